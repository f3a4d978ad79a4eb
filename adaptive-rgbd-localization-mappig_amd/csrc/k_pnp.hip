// PnPSolver::Compute for gfx950 (Odometry/pnpsolver.cpp:17-214): motion-only
// bundle adjustment of one SE3Expmap vertex with mono / stereo reprojection
// edges, Huber kernel, 4 rounds x optimize(10) with chi2 re-classification,
// g2o OptimizationAlgorithmLevenberg + LinearSolverDense (Eigen LDLT)
// semantics. One 256-thread workgroup per frame pair;
// per-edge work is spread over lanes and summed with a fixed-order tree
// (deterministic run to run; agrees with the sequential oracle to rounding).
#include "odo_device.h"
#include "odo_internal.h"

namespace odo {

#define PNP_THREADS 256

struct Quat {
    double x, y, z, w;
};
struct SE3 {
    Quat q;
    double t[3];
};

ODO_INLINE void cross3(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
ODO_INLINE void qrot(const Quat& q, const double v[3], double o[3]) {
    const double qv[3] = {q.x, q.y, q.z};
    double uv[3], uv2[3];
    cross3(qv, v, uv);
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    cross3(qv, uv, uv2);
    for (int i = 0; i < 3; i++) o[i] = v[i] + q.w * uv[i] + uv2[i];
}
ODO_INLINE Quat qmul(const Quat& a, const Quat& b) {
    return Quat{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
                a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
ODO_INLINE Quat quat_from_R(const double m[3][3]) {
    Quat q;
    double t = sum3d(m[0][0], m[1][1], m[2][2]);
    if (t > 0) {
        t = sqrt(t + 1.0);
        q.w = 0.5 * t;
        t = 0.5 / t;
        q.x = (m[2][1] - m[1][2]) * t;
        q.y = (m[0][2] - m[2][0]) * t;
        q.z = (m[1][0] - m[0][1]) * t;
    } else {
        int i = 0;
        if (m[1][1] > m[0][0]) i = 1;
        if (m[2][2] > m[i][i]) i = 2;
        int j = (i + 1) % 3, k = (j + 1) % 3;
        t = sqrt(m[i][i] - m[j][j] - m[k][k] + 1.0);
        double c[3];
        c[i] = 0.5 * t;
        t = 0.5 / t;
        q.w = (m[k][j] - m[j][k]) * t;
        c[j] = (m[j][i] + m[i][j]) * t;
        c[k] = (m[k][i] + m[i][k]) * t;
        q.x = c[0];
        q.y = c[1];
        q.z = c[2];
    }
    return q;
}
ODO_INLINE void quat_to_R(const Quat& q, double r[3][3]) {
    const double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    r[0][0] = 1 - (tyy + tzz);
    r[0][1] = txy - twz;
    r[0][2] = txz + twy;
    r[1][0] = txy + twz;
    r[1][1] = 1 - (txx + tzz);
    r[1][2] = tyz - twx;
    r[2][0] = txz - twy;
    r[2][1] = tyz + twx;
    r[2][2] = 1 - (txx + tyy);
}
ODO_INLINE void normalize_rot(SE3& s) {
    if (s.q.w < 0) {
        s.q.x = -s.q.x;
        s.q.y = -s.q.y;
        s.q.z = -s.q.z;
        s.q.w = -s.q.w;
    }
    double n = sqrt((s.q.x * s.q.x + s.q.y * s.q.y) + (s.q.z * s.q.z + s.q.w * s.q.w));
    s.q.x /= n;
    s.q.y /= n;
    s.q.z /= n;
    s.q.w /= n;
}
ODO_INLINE SE3 se3_mul(const SE3& a, const SE3& b) {
    SE3 r = a;
    double rt[3];
    qrot(a.q, b.t, rt);
    for (int i = 0; i < 3; i++) r.t[i] += rt[i];
    r.q = qmul(a.q, b.q);
    normalize_rot(r);
    return r;
}
ODO_INLINE SE3 se3_exp(const double u[6]) {
    const double w[3] = {u[0], u[1], u[2]};
    const double up[3] = {u[3], u[4], u[5]};
    double theta = sqrt(sum3d(w[0] * w[0], w[1] * w[1], w[2] * w[2]));
    double O[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    double O2[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) O2[i][j] = sum3d(O[i][0] * O[0][j], O[i][1] * O[1][j], O[i][2] * O[2][j]);
    double R[3][3], V[3][3];
    if (theta < 0.00001) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = ((i == j ? 1.0 : 0.0) + O[i][j]) + O2[i][j];
                V[i][j] = R[i][j];
            }
    } else {
        double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
        double c = (theta - sin(theta)) / (theta * theta * theta);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = ((i == j ? 1.0 : 0.0) + a * O[i][j]) + b * O2[i][j];
                V[i][j] = ((i == j ? 1.0 : 0.0) + b * O[i][j]) + c * O2[i][j];
            }
    }
    SE3 s;
    for (int i = 0; i < 3; i++) s.t[i] = sum3d(V[i][0] * up[0], V[i][1] * up[1], V[i][2] * up[2]);
    s.q = quat_from_R(R);
    normalize_rot(s);
    return s;
}
ODO_INLINE void se3_map(const SE3& T, const double p[3], double o[3]) {
    qrot(T.q, p, o);
    for (int i = 0; i < 3; i++) o[i] += T.t[i];
}

// Eigen LDLT with diagonal pivoting on a 6x6 (one thread).
ODO_INLINE bool ldlt_solve6(const double Ain[6][6], const double b[6], double x[6]) {
    const int n = 6;
    double m[6][6];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < 6; j++) m[i][j] = Ain[i][j];
    int tr[6];
    int sign = 0;
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = fabs(m[k][k]);
        for (int i = k + 1; i < n; i++)
            if (fabs(m[i][i]) > bv) {
                bv = fabs(m[i][i]);
                big = i;
            }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) {
                double a = m[k][j];
                m[k][j] = m[big][j];
                m[big][j] = a;
            }
            for (int i = big + 1; i < n; i++) {
                double a = m[i][k];
                m[i][k] = m[i][big];
                m[i][big] = a;
            }
            double a = m[k][k];
            m[k][k] = m[big][big];
            m[big][big] = a;
            for (int i = k + 1; i < big; i++) {
                double tmp = m[i][k];
                m[i][k] = m[big][i];
                m[big][i] = tmp;
            }
        }
        double temp[6];
        if (k > 0) {
            for (int j = 0; j < k; j++) temp[j] = m[j][j] * m[k][j];
            double s = 0;
            for (int j = 0; j < k; j++) s += m[k][j] * temp[j];
            m[k][k] -= s;
            for (int i = k + 1; i < n; i++) {
                double tt = 0;
                for (int j = 0; j < k; j++) tt += m[i][j] * temp[j];
                m[i][k] -= tt;
            }
        }
        double akk = m[k][k];
        bool valid = fabs(akk) > 0;
        if (k == 0 && !valid) return false;
        if (valid)
            for (int i = k + 1; i < n; i++) m[i][k] /= akk;
        if (sign == 1) {
            if (akk < 0) sign = 3;
        } else if (sign == 2) {
            if (akk > 0) sign = 3;
        } else if (sign == 0) {
            if (akk > 0) sign = 1;
            else if (akk < 0) sign = 2;
        }
    }
    if (!(sign == 1 || sign == 0)) return false;
    double y[6];
    for (int i = 0; i < 6; i++) y[i] = b[i];
    for (int k = 0; k < n; k++) {
        double a = y[k];
        y[k] = y[tr[k]];
        y[tr[k]] = a;
    }
    for (int i = 0; i < n; i++) {
        double s = 0;
        for (int j = 0; j < i; j++) s += m[i][j] * y[j];
        y[i] -= s;
    }
    for (int i = 0; i < n; i++) {
        if (fabs(m[i][i]) > 2.2250738585072014e-308) y[i] /= m[i][i];
        else y[i] = 0;
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = 0;
        for (int j = i + 1; j < n; j++) s += m[j][i] * y[j];
        y[i] -= s;
    }
    for (int k = n - 1; k >= 0; k--) {
        double a = y[k];
        y[k] = y[tr[k]];
        y[tr[k]] = a;
    }
    for (int i = 0; i < 6; i++) x[i] = y[i];
    return true;
}

struct PEdge {
    double Xw[3];
    double obs[3];
    double info;
    double delta;
    double err[3];
    int stereo;
    int level;
    int robust;
    int idx;  // F2 keypoint index
};

// ----- fixed-order block reduction of NV doubles (lane-serial, xor butterfly, waves in order)
template <int NV>
ODO_INLINE void block_reduce(double (&v)[NV], double* red /* 4*NV */) {
#pragma unroll
    for (int k = 0; k < NV; k++) {
        double x = v[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        v[k] = x;
    }
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0)
        for (int k = 0; k < NV; k++) red[wave * NV + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; k++) v[k] = ((red[k] + red[NV + k]) + red[2 * NV + k]) + red[3 * NV + k];
    __syncthreads();
}

struct PnPCam {
    double fx, fy, cx, cy, bf;
};

ODO_INLINE void edge_error(PEdge& e, const SE3& T, const PnPCam& c) {
    double Xc[3];
    se3_map(T, e.Xw, Xc);
    if (!e.stereo) {
        double px = Xc[0] / Xc[2], py = Xc[1] / Xc[2];
        e.err[0] = e.obs[0] - (px * c.fx + c.cx);
        e.err[1] = e.obs[1] - (py * c.fy + c.cy);
        e.err[2] = 0;
    } else {
        const float invz = (float)(1.0 / Xc[2]);
        const double iz = (double)invz;
        double r0 = Xc[0] * iz * c.fx + c.cx;
        double r1 = Xc[1] * iz * c.fy + c.cy;
        double r2 = r0 - c.bf * iz;
        e.err[0] = e.obs[0] - r0;
        e.err[1] = e.obs[1] - r1;
        e.err[2] = e.obs[2] - r2;
    }
}
ODO_INLINE double edge_chi2(const PEdge& e) {
    if (!e.stereo) return e.err[0] * (e.info * e.err[0]) + e.err[1] * (e.info * e.err[1]);
    return sum3d(e.err[0] * (e.info * e.err[0]), e.err[1] * (e.info * e.err[1]), e.err[2] * (e.info * e.err[2]));
}
ODO_INLINE void huber(const PEdge& e, double chi, double rho[3]) {
    double dsqr = e.delta * e.delta;
    if (chi <= dsqr) {
        rho[0] = chi;
        rho[1] = 1.;
        rho[2] = 0.;
    } else {
        double sq = sqrt(chi);
        rho[0] = 2 * sq * e.delta - dsqr;
        rho[1] = e.delta / sq;
        rho[2] = -0.5 * rho[1] / chi;
    }
}

__global__ void __launch_bounds__(PNP_THREADS) k_pnp(const int32_t* __restrict__ f2_src, const float* __restrict__ xyz,
                                                     const float* __restrict__ kun, const float* __restrict__ ur,
                                                     const int* __restrict__ nkp, int kp_cap, int slot0,
                                                     FrameCalib cal, const float* __restrict__ T12,
                                                     const int* __restrict__ pair_valid, const int* __restrict__ n_matches,
                                                     int min_matches,
                                                     PEdge* __restrict__ edges_g, odo_pair_result* __restrict__ res,
                                                     uint8_t* __restrict__ inlier_mask) {
    const int p = blockIdx.x;
    const int t = threadIdx.x;
    __shared__ double red[4 * 28];
    __shared__ int s_scan[PNP_THREADS];
    __shared__ SE3 s_T, s_backup, s_T0;
    __shared__ double s_H[6][6], s_b[6], s_x[6];
    __shared__ double s_lambda, s_ni, s_curChi, s_rho;
    __shared__ int s_ok2, s_stop, s_qmax, s_nedges, s_accept;
    odo_pair_result* R = res + p;
    const int s1 = slot0 + p, s2 = slot0 + p + 1;
    const int n2 = nkp[s2];
    uint8_t* mask = inlier_mask + (size_t)p * kp_cap;
    for (int i = t; i < n2; i += PNP_THREADS) mask[i] = 0;
    const float* T0 = T12 + (size_t)p * 16;
    if (t == 0) {
        for (int i = 0; i < 16; i++) R->Tcw[i] = T0[i];
        R->pnp_inliers = 0;
    }
    if (!pair_valid[p] || n_matches[p] < min_matches) return;
    // ---- edges: F2 keypoints holding a landmark, index order (pnpsolver.cpp:57-135)
    const int32_t* src = f2_src + (size_t)p * kp_cap;
    const float* X1 = xyz + (size_t)s1 * kp_cap * 3;
    const float* K2 = kun + (size_t)s2 * kp_cap * 2;
    const float* U2 = ur + (size_t)s2 * kp_cap;
    PEdge* E = edges_g + (size_t)p * kp_cap;
    const float deltaMono = (float)sqrt(5.991), deltaStereo = (float)sqrt(7.815);  // pnpsolver.cpp:51-52
    int base = 0;
    for (int c0 = 0; c0 < n2; c0 += PNP_THREADS) {
        const int i = c0 + t;
        const int has = (i < n2 && src[i] >= 0) ? 1 : 0;
        s_scan[t] = has;
        __syncthreads();
        for (int off = 1; off < PNP_THREADS; off <<= 1) {
            int a = t >= off ? s_scan[t - off] : 0;
            __syncthreads();
            s_scan[t] += a;
            __syncthreads();
        }
        const int incl = s_scan[t], tot = s_scan[PNP_THREADS - 1];
        if (has) {
            PEdge e;
            const int s = src[i];
            for (int k = 0; k < 3; k++) e.Xw[k] = (double)X1[3 * s + k];
            const float urv = U2[i];
            e.stereo = !(urv < 0);
            e.obs[0] = K2[2 * i];
            e.obs[1] = K2[2 * i + 1];
            e.obs[2] = e.stereo ? (double)urv : 0.0;
            const float zw = X1[3 * s + 2];
            const float sigma = 1.0f / (zw * zw);
            e.info = sigma;
            e.delta = e.stereo ? (double)deltaStereo : (double)deltaMono;
            e.level = 0;
            e.robust = 1;
            e.err[0] = e.err[1] = e.err[2] = 0;
            e.idx = i;
            E[base + incl - 1] = e;
        }
        base += tot;
        __syncthreads();
    }
    const int ne = base;
    if (ne < 3) {
        for (int k = t; k < ne; k += PNP_THREADS) mask[E[k].idx] = 1;  // set inlier at edge creation
        return;
    }
    PnPCam cam{(double)cal.fx, (double)cal.fy, (double)cal.cx, (double)cal.cy, (double)cal.mbf};
    if (t == 0) {
        double R0[3][3], t0[3];
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) R0[i][j] = (double)T0[i * 4 + j];
            t0[i] = (double)T0[i * 4 + 3];
        }
        s_T0.q = quat_from_R(R0);
        for (int i = 0; i < 3; i++) s_T0.t[i] = t0[i];
        normalize_rot(s_T0);
    }
    __syncthreads();
    const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        if (t == 0) s_T = s_T0;
        __syncthreads();
        // ---------------- optimize(10)
        for (int iter = 0; iter < 10; iter++) {
            // computeActiveErrors + activeRobustChi2 + buildSystem at s_T
            const SE3 T = s_T;
            double acc[28];
            for (int k = 0; k < 28; k++) acc[k] = 0;
            for (int k = t; k < ne; k += PNP_THREADS) {
                PEdge e = E[k];
                if (e.level != 0) continue;
                edge_error(e, T, cam);
                E[k].err[0] = e.err[0];
                E[k].err[1] = e.err[1];
                E[k].err[2] = e.err[2];
                const double c2 = edge_chi2(e);
                double rho[3] = {c2, 1.0, 0.0};
                if (e.robust) huber(e, c2, rho);
                acc[27] += rho[0];
                double Xc[3];
                se3_map(T, e.Xw, Xc);
                const double x = Xc[0], y = Xc[1], invz = 1.0 / Xc[2], invz_2 = invz * invz;
                double J[3][6];
                J[0][0] = x * y * invz_2 * cam.fx;
                J[0][1] = -(1 + (x * x * invz_2)) * cam.fx;
                J[0][2] = y * invz * cam.fx;
                J[0][3] = -invz * cam.fx;
                J[0][4] = 0;
                J[0][5] = x * invz_2 * cam.fx;
                J[1][0] = (1 + y * y * invz_2) * cam.fy;
                J[1][1] = -x * y * invz_2 * cam.fy;
                J[1][2] = -x * invz * cam.fy;
                J[1][3] = 0;
                J[1][4] = -invz * cam.fy;
                J[1][5] = y * invz_2 * cam.fy;
                const int D = e.stereo ? 3 : 2;
                if (e.stereo) {
                    J[2][0] = J[0][0] - cam.bf * y * invz_2;
                    J[2][1] = J[0][1] + cam.bf * x * invz_2;
                    J[2][2] = J[0][2];
                    J[2][3] = J[0][3];
                    J[2][4] = 0;
                    J[2][5] = J[0][5] - cam.bf * invz_2;
                }
                const double r1 = rho[1];
                const double wo = r1 * e.info;
                int h = 0;
                for (int a = 0; a < 6; a++) {
                    double s = 0;
                    for (int kk = 0; kk < D; kk++) s += J[kk][a] * (e.info * e.err[kk]);
                    acc[21 + a] -= r1 * s;
                    for (int c = a; c < 6; c++) {
                        double hh = 0;
                        for (int kk = 0; kk < D; kk++) hh += J[kk][a] * wo * J[kk][c];
                        acc[h++] += hh;
                    }
                }
            }
            block_reduce<28>(acc, red);
            if (t == 0) {
                int h = 0;
                for (int a = 0; a < 6; a++)
                    for (int c = a; c < 6; c++) {
                        s_H[a][c] = acc[h];
                        s_H[c][a] = acc[h];
                        h++;
                    }
                for (int a = 0; a < 6; a++) s_b[a] = acc[21 + a];
                s_curChi = acc[27];
                if (iter == 0) {
                    double mx = 0;
                    for (int j = 0; j < 6; j++) mx = fmax(fabs(s_H[j][j]), mx);
                    s_lambda = 1e-5 * mx;
                    s_ni = 2;
                }
                s_qmax = 0;
                s_stop = 0;
            }
            __syncthreads();
            // LM trials (OptimizationAlgorithmLevenberg::solve)
            while (true) {
                if (t == 0) {
                    s_backup = s_T;
                    double Hl[6][6];
                    for (int a = 0; a < 6; a++)
                        for (int c = 0; c < 6; c++) Hl[a][c] = s_H[a][c];
                    for (int j = 0; j < 6; j++) Hl[j][j] += s_lambda;
                    double x[6] = {0, 0, 0, 0, 0, 0};
                    s_ok2 = ldlt_solve6(Hl, s_b, x) ? 1 : 0;
                    for (int j = 0; j < 6; j++) s_x[j] = x[j];
                    s_T = se3_mul(se3_exp(x), s_T);
                }
                __syncthreads();
                const SE3 Tn = s_T;
                double chi[1] = {0};
                for (int k = t; k < ne; k += PNP_THREADS) {
                    PEdge e = E[k];
                    if (e.level != 0) continue;
                    edge_error(e, Tn, cam);
                    E[k].err[0] = e.err[0];
                    E[k].err[1] = e.err[1];
                    E[k].err[2] = e.err[2];
                    const double c2 = edge_chi2(e);
                    if (e.robust) {
                        double rho[3];
                        huber(e, c2, rho);
                        chi[0] += rho[0];
                    } else chi[0] += c2;
                }
                block_reduce<1>(chi, red);
                if (t == 0) {
                    double tempChi = chi[0];
                    if (!s_ok2) tempChi = 1.7976931348623157e308;
                    double rho = s_curChi - tempChi;
                    double scale = 0;
                    for (int j = 0; j < 6; j++) scale += s_x[j] * (s_lambda * s_x[j] + s_b[j]);
                    scale += 1e-3;
                    rho /= scale;
                    if (rho > 0 && isfinite(tempChi)) {
                        double alpha = 1. - pow((2 * rho - 1), 3);
                        alpha = fmin(alpha, 2. / 3.);
                        double sf = fmax(1. / 3., alpha);
                        s_lambda *= sf;
                        s_ni = 2;
                        s_curChi = tempChi;
                    } else {
                        s_lambda *= s_ni;
                        s_ni *= 2;
                        s_T = s_backup;
                    }
                    s_qmax++;
                    s_rho = rho;
                    s_accept = (rho < 0 && s_qmax < 10) ? 0 : 1;
                    if (s_accept && (s_qmax == 10 || rho == 0)) s_stop = 1;
                }
                __syncthreads();
                if (s_accept) break;
            }
            if (s_stop) break;
        }
        // ---------------- classification (pnpsolver.cpp:149-205)
        const SE3 T = s_T;
        double bad[1] = {0};
        for (int k = t; k < ne; k += PNP_THREADS) {
            PEdge e = E[k];
            const int idx = e.idx;
            if (mask[idx] == 2) {  // outlier from the previous round: recompute at current estimate
                edge_error(e, T, cam);
                E[k].err[0] = e.err[0];
                E[k].err[1] = e.err[1];
                E[k].err[2] = e.err[2];
            }
            const float chi2 = (float)edge_chi2(e);
            const float th = e.stereo ? chi2Stereo : chi2Mono;
            if (chi2 > th) {
                mask[idx] = 2;
                E[k].level = 1;
                bad[0] += 1;
            } else {
                mask[idx] = 1;
                E[k].level = 0;
            }
            if (it == 2) E[k].robust = 0;
        }
        block_reduce<1>(bad, red);
        nBad = (int)bad[0];
        if (ne < 10) break;
    }
    if (t == 0) {
        double Rm[3][3];
        quat_to_R(s_T.q, Rm);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) R->Tcw[i * 4 + j] = (float)Rm[i][j];
            R->Tcw[i * 4 + 3] = (float)s_T.t[i];
        }
        R->Tcw[12] = R->Tcw[13] = R->Tcw[14] = 0.f;
        R->Tcw[15] = 1.f;
        R->pnp_inliers = ne - nBad;
    }
    __syncthreads();
    for (int i = t; i < n2; i += PNP_THREADS) mask[i] = mask[i] == 1 ? 1 : 0;
}

}  // namespace odo

namespace odo {
size_t pnp_edge_bytes() { return sizeof(PEdge); }
void launch_pnp(hipStream_t st, const int32_t* f2_src, const float* xyz, const float* kun, const float* ur,
                const int* nkp, int kp_cap, int slot0, FrameCalib cal, const float* T12, const int* pair_valid,
                const int* n_matches, int min_matches, void* edges, odo_pair_result* res, uint8_t* inlier_mask,
                int npairs) {
    hipLaunchKernelGGL(k_pnp, dim3(npairs), dim3(PNP_THREADS), 0, st, f2_src, xyz, kun, ur, nkp, kp_cap, slot0, cal,
                       T12, pair_valid, n_matches, min_matches, (PEdge*)edges, res, inlier_mask);
}
}  // namespace odo

// ============================================================ Kabsch::Compute
// Odometry/kabsch.cpp:14-57 (dead code in the reference, exported for
// completeness): centroids, A = (A-cA)^T (B-cB), JacobiSVD (same 3x3 Jacobi as
// the RANSAC fit), R = W diag(1,1,sgn det A) V^T, t = -R cA + cB. One
// workgroup; sums use the fixed-order block reduction.
namespace odo {
__global__ void __launch_bounds__(PNP_THREADS) k_kabsch(const float* __restrict__ A, const float* __restrict__ B, int n,
                                                        float* __restrict__ T) {
    __shared__ double red[4 * 28];
    const int t = threadIdx.x;
    if (n == 0) {
        if (t < 16) T[t] = (t % 5 == 0) ? 1.f : 0.f;
        return;
    }
    double s[6] = {0, 0, 0, 0, 0, 0};
    for (int i = t; i < n; i += PNP_THREADS)
        for (int k = 0; k < 3; k++) {
            s[k] += A[3 * i + k];
            s[3 + k] += B[3 * i + k];
        }
    block_reduce<6>(s, red);
    float cA[3], cB[3];
    for (int k = 0; k < 3; k++) {
        cA[k] = (float)s[k] / (float)n;
        cB[k] = (float)s[3 + k] / (float)n;
    }
    double m[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = t; i < n; i += PNP_THREADS)
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) m[a * 3 + b] += (double)((A[3 * i + a] - cA[a]) * (B[3 * i + b] - cB[b]));
    block_reduce<9>(m, red);
    if (t == 0) {
        float M[3][3], Vm[3][3], S[3], Wm[3][3];
        for (int i = 0; i < 9; i++) M[i / 3][i % 3] = (float)m[i];
        svd3(M, Vm, S, Wm);  // V = svd.matrixU(), W = svd.matrixV()
        const float d = det3(M);
        const float sg = (d != 0.f) ? (float)((d > 0.f) - (d < 0.f)) : 1.f;
        float R[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = Wm[i][0] * Vm[j][0] + Wm[i][1] * Vm[j][1] + Wm[i][2] * sg * Vm[j][2];
        for (int i = 0; i < 3; i++) {
            const float tt = (R[i][0] * -cA[0] + R[i][1] * -cA[1] + R[i][2] * -cA[2]) + cB[i];
            for (int j = 0; j < 3; j++) T[i * 4 + j] = R[i][j];
            T[i * 4 + 3] = tt;
        }
        T[12] = T[13] = T[14] = 0.f;
        T[15] = 1.f;
    }
}
void launch_kabsch(hipStream_t st, const float* A, const float* B, int n, float* T) {
    hipLaunchKernelGGL(k_kabsch, dim3(1), dim3(PNP_THREADS), 0, st, A, B, n, T);
}
}  // namespace odo
