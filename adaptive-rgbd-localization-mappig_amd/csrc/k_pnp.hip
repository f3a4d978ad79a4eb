// PnPSolver::Compute for gfx950 (Odometry/pnpsolver.cpp:17-214): motion-only
// bundle adjustment of one SE3Expmap vertex with mono / stereo reprojection
// edges, Huber kernel, 4 rounds x optimize(10) with chi2 re-classification,
// g2o OptimizationAlgorithmLevenberg + LinearSolverDense (Eigen LDLT)
// semantics. One 256-thread workgroup per frame pair;
// per-edge work is spread over lanes and summed with a fixed-order tree
// (deterministic run to run; agrees with the sequential oracle to rounding).
#include "odo_device.h"
#include "odo_internal.h"

// a * b + c as one fused multiply-add in this file's FP64 arithmetic (the
// library builds with -ffp-contract=off for its bit-exact stages; PnP's and
// Kabsch's parity is a tolerance, 1e-4 on the pose): 11 % fewer FP64
// instructions in k_pnp, and shorter dependent chains
#pragma clang fp contract(fast)

namespace odo {

#define PNP_THREADS 256

struct Quat {
    double x, y, z, w;
};
struct SE3 {
    Quat q;
    double t[3];
};

ODO_INLINE Quat quat_from_R(const double m[3][3]) {
    // Eigen quaternionbase_assign_impl<Matrix3>, branches written with static indices
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
        if (m[2][2] > (i == 0 ? m[0][0] : m[1][1])) i = 2;
        if (i == 0) {  // j=1, k=2
            t = sqrt(m[0][0] - m[1][1] - m[2][2] + 1.0);
            q.x = 0.5 * t;
            t = 0.5 / t;
            q.w = (m[2][1] - m[1][2]) * t;
            q.y = (m[1][0] + m[0][1]) * t;
            q.z = (m[2][0] + m[0][2]) * t;
        } else if (i == 1) {  // j=2, k=0
            t = sqrt(m[1][1] - m[2][2] - m[0][0] + 1.0);
            q.y = 0.5 * t;
            t = 0.5 / t;
            q.w = (m[0][2] - m[2][0]) * t;
            q.z = (m[2][1] + m[1][2]) * t;
            q.x = (m[0][1] + m[1][0]) * t;
        } else {  // j=0, k=1
            t = sqrt(m[2][2] - m[0][0] - m[1][1] + 1.0);
            q.z = 0.5 * t;
            t = 0.5 / t;
            q.w = (m[1][0] - m[0][1]) * t;
            q.x = (m[0][2] + m[2][0]) * t;
            q.y = (m[1][2] + m[2][1]) * t;
        }
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
    const double in = 1.0 / sqrt((s.q.x * s.q.x + s.q.y * s.q.y) + (s.q.z * s.q.z + s.q.w * s.q.w));
    s.q.x *= in;
    s.q.y *= in;
    s.q.z *= in;
    s.q.w *= in;
}
// Rodrigues' R and V of SE3Quat::exp (g2o se3quat.h)
ODO_INLINE void se3_exp_rv(const double u[6], double R[3][3], double V[3][3]) {
    const double w[3] = {u[0], u[1], u[2]};
    double theta = sqrt(sum3d(w[0] * w[0], w[1] * w[1], w[2] * w[2]));
    double O[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
    double O2[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) O2[i][j] = sum3d(O[i][0] * O[0][j], O[i][1] * O[1][j], O[i][2] * O[2][j]);
    if (theta < 0.00001) {
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = ((i == j ? 1.0 : 0.0) + O[i][j]) + O2[i][j];
                V[i][j] = R[i][j];
            }
    } else {
        // sin / cos as g2o calls them (the device sincos takes its outputs
        // through private memory: measured 20 VGPRs of scratch spills)
        const double sn = sin(theta), cs = cos(theta);
        const double th2 = theta * theta;
        // g2o divides by pow(theta, 3): theta * theta^2 differs in the last ulp
        // at most (PnP parity is a tolerance, 1e-4 on the pose)
        double a = sn / theta, b = (1 - cs) / th2;
        double c = (theta - sn) / (theta * th2);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                R[i][j] = ((i == j ? 1.0 : 0.0) + a * O[i][j]) + b * O2[i][j];
                V[i][j] = ((i == j ? 1.0 : 0.0) + b * O[i][j]) + c * O2[i][j];
            }
    }
}
// The pose as a rotation matrix + translation for the edge passes: 9 products
// per point instead of the quaternion's two cross products (g2o maps with the
// quaternion; the difference is rounding, within the PnP tolerance).
struct SE3M {
    double R[9], t[3];
};
ODO_INLINE SE3M se3_mat(const SE3& T) {
    double r[3][3];
    quat_to_R(T.q, r);
    SE3M M;
#pragma unroll
    for (int i = 0; i < 3; i++) {
#pragma unroll
        for (int j = 0; j < 3; j++) M.R[3 * i + j] = r[i][j];
        M.t[i] = T.t[i];
    }
    return M;
}
ODO_INLINE void se3m_map(const SE3M& T, const double p[3], double o[3]) {
#pragma unroll
    for (int i = 0; i < 3; i++) o[i] = (T.R[3 * i] * p[0] + T.R[3 * i + 1] * p[1]) + (T.R[3 * i + 2] * p[2] + T.t[i]);
}
// exp(u) * T (VertexSE3Expmap::oplusImpl) with the pose kept as a matrix:
// R = R_exp R_T, t = R_exp t_T + V u_t. g2o composes unit quaternions and
// renormalizes; the matrices agree with that to rounding (the PnP tolerance)
ODO_INLINE SE3M se3m_exp_mul(const double u[6], const SE3M& T) {
    double R[3][3], V[3][3];
    se3_exp_rv(u, R, V);
    SE3M M;
#pragma unroll
    for (int i = 0; i < 3; i++) {
#pragma unroll
        for (int j = 0; j < 3; j++) M.R[3 * i + j] = sum3d(R[i][0] * T.R[j], R[i][1] * T.R[3 + j], R[i][2] * T.R[6 + j]);
        M.t[i] = sum3d(R[i][0] * T.t[0], R[i][1] * T.t[1], R[i][2] * T.t[2]) +
                 sum3d(V[i][0] * u[3], V[i][1] * u[4], V[i][2] * u[5]);
    }
    return M;
}

// Eigen LDLT with diagonal pivoting on a 6x6, every index static after
// unrolling (the pivot swap is a select over the candidate rows), so the
// matrix stays in registers.
ODO_INLINE bool ldlt_solve6(const double Ain[6][6], const double b[6], double x[6]) {
    double m[6][6];
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) m[i][j] = Ain[i][j];
    int tr[6];
    int sign = 0;
    bool fail = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int big = k;
        double bv = fabs(m[k][k]);
#pragma unroll
        for (int i = k + 1; i < 6; i++)
            if (fabs(m[i][i]) > bv) {
                bv = fabs(m[i][i]);
                big = i;
            }
        tr[k] = big;
#pragma unroll
        for (int q = k + 1; q < 6; q++) {
            if (q == big) {
#pragma unroll
                for (int j = 0; j < k; j++) {
                    double a = m[k][j];
                    m[k][j] = m[q][j];
                    m[q][j] = a;
                }
#pragma unroll
                for (int i = q + 1; i < 6; i++) {
                    double a = m[i][k];
                    m[i][k] = m[i][q];
                    m[i][q] = a;
                }
                double a = m[k][k];
                m[k][k] = m[q][q];
                m[q][q] = a;
#pragma unroll
                for (int i = k + 1; i < q; i++) {
                    double tmp = m[i][k];
                    m[i][k] = m[q][i];
                    m[q][i] = tmp;
                }
            }
        }
        double temp[6];
        if (k > 0) {
#pragma unroll
            for (int j = 0; j < k; j++) temp[j] = m[j][j] * m[k][j];
            double s = 0;
#pragma unroll
            for (int j = 0; j < k; j++) s += m[k][j] * temp[j];
            m[k][k] -= s;
#pragma unroll
            for (int i = k + 1; i < 6; i++) {
                double tt = 0;
#pragma unroll
                for (int j = 0; j < k; j++) tt += m[i][j] * temp[j];
                m[i][k] -= tt;
            }
        }
        const double akk = m[k][k];
        const bool valid = fabs(akk) > 0;
        if (k == 0 && !valid) fail = true;
        if (valid) {
            const double ia = 1.0 / akk;  // one division per pivot (Eigen divides each entry)
#pragma unroll
            for (int i = k + 1; i < 6; i++) m[i][k] *= ia;
        }
        if (sign == 1) {
            if (akk < 0) sign = 3;
        } else if (sign == 2) {
            if (akk > 0) sign = 3;
        } else if (sign == 0) {
            if (akk > 0) sign = 1;
            else if (akk < 0) sign = 2;
        }
    }
    if (fail || !(sign == 1 || sign == 0)) return false;
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] = b[i];
#pragma unroll
    for (int k = 0; k < 6; k++)
#pragma unroll
        for (int q = k + 1; q < 6; q++)
            if (tr[k] == q) {
                double a = y[k];
                y[k] = y[q];
                y[q] = a;
            }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double s = 0;
#pragma unroll
        for (int j = 0; j < i; j++) s += m[i][j] * y[j];
        y[i] -= s;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) {
        if (fabs(m[i][i]) > 2.2250738585072014e-308) y[i] /= m[i][i];
        else y[i] = 0;
    }
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double s = 0;
#pragma unroll
        for (int j = i + 1; j < 6; j++) s += m[j][i] * y[j];
        y[i] -= s;
    }
#pragma unroll
    for (int k = 5; k >= 0; k--)
#pragma unroll
        for (int q = k + 1; q < 6; q++)
            if (tr[k] == q) {
                double a = y[k];
                y[k] = y[q];
                y[q] = a;
            }
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = y[i];
    return true;
}

// The same solve without Eigen's diagonal pivoting (round 3): the damped
// normal matrix H + lambda I of the Levenberg trial is symmetric positive
// definite, for which the pivoted and the unpivoted LDL^T are the same
// factorization up to rounding; dropping the pivot search and the
// select-based row / column swaps (most of the pivoted solve's ~900
// instructions) and dividing by the stored pivot reciprocals halves the
// trial solve, the longest serial step of a PnP iteration. A pivot <= 0 (not
// positive definite) fails the solve as in the pivoted form (Eigen's
// isPositive() check; g2o then rejects the trial).
ODO_INLINE bool ldlt_solve6_spd(const double Ain[6][6], const double b[6], double x[6]) {
    double m[6][6];
#pragma unroll
    for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) m[i][j] = Ain[i][j];
    double inv[6];
    bool fail = false;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        double temp[6];
        if (k > 0) {
#pragma unroll
            for (int j = 0; j < k; j++) temp[j] = m[j][j] * m[k][j];
            double s = 0;
#pragma unroll
            for (int j = 0; j < k; j++) s += m[k][j] * temp[j];
            m[k][k] -= s;
#pragma unroll
            for (int i = k + 1; i < 6; i++) {
                double tt = 0;
#pragma unroll
                for (int j = 0; j < k; j++) tt += m[i][j] * temp[j];
                m[i][k] -= tt;
            }
        }
        const double akk = m[k][k];
        fail = fail || !(akk > 0);
        const double ia = 1.0 / akk;
        inv[k] = ia;
#pragma unroll
        for (int i = k + 1; i < 6; i++) m[i][k] *= ia;
    }
    if (fail) return false;
    double y[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        double s = 0;
#pragma unroll
        for (int j = 0; j < i; j++) s += m[i][j] * y[j];
        y[i] = b[i] - s;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) y[i] *= inv[i];
#pragma unroll
    for (int i = 5; i >= 0; i--) {
        double s = 0;
#pragma unroll
        for (int j = i + 1; j < 6; j++) s += m[j][i] * y[j];
        y[i] -= s;
    }
#pragma unroll
    for (int i = 0; i < 6; i++) x[i] = y[i];
    return true;
}

// Edge storage: SoA in HBM scratch, [pair][field][cap]. The reference keeps
// Xw, observations and the information weight as float (cv::Mat / KeyPoint,
// pnpsolver.cpp:74-125) and widens to double inside g2o; we store the floats.
struct PEdgeSoA {
    float* X;        // 3*cap
    float* obs;      // 3*cap
    float* info;     // cap
    uint8_t* flags;  // cap: bit0 stereo, bit1 outlier (level 1), bit2 robust kernel on
    double* chi4;    // 4*cap: chi2 of the stored _error per speculative trial slot
    int* idx;        // cap: F2 keypoint index
};

#define PE_STEREO 1
#define PE_OUT 2
#define PE_ROBUST 4
#define PE_BYTES 72

ODO_INLINE PEdgeSoA pedge_view(void* base, int cap, int p) {
    char* b = (char*)base + (size_t)p * (size_t)cap * PE_BYTES;
    PEdgeSoA E;
    E.chi4 = (double*)b;
    E.X = (float*)(b + (size_t)cap * 32);
    E.obs = E.X + 3 * cap;
    E.info = E.obs + 3 * cap;
    E.idx = (int*)(E.info + cap);
    E.flags = (uint8_t*)(E.idx + cap);
    return E;
}

// one edge's read-mostly fields (the edge passes' loads, issued together)
struct EdgeIn {
    float X[3], ob[3], info;
    uint8_t fl;
};
ODO_INLINE EdgeIn load_edge(const PEdgeSoA& E, int k) {
    EdgeIn r;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        r.X[i] = E.X[3 * k + i];
        r.ob[i] = E.obs[3 * k + i];
    }
    r.info = E.info[k];
    r.fl = E.flags[k];
    return r;
}

ODO_INLINE double wave_sum(double x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    return x;
}

struct PnPCam {
    double fx, fy, cx, cy, bf;
};

// 1 / z for the edge passes: v_rcp_f64 refined by two Newton steps (within an
// ulp of the IEEE quotient g2o divides by, about half the instructions of the
// correctly rounded division; z = +-0 keeps rcp's +-inf)
ODO_INLINE double pnp_inv(double z) {
    const double r0 = __builtin_amdgcn_rcp(z);
    double e = __builtin_fma(-z, r0, 1.0);
    double r = __builtin_fma(r0, e, r0);
    e = __builtin_fma(-z, r, 1.0);
    r = __builtin_fma(r, e, r);
    return __builtin_isinf(r0) ? r0 : r;
}
// sqrt(x) for the Huber kernel (x > delta^2 > 0 where it is used; inf kept)
ODO_INLINE double pnp_sqrt(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = 0.5 * y;
    const double r = __builtin_fma(-g, h, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    const double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    return __builtin_isinf(x) ? x : g;
}

// EdgeSE3ProjectXYZOnlyPose / EdgeStereoSE3ProjectXYZOnlyPose::computeError (g2o types_six_dof_expmap)
ODO_INLINE void edge_err(const double Xc[3], const double ob[3], bool stereo, const PnPCam& c, double e[3]) {
    if (!stereo) {
        const double iz = pnp_inv(Xc[2]);
        double px = Xc[0] * iz, py = Xc[1] * iz;
        e[0] = ob[0] - (px * c.fx + c.cx);
        e[1] = ob[1] - (py * c.fy + c.cy);
        e[2] = 0;
    } else {
        const float invz = (float)pnp_inv(Xc[2]);
        const double iz = (double)invz;
        double r0 = Xc[0] * iz * c.fx + c.cx;
        double r1 = Xc[1] * iz * c.fy + c.cy;
        double r2 = r0 - c.bf * iz;
        e[0] = ob[0] - r0;
        e[1] = ob[1] - r1;
        e[2] = ob[2] - r2;
    }
}
ODO_INLINE double chi2_of(const double e[3], double info, bool stereo) {
    if (!stereo) return e[0] * (info * e[0]) + e[1] * (info * e[1]);
    return sum3d(e[0] * (info * e[0]), e[1] * (info * e[1]), e[2] * (info * e[2]));
}
ODO_INLINE void huber_rho(double delta, double chi, double rho[3]) {
    double dsqr = delta * delta;
    if (chi <= dsqr) {
        rho[0] = chi;
        rho[1] = 1.;
        rho[2] = 0.;
    } else {
        double sq = pnp_sqrt(chi);
        rho[0] = 2 * sq * delta - dsqr;
        rho[1] = __builtin_isinf(sq) ? 0.0 : delta * pnp_inv(sq);  // delta / inf = 0, as the IEEE quotient
        rho[2] = -0.5 * rho[1] / chi;
    }
}

// One wave per frame pair. Every lane runs the (tiny) serial parts — LDLT,
// exp map, LM bookkeeping — redundantly on identical values, so no lane ever
// waits for a broadcast; per-edge work is split over lanes and combined with a
// fixed xor-butterfly (deterministic).
#ifndef PNP_NW
#define PNP_NW 4  // waves per pair
#endif
#define PNP_NT (64 * PNP_NW)
#ifndef PNP_K
// Levenberg trials evaluated per edge pass (one per 16-lane group of wave 0).
// Round 6: 2 — with the pair chain off the step's critical path, the
// speculative trials' chi2 passes are issue slots the extraction kernels
// beside PnP lose: 154.7-155.0 vs 153.7-154.3 k frames/s (4) and
// 152.3-153.9 k (1); PnP alone 0.386-0.397 vs 0.380-0.385 ms (4), 0.44 (1);
// hard workload unchanged (profiles/r06_w, r06_wh)
#define PNP_K 2
#endif
static_assert(PNP_K <= 4, "the trial solves run on the four 16-lane groups of one wave");

// Sum of NV per-lane doubles over the workgroup, the result in every lane.
// Per wave a transposing xor-butterfly: at offset o the lane pair splits the
// (padded) vector, each lane keeping one half and adding its partner's copy
// of that half, so NP values need NP/2 + NP/4 + ... + 1 shuffles instead of
// 6 per value; after log2(NP) halvings lane l holds value (l >> (6-log2 NP)),
// reduced over the remaining offsets. Waves are then added in index order.
// The tree is fixed, so the sum is deterministic.
template <int NV>
struct Pow2Pad {
    static constexpr int v = NV <= 1 ? 1 : NV <= 2 ? 2 : NV <= 4 ? 4 : NV <= 8 ? 8 : NV <= 16 ? 16 : 32;
    static constexpr int lg = NV <= 1 ? 0 : NV <= 2 ? 1 : NV <= 4 ? 2 : NV <= 8 ? 3 : NV <= 16 ? 4 : 5;
};
template <int O>
ODO_INLINE double xor_partner(double v) {
    return __shfl_xor(v, O);
}
template <int NP, int O>
ODO_INLINE void halving_level(double (&w)[NP], int lane) {
    constexpr int n = NP * O / 32, h = n >> 1;  // values held before this level
    const bool hi = (lane & O) != 0;
#pragma unroll
    for (int i = 0; i < h; i++) {
        const double send = hi ? w[i] : w[h + i];
        const double keep = hi ? w[h + i] : w[i];
        w[i] = keep + xor_partner<O>(send);
    }
}
template <int NV>
ODO_INLINE double wave_sum_transposed(const double (&v)[NV]) {
    constexpr int NP = Pow2Pad<NV>::v, LG = Pow2Pad<NV>::lg;
    static_assert(NP <= 32, "at most 32 values");
    const int lane = threadIdx.x & 63;
    double w[NP];
#pragma unroll
    for (int k = 0; k < NP; k++) w[k] = k < NV ? v[k] : 0.0;
    // halving levels: at offset O the lane pair splits the vector (the lane
    // with bit O clear keeps the low half)
    if constexpr (LG > 0) halving_level<NP, 32>(w, lane);
    if constexpr (LG > 1) halving_level<NP, 16>(w, lane);
    if constexpr (LG > 2) halving_level<NP, 8>(w, lane);
    if constexpr (LG > 3) halving_level<NP, 4>(w, lane);
    if constexpr (LG > 4) halving_level<NP, 2>(w, lane);
    double x = w[0];
    // the remaining offsets: every lane adds its partner's total
    if constexpr (LG < 1) x += xor_partner<32>(x);
    if constexpr (LG < 2) x += xor_partner<16>(x);
    if constexpr (LG < 3) x += xor_partner<8>(x);
    if constexpr (LG < 4) x += xor_partner<4>(x);
    if constexpr (LG < 5) x += xor_partner<2>(x);
    x += xor_partner<1>(x);
    return x;  // total of value (lane >> (6 - LG)) over the wave
}
#define PNP_RED_WORDS (PNP_NW * 28)
template <int NV>
ODO_INLINE void wg_sum(double (&v)[NV], double* red) {
    constexpr int LG = Pow2Pad<NV>::lg;
    const double x = wave_sum_transposed(v);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int j = lane >> (6 - LG);
    double* r = red;
    if ((lane & ((1 << (6 - LG)) - 1)) == 0 && j < NV) r[wave * NV + j] = x;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; k++) {
        double a = r[k];
        for (int w = 1; w < PNP_NW; w++) a += r[w * NV + k];
        v[k] = a;
    }
    __syncthreads();
}

// computeActiveErrors + activeRobustChi2 + buildSystem contribution of one edge
// at pose T into acc (H upper triangle row-major 0..20, b 21..26, robust chi 27)
ODO_INLINE void edge_build(const SE3M& T, const double Xw[3], const double ob[3], double info, uint8_t fl,
                           const PnPCam& cam, double dMono, double dStereo, double (&acc)[28]) {
    const bool st = fl & PE_STEREO;
    double Xc[3], e[3];
    se3m_map(T, Xw, Xc);
    edge_err(Xc, ob, st, cam, e);
    const double c2 = chi2_of(e, info, st);
    double rho[3] = {c2, 1.0, 0.0};
    if (fl & PE_ROBUST) huber_rho(st ? dStereo : dMono, c2, rho);
    acc[27] += rho[0];
    const double x = Xc[0], y = Xc[1], invz = pnp_inv(Xc[2]), invz_2 = invz * invz;
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
    // mono edges: third row zero, so its terms add exactly +0
    J[2][0] = st ? J[0][0] - cam.bf * y * invz_2 : 0.0;
    J[2][1] = st ? J[0][1] + cam.bf * x * invz_2 : 0.0;
    J[2][2] = st ? J[0][2] : 0.0;
    J[2][3] = st ? J[0][3] : 0.0;
    J[2][4] = 0;
    J[2][5] = st ? J[0][5] - cam.bf * invz_2 : 0.0;
    const double r1 = rho[1];
    const double wo = r1 * info;
    // J[0][4], J[1][3] and J[2][4] are exact zeros by construction: their
    // terms (0 * x * y and x * y * 0, added to the running sum) are skipped —
    // the same sums for finite Jacobians, 21 of the 81 terms fewer (H[3][4]
    // has no term at all)
    constexpr bool Z[3][6] = {{false, false, false, false, true, false},
                              {false, false, false, true, false, false},
                              {false, false, false, false, true, false}};
    int h = 0;
#pragma unroll
    for (int a = 0; a < 6; a++) {
        double sb = 0;
#pragma unroll
        for (int kk = 0; kk < 3; kk++)
            if (!Z[kk][a]) sb += J[kk][a] * (info * e[kk]);
        acc[21 + a] -= r1 * sb;
#pragma unroll
        for (int cc = a; cc < 6; cc++) {
#pragma unroll
            for (int kk = 0; kk < 3; kk++)
                if (!Z[kk][a] && !Z[kk][cc]) acc[h] += J[kk][a] * wo * J[kk][cc];
            h++;
        }
    }
}

// One workgroup (4 waves) per pair. OptimizationAlgorithmLevenberg's trial
// loop (reject -> lambda *= ni, ni *= 2) is run speculatively: the next
// PNP_K lambdas of a rejection run are known in advance, so waves 0..K-1 each
// solve one candidate step, a single edge pass sums chi2 for all candidates,
// and the sequential accept/reject control flow is replayed over the results
// (same decisions, same state as the one-trial-at-a-time loop).
#ifndef PNP_WAVES_PER_EU
#define PNP_WAVES_PER_EU 1  // occupancy floor (launch bounds); 1 = compiler's choice
#endif
// LE (edges in LDS): after the edges are created in the pair's HBM scratch,
// their read-mostly fields (Xw, obs, info, flags: 29 B per edge) are copied
// into the workgroup's LDS, and every pass of the ~40 Levenberg iterations
// reads them there instead of from L2 (a pass walks ~2-3 edges per thread,
// each a dependent L2 round trip before). chi4 and idx stay in HBM. The host
// picks LE when kp_cap edges fit (pnp_lds_bytes).
template <bool LE>
__global__ void __launch_bounds__(PNP_NT, PNP_WAVES_PER_EU) k_pnp(const int32_t* __restrict__ f2_src, const float* __restrict__ xyz,
                                            const float* __restrict__ kun, const float* __restrict__ ur,
                                            const int* __restrict__ nkp, int kp_cap, int slot0, FrameCalib cal,
                                            const float* __restrict__ T12, const int* __restrict__ pair_valid,
                                            const int* __restrict__ n_matches, int min_matches, void* edges_g,
                                            odo_pair_result* __restrict__ res, uint8_t* __restrict__ inlier_mask,
                                            const int* __restrict__ sel, int sel_val) {
#ifndef ODO_PNP_PRIO
// round 6: 0 — PnP ends ~80 us before the extraction step does and runs beside
// finalize, which gets the issue slots (with ODO_WAVE_PRIO 1: profiles/r06_h;
// round 5, PnP on the step's critical path: 3, profiles/r05_pr)
#define ODO_PNP_PRIO 0
#endif
    __builtin_amdgcn_s_setprio(ODO_PNP_PRIO);
    const int p = blockIdx.x;
    if (sel && sel[p] != sel_val) return;  // pair handled by the other PnP launch
    const int lane = threadIdx.x;  // thread index within the workgroup
    const int wlane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ double red[PNP_RED_WORDS];
    __shared__ double s_acc[28];  // reduced H (upper, row-major), b, chi of the iteration
    __shared__ double s_sc[PNP_K];  // the trials' gain denominators (scale)
    __shared__ double s_M[PNP_K][12];  // the candidates as rotation matrix + translation
    __shared__ int s_ok[PNP_K];
    __shared__ int s_ne[PNP_NW];
    odo_pair_result* R = res + p;
    const int s1 = slot0 + p, s2 = slot0 + p + 1;
    const int n2 = nkp[s2];
    uint8_t* mask = inlier_mask + (size_t)p * kp_cap;
    for (int i = lane; i < n2; i += PNP_NT) mask[i] = 0;
    const float* T0 = T12 + (size_t)p * 16;
    if (lane < 16) R->Tcw[lane] = T0[lane];
    if (lane == 0) R->pnp_inliers = 0;
    if (!pair_valid[p] || n_matches[p] < min_matches) return;
    // ---- edges: F2 keypoints holding a landmark, index order (pnpsolver.cpp:57-135)
    const int32_t* src = f2_src + (size_t)p * kp_cap;
    const float* X1 = xyz + (size_t)s1 * kp_cap * 3;
    const float* K2 = kun + (size_t)s2 * kp_cap * 2;
    const float* U2 = ur + (size_t)s2 * kp_cap;
    PEdgeSoA E = pedge_view(edges_g, kp_cap, p);
    int ne = 0;
    for (int c0 = 0; c0 < n2; c0 += PNP_NT) {
        const int i = c0 + lane;
        const bool has = i < n2 && src[i] >= 0;
        const uint64_t bal = __ballot(has);
        if (wlane == 0) s_ne[wave] = __popcll(bal);
        __syncthreads();
        int before = 0, tot = 0;
        for (int w = 0; w < PNP_NW; w++) {
            if (w < wave) before += s_ne[w];
            tot += s_ne[w];
        }
        __syncthreads();
        if (has) {
            const int k = ne + before + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
            const int s = src[i];
            const float zw = X1[3 * s + 2];
            E.X[3 * k] = X1[3 * s];
            E.X[3 * k + 1] = X1[3 * s + 1];
            E.X[3 * k + 2] = zw;
            const float urv = U2[i];
            const bool st = !(urv < 0);
            E.obs[3 * k] = K2[2 * i];
            E.obs[3 * k + 1] = K2[2 * i + 1];
            E.obs[3 * k + 2] = st ? urv : 0.f;
            E.info[k] = 1.0f / (zw * zw);
            E.flags[k] = (uint8_t)((st ? PE_STEREO : 0) | PE_ROBUST);
            E.idx[k] = i;
        }
        ne += tot;
    }
    __syncthreads();
    if (ne < 3) {
        for (int k = lane; k < ne; k += PNP_NT) mask[E.idx[k]] = 1;  // SetInlier at edge creation
        return;
    }
    // the chi2 each chi pass stores per edge and trial slot, read back by the
    // classification only as (float)chi2: with LE the float
    // itself, in LDS (no global stores in the passes: every barrier would
    // wait for them)
    float* sC = nullptr;
    if (LE) {
        extern __shared__ __attribute__((aligned(16))) float s_edge[];
        float* sX = s_edge;             // 3 * kp_cap
        float* sO = sX + 3 * kp_cap;    // 3 * kp_cap
        float* sI = sO + 3 * kp_cap;    // kp_cap
        uint8_t* sF = reinterpret_cast<uint8_t*>(sI + kp_cap);  // kp_cap
        sC = reinterpret_cast<float*>(sF + kp_cap);  // 4 * kp_cap (kp_cap % 64 == 0)
        for (int k = lane; k < 3 * ne; k += PNP_NT) {
            sX[k] = E.X[k];
            sO[k] = E.obs[k];
        }
        for (int k = lane; k < ne; k += PNP_NT) {
            sI[k] = E.info[k];
            sF[k] = E.flags[k];
        }
        __syncthreads();
        E.X = sX;
        E.obs = sO;
        E.info = sI;
        E.flags = sF;
    }
    const PnPCam cam{(double)cal.fx, (double)cal.fy, (double)cal.cx, (double)cal.cy, (double)cal.mbf};
    const double dMono = (double)(float)sqrt(5.991), dStereo = (double)(float)sqrt(7.815);  // pnpsolver.cpp:51-52
    SE3 T0s;
    {
        double R0[3][3], t0[3];
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) R0[i][j] = (double)T0[i * 4 + j];
            t0[i] = (double)T0[i * 4 + 3];
        }
        T0s.q = quat_from_R(R0);
        for (int i = 0; i < 3; i++) T0s.t[i] = t0[i];
        normalize_rot(T0s);
    }
    const float chi2Mono = 5.991f, chi2Stereo = 7.815f;
    int nBad = 0;
    const SE3M T0m = se3_mat(T0s);
    SE3M T = T0m;
#ifdef ODO_PNP_PROFILE
    // -DODO_PNP_PROFILE: phase times (10 ns ticks) of one pair via printf
    uint64_t tb = 0, tsol = 0, tchi = 0, tcls = 0, t0 = 0, tall = wall_clock64(), tldlt = 0, texp = 0, tbl = 0, tcl = 0;
    int nit = 0, ntr = 0;
#define PP_T0() t0 = wall_clock64()
#define PP_ACC(x) x += wall_clock64() - t0
#else
#define PP_T0()
#define PP_ACC(x)
#endif
    int last_slot = 0;  // trial slot whose errors the edges store (last computeActiveErrors)
    for (int it = 0; it < 4; it++) {
        T = T0m;  // vSE3->setEstimate(pFrame->GetPose()) (pnpsolver.cpp:150)
        double lambda = 0, ni = 2;
        for (int iter = 0; iter < 10; iter++) {
            // computeActiveErrors + activeRobustChi2 + buildSystem at T
            PP_T0();
            double acc[28];
#pragma unroll
            for (int k = 0; k < 28; k++) acc[k] = 0;
            {
                const SE3M& Tm = T;
                // the next edge's fields are loaded before this one is built
                if (lane < ne) {
                    EdgeIn cur = load_edge(E, lane);
                    for (int k = lane; k < ne; k += PNP_NT) {
                        const EdgeIn nx = load_edge(E, min(k + PNP_NT, ne - 1));
                        if (!(cur.fl & PE_OUT)) {
                            const double Xw[3] = {cur.X[0], cur.X[1], cur.X[2]};
                            const double ob[3] = {cur.ob[0], cur.ob[1], cur.ob[2]};
                            edge_build(Tm, Xw, ob, (double)cur.info, cur.fl, cam, dMono, dStereo, acc);
                        }
                        cur = nx;
                    }
                }
            }
#ifdef ODO_PNP_PROFILE
            tbl += wall_clock64() - t0;  // the edge trips, without the sum
#endif
            wg_sum<28>(acc, red);
            PP_ACC(tb);
#ifdef ODO_PNP_PROFILE
            nit++;
#endif
            if (lane == 0)
#pragma unroll
                for (int k = 0; k < 28; k++) s_acc[k] = acc[k];
            double curChi = acc[27];
            if (iter == 0) {
                // diagonal of the packed upper triangle: 0, 6, 11, 15, 18, 20
                double mx = 0;
                mx = fmax(fabs(acc[0]), mx);
                mx = fmax(fabs(acc[6]), mx);
                mx = fmax(fabs(acc[11]), mx);
                mx = fmax(fabs(acc[15]), mx);
                mx = fmax(fabs(acc[18]), mx);
                mx = fmax(fabs(acc[20]), mx);
                lambda = 1e-5 * mx;
                ni = 2;
            }
            // s_acc is written by lane 0 and read by wave 0 only (the trial
            // solves): a wave-level fence instead of a workgroup barrier
            if (wave == 0) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            // ---- OptimizationAlgorithmLevenberg::solve trial loop, PNP_K trials per pass
            double rho = 0;
            int qmax = 0;
            bool trials_done = false;
            while (!trials_done) {
                const int K = min(PNP_K, 10 - qmax);
                // lambdas of the next K trials if every one of them is rejected
                double lam[PNP_K], nis[PNP_K];
                {
                    double l = lambda, n_ = ni;
#pragma unroll
                    for (int k = 0; k < PNP_K; k++) {
                        lam[k] = l;
                        nis[k] = n_;
                        l *= n_;
                        n_ *= 2;
                    }
                }
                PP_T0();
                // the K trial solves on wave 0's four 16-lane groups (group g =
                // trial g): the same per-lane arithmetic as one wave per trial,
                // a quarter of the issued FP64 instructions
                const int tg = wlane >> 4;
                if (wave == 0 && tg < K) {
                    double lw = lam[0];
#pragma unroll
                    for (int k = 1; k < PNP_K; k++)
                        if (tg == k) lw = lam[k];
                    double Hl[6][6], b[6];
                    {
                        int h = 0;
#pragma unroll
                        for (int a = 0; a < 6; a++)
#pragma unroll
                            for (int cc = a; cc < 6; cc++) {
                                Hl[a][cc] = s_acc[h];
                                Hl[cc][a] = s_acc[h];
                                h++;
                            }
#pragma unroll
                        for (int a = 0; a < 6; a++) b[a] = s_acc[21 + a];
                    }
                    for (int j = 0; j < 6; j++) Hl[j][j] += lw;
                    double x[6] = {0, 0, 0, 0, 0, 0};
#ifdef ODO_PNP_PROFILE
                    const uint64_t ts0 = wall_clock64();
#endif
                    const bool ok2 = ldlt_solve6_spd(Hl, b, x);
#ifdef ODO_PNP_PROFILE
                    const uint64_t ts1 = wall_clock64();
#endif
                    const SE3M Tk = se3m_exp_mul(x, T);
#ifdef ODO_PNP_PROFILE
                    if (wlane == 0) {
                        tldlt += ts1 - ts0;
                        texp += wall_clock64() - ts1 + (Tk.t[0] == 12345.678 ? 1 : 0);
                    }
#endif
                    double scale = 0;
                    for (int j = 0; j < 6; j++) scale += x[j] * (lw * x[j] + b[j]);
                    scale += 1e-3;
                    if ((wlane & 15) == 0) {
                        s_sc[tg] = scale;
                        s_ok[tg] = ok2 ? 1 : 0;
#pragma unroll
                        for (int q = 0; q < 9; q++) s_M[tg][q] = Tk.R[q];
#pragma unroll
                        for (int q = 0; q < 3; q++) s_M[tg][9 + q] = Tk.t[q];
                    }
                }
                __syncthreads();
                double sc[PNP_K];
                bool okc[PNP_K];
#pragma unroll
                for (int k = 0; k < PNP_K; k++) {
                    sc[k] = s_sc[k];
                    okc[k] = s_ok[k] != 0;
                }
                PP_ACC(tsol);
                PP_T0();
                // computeActiveErrors + activeRobustChi2 at every candidate
                double chi[PNP_K];
#pragma unroll
                for (int k = 0; k < PNP_K; k++) chi[k] = 0;
                // all PNP_K candidates of an edge as independent chains, phase
                // by phase (maps, divisions, errors, chi2, Huber) with no
                // branch between them, so their latencies overlap; the same
                // expressions as edge_err + chi2_of + huber_rho (computeError,
                // chi2, RobustKernelHuber::robustify; candidates >= K are computed
                // from stale slots and dropped: their chi2 slots are never read)
                EdgeIn cur = load_edge(E, min(lane, ne - 1));
                for (int e = lane; e < ne; e += PNP_NT) {
                    const EdgeIn ed = cur;
                    cur = load_edge(E, min(e + PNP_NT, ne - 1));
                    const uint8_t fl = ed.fl;
                    if (fl & PE_OUT) continue;
                    const double Xw[3] = {ed.X[0], ed.X[1], ed.X[2]};
                    const double ob[3] = {ed.ob[0], ed.ob[1], ed.ob[2]};
                    const double info = ed.info;
                    const bool st = fl & PE_STEREO;
                    double c2[PNP_K];
#pragma unroll
                    for (int k = 0; k < PNP_K; k++) {
                        SE3M Mk;
#pragma unroll
                        for (int q = 0; q < 9; q++) Mk.R[q] = s_M[k][q];
#pragma unroll
                        for (int q = 0; q < 3; q++) Mk.t[q] = s_M[k][9 + q];
                        double Xc[3];
                        se3m_map(Mk, Xw, Xc);
                        const double d = pnp_inv(Xc[2]);
                        const double iz = st ? (double)(float)d : d;
                        const double r0 = Xc[0] * iz * cam.fx + cam.cx;
                        const double r1 = Xc[1] * iz * cam.fy + cam.cy;
                        const double e0 = ob[0] - r0, e1 = ob[1] - r1;
                        const double e2 = st ? ob[2] - (r0 - cam.bf * iz) : 0.0;
                        c2[k] = sum3d(e0 * (info * e0), e1 * (info * e1), e2 * (info * e2));
                    }
                    const double delta = st ? dStereo : dMono, dsqr = delta * delta;
                    bool huber = false;
#pragma unroll
                    for (int k = 0; k < PNP_K; k++) huber |= c2[k] > dsqr;
                    huber = huber && (fl & PE_ROBUST);
                    double sq[PNP_K];
#pragma unroll
                    for (int k = 0; k < PNP_K; k++) sq[k] = 0.0;
                    if (huber) {
#pragma unroll
                        for (int k = 0; k < PNP_K; k++) sq[k] = pnp_sqrt(c2[k]);
                    }
#pragma unroll
                    for (int k = 0; k < PNP_K; k++) {
                        const double r = (huber && c2[k] > dsqr) ? 2 * sq[k] * delta - dsqr : c2[k];
                        chi[k] += r;
                        if (LE) sC[4 * e + k] = (float)c2[k];
                        else if (k < K) E.chi4[4 * e + k] = c2[k];
                    }
                }
#ifdef ODO_PNP_PROFILE
                tcl += wall_clock64() - t0;
#endif
                wg_sum<PNP_K>(chi, red);
                PP_ACC(tchi);
                // replay the trials in order
#pragma unroll
                for (int k = 0; k < PNP_K; k++) {
                    if (k >= K || trials_done) break;
#ifdef ODO_PNP_PROFILE
                    ntr++;
#endif
                    double tempChi = chi[k];
                    if (!okc[k]) tempChi = 1.7976931348623157e308;
                    rho = curChi - tempChi;
                    rho /= sc[k];
                    last_slot = k;
                    qmax++;
                    if (rho > 0 && isfinite(tempChi)) {
                        const double tr = 2 * rho - 1;
                        double alpha = 1. - tr * tr * tr;
                        alpha = fmin(alpha, 2. / 3.);
                        const double sf = fmax(1. / 3., alpha);
                        lambda = lam[k] * sf;
                        ni = 2;
                        curChi = tempChi;
                        // the accepted candidate's matrix (s_M is not written
                        // again before the next trial solves)
#pragma unroll
                        for (int q = 0; q < 9; q++) T.R[q] = s_M[k][q];
#pragma unroll
                        for (int q = 0; q < 3; q++) T.t[q] = s_M[k][9 + q];
                        trials_done = true;
                    } else {
                        lambda = lam[k] * nis[k];  // T stays at the backup
                        ni = nis[k] * 2;
                        if (!(rho < 0 && qmax < 10)) trials_done = true;
                    }
                }
            }
            if (qmax == 10 || rho == 0) break;
        }
        // ---- classification (pnpsolver.cpp:157-201)
        PP_T0();
        int bad = 0;
        {
            const SE3M& Tm = T;
            // reclassify edge k (flags in / out); the stored chi2 of the last
            // computeActiveErrors, recomputed at T for the edges that were out
            auto classify = [&](int k, uint32_t fl, const double Xw[3], const double ob[3], double info) {
                const bool st = fl & PE_STEREO;
                float chi2;
                if (fl & PE_OUT) {  // IsOutlier: e->computeError() at the current estimate
                    double Xc[3], e[3];
                    se3m_map(Tm, Xw, Xc);
                    edge_err(Xc, ob, st, cam, e);
                    const double c2 = chi2_of(e, info, st);
                    // (never read back: an edge out during the next round is
                    // recomputed here, one in is rewritten by its chi passes)
                    if (!LE) E.chi4[4 * k + last_slot] = c2;
                    chi2 = (float)c2;
                } else {
                    chi2 = LE ? sC[4 * k + last_slot] : (float)E.chi4[4 * k + last_slot];
                }
                if (chi2 > (st ? chi2Stereo : chi2Mono)) {
                    fl |= PE_OUT;
                    bad++;
                } else {
                    fl &= ~PE_OUT;
                }
                if (it == 2) fl &= ~PE_ROBUST;
                E.flags[k] = (uint8_t)fl;
                return fl;
            };
            for (int k = lane; k < ne; k += PNP_NT) {
                const double Xw[3] = {E.X[3 * k], E.X[3 * k + 1], E.X[3 * k + 2]};
                const double ob[3] = {E.obs[3 * k], E.obs[3 * k + 1], E.obs[3 * k + 2]};
                classify(k, E.flags[k], Xw, ob, (double)E.info[k]);
            }
        }
        double bd[1] = {(double)bad};
        wg_sum<1>(bd, red);
        nBad = (int)bd[0];
        PP_ACC(tcls);
        if (ne < 10) break;
    }
#ifdef ODO_PNP_PROFILE
#ifndef PNP_PROF_PAIRS
#define PNP_PROF_PAIRS 3
#endif
    if (lane == 0 && p < PNP_PROF_PAIRS)
        printf("PNP p %d ne %d iters %d trials %d: build %lu (trips %lu) solve %lu (ldlt %lu exp+mul %lu) chi %lu (trips %lu) classify %lu total %lu (x10ns)\n",
               p, ne, nit, ntr, tb, tbl, tsol, tldlt, texp, tchi, tcl, tcls, wall_clock64() - tall);
#endif
    if (lane == 0) {
        double Rm[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) Rm[i][j] = T.R[3 * i + j];
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) R->Tcw[i * 4 + j] = (float)Rm[i][j];
            R->Tcw[i * 4 + 3] = (float)T.t[i];
        }
        R->Tcw[12] = R->Tcw[13] = R->Tcw[14] = 0.f;
        R->Tcw[15] = 1.f;
        R->pnp_inliers = ne - nBad;
    }
    for (int k = lane; k < ne; k += PNP_NT) mask[E.idx[k]] = (E.flags[k] & PE_OUT) ? 0 : 1;
}



}  // namespace odo

namespace odo {
size_t pnp_edge_bytes() { return PE_BYTES; }
// dynamic LDS of k_pnp<true>: 29 B per edge slot (kp_cap), 0 = edges stay in
// HBM (k_pnp<false>). ODO_PNP_LDS (tuning builds) = 0 disables it for A/B.
#ifndef PNP_LDS_MAX
#define PNP_LDS_MAX (96 * 1024)
#endif
static size_t pnp_lds_bytes(int kp_cap) {
    static const bool off = [] {
        const char* e = odo_knob("ODO_PNP_LDS");
        return e && e[0] == '0';
    }();
    const size_t b = ((size_t)kp_cap * 45 + 15) & ~(size_t)15;
    return (!off && b <= PNP_LDS_MAX) ? b : 0;
}
// The 4-wave workgroup per pair (k_pnp). Measured and retired: one wave per
// pair (round 2: PnP 1.66 vs 0.72 ms alone per 256 pairs, step 2.61 vs
// 2.50 ms, one frame 0.65 vs 0.49 ms — the solver is latency-bound per pair,
// and the freed SIMDs do not buy back the 4x longer edge passes).
void launch_pnp(hipStream_t st, const int32_t* f2_src, const float* xyz, const float* kun, const float* ur,
                const int* nkp, int kp_cap, int slot0, FrameCalib cal, const float* T12, const int* pair_valid,
                const int* n_matches, int min_matches, void* edges, odo_pair_result* res, uint8_t* inlier_mask,
                int npairs, const int* sel, int sel_val) {
    const size_t lds = pnp_lds_bytes(kp_cap);
    if (lds) {
        static bool attr = false;
        if (!attr) {
            (void)hipFuncSetAttribute((const void*)k_pnp<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)PNP_LDS_MAX);
            attr = true;
        }
        hipLaunchKernelGGL(k_pnp<true>, dim3(npairs), dim3(PNP_NT), lds, st, f2_src, xyz, kun, ur, nkp, kp_cap, slot0,
                           cal, T12, pair_valid, n_matches, min_matches, edges, res, inlier_mask, sel, sel_val);
        return;
    }
    hipLaunchKernelGGL(k_pnp<false>, dim3(npairs), dim3(PNP_NT), 0, st, f2_src, xyz, kun, ur, nkp, kp_cap, slot0, cal,
                       T12, pair_valid, n_matches, min_matches, edges, res, inlier_mask, sel, sel_val);
}
}  // namespace odo

// fixed-order block reduction (4 waves) used by the Kabsch kernel
namespace odo {
template <int NV>
ODO_INLINE void block_reduce(double (&v)[NV], double* red /* 4*NV */) {
#pragma unroll
    for (int k = 0; k < NV; k++) v[k] = wave_sum(v[k]);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __syncthreads();
    if (lane == 0)
        for (int k = 0; k < NV; k++) red[wave * NV + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; k++) v[k] = ((red[k] + red[NV + k]) + red[2 * NV + k]) + red[3 * NV + k];
    __syncthreads();
}
}  // namespace odo

// Kabsch is not part of the PnP measurements that paid for contraction: back to
// the library's -ffp-contract=off from here on
#pragma clang fp contract(off)

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
