// GeneralizedICP::Compute(source, target, guess) (Odometry/generalizedicp.cpp:
// 30-39, 65-89; the ADAPTIVE_RICP fallback of odometry.cpp:46-78; SURVEY §8(f)
// rank 4): pcl::GeneralizedIterativeClosestPoint<PointXYZ, PointXYZ> on the GPU.
//   k_gicp_cov  one lane per point: the 20 nearest points of its own cloud
//               (brute force, float squared distances, ties to the lower
//               index), mean / covariance in double, eigenvalues replaced by
//               (1, 1, 1e-3) (computeCovariances);
//   k_gicp      one 4-wave workgroup runs computeTransformation: per ICP iteration the
//               nearest target point of every transformed source point
//               (lane-strided brute force), the Mahalanobis matrices
//               (R C1 R^T + C2)^-1 of the pairs within the distance threshold,
//               compaction in source order (ballot prefix), then
//               estimateRigidTransformationBFGS: BFGS2 + Fletcher's line search
//               with identical control flow on all lanes, the cost and gradient
//               as thread-strided partial sums, the four waves' partials of a
//               lane position added in order, an xor butterfly read on lane 0
//               (oracle/gicp_ref.cpp's sum256), and the convergence test.
// The restatement, its pinned choices and the oracle are in oracle/gicp_ref.cpp
// (PCL is absent: parity with the library is unpinned).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>

#include "odo_internal.h"
#include "odo_linalg.h"

namespace odo {
namespace {

constexpr int GI_K = 20;
constexpr int GI_LANES = 64;
constexpr int GI_THREADS = 256;  // the ICP / BFGS workgroup: 4 waves share every pass over the correspondences
constexpr int GI_WAVES = GI_THREADS / GI_LANES;
constexpr int GI_NV = 12;        // values reduced per gradient evaluation
constexpr int GI_STAGE = 4096;   // clouds up to this many points are staged in LDS (48 KB)

__device__ __forceinline__ double s3(double a, double b, double c) { return a + (b + c); }

__device__ __forceinline__ float dist2f(const float* a, const float* b) {
    float r = 0.f, d;
    d = a[0] - b[0];
    r += d * d;
    d = a[1] - b[1];
    r += d * d;
    d = a[2] - b[2];
    r += d * d;
    return r;
}

// computeCovariances for point q of a cloud P of n points (LDS or global)
__device__ __forceinline__ void cov_point(const float* __restrict__ P, int n, int q, double eps,
                                          double* __restrict__ C) {
    // the sorted top 20 in registers: +inf padding stands for "fewer than 20
    // so far", a candidate is inserted after equal distances (ties to the lower
    // index, as the scan is in index order)
    float nd[GI_K];
    int nn[GI_K];
#pragma unroll
    for (int j = 0; j < GI_K; j++) {
        nd[j] = __builtin_inff();
        nn[j] = 0;
    }
    const float pq[3] = {P[3 * q], P[3 * q + 1], P[3 * q + 2]};
    for (int i = 0; i < n; i++) {
        const float pi[3] = {P[3 * i], P[3 * i + 1], P[3 * i + 2]};
        const float d = dist2f(pq, pi);
        if (!(d < nd[GI_K - 1])) continue;
#pragma unroll
        for (int j = GI_K - 1; j > 0; j--) {
            const bool up = d < nd[j - 1];
            const bool here = !up && d < nd[j];
            nd[j] = up ? nd[j - 1] : (here ? d : nd[j]);
            nn[j] = up ? nn[j - 1] : (here ? i : nn[j]);
        }
        if (d < nd[0]) {
            nd[0] = d;
            nn[0] = i;
        }
    }
    double mean[3] = {0, 0, 0}, cov[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < GI_K; j++) {
        const float* pt = P + 3 * nn[j];
        const float x = pt[0], y = pt[1], z = pt[2];
        mean[0] += x;
        mean[1] += y;
        mean[2] += z;
        cov[0] += x * x;
        cov[3] += y * x;
        cov[4] += y * y;
        cov[6] += z * x;
        cov[7] += z * y;
        cov[8] += z * z;
    }
#pragma unroll
    for (int a = 0; a < 3; a++) mean[a] /= (double)GI_K;
#pragma unroll
    for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = 0; b <= a; b++) {
            cov[a * 3 + b] /= (double)GI_K;
            cov[a * 3 + b] -= mean[a] * mean[b];
            cov[b * 3 + a] = cov[a * 3 + b];
        }
    double w[3], V[9];
    svdj<3, 3>(cov, w, nullptr, V);
    double out[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const double v = c == 2 ? eps : 1.;
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) out[a * 3 + b] += (v * V[a * 3 + c]) * V[b * 3 + c];
    }
#pragma unroll
    for (int k = 0; k < 9; k++) C[9 * q + k] = out[k];
}

// grid (point blocks, problems, 2): z = 0 the target clouds, z = 1 the sources
__global__ __launch_bounds__(64) void k_gicp_cov(const float* __restrict__ src, const int* __restrict__ soffs,
                                                 double* __restrict__ Cs, const float* __restrict__ tgt,
                                                 const int* __restrict__ toffs, double* __restrict__ Ct, double eps) {
    const int pb = blockIdx.y;
    const int* offs = blockIdx.z ? soffs : toffs;
    const int n = offs[pb + 1] - offs[pb];
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    // whole blocks leave together (the staging below needs every thread)
    if ((int)(blockIdx.x * blockDim.x) >= n || soffs[pb + 1] - soffs[pb] < 20 || toffs[pb + 1] - toffs[pb] < 20) return;
    const float* __restrict__ Pg = (blockIdx.z ? src : tgt) + 3 * (size_t)offs[pb];
    double* __restrict__ C = (blockIdx.z ? Cs : Ct) + 9 * (size_t)offs[pb];
    if (n <= GI_STAGE) {  // the whole cloud in LDS: the scan reads it with uniform addresses
        __shared__ float cst[3 * GI_STAGE];
        for (int i = threadIdx.x; i < 3 * n; i += blockDim.x) cst[i] = Pg[i];
        __syncthreads();
        if (q < n) cov_point(cst, n, q, eps, C);
    } else if (q < n) {
        cov_point(Pg, n, q, eps, C);
    }
}

__device__ void inv3(const double* m, double* r) {
#define M_(i, j) m[(i) * 3 + (j)]
#define COF(i, j) (M_(((i) + 1) % 3, ((j) + 1) % 3) * M_(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M_(((i) + 1) % 3, ((j) + 2) % 3) * M_(((i) + 2) % 3, ((j) + 1) % 3))
    const double c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
    const double det = s3(c0 * M_(0, 0), c1 * M_(1, 0), c2 * M_(2, 0));
    const double invdet = 1.0 / det;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) r[i * 3 + j] = COF(j, i) * invdet;
#undef COF
#undef M_
}

__device__ __forceinline__ void xform4f(const float* T, const float* p, float* o) {
#pragma unroll
    for (int i = 0; i < 3; i++) o[i] = ((T[4 * i] * p[0] + T[4 * i + 1] * p[1]) + T[4 * i + 2] * p[2]) + T[4 * i + 3];
}

// applyState on the identity base (AngleAxisf Z * Y * X via quaternions)
__device__ void apply_state(const double* x, float* T) {
    float q[3][4];
    const float a[3] = {(float)x[5], (float)x[4], (float)x[3]};
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float h = 0.5f * a[k];
        const float c = (float)cos((double)h), s = (float)sin((double)h);  // float trig via double (pinned)
        q[k][0] = c;
        q[k][1] = k == 2 ? s : 0.f;
        q[k][2] = k == 1 ? s : 0.f;
        q[k][3] = k == 0 ? s : 0.f;
    }
    auto mul = [](const float* A, const float* B, float* o) {
        o[0] = A[0] * B[0] - A[1] * B[1] - A[2] * B[2] - A[3] * B[3];
        o[1] = A[0] * B[1] + A[1] * B[0] + A[2] * B[3] - A[3] * B[2];
        o[2] = A[0] * B[2] + A[2] * B[0] + A[3] * B[1] - A[1] * B[3];
        o[3] = A[0] * B[3] + A[3] * B[0] + A[1] * B[2] - A[2] * B[1];
    };
    float zy[4], r[4];
    mul(q[0], q[1], zy);
    mul(zy, q[2], r);
    const float w = r[0], qx = r[1], qy = r[2], qz = r[3];
    const float tx = 2.f * qx, ty = 2.f * qy, tz = 2.f * qz;
    const float twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * qx, txy = ty * qx, txz = tz * qx;
    const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    const float R[9] = {1.f - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1.f - (txx + tzz),
                        tyz - twx,         txz - twy, tyz + twx, 1.f - (txx + tyy)};
#pragma unroll
    for (int i = 0; i < 3; i++) {
#pragma unroll
        for (int j = 0; j < 3; j++) T[4 * i + j] = R[3 * i + j];
        T[4 * i + 3] = 0.f + (float)x[i];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
}

// oracle/gicp_ref.cpp's sum256: thread t's partial over k = t, t + 256, ...;
// lane l of wave 0 adds the four waves' partials of position l in wave order,
// then an xor butterfly read on lane 0; the NV results are broadcast via LDS.
template <int NV>
__device__ void block_sum256(double* v, double (*red)[GI_THREADS], double* out) {
#pragma unroll
    for (int k = 0; k < NV; k++) red[k][threadIdx.x] = v[k];
    __syncthreads();
    if (threadIdx.x < GI_LANES) {
#pragma unroll
        for (int k = 0; k < NV; k++) {
            double z = ((red[k][threadIdx.x] + red[k][threadIdx.x + 64]) + red[k][threadIdx.x + 128]) +
                       red[k][threadIdx.x + 192];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) z += __shfl_xor(z, o, GI_LANES);
            if (threadIdx.x == 0) out[k] = z;
        }
    }
    __syncthreads();
}

struct GiProblem {
    const float* src;  // source after the guess
    const float* tgt;
    const int* is;
    const int* it;
    const double* M;
    int m;
    double (*red)[GI_THREADS];  // LDS [GI_NV][GI_THREADS]
    double* bc;                 // LDS [GI_NV]
};

__device__ double gi_cost(const GiProblem& P, const double* x) {
    float T[16];
    apply_state(x, T);
    double part = 0.0;
    for (int k = threadIdx.x; k < P.m; k += GI_THREADS) {
        const int si = P.is[k];
        const float ps[3] = {P.src[3 * si], P.src[3 * si + 1], P.src[3 * si + 2]};
        float pp[3];
        xform4f(T, ps, pp);
        const float* q = P.tgt + 3 * P.it[k];
        const double r[3] = {(double)(pp[0] - q[0]), (double)(pp[1] - q[1]), (double)(pp[2] - q[2])};
        const double* M = P.M + 9 * si;
        double t[3];
#pragma unroll
        for (int i = 0; i < 3; i++) t[i] = s3(M[3 * i] * r[0], M[3 * i + 1] * r[1], M[3 * i + 2] * r[2]);
        part += s3(r[0] * t[0], r[1] * t[1], r[2] * t[2]);
    }
    block_sum256<1>(&part, P.red, P.bc);
    return P.bc[0] / P.m;
}

__device__ void gi_grad(const GiProblem& P, const double* x, double* g) {
    float T[16];
    apply_state(x, T);
    double part[12];
#pragma unroll
    for (int i = 0; i < 12; i++) part[i] = 0.0;
    for (int k = threadIdx.x; k < P.m; k += GI_THREADS) {
        const int si = P.is[k];
        const float ps[3] = {P.src[3 * si], P.src[3 * si + 1], P.src[3 * si + 2]};
        float pp[3];
        xform4f(T, ps, pp);
        const float* q = P.tgt + 3 * P.it[k];
        const double r[3] = {(double)(pp[0] - q[0]), (double)(pp[1] - q[1]), (double)(pp[2] - q[2])};
        const double* M = P.M + 9 * si;
        double t[3];
#pragma unroll
        for (int i = 0; i < 3; i++) t[i] = s3(M[3 * i] * r[0], M[3 * i + 1] * r[1], M[3 * i + 2] * r[2]);
#pragma unroll
        for (int i = 0; i < 3; i++) part[i] += t[i];
#pragma unroll
        for (int a = 0; a < 3; a++)
#pragma unroll
            for (int b = 0; b < 3; b++) part[3 + 3 * a + b] += (double)ps[a] * t[b];
    }
    double Rm[9];
    block_sum256<GI_NV>(part, P.red, P.bc);
#pragma unroll
    for (int i = 0; i < 3; i++) g[i] = P.bc[i] * (2.0 / P.m);
#pragma unroll
    for (int i = 0; i < 9; i++) Rm[i] = P.bc[3 + i] * (2.0 / P.m);
    const double phi = x[3], theta = x[4], psi = x[5];
    const double cphi = cos(phi), sphi = sin(phi), ctheta = cos(theta), stheta = sin(theta), cpsi = cos(psi),
                 spsi = sin(psi);
    const double d[3][9] = {{0., sphi * spsi + cphi * cpsi * stheta, cphi * spsi - cpsi * sphi * stheta,
                             0., -cpsi * sphi + cphi * spsi * stheta, -cphi * cpsi - sphi * spsi * stheta,
                             0., cphi * ctheta, -ctheta * sphi},
                            {-cpsi * stheta, cpsi * ctheta * sphi, cphi * cpsi * ctheta,
                             -spsi * stheta, ctheta * sphi * spsi, cphi * ctheta * spsi,
                             -ctheta, -sphi * stheta, -cphi * stheta},
                            {-ctheta * spsi, -cphi * cpsi - sphi * spsi * stheta, cpsi * sphi - cphi * spsi * stheta,
                             cpsi * ctheta, -cphi * spsi + cpsi * sphi * stheta, sphi * spsi + cphi * cpsi * stheta,
                             0., 0., 0.}};
#pragma unroll
    for (int c = 0; c < 3; c++) {
        double r = 0.;
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) r += d[c][3 * j + i] * Rm[3 * i + j];
        g[3 + c] = r;
    }
}

enum { ST_NOT_STARTED = -2, ST_RUNNING = -1, ST_SUCCESS = 0, ST_NO_PROGRESS = 1 };

// bfgs.h on every lane of the wave (uniform control flow, wave-summed values)
struct GiBfgs {
    GiProblem P;
    double x0[6], p[6], g0[6], dx0[6], dg0[6], gradient[6];
    double f, fp0, g0norm, pnorm, delta_f;
    double x_alpha[6], g_alpha[6], f_alpha, df_alpha, f_key, g_key, df_key;

    __device__ static double dot6(const double* a, const double* b) {
        double s = 0;
#pragma unroll
        for (int i = 0; i < 6; i++) s += a[i] * b[i];
        return s;
    }
    __device__ static double norm6(const double* a) { return sqrt(dot6(a, a)); }
    __device__ void moveTo(double alpha) {
#pragma unroll
        for (int i = 0; i < 6; i++) x_alpha[i] = x0[i] + alpha * p[i];
    }
    __device__ double slope() { return dot6(g_alpha, p); }
    __device__ double applyF(double alpha) {
        if (alpha == f_key) return f_alpha;
        moveTo(alpha);
        f_alpha = gi_cost(P, x_alpha);
        f_key = alpha;
        return f_alpha;
    }
    __device__ double applyDF(double alpha) {
        if (alpha == df_key) return df_alpha;
        moveTo(alpha);
        if (alpha != g_key) {
            gi_grad(P, x_alpha, g_alpha);
            g_key = alpha;
        }
        df_alpha = slope();
        df_key = alpha;
        return df_alpha;
    }
    __device__ static double cubic(double c0, double c1, double c2, double c3, double z) {
        return c0 + z * (c1 + z * (c2 + z * c3));
    }
    __device__ static void checkExtremum(double c0, double c1, double c2, double c3, double x, double& xmin,
                                         double& fmin) {
        const double y = cubic(c0, c1, c2, c3, x);
        if (y < fmin) {
            xmin = x;
            fmin = y;
        }
    }
    __device__ static int solve_quadratic(double a, double b, double c, double* x0, double* x1) {
        if (a == 0) {
            if (b == 0) return 0;
            *x0 = -c / b;
            return 1;
        }
        const double disc = b * b - 4 * a * c;
        if (disc > 0) {
            if (b == 0) {
                const double r = sqrt(-c / a);
                *x0 = -r;
                *x1 = r;
            } else {
                const double sgnb = (b > 0 ? 1 : -1);
                const double temp = -0.5 * (b + sgnb * sqrt(disc));
                const double r1 = temp / a, r2 = c / temp;
                if (r1 < r2) {
                    *x0 = r1;
                    *x1 = r2;
                } else {
                    *x0 = r2;
                    *x1 = r1;
                }
            }
            return 2;
        } else if (disc == 0) {
            *x0 = -0.5 * b / a;
            *x1 = -0.5 * b / a;
            return 2;
        }
        return 0;
    }
    __device__ static double cubicInterp(double f0, double fp0, double f1, double fp1, double zl, double zh) {
        const double eta = 3 * (f1 - f0) - 2 * fp0 - fp1;
        const double xi = fp0 + fp1 - 2 * (f1 - f0);
        const double c0 = f0, c1 = fp0, c2 = eta, c3 = xi;
        double zmin = zl, fmin = cubic(c0, c1, c2, c3, zl);
        checkExtremum(c0, c1, c2, c3, zh, zmin, fmin);
        double z0 = 0, z1 = 0;
        const int n = solve_quadratic(3 * c3, 2 * c2, c1, &z0, &z1);
        if (n == 2) {
            if (z0 > zl && z0 < zh) checkExtremum(c0, c1, c2, c3, z0, zmin, fmin);
            if (z1 > zl && z1 < zh) checkExtremum(c0, c1, c2, c3, z1, zmin, fmin);
        } else if (n == 1) {
            if (z0 > zl && z0 < zh) checkExtremum(c0, c1, c2, c3, z0, zmin, fmin);
        }
        return zmin;
    }
    __device__ static double quadraticInterp(double f0, double fp0, double f1, double zl, double zh) {
        const double fl = f0 + zl * (fp0 + zl * (f1 - f0 - fp0));
        const double fh = f0 + zh * (fp0 + zh * (f1 - f0 - fp0));
        const double c = 2 * (f1 - f0 - fp0);
        double zmin = zl, fmin = fl;
        if (fh < fmin) {
            zmin = zh;
            fmin = fh;
        }
        if (c > 0) {
            const double z = -fp0 / c;
            if (z > zl && z < zh) {
                const double ff = f0 + z * (fp0 + z * (f1 - f0 - fp0));
                if (ff < fmin) {
                    zmin = z;
                    fmin = ff;
                }
            }
        }
        return zmin;
    }
    __device__ static double interpolate(double a, double fa, double fpa, double b, double fb, double fpb, double xmin,
                                         double xmax) {
        double zmin = (xmin - a) / (b - a), zmax = (xmax - a) / (b - a);
        if (zmin > zmax) {
            const double t = zmin;
            zmin = zmax;
            zmax = t;
        }
        double z;
        if (!isnan(fpb))  // order 3
            z = cubicInterp(fa, fpa * (b - a), fb, fpb * (b - a), zmin, zmax);
        else
            z = quadraticInterp(fa, fpa * (b - a), fb, zmin, zmax);
        return a + z * (b - a);
    }
    __device__ int lineSearch(double alpha1, double* alpha_new) {
        const double rho = 0.01, sigma = 0.01, tau1 = 9, tau2 = 0.05, tau3 = 0.5;
        double falpha, fpalpha, delta, alpha_next;
        double alpha = alpha1, alpha_prev = 0.0;
        int i = 0;
        const double f0 = applyF(0.0), fp0l = applyDF(0.0);
        double falpha_prev = f0, fpalpha_prev = fp0l;
        double a = 0.0, b = alpha, fa = f0, fb = 0.0, fpa = fp0l, fpb = 0.0;
        const double qnan = __builtin_nan("");
        while (i++ < 100) {
            falpha = applyF(alpha);
            if (falpha > f0 + alpha * rho * fp0l || falpha >= falpha_prev) {
                a = alpha_prev;
                fa = falpha_prev;
                fpa = fpalpha_prev;
                b = alpha;
                fb = falpha;
                fpb = qnan;
                break;
            }
            fpalpha = applyDF(alpha);
            if (fabs(fpalpha) <= -sigma * fp0l) {
                *alpha_new = alpha;
                return ST_SUCCESS;
            }
            if (fpalpha >= 0) {
                a = alpha;
                fa = falpha;
                fpa = fpalpha;
                b = alpha_prev;
                fb = falpha_prev;
                fpb = fpalpha_prev;
                break;
            }
            delta = alpha - alpha_prev;
            alpha_next = interpolate(alpha_prev, falpha_prev, fpalpha_prev, alpha, falpha, fpalpha, alpha + delta,
                                     alpha + tau1 * delta);
            alpha_prev = alpha;
            falpha_prev = falpha;
            fpalpha_prev = fpalpha;
            alpha = alpha_next;
        }
        while (i++ < 100) {
            delta = b - a;
            alpha = interpolate(a, fa, fpa, b, fb, fpb, a + tau2 * delta, b - tau3 * delta);
            falpha = applyF(alpha);
            if ((a - alpha) * fpa <= DBL_EPSILON) return ST_NO_PROGRESS;
            if (falpha > f0 + rho * alpha * fp0l || falpha >= fa) {
                b = alpha;
                fb = falpha;
                fpb = qnan;
            } else {
                fpalpha = applyDF(alpha);
                if (fabs(fpalpha) <= -sigma * fp0l) {
                    *alpha_new = alpha;
                    return ST_SUCCESS;
                }
                if (((b - a) >= 0 && fpalpha >= 0) || ((b - a) <= 0 && fpalpha <= 0)) {
                    b = a;
                    fb = fa;
                    fpb = fpa;
                    a = alpha;
                    fa = falpha;
                    fpa = fpalpha;
                } else {
                    a = alpha;
                    fa = falpha;
                    fpa = fpalpha;
                }
            }
        }
        return ST_SUCCESS;
    }
    __device__ void minimizeInit(const double* x) {
        delta_f = 0;
        f = gi_cost(P, x);
        gi_grad(P, x, gradient);
#pragma unroll
        for (int i = 0; i < 6; i++) {
            x0[i] = x[i];
            g0[i] = gradient[i];
        }
        g0norm = norm6(g0);
#pragma unroll
        for (int i = 0; i < 6; i++) p[i] = gradient[i] * (-1 / g0norm);
        pnorm = norm6(p);
        fp0 = -g0norm;
#pragma unroll
        for (int i = 0; i < 6; i++) {
            x_alpha[i] = x0[i];
            g_alpha[i] = g0[i];
        }
        f_alpha = f;
        f_key = 0;
        g_key = 0;
        df_alpha = slope();
        df_key = 0;
    }
    __device__ int minimizeOneStep(double* x) {
        double alpha = 0.0, alpha1;
        const double f0 = f;
        if (pnorm == 0.0 || g0norm == 0.0 || fp0 == 0) return ST_NOT_STARTED;
        if (delta_f < 0) {
            const double del = fmax(-delta_f, 10 * DBL_EPSILON * fabs(f0));
            alpha1 = fmin(1.0, 2.0 * del / (-fp0));
        } else {
            alpha1 = 1.0;  // |step_size|
        }
        const int st = lineSearch(alpha1, &alpha);
        if (st != ST_SUCCESS) return st;
        applyF(alpha);  // updatePosition
        applyDF(alpha);
#pragma unroll
        for (int i = 0; i < 6; i++) {
            x[i] = x_alpha[i];
            gradient[i] = g_alpha[i];
        }
        f = f_alpha;
        delta_f = f - f0;
#pragma unroll
        for (int i = 0; i < 6; i++) {
            dx0[i] = x[i] - x0[i];
            dg0[i] = gradient[i] - g0[i];
        }
        const double dxg = dot6(dx0, gradient), dgg = dot6(dg0, gradient), dxdg = dot6(dx0, dg0);
        const double dgnorm = norm6(dg0);
        double A, B;
        if (dxdg != 0) {
            B = dxg / dxdg;
            A = -(1.0 + dgnorm * dgnorm / dxdg) * B + dgg / dxdg;
        } else {
            B = 0;
            A = 0;
        }
#pragma unroll
        for (int i = 0; i < 6; i++) p[i] = (gradient[i] + (-A) * dx0[i]) + (-B) * dg0[i];
#pragma unroll
        for (int i = 0; i < 6; i++) {
            g0[i] = gradient[i];
            x0[i] = x[i];
        }
        g0norm = norm6(g0);
        pnorm = norm6(p);
        const double dir = (dot6(p, gradient) >= 0.0) ? -1.0 : +1.0;
#pragma unroll
        for (int i = 0; i < 6; i++) p[i] *= dir / pnorm;
        pnorm = norm6(p);
        fp0 = dot6(p, g0);
#pragma unroll
        for (int i = 0; i < 6; i++) {  // changeDirection
            x_alpha[i] = x0[i];
            g_alpha[i] = g0[i];
        }
        f_key = 0.0;
        g_key = 0.0;
        df_alpha = slope();
        df_key = 0.0;
        return ST_SUCCESS;
    }
};

// out[4]: converged, iterations, n_corr, (pad); T12[16]
// nearest point of T (n points, LDS or global) to q: strict <, ties to the lower index
__device__ __forceinline__ int nn_search(const float* __restrict__ T, int n, const float* q, float* bdo) {
    float bd = dist2f(q, T);
    int best = 0;
    for (int j = 1; j < n; j++) {
        const float tj[3] = {T[3 * j], T[3 * j + 1], T[3 * j + 2]};
        const float d = dist2f(q, tj);
        if (d < bd) {
            bd = d;
            best = j;
        }
    }
    *bdo = bd;
    return best;
}

// one workgroup per problem of the batch
__global__ __launch_bounds__(GI_THREADS) void k_gicp(const float* __restrict__ src, const float* __restrict__ tgt,
                                                   const double* __restrict__ Cs, const double* __restrict__ Ct,
                                                   float* __restrict__ outp, double* __restrict__ Mah,
                                                   int* __restrict__ is, int* __restrict__ it, GicpArgs A,
                                                   float* __restrict__ T12, int* __restrict__ outi) {
    __shared__ double red[GI_NV][GI_THREADS];
    __shared__ double bc[GI_NV];
    __shared__ int wcnt[GI_WAVES];
    const int lane = threadIdx.x & (GI_LANES - 1), wave = threadIdx.x / GI_LANES;
    const int pb = blockIdx.x;
    const int s0 = A.soffs[pb], t0 = A.toffs[pb];
    const int ns = A.soffs[pb + 1] - s0, nt = A.toffs[pb + 1] - t0;
    const float* guess = A.guess + 16 * pb;
    T12 += 16 * pb;
    outi += 4 * pb;
    if (ns < 20 || nt < 20) {  // generalizedicp.cpp:33
        if (threadIdx.x < 16) T12[threadIdx.x] = threadIdx.x % 5 == 0 ? 1.f : 0.f;
        if (threadIdx.x < 4) outi[threadIdx.x] = 0;
        return;
    }
    src += 3 * (size_t)s0;
    outp += 3 * (size_t)s0;
    Cs += 9 * (size_t)s0;
    Mah += 9 * (size_t)s0;
    is += s0;
    it += s0;
    tgt += 3 * (size_t)t0;
    Ct += 9 * (size_t)t0;
    for (int i = threadIdx.x; i < ns; i += GI_THREADS) {  // transformPointCloud(output, output, guess)
        const float p0 = src[3 * i], p1 = src[3 * i + 1], p2 = src[3 * i + 2];
#pragma unroll
        for (int r = 0; r < 3; r++)
            outp[3 * i + r] = guess[4 * r] * p0 + guess[4 * r + 1] * p1 + guess[4 * r + 2] * p2 + guess[4 * r + 3];
    }
    __syncthreads();
    float Tcur[16], Tprev[16];
#pragma unroll
    for (int i = 0; i < 16; i++) Tcur[i] = Tprev[i] = i % 5 == 0 ? 1.f : 0.f;
    const double dist_threshold = A.max_corr_dist * A.max_corr_dist;
    int nr_iterations = 0, conv = 0, ncorr = 0;
    while (!conv) {
        double R[9];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) {
                double s = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) s += double(Tcur[4 * i + k]) * double(guess[4 * k + j]);
                R[3 * i + j] = s;
            }
        int base = 0;
        for (int i0 = 0; i0 < ns; i0 += GI_THREADS) {
            const int i = i0 + threadIdx.x;
            bool hit = false;
            int best = 0;
            if (i < ns) {
                const float pi[3] = {outp[3 * i], outp[3 * i + 1], outp[3 * i + 2]};
                float q[3];
                xform4f(Tcur, pi, q);
                float bd;
                best = nn_search(tgt, nt, q, &bd);  // (an LDS-staged target measured no faster)
                if ((double)bd < dist_threshold) {
                    hit = true;
                    const double* C1 = Cs + 9 * i;
                    const double* C2 = Ct + 9 * best;
                    double M[9], tmp[9];
#pragma unroll
                    for (int a = 0; a < 3; a++)
#pragma unroll
                        for (int b = 0; b < 3; b++)
                            M[3 * a + b] = s3(R[3 * a] * C1[b], R[3 * a + 1] * C1[3 + b], R[3 * a + 2] * C1[6 + b]);
#pragma unroll
                    for (int a = 0; a < 3; a++)
#pragma unroll
                        for (int b = 0; b < 3; b++) {
                            tmp[3 * a + b] = s3(M[3 * a] * R[3 * b], M[3 * a + 1] * R[3 * b + 1], M[3 * a + 2] * R[3 * b + 2]);
                            tmp[3 * a + b] += C2[3 * a + b];
                        }
                    double Mi[9];
                    inv3(tmp, Mi);
#pragma unroll
                    for (int k = 0; k < 9; k++) Mah[9 * i + k] = Mi[k];
                }
            }
            // compaction in source order: ballot within the wave, wave counts in order
            const uint64_t bal = __ballot(hit);
            if (lane == 0) wcnt[wave] = __popcll(bal);
            __syncthreads();
            int pre = base, tot = 0;
#pragma unroll
            for (int w = 0; w < GI_WAVES; w++) {
                if (w < wave) pre += wcnt[w];
                tot += wcnt[w];
            }
            const int pos = pre + __popcll(bal & ((1ull << lane) - 1ull));
            if (hit) {
                is[pos] = i;
                it[pos] = best;
            }
            base += tot;
            __syncthreads();
        }
        __threadfence_block();
        __syncthreads();
        ncorr = base;
#pragma unroll
        for (int i = 0; i < 16; i++) Tprev[i] = Tcur[i];
        if (base < 4) break;  // NotEnoughPointsException: caught, not converged
        double x[6] = {Tcur[3], Tcur[7], Tcur[11], (double)(float)atan2((double)Tcur[9], (double)Tcur[10]), (double)(float)asin(-(double)Tcur[8]),
                       (double)(float)atan2((double)Tcur[4], (double)Tcur[0])};
        GiBfgs bf;
        bf.P = GiProblem{outp, tgt, is, it, Mah, base, red, bc};
        bf.minimizeInit(x);
        int inner = 0, result;
        do {
            inner++;
            result = bf.minimizeOneStep(x);
            if (result) break;
            double gn = 0;
#pragma unroll
            for (int k = 0; k < 6; k++) gn += bf.gradient[k] * bf.gradient[k];
            result = sqrt(gn) < 1e-2 ? ST_SUCCESS : ST_RUNNING;
        } while (result == ST_RUNNING && inner < A.max_inner);
        if (!(result == ST_NO_PROGRESS || result == ST_SUCCESS || inner == A.max_inner)) break;
        apply_state(x, Tcur);
        double delta = 0.;
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int l = 0; l < 4; l++) {
                const double ratio = (k < 3 && l < 3) ? 1. / 2e-3 : 1. / 1e-9;
                const double c_delta = ratio * fabsf(Tprev[4 * k + l] - Tcur[4 * k + l]);
                if (c_delta > delta) delta = c_delta;
            }
        nr_iterations++;
        if (nr_iterations >= A.max_iterations || delta < 1) {
            conv = 1;
#pragma unroll
            for (int i = 0; i < 16; i++) Tprev[i] = Tcur[i];
        }
    }
    if (threadIdx.x == 0) {
        outi[0] = conv;
        outi[1] = nr_iterations;
        outi[2] = ncorr;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++)
                T12[4 * i + j] = conv ? ((Tprev[4 * i] * guess[j] + Tprev[4 * i + 1] * guess[4 + j]) +
                                         Tprev[4 * i + 2] * guess[8 + j]) + Tprev[4 * i + 3] * guess[12 + j]
                                      : (i == j ? 1.f : 0.f);
    }
}

}  // namespace

void launch_gicp(hipStream_t st, const float* src, const float* tgt, int nprob, int max_ns, int max_nt, double* Cs,
                 double* Ct, float* outp, double* Mah, int* is, int* it, GicpArgs args, float* T12, int* outi) {
    const int nbx = (std::max(max_ns, max_nt) + 63) / 64;
    hipLaunchKernelGGL(k_gicp_cov, dim3(nbx, nprob, 2), dim3(64), 0, st, src, args.soffs, Cs, tgt, args.toffs, Ct,
                       1e-3);
    hipLaunchKernelGGL(k_gicp, dim3(nprob), dim3(GI_THREADS), 0, st, src, tgt, Cs, Ct, outp, Mah, is, it, args, T12,
                       outi);
}

}  // namespace odo
