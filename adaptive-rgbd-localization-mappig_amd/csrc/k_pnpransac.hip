// PnPRansac::Compute (Odometry/pnpransac.cpp:11-51): cv::solvePnPRansac(v3D,
// v2D, mK, noDist, r, t, false, 500, 3.0f, 0.85, inliers) on the GPU
// (SURVEY §8(f) rank 4). OpenCV 3.4's RANSACPointSetRegistrator::run is a
// sequential loop whose only cross-iteration state is (maxGoodCount, niters);
// the minimal sets come from cv::RNG independently of the models. So:
//   k_pr_subsets  one lane draws every hypothesis' 5 distinct indices
//                 (cv::RNG(-1).uniform(0, n), getSubset's retry rule);
//   k_pr_epnp     16 lanes per hypothesis (row-parallel 12x12 Jacobi, the rest
//                 replicated on the group): EPnP on its 5 points (epnp.cpp:
//                 control points, barycentrics, 12x12 M^T M eigenvectors, the
//                 three beta approximations + 5 Gauss-Newton steps, best
//                 reprojection), Rodrigues -> (rvec, tvec) and the rotation
//                 projectPoints rebuilds from rvec;
//   k_pr_count    one workgroup per hypothesis: computeError (projectPoints in
//                 double, stored as float, L2SQR in float) and findInliers
//                 (err <= 9) for every point -> inlier bytes + count;
//   k_pr_fold     one lane replays run()'s loop over the counts in order:
//                 goodCount > max(maxGoodCount, 4) -> best, niters =
//                 RANSACUpdateNumIters(0.85, outlier ratio, 5, niters);
//   k_pr_refine   one wave: solvePnP(ITERATIVE, useExtrinsicGuess = false, as
//                 pnpransac.cpp:34 passes) on the best model's inliers =
//                 cvFindExtrinsicCameraParams2's own start (DLT / homography,
//                 extrinsic_init) then CvLevMarq (20 iterations, FLT_EPSILON)
//                 over cvProjectPoints2 residuals and Jacobians; J^T J, J^T e
//                 and |e| reduced in a fixed lane-shuffle order.
// All hypotheses up to `iterations` are evaluated (the fold decides how many
// were visited), like the Ransac::Iterate kernels. The per-hypothesis math is
// double precision IEEE +,-,*,/,sqrt in the oracle's operation order
// (-ffp-contract=off), so the models agree with oracle/pnpransac_ref.cpp up to
// the device libm's cos/sin/acos.
#include <hip/hip_runtime.h>

#include <cfloat>

#include "odo_internal.h"
#include "odo_linalg.h"

namespace odo {
namespace {

constexpr int PR_MODEL_POINTS = 5;
constexpr int PR_COUNT_THREADS = 256;
constexpr int PR_REFINE_THREADS = 64;  // one wave: the LM reductions need no LDS round

struct PrK {
    double fx, fy, cx, cy;
};

// The 12 x 12 M^T M of EPnP, row-parallel: a group of 16 lanes per
// hypothesis, lane r < 12 holding row r of A and of V (lanes 12..15 hold
// zeros). The column dot products of a rotation are xor-butterfly sums over the
// group taken from its first lane (tree16 in oracle/pnpransac_ref.cpp follows
// the same association); the rotations are lane-local, in svdj's order.
constexpr int PR_EPNP_GROUP = 16;
constexpr int PR_EPNP_THREADS = 64;
__device__ __forceinline__ double group_sum16(double x) {
    x += __shfl_xor(x, 8, PR_EPNP_GROUP);
    x += __shfl_xor(x, 4, PR_EPNP_GROUP);
    x += __shfl_xor(x, 2, PR_EPNP_GROUP);
    x += __shfl_xor(x, 1, PR_EPNP_GROUP);
    return __shfl(x, 0, PR_EPNP_GROUP);
}

__device__ void svdj12_rows(double* arow, double* vrow, int r, int* ord) {
#pragma unroll
    for (int j = 0; j < 12; j++) vrow[j] = (r == j) ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; sweep++) {
        int changed = 0;
#pragma unroll
        for (int p = 0; p < 11; p++)
#pragma unroll
            for (int q = p + 1; q < 12; q++) {
                const double ap0 = arow[p], aq0 = arow[q];
                const double alpha = group_sum16(ap0 * ap0);
                const double beta = group_sum16(aq0 * aq0);
                const double gamma = group_sum16(ap0 * aq0);
                if (gamma == 0.0 || fabs(gamma) <= DBL_EPSILON * sqrt(alpha * beta)) continue;
                changed = 1;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
                arow[p] = c * ap0 - s * aq0;
                arow[q] = s * ap0 + c * aq0;
                const double vp = vrow[p], vq = vrow[q];
                vrow[p] = c * vp - s * vq;
                vrow[q] = s * vp + c * vq;
            }
        if (!changed) break;
    }
    double ww[12];
#pragma unroll
    for (int j = 0; j < 12; j++) {
        ww[j] = sqrt(group_sum16(arow[j] * arow[j]));
        ord[j] = j;
    }
#pragma unroll
    for (int j = 0; j < 12; j++) {
        int b = j;
        double wb = ww[j];
#pragma unroll
        for (int k = j + 1; k < 12; k++)
            if (ww[k] > wb) {
                b = k;
                wb = ww[k];
            }
#pragma unroll
        for (int k = j + 1; k < 12; k++)
            if (k == b) {
                const double tw = ww[j];
                ww[j] = ww[k];
                ww[k] = tw;
                const int to = ord[j];
                ord[j] = ord[k];
                ord[k] = to;
            }
    }
}

// cvSolve(A, b, x, CV_SVD): least squares over w > n * DBL_EPSILON * w[0]
template <int M, int N>
__device__ void svd_solve(const double* A, const double* b, double* x) {
    double w[N], U[M * N], V[N * N];
    svdj<M, N>(A, w, U, V);
    const double thr = N * DBL_EPSILON * w[0];
    double y[N];
#pragma unroll
    for (int j = 0; j < N; j++) {
        double s = 0;
#pragma unroll
        for (int i = 0; i < M; i++) s += U[i * N + j] * b[i];
        y[j] = w[j] > thr ? s / w[j] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < N; i++) {
        double s = 0;
#pragma unroll
        for (int j = 0; j < N; j++) s += V[i * N + j] * y[j];
        x[i] = s;
    }
}

__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// cvRodrigues2 vector -> matrix (+ dRdr[i*9+k] = dR_k/dr_i)
__device__ void rod_v2m(const double* r, double* R, double* J) {
    const double theta = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; k++) R[k] = k % 4 == 0 ? 1.0 : 0.0;
        if (J) {
            for (int k = 0; k < 27; k++) J[k] = 0.0;
            J[5] = 1;
            J[7] = -1;
            J[11] = -1;
            J[15] = 1;
            J[19] = 1;
            J[21] = -1;
        }
        return;
    }
    const double c = cos(theta), s = sin(theta), c1 = 1. - c;
    const double itheta = theta ? 1. / theta : 0.;
    const double rx = r[0] * itheta, ry = r[1] * itheta, rz = r[2] * itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rx_[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 9; k++) R[k] = c * I[k] + c1 * rrt[k] + s * rx_[k];
    if (J) {
        const double drrt[27] = {rx + rx, ry, rz, ry, 0, 0, rz, 0, 0, 0, rx, 0, rx, ry + ry, rz, 0, rz, 0,
                                 0, 0, rx, 0, 0, ry, rx, ry, rz + rz};
        const double drx_[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0,
                                 0, -1, 0, 1, 0, 0, 0, 0, 0};
        for (int i = 0; i < 3; i++) {
            const double ri = i == 0 ? rx : i == 1 ? ry : rz;
            const double a0 = -s * ri, a1 = (s - 2 * c1 * itheta) * ri, a2 = c1 * itheta;
            const double a3 = (c - s * itheta) * ri, a4 = s * itheta;
            for (int k = 0; k < 9; k++)
                J[i * 9 + k] = a0 * I[k] + a1 * rrt[k] + a2 * drrt[i * 9 + k] + a3 * rx_[k] + a4 * drx_[i * 9 + k];
        }
    }
}

// cvRodrigues2 matrix -> vector (R := U V^T first)
__device__ void rod_m2v(const double* Rin, double* r) {
    double w[3], U[9], V[9], R[9];
    svdj<3, 3>(Rin, w, U, V);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i * 3 + j] = U[i * 3 + 0] * V[j * 3 + 0] + U[i * 3 + 1] * V[j * 3 + 1] + U[i * 3 + 2] * V[j * 3 + 2];
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = sqrt(t > 0 ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta;
            ry *= theta;
            rz *= theta;
        }
    } else {
        double vth = 1 / (2 * s);
        vth *= theta;
        rx *= vth;
        ry *= vth;
        rz *= vth;
    }
    r[0] = rx;
    r[1] = ry;
    r[2] = rz;
}

// cvProjectPoints2 of one point without distortion (+ Jacobian rows)
__device__ __forceinline__ void project_pt(const double* R, const double* dRdr, const double* t, const PrK& K,
                                           double X, double Y, double Z, double* u, double* v, double* Ju,
                                           double* Jv) {
    double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    z = z ? 1. / z : 1;
    x *= z;
    y *= z;
    *u = x * K.fx + K.cx;
    *v = y * K.fy + K.cy;
    if (Ju) {
        Ju[3] = K.fx * z;
        Ju[4] = K.fx * 0.0;
        Ju[5] = K.fx * (-x * z);
        Jv[3] = K.fy * 0.0;
        Jv[4] = K.fy * z;
        Jv[5] = K.fy * (-y * z);
        for (int j = 0; j < 3; j++) {
            const double* d = dRdr + 9 * j;
            const double dx0 = X * d[0] + Y * d[1] + Z * d[2];
            const double dy0 = X * d[3] + Y * d[4] + Z * d[5];
            const double dz0 = X * d[6] + Y * d[7] + Z * d[8];
            Ju[j] = K.fx * (z * (dx0 - x * dz0));
            Jv[j] = K.fy * (z * (dy0 - y * dz0));
        }
    }
}

// ------------------------------------------------ EPnP on the 5 points (epnp.cpp)
struct Epnp5 {
    double pws[15], us[10];
    double alphas[20], pcs[15];
    double cws[4][3], ccs[4][3];
    double fu, fv, uc, vc;

    __device__ void choose_control_points() {
        cws[0][0] = cws[0][1] = cws[0][2] = 0;
        for (int i = 0; i < PR_MODEL_POINTS; i++)
            for (int j = 0; j < 3; j++) cws[0][j] += pws[3 * i + j];
        for (int j = 0; j < 3; j++) cws[0][j] /= PR_MODEL_POINTS;
        double PtP[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < PR_MODEL_POINTS; i++) {
            double d[3];
            for (int j = 0; j < 3; j++) d[j] = pws[3 * i + j] - cws[0][j];
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) PtP[a * 3 + b] += d[a] * d[b];
        }
        double dc[3], V[9];
        svdj<3, 3>(PtP, dc, nullptr, V);
        for (int i = 1; i < 4; i++) {
            const double k = sqrt(dc[i - 1] / PR_MODEL_POINTS);
            for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * V[j * 3 + (i - 1)];
        }
    }
    __device__ void compute_barycentric_coordinates() {
        double cc[9], w[3], U[9], V[9], ci[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
        svdj<3, 3>(cc, w, U, V);
        const double thr = 3 * DBL_EPSILON * w[0];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                double s = 0;
                for (int k = 0; k < 3; k++) s += V[i * 3 + k] * (w[k] > thr ? 1.0 / w[k] : 0.0) * U[j * 3 + k];
                ci[i * 3 + j] = s;
            }
        for (int i = 0; i < PR_MODEL_POINTS; i++) {
            const double* pi = pws + 3 * i;
            double* a = alphas + 4 * i;
            for (int j = 0; j < 3; j++)
                a[1 + j] = ci[3 * j] * (pi[0] - cws[0][0]) + ci[3 * j + 1] * (pi[1] - cws[0][1]) +
                           ci[3 * j + 2] * (pi[2] - cws[0][2]);
            a[0] = 1.0f - a[1] - a[2] - a[3];
        }
    }
    __device__ double compute_R_and_t(const double* ut, const double* betas, double R[3][3], double t[3]) {
        for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
        for (int i = 0; i < 4; i++) {
            const double* v = ut + 12 * (3 - i);  // ut4 row 11 - i
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
        }
        for (int i = 0; i < PR_MODEL_POINTS; i++) {
            const double* a = alphas + 4 * i;
            for (int j = 0; j < 3; j++)
                pcs[3 * i + j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
        }
        if (pcs[2] < 0.0) {  // solve_for_sign
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
            for (int i = 0; i < 3 * PR_MODEL_POINTS; i++) pcs[i] = -pcs[i];
        }
        // estimate_R_and_t
        double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
        for (int i = 0; i < PR_MODEL_POINTS; i++)
            for (int j = 0; j < 3; j++) {
                pc0[j] += pcs[3 * i + j];
                pw0[j] += pws[3 * i + j];
            }
        for (int j = 0; j < 3; j++) {
            pc0[j] /= PR_MODEL_POINTS;
            pw0[j] /= PR_MODEL_POINTS;
        }
        double abt[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        for (int i = 0; i < PR_MODEL_POINTS; i++) {
            const double* pc = pcs + 3 * i;
            const double* pw = pws + 3 * i;
            for (int j = 0; j < 3; j++) {
                abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
                abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
                abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
            }
        }
        double d[3], u[9], v[9];
        svdj<3, 3>(abt, d, u, v);
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = dot3(u + 3 * i, v + 3 * j);
        const double det = R[0][0] * R[1][1] * R[2][2] + R[0][1] * R[1][2] * R[2][0] + R[0][2] * R[1][0] * R[2][1] -
                           R[0][2] * R[1][1] * R[2][0] - R[0][1] * R[1][0] * R[2][2] - R[0][0] * R[1][2] * R[2][1];
        if (det < 0) {
            R[2][0] = -R[2][0];
            R[2][1] = -R[2][1];
            R[2][2] = -R[2][2];
        }
        t[0] = pc0[0] - dot3(R[0], pw0);
        t[1] = pc0[1] - dot3(R[1], pw0);
        t[2] = pc0[2] - dot3(R[2], pw0);
        // reprojection_error
        double sum2 = 0.0;
        for (int i = 0; i < PR_MODEL_POINTS; i++) {
            const double* pw = pws + 3 * i;
            const double Xc = dot3(R[0], pw) + t[0], Yc = dot3(R[1], pw) + t[1];
            const double inv_Zc = 1.0 / (dot3(R[2], pw) + t[2]);
            const double ue = uc + fu * Xc * inv_Zc, ve = vc + fv * Yc * inv_Zc;
            const double uu = us[2 * i], vv = us[2 * i + 1];
            sum2 += sqrt((uu - ue) * (uu - ue) + (vv - ve) * (vv - ve));
        }
        return sum2 / PR_MODEL_POINTS;
    }
};

// ut4 = rows 8..11 of epnp.cpp's ut (the four smallest singular vectors)
__device__ void compute_L_6x10(const double* ut4, double* l) {
    const double* v[4] = {ut4 + 12 * 3, ut4 + 12 * 2, ut4 + 12 * 1, ut4};
    double dv[4][6][3];
    for (int i = 0; i < 4; i++) {
        int a = 0, b = 1;
        for (int j = 0; j < 6; j++) {
            for (int k = 0; k < 3; k++) dv[i][j][k] = v[i][3 * a + k] - v[i][3 * b + k];
            b++;
            if (b > 3) {
                a++;
                b = a + 1;
            }
        }
    }
    for (int i = 0; i < 6; i++) {
        double* row = l + 10 * i;
        row[0] = dot3(dv[0][i], dv[0][i]);
        row[1] = 2.0f * dot3(dv[0][i], dv[1][i]);
        row[2] = dot3(dv[1][i], dv[1][i]);
        row[3] = 2.0f * dot3(dv[0][i], dv[2][i]);
        row[4] = 2.0f * dot3(dv[1][i], dv[2][i]);
        row[5] = dot3(dv[2][i], dv[2][i]);
        row[6] = 2.0f * dot3(dv[0][i], dv[3][i]);
        row[7] = 2.0f * dot3(dv[1][i], dv[3][i]);
        row[8] = 2.0f * dot3(dv[2][i], dv[3][i]);
        row[9] = dot3(dv[3][i], dv[3][i]);
    }
}

__device__ __forceinline__ double dist2(const double* a, const double* b) {
    return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
}

__device__ void betas_approx(const double* l, const double* rho, int which, double* betas) {
    const int nc = which == 1 ? 4 : which == 2 ? 3 : 5;
    int cols[5] = {0, 1, 2, 3, 4};
    if (which == 1) {
        cols[2] = 3;
        cols[3] = 6;
    }
    double L[30], b[5];
    for (int i = 0; i < 6; i++)
        for (int j = 0; j < nc; j++) L[i * nc + j] = l[10 * i + cols[j]];
    if (which == 1)
        svd_solve<6, 4>(L, rho, b);
    else if (which == 2)
        svd_solve<6, 3>(L, rho, b);
    else
        svd_solve<6, 5>(L, rho, b);
    if (which == 1) {
        if (b[0] < 0) {
            betas[0] = sqrt(-b[0]);
            betas[1] = -b[1] / betas[0];
            betas[2] = -b[2] / betas[0];
            betas[3] = -b[3] / betas[0];
        } else {
            betas[0] = sqrt(b[0]);
            betas[1] = b[1] / betas[0];
            betas[2] = b[2] / betas[0];
            betas[3] = b[3] / betas[0];
        }
        return;
    }
    if (b[0] < 0) {
        betas[0] = sqrt(-b[0]);
        betas[1] = (b[2] < 0) ? sqrt(-b[2]) : 0.0;
    } else {
        betas[0] = sqrt(b[0]);
        betas[1] = (b[2] > 0) ? sqrt(b[2]) : 0.0;
    }
    if (b[1] < 0) betas[0] = -betas[0];
    betas[2] = which == 3 ? b[3] / betas[0] : 0.0;
    betas[3] = 0.0;
}

// epnp.cpp qr_solve (6 x 4 Householder), with its column scan as written
__device__ void qr_solve(double* A, double* b, double* X) {
    const int nr = 6, nc = 4;
    double A1[4], A2[4];
    for (int k = 0; k < nc; k++) {
        double* ppAkk = A + k * (nc + 1);
        double* ppAik = ppAkk;
        double eta = fabs(*ppAik);
        for (int i = k + 1; i < nr; i++) {
            const double elt = fabs(*ppAik);
            if (eta < elt) eta = elt;
            ppAik += nc;
        }
        if (eta == 0) {
            A1[k] = A2[k] = 0.0;
            return;
        }
        double sum = 0.0;
        const double inv_eta = 1. / eta;
        ppAik = ppAkk;
        for (int i = k; i < nr; i++) {
            *ppAik *= inv_eta;
            sum += *ppAik * *ppAik;
            ppAik += nc;
        }
        double sigma = sqrt(sum);
        if (*ppAkk < 0) sigma = -sigma;
        *ppAkk += sigma;
        A1[k] = sigma * *ppAkk;
        A2[k] = -eta * sigma;
        for (int j = k + 1; j < nc; j++) {
            double* p = ppAkk;
            double s = 0;
            for (int i = k; i < nr; i++) {
                s += *p * p[j - k];
                p += nc;
            }
            const double tau = s / A1[k];
            p = ppAkk;
            for (int i = k; i < nr; i++) {
                p[j - k] -= tau * *p;
                p += nc;
            }
        }
    }
    for (int j = 0; j < nc; j++) {
        double* p = A + j * (nc + 1);
        double tau = 0;
        for (int i = j; i < nr; i++) {
            tau += *p * b[i];
            p += nc;
        }
        tau /= A1[j];
        p = A + j * (nc + 1);
        for (int i = j; i < nr; i++) {
            b[i] -= tau * *p;
            p += nc;
        }
    }
    X[nc - 1] = b[nc - 1] / A2[nc - 1];
    for (int i = nc - 2; i >= 0; i--) {
        const double* p = A + i * nc + (i + 1);
        double s = 0;
        for (int j = i + 1; j < nc; j++) {
            s += *p * X[j];
            p++;
        }
        X[i] = (b[i] - s) / A2[i];
    }
}

__device__ void gauss_newton(const double* l, const double* rho, double* betas) {
    for (int k = 0; k < 5; k++) {
        double A[24], b[6], x[4] = {0, 0, 0, 0};
        for (int i = 0; i < 6; i++) {
            const double* r = l + i * 10;
            double* a = A + i * 4;
            a[0] = 2 * r[0] * betas[0] + r[1] * betas[1] + r[3] * betas[2] + r[6] * betas[3];
            a[1] = r[1] * betas[0] + 2 * r[2] * betas[1] + r[4] * betas[2] + r[7] * betas[3];
            a[2] = r[3] * betas[0] + r[4] * betas[1] + 2 * r[5] * betas[2] + r[8] * betas[3];
            a[3] = r[6] * betas[0] + r[7] * betas[1] + r[8] * betas[2] + 2 * r[9] * betas[3];
            b[i] = rho[i] - (r[0] * betas[0] * betas[0] + r[1] * betas[0] * betas[1] + r[2] * betas[1] * betas[1] +
                             r[3] * betas[0] * betas[2] + r[4] * betas[1] * betas[2] + r[5] * betas[2] * betas[2] +
                             r[6] * betas[0] * betas[3] + r[7] * betas[1] * betas[3] + r[8] * betas[2] * betas[3] +
                             r[9] * betas[3] * betas[3]);
        }
        qr_solve(A, b, x);
        for (int i = 0; i < 4; i++) betas[i] += x[i];
    }
}

// ------------------------------------------------------------------ kernels
// cv::RNG draws on one lane: the multiply-with-carry step, x % n through a
// double reciprocal with one correction (exact for x < 2^32), getSubset's
// rule (a draw equal to an earlier index of the same subset is drawn again).
constexpr int PR_RNG_THREADS = 64;
// Problems of a batch: problem p owns points [offs[p], offs[p + 1]); problems
// with fewer than 10 points are skipped (pnpransac.cpp:30).
__global__ __launch_bounds__(PR_RNG_THREADS) void k_pr_subsets(const int* __restrict__ offs, int nprob, int H,
                                                               int* __restrict__ idx) {
    const int pb = blockIdx.x * blockDim.x + threadIdx.x;
    if (pb >= nprob) return;
    const int n = offs[pb + 1] - offs[pb];
    if (n < 10) return;
    idx += (size_t)pb * H * PR_MODEL_POINTS;
    const double inv = 1.0 / (double)n;
    uint64_t state = ~(uint64_t)0;  // RNG rng((uint64)-1), ptsetreg.cpp run()
    for (int h = 0; h < H; h++) {
        int sub[PR_MODEL_POINTS];
#pragma unroll
        for (int i = 0; i < PR_MODEL_POINTS; i++) {
            int v;
            for (;;) {
                state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
                // x % n: the double quotient is floor(x / n) or one off, the
                // 32-bit remainder (mod 2^32) is corrected once either way
                const uint32_t x = (uint32_t)state;
                const uint32_t q = (uint32_t)((double)x * inv);
                int rem = (int)(x - q * (uint32_t)n);
                if (rem < 0)
                    rem += n;
                else if (rem >= n)
                    rem -= n;
                v = rem;
                bool dup = false;
#pragma unroll
                for (int j = 0; j < i; j++) dup |= sub[j] == v;
                if (!dup) break;
            }
            sub[i] = v;
        }
#pragma unroll
        for (int i = 0; i < PR_MODEL_POINTS; i++) idx[h * PR_MODEL_POINTS + i] = sub[i];
    }
}

__global__ __launch_bounds__(PR_EPNP_THREADS) void k_pr_epnp(const float* __restrict__ Xw,
                                                             const float* __restrict__ uv,
                                                             const int* __restrict__ offs, const int* __restrict__ idx,
                                                             int H, int h0, int h1, const int* __restrict__ fstate,
                                                             PrK K, double* __restrict__ model,
                                                             double* __restrict__ Rproj) {
    const int r = threadIdx.x & (PR_EPNP_GROUP - 1);
    const int h = h0 + blockIdx.x * (PR_EPNP_THREADS / PR_EPNP_GROUP) + (threadIdx.x >> 4);
    const int pb = blockIdx.y;
    // whole 16-lane groups leave together; with a fold state, hypotheses at or
    // past the problem's current niters are never visited (niters only shrinks)
    if (h >= h1 || offs[pb + 1] - offs[pb] < 10 || (fstate && h >= fstate[4 * pb + 3])) return;
    Xw += 3 * (size_t)offs[pb];
    uv += 2 * (size_t)offs[pb];
    idx += (size_t)pb * H * PR_MODEL_POINTS;
    model += (size_t)pb * H * 6;
    Rproj += (size_t)pb * H * 9;
    // every lane of the group runs the small steps redundantly (identical
    // arithmetic), lane r < 12 owns row r of the 12 x 12 eigenproblem
    Epnp5 e;
    e.fu = K.fx;
    e.fv = K.fy;
    e.uc = K.cx;
    e.vc = K.cy;
    for (int i = 0; i < PR_MODEL_POINTS; i++) {
        const int p = idx[h * PR_MODEL_POINTS + i];
        for (int k = 0; k < 3; k++) e.pws[3 * i + k] = (double)Xw[3 * p + k];
        e.us[2 * i] = (double)uv[2 * p];
        e.us[2 * i + 1] = (double)uv[2 * p + 1];
    }
    e.choose_control_points();
    e.compute_barycentric_coordinates();
    // row r of M^T M: sum over the M rows 2i, 2i+1 in order (fill_M)
    double arow[12], vrow[12];
#pragma unroll
    for (int j = 0; j < 12; j++) arow[j] = 0.0;
    for (int i = 0; i < PR_MODEL_POINTS; i++) {
        const double* as = e.alphas + 4 * i;
        double M1[12], M2[12];
        const double uu = e.us[2 * i], vv = e.us[2 * i + 1];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            M1[3 * j] = as[j] * e.fu;
            M1[3 * j + 1] = 0.0;
            M1[3 * j + 2] = as[j] * (e.uc - uu);
            M2[3 * j] = 0.0;
            M2[3 * j + 1] = as[j] * e.fv;
            M2[3 * j + 2] = as[j] * (e.vc - vv);
        }
        double m1r = 0.0, m2r = 0.0;
#pragma unroll
        for (int j = 0; j < 12; j++)
            if (j == r) {
                m1r = M1[j];
                m2r = M2[j];
            }
#pragma unroll
        for (int j = 0; j < 12; j++) {
            arow[j] += m1r * M1[j];
            arow[j] += m2r * M2[j];
        }
    }
    if (r >= 12)
#pragma unroll
        for (int j = 0; j < 12; j++) arow[j] = 0.0;
    int ord[12];
    svdj12_rows(arow, vrow, r, ord);
    // ut rows 8..11 (the four smallest singular vectors) = V columns ord[8..11]
    double ut[48];  // ut4[(k) * 12 + j] = V(j, ord[8 + k]), V row j on lane j
#pragma unroll
    for (int k = 0; k < 4; k++) {
        double mine = 0.0;
#pragma unroll
        for (int c = 0; c < 12; c++)
            if (c == ord[8 + k]) mine = vrow[c];
#pragma unroll
        for (int j = 0; j < 12; j++) ut[k * 12 + j] = __shfl(mine, j, PR_EPNP_GROUP);
    }
    double l[60], rho[6];
    compute_L_6x10(ut, l);
    rho[0] = dist2(e.cws[0], e.cws[1]);
    rho[1] = dist2(e.cws[0], e.cws[2]);
    rho[2] = dist2(e.cws[0], e.cws[3]);
    rho[3] = dist2(e.cws[1], e.cws[2]);
    rho[4] = dist2(e.cws[1], e.cws[3]);
    rho[5] = dist2(e.cws[2], e.cws[3]);
    double bestR[3][3], bestt[3], bestErr = 0;
    for (int w = 1; w <= 3; w++) {
        double betas[4], R[3][3], t[3];
        betas_approx(l, rho, w, betas);
        gauss_newton(l, rho, betas);
        const double err = e.compute_R_and_t(ut, betas, R, t);
        if (w == 1 || err < bestErr) {  // N = 1; rep[2] < rep[1] -> 2; rep[3] < rep[N] -> 3
            bestErr = err;
            for (int a = 0; a < 3; a++) {
                bestt[a] = t[a];
                for (int b = 0; b < 3; b++) bestR[a][b] = R[a][b];
            }
        }
    }
    double rv[3], Rp[9];
    rod_m2v(&bestR[0][0], rv);
    rod_v2m(rv, Rp, nullptr);
    if (r != 0) return;
    double* mo = model + 6 * h;
    mo[0] = rv[0];
    mo[1] = rv[1];
    mo[2] = rv[2];
    mo[3] = bestt[0];
    mo[4] = bestt[1];
    mo[5] = bestt[2];
    for (int k = 0; k < 9; k++) Rproj[9 * h + k] = Rp[k];
}

__global__ __launch_bounds__(PR_COUNT_THREADS) void k_pr_count(const float* __restrict__ Xw,
                                                               const float* __restrict__ uv,
                                                               const int* __restrict__ offs, int H, int h0,
                                                               const int* __restrict__ fstate, PrK K, float thr,
                                                               const double* __restrict__ model,
                                                               const double* __restrict__ Rproj,
                                                               uint8_t* __restrict__ mask, int* __restrict__ good) {
    const int h = h0 + blockIdx.x, pb = blockIdx.y;
    const int n = offs[pb + 1] - offs[pb];
    if (n < 10 || (fstate && h >= fstate[4 * pb + 3])) return;
    Xw += 3 * (size_t)offs[pb];
    uv += 2 * (size_t)offs[pb];
    model += (size_t)pb * H * 6;
    Rproj += (size_t)pb * H * 9;
    mask += (size_t)H * offs[pb];
    good += (size_t)pb * H;
    __shared__ int wsum[PR_COUNT_THREADS / 64];
    double R[9], t[3];
    for (int k = 0; k < 9; k++) R[k] = Rproj[9 * h + k];
    for (int k = 0; k < 3; k++) t[k] = model[6 * h + 3 + k];
    uint8_t* mrow = mask + (size_t)h * n;
    int cnt = 0;
    for (int i = threadIdx.x; i < n; i += PR_COUNT_THREADS) {
        double u, v;
        project_pt(R, nullptr, t, K, (double)Xw[3 * i], (double)Xw[3 * i + 1], (double)Xw[3 * i + 2], &u, &v,
                   nullptr, nullptr);
        const float dx = uv[2 * i] - (float)u, dy = uv[2 * i + 1] - (float)v;
        const float e2 = dx * dx + dy * dy;
        const int f = e2 <= thr;
        mrow[i] = (uint8_t)f;
        cnt += f;
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        int s = 0;
        for (int w = 0; w < PR_COUNT_THREADS / 64; w++) s += wsum[w];
        good[h] = s;
    }
}

__device__ int update_num_iters(double p, double ep, int modelPoints, int maxIters) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - pow(1. - ep, (double)modelPoints);
    if (denom < DBL_MIN) return 0;
    num = log(num);
    denom = log(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)rint(num / denom);
}

// state[4p]: [0] = best hypothesis (-1: none), [1] = iterations visited so
// far, [2] = maxGoodCount, [3] = niters. Folds hypotheses [h0, h1) in order,
// continuing the state of earlier chunks (h0 = 0 starts it).
__global__ void k_pr_fold(const int* __restrict__ good, const int* __restrict__ offs, int nprob, int H, int h0,
                          int h1, double confidence, int* __restrict__ state) {
    const int pb = blockIdx.x * blockDim.x + threadIdx.x;
    if (pb >= nprob) return;
    const int n = offs[pb + 1] - offs[pb];
    good += (size_t)pb * H;
    state += 4 * pb;
    if (n < 10) {
        state[0] = -1;
        state[1] = 0;
        state[2] = 0;
        state[3] = 0;
        return;
    }
    int niters, maxGood, best, iter;
    if (h0 == 0) {
        niters = H > 1 ? H : 1;
        maxGood = 0;
        best = -1;
        iter = 0;
    } else {
        best = state[0];
        iter = state[1];
        maxGood = state[2];
        niters = state[3];
        if (iter < h0) return;  // the fold ended in an earlier chunk
    }
    for (; iter < niters && iter < h1; iter++) {
        const int g = good[iter];
        if (g > (maxGood > PR_MODEL_POINTS - 1 ? maxGood : PR_MODEL_POINTS - 1)) {
            best = iter;
            maxGood = g;
            niters = update_num_iters(confidence, (double)(n - g) / n, PR_MODEL_POINTS, niters);
        }
    }
    state[0] = best;
    state[1] = iter;
    state[2] = maxGood;
    state[3] = niters;
}

// fixed-order workgroup sum of NV doubles per thread (wave shuffles, then waves in order)
template <int NV>
__device__ void block_sum(double* v, double (*wred)[NV], double* out) {
    for (int k = 0; k < NV; k++)
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_down(v[k], o, 64);
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < NV; k++) wred[threadIdx.x >> 6][k] = v[k];
    __syncthreads();
    for (int k = threadIdx.x; k < NV; k += PR_REFINE_THREADS) {  // NV may exceed the thread count
        double s = wred[0][k];
        for (int w = 1; w < PR_REFINE_THREADS / 64; w++) s += wred[w][k];
        out[k] = s;
    }
    __syncthreads();
}

// residual pass over the inliers: with J -> red[0..35] = J^T J, [36..41] = J^T e, [42] = |e|^2
__device__ void lm_pass(const float* __restrict__ Xw, const float* __restrict__ uv, const uint8_t* __restrict__ m,
                        int n, const PrK& K, const double* p, bool withJ, double (*wred)[43], double* red) {
    double R[9], dRdr[27];
    rod_v2m(p, R, withJ ? dRdr : nullptr);
    double acc[43];
    for (int k = 0; k < 43; k++) acc[k] = 0.0;
    for (int i = threadIdx.x; i < n; i += PR_REFINE_THREADS) {
        if (!m[i]) continue;
        double u, v, Ju[6], Jv[6];
        project_pt(R, dRdr, p + 3, K, (double)Xw[3 * i], (double)Xw[3 * i + 1], (double)Xw[3 * i + 2], &u, &v,
                   withJ ? Ju : nullptr, withJ ? Jv : nullptr);
        const double eu = u - (double)uv[2 * i], ev = v - (double)uv[2 * i + 1];
        acc[42] += eu * eu;
        acc[42] += ev * ev;
        if (withJ)
            for (int a = 0; a < 6; a++) {
                for (int b = 0; b < 6; b++) {
                    acc[a * 6 + b] += Ju[a] * Ju[b];
                    acc[a * 6 + b] += Jv[a] * Jv[b];
                }
                acc[36 + a] += Ju[a] * eu;
                acc[36 + a] += Jv[a] * ev;
            }
    }
    if (withJ) {
        block_sum<43>(acc, wred, red);
    } else {
        // only |e|^2: reuse the 43-wide path for slot 42 alone
        double one[1] = {acc[42]};
        for (int o = 32; o > 0; o >>= 1) one[0] += __shfl_down(one[0], o, 64);
        if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6][42] = one[0];
        __syncthreads();
        if (threadIdx.x == 0) {
            double s = wred[0][42];
            for (int w = 1; w < PR_REFINE_THREADS / 64; w++) s += wred[w][42];
            red[42] = s;
        }
        __syncthreads();
    }
}

// ------------------------- cvFindExtrinsicCameraParams2, unseeded (calibration.cpp)
// The final solvePnP of solvePnPRansac gets the caller's useExtrinsicGuess,
// false at pnpransac.cpp:34, so the LM starts from cvFindExtrinsicCameraParams2's
// own initial pose (extrinsic_init in oracle/pnpransac_ref.cpp, same
// operation order): centroid + scatter of the object points (wave sums over
// the inliers, point i on lane i % 64), 3x3 SVD -> planar or not; non-planar:
// the DLT's 12 x 12 L^T L (78 wave sums), its smallest singular vector (by
// inverse iteration: the same vector as the oracle's Jacobi SVD up to
// rounding), [R | t] from it;
// planar: the homography path on lane 0 (rare: coplanar landmarks), its
// matrices in LDS.

// one-sided Jacobi SVD on LDS arrays, one lane (oracle svdj's loop order):
// a (m x n) is destroyed; w (n), V (n x n by columns), U (m x n) if non-null
__device__ void svdj_lds(int m, int n, double* a, double* v, double* w, double* U, double* V, double* ww, int* ord) {
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) v[i * n + j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; sweep++) {
        int changed = 0;
        for (int p = 0; p < n - 1; p++)
            for (int q = p + 1; q < n; q++) {
                double alpha = 0, beta = 0, gamma = 0;
                for (int i = 0; i < m; i++) {
                    const double ap = a[i * n + p], aq = a[i * n + q];
                    alpha += ap * ap;
                    beta += aq * aq;
                    gamma += ap * aq;
                }
                if (gamma == 0.0 || fabs(gamma) <= DBL_EPSILON * sqrt(alpha * beta)) continue;
                changed = 1;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
                for (int i = 0; i < m; i++) {
                    const double ap = a[i * n + p], aq = a[i * n + q];
                    a[i * n + p] = c * ap - sn * aq;
                    a[i * n + q] = sn * ap + c * aq;
                }
                for (int i = 0; i < n; i++) {
                    const double vp = v[i * n + p], vq = v[i * n + q];
                    v[i * n + p] = c * vp - sn * vq;
                    v[i * n + q] = sn * vp + c * vq;
                }
            }
        if (!changed) break;
    }
    for (int j = 0; j < n; j++) {
        double sq = 0;
        for (int i = 0; i < m; i++) sq += a[i * n + j] * a[i * n + j];
        ww[j] = sqrt(sq);
        ord[j] = j;
    }
    for (int j = 0; j < n; j++) {
        int b = j;
        for (int k = j + 1; k < n; k++)
            if (ww[ord[k]] > ww[ord[b]]) b = k;
        const int t = ord[j];
        ord[j] = ord[b];
        ord[b] = t;
    }
    for (int j = 0; j < n; j++) {
        const int c = ord[j];
        w[j] = ww[c];
        const double inv = ww[c] > 0 ? 1.0 / ww[c] : 0.0;
        if (U)
            for (int i = 0; i < m; i++) U[i * n + j] = a[i * n + c] * inv;
        for (int i = 0; i < n; i++) V[i * n + j] = v[i * n + c];
    }
}

struct HomLds {  // lane-0 scratch of the planar start
    double a[81], v[81], U[81], V[81], w[9], ww[9];
    int ord[9];
    double A[64], Ap[64];
};

// svd_solve (cvSolve CV_SVD) of the n x n Ap against b, on LDS
__device__ void svd_solve_lds(int n, HomLds& h, const double* b, double* x) {
    for (int k = 0; k < n * n; k++) h.a[k] = h.Ap[k];
    svdj_lds(n, n, h.a, h.v, h.w, h.U, h.V, h.ww, h.ord);
    const double thr = n * DBL_EPSILON * h.w[0];
    double y[8];
    for (int j = 0; j < n; j++) {
        double sacc = 0;
        for (int i = 0; i < n; i++) sacc += h.U[i * n + j] * b[i];
        y[j] = h.w[j] > thr ? sacc / h.w[j] : 0.0;
    }
    for (int i = 0; i < n; i++) {
        double sacc = 0;
        for (int j = 0; j < n; j++) sacc += h.V[i * n + j] * y[j];
        x[i] = sacc;
    }
}

__device__ __forceinline__ double det3d(const double* a) {
    return a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6]);
}

// the planar point (Rt M + T).xy as float and the normalised image point as float
__device__ __forceinline__ void hom_pts(const float* Xw, const float* uv, int i, const double* Rt, const double* T,
                                        const PrK& K, double ifx, double ify, float* Mf, float* mf) {
    const double s0 = Xw[3 * i], s1 = Xw[3 * i + 1], s2 = Xw[3 * i + 2];
    Mf[0] = (float)(Rt[0] * s0 + Rt[1] * s1 + Rt[2] * s2 + T[0]);
    Mf[1] = (float)(Rt[3] * s0 + Rt[4] * s1 + Rt[5] * s2 + T[1]);
    mf[0] = (float)(((double)uv[2 * i] - K.cx) * ifx);
    mf[1] = (float)(((double)uv[2 * i + 1] - K.cy) * ify);
}

// cv::findHomography(Mxy, mn, 0) (oracle find_homography): lane 0
__device__ bool find_homography_lane(const float* Xw, const float* uv, const uint8_t* m, int n, int ni,
                                     const double* Rt, const double* T, const PrK& K, double ifx, double ify,
                                     HomLds& hs, double* H) {
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
    float Mf[2], mf[2];
    for (int i = 0; i < n; i++) {
        if (!m[i]) continue;
        hom_pts(Xw, uv, i, Rt, T, K, ifx, ify, Mf, mf);
        cmx += mf[0];
        cmy += mf[1];
        cMx += Mf[0];
        cMy += Mf[1];
    }
    cmx /= ni;
    cmy /= ni;
    cMx /= ni;
    cMy /= ni;
    for (int i = 0; i < n; i++) {
        if (!m[i]) continue;
        hom_pts(Xw, uv, i, Rt, T, K, ifx, ify, Mf, mf);
        smx += fabs(mf[0] - cmx);
        smy += fabs(mf[1] - cmy);
        sMx += fabs(Mf[0] - cMx);
        sMy += fabs(Mf[1] - cMy);
    }
    if (fabs(smx) < DBL_EPSILON || fabs(smy) < DBL_EPSILON || fabs(sMx) < DBL_EPSILON || fabs(sMy) < DBL_EPSILON)
        return false;
    smx = ni / smx;
    smy = ni / smy;
    sMx = ni / sMx;
    sMy = ni / sMy;
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double* LtL = hs.a;
    for (int k = 0; k < 81; k++) LtL[k] = 0;
    for (int i = 0; i < n; i++) {
        if (!m[i]) continue;
        hom_pts(Xw, uv, i, Rt, T, K, ifx, ify, Mf, mf);
        const double x = (mf[0] - cmx) * smx, y = (mf[1] - cmy) * smy;
        const double X = (Mf[0] - cMx) * sMx, Y = (Mf[1] - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        for (int j = 0; j < 9; j++)
            for (int k = j; k < 9; k++) LtL[j * 9 + k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    for (int j = 0; j < 9; j++)
        for (int k = 0; k < j; k++) LtL[j * 9 + k] = LtL[k * 9 + j];
    svdj_lds(9, 9, hs.a, hs.v, hs.w, hs.U, hs.V, hs.ww, hs.ord);
    double H0[9], Ht[9];
    for (int k = 0; k < 9; k++) H0[k] = hs.V[k * 9 + 8];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++)
            Ht[r * 3 + c] = invHnorm[r * 3 + 0] * H0[0 * 3 + c] + invHnorm[r * 3 + 1] * H0[1 * 3 + c] +
                            invHnorm[r * 3 + 2] * H0[2 * 3 + c];
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++)
            H0[r * 3 + c] = Ht[r * 3 + 0] * Hnorm2[0 * 3 + c] + Ht[r * 3 + 1] * Hnorm2[1 * 3 + c] +
                            Ht[r * 3 + 2] * Hnorm2[2 * 3 + c];
    const double s22 = 1. / H0[8];
    for (int k = 0; k < 9; k++) H[k] = H0[k] * s22;
    if (ni <= 4) return true;
    // LMSolverImpl::run over h[0..7], streaming the residuals / Jacobian rows
    // (J^T J, J^T r, |r|^2 and max |r| in point order)
    double x8[8], xd[8], v[8], D[8], d[8];
    for (int k = 0; k < 8; k++) x8[k] = H[k];
    auto pass = [&](const double* h, bool withJ, double* S, double* rinf) {
        if (withJ) {
            for (int k = 0; k < 64; k++) hs.A[k] = 0;
            for (int k = 0; k < 8; k++) v[k] = 0;
        }
        double s2 = 0, mx = 0;
        for (int i = 0; i < n; i++) {
            if (!m[i]) continue;
            hom_pts(Xw, uv, i, Rt, T, K, ifx, ify, Mf, mf);
            const double Mx = Mf[0], My = Mf[1];
            double ww = h[6] * Mx + h[7] * My + 1.;
            ww = fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
            const double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
            const double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
            const double r0 = xi - mf[0], r1 = yi - mf[1];
            if (withJ) {
                const double Jx[8] = {Mx * ww, My * ww, ww, 0., 0., 0., -Mx * ww * xi, -My * ww * xi};
                const double Jy[8] = {0., 0., 0., Mx * ww, My * ww, ww, -Mx * ww * yi, -My * ww * yi};
                for (int a = 0; a < 8; a++) {
                    for (int b = 0; b < 8; b++) {
                        hs.A[a * 8 + b] += Jx[a] * Jx[b];
                        hs.A[a * 8 + b] += Jy[a] * Jy[b];
                    }
                    v[a] += Jx[a] * r0;
                    v[a] += Jy[a] * r1;
                }
            }
            s2 += r0 * r0;
            s2 += r1 * r1;
            mx = fmax(mx, fmax(fabs(r0), fabs(r1)));
        }
        *S = s2;
        if (rinf) *rinf = mx;
    };
    double S, rinf;
    pass(x8, true, &S, &rinf);
    for (int i = 0; i < 8; i++) D[i] = hs.A[i * 9];
    const double Rlo = 0.25, Rhi = 0.75;
    double lambda = 1, lc = 0.75;
    int iter = 0;
    for (;;) {
        for (int k = 0; k < 64; k++) hs.Ap[k] = hs.A[k];
        for (int i = 0; i < 8; i++) hs.Ap[i * 9] += lambda * D[i];
        svd_solve_lds(8, hs, v, d);
        for (int i = 0; i < 8; i++) xd[i] = x8[i] - d[i];
        double Sd;
        pass(xd, false, &Sd, nullptr);
        double dS = 0;
        for (int i = 0; i < 8; i++) {
            double t = 0;
            for (int k = 0; k < 8; k++) t += hs.A[i * 8 + k] * d[k];
            dS += d[i] * (2 * v[i] - t);
        }
        const double R = (S - Sd) / (fabs(dS) > DBL_EPSILON ? dS : 1);
        if (R > Rhi) {
            lambda *= 0.5;
            if (lambda < lc) lambda = 0;
        } else if (R < Rlo) {
            double t = 0;
            for (int i = 0; i < 8; i++) t += d[i] * v[i];
            double nu = (Sd - S) / (fabs(t) > DBL_EPSILON ? t : 1) + 2;
            nu = fmin(fmax(nu, 2.), 10.);
            if (lambda == 0) {
                for (int k = 0; k < 64; k++) hs.a[k] = hs.A[k];
                svdj_lds(8, 8, hs.a, hs.v, hs.w, hs.U, hs.V, hs.ww, hs.ord);
                const double thr = 8 * DBL_EPSILON * hs.w[0];
                double maxval = DBL_EPSILON;
                for (int i = 0; i < 8; i++) {
                    double dii = 0;
                    for (int k = 0; k < 8; k++)
                        if (hs.w[k] > thr) dii += hs.V[i * 8 + k] * hs.U[i * 8 + k] / hs.w[k];
                    maxval = fmax(maxval, fabs(dii));
                }
                lambda = lc = 1. / maxval;
                nu *= 0.5;
            }
            lambda *= nu;
        }
        if (Sd < S) {
            S = Sd;
            for (int k = 0; k < 8; k++) x8[k] = xd[k];
            pass(x8, true, &S, &rinf);
        }
        iter++;
        double dinf = 0;
        for (int i = 0; i < 8; i++) dinf = fmax(dinf, fabs(d[i]));
        if (!(iter < 10 && dinf >= FLT_EPSILON && rinf >= FLT_EPSILON)) break;
    }
    for (int k = 0; k < 8; k++) H[k] = x8[k];
    H[8] = 1.;
    return true;
}

// -> sp[0..5] = (rvec, tvec): the whole wave calls it. Returns false where
// cvFindExtrinsicCameraParams2's DLT branch asserts count >= 6 (non-planar
// points, ni = 5: solvePnPRansac accepts a model with goodCount > 4), i.e.
// where OpenCV throws cv::Exception out of solvePnPRansac.
__device__ bool extrinsic_init(const float* __restrict__ Xw, const float* __restrict__ uv,
                               const uint8_t* __restrict__ m, int n, int ni, const PrK& K, double* sp) {
    __shared__ double s_red[78];
    __shared__ double wred[1][78];
    __shared__ double s_mc[3];
    __shared__ int s_planar;
    __shared__ double s_Rt[9], s_T[3];
    __shared__ HomLds hs;
    const int lane = threadIdx.x;
    const double ifx = 1. / K.fx, ify = 1. / K.fy;
    {
        double v[3] = {0, 0, 0};
        for (int i = lane; i < n; i += PR_REFINE_THREADS) {
            if (!m[i]) continue;
            for (int k = 0; k < 3; k++) v[k] += (double)Xw[3 * i + k];
        }
        block_sum<3>(v, (double(*)[3])wred, s_red);
        if (lane < 3) s_mc[lane] = s_red[lane] / ni;
        __syncthreads();
    }
    const double Mc[3] = {s_mc[0], s_mc[1], s_mc[2]};
    {
        double v[6] = {0, 0, 0, 0, 0, 0};
        for (int i = lane; i < n; i += PR_REFINE_THREADS) {
            if (!m[i]) continue;
            const double d0 = (double)Xw[3 * i] - Mc[0], d1 = (double)Xw[3 * i + 1] - Mc[1],
                         d2 = (double)Xw[3 * i + 2] - Mc[2];
            v[0] += d0 * d0;
            v[1] += d0 * d1;
            v[2] += d0 * d2;
            v[3] += d1 * d1;
            v[4] += d1 * d2;
            v[5] += d2 * d2;
        }
        block_sum<6>(v, (double(*)[6])wred, s_red);
    }
    if (lane == 0) {
        const double MM[9] = {s_red[0], s_red[1], s_red[2], s_red[1], s_red[3], s_red[4], s_red[2], s_red[4], s_red[5]};
        double W[3], Um[9], Vm[9];
        svdj<3, 3>(MM, W, Um, Vm);
        s_planar = W[2] / W[1] < 1e-3;
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) s_Rt[r * 3 + c] = Vm[c * 3 + r];
    }
    __syncthreads();
    if (!s_planar && ni < 6) return false;  // CV_Assert(count >= 6) (calibration.cpp, DLT branch)
    double R[9], t[3];
    if (!s_planar) {
        double v[78];
        for (int k = 0; k < 78; k++) v[k] = 0;
        for (int i = lane; i < n; i += PR_REFINE_THREADS) {
            if (!m[i]) continue;
            const double x = -(((double)uv[2 * i] - K.cx) * ifx), y = -(((double)uv[2 * i + 1] - K.cy) * ify);
            const double X = Xw[3 * i], Y = Xw[3 * i + 1], Z = Xw[3 * i + 2];
            const double L1[12] = {X, Y, Z, 1., 0., 0., 0., 0., x * X, x * Y, x * Z, x};
            const double L2[12] = {0., 0., 0., 0., X, Y, Z, 1., y * X, y * Y, y * Z, y};
            int k = 0;
#pragma unroll
            for (int r = 0; r < 12; r++)
#pragma unroll
                for (int c = r; c < 12; c++, k++) {
                    v[k] += L1[r] * L1[c];
                    v[k] += L2[r] * L2[c];
                }
        }
        block_sum<78>(v, wred, s_red);
        if (lane == 0) {
            // row 11 of cvSVD(L^T L)'s V^T = the eigenvector of the smallest
            // eigenvalue, here by inverse iteration (the oracle runs the
            // Jacobi SVD of OpenCV's cvSVD; a 12 x 12 Jacobi is ~0.4 ms of
            // dependent sqrt / div chains on the GPU, this ~20 us): Cholesky
            // of L^T L + delta I (the shift keeps it positive definite on
            // noise-free data and leaves the eigenvectors unchanged), six
            // solves from a fixed start vector, unit norm; the sign is fixed
            // below by det(R) > 0 as in calibration.cpp. Agreement with the
            // oracle's refined pose: 1e-7 (tests/test_pnpransac.py).
            double* A = hs.a;  // 12 x 12 Cholesky factor (lower)
            double tr = 0;
            for (int r = 0; r < 12; r++) tr += s_red[r * 12 - r * (r - 1) / 2];
            const double delta = 1e-13 * tr + DBL_MIN;
            for (int r = 0; r < 12; r++)
                for (int c = 0; c <= r; c++) A[r * 12 + c] = s_red[c * 12 - c * (c - 1) / 2 + (r - c)] + (r == c ? delta : 0.0);
            for (int c = 0; c < 12; c++) {
                double d = A[c * 12 + c];
                for (int k = 0; k < c; k++) d -= A[c * 12 + k] * A[c * 12 + k];
                d = sqrt(fmax(d, DBL_MIN));
                A[c * 12 + c] = d;
                const double id = 1.0 / d;
                for (int r = c + 1; r < 12; r++) {
                    double e = A[r * 12 + c];
                    for (int k = 0; k < c; k++) e -= A[r * 12 + k] * A[c * 12 + k];
                    A[r * 12 + c] = e * id;
                }
            }
            double x[12];
            for (int k = 0; k < 12; k++) x[k] = 1.0 + 0.1 * k;  // fixed start
            for (int it = 0; it < 6; it++) {
                for (int r = 0; r < 12; r++) {  // L y = x
                    double e = x[r];
                    for (int k = 0; k < r; k++) e -= A[r * 12 + k] * x[k];
                    x[r] = e / A[r * 12 + r];
                }
                for (int r = 11; r >= 0; r--) {  // L^T z = y
                    double e = x[r];
                    for (int k = r + 1; k < 12; k++) e -= A[k * 12 + r] * x[k];
                    x[r] = e / A[r * 12 + r];
                }
                double nx = 0;
                for (int k = 0; k < 12; k++) nx += x[k] * x[k];
                nx = 1.0 / sqrt(nx);
                for (int k = 0; k < 12; k++) x[k] *= nx;
            }
            double RRt[12];
            for (int k = 0; k < 12; k++) RRt[k] = x[k];
            double RR[9] = {RRt[0], RRt[1], RRt[2], RRt[4], RRt[5], RRt[6], RRt[8], RRt[9], RRt[10]};
            if (det3d(RR) < 0) {
                for (int k = 0; k < 12; k++) RRt[k] = -RRt[k];
                for (int k = 0; k < 9; k++) RR[k] = -RR[k];
            }
            double sc = 0;
            for (int k = 0; k < 9; k++) sc += RR[k] * RR[k];
            sc = sqrt(sc);
            double w3[3], U3[9], V3[9];
            svdj<3, 3>(RR, w3, U3, V3);
            double nr = 0;
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++) {
                    R[r * 3 + c] =
                        U3[r * 3] * V3[c * 3] + U3[r * 3 + 1] * V3[c * 3 + 1] + U3[r * 3 + 2] * V3[c * 3 + 2];
                    nr += R[r * 3 + c] * R[r * 3 + c];
                }
            const double f = sqrt(nr) / sc;
            t[0] = RRt[3] * f;
            t[1] = RRt[7] * f;
            t[2] = RRt[11] * f;
        }
    } else if (lane == 0) {
        double Rt[9];
        for (int k = 0; k < 9; k++) Rt[k] = s_Rt[k];
        if (Rt[2] * Rt[2] + Rt[5] * Rt[5] < 1e-10)
            for (int k = 0; k < 9; k++) Rt[k] = k % 4 == 0 ? 1.0 : 0.0;
        if (det3d(Rt) < 0)
            for (int k = 0; k < 9; k++) Rt[k] = -Rt[k];
        double T[3];
        for (int r = 0; r < 3; r++) T[r] = -(Rt[r * 3] * Mc[0] + Rt[r * 3 + 1] * Mc[1] + Rt[r * 3 + 2] * Mc[2]);
        double h[9];
        bool okh = find_homography_lane(Xw, uv, m, n, ni, Rt, T, K, ifx, ify, hs, h);
        for (int k = 0; k < 9 && okh; k++) okh = isfinite(h[k]);
        if (okh) {
            const double h1n = sqrt(h[0] * h[0] + h[3] * h[3] + h[6] * h[6]);
            const double h2n = sqrt(h[1] * h[1] + h[4] * h[4] + h[7] * h[7]);
            const double s1 = 1. / fmax(h1n, DBL_EPSILON), s2 = 1. / fmax(h2n, DBL_EPSILON);
            const double s3 = 2. / fmax(h1n + h2n, DBL_EPSILON);
            double Hm[9];
            for (int r = 0; r < 3; r++) {
                Hm[r * 3] = h[r * 3] * s1;
                Hm[r * 3 + 1] = h[r * 3 + 1] * s2;
                t[r] = h[r * 3 + 2] * s3;
            }
            Hm[2] = Hm[3] * Hm[7] - Hm[6] * Hm[4];
            Hm[5] = Hm[6] * Hm[1] - Hm[0] * Hm[7];
            Hm[8] = Hm[0] * Hm[4] - Hm[3] * Hm[1];
            double rv[3], Hr[9];
            rod_m2v(Hm, rv);
            rod_v2m(rv, Hr, nullptr);
            for (int r = 0; r < 3; r++) t[r] = Hr[r * 3] * T[0] + Hr[r * 3 + 1] * T[1] + Hr[r * 3 + 2] * T[2] + t[r];
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++)
                    R[r * 3 + c] = Hr[r * 3] * Rt[c] + Hr[r * 3 + 1] * Rt[3 + c] + Hr[r * 3 + 2] * Rt[6 + c];
        } else {
            for (int k = 0; k < 9; k++) R[k] = k % 4 == 0 ? 1.0 : 0.0;
            t[0] = t[1] = t[2] = 0;
        }
    }
    if (lane == 0) {
        double r[3];
        rod_m2v(R, r);
        for (int k = 0; k < 3; k++) {
            sp[k] = r[k];
            sp[3 + k] = t[k];
        }
    }
    __syncthreads();
    return true;
}

__global__ __launch_bounds__(PR_REFINE_THREADS) void k_pr_refine(const float* __restrict__ Xw,
                                                                 const float* __restrict__ uv,
                                                                 const int* __restrict__ offs, int H, PrK K,
                                                                 const uint8_t* __restrict__ mask,
                                                                 const double* __restrict__ model,
                                                                 const int* __restrict__ state,
                                                                 odo_pnp_ransac_result* __restrict__ res,
                                                                 uint8_t* __restrict__ mask_out) {
    __shared__ double wred[PR_REFINE_THREADS / 64][43];
    __shared__ double red[43];
    __shared__ double sp[6], sprev[6];
    const int pb = blockIdx.x;
    const int n = offs[pb + 1] - offs[pb];
    Xw += 3 * (size_t)offs[pb];
    uv += 2 * (size_t)offs[pb];
    mask += (size_t)H * offs[pb];
    model += (size_t)pb * H * 6;
    state += 4 * pb;
    res += pb;
    mask_out += offs[pb];
    const int best = state[0];
    if (best < 0 || state[2] <= 0) {
        if (threadIdx.x == 0) {
            for (int k = 0; k < 3; k++) res->rvec[k] = res->tvec[k] = res->model_rvec[k] = res->model_tvec[k] = 0.0;
            for (int k = 0; k < 16; k++) res->Tcw[k] = 0.f;
            res->ok = 0;
            res->n_inliers = 0;
            res->best_iter = best;
            res->iterations_visited = state[1];
        }
        for (int i = threadIdx.x; i < n; i += PR_REFINE_THREADS) mask_out[i] = 0;
        return;
    }
    const uint8_t* m = mask + (size_t)best * n;
    for (int i = threadIdx.x; i < n; i += PR_REFINE_THREADS) mask_out[i] = m[i];
    // solvePnP(inliers, useExtrinsicGuess = false) (pnpransac.cpp:34): the
    // LM starts from cvFindExtrinsicCameraParams2's own pose, not the model
    if (!extrinsic_init(Xw, uv, m, n, state[2], K, sp)) {
        // the refinement would throw (non-planar inliers, fewer than 6): no
        // pose; the model, mask and counts are reported, ok = -1
        if (threadIdx.x == 0) {
            for (int k = 0; k < 3; k++) {
                res->rvec[k] = res->tvec[k] = 0.0;
                res->model_rvec[k] = model[6 * best + k];
                res->model_tvec[k] = model[6 * best + 3 + k];
            }
            for (int k = 0; k < 16; k++) res->Tcw[k] = 0.f;
            res->ok = -1;
            res->n_inliers = state[2];
            res->best_iter = best;
            res->iterations_visited = state[1];
        }
        return;
    }
    double lambdaLg10 = -3, prevErrNorm = DBL_MAX;
    double JtJ[36], JtErr[6];
    int iters = 0;
    for (;;) {
        double p[6];
        for (int k = 0; k < 6; k++) p[k] = sp[k];
        lm_pass(Xw, uv, m, n, K, p, true, wred, red);
        const double e0 = sqrt(red[42]);
        for (int k = 0; k < 36; k++) JtJ[k] = red[k];
        for (int k = 0; k < 6; k++) JtErr[k] = red[36 + k];
        for (int k = 0; k < 6; k++) p[k] = sp[k];  // prevParam
        // step(): param = prev - solve((JtJ with diag * (1 + lambda)), JtErr)
        auto step = [&]() {
            if (threadIdx.x == 0) {
                const double lambda = exp(lambdaLg10 * log(10.));
                double A[36], x[6];
                for (int k = 0; k < 36; k++) A[k] = JtJ[k];
                for (int i = 0; i < 6; i++) A[i * 7] *= 1. + lambda;
                svd_solve<6, 6>(A, JtErr, x);
                for (int i = 0; i < 6; i++) sp[i] = p[i] - x[i];
            }
            __syncthreads();
        };
        if (threadIdx.x < 6) sprev[threadIdx.x] = p[threadIdx.x];
        step();
        if (iters == 0) prevErrNorm = e0;
        double q[6];
        for (int k = 0; k < 6; k++) q[k] = sp[k];
        lm_pass(Xw, uv, m, n, K, q, false, wred, red);
        double errNorm = sqrt(red[42]);
        while (errNorm > prevErrNorm && ++lambdaLg10 <= 16) {
            step();
            for (int k = 0; k < 6; k++) q[k] = sp[k];
            lm_pass(Xw, uv, m, n, K, q, false, wred, red);
            errNorm = sqrt(red[42]);
        }
        lambdaLg10 = lambdaLg10 - 1 > -16 ? lambdaLg10 - 1 : -16;
        double dn = 0, pn = 0;
        for (int i = 0; i < 6; i++) {
            dn += (sp[i] - sprev[i]) * (sp[i] - sprev[i]);
            pn += sprev[i] * sprev[i];
        }
        if (++iters >= 20 || sqrt(dn) / (sqrt(pn) + DBL_EPSILON) < FLT_EPSILON) break;
        prevErrNorm = errNorm;
    }
    if (threadIdx.x == 0) {
        double R[9];
        double p[6];
        for (int k = 0; k < 6; k++) p[k] = sp[k];
        rod_v2m(p, R, nullptr);
        for (int k = 0; k < 3; k++) {
            res->rvec[k] = p[k];
            res->tvec[k] = p[3 + k];
            res->model_rvec[k] = model[6 * best + k];
            res->model_tvec[k] = model[6 * best + 3 + k];
        }
        for (int r = 0; r < 3; r++) {
            for (int k = 0; k < 3; k++) res->Tcw[4 * r + k] = (float)R[3 * r + k];
            res->Tcw[4 * r + 3] = (float)p[3 + r];
        }
        res->Tcw[12] = res->Tcw[13] = res->Tcw[14] = 0.f;
        res->Tcw[15] = 1.f;
        res->ok = 1;
        res->n_inliers = state[2];
        res->best_iter = best;
        res->iterations_visited = state[1];
    }
}

}  // namespace

int pnp_ransac_max_points() { return 1 << 16; }

// One problem: every hypothesis at once (the per-hypothesis chains are the
// latency). A batch: chunks of PR_CHUNK hypotheses, each chunk's EPnP and
// counts skipping the problems whose fold has already stopped, so the work
// follows the visited hypotheses (typically a fraction of `iterations`).
constexpr int PR_CHUNK = 64;
void launch_pnp_ransac(hipStream_t st, const float* Xw, const float* uv, const int* offs, int nprob,
                       const float K4[4], int H, float reproj_err, double confidence, int* idx, double* model,
                       double* Rproj, uint8_t* mask, int* good, int* state, odo_pnp_ransac_result* res,
                       uint8_t* mask_out) {
    const PrK K{(double)K4[0], (double)K4[1], (double)K4[2], (double)K4[3]};
    const float thr = (float)((double)reproj_err * (double)reproj_err);
    const int pblocks = (nprob + 63) / 64;
    hipLaunchKernelGGL(k_pr_subsets, dim3(pblocks), dim3(PR_RNG_THREADS), 0, st, offs, nprob, H, idx);
    const int hyp_per_block = PR_EPNP_THREADS / PR_EPNP_GROUP;
    const int chunk = nprob > 1 ? PR_CHUNK : H;
    for (int h0 = 0; h0 < H; h0 += chunk) {
        const int h1 = h0 + chunk < H ? h0 + chunk : H;
        const int* fs = h0 == 0 ? nullptr : state;
        hipLaunchKernelGGL(k_pr_epnp, dim3((h1 - h0 + hyp_per_block - 1) / hyp_per_block, nprob),
                           dim3(PR_EPNP_THREADS), 0, st, Xw, uv, offs, idx, H, h0, h1, fs, K, model, Rproj);
        hipLaunchKernelGGL(k_pr_count, dim3(h1 - h0, nprob), dim3(PR_COUNT_THREADS), 0, st, Xw, uv, offs, H, h0, fs,
                           K, thr, model, Rproj, mask, good);
        hipLaunchKernelGGL(k_pr_fold, dim3(pblocks), dim3(64), 0, st, good, offs, nprob, H, h0, h1, confidence,
                           state);
    }
    hipLaunchKernelGGL(k_pr_refine, dim3(nprob), dim3(PR_REFINE_THREADS), 0, st, Xw, uv, offs, H, K, mask, model,
                       state, res, mask_out);
}

}  // namespace odo
