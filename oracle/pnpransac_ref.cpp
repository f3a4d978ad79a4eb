// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). CPU restatement of
//   PnPRansac::Compute                        Odometry/pnpransac.cpp:11-51
// i.e. cv::solvePnPRansac(v3D, v2D, mK, noDist, r, t, false, 500, 3.0f, 0.85,
// inliers) of OpenCV 3.4 (calib3d: solvepnp.cpp, ptsetreg.cpp
// RANSACPointSetRegistrator, epnp.cpp, calibration.cpp cvProjectPoints2 /
// cvRodrigues2 / cvFindExtrinsicCameraParams2 + CvLevMarq). OpenCV is absent
// from this image: its internals are restated from its published source as
// recalled (parity UNPINNED, like every OpenCV boundary here). Pinned choices
// (DESIGN.md §4 "PnPRansac"):
//   * the EPnP kernel takes the keypoints in pixels (undistortPoints with
//     P = K and no distortion is the identity map);
//   * cvSVD / cvSolve(CV_SVD) / cvInvert(CV_SVD) are one-sided (Hestenes)
//     Jacobi SVDs in double, singular values sorted descending;
//   * the final refinement is solvePnP(inliers, SOLVEPNP_ITERATIVE,
//     useExtrinsicGuess = false), as pnpransac.cpp:34 passes false: OpenCV
//     3.4's solvePnPRansac hands the inliers to solvePnP with the caller's
//     flag, so cvFindExtrinsicCameraParams2 builds its own start (extrinsic_init:
//     DLT for non-planar point sets, the homography decomposition for planar
//     ones) and CvLevMarq refines from there; its 6x6 damped normal equations
//     are solved with the same SVD (solve(..., DECOMP_SVD));
//   * sums over the inlier points run in the GPU's order (lane i % 64 of one
//     wave accumulates point i, then a shuffle-down tree: wsum64), and the
//     12 x 12 DLT eigenproblem uses svdj12 (tree16), as the EPnP one.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

// ---------------------------------------------------------------- cv::RNG
struct CvRng {
    uint64_t state;
    unsigned next() {
        state = (uint64_t)(unsigned)state * 4164903690U + (unsigned)(state >> 32);
        return (unsigned)state;
    }
    int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + a); }
};

// ------------------------------------------- one-sided Jacobi SVD (double)
// A (m x n, m >= n, row-major) = U diag(w) V^T; w descending; U m x n, V n x n
// (columns). Used for every cvSVD / cvSolve / cvInvert of the path.
void svdj(int m, int n, const double* A, double* w, double* U, double* V) {
    double a[12 * 12], v[12 * 12];
    memcpy(a, A, sizeof(double) * m * n);
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
                if (gamma == 0.0 || std::fabs(gamma) <= DBL_EPSILON * std::sqrt(alpha * beta)) continue;
                changed = 1;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
                for (int i = 0; i < m; i++) {
                    const double ap = a[i * n + p], aq = a[i * n + q];
                    a[i * n + p] = c * ap - s * aq;
                    a[i * n + q] = s * ap + c * aq;
                }
                for (int i = 0; i < n; i++) {
                    const double vp = v[i * n + p], vq = v[i * n + q];
                    v[i * n + p] = c * vp - s * vq;
                    v[i * n + q] = s * vp + c * vq;
                }
            }
        if (!changed) break;
    }
    double ww[12];
    for (int j = 0; j < n; j++) {
        double s = 0;
        for (int i = 0; i < m; i++) s += a[i * n + j] * a[i * n + j];
        ww[j] = std::sqrt(s);
    }
    int ord[12];
    for (int j = 0; j < n; j++) ord[j] = j;
    for (int j = 0; j < n; j++) {  // selection sort, descending, first maximum wins
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
        for (int i = 0; i < m; i++) U[i * n + j] = a[i * n + c] * inv;
        for (int i = 0; i < n; i++) V[i * n + j] = v[i * n + c];
    }
}

// The sum of 12 row values as the GPU's 16-lane xor butterfly forms it on its
// first lane (rows 12..15 are zero): ((x0+x8)+(x4+x12)) + ((x2+x10)+(x6+x14))
// + ... — the summation order of the 12 x 12 EPnP eigenproblem (pinned choice).
double tree16(const double* x) {
    double y[16];
    for (int i = 0; i < 16; i++) y[i] = i < 12 ? x[i] : 0.0;
    for (int o = 8; o >= 1; o >>= 1) {
        double z[16];
        for (int i = 0; i < 16; i++) z[i] = y[i] + y[i ^ o];
        memcpy(y, z, sizeof(y));
    }
    return y[0];
}

// svdj for the 12 x 12 M^T M with tree16 column sums; V only.
void svdj12(const double* A, double* w, double* V) {
    double a[144], v[144];
    memcpy(a, A, sizeof(a));
    for (int i = 0; i < 12; i++)
        for (int j = 0; j < 12; j++) v[i * 12 + j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; sweep++) {
        int changed = 0;
        for (int p = 0; p < 11; p++)
            for (int q = p + 1; q < 12; q++) {
                double pp[12], qq[12], pq[12];
                for (int i = 0; i < 12; i++) {
                    const double ap = a[i * 12 + p], aq = a[i * 12 + q];
                    pp[i] = ap * ap;
                    qq[i] = aq * aq;
                    pq[i] = ap * aq;
                }
                const double alpha = tree16(pp), beta = tree16(qq), gamma = tree16(pq);
                if (gamma == 0.0 || std::fabs(gamma) <= DBL_EPSILON * std::sqrt(alpha * beta)) continue;
                changed = 1;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
                for (int i = 0; i < 12; i++) {
                    const double ap = a[i * 12 + p], aq = a[i * 12 + q];
                    a[i * 12 + p] = c * ap - s * aq;
                    a[i * 12 + q] = s * ap + c * aq;
                }
                for (int i = 0; i < 12; i++) {
                    const double vp = v[i * 12 + p], vq = v[i * 12 + q];
                    v[i * 12 + p] = c * vp - s * vq;
                    v[i * 12 + q] = s * vp + c * vq;
                }
            }
        if (!changed) break;
    }
    double ww[12];
    for (int j = 0; j < 12; j++) {
        double sq[12];
        for (int i = 0; i < 12; i++) sq[i] = a[i * 12 + j] * a[i * 12 + j];
        ww[j] = std::sqrt(tree16(sq));
    }
    int ord[12];
    for (int j = 0; j < 12; j++) ord[j] = j;
    for (int j = 0; j < 12; j++) {
        int b = j;
        for (int k = j + 1; k < 12; k++)
            if (ww[ord[k]] > ww[ord[b]]) b = k;
        const int t = ord[j];
        ord[j] = ord[b];
        ord[b] = t;
    }
    for (int j = 0; j < 12; j++) {
        w[j] = ww[ord[j]];
        for (int i = 0; i < 12; i++) V[i * 12 + j] = v[i * 12 + ord[j]];
    }
}

// cvSolve(A, b, x, CV_SVD) for m x n (m >= n): x = V diag(1/w) U^T b over
// singular values above n * DBL_EPSILON * w[0].
void svd_solve(int m, int n, const double* A, const double* b, double* x) {
    double w[12], U[12 * 12], V[12 * 12];
    svdj(m, n, A, w, U, V);
    const double thr = n * DBL_EPSILON * w[0];
    double y[12];
    for (int j = 0; j < n; j++) {
        double s = 0;
        for (int i = 0; i < m; i++) s += U[i * n + j] * b[i];
        y[j] = w[j] > thr ? s / w[j] : 0.0;
    }
    for (int i = 0; i < n; i++) {
        double s = 0;
        for (int j = 0; j < n; j++) s += V[i * n + j] * y[j];
        x[i] = s;
    }
}

inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// ------------------------------------------------------------ cvRodrigues2
// vector -> matrix (+ 3x9 jacobian dRdr[i*9+k] = dR_k/dr_i), calibration.cpp
void rodrigues_v2m(const double r[3], double R[9], double* J) {
    const double theta = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (theta < DBL_EPSILON) {
        for (int k = 0; k < 9; k++) R[k] = k % 4 == 0 ? 1.0 : 0.0;
        if (J) {
            static const double J0[27] = {0, 0, 0, 0, 0, 1, 0, -1, 0, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 1, 0, -1, 0, 0, 0, 0, 0};
            memcpy(J, J0, sizeof(J0));
        }
        return;
    }
    const double c = std::cos(theta), s = std::sin(theta), c1 = 1. - c;
    const double itheta = theta ? 1. / theta : 0.;
    const double rx = r[0] * itheta, ry = r[1] * itheta, rz = r[2] * itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rx_[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    static const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    for (int k = 0; k < 9; k++) R[k] = c * I[k] + c1 * rrt[k] + s * rx_[k];
    if (J) {
        const double drrt[27] = {rx + rx, ry, rz, ry, 0, 0, rz, 0, 0, 0, rx, 0, rx, ry + ry, rz, 0, rz, 0,
                                 0, 0, rx, 0, 0, ry, rx, ry, rz + rz};
        static const double drx_[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0,
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

// matrix -> vector (R re-orthonormalised as U V^T first)
void rodrigues_m2v(const double Rin[9], double r[3]) {
    double w[3], U[9], V[9], R[9];
    svdj(3, 3, Rin, w, U, V);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i * 3 + j] = U[i * 3 + 0] * V[j * 3 + 0] + U[i * 3 + 1] * V[j * 3 + 1] + U[i * 3 + 2] * V[j * 3 + 2];
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = std::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t = (R[0] + 1) * 0.5;
            rx = std::sqrt(t > 0 ? t : 0.);
            t = (R[4] + 1) * 0.5;
            ry = std::sqrt(t > 0 ? t : 0.) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = std::sqrt(t > 0 ? t : 0.) * (R[2] < 0 ? -1. : 1.);
            if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
            theta /= std::sqrt(rx * rx + ry * ry + rz * rz);
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

// cvProjectPoints2 of one point, zero distortion: (u, v) and optionally the
// rows du/d(r,t), dv/d(r,t) (R and dRdr from rodrigues_v2m of the same r).
inline void project_pt(const double R[9], const double* dRdr, const double t[3], const double K[4], const double M[3],
                       double* u, double* v, double* Ju, double* Jv) {
    const double X = M[0], Y = M[1], Z = M[2];
    double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    z = z ? 1. / z : 1;
    x *= z;
    y *= z;
    *u = x * K[0] + K[2];
    *v = y * K[1] + K[3];
    if (Ju) {
        const double dxdt[3] = {z, 0, -x * z}, dydt[3] = {0, z, -y * z};
        for (int j = 0; j < 3; j++) {
            Ju[3 + j] = K[0] * dxdt[j];
            Jv[3 + j] = K[1] * dydt[j];
        }
        for (int j = 0; j < 3; j++) {
            const double* d = dRdr + 9 * j;
            const double dx0 = X * d[0] + Y * d[1] + Z * d[2];
            const double dy0 = X * d[3] + Y * d[4] + Z * d[5];
            const double dz0 = X * d[6] + Y * d[7] + Z * d[8];
            const double dxdr = z * (dx0 - x * dz0), dydr = z * (dy0 - y * dz0);
            Ju[j] = K[0] * dxdr;
            Jv[j] = K[1] * dydr;
        }
    }
}

// -------------------------------------------------------------- epnp.cpp
struct Epnp {
    int n;
    const double* pws;  // n x 3
    const double* us;   // n x 2
    double fu, fv, uc, vc;
    double alphas[4 * 64], pcs[3 * 64];
    double cws[4][3], ccs[4][3];

    void choose_control_points() {
        cws[0][0] = cws[0][1] = cws[0][2] = 0;
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) cws[0][j] += pws[3 * i + j];
        for (int j = 0; j < 3; j++) cws[0][j] /= n;
        double PtP[9] = {0};
        for (int i = 0; i < n; i++) {  // cvMulTransposed(PW0, PW0tPW0, 1)
            double d[3];
            for (int j = 0; j < 3; j++) d[j] = pws[3 * i + j] - cws[0][j];
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) PtP[a * 3 + b] += d[a] * d[b];
        }
        double dc[3], U[9], V[9];
        svdj(3, 3, PtP, dc, U, V);
        for (int i = 1; i < 4; i++) {
            const double k = std::sqrt(dc[i - 1] / n);
            for (int j = 0; j < 3; j++) cws[i][j] = cws[0][j] + k * V[j * 3 + (i - 1)];  // uct row i-1 (symmetric: V)
        }
    }
    void compute_barycentric_coordinates() {
        double cc[9], w[3], U[9], V[9], ci[9];
        for (int i = 0; i < 3; i++)
            for (int j = 1; j < 4; j++) cc[3 * i + j - 1] = cws[j][i] - cws[0][i];
        svdj(3, 3, cc, w, U, V);  // cvInvert(CC, CC_inv, CV_SVD): V diag(1/w) U^T
        const double thr = 3 * DBL_EPSILON * w[0];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                double s = 0;
                for (int k = 0; k < 3; k++) s += V[i * 3 + k] * (w[k] > thr ? 1.0 / w[k] : 0.0) * U[j * 3 + k];
                ci[i * 3 + j] = s;
            }
        for (int i = 0; i < n; i++) {
            const double* pi = pws + 3 * i;
            double* a = alphas + 4 * i;
            for (int j = 0; j < 3; j++)
                a[1 + j] = ci[3 * j] * (pi[0] - cws[0][0]) + ci[3 * j + 1] * (pi[1] - cws[0][1]) +
                           ci[3 * j + 2] * (pi[2] - cws[0][2]);
            a[0] = 1.0f - a[1] - a[2] - a[3];
        }
    }
    void compute_ccs(const double* betas, const double* ut) {
        for (int i = 0; i < 4; i++) ccs[i][0] = ccs[i][1] = ccs[i][2] = 0.0f;
        for (int i = 0; i < 4; i++) {
            const double* v = ut + 12 * (11 - i);
            for (int j = 0; j < 4; j++)
                for (int k = 0; k < 3; k++) ccs[j][k] += betas[i] * v[3 * j + k];
        }
    }
    void compute_pcs() {
        for (int i = 0; i < n; i++) {
            const double* a = alphas + 4 * i;
            double* pc = pcs + 3 * i;
            for (int j = 0; j < 3; j++) pc[j] = a[0] * ccs[0][j] + a[1] * ccs[1][j] + a[2] * ccs[2][j] + a[3] * ccs[3][j];
        }
    }
    void solve_for_sign() {
        if (pcs[2] < 0.0) {
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 3; j++) ccs[i][j] = -ccs[i][j];
            for (int i = 0; i < 3 * n; i++) pcs[i] = -pcs[i];
        }
    }
    void estimate_R_and_t(double R[3][3], double t[3]) {
        double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
        for (int i = 0; i < n; i++)
            for (int j = 0; j < 3; j++) {
                pc0[j] += pcs[3 * i + j];
                pw0[j] += pws[3 * i + j];
            }
        for (int j = 0; j < 3; j++) {
            pc0[j] /= n;
            pw0[j] /= n;
        }
        double abt[9] = {0};
        for (int i = 0; i < n; i++) {
            const double* pc = pcs + 3 * i;
            const double* pw = pws + 3 * i;
            for (int j = 0; j < 3; j++) {
                abt[3 * j] += (pc[j] - pc0[j]) * (pw[0] - pw0[0]);
                abt[3 * j + 1] += (pc[j] - pc0[j]) * (pw[1] - pw0[1]);
                abt[3 * j + 2] += (pc[j] - pc0[j]) * (pw[2] - pw0[2]);
            }
        }
        double d[3], u[9], v[9];
        svdj(3, 3, abt, d, u, v);
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
    }
    double reprojection_error(const double R[3][3], const double t[3]) {
        double sum2 = 0.0;
        for (int i = 0; i < n; i++) {
            const double* pw = pws + 3 * i;
            const double Xc = dot3(R[0], pw) + t[0], Yc = dot3(R[1], pw) + t[1];
            const double inv_Zc = 1.0 / (dot3(R[2], pw) + t[2]);
            const double ue = uc + fu * Xc * inv_Zc, ve = vc + fv * Yc * inv_Zc;
            const double u = us[2 * i], v = us[2 * i + 1];
            sum2 += std::sqrt((u - ue) * (u - ue) + (v - ve) * (v - ve));
        }
        return sum2 / n;
    }
    double compute_R_and_t(const double* ut, const double* betas, double R[3][3], double t[3]) {
        compute_ccs(betas, ut);
        compute_pcs();
        solve_for_sign();
        estimate_R_and_t(R, t);
        return reprojection_error(R, t);
    }
    static void compute_L_6x10(const double* ut, double* l) {
        const double* v[4] = {ut + 12 * 11, ut + 12 * 10, ut + 12 * 9, ut + 12 * 8};
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
    static double dist2(const double* a, const double* b) {
        return (a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]);
    }
    void compute_rho(double* rho) {
        rho[0] = dist2(cws[0], cws[1]);
        rho[1] = dist2(cws[0], cws[2]);
        rho[2] = dist2(cws[0], cws[3]);
        rho[3] = dist2(cws[1], cws[2]);
        rho[4] = dist2(cws[1], cws[3]);
        rho[5] = dist2(cws[2], cws[3]);
    }
    static void betas_approx(const double* l, const double* rho, int which, double* betas) {
        static const int cols1[4] = {0, 1, 3, 6}, cols2[3] = {0, 1, 2}, cols3[5] = {0, 1, 2, 3, 4};
        const int nc = which == 1 ? 4 : which == 2 ? 3 : 5;
        const int* cols = which == 1 ? cols1 : which == 2 ? cols2 : cols3;
        double L[6 * 5], b[5];
        for (int i = 0; i < 6; i++)
            for (int j = 0; j < nc; j++) L[i * nc + j] = l[10 * i + cols[j]];
        svd_solve(6, nc, L, rho, b);
        if (which == 1) {
            if (b[0] < 0) {
                betas[0] = std::sqrt(-b[0]);
                betas[1] = -b[1] / betas[0];
                betas[2] = -b[2] / betas[0];
                betas[3] = -b[3] / betas[0];
            } else {
                betas[0] = std::sqrt(b[0]);
                betas[1] = b[1] / betas[0];
                betas[2] = b[2] / betas[0];
                betas[3] = b[3] / betas[0];
            }
            return;
        }
        if (b[0] < 0) {
            betas[0] = std::sqrt(-b[0]);
            betas[1] = (b[2] < 0) ? std::sqrt(-b[2]) : 0.0;
        } else {
            betas[0] = std::sqrt(b[0]);
            betas[1] = (b[2] > 0) ? std::sqrt(b[2]) : 0.0;
        }
        if (b[1] < 0) betas[0] = -betas[0];
        betas[2] = which == 3 ? b[3] / betas[0] : 0.0;
        betas[3] = 0.0;
    }
    // qr_solve of epnp.cpp (Householder, including its eta scan of the column)
    static void qr_solve(double* A, double* b, double* X) {
        const int nr = 6, nc = 4;
        double A1[6], A2[6];
        double* pA = A;
        double* ppAkk = pA;
        for (int k = 0; k < nc; k++) {
            double* ppAik = ppAkk;
            double eta = std::fabs(*ppAik);
            for (int i = k + 1; i < nr; i++) {
                const double elt = std::fabs(*ppAik);
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
            double sigma = std::sqrt(sum);
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
            ppAkk += nc + 1;
        }
        double* ppAjj = pA;
        for (int j = 0; j < nc; j++) {
            double* p = ppAjj;
            double tau = 0;
            for (int i = j; i < nr; i++) {
                tau += *p * b[i];
                p += nc;
            }
            tau /= A1[j];
            p = ppAjj;
            for (int i = j; i < nr; i++) {
                b[i] -= tau * *p;
                p += nc;
            }
            ppAjj += nc + 1;
        }
        X[nc - 1] = b[nc - 1] / A2[nc - 1];
        for (int i = nc - 2; i >= 0; i--) {
            const double* p = pA + i * nc + (i + 1);
            double s = 0;
            for (int j = i + 1; j < nc; j++) {
                s += *p * X[j];
                p++;
            }
            X[i] = (b[i] - s) / A2[i];
        }
    }
    static void gauss_newton(const double* l, const double* rho, double* betas) {
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
    void compute_pose(double R[3][3], double t[3]) {
        choose_control_points();
        compute_barycentric_coordinates();
        std::vector<double> M((size_t)2 * n * 12);
        for (int i = 0; i < n; i++) {  // fill_M
            const double* as = alphas + 4 * i;
            double* M1 = M.data() + (size_t)(2 * i) * 12;
            double* M2 = M1 + 12;
            const double u = us[2 * i], v = us[2 * i + 1];
            for (int j = 0; j < 4; j++) {
                M1[3 * j] = as[j] * fu;
                M1[3 * j + 1] = 0.0;
                M1[3 * j + 2] = as[j] * (uc - u);
                M2[3 * j] = 0.0;
                M2[3 * j + 1] = as[j] * fv;
                M2[3 * j + 2] = as[j] * (vc - v);
            }
        }
        double mtm[144] = {0};
        for (int r = 0; r < 2 * n; r++)  // cvMulTransposed(M, MtM, 1)
            for (int a = 0; a < 12; a++)
                for (int b = 0; b < 12; b++) mtm[a * 12 + b] += M[(size_t)r * 12 + a] * M[(size_t)r * 12 + b];
        double d[12], V[144], ut[144];
        svdj12(mtm, d, V);
        for (int i = 0; i < 12; i++)
            for (int j = 0; j < 12; j++) ut[i * 12 + j] = V[j * 12 + i];  // symmetric PSD: U = V
        double l[60], rho[6];
        compute_L_6x10(ut, l);
        compute_rho(rho);
        double Betas[4][4], rep[4], Rs[4][3][3], ts[4][3];
        for (int w = 1; w <= 3; w++) {
            betas_approx(l, rho, w, Betas[w]);
            gauss_newton(l, rho, Betas[w]);
            rep[w] = compute_R_and_t(ut, Betas[w], Rs[w], ts[w]);
        }
        int N = 1;
        if (rep[2] < rep[1]) N = 2;
        if (rep[3] < rep[N]) N = 3;
        memcpy(R, Rs[N], sizeof(Rs[N]));
        memcpy(t, ts[N], sizeof(ts[N]));
    }
};

// ---------------------------------------------- RANSACUpdateNumIters (ptsetreg.cpp)
int update_num_iters(double p, double ep, int modelPoints, int maxIters) {
    p = p > 0. ? p : 0.;
    p = p < 1. ? p : 1.;
    ep = ep > 0. ? ep : 0.;
    ep = ep < 1. ? ep : 1.;
    double num = 1. - p > DBL_MIN ? 1. - p : DBL_MIN;
    double denom = 1. - std::pow(1. - ep, modelPoints);
    if (denom < DBL_MIN) return 0;
    num = std::log(num);
    denom = std::log(denom);
    return denom >= 0 || -num >= maxIters * (-denom) ? maxIters : (int)lrint(num / denom);
}

// The RANSAC model of one minimal set: solvePnP(EPNP) -> (rvec, tvec)
void epnp_model(const double* pw, const double* uv, int n, const double K[4], double model[6]) {
    Epnp e;
    e.n = n;
    e.pws = pw;
    e.us = uv;
    e.fu = K[0];
    e.fv = K[1];
    e.uc = K[2];
    e.vc = K[3];
    double R[3][3], t[3];
    e.compute_pose(R, t);
    rodrigues_m2v(&R[0][0], model);
    model[3] = t[0];
    model[4] = t[1];
    model[5] = t[2];
}

// cvFindExtrinsicCameraParams2 with useExtrinsicGuess: CvLevMarq(6, 2n,
// (EPS+ITER, 20, FLT_EPSILON)) over cvProjectPoints2 residuals.
void refine_lm(const double* M, const double* m, int n, const double K[4], double param[6]) {
    double prev[6], JtJ[36], JtErr[6];
    double lambdaLg10 = -3, prevErrNorm = DBL_MAX;
    int iters = 0;
    auto residuals = [&](const double* p, bool withJ) -> double {
        double R[9], dRdr[27];
        rodrigues_v2m(p, R, withJ ? dRdr : nullptr);
        if (withJ) {
            memset(JtJ, 0, sizeof(JtJ));
            memset(JtErr, 0, sizeof(JtErr));
        }
        double e2 = 0;
        for (int i = 0; i < n; i++) {
            double u, v, Ju[6], Jv[6];
            project_pt(R, dRdr, p + 3, K, M + 3 * i, &u, &v, withJ ? Ju : nullptr, withJ ? Jv : nullptr);
            const double eu = u - m[2 * i], ev = v - m[2 * i + 1];
            e2 += eu * eu;
            e2 += ev * ev;
            if (withJ)
                for (int a = 0; a < 6; a++) {
                    for (int b = 0; b < 6; b++) {
                        JtJ[a * 6 + b] += Ju[a] * Ju[b];
                        JtJ[a * 6 + b] += Jv[a] * Jv[b];
                    }
                    JtErr[a] += Ju[a] * eu;
                    JtErr[a] += Jv[a] * ev;
                }
        }
        return std::sqrt(e2);
    };
    auto step = [&]() {
        const double lambda = std::exp(lambdaLg10 * std::log(10.));
        double A[36], x[6];
        memcpy(A, JtJ, sizeof(A));
        for (int i = 0; i < 6; i++) A[i * 7] *= 1. + lambda;
        svd_solve(6, 6, A, JtErr, x);
        for (int i = 0; i < 6; i++) param[i] = prev[i] - x[i];
    };
    for (;;) {
        // CALC_J
        const double e0 = residuals(param, true);
        memcpy(prev, param, sizeof(prev));
        step();
        if (iters == 0) prevErrNorm = e0;
        // CHECK_ERR
        double errNorm = residuals(param, false);
        while (errNorm > prevErrNorm && ++lambdaLg10 <= 16) {
            step();
            errNorm = residuals(param, false);
        }
        lambdaLg10 = lambdaLg10 - 1 > -16 ? lambdaLg10 - 1 : -16;
        double dn = 0, pn = 0;
        for (int i = 0; i < 6; i++) {
            dn += (param[i] - prev[i]) * (param[i] - prev[i]);
            pn += prev[i] * prev[i];
        }
        if (++iters >= 20 || std::sqrt(dn) / (std::sqrt(pn) + DBL_EPSILON) < FLT_EPSILON) break;
        prevErrNorm = errNorm;
    }
}

// ----------------------------------- sums in the GPU's one-wave order
// K running sums over n items: item i is added on lane i % 64 (in item
// order), then lanes combine with the shuffle-down tree (offsets 32 .. 1) and
// lane 0 holds the total (k_pnpransac.hip block_sum / wave_sums).
struct WSum64 {
    int K;
    std::vector<double> acc;  // [64][K]
    explicit WSum64(int k) : K(k), acc(64 * (size_t)k, 0.0) {}
    double* lane(int key) { return &acc[(size_t)(key & 63) * K]; }
    void total(double* out) {
        for (int o = 32; o > 0; o >>= 1)
            for (int l = 0; l < o; l++)
                for (int k = 0; k < K; k++) acc[(size_t)l * K + k] += acc[(size_t)(l + o) * K + k];
        for (int k = 0; k < K; k++) out[k] = acc[k];
    }
};

inline double det3(const double* a) {
    return a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) + a[2] * (a[3] * a[7] - a[4] * a[6]);
}

// cv::findHomography(src, dst, 0) on float points (findHomography converts
// its inputs to CV_32F): HomographyEstimatorCallback::runKernel (normalised
// DLT: centroids, mean absolute deviations, 9 x 9 LtL, eigenvector of the
// smallest eigenvalue, denormalised, scaled to h22 = 1), then LMSolver with
// HomographyRefineCallback (8 parameters, 10 iterations, epsx = epsf =
// FLT_EPSILON; solve / invert with DECOMP_EIG taken as the SVD solve).
// Returns false when the kernel fails (degenerate spread).
bool find_homography(const float* M, const float* m, int n, double H[9]) {
    double cMx = 0, cMy = 0, cmx = 0, cmy = 0, sMx = 0, sMy = 0, smx = 0, smy = 0;
    for (int i = 0; i < n; i++) {
        cmx += m[2 * i];
        cmy += m[2 * i + 1];
        cMx += M[2 * i];
        cMy += M[2 * i + 1];
    }
    cmx /= n;
    cmy /= n;
    cMx /= n;
    cMy /= n;
    for (int i = 0; i < n; i++) {
        smx += std::fabs(m[2 * i] - cmx);
        smy += std::fabs(m[2 * i + 1] - cmy);
        sMx += std::fabs(M[2 * i] - cMx);
        sMy += std::fabs(M[2 * i + 1] - cMy);
    }
    if (std::fabs(smx) < DBL_EPSILON || std::fabs(smy) < DBL_EPSILON || std::fabs(sMx) < DBL_EPSILON ||
        std::fabs(sMy) < DBL_EPSILON)
        return false;
    smx = n / smx;
    smy = n / smy;
    sMx = n / sMx;
    sMy = n / sMy;
    const double invHnorm[9] = {1. / smx, 0, cmx, 0, 1. / smy, cmy, 0, 0, 1};
    const double Hnorm2[9] = {sMx, 0, -cMx * sMx, 0, sMy, -cMy * sMy, 0, 0, 1};
    double LtL[81] = {0};
    for (int i = 0; i < n; i++) {
        const double x = (m[2 * i] - cmx) * smx, y = (m[2 * i + 1] - cmy) * smy;
        const double X = (M[2 * i] - cMx) * sMx, Y = (M[2 * i + 1] - cMy) * sMy;
        const double Lx[9] = {X, Y, 1, 0, 0, 0, -x * X, -x * Y, -x};
        const double Ly[9] = {0, 0, 0, X, Y, 1, -y * X, -y * Y, -y};
        for (int j = 0; j < 9; j++)
            for (int k = j; k < 9; k++) LtL[j * 9 + k] += Lx[j] * Lx[k] + Ly[j] * Ly[k];
    }
    for (int j = 0; j < 9; j++)
        for (int k = 0; k < j; k++) LtL[j * 9 + k] = LtL[k * 9 + j];
    double w[9], U[81], V[81];
    svdj(9, 9, LtL, w, U, V);  // eigen() of the symmetric PSD LtL: eigenvalues descending
    double H0[9], Ht[9];
    for (int k = 0; k < 9; k++) H0[k] = V[k * 9 + 8];
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
    if (n <= 4) return true;
    // LMSolverImpl::run over h[0..7] (h22 = 1)
    auto compute = [&](const double* h, double* r, double* J) {
        for (int i = 0; i < n; i++) {
            const double Mx = M[2 * i], My = M[2 * i + 1];
            double ww = h[6] * Mx + h[7] * My + 1.;
            ww = std::fabs(ww) > DBL_EPSILON ? 1. / ww : 0;
            const double xi = (h[0] * Mx + h[1] * My + h[2]) * ww;
            const double yi = (h[3] * Mx + h[4] * My + h[5]) * ww;
            r[2 * i] = xi - m[2 * i];
            r[2 * i + 1] = yi - m[2 * i + 1];
            if (J) {
                double* j0 = J + 16 * i;
                j0[0] = Mx * ww;
                j0[1] = My * ww;
                j0[2] = ww;
                j0[3] = j0[4] = j0[5] = 0.;
                j0[6] = -Mx * ww * xi;
                j0[7] = -My * ww * xi;
                j0[8] = j0[9] = j0[10] = 0.;
                j0[11] = Mx * ww;
                j0[12] = My * ww;
                j0[13] = ww;
                j0[14] = -Mx * ww * yi;
                j0[15] = -My * ww * yi;
            }
        }
    };
    std::vector<double> r(2 * n), rd(2 * n), J(16 * (size_t)n);
    double x[8], xd[8], A[64], Ap[64], v[8], D[8], d[8];
    memcpy(x, H, sizeof(x));
    auto normals = [&]() {
        for (int a = 0; a < 8; a++) {
            for (int b = 0; b < 8; b++) {
                double sacc = 0;
                for (int k = 0; k < 2 * n; k++) sacc += J[(size_t)k * 8 + a] * J[(size_t)k * 8 + b];
                A[a * 8 + b] = sacc;
            }
            double sv = 0;
            for (int k = 0; k < 2 * n; k++) sv += J[(size_t)k * 8 + a] * r[k];
            v[a] = sv;
        }
    };
    auto l2sq = [&](const std::vector<double>& e) {
        double s2 = 0;
        for (double t : e) s2 += t * t;
        return s2;
    };
    compute(x, r.data(), J.data());
    double S = l2sq(r);
    normals();
    for (int i = 0; i < 8; i++) D[i] = A[i * 9];
    const double Rlo = 0.25, Rhi = 0.75;
    double lambda = 1, lc = 0.75;
    int iter = 0;
    for (;;) {
        memcpy(Ap, A, sizeof(Ap));
        for (int i = 0; i < 8; i++) Ap[i * 9] += lambda * D[i];
        svd_solve(8, 8, Ap, v, d);
        for (int i = 0; i < 8; i++) xd[i] = x[i] - d[i];
        compute(xd, rd.data(), nullptr);
        const double Sd = l2sq(rd);
        double dS = 0;
        for (int i = 0; i < 8; i++) {
            double t = 0;
            for (int k = 0; k < 8; k++) t += A[i * 8 + k] * d[k];
            dS += d[i] * (2 * v[i] - t);  // temp_d = -A d + 2 v
        }
        const double R = (S - Sd) / (std::fabs(dS) > DBL_EPSILON ? dS : 1);
        if (R > Rhi) {
            lambda *= 0.5;
            if (lambda < lc) lambda = 0;
        } else if (R < Rlo) {
            double t = 0;
            for (int i = 0; i < 8; i++) t += d[i] * v[i];
            double nu = (Sd - S) / (std::fabs(t) > DBL_EPSILON ? t : 1) + 2;
            nu = std::min(std::max(nu, 2.), 10.);
            if (lambda == 0) {
                // invert(A, Ap, DECOMP_EIG): the diagonal of the (pseudo) inverse
                double w8[8], U8[64], V8[64];
                svdj(8, 8, A, w8, U8, V8);
                const double thr = 8 * DBL_EPSILON * w8[0];
                double maxval = DBL_EPSILON;
                for (int i = 0; i < 8; i++) {
                    double dii = 0;
                    for (int k = 0; k < 8; k++)
                        if (w8[k] > thr) dii += V8[i * 8 + k] * U8[i * 8 + k] / w8[k];
                    maxval = std::max(maxval, std::fabs(dii));
                }
                lambda = lc = 1. / maxval;
                nu *= 0.5;
            }
            lambda *= nu;
        }
        if (Sd < S) {
            S = Sd;
            std::swap(x, xd);
            compute(x, r.data(), J.data());
            normals();
        }
        iter++;
        double dinf = 0, rinf = 0;
        for (int i = 0; i < 8; i++) dinf = std::max(dinf, std::fabs(d[i]));
        for (double t : r) rinf = std::max(rinf, std::fabs(t));
        if (!(iter < 10 && dinf >= FLT_EPSILON && rinf >= FLT_EPSILON)) break;
    }
    memcpy(H, x, sizeof(x));
    H[8] = 1.;
    return true;
}

// cvFindExtrinsicCameraParams2's initial pose without an extrinsic guess
// (calibration.cpp): normalised image points mn = ((u - cx) / fx, (v - cy) /
// fy) (cvUndistortPoints, no distortion); centroid Mc and scatter MM of the
// object points, cvSVD(MM) -> W, V^T. W2 / W1 < 1e-3: planar — rotate the
// points into their plane (V^T, T = -V^T Mc), find the homography to mn, take
// R from its first two columns (Rodrigues round trip) and t from the third;
// otherwise DLT — the 2n x 12 system L, the eigenvector of L^T L of the
// smallest eigenvalue as [R | t] up to scale and sign (det(R) > 0),
// R := U V^T of its SVD, t scaled by |R| / |RR|. -> param = (rvec, tvec).
// key[i]: the lane of point i (its index among all RANSAC points: the GPU
// walks the inlier mask over them); null = i. Returns false (param untouched)
// where the DLT branch's CV_Assert(count >= 6) fails: non-planar points and
// n < 6, which OpenCV reports by throwing cv::Exception.
bool extrinsic_init(const double* M, const double* m, int n, const double K[4], double param[6],
                    const int* key = nullptr) {
    auto L = [&](int i) { return key ? key[i] : i; };
    const double ifx = 1. / K[0], ify = 1. / K[1];
    std::vector<double> mn(2 * (size_t)n);
    for (int i = 0; i < n; i++) {
        mn[2 * i] = (m[2 * i] - K[2]) * ifx;
        mn[2 * i + 1] = (m[2 * i + 1] - K[3]) * ify;
    }
    double Mc[3];
    {
        WSum64 s(3);
        for (int i = 0; i < n; i++)
            for (int k = 0; k < 3; k++) s.lane(L(i))[k] += M[3 * i + k];
        s.total(Mc);
        for (int k = 0; k < 3; k++) Mc[k] /= n;
    }
    double MM[9];
    {
        WSum64 s(6);
        for (int i = 0; i < n; i++) {
            const double d0 = M[3 * i] - Mc[0], d1 = M[3 * i + 1] - Mc[1], d2 = M[3 * i + 2] - Mc[2];
            double* a = s.lane(L(i));
            a[0] += d0 * d0;
            a[1] += d0 * d1;
            a[2] += d0 * d2;
            a[3] += d1 * d1;
            a[4] += d1 * d2;
            a[5] += d2 * d2;
        }
        double t[6];
        s.total(t);
        const double full[9] = {t[0], t[1], t[2], t[1], t[3], t[4], t[2], t[4], t[5]};
        memcpy(MM, full, sizeof(MM));
    }
    double W[3], Um[9], Vm[9];
    svdj(3, 3, MM, W, Um, Vm);
    double R[9], t[3];
    if (W[2] / W[1] < 1e-3) {
        // planar: R_transform = V^T (rows = right singular vectors)
        double Rt[9];
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) Rt[r * 3 + c] = Vm[c * 3 + r];
        if (Rt[2] * Rt[2] + Rt[5] * Rt[5] < 1e-10)
            for (int k = 0; k < 9; k++) Rt[k] = k % 4 == 0 ? 1.0 : 0.0;
        if (det3(Rt) < 0)
            for (int k = 0; k < 9; k++) Rt[k] = -Rt[k];
        double T[3];
        for (int r = 0; r < 3; r++) T[r] = -(Rt[r * 3] * Mc[0] + Rt[r * 3 + 1] * Mc[1] + Rt[r * 3 + 2] * Mc[2]);
        std::vector<float> Mxy(2 * (size_t)n), mnf(2 * (size_t)n);
        for (int i = 0; i < n; i++) {
            const double* src = M + 3 * i;
            Mxy[2 * i] = (float)(Rt[0] * src[0] + Rt[1] * src[1] + Rt[2] * src[2] + T[0]);
            Mxy[2 * i + 1] = (float)(Rt[3] * src[0] + Rt[4] * src[1] + Rt[5] * src[2] + T[1]);
            mnf[2 * i] = (float)mn[2 * i];
            mnf[2 * i + 1] = (float)mn[2 * i + 1];
        }
        double h[9];
        bool okh = find_homography(Mxy.data(), mnf.data(), n, h);
        for (int k = 0; k < 9 && okh; k++) okh = std::isfinite(h[k]);
        if (okh) {
            const double h1n = std::sqrt(h[0] * h[0] + h[3] * h[3] + h[6] * h[6]);
            const double h2n = std::sqrt(h[1] * h[1] + h[4] * h[4] + h[7] * h[7]);
            const double s1 = 1. / std::max(h1n, DBL_EPSILON), s2 = 1. / std::max(h2n, DBL_EPSILON);
            const double s3 = 2. / std::max(h1n + h2n, DBL_EPSILON);
            double Hm[9];
            for (int r = 0; r < 3; r++) {
                Hm[r * 3] = h[r * 3] * s1;
                Hm[r * 3 + 1] = h[r * 3 + 1] * s2;
                t[r] = h[r * 3 + 2] * s3;
            }
            // third column = h1 x h2
            Hm[2] = Hm[3] * Hm[7] - Hm[6] * Hm[4];
            Hm[5] = Hm[6] * Hm[1] - Hm[0] * Hm[7];
            Hm[8] = Hm[0] * Hm[4] - Hm[3] * Hm[1];
            double rv[3], Hr[9];
            rodrigues_m2v(Hm, rv);
            rodrigues_v2m(rv, Hr, nullptr);
            for (int r = 0; r < 3; r++) t[r] = Hr[r * 3] * T[0] + Hr[r * 3 + 1] * T[1] + Hr[r * 3 + 2] * T[2] + t[r];
            for (int r = 0; r < 3; r++)
                for (int c = 0; c < 3; c++)
                    R[r * 3 + c] = Hr[r * 3] * Rt[c] + Hr[r * 3 + 1] * Rt[3 + c] + Hr[r * 3 + 2] * Rt[6 + c];
        } else {
            for (int k = 0; k < 9; k++) R[k] = k % 4 == 0 ? 1.0 : 0.0;
            t[0] = t[1] = t[2] = 0;
        }
    } else {
        // non-planar: DLT (calibration.cpp: CV_Assert(count >= 6))
        if (n < 6) return false;
        WSum64 s(78);
        for (int i = 0; i < n; i++) {
            const double x = -mn[2 * i], y = -mn[2 * i + 1];
            const double X = M[3 * i], Y = M[3 * i + 1], Z = M[3 * i + 2];
            const double L1[12] = {X, Y, Z, 1., 0., 0., 0., 0., x * X, x * Y, x * Z, x};
            const double L2[12] = {0., 0., 0., 0., X, Y, Z, 1., y * X, y * Y, y * Z, y};
            double* a = s.lane(L(i));
            int k = 0;
            for (int r = 0; r < 12; r++)
                for (int c = r; c < 12; c++, k++) {
                    a[k] += L1[r] * L1[c];
                    a[k] += L2[r] * L2[c];
                }
        }
        double u[78], LL[144];
        s.total(u);
        for (int r = 0, k = 0; r < 12; r++)
            for (int c = r; c < 12; c++, k++) LL[r * 12 + c] = LL[c * 12 + r] = u[k];
        double w12[12], V12[144];
        svdj12(LL, w12, V12);
        double RRt[12];
        for (int k = 0; k < 12; k++) RRt[k] = V12[k * 12 + 11];  // row 11 of V^T
        double RR[9] = {RRt[0], RRt[1], RRt[2], RRt[4], RRt[5], RRt[6], RRt[8], RRt[9], RRt[10]};
        if (det3(RR) < 0) {
            for (int k = 0; k < 12; k++) RRt[k] = -RRt[k];
            for (int k = 0; k < 9; k++) RR[k] = -RR[k];
        }
        double sc = 0;
        for (int k = 0; k < 9; k++) sc += RR[k] * RR[k];
        sc = std::sqrt(sc);
        double w3[3], U3[9], V3[9];
        svdj(3, 3, RR, w3, U3, V3);
        double nr = 0;
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) {
                R[r * 3 + c] = U3[r * 3] * V3[c * 3] + U3[r * 3 + 1] * V3[c * 3 + 1] + U3[r * 3 + 2] * V3[c * 3 + 2];
                nr += R[r * 3 + c] * R[r * 3 + c];
            }
        const double f = std::sqrt(nr) / sc;
        t[0] = RRt[3] * f;
        t[1] = RRt[7] * f;
        t[2] = RRt[11] * f;
    }
    rodrigues_m2v(R, param);
    param[3] = t[0];
    param[4] = t[1];
    param[5] = t[2];
    return true;
}

}  // namespace

extern "C" {

void oracle_cvrng_stream(uint64_t state, int a, int b, int n, int32_t* out) {
    CvRng r{state};
    for (int i = 0; i < n; i++) out[i] = r.uniform(a, b);
}

int oracle_ransac_update_num_iters(double p, double ep, int model_points, int max_iters) {
    return update_num_iters(p, ep, model_points, max_iters);
}

void oracle_rodrigues(const double r[3], double R[9], double* dRdr) { rodrigues_v2m(r, R, dRdr); }
void oracle_rodrigues_inv(const double R[9], double r[3]) { rodrigues_m2v(R, r); }

void oracle_epnp(const double* pw, const double* uv, int n, const double K[4], double model[6]) {
    epnp_model(pw, uv, n, K, model);
}

void oracle_pnp_refine(const double* M, const double* m, int n, const double K[4], double param[6]) {
    refine_lm(M, m, n, K, param);
}

int oracle_pnp_extrinsic_init(const double* M, const double* m, int n, const double K[4], double param[6]) {
    return extrinsic_init(M, m, n, K, param) ? 1 : 0;
}

int oracle_pnp_ransac(const float* Xw, const float* uv, int n, const odo_calib* c, int iterations, float reproj_err,
                      double confidence, double model_out[6], double rt_out[6], float* Tcw, uint8_t* mask,
                      int* n_inliers, int* best_iter, int* niters_out, int* good_counts) {
    *n_inliers = 0;
    *best_iter = -1;
    *niters_out = 0;
    if (n < 10) return 0;  // pnpransac.cpp:30
    const int modelPoints = 5;
    const double K[4] = {c->fx, c->fy, c->cx, c->cy};
    CvRng rng{~(uint64_t)0};
    int niters = iterations > 1 ? iterations : 1, maxGoodCount = 0;
    const float thr = (float)((double)reproj_err * (double)reproj_err);
    std::vector<uint8_t> cur(n), best(n, 0);
    double bestModel[6] = {0};
    int iter;
    for (iter = 0; iter < niters; iter++) {
        // getSubset(m1, m2, ms1, ms2, rng, 10000): distinct indices, checkSubset = true
        int idx[5];
        for (int i = 0; i < modelPoints; i++) {
            for (;;) {
                idx[i] = rng.uniform(0, n);
                int j;
                for (j = 0; j < i; j++)
                    if (idx[i] == idx[j]) break;
                if (j == i) break;
            }
        }
        double pw[15], us[10], model[6];
        for (int i = 0; i < modelPoints; i++) {
            for (int k = 0; k < 3; k++) pw[3 * i + k] = (double)Xw[3 * idx[i] + k];
            us[2 * i] = (double)uv[2 * idx[i]];
            us[2 * i + 1] = (double)uv[2 * idx[i] + 1];
        }
        epnp_model(pw, us, modelPoints, K, model);
        // findInliers: computeError = projectPoints (float out) -> L2SQR in float
        double R[9];
        rodrigues_v2m(model, R, nullptr);
        int good = 0;
        for (int i = 0; i < n; i++) {
            const double M[3] = {(double)Xw[3 * i], (double)Xw[3 * i + 1], (double)Xw[3 * i + 2]};
            double u, v;
            project_pt(R, nullptr, model + 3, K, M, &u, &v, nullptr, nullptr);
            const float dx = uv[2 * i] - (float)u, dy = uv[2 * i + 1] - (float)v;
            const float e = dx * dx + dy * dy;
            cur[i] = e <= thr;
            good += cur[i];
        }
        if (good_counts && iter < iterations) good_counts[iter] = good;
        if (good > (maxGoodCount > modelPoints - 1 ? maxGoodCount : modelPoints - 1)) {
            std::swap(cur, best);
            memcpy(bestModel, model, sizeof(bestModel));
            maxGoodCount = good;
            *best_iter = iter;
            niters = update_num_iters(confidence, (double)(n - good) / n, modelPoints, niters);
        }
    }
    *niters_out = iter;
    if (maxGoodCount <= 0) return 0;
    memcpy(model_out, bestModel, sizeof(bestModel));
    // refinement on the inliers (float -> double as convertTo(CV_64F))
    std::vector<double> Mi, mi;
    std::vector<int> key;
    for (int i = 0; i < n; i++)
        if (best[i]) {
            for (int k = 0; k < 3; k++) Mi.push_back((double)Xw[3 * i + k]);
            mi.push_back((double)uv[2 * i]);
            mi.push_back((double)uv[2 * i + 1]);
            key.push_back(i);
        }
    const int ni = (int)(mi.size() / 2);
    // solvePnP(..., useExtrinsicGuess = false): cvFindExtrinsicCameraParams2's own start
    double p[6];
    if (mask) memcpy(mask, best.data(), n);
    *n_inliers = maxGoodCount;
    if (!extrinsic_init(Mi.data(), mi.data(), ni, K, p, key.data())) {
        // solvePnP's cvFindExtrinsicCameraParams2 throws (non-planar, 5
        // inliers): the exception leaves solvePnPRansac, and PnPRansac::Compute
        // does not catch it. Reported as -1: no pose.
        memset(rt_out, 0, 6 * sizeof(double));
        memset(Tcw, 0, 16 * sizeof(float));
        return -1;
    }
    refine_lm(Mi.data(), mi.data(), ni, K, p);
    memcpy(rt_out, p, sizeof(p));
    // Converter::toHomogeneous(r, t)
    double R[9];
    rodrigues_v2m(p, R, nullptr);
    for (int r = 0; r < 3; r++) {
        for (int k = 0; k < 3; k++) Tcw[4 * r + k] = (float)R[3 * r + k];
        Tcw[4 * r + 3] = (float)p[3 + r];
    }
    Tcw[12] = Tcw[13] = Tcw[14] = 0.f;
    Tcw[15] = 1.f;
    return 1;
}

}  // extern "C"
