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
//     useExtrinsicGuess = true) seeded with the RANSAC model, whose 6x6 damped
//     normal equations are solved with the same SVD (solve(..., DECOMP_SVD)).
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
    for (int i = 0; i < n; i++)
        if (best[i]) {
            for (int k = 0; k < 3; k++) Mi.push_back((double)Xw[3 * i + k]);
            mi.push_back((double)uv[2 * i]);
            mi.push_back((double)uv[2 * i + 1]);
        }
    const int ni = (int)(mi.size() / 2);
    double p[6];
    memcpy(p, bestModel, sizeof(p));
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
    if (mask) memcpy(mask, best.data(), n);
    *n_inliers = maxGoodCount;
    return 1;
}

}  // extern "C"
