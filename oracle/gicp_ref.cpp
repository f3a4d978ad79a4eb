// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). CPU restatement of
//   GeneralizedICP::Compute(source, target, guess)   Odometry/generalizedicp.cpp:30-39, 65-89
// i.e. pcl::GeneralizedIterativeClosestPoint<PointXYZ, PointXYZ> of PCL 1.8
// (gicp.hpp computeCovariances / computeTransformation /
// estimateRigidTransformationBFGS / applyState / computeRDerivative, bfgs.h's
// BFGS2 with Fletcher's line search) with the settings of generalizedicp.cpp:11-22
// and odometry.cpp:15 (max iterations, max correspondence distance, euclidean
// fitness epsilon 1, transformation epsilon 1e-9; PCL defaults k = 20,
// epsilon 1e-3, rotation epsilon 2e-3, 20 BFGS iterations, gradient tol 1e-2).
// PCL is absent from this image: restated from its published source as
// recalled (parity UNPINNED). Pinned choices (DESIGN.md §4 "GICP"):
//   * k-d tree searches are exact brute force, ties to the lower index; squared
//     distances in float, x then y then z (FLANN L2_Simple);
//   * the 3x3 covariance eigenvectors come from the one-sided Jacobi SVD (V);
//   * Eigen fixed-size-3 sums associate as p0 + (p1 + p2); Matrix4f * Vector4f
//     accumulates column by column; AngleAxisf products via quaternions;
//   * float cos / sin / atan2 / asin (AngleAxisf, the initial Euler angles) are
//     the double functions rounded to float;
//   * every sum over correspondences (cost, gradient) is the 256-thread form of
//     the GPU: thread t sums k = t, t + 256, ... in order, lane position l adds
//     the partials of threads l, l + 64, l + 128, l + 192 in that order, then an
//     xor butterfly 32 .. 1 read on lane 0 (sum256 below).
#include <cfloat>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "oracle.h"

namespace {

inline double s3(double a, double b, double c) { return a + (b + c); }

// one-sided Jacobi SVD of a 3x3 (same rotations as pnpransac_ref.cpp's svdj); V by columns, w descending
void svd3_v(const double* A, double* w, double* V) {
    double a[9], v[9];
    memcpy(a, A, sizeof(a));
    for (int i = 0; i < 9; i++) v[i] = i % 4 == 0 ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; sweep++) {
        int changed = 0;
        for (int p = 0; p < 2; p++)
            for (int q = p + 1; q < 3; q++) {
                double alpha = 0, beta = 0, gamma = 0;
                for (int i = 0; i < 3; i++) {
                    const double ap = a[i * 3 + p], aq = a[i * 3 + q];
                    alpha += ap * ap;
                    beta += aq * aq;
                    gamma += ap * aq;
                }
                if (gamma == 0.0 || std::fabs(gamma) <= DBL_EPSILON * std::sqrt(alpha * beta)) continue;
                changed = 1;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / std::sqrt(1.0 + t * t), s = c * t;
                for (int i = 0; i < 3; i++) {
                    const double ap = a[i * 3 + p], aq = a[i * 3 + q];
                    a[i * 3 + p] = c * ap - s * aq;
                    a[i * 3 + q] = s * ap + c * aq;
                    const double vp = v[i * 3 + p], vq = v[i * 3 + q];
                    v[i * 3 + p] = c * vp - s * vq;
                    v[i * 3 + q] = s * vp + c * vq;
                }
            }
        if (!changed) break;
    }
    double ww[3];
    int ord[3] = {0, 1, 2};
    for (int j = 0; j < 3; j++) ww[j] = std::sqrt(a[j] * a[j] + a[3 + j] * a[3 + j] + a[6 + j] * a[6 + j]);
    for (int j = 0; j < 3; j++) {
        int b = j;
        for (int k = j + 1; k < 3; k++)
            if (ww[ord[k]] > ww[ord[b]]) b = k;
        const int t = ord[j];
        ord[j] = ord[b];
        ord[b] = t;
    }
    for (int j = 0; j < 3; j++) {
        w[j] = ww[ord[j]];
        for (int i = 0; i < 3; i++) V[i * 3 + j] = v[i * 3 + ord[j]];
    }
}

inline float dist2f(const float* a, const float* b) {
    float r = 0.f, d;
    d = a[0] - b[0];
    r += d * d;
    d = a[1] - b[1];
    r += d * d;
    d = a[2] - b[2];
    r += d * d;
    return r;
}

// computeCovariances: k nearest (incl. the point), mean / covariance in double
// with float products, eigenvalues replaced by (1, 1, epsilon)
void covariances(const float* P, int n, int k, double eps, double* C) {
    std::vector<int> nn(k);
    std::vector<float> nd(k);
    for (int q = 0; q < n; q++) {
        int cnt = 0;
        for (int i = 0; i < n; i++) {  // insertion into the sorted top k, ties to the lower index
            const float d = dist2f(P + 3 * q, P + 3 * i);
            if (cnt == k && !(d < nd[k - 1])) continue;
            int pos = cnt < k ? cnt : k - 1;
            while (pos > 0 && d < nd[pos - 1]) {
                if (pos < k) {
                    nd[pos] = nd[pos - 1];
                    nn[pos] = nn[pos - 1];
                }
                pos--;
            }
            nd[pos] = d;
            nn[pos] = i;
            if (cnt < k) cnt++;
        }
        double mean[3] = {0, 0, 0}, cov[9] = {0};
        for (int j = 0; j < k; j++) {
            const float* pt = P + 3 * nn[j];
            mean[0] += pt[0];
            mean[1] += pt[1];
            mean[2] += pt[2];
            cov[0] += pt[0] * pt[0];
            cov[3] += pt[1] * pt[0];
            cov[4] += pt[1] * pt[1];
            cov[6] += pt[2] * pt[0];
            cov[7] += pt[2] * pt[1];
            cov[8] += pt[2] * pt[2];
        }
        for (int a = 0; a < 3; a++) mean[a] /= (double)k;
        for (int a = 0; a < 3; a++)
            for (int b = 0; b <= a; b++) {
                cov[a * 3 + b] /= (double)k;
                cov[a * 3 + b] -= mean[a] * mean[b];
                cov[b * 3 + a] = cov[a * 3 + b];
            }
        double w[3], U[9];
        svd3_v(cov, w, U);
        double* out = C + 9 * q;
        for (int i = 0; i < 9; i++) out[i] = 0.0;
        for (int c = 0; c < 3; c++) {
            const double v = c == 2 ? eps : 1.;
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) out[a * 3 + b] += (v * U[a * 3 + c]) * U[b * 3 + c];
        }
    }
}

// Eigen Matrix3d::inverse (cofactors, invdet)
void inv3(const double* m, double* r) {
    auto M = [&](int i, int j) { return m[i * 3 + j]; };
    auto cof = [&](int i, int j) {
        const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
        return M(i1, j1) * M(i2, j2) - M(i1, j2) * M(i2, j1);
    };
    const double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
    const double det = s3(c0 * M(0, 0), c1 * M(1, 0), c2 * M(2, 0));
    const double invdet = 1.0 / det;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r[i * 3 + j] = cof(j, i) * invdet;
}

// Matrix4f * (x, y, z, 1): column by column
inline void xform4f(const float* T, const float* p, float* o) {
    for (int i = 0; i < 3; i++) o[i] = ((T[4 * i] * p[0] + T[4 * i + 1] * p[1]) + T[4 * i + 2] * p[2]) + T[4 * i + 3];
}

// applyState on the identity base: R = AngleAxisf(x5, Z) * AngleAxisf(x4, Y) * AngleAxisf(x3, X)
void apply_state(const double* x, float* T) {
    float q[3][4];  // (w, x, y, z) of the Z, Y, X rotations
    const float a[3] = {(float)x[5], (float)x[4], (float)x[3]};
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
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T[4 * i + j] = R[3 * i + j];
        T[4 * i + 3] = 0.f + (float)x[i];
    }
    T[12] = T[13] = T[14] = 0.f;
    T[15] = 1.f;
}

// the GPU's 256-thread sum of values v[0..m) (see the header)
double sum256(const std::vector<double>& v) {
    double t256[256], y[64];
    for (int t = 0; t < 256; t++) {
        double s = 0.0;
        for (size_t k = t; k < v.size(); k += 256) s += v[k];
        t256[t] = s;
    }
    for (int l = 0; l < 64; l++) y[l] = ((t256[l] + t256[l + 64]) + t256[l + 128]) + t256[l + 192];
    for (int o = 32; o >= 1; o >>= 1) {
        double z[64];
        for (int i = 0; i < 64; i++) z[i] = y[i] + y[i ^ o];
        memcpy(y, z, sizeof(y));
    }
    return y[0];
}

struct Problem {
    const float* src;  // output (source after the guess)
    const float* tgt;
    const int* is;
    const int* it;
    const double* M;  // Mahalanobis per source index
    int m;
};

double cost(const Problem& P, const double* x) {
    float T[16];
    apply_state(x, T);
    std::vector<double> v(P.m);
    for (int k = 0; k < P.m; k++) {
        float pp[3];
        xform4f(T, P.src + 3 * P.is[k], pp);
        const float* q = P.tgt + 3 * P.it[k];
        const double r[3] = {(double)(pp[0] - q[0]), (double)(pp[1] - q[1]), (double)(pp[2] - q[2])};
        const double* M = P.M + 9 * P.is[k];
        double t[3];
        for (int i = 0; i < 3; i++) t[i] = s3(M[3 * i] * r[0], M[3 * i + 1] * r[1], M[3 * i + 2] * r[2]);
        v[k] = s3(r[0] * t[0], r[1] * t[1], r[2] * t[2]);
    }
    return sum256(v) / P.m;
}

void grad(const Problem& P, const double* x, double* g) {
    float T[16];
    apply_state(x, T);
    std::vector<double> v[12];
    for (auto& a : v) a.resize(P.m);
    for (int k = 0; k < P.m; k++) {
        float pp[3];
        const float* ps = P.src + 3 * P.is[k];
        xform4f(T, ps, pp);
        const float* q = P.tgt + 3 * P.it[k];
        const double r[3] = {(double)(pp[0] - q[0]), (double)(pp[1] - q[1]), (double)(pp[2] - q[2])};
        const double* M = P.M + 9 * P.is[k];
        double t[3];
        for (int i = 0; i < 3; i++) t[i] = s3(M[3 * i] * r[0], M[3 * i + 1] * r[1], M[3 * i + 2] * r[2]);
        for (int i = 0; i < 3; i++) v[i][k] = t[i];
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) v[3 + 3 * a + b][k] = (double)ps[a] * t[b];
    }
    double Rm[9];
    for (int i = 0; i < 3; i++) g[i] = sum256(v[i]) * (2.0 / P.m);
    for (int i = 0; i < 9; i++) Rm[i] = sum256(v[3 + i]) * (2.0 / P.m);
    // computeRDerivative
    const double phi = x[3], theta = x[4], psi = x[5];
    const double cphi = cos(phi), sphi = sin(phi), ctheta = cos(theta), stheta = sin(theta), cpsi = cos(psi),
                 spsi = sin(psi);
    const double dPhi[9] = {0., sphi * spsi + cphi * cpsi * stheta, cphi * spsi - cpsi * sphi * stheta,
                            0., -cpsi * sphi + cphi * spsi * stheta, -cphi * cpsi - sphi * spsi * stheta,
                            0., cphi * ctheta, -ctheta * sphi};
    const double dTheta[9] = {-cpsi * stheta, cpsi * ctheta * sphi, cphi * cpsi * ctheta,
                              -spsi * stheta, ctheta * sphi * spsi, cphi * ctheta * spsi,
                              -ctheta, -sphi * stheta, -cphi * stheta};
    const double dPsi[9] = {-ctheta * spsi, -cphi * cpsi - sphi * spsi * stheta, cpsi * sphi - cphi * spsi * stheta,
                            cpsi * ctheta, -cphi * spsi + cpsi * sphi * stheta, sphi * spsi + cphi * cpsi * stheta,
                            0., 0., 0.};
    const double* d[3] = {dPhi, dTheta, dPsi};
    for (int c = 0; c < 3; c++) {  // matricesInnerProd: r += mat1(j, i) * mat2(i, j)
        double r = 0.;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) r += d[c][3 * j + i] * Rm[3 * i + j];
        g[3 + c] = r;
    }
}

// ---- bfgs.h (BFGS2 with Fletcher's line search, GSL lineage)
enum { ST_NEG_EPS = -3, ST_NOT_STARTED = -2, ST_RUNNING = -1, ST_SUCCESS = 0, ST_NO_PROGRESS = 1 };

struct Bfgs {
    const Problem& P;
    double x0[6], p[6], g0[6], dx0[6], dg0[6], gradient[6];
    double f, fp0, g0norm, pnorm, delta_f;
    // cached line point
    double x_alpha[6], g_alpha[6], f_alpha, df_alpha;
    double f_key, g_key, df_key;
    const double rho = 0.01, sigma = 0.01, tau1 = 9, tau2 = 0.05, tau3 = 0.5, step_size = 1.0;
    const int order = 3;
    explicit Bfgs(const Problem& pr) : P(pr) {}

    static double dot6(const double* a, const double* b) {
        double s = 0;
        for (int i = 0; i < 6; i++) s += a[i] * b[i];
        return s;
    }
    static double norm6(const double* a) { return std::sqrt(dot6(a, a)); }

    void moveTo(double alpha) {
        for (int i = 0; i < 6; i++) x_alpha[i] = x0[i] + alpha * p[i];
    }
    double slope() { return dot6(g_alpha, p); }
    double applyF(double alpha) {
        if (alpha == f_key) return f_alpha;
        moveTo(alpha);
        f_alpha = cost(P, x_alpha);
        f_key = alpha;
        return f_alpha;
    }
    double applyDF(double alpha) {
        if (alpha == df_key) return df_alpha;
        moveTo(alpha);
        if (alpha != g_key) {
            grad(P, x_alpha, g_alpha);
            g_key = alpha;
        }
        df_alpha = slope();
        df_key = alpha;
        return df_alpha;
    }
    void updatePosition(double alpha, double* x, double* fo, double* g) {
        applyF(alpha);
        applyDF(alpha);
        memcpy(x, x_alpha, sizeof(x_alpha));
        *fo = f_alpha;
        memcpy(g, g_alpha, sizeof(g_alpha));
    }
    void changeDirection() {
        memcpy(x_alpha, x0, sizeof(x0));
        f_key = 0.0;
        memcpy(g_alpha, g0, sizeof(g0));
        g_key = 0.0;
        df_alpha = slope();
        df_key = 0.0;
    }

    static double cubic(double c0, double c1, double c2, double c3, double z) { return c0 + z * (c1 + z * (c2 + z * c3)); }
    static void checkExtremum(double c0, double c1, double c2, double c3, double x, double& xmin, double& fmin) {
        const double y = cubic(c0, c1, c2, c3, x);
        if (y < fmin) {
            xmin = x;
            fmin = y;
        }
    }
    static int solve_quadratic(double a, double b, double c, double* x0, double* x1) {
        if (a == 0) {
            if (b == 0) return 0;
            *x0 = -c / b;
            return 1;
        }
        const double disc = b * b - 4 * a * c;
        if (disc > 0) {
            if (b == 0) {
                const double r = std::sqrt(-c / a);
                *x0 = -r;
                *x1 = r;
            } else {
                const double sgnb = (b > 0 ? 1 : -1);
                const double temp = -0.5 * (b + sgnb * std::sqrt(disc));
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
    static double cubicInterp(double f0, double fp0, double f1, double fp1, double zl, double zh) {
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
    static double quadraticInterp(double f0, double fp0, double f1, double zl, double zh) {
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
    double interpolate(double a, double fa, double fpa, double b, double fb, double fpb, double xmin, double xmax) {
        double zmin = (xmin - a) / (b - a), zmax = (xmax - a) / (b - a);
        if (zmin > zmax) {
            const double t = zmin;
            zmin = zmax;
            zmax = t;
        }
        double z;
        if (order > 2 && !std::isnan(fpb))
            z = cubicInterp(fa, fpa * (b - a), fb, fpb * (b - a), zmin, zmax);
        else
            z = quadraticInterp(fa, fpa * (b - a), fb, zmin, zmax);
        return a + z * (b - a);
    }
    int lineSearch(double alpha1, double* alpha_new) {
        double falpha, fpalpha, delta, alpha_next;
        double alpha = alpha1, alpha_prev = 0.0;
        int i = 0;
        const double f0 = applyF(0.0), fp0l = applyDF(0.0);
        double falpha_prev = f0, fpalpha_prev = fp0l;
        double a = 0.0, b = alpha, fa = f0, fb = 0.0, fpa = fp0l, fpb = 0.0;
        const double qnan = std::numeric_limits<double>::quiet_NaN();
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
            if (std::fabs(fpalpha) <= -sigma * fp0l) {
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
            if ((a - alpha) * fpa <= std::numeric_limits<double>::epsilon()) return ST_NO_PROGRESS;
            if (falpha > f0 + rho * alpha * fp0l || falpha >= fa) {
                b = alpha;
                fb = falpha;
                fpb = qnan;
            } else {
                fpalpha = applyDF(alpha);
                if (std::fabs(fpalpha) <= -sigma * fp0l) {
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
    void minimizeInit(const double* x) {
        delta_f = 0;
        f = cost(P, x);
        grad(P, x, gradient);
        memcpy(x0, x, sizeof(x0));
        memcpy(g0, gradient, sizeof(g0));
        g0norm = norm6(g0);
        for (int i = 0; i < 6; i++) p[i] = gradient[i] * (-1 / g0norm);
        pnorm = norm6(p);
        fp0 = -g0norm;
        memcpy(x_alpha, x0, sizeof(x0));
        f_alpha = f;
        f_key = 0;
        memcpy(g_alpha, g0, sizeof(g0));
        g_key = 0;
        df_alpha = slope();
        df_key = 0;
    }
    int minimizeOneStep(double* x) {
        double alpha = 0.0, alpha1;
        const double f0 = f;
        if (pnorm == 0.0 || g0norm == 0.0 || fp0 == 0) return ST_NOT_STARTED;
        if (delta_f < 0) {
            const double del = std::max(-delta_f, 10 * std::numeric_limits<double>::epsilon() * std::fabs(f0));
            alpha1 = std::min(1.0, 2.0 * del / (-fp0));
        } else {
            alpha1 = std::fabs(step_size);
        }
        const int st = lineSearch(alpha1, &alpha);
        if (st != ST_SUCCESS) return st;
        updatePosition(alpha, x, &f, gradient);
        delta_f = f - f0;
        {
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
            for (int i = 0; i < 6; i++) p[i] = (gradient[i] + (-A) * dx0[i]) + (-B) * dg0[i];  // memcpy, daxpy, daxpy
        }
        memcpy(g0, gradient, sizeof(g0));
        memcpy(x0, x, sizeof(x0));
        g0norm = norm6(g0);
        pnorm = norm6(p);
        const double dir = (dot6(p, gradient) >= 0.0) ? -1.0 : +1.0;
        for (int i = 0; i < 6; i++) p[i] *= dir / pnorm;
        pnorm = norm6(p);
        fp0 = dot6(p, g0);
        changeDirection();
        return ST_SUCCESS;
    }
};

}  // namespace

extern "C" {

void oracle_gicp_covariances(const float* P, int n, double* C) { covariances(P, n, 20, 1e-3, C); }

int oracle_gicp(const float* src, int ns, const float* tgt, int nt, const float* guess, int max_iterations,
                double max_corr_dist, float* T12, int* converged, int* iterations, int* n_corr) {
    *converged = 0;
    *iterations = 0;
    *n_corr = 0;
    for (int i = 0; i < 16; i++) T12[i] = i % 5 == 0 ? 1.f : 0.f;
    if (ns < 20 || nt < 20) return 0;  // generalizedicp.cpp:33
    std::vector<double> Ct((size_t)nt * 9), Cs((size_t)ns * 9), Mah((size_t)ns * 9);
    covariances(tgt, nt, 20, 1e-3, Ct.data());
    covariances(src, ns, 20, 1e-3, Cs.data());
    for (int i = 0; i < ns; i++)
        for (int k = 0; k < 9; k++) Mah[9 * i + k] = k % 4 == 0 ? 1.0 : 0.0;
    // output = source transformed by the guess (transformPointCloud, float)
    std::vector<float> out((size_t)3 * ns);
    for (int i = 0; i < ns; i++) {
        const float* p = src + 3 * i;
        for (int r = 0; r < 3; r++)
            out[3 * i + r] = guess[4 * r] * p[0] + guess[4 * r + 1] * p[1] + guess[4 * r + 2] * p[2] + guess[4 * r + 3];
    }
    float Tcur[16], Tprev[16];
    for (int i = 0; i < 16; i++) Tcur[i] = Tprev[i] = i % 5 == 0 ? 1.f : 0.f;
    const double dist_threshold = max_corr_dist * max_corr_dist;
    const double rotation_epsilon = 2e-3, transformation_epsilon = 1e-9;
    int nr_iterations = 0, conv = 0;
    std::vector<int> is, it;
    while (!conv) {
        is.clear();
        it.clear();
        double R[9];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                double s = 0;
                for (int k = 0; k < 4; k++) s += double(Tcur[4 * i + k]) * double(guess[4 * k + j]);
                R[3 * i + j] = s;
            }
        for (int i = 0; i < ns; i++) {
            float q[3];
            xform4f(Tcur, out.data() + 3 * i, q);
            int best = 0;
            float bd = dist2f(q, tgt);
            for (int j = 1; j < nt; j++) {
                const float d = dist2f(q, tgt + 3 * j);
                if (d < bd) {
                    bd = d;
                    best = j;
                }
            }
            if ((double)bd < dist_threshold) {
                const double* C1 = Cs.data() + 9 * i;
                const double* C2 = Ct.data() + 9 * best;
                double M[9], tmp[9];
                for (int a = 0; a < 3; a++)
                    for (int b = 0; b < 3; b++) M[3 * a + b] = s3(R[3 * a] * C1[b], R[3 * a + 1] * C1[3 + b], R[3 * a + 2] * C1[6 + b]);
                for (int a = 0; a < 3; a++)
                    for (int b = 0; b < 3; b++) {
                        tmp[3 * a + b] = s3(M[3 * a] * R[3 * b], M[3 * a + 1] * R[3 * b + 1], M[3 * a + 2] * R[3 * b + 2]);
                        tmp[3 * a + b] += C2[3 * a + b];
                    }
                inv3(tmp, Mah.data() + 9 * i);
                is.push_back(i);
                it.push_back(best);
            }
        }
        *n_corr = (int)is.size();
        memcpy(Tprev, Tcur, sizeof(Tcur));
        // estimateRigidTransformationBFGS
        if (is.size() < 4) break;  // NotEnoughPointsException -> caught, not converged
        double x[6] = {Tcur[3], Tcur[7], Tcur[11], (double)(float)atan2((double)Tcur[9], (double)Tcur[10]), (double)(float)asin(-(double)Tcur[8]),
                       (double)(float)atan2((double)Tcur[4], (double)Tcur[0])};
        Problem P{out.data(), tgt, is.data(), it.data(), Mah.data(), (int)is.size()};
        Bfgs bfgs(P);
        bfgs.minimizeInit(x);
        int inner = 0, result;
        do {
            inner++;
            result = bfgs.minimizeOneStep(x);
            if (result) break;
            double gn = 0;
            for (int k = 0; k < 6; k++) gn += bfgs.gradient[k] * bfgs.gradient[k];
            result = std::sqrt(gn) < 1e-2 ? ST_SUCCESS : ST_RUNNING;
        } while (result == ST_RUNNING && inner < 20);
        if (!(result == ST_NO_PROGRESS || result == ST_SUCCESS || inner == 20)) break;  // SolverDidntConverge
        apply_state(x, Tcur);
        double delta = 0.;
        for (int k = 0; k < 4; k++)
            for (int l = 0; l < 4; l++) {
                const double ratio = (k < 3 && l < 3) ? 1. / rotation_epsilon : 1. / transformation_epsilon;
                const double c_delta = ratio * std::fabs(Tprev[4 * k + l] - Tcur[4 * k + l]);
                if (c_delta > delta) delta = c_delta;
            }
        nr_iterations++;
        if (nr_iterations >= max_iterations || delta < 1) {
            conv = 1;
            memcpy(Tprev, Tcur, sizeof(Tcur));
        }
    }
    *iterations = nr_iterations;
    *converged = conv;
    if (!conv) return 0;
    // final_transformation_ = previous_transformation_ * guess (Matrix4f product)
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            T12[4 * i + j] = ((Tprev[4 * i] * guess[j] + Tprev[4 * i + 1] * guess[4 + j]) + Tprev[4 * i + 2] * guess[8 + j]) +
                             Tprev[4 * i + 3] * guess[12 + j];
    return 1;
}

}  // extern "C"
