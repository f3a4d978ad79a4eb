// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). CPU restatement of the
// reference's frame geometry, matching and pose estimation:
//   Frame::ExtractFeatures / UndistortKeyPoints  Core/frame.cpp:135-170, 286-313
//   Matcher::KnnMatch(Frame&,Frame&)             Features/matcher.cpp:55-88
//   Tracking::UpdateLastFrame (VO landmarks)     System/tracking.cpp:136-191
//   Ransac::Iterate / SampleMatches / ...        Odometry/ransac.cpp:155-421
//   PnPSolver::Compute                           Odometry/pnpsolver.cpp:17-214
//   Kabsch::Compute                              Odometry/kabsch.cpp:14-57
// Third-party semantics (cv::undistortPoints, BFMatcher, PCL
// TransformationFromCorrespondences, Eigen JacobiSVD/LLT/LDLT, g2o
// Levenberg-Marquardt) restated per SURVEY.md Appendix A; arithmetic order
// choices recorded in DESIGN.md §4.
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <limits>
#include <set>
#include <utility>
#include <vector>

#include "oracle.h"

namespace {

// ------------------------------------------------------------ small linalg
struct V3f { float v[3]; float& operator[](int i) { return v[i]; } float operator[](int i) const { return v[i]; } };
struct M3f { float m[3][3]; };
struct V3d { double v[3]; double& operator[](int i) { return v[i]; } double operator[](int i) const { return v[i]; } };
struct M3d { double m[3][3]; };

// Eigen fixed-size-3 reduction order (redux_novec_unroller): p0 + (p1 + p2)
inline float sum3(float a, float b, float c) { return a + (b + c); }
inline double sum3(double a, double b, double c) { return a + (b + c); }

// ------------------------------------------------------------ App. A.8 SVD
// Eigen 3.3 JacobiSVD<Matrix3f>(ComputeFullU|ComputeFullV), square case.
struct Rot { float c, s; };

inline void rot_rows(float W[3][3], int p, int q, Rot j) {  // applyOnTheLeft(p,q,j)
    if (j.c == 1.f && j.s == 0.f) return;
    for (int i = 0; i < 3; i++) {
        float xi = W[p][i], yi = W[q][i];
        W[p][i] = j.c * xi + j.s * yi;
        W[q][i] = -j.s * xi + j.c * yi;
    }
}
inline void rot_cols(float W[3][3], int p, int q, Rot j) {  // applyOnTheRight(p,q,j): uses j^T
    Rot t{j.c, -j.s};
    if (t.c == 1.f && t.s == 0.f) return;
    for (int i = 0; i < 3; i++) {
        float xi = W[i][p], yi = W[i][q];
        W[i][p] = t.c * xi + t.s * yi;
        W[i][q] = -t.s * xi + t.c * yi;
    }
}

Rot make_jacobi(float x, float y, float z) {
    float deno = 2.f * std::abs(y);
    if (deno < FLT_MIN) return Rot{1.f, 0.f};
    float tau = (x - z) / deno;
    float w = sqrtf(tau * tau + 1.f);
    float t = tau > 0.f ? 1.f / (tau + w) : 1.f / (tau - w);
    float sign_t = t > 0.f ? 1.f : -1.f;
    float n = 1.f / sqrtf(t * t + 1.f);
    Rot r;
    r.s = ((-sign_t) * (y / std::abs(y))) * std::abs(t) * n;
    r.c = n;
    return r;
}

void real_2x2_jacobi_svd(const float W[3][3], int p, int q, Rot* jl, Rot* jr) {
    float m[2][2] = {{W[p][p], W[p][q]}, {W[q][p], W[q][q]}};
    Rot rot1;
    float t = m[0][0] + m[1][1];
    float d = m[1][0] - m[0][1];
    if (std::abs(d) < FLT_MIN) {
        rot1.s = 0.f;
        rot1.c = 1.f;
    } else {
        float u = t / d;
        float tmp = sqrtf(1.f + u * u);
        rot1.s = 1.f / tmp;
        rot1.c = u / tmp;
    }
    // m.applyOnTheLeft(0,1,rot1)
    if (!(rot1.c == 1.f && rot1.s == 0.f)) {
        for (int i = 0; i < 2; i++) {
            float xi = m[0][i], yi = m[1][i];
            m[0][i] = rot1.c * xi + rot1.s * yi;
            m[1][i] = -rot1.s * xi + rot1.c * yi;
        }
    }
    *jr = make_jacobi(m[0][0], m[0][1], m[1][1]);
    // j_left = rot1 * j_right^T ; (c1,s1)*(c2,s2) = (c1 c2 - s1 s2, c1 s2 + s1 c2)
    float c2 = jr->c, s2 = -jr->s;
    jl->c = rot1.c * c2 - rot1.s * s2;
    jl->s = rot1.c * s2 + rot1.s * c2;
}

void svd3(const float A[3][3], float U[3][3], float S[3], float V[3][3]) {
    const float precision = 2.f * FLT_EPSILON;
    const float considerAsZero = FLT_MIN;
    float scale = 0.f;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) scale = std::max(scale, std::abs(A[i][j]));
    if (scale == 0.f) scale = 1.f;
    float W[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            W[i][j] = A[i][j] / scale;
            U[i][j] = (i == j) ? 1.f : 0.f;
            V[i][j] = (i == j) ? 1.f : 0.f;
        }
    float maxDiag = std::max(std::abs(W[0][0]), std::max(std::abs(W[1][1]), std::abs(W[2][2])));
    bool finished = false;
    int sweeps = 0;
    while (!finished && sweeps < 100) {
        finished = true;
        sweeps++;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                float threshold = std::max(considerAsZero, precision * maxDiag);
                if (std::abs(W[p][q]) > threshold || std::abs(W[q][p]) > threshold) {
                    finished = false;
                    Rot jl, jr;
                    real_2x2_jacobi_svd(W, p, q, &jl, &jr);
                    rot_rows(W, p, q, jl);
                    rot_cols(U, p, q, Rot{jl.c, -jl.s});  // U.applyOnTheRight(p,q,j_left.transpose())
                    rot_cols(W, p, q, jr);
                    rot_cols(V, p, q, jr);
                    maxDiag = std::max(maxDiag, std::max(std::abs(W[p][p]), std::abs(W[q][q])));
                }
            }
    }
    for (int i = 0; i < 3; i++) {
        float a = W[i][i];
        S[i] = std::abs(a);
        if (a < 0.f)
            for (int r = 0; r < 3; r++) U[r][i] = -U[r][i];
    }
    for (int i = 0; i < 3; i++) S[i] *= scale;
    for (int i = 0; i < 3; i++) {
        int pos = i;
        float mx = S[i];
        for (int k = i + 1; k < 3; k++)
            if (S[k] > mx) { mx = S[k]; pos = k; }
        if (mx == 0.f) break;
        if (pos != i) {
            std::swap(S[i], S[pos]);
            for (int r = 0; r < 3; r++) {
                std::swap(U[r][i], U[r][pos]);
                std::swap(V[r][i], V[r][pos]);
            }
        }
    }
}

inline float det3(const float M[3][3]) {
    // Eigen determinant_impl<3>: bruteforce_det3_helper(0,1,2) - (1,0,2) + (2,0,1)
    auto h = [&](int a, int b, int c) { return M[0][a] * (M[1][b] * M[2][c] - M[1][c] * M[2][b]); };
    return h(0, 1, 2) - h(1, 0, 2) + h(2, 0, 1);
}

// ------------------------------------------------------------ App. A.7 TFC
struct TFC {
    float accW = 0.f;
    float mean1[3] = {0, 0, 0}, mean2[3] = {0, 0, 0};
    float cov[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    void add(const float p[3], const float q[3], float w) {
        if (w == 0.0f) return;
        accW += w;
        float alpha = w / accW;
        float d1[3], d2[3];
        for (int i = 0; i < 3; i++) {
            d1[i] = p[i] - mean1[i];
            d2[i] = q[i] - mean2[i];
        }
        for (int i = 0; i < 3; i++)
            // Eigen 3.3 rewrites "alpha * (d2 * d1^T)" as "(alpha * d2) * d1^T"
            // (ProductEvaluators.h, scalar*(A*B) rule).
            for (int j = 0; j < 3; j++) cov[i][j] = (1.0f - alpha) * (cov[i][j] + (alpha * d2[i]) * d1[j]);
        for (int i = 0; i < 3; i++) {
            mean1[i] += alpha * d1[i];
            mean2[i] += alpha * d2[i];
        }
    }
    void get(float T[16]) const {
        float U[3][3], S[3], V[3][3];
        svd3(cov, U, S, V);
        float s22 = (det3(U) * det3(V) < 0.0f) ? -1.0f : 1.0f;
        float US[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) {
                // (U*S)(i,j) = U(i,0)S(0,j) + (U(i,1)S(1,j) + U(i,2)S(2,j))
                float Sd[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, s22}};
                US[i][j] = sum3(U[i][0] * Sd[0][j], U[i][1] * Sd[1][j], U[i][2] * Sd[2][j]);
            }
        float R[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R[i][j] = sum3(US[i][0] * V[j][0], US[i][1] * V[j][1], US[i][2] * V[j][2]);
        float t[3];
        for (int i = 0; i < 3; i++) t[i] = mean2[i] - sum3(R[i][0] * mean1[0], R[i][1] * mean1[1], R[i][2] * mean1[2]);
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++) T[i * 4 + j] = R[i][j];
            T[i * 4 + 3] = t[i];
        }
        T[12] = T[13] = T[14] = 0.f;
        T[15] = 1.f;
    }
};

// ------------------------------------------------------------ frame geometry
// cv::undistortPoints(src, dst, K, D(k1,k2,p1,p2,k3), noArray(), K), 5 iterations, double.
void undistort_point(float u, float v, const odo_calib& c, float* uo, float* vo) {
    const double fx = c.fx, fy = c.fy, cx = c.cx, cy = c.cy;
    const double ifx = 1. / fx, ify = 1. / fy;
    const double k[5] = {c.k1, c.k2, c.p1, c.p2, c.k3};
    double x = u, y = v;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < 5; j++) {
        double r2 = x * x + y * y;
        double icdist = 1 / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    double xx = fx * x + cx;
    double yy = fy * y + cy;
    *uo = (float)xx;
    *vo = (float)yy;
}

// ------------------------------------------------------------ matching
inline int hamming32(const uint8_t* a, const uint8_t* b) {
    // cv::norm(NORM_HAMMING) over 256 bits, 64-bit words
    uint64_t x[4], y[4];
    memcpy(x, a, 32);
    memcpy(y, b, 32);
    return __builtin_popcountll(x[0] ^ y[0]) + __builtin_popcountll(x[1] ^ y[1]) +
           __builtin_popcountll(x[2] ^ y[2]) + __builtin_popcountll(x[3] ^ y[3]);
}

// ------------------------------------------------------------ RANSAC
struct DM {
    int queryIdx, trainIdx, imgIdx;
    float distance;
    bool operator<(const DM& o) const { return distance < o.distance; }  // cv::DMatch::operator<
};

struct RansacState {
    const float* xyz1;
    const float* xyz2;
    odo_ransac_params p;
    odo_rng* rng;
    double* latch;
    // algorithmic work of the visited iterations
    int n_sweeps = 0;      // ComputeInliersAndError calls
    int n_fit_points = 0;  // points added to TransformationFromCorrespondences
};

int32_t rng_next(odo_rng* r);

double depth_covariance(RansacState& S, double depth) {
    // ransac.cpp:416-421: function-local statics latch on the first call
    if (std::isnan(*S.latch)) {
        double stddev = 0.01 * depth * depth;
        *S.latch = stddev * stddev;
    }
    return *S.latch;
}

double error_function2(RansacState& S, const float x1[3], const float x2[3], const double T[4][4]) {
    // ransac.cpp:350-414
    static const double cam_angle_x = 58.0 / 180.0 * M_PI;
    static const double cam_angle_y = 45.0 / 180.0 * M_PI;
    static const double cam_resol_x = 640;
    static const double cam_resol_y = 480;
    static const double raster_stddev_x = 3 * tan(cam_angle_x / cam_resol_x);
    static const double raster_stddev_y = 3 * tan(cam_angle_y / cam_resol_y);
    static const double raster_cov_x = raster_stddev_x * raster_stddev_x;
    static const double raster_cov_y = raster_stddev_y * raster_stddev_y;
    if (std::isnan(x1[2]) || std::isnan(x2[2])) return std::numeric_limits<double>::max();
    const double a[4] = {x1[0], x1[1], x1[2], 1.0};
    const double mu2[3] = {x2[0], x2[1], x2[2]};
    double m12[3];
    for (int i = 0; i < 4 - 1; i++)  // (tf_12 * x_1).head<3>(): ((p0+p1)+p2)+p3
        m12[i] = ((T[i][0] * a[0] + T[i][1] * a[1]) + T[i][2] * a[2]) + T[i][3] * a[3];
    {
        double d0 = m12[0] - mu2[0], d1 = m12[1] - mu2[1], d2 = m12[2] - mu2[2];
        double delta_sq_norm = sum3(d0 * d0, d1 * d1, d2 * d2);
        double sigma_max_1 = std::max(raster_cov_x, depth_covariance(S, a[2]));
        double sigma_max_2 = std::max(raster_cov_x, depth_covariance(S, mu2[2]));
        if (delta_sq_norm > 2.0 * (sigma_max_1 + sigma_max_2)) return std::numeric_limits<double>::max();
    }
    double R[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R[i][j] = T[i][j];
    double cov1[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}, cov2[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    cov1[0][0] = raster_cov_x * a[2];
    cov1[1][1] = raster_cov_y * a[2];
    cov1[2][2] = depth_covariance(S, a[2]);
    cov2[0][0] = raster_cov_x * mu2[2];
    cov2[1][1] = raster_cov_y * mu2[2];
    cov2[2][2] = depth_covariance(S, mu2[2]);
    double RtC[3][3], C1[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) RtC[i][j] = sum3(R[0][i] * cov1[0][j], R[1][i] * cov1[1][j], R[2][i] * cov1[2][j]);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) C1[i][j] = sum3(RtC[i][0] * R[0][j], RtC[i][1] * R[1][j], RtC[i][2] * R[2][j]);
    double delta[3] = {m12[0] - mu2[0], m12[1] - mu2[1], m12[2] - mu2[2]};
    if (std::isnan(delta[2])) return std::numeric_limits<double>::max();
    double A[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) A[i][j] = C1[i][j] + cov2[i][j];
    // Eigen LLT<Matrix3d> (lower, unblocked) on the lower triangle.
    double L[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) L[i][j] = A[i][j];
    {
        // k = 0
        double x = L[0][0];
        bool ok = x > 0;
        if (ok) {
            L[0][0] = x = sqrt(x);
            L[1][0] /= x;
            L[2][0] /= x;
            // k = 1
            x = L[1][1] - L[1][0] * L[1][0];
            ok = x > 0;
            if (ok) {
                L[1][1] = x = sqrt(x);
                L[2][1] -= L[2][0] * L[1][0];
                L[2][1] /= x;
                // k = 2
                x = L[2][2] - (L[2][0] * L[2][0] + L[2][1] * L[2][1]);
                ok = x > 0;
                if (ok) L[2][2] = sqrt(x);
            }
        }
        (void)ok;  // Eigen's solve() ignores info(); the partially factored matrix is used
    }
    // solveInPlace: L y = delta (unrolled, row dot form), then L^T x = y.
    double y0 = delta[0] / L[0][0];
    double y1 = (delta[1] - L[1][0] * y0) / L[1][1];
    double y2 = (delta[2] - (L[2][0] * y0 + L[2][1] * y1)) / L[2][2];
    double z2 = y2 / L[2][2];
    double z1 = (y1 - L[2][1] * z2) / L[1][1];
    double z0 = (y0 - (L[1][0] * z1 + L[2][0] * z2)) / L[0][0];
    double d2 = sum3(delta[0] * z0, delta[1] * z1, delta[2] * z2);
    if (!(d2 >= 0.0)) return std::numeric_limits<double>::max();
    return d2;
}

double compute_inliers_and_error(RansacState& S, const std::vector<DM>& m12, const float T[16],
                                 std::vector<DM>& inl) {
    // ransac.cpp:315-348
    inl.clear();
    double meanError = 0.0;
    double Td[4][4];
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) Td[i][j] = (double)T[i * 4 + j];
    const float th = S.p.max_mahalanobis * S.p.max_mahalanobis;
    S.n_sweeps++;
    for (const DM& m : m12) {
        const float* o = &S.xyz1[3 * m.queryIdx];
        const float* t = &S.xyz2[3 * m.trainIdx];
        if (o[2] == 0.0f || t[0] == 0.0f) continue;  // sic: target.x (ransac.cpp:326)
        double d = error_function2(S, o, t, Td);
        if (d > th) continue;
        if (!(d >= 0.0)) continue;
        meanError += d;
        inl.push_back(m);
    }
    if (inl.size() < 3) meanError = 1e9;
    else {
        meanError /= inl.size();
        meanError = sqrt(meanError);
    }
    return meanError;
}

void transform_from_matches(RansacState& S, const std::vector<DM>& v, float T[16]) {
    // ransac.cpp:295-313
    TFC tfc;
    for (const DM& m : v) {
        const float* f = &S.xyz1[3 * m.queryIdx];
        const float* t = &S.xyz2[3 * m.trainIdx];
        if (std::isnan(f[2]) || std::isnan(t[2])) continue;
        float weight = 1.0f / (f[2] * t[2]);
        tfc.add(f, t, weight);
        S.n_fit_points++;
    }
    tfc.get(T);
}

std::vector<DM> sample_matches(RansacState& S, const std::vector<DM>& v) {
    // ransac.cpp:269-293
    std::set<size_t> ids;
    int safety = 0;
    while (ids.size() < (size_t)S.p.sample_size && v.size() >= (size_t)S.p.sample_size) {
        int id1 = rng_next(S.rng) % v.size();
        int id2 = rng_next(S.rng) % v.size();
        if (id1 > id2) id1 = id2;
        ids.insert(id1);
        if (++safety > 10000) break;
    }
    std::vector<DM> out;
    for (size_t id : ids) out.push_back(v[id]);
    return out;
}

bool ransac_iterate(RansacState& S, const std::vector<DM>& m12, float T12[16], float* rmse_out,
                    std::vector<DM>& inliers, int* visited, int* n_good) {
    // ransac.cpp:155-267
    std::vector<DM> mvInliers;
    float rmse = 1e6;
    float mT12[16];
    for (int i = 0; i < 16; i++) mT12[i] = (i % 5 == 0) ? 1.f : 0.f;
    *visited = 0;
    *n_good = 0;
    auto finish = [&](bool r) {
        memcpy(T12, mT12, sizeof(mT12));
        *rmse_out = rmse;
        inliers = mvInliers;
        return r;
    };
    const size_t minInl = (size_t)S.p.min_inlier_th;
    if (m12.size() < minInl) return finish(false);
    std::vector<DM> good;
    for (const DM& m : m12) {
        const float* s = &S.xyz1[3 * m.queryIdx];
        const float* t = &S.xyz2[3 * m.trainIdx];
        if (S.p.check_depth) {
            if (std::isnan(s[2]) || std::isnan(t[2])) continue;
            if (s[2] <= 0 || t[2] <= 0) continue;
        }
        good.push_back(m);
    }
    *n_good = (int)good.size();
    if (good.size() < minInl) return finish(false);
    int validIters = 0;
    double inlierError;
    std::sort(good.begin(), good.end());
    for (int n = 0; (n < S.p.iterations && good.size() >= (size_t)S.p.sample_size); n++) {
        double refinedError = 1e6;
        std::vector<DM> refined;
        std::vector<DM> inl = sample_matches(S, good);
        float refinedT[16];
        for (int i = 0; i < 16; i++) refinedT[i] = (i % 5 == 0) ? 1.f : 0.f;
        (*visited)++;
        for (int refinements = 1; refinements < 20; refinements++) {
            float T[16];
            transform_from_matches(S, inl, T);
            inlierError = compute_inliers_and_error(S, good, T, inl);
            if (inl.size() < minInl || inlierError > S.p.max_mahalanobis) break;
            if (inl.size() >= refined.size() && inlierError <= refinedError) {
                size_t prev = refined.size();
                memcpy(refinedT, T, sizeof(T));
                refined = inl;
                refinedError = inlierError;
                if (inl.size() == prev) break;
            } else break;
        }
        if (refined.size() > 0) {
            validIters++;
            if (refinedError <= rmse && refined.size() >= mvInliers.size() && refined.size() >= minInl) {
                rmse = refinedError;
                memcpy(mT12, refinedT, sizeof(refinedT));
                mvInliers = refined;
                if (refined.size() > good.size() * 0.5) n += 10;
                if (refined.size() > good.size() * 0.75) n += 10;
                if (refined.size() > good.size() * 0.8) break;
            }
        }
    }
    if (validIters == 0) {
        float I[16];
        for (int i = 0; i < 16; i++) I[i] = (i % 5 == 0) ? 1.f : 0.f;
        std::vector<DM> inl;
        inlierError = compute_inliers_and_error(S, good, I, inl);
        if (inl.size() > minInl && inlierError < S.p.max_mahalanobis) {
            memcpy(mT12, I, sizeof(I));
            mvInliers = inl;
            rmse += inlierError;
        }
    }
    return finish(mvInliers.size() >= minInl);
}

// ------------------------------------------------------------ g2o restatement
struct Quat { double x, y, z, w; };

Quat qmul(const Quat& a, const Quat& b) {
    return Quat{a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y, a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
                a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x, a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z};
}
void cross(const double a[3], const double b[3], double o[3]) {
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}
void qrot(const Quat& q, const double v[3], double o[3]) {  // Eigen _transformVector
    const double qv[3] = {q.x, q.y, q.z};
    double uv[3], uv2[3];
    cross(qv, v, uv);
    for (int i = 0; i < 3; i++) uv[i] += uv[i];
    cross(qv, uv, uv2);
    for (int i = 0; i < 3; i++) o[i] = v[i] + q.w * uv[i] + uv2[i];
}
Quat quat_from_R(const double m[3][3]) {  // Eigen quaternionbase_assign_impl<Matrix3>
    Quat q;
    double t = sum3(m[0][0], m[1][1], m[2][2]);
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
void quat_to_R(const Quat& q, double r[3][3]) {
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
struct SE3 {
    Quat q;
    double t[3];
    void normalize_rotation() {
        if (q.w < 0) { q.x = -q.x; q.y = -q.y; q.z = -q.z; q.w = -q.w; }
        double n = sqrt((q.x * q.x + q.y * q.y) + (q.z * q.z + q.w * q.w));
        q.x /= n; q.y /= n; q.z /= n; q.w /= n;
    }
    static SE3 from_Rt(const double R[3][3], const double tt[3]) {
        SE3 s;
        s.q = quat_from_R(R);
        for (int i = 0; i < 3; i++) s.t[i] = tt[i];
        s.normalize_rotation();
        return s;
    }
    void map(const double p[3], double o[3]) const {
        qrot(q, p, o);
        for (int i = 0; i < 3; i++) o[i] += t[i];
    }
    SE3 operator*(const SE3& b) const {
        SE3 r = *this;
        double rt[3];
        qrot(q, b.t, rt);
        for (int i = 0; i < 3; i++) r.t[i] += rt[i];
        r.q = qmul(q, b.q);
        r.normalize_rotation();
        return r;
    }
    static SE3 exp(const double u[6]) {
        const double w[3] = {u[0], u[1], u[2]};
        const double up[3] = {u[3], u[4], u[5]};
        double theta = sqrt(sum3(w[0] * w[0], w[1] * w[1], w[2] * w[2]));
        double O[3][3] = {{0, -w[2], w[1]}, {w[2], 0, -w[0]}, {-w[1], w[0], 0}};
        double O2[3][3];
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) O2[i][j] = sum3(O[i][0] * O[0][j], O[i][1] * O[1][j], O[i][2] * O[2][j]);
        double R[3][3], V[3][3];
        if (theta < 0.00001) {
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) R[i][j] = ((i == j ? 1.0 : 0.0) + O[i][j]) + O2[i][j];
            memcpy(V, R, sizeof(R));
        } else {
            double a = sin(theta) / theta, b = (1 - cos(theta)) / (theta * theta);
            double c = (theta - sin(theta)) / pow(theta, 3);
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    R[i][j] = ((i == j ? 1.0 : 0.0) + a * O[i][j]) + b * O2[i][j];
                    V[i][j] = ((i == j ? 1.0 : 0.0) + b * O[i][j]) + c * O2[i][j];
                }
        }
        double tt[3];
        for (int i = 0; i < 3; i++) tt[i] = sum3(V[i][0] * up[0], V[i][1] * up[1], V[i][2] * up[2]);
        SE3 s;
        s.q = quat_from_R(R);
        for (int i = 0; i < 3; i++) s.t[i] = tt[i];
        s.normalize_rotation();
        return s;
    }
};

struct Edge {
    bool stereo;
    double Xw[3];
    double obs[3];
    double info;      // sigma (information = sigma * I)
    double err[3];    // stored _error
    int level;        // 0 active, 1 outlier
    bool robust;
    double delta;     // Huber delta
};

struct PnPProblem {
    double fx, fy, cx, cy, bf;
    std::vector<Edge> edges;

    void compute_error(Edge& e, const SE3& T) const {
        double Xc[3];
        T.map(e.Xw, Xc);
        if (!e.stereo) {
            double px = Xc[0] / Xc[2], py = Xc[1] / Xc[2];
            e.err[0] = e.obs[0] - (px * fx + cx);
            e.err[1] = e.obs[1] - (py * fy + cy);
            e.err[2] = 0;
        } else {
            const float invz = 1.0f / Xc[2];
            double r0 = Xc[0] * invz * fx + cx;
            double r1 = Xc[1] * invz * fy + cy;
            double r2 = r0 - bf * invz;
            e.err[0] = e.obs[0] - r0;
            e.err[1] = e.obs[1] - r1;
            e.err[2] = e.obs[2] - r2;
        }
    }
    static double chi2(const Edge& e) {
        if (!e.stereo) return e.err[0] * (e.info * e.err[0]) + e.err[1] * (e.info * e.err[1]);
        return sum3(e.err[0] * (e.info * e.err[0]), e.err[1] * (e.info * e.err[1]), e.err[2] * (e.info * e.err[2]));
    }
    static void robustify(const Edge& e, double chi, double rho[3]) {
        double dsqr = e.delta * e.delta;
        if (chi <= dsqr) { rho[0] = chi; rho[1] = 1.; rho[2] = 0.; }
        else {
            double sq = sqrt(chi);
            rho[0] = 2 * sq * e.delta - dsqr;
            rho[1] = e.delta / sq;
            rho[2] = -0.5 * rho[1] / chi;
        }
    }
    void jacobian(const Edge& e, const SE3& T, double J[3][6]) const {
        double Xc[3];
        T.map(e.Xw, Xc);
        double x = Xc[0], y = Xc[1], invz = 1.0 / Xc[2], invz_2 = invz * invz;
        J[0][0] = x * y * invz_2 * fx;
        J[0][1] = -(1 + (x * x * invz_2)) * fx;
        J[0][2] = y * invz * fx;
        J[0][3] = -invz * fx;
        J[0][4] = 0;
        J[0][5] = x * invz_2 * fx;
        J[1][0] = (1 + y * y * invz_2) * fy;
        J[1][1] = -x * y * invz_2 * fy;
        J[1][2] = -x * invz * fy;
        J[1][3] = 0;
        J[1][4] = -invz * fy;
        J[1][5] = y * invz_2 * fy;
        if (e.stereo) {
            J[2][0] = J[0][0] - bf * y * invz_2;
            J[2][1] = J[0][1] + bf * x * invz_2;
            J[2][2] = J[0][2];
            J[2][3] = J[0][3];
            J[2][4] = 0;
            J[2][5] = J[0][5] - bf * invz_2;
        }
    }
    double active_robust_chi2() const {
        double chi = 0;
        for (const Edge& e : edges) {
            if (e.level != 0) continue;
            double c = chi2(e);
            if (e.robust) {
                double rho[3];
                robustify(e, c, rho);
                chi += rho[0];
            } else chi += c;
        }
        return chi;
    }
    void compute_active_errors(const SE3& T) {
        for (Edge& e : edges)
            if (e.level == 0) compute_error(e, T);
    }
    void build_system(const SE3& T, double H[6][6], double b[6]) const {
        memset(H, 0, sizeof(double) * 36);
        memset(b, 0, sizeof(double) * 6);
        for (const Edge& e : edges) {
            if (e.level != 0) continue;
            double J[3][6];
            jacobian(e, T, J);
            int D = e.stereo ? 3 : 2;
            double w = e.info, r1 = 1.0;
            if (e.robust) {
                double rho[3];
                robustify(e, chi2(e), rho);
                r1 = rho[1];
            }
            double wo = r1 * e.info;  // robustInformation
            for (int a = 0; a < 6; a++) {
                double s = 0;
                for (int k = 0; k < D; k++) s += J[k][a] * (w * e.err[k]);
                b[a] -= r1 * s;
                for (int c = 0; c < 6; c++) {
                    double h = 0;
                    for (int k = 0; k < D; k++) h += J[k][a] * wo * J[k][c];
                    H[a][c] += h;
                }
            }
        }
    }
};

// Eigen LDLT (lower, diagonal pivoting) solve of a 6x6 SPD system.
bool ldlt_solve6(const double Ain[6][6], const double b[6], double x[6]) {
    const int n = 6;
    double m[6][6];
    memcpy(m, Ain, sizeof(m));
    int tr[6];
    int sign = 0;  // 0 zero, 1 pos semidef, 2 neg semidef, 3 indefinite
    for (int k = 0; k < n; ++k) {
        int big = k;
        double bv = std::abs(m[k][k]);
        for (int i = k + 1; i < n; i++)
            if (std::abs(m[i][i]) > bv) { bv = std::abs(m[i][i]); big = i; }
        tr[k] = big;
        if (k != big) {
            for (int j = 0; j < k; j++) std::swap(m[k][j], m[big][j]);
            for (int i = big + 1; i < n; i++) std::swap(m[i][k], m[i][big]);
            std::swap(m[k][k], m[big][big]);
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
                double t = 0;
                for (int j = 0; j < k; j++) t += m[i][j] * temp[j];
                m[i][k] -= t;
            }
        }
        double akk = m[k][k];
        bool valid = std::abs(akk) > 0;
        if (k == 0 && !valid) return false;
        if (valid)
            for (int i = k + 1; i < n; i++) m[i][k] /= akk;
        if (sign == 1) { if (akk < 0) sign = 3; }
        else if (sign == 2) { if (akk > 0) sign = 3; }
        else if (sign == 0) { if (akk > 0) sign = 1; else if (akk < 0) sign = 2; }
    }
    if (!(sign == 1 || sign == 0)) return false;
    double y[6];
    memcpy(y, b, sizeof(y));
    for (int k = 0; k < n; k++) std::swap(y[k], y[tr[k]]);
    for (int i = 0; i < n; i++) {
        double s = 0;
        for (int j = 0; j < i; j++) s += m[i][j] * y[j];
        y[i] -= s;
    }
    for (int i = 0; i < n; i++) {
        if (std::abs(m[i][i]) > DBL_MIN) y[i] /= m[i][i];
        else y[i] = 0;
    }
    for (int i = n - 1; i >= 0; i--) {
        double s = 0;
        for (int j = i + 1; j < n; j++) s += m[j][i] * y[j];
        y[i] -= s;
    }
    for (int k = n - 1; k >= 0; k--) std::swap(y[k], y[tr[k]]);
    memcpy(x, y, sizeof(y));
    return true;
}

// SparseOptimizer::optimize(iterations) with OptimizationAlgorithmLevenberg.
void lm_optimize(PnPProblem& P, SE3& T, int iterations) {
    double lambda = 0, ni = 2;
    for (int it = 0; it < iterations; it++) {
        P.compute_active_errors(T);
        double currentChi = P.active_robust_chi2();
        double H[6][6], b[6];
        P.build_system(T, H, b);
        if (it == 0) {
            double mx = 0;
            for (int j = 0; j < 6; j++) mx = std::max(std::abs(H[j][j]), mx);
            lambda = 1e-5 * mx;
            ni = 2;
        }
        double rho = 0;
        int qmax = 0;
        do {
            SE3 backup = T;
            double Hl[6][6];
            memcpy(Hl, H, sizeof(H));
            for (int j = 0; j < 6; j++) Hl[j][j] += lambda;
            double x[6] = {0, 0, 0, 0, 0, 0};
            bool ok2 = ldlt_solve6(Hl, b, x);
            T = SE3::exp(x) * T;
            P.compute_active_errors(T);
            double tempChi = P.active_robust_chi2();
            if (!ok2) tempChi = std::numeric_limits<double>::max();
            rho = currentChi - tempChi;
            double scale = 0;
            for (int j = 0; j < 6; j++) scale += x[j] * (lambda * x[j] + b[j]);
            scale += 1e-3;
            rho /= scale;
            if (rho > 0 && std::isfinite(tempChi)) {
                double alpha = 1. - pow((2 * rho - 1), 3);
                alpha = std::min(alpha, 2. / 3.);
                double scaleFactor = std::max(1. / 3., alpha);
                lambda *= scaleFactor;
                ni = 2;
                currentChi = tempChi;
            } else {
                lambda *= ni;
                ni *= 2;
                T = backup;
            }
            qmax++;
        } while (rho < 0 && qmax < 10);
        if (qmax == 10 || rho == 0) break;
    }
}

int pnp_compute(const float* Xw, const float* obs, int n, const odo_calib& c, const float Tcw[16],
                float Tout[16], uint8_t* outlier) {
    // pnpsolver.cpp:17-214
    PnPProblem P;
    P.fx = (double)c.fx;
    P.fy = (double)c.fy;
    P.cx = (double)c.cx;
    P.cy = (double)c.cy;
    P.bf = (double)c.mbf;
    const float deltaMono = sqrt(5.991);
    const float deltaStereo = sqrt(7.815);
    int nInitial = 0;
    for (int i = 0; i < n; i++) {
        Edge e;
        e.stereo = !(obs[3 * i + 2] < 0);
        nInitial++;
        outlier[i] = 0;
        for (int k = 0; k < 3; k++) e.Xw[k] = Xw[3 * i + k];
        e.obs[0] = obs[3 * i];
        e.obs[1] = obs[3 * i + 1];
        e.obs[2] = e.stereo ? obs[3 * i + 2] : 0;
        const float sigma = 1.0f / (Xw[3 * i + 2] * Xw[3 * i + 2]);
        e.info = sigma;
        e.robust = true;
        e.delta = e.stereo ? deltaStereo : deltaMono;
        e.level = 0;
        e.err[0] = e.err[1] = e.err[2] = 0;
        P.edges.push_back(e);
    }
    if (nInitial < 3) {
        memcpy(Tout, Tcw, sizeof(float) * 16);
        return 0;
    }
    const float chi2Mono[4] = {5.991, 5.991, 5.991, 5.991};
    const float chi2Stereo[4] = {7.815, 7.815, 7.815, 7.815};
    double R0[3][3], t0[3];
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) R0[i][j] = Tcw[i * 4 + j];
        t0[i] = Tcw[i * 4 + 3];
    }
    SE3 T;
    int nBad = 0;
    for (int it = 0; it < 4; it++) {
        T = SE3::from_Rt(R0, t0);
        lm_optimize(P, T, 10);
        nBad = 0;
        // mono edges first, then stereo (pnpsolver.cpp:157-201)
        for (int pass = 0; pass < 2; pass++) {
            for (int i = 0; i < n; i++) {
                Edge& e = P.edges[i];
                if (e.stereo != (pass == 1)) continue;
                if (outlier[i]) P.compute_error(e, T);
                const float chi2 = PnPProblem::chi2(e);
                const float th = e.stereo ? chi2Stereo[it] : chi2Mono[it];
                if (chi2 > th) {
                    outlier[i] = 1;
                    e.level = 1;
                    nBad++;
                } else {
                    outlier[i] = 0;
                    e.level = 0;
                }
                if (it == 2) e.robust = false;
            }
        }
        if ((int)P.edges.size() < 10) break;
    }
    double R[3][3];
    quat_to_R(T.q, R);
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) Tout[i * 4 + j] = (float)R[i][j];
        Tout[i * 4 + 3] = (float)T.t[i];
    }
    Tout[12] = Tout[13] = Tout[14] = 0.f;
    Tout[15] = 1.f;
    return nInitial - nBad;
}

// ------------------------------------------------------------ glibc rand
void to_random_data(odo_rng* r, struct random_data* rd) {
    memset(rd, 0, sizeof(*rd));
    rd->state = r->state;
    rd->fptr = r->state + r->fpos;
    rd->rptr = r->state + r->rpos;
    rd->rand_type = 3;
    rd->rand_deg = 31;
    rd->rand_sep = 3;
    rd->end_ptr = r->state + 31;
}

int32_t rng_next(odo_rng* r) {
    struct random_data rd;
    to_random_data(r, &rd);
    int32_t out;
    random_r(&rd, &out);
    r->fpos = (int)(rd.fptr - r->state);
    r->rpos = (int)(rd.rptr - r->state);
    return out;
}

}  // namespace

// ================================================================ C API
extern "C" {

// std::sort(vector<cv::DMatch>) as in Ransac::Iterate (ransac.cpp:199):
// libstdc++ introsort by distance (cv::DMatch::operator<), unstable.
void oracle_sort_dmatch(void* v, int n) {
    DM* a = static_cast<DM*>(v);
    std::sort(a, a + n);
}

void oracle_frame_geometry(const orb_kp* kps, int n, const float* depth, int w, int h,
                           const odo_calib* c, float* kps_un, float* xyz, float* u_right) {
    (void)h;
    const float invfx = 1.0f / c->fx, invfy = 1.0f / c->fy;
    for (int i = 0; i < n; i++) {
        float uu = kps[i].x, vv = kps[i].y;
        if (c->k1 == 0.0f) {
            kps_un[2 * i] = uu;
            kps_un[2 * i + 1] = vv;
        } else {
            undistort_point(uu, vv, *c, &kps_un[2 * i], &kps_un[2 * i + 1]);
        }
        xyz[3 * i] = xyz[3 * i + 1] = xyz[3 * i + 2] = 0.f;
        u_right[i] = -1;
        const float z = depth[(size_t)((int)vv) * w + (int)uu];
        if (z > 0) {
            u_right[i] = kps_un[2 * i] - c->mbf / z;
            xyz[3 * i] = (kps_un[2 * i] - c->cx) * z * invfx;
            xyz[3 * i + 1] = (kps_un[2 * i + 1] - c->cy) * z * invfy;
            xyz[3 * i + 2] = z;
        }
    }
}

int oracle_extract_frame(const uint8_t* bgr, const uint16_t* depth, int w, int h,
                         const odo_orb_params* p, const odo_calib* c, orb_kp* kps, uint8_t* desc,
                         float* kps_un, float* xyz, float* u_right, int cap) {
    std::vector<uint8_t> gray((size_t)w * h);
    std::vector<float> z((size_t)w * h);
    oracle_bgr2gray(bgr, w, h, 3 * w, gray.data());
    oracle_depth_to_f32(depth, w * h, c->depth_factor, z.data());
    int n = oracle_orb_extract(gray.data(), w, h, p, kps, desc, cap);
    int m = std::min(n, cap);
    oracle_frame_geometry(kps, m, z.data(), w, h, c, kps_un, xyz, u_right);
    return n;
}

int oracle_extract_frame_adaptive(const uint8_t* bgr, const uint16_t* depth, int w, int h,
                                  const odo_adaptive_params* p, double* thresh, const odo_calib* c,
                                  orb_kp* kps, uint8_t* desc, float* kps_un, float* xyz, float* u_right,
                                  int cap) {
    std::vector<uint8_t> gray((size_t)w * h);
    std::vector<float> z((size_t)w * h);
    oracle_bgr2gray(bgr, w, h, 3 * w, gray.data());
    oracle_depth_to_f32(depth, w * h, c->depth_factor, z.data());
    int n = oracle_adaptive_extract(gray.data(), w, h, p, thresh, kps, desc, cap, nullptr);
    int m = std::min(n, cap);
    oracle_frame_geometry(kps, m, z.data(), w, h, c, kps_un, xyz, u_right);
    return n;
}

// The same with the cv::ORB inner detector (Extractor(ORB, ORB, ADAPTIVE)).
int oracle_extract_frame_adaptive_orb(const uint8_t* bgr, const uint16_t* depth, int w, int h,
                                      const odo_adaptive_params* p, double* thresh, const odo_calib* c,
                                      orb_kp* kps, uint8_t* desc, float* kps_un, float* xyz, float* u_right,
                                      int cap) {
    std::vector<uint8_t> gray((size_t)w * h);
    std::vector<float> z((size_t)w * h);
    oracle_bgr2gray(bgr, w, h, 3 * w, gray.data());
    oracle_depth_to_f32(depth, w * h, c->depth_factor, z.data());
    int n = oracle_adaptive_orb_extract(gray.data(), w, h, p, thresh, kps, desc, cap, nullptr);
    int m = std::min(n, cap);
    oracle_frame_geometry(kps, m, z.data(), w, h, c, kps_un, xyz, u_right);
    return n;
}

// Frame::ComputeImageBounds (frame.cpp:315-349): undistorted image corners.
void oracle_image_bounds(const odo_calib* c, int w, int h, float* b) {
    if (c->k1 != 0.0f) {
        const float cu[4] = {0.f, (float)w, 0.f, (float)w}, cv_[4] = {0.f, 0.f, (float)h, (float)h};
        float u[4], v[4];
        for (int i = 0; i < 4; i++) undistort_point(cu[i], cv_[i], *c, &u[i], &v[i]);
        b[0] = std::min(u[0], u[2]);
        b[1] = std::max(u[1], u[3]);
        b[2] = std::min(v[0], v[1]);
        b[3] = std::max(v[2], v[3]);
    } else {
        b[0] = 0.f;
        b[1] = (float)w;
        b[2] = 0.f;
        b[3] = (float)h;
    }
}

// Tracking::SearchLocalLMs (tracking.cpp:368-405): Frame::isInFrustum
// (frame.cpp:100-133) on every landmark neither bad nor already seen by the
// frame, then Matcher(0.8f)::ProjectionMatch(frame, landmarks, th)
// (matcher.cpp:90-145, TH_HIGH = 100, matcher.cpp:15-17) with
// GetFeaturesInArea's linear scan (frame.cpp:258-274). mRcw * P + mtcw is one
// folded cv::gemm (float data, double accumulation, one rounding). slot_taken:
// the frame slot holds a landmark with Observations() > 0. Outputs: slot_lm =
// landmark index added to the slot (AddLandmark) or -1; proj = (u, v, uR) of
// in-view landmarks (mTrackProjX/Y/XR), NaN otherwise. Returns nmatches.
int oracle_projection_match(const float* Tcw, const odo_landmark* lms, int nL, const float* kun,
                            const int32_t* octave, const uint8_t* desc, int n, const uint8_t* slot_taken,
                            const odo_calib* c, const float* bounds, float th, float nnratio, int32_t* slot_lm,
                            float* proj) {
    std::vector<uint8_t> taken(slot_taken, slot_taken + n);
    for (int j = 0; j < n; j++) slot_lm[j] = -1;
    std::vector<uint8_t> inview(nL, 0);
    const float nan = std::numeric_limits<float>::quiet_NaN();
    for (int i = 0; i < nL; i++) {
        proj[3 * i] = proj[3 * i + 1] = proj[3 * i + 2] = nan;
        const odo_landmark& L = lms[i];
        if (L.flags & (ODO_LM_BAD | ODO_LM_SEEN)) continue;
        float Pc[3];
        for (int k = 0; k < 3; k++)
            Pc[k] = (float)((((double)Tcw[4 * k] * L.X[0] + (double)Tcw[4 * k + 1] * L.X[1]) +
                             (double)Tcw[4 * k + 2] * L.X[2]) + (double)Tcw[4 * k + 3]);
        if (Pc[2] < 0.0f) continue;
        const float invz = 1.0f / Pc[2];
        const float u = c->fx * Pc[0] * invz + c->cx;
        const float v = c->fy * Pc[1] * invz + c->cy;
        if (u < bounds[0] || u > bounds[1]) continue;
        if (v < bounds[2] || v > bounds[3]) continue;
        inview[i] = 1;
        proj[3 * i] = u;
        proj[3 * i + 1] = v;
        proj[3 * i + 2] = u - c->mbf * invz;
    }
    const double TH_HIGH = 100.0;
    int nmatches = 0;
    for (int i = 0; i < nL; i++) {
        if (!inview[i]) continue;
        const odo_landmark& L = lms[i];
        if (L.flags & ODO_LM_BAD) continue;
        const float x = proj[3 * i], y = proj[3 * i + 1];
        std::vector<int> idx;
        for (int j = 0; j < n; j++) {
            const float distx = kun[2 * j] - x, disty = kun[2 * j + 1] - y;
            if (fabsf(distx) < th && fabsf(disty) < th) idx.push_back(j);
        }
        if (idx.empty()) continue;
        double best1 = std::numeric_limits<double>::max(), best2 = best1;
        int lvl1 = -1, lvl2 = -1, bidx = -1;
        for (int j : idx) {
            if (taken[j]) continue;
            const double d = (double)hamming32(L.desc, desc + 32 * (size_t)j);
            if (d < best1) {
                best2 = best1;
                best1 = d;
                lvl2 = lvl1;
                lvl1 = octave[j];
                bidx = j;
            } else if (d < best2) {
                lvl2 = octave[j];
                best2 = d;
            }
        }
        if (best1 <= TH_HIGH) {
            if (lvl1 == lvl2 && best1 > nnratio * best2) continue;
            slot_lm[bidx] = i;
            taken[bidx] = (L.flags & ODO_LM_HAS_OBS) ? 1 : 0;
            nmatches++;
        }
    }
    return nmatches;
}

void oracle_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx, int32_t* dist) {
    for (int i = 0; i < nq; i++) {
        int nidx[2] = {-1, -1};
        int dd[2] = {INT32_MAX, INT32_MAX};
        for (int j = 0; j < nt; j++) {
            int d = hamming32(q + 32 * (size_t)i, t + 32 * (size_t)j);
            if (d < dd[1]) {
                int k;
                for (k = 0; k >= 0 && dd[k] > d; k--) {
                    nidx[k + 1] = nidx[k];
                    dd[k + 1] = dd[k];
                }
                nidx[k + 1] = j;
                dd[k + 1] = d;
            }
        }
        idx[2 * i] = nidx[0];
        idx[2 * i + 1] = nidx[1];
        dist[2 * i] = dd[0];
        dist[2 * i + 1] = dd[1];
    }
}

int oracle_knn_match(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float ratio,
                     const uint8_t* f1_has_lm, const uint8_t* f1_outlier, const int32_t* f1_lm_obs,
                     int32_t* f2_lm_obs, int32_t* f2_lm_src, uint8_t* f2_outlier, odo_dmatch* out,
                     int cap) {
    std::vector<int32_t> idx(2 * (size_t)n1), dist(2 * (size_t)n1);
    oracle_knn2(d1, n1, d2, n2, idx.data(), dist.data());
    int nm = 0;
    for (int i = 0; i < n1; i++) {
        // m1 = matchesKnn[i][0], m2 = matchesKnn[i][1]; with n2 < 2 the
        // reference indexes past the list (UB): a missing neighbour counts as
        // distance INT_MAX here (pinned).
        if (idx[2 * i] < 0) continue;
        const float dd0 = (float)dist[2 * i];
        const float dd1 = (float)dist[2 * i + 1];
        if (dd0 < ratio * dd1) {
            const int i1 = i, i2 = idx[2 * i];
            if (!f1_has_lm[i1]) continue;
            if (f1_outlier[i1]) continue;
            if (f2_lm_obs[i2] >= 0 && f2_lm_obs[i2] > 0) continue;
            f2_lm_obs[i2] = f1_lm_obs[i1];
            f2_lm_src[i2] = i1;
            f2_outlier[i2] = 1;
            if (nm < cap) out[nm] = odo_dmatch{i1, i2, 0, dd0};
            nm++;
        }
    }
    return nm;
}

int oracle_vo_landmarks(const float* xyz, int n, float th_depth_m, uint8_t* has_lm) {
    std::vector<std::pair<float, size_t>> v;
    for (int i = 0; i < n; i++) {
        has_lm[i] = 0;
        float z = xyz[3 * i + 2];
        if (z > 0) v.push_back(std::make_pair(z, (size_t)i));
    }
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    int nPoints = 0;
    for (size_t j = 0; j < v.size(); j++) {
        has_lm[v[j].second] = 1;
        nPoints++;
        if (v[j].first > th_depth_m && nPoints > 100) break;
    }
    return nPoints;
}

void oracle_rng_seed(odo_rng* r, uint32_t seed) {
    char statebuf[128];  // per call: the oracle is called from several threads at once
    struct random_data rd;
    memset(&rd, 0, sizeof(rd));
    initstate_r(seed, statebuf, sizeof(statebuf), &rd);  // TYPE_3, seeded via srandom_r
    memcpy(r->state, rd.state, sizeof(r->state));
    r->fpos = (int)(rd.fptr - rd.state);
    r->rpos = (int)(rd.rptr - rd.state);
}

int32_t oracle_rng_next(odo_rng* r) { return rng_next(r); }

void oracle_libc_rand_stream(uint32_t seed, int n, int32_t* out) {
    srand(seed);
    for (int i = 0; i < n; i++) out[i] = rand();
}

// work counters of the calling thread's last oracle_ransac (measurement only)
static thread_local int g_last_sweeps = 0, g_last_fit_points = 0;

void oracle_last_ransac_work(int* sweeps, int* fit_points) {
    *sweeps = g_last_sweeps;
    *fit_points = g_last_fit_points;
}

int oracle_ransac(const odo_dmatch* m12, int n12, const float* xyz1, const float* xyz2,
                  const odo_ransac_params* p, odo_rng* rng, double* latch, float* T12, float* rmse,
                  odo_dmatch* inliers, int* n_inliers, int* visited, int* n_good) {
    RansacState S{xyz1, xyz2, *p, rng, latch};
    std::vector<DM> m(n12);
    for (int i = 0; i < n12; i++) m[i] = DM{m12[i].queryIdx, m12[i].trainIdx, m12[i].imgIdx, m12[i].distance};
    std::vector<DM> inl;
    bool ok = ransac_iterate(S, m, T12, rmse, inl, visited, n_good);
    g_last_sweeps = S.n_sweeps;
    g_last_fit_points = S.n_fit_points;
    for (size_t i = 0; i < inl.size(); i++)
        inliers[i] = odo_dmatch{inl[i].queryIdx, inl[i].trainIdx, inl[i].imgIdx, inl[i].distance};
    *n_inliers = (int)inl.size();
    return ok ? 1 : 0;
}

// Hypotheses mode: the refinement loop of ransac.cpp:201-231
// for visited iterations [h0, h1) only, from the same rand() stream (samples
// of iterations < h0 are drawn and discarded); no fold. rng is not advanced.
int oracle_ransac_hyps(const odo_dmatch* m12, int n12, const float* xyz1, const float* xyz2,
                       const odo_ransac_params* p, const odo_rng* rng_in, double* latch, int h0, int h1,
                       odo_hyp_summary* out) {
    odo_rng rng = *rng_in;
    RansacState S{xyz1, xyz2, *p, &rng, latch};
    for (int h = h0; h < h1; h++) out[h - h0] = odo_hyp_summary{1e6, 0, 0, {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0}};
    const size_t minInl = (size_t)p->min_inlier_th;
    if ((size_t)n12 < minInl) return 0;
    std::vector<DM> good;
    for (int i = 0; i < n12; i++) {
        const DM m{m12[i].queryIdx, m12[i].trainIdx, m12[i].imgIdx, m12[i].distance};
        const float* s = &xyz1[3 * m.queryIdx];
        const float* t = &xyz2[3 * m.trainIdx];
        if (p->check_depth) {
            if (std::isnan(s[2]) || std::isnan(t[2])) continue;
            if (s[2] <= 0 || t[2] <= 0) continue;
        }
        good.push_back(m);
    }
    if (good.size() < minInl) return 0;
    std::sort(good.begin(), good.end());
    for (int h = 0; h < h1 && good.size() >= (size_t)p->sample_size; h++) {
        std::vector<DM> inl = sample_matches(S, good);
        if (h < h0) continue;
        double refinedError = 1e6;
        std::vector<DM> refined;
        float refinedT[16];
        for (int i = 0; i < 16; i++) refinedT[i] = (i % 5 == 0) ? 1.f : 0.f;
        for (int refinements = 1; refinements < 20; refinements++) {
            float T[16];
            transform_from_matches(S, inl, T);
            const double inlierError = compute_inliers_and_error(S, good, T, inl);
            if (inl.size() < minInl || inlierError > p->max_mahalanobis) break;
            if (inl.size() >= refined.size() && inlierError <= refinedError) {
                const size_t prev = refined.size();
                memcpy(refinedT, T, sizeof(T));
                refined = inl;
                refinedError = inlierError;
                if (inl.size() == prev) break;
            } else break;
        }
        odo_hyp_summary& o = out[h - h0];
        o.err = refinedError;
        o.cnt = (int)refined.size();
        memcpy(o.T, refinedT, 48);
    }
    return (int)good.size();
}

void oracle_tfc(const float* src, const float* tgt, const float* w, int n, float* T) {
    TFC t;
    for (int i = 0; i < n; i++) t.add(&src[3 * i], &tgt[3 * i], w[i]);
    t.get(T);
}

void oracle_svd3(const float* A, float* U, float* S, float* V) {
    float a[3][3], u[3][3], v[3][3];
    for (int i = 0; i < 9; i++) a[i / 3][i % 3] = A[i];
    svd3(a, u, S, v);
    for (int i = 0; i < 9; i++) {
        U[i] = u[i / 3][i % 3];
        V[i] = v[i / 3][i % 3];
    }
}

int oracle_pnp(const float* Xw, const float* obs, int n, const odo_calib* c, const float* Tcw_init,
               float* Tcw_out, uint8_t* outlier) {
    return pnp_compute(Xw, obs, n, *c, Tcw_init, Tcw_out, outlier);
}

void oracle_kabsch(const float* A, const float* B, int n, float* T) {
    // kabsch.cpp:14-57
    for (int i = 0; i < 16; i++) T[i] = (i % 5 == 0) ? 1.f : 0.f;
    if (n == 0) return;
    float cA[3], cB[3];
    for (int k = 0; k < 3; k++) {
        float sa = 0, sb = 0;
        for (int i = 0; i < n; i++) { sa += A[3 * i + k]; sb += B[3 * i + k]; }
        cA[k] = sa / n;
        cB[k] = sb / n;
    }
    float M[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            float s = 0;
            for (int i = 0; i < n; i++) s += (A[3 * i + a] - cA[a]) * (B[3 * i + b] - cB[b]);
            M[a][b] = s;
        }
    float Vm[3][3], S[3], Wm[3][3];
    svd3(M, Vm, S, Wm);  // V = svd.matrixU(), W = svd.matrixV()
    float d = det3(M);
    float sg = (d != 0) ? ((d > 0) - (d < 0)) : 1.f;
    float R[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            float s = 0;
            for (int k = 0; k < 3; k++) s += Wm[i][k] * (k == 2 ? sg : 1.f) * Vm[j][k];
            R[i][j] = s;
        }
    for (int i = 0; i < 3; i++) {
        float t = 0;
        for (int k = 0; k < 3; k++) t += R[i][k] * (-cA[k]);
        t += cB[i];
        for (int j = 0; j < 3; j++) T[i * 4 + j] = R[i][j];
        T[i * 4 + 3] = t;
    }
}

int oracle_track_pair(const orb_kp* k1, const uint8_t* d1, const float* xyz1, int n1,
                      const orb_kp* k2, const uint8_t* d2, const float* kun2, const float* xyz2,
                      const float* ur2, int n2, const odo_calib* c, float ratio,
                      const odo_ransac_params* rp, uint32_t seed, double* latch, odo_pair_result* res,
                      uint8_t* inlier_mask, odo_dmatch* matches, int cap,
                      odo_dmatch* ransac_inliers, int* n_ransac_inliers) {
    (void)k1;
    (void)k2;
    memset(res, 0, sizeof(*res));
    // F1 = last frame with pose I and fresh VO landmarks (tracking.cpp:146-190)
    std::vector<uint8_t> has_lm(n1), out1(n1, 0);
    std::vector<int32_t> obs1(n1, 0);
    const float mThDepth = c->mbf * c->th_depth / c->fx;
    res->n_queries = oracle_vo_landmarks(xyz1, n1, mThDepth, has_lm.data());
    std::vector<int32_t> lm_obs2(n2, -1), lm_src2(n2, -1);
    std::vector<uint8_t> out2(n2, 0);
    std::vector<odo_dmatch> m(std::max(n1, 1));
    int nm = oracle_knn_match(d1, n1, d2, n2, ratio, has_lm.data(), out1.data(), obs1.data(),
                              lm_obs2.data(), lm_src2.data(), out2.data(), m.data(), n1);
    res->n_matches = nm;
    for (int i = 0; i < std::min(nm, cap); i++) matches[i] = m[i];
    float I[16];
    for (int i = 0; i < 16; i++) I[i] = (i % 5 == 0) ? 1.f : 0.f;
    memcpy(res->T12, I, sizeof(I));
    memcpy(res->Tcw, I, sizeof(I));
    res->rmse = 1e6f;
    for (int i = 0; i < n2; i++) inlier_mask[i] = 0;
    if (n_ransac_inliers) *n_ransac_inliers = 0;
    if (nm < 20) return nm;  // TrackFrame: nmatches < 20 -> return (tracking.cpp:201)
    odo_rng rng;
    oracle_rng_seed(&rng, seed);
    std::vector<odo_dmatch> inl(nm);
    int ninl = 0, visited = 0, ngood = 0;
    res->ransac_ok = oracle_ransac(m.data(), nm, xyz1, xyz2, rp, &rng, latch, res->T12, &res->rmse,
                                   inl.data(), &ninl, &visited, &ngood);
    res->n_inliers = ninl;
    // Ransac::mvInliers (ransac.cpp:240 / 258): read by DrawMatches
    // (tracking.cpp:205) and copied into F2's flags in RANSAC mode
    // (odometry.cpp:75-76)
    if (ransac_inliers && n_ransac_inliers) {
        const int nc = std::min(ninl, cap);
        for (int i = 0; i < nc; i++) ransac_inliers[i] = inl[i];
        *n_ransac_inliers = nc;
    }
    res->visited = visited;
    res->n_good = ngood;
    res->n_sweeps = g_last_sweeps;
    res->n_fit_points = g_last_fit_points;
    // Odometry::Compute ADAPTIVE_RBA: Tcw2 = T12 * Tcw1 (= T12), then PnP on F2
    std::vector<float> Xw, ob;
    std::vector<int> eidx;
    for (int i = 0; i < n2; i++) {
        if (lm_src2[i] < 0) continue;
        const int s = lm_src2[i];
        Xw.insert(Xw.end(), {xyz1[3 * s], xyz1[3 * s + 1], xyz1[3 * s + 2]});
        ob.insert(ob.end(), {kun2[2 * i], kun2[2 * i + 1], ur2[i]});
        eidx.push_back(i);
    }
    std::vector<uint8_t> eout(eidx.size(), 0);
    res->pnp_inliers = pnp_compute(Xw.data(), ob.data(), (int)eidx.size(), *c, res->T12, res->Tcw,
                                   eout.data());
    // PnPSolver sets every landmark slot inlier at edge creation (pnpsolver.cpp:63,98),
    // so with < 3 edges they stay inlier and the pose stays T12.
    for (size_t k = 0; k < eidx.size(); k++) inlier_mask[eidx[k]] = eout[k] ? 0 : 1;
    return nm;
}

}  // extern "C"
