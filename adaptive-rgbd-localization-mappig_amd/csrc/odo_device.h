// Device-side scalar math for the MI355X odometry kernels (gfx950).
//
// Every routine here restates a third-party or reference computation with a
// FIXED operation order so that float/double
// results are bit-identical to the CPU oracle; the library is compiled with
// -ffp-contract=off so no FMA contraction reorders rounding.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define ODO_INLINE __device__ __forceinline__

// s_setprio level of the latency-bound pair kernels (pair match, RANSAC) so
// their waves issue ahead of co-resident extraction waves. Round 6: 1 (3
// until round 5, when the pair chain was longer than the extraction step;
// with the 512-thread pyramid it fits inside the step with slack, and at 1
// the extraction kernels issue more: +0.3-0.9 % on the default workload and
// +1.1 % on the hard one, profiles/r06_f, r06_g, r06_h)
#ifndef ODO_WAVE_PRIO
#define ODO_WAVE_PRIO 1
#endif

namespace odo {

// ----------------------------------------------------------------- rounding
ODO_INLINE int cv_round(float v) { return __float2int_rn(v); }  // cvRound: half to even
ODO_INLINE int cv_floor(float v) { int i = (int)v; return i - (i > v); }

// --------------------------------------------------------- fastAtan2 (A.5)
ODO_INLINE float fast_atan2(float y, float x) {
    const float k = (float)(180.0 / 3.14159265358979323846);
    const float p1 = 0.9997878412794807f * k;
    const float p3 = -0.3258083974640975f * k;
    const float p5 = 0.1555786518463281f * k;
    const float p7 = -0.04432655554792128f * k;
    const float eps = (float)2.220446049250313080847e-16;
    float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + eps);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + eps);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// ---------------------------------------------- Eigen JacobiSVD<3x3f> (A.8)
struct Rot {
    float c, s;
};

ODO_INLINE float sum3f(float a, float b, float c) { return a + (b + c); }
ODO_INLINE double sum3d(double a, double b, double c) { return a + (b + c); }

ODO_INLINE void rot_rows(float W[3][3], int p, int q, Rot j) {
    if (j.c == 1.f && j.s == 0.f) return;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float xi = W[p][i], yi = W[q][i];
        W[p][i] = j.c * xi + j.s * yi;
        W[q][i] = -j.s * xi + j.c * yi;
    }
}
ODO_INLINE void rot_cols(float W[3][3], int p, int q, Rot j) {
    Rot t{j.c, -j.s};
    if (t.c == 1.f && t.s == 0.f) return;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float xi = W[i][p], yi = W[i][q];
        W[i][p] = t.c * xi + t.s * yi;
        W[i][q] = -t.s * xi + t.c * yi;
    }
}
ODO_INLINE Rot make_jacobi(float x, float y, float z) {
    float deno = 2.f * fabsf(y);
    if (deno < 1.17549435082228750797e-38f) return Rot{1.f, 0.f};
    float tau = (x - z) / deno;
    float w = sqrtf(tau * tau + 1.f);
    float t = tau > 0.f ? 1.f / (tau + w) : 1.f / (tau - w);
    float sign_t = t > 0.f ? 1.f : -1.f;
    float n = 1.f / sqrtf(t * t + 1.f);
    Rot r;
    r.s = ((-sign_t) * (y / fabsf(y))) * fabsf(t) * n;
    r.c = n;
    return r;
}
ODO_INLINE void real_2x2_jacobi_svd(const float W[3][3], int p, int q, Rot* jl, Rot* jr) {
    float m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
    Rot rot1;
    float t = m00 + m11;
    float d = m10 - m01;
    if (fabsf(d) < 1.17549435082228750797e-38f) {
        rot1.s = 0.f;
        rot1.c = 1.f;
    } else {
        float u = t / d;
        float tmp = sqrtf(1.f + u * u);
        rot1.s = 1.f / tmp;
        rot1.c = u / tmp;
    }
    if (!(rot1.c == 1.f && rot1.s == 0.f)) {
        float x0 = m00, y0 = m10;
        m00 = rot1.c * x0 + rot1.s * y0;
        m10 = -rot1.s * x0 + rot1.c * y0;
        float x1 = m01, y1 = m11;
        m01 = rot1.c * x1 + rot1.s * y1;
        m11 = -rot1.s * x1 + rot1.c * y1;
    }
    *jr = make_jacobi(m00, m01, m11);
    float c2 = jr->c, s2 = -jr->s;
    jl->c = rot1.c * c2 - rot1.s * s2;
    jl->s = rot1.c * s2 + rot1.s * c2;
}

ODO_INLINE void svd3(const float A[3][3], float U[3][3], float S[3], float V[3][3]) {
    const float precision = 2.f * 1.1920928955078125e-07f;
    const float considerAsZero = 1.17549435082228750797e-38f;
    float scale = 0.f;
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) scale = fmaxf(scale, fabsf(A[i][j]));
    if (scale == 0.f) scale = 1.f;
    float W[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
            W[i][j] = A[i][j] / scale;
            U[i][j] = (i == j) ? 1.f : 0.f;
            V[i][j] = (i == j) ? 1.f : 0.f;
        }
    float maxDiag = fmaxf(fabsf(W[0][0]), fmaxf(fabsf(W[1][1]), fabsf(W[2][2])));
    bool finished = false;
    int sweeps = 0;
    while (!finished && sweeps < 100) {
        finished = true;
        sweeps++;
        for (int p = 1; p < 3; ++p)
            for (int q = 0; q < p; ++q) {
                float threshold = fmaxf(considerAsZero, precision * maxDiag);
                if (fabsf(W[p][q]) > threshold || fabsf(W[q][p]) > threshold) {
                    finished = false;
                    Rot jl, jr;
                    real_2x2_jacobi_svd(W, p, q, &jl, &jr);
                    rot_rows(W, p, q, jl);
                    rot_cols(U, p, q, Rot{jl.c, -jl.s});
                    rot_cols(W, p, q, jr);
                    rot_cols(V, p, q, jr);
                    maxDiag = fmaxf(maxDiag, fmaxf(fabsf(W[p][p]), fabsf(W[q][q])));
                }
            }
    }
#pragma unroll
    for (int i = 0; i < 3; i++) {
        float a = W[i][i];
        S[i] = fabsf(a);
        if (a < 0.f)
#pragma unroll
            for (int r = 0; r < 3; r++) U[r][i] = -U[r][i];
    }
#pragma unroll
    for (int i = 0; i < 3; i++) S[i] *= scale;
    for (int i = 0; i < 3; i++) {
        int pos = i;
        float mx = S[i];
        for (int k = i + 1; k < 3; k++)
            if (S[k] > mx) {
                mx = S[k];
                pos = k;
            }
        if (mx == 0.f) break;
        if (pos != i) {
            float t = S[i];
            S[i] = S[pos];
            S[pos] = t;
            for (int r = 0; r < 3; r++) {
                float a = U[r][i];
                U[r][i] = U[r][pos];
                U[r][pos] = a;
                float b = V[r][i];
                V[r][i] = V[r][pos];
                V[r][pos] = b;
            }
        }
    }
}

ODO_INLINE float det3(const float M[3][3]) {
    float h012 = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]);
    float h102 = M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]);
    float h201 = M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
    return h012 - h102 + h201;
}

// ------------------------------------------------ PCL TFC (A.7) accumulator
// w / aw of the TFC recurrence: LLVM's f32 division sequence without its
// v_div_scale / v_div_fixup (rcp, one Newton step, two Markstein corrections,
// the last as a plain fma where v_div_fmas adds no scale). They are inactive,
// so the quotient is the same bits, when the numerator lies in [2^-20, 2^20]
// and the denominator in [2^-20, 2^40] (no operand scaling below an exponent
// difference of 96, a normal quotient in (0, 1]): every weight a pair's TFC
// adds in that range (k_ransac_prep's guard, RState.efast), a sum of at most
// 2^20 of them (k_ransac_lanes' fast-form launch, LN_TFAST)
template <bool FAST>
ODO_INLINE float tfc_div(float a, float b) {
    if (!FAST) return a / b;
    float y = __builtin_amdgcn_rcpf(b);
    const float e = __builtin_fmaf(-b, y, 1.0f);
    y = __builtin_fmaf(e, y, y);
    float q = a * y;
    float r = __builtin_fmaf(-b, q, a);
    q = __builtin_fmaf(r, y, q);
    r = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(r, y, q);
}
struct TFC {
    float accW;
    float m1[3], m2[3];
    float cov[3][3];
    ODO_INLINE void reset() {
        accW = 0.f;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            m1[i] = m2[i] = 0.f;
#pragma unroll
            for (int j = 0; j < 3; j++) cov[i][j] = 0.f;
        }
    }
    template <bool FD = false>
    ODO_INLINE void add(float px, float py, float pz, float qx, float qy, float qz, float w) {
        if (w == 0.0f) return;
        accW += w;
        float alpha = tfc_div<FD>(w, accW);
        float d1[3] = {px - m1[0], py - m1[1], pz - m1[2]};
        float d2[3] = {qx - m2[0], qy - m2[1], qz - m2[2]};
        const float oma = 1.0f - alpha;
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const float ad2 = alpha * d2[i];
#pragma unroll
            for (int j = 0; j < 3; j++) cov[i][j] = oma * (cov[i][j] + ad2 * d1[j]);
        }
#pragma unroll
        for (int i = 0; i < 3; i++) {
            m1[i] += alpha * d1[i];
            m2[i] += alpha * d2[i];
        }
    }
    // add() when `in`, else nothing, as straight-line code (selects): the
    // same operations on the same values for an added point, so a caller can
    // unroll over points and let the next points' divisions overlap this one's
    // updates
    template <bool FD = false>
    ODO_INLINE void add_sel(float px, float py, float pz, float qx, float qy, float qz, float w, bool in) {
        const bool u = in & (w != 0.0f);
        const float aw = accW + w;
        const float alpha = tfc_div<FD>(w, aw);
        const float d1[3] = {px - m1[0], py - m1[1], pz - m1[2]};
        const float d2[3] = {qx - m2[0], qy - m2[1], qz - m2[2]};
        const float oma = 1.0f - alpha;
        if (FD) {
            // guarded launch (finite coordinates): a point the lane does not
            // add updates with alpha = 0, 1 - alpha = 1, which leaves every
            // accumulator's bits as they are — x + (+-0) = x, as none of them
            // is ever -0 (they start at +0, and a sum is -0 only when both
            // terms are) — so 2 selects replace the 15 below
            const float al = u ? alpha : 0.0f, om = u ? oma : 1.0f;
#pragma unroll
            for (int i = 0; i < 3; i++) {
                const float ad2 = al * d2[i];
#pragma unroll
                for (int j = 0; j < 3; j++) cov[i][j] = om * (cov[i][j] + ad2 * d1[j]);
            }
#pragma unroll
            for (int i = 0; i < 3; i++) {
                m1[i] = m1[i] + al * d1[i];
                m2[i] = m2[i] + al * d2[i];
            }
            accW = u ? aw : accW;
            return;
        }
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const float ad2 = alpha * d2[i];
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const float nc = oma * (cov[i][j] + ad2 * d1[j]);
                cov[i][j] = u ? nc : cov[i][j];
            }
        }
#pragma unroll
        for (int i = 0; i < 3; i++) {
            const float n1 = m1[i] + alpha * d1[i], n2 = m2[i] + alpha * d2[i];
            m1[i] = u ? n1 : m1[i];
            m2[i] = u ? n2 : m2[i];
        }
        accW = u ? aw : accW;
    }
    // getTransformation(): row-major 3x4 [R|t]
    ODO_INLINE void get(float T[12]) const {
        float U[3][3], S[3], V[3][3];
        svd3(cov, U, S, V);
        float s22 = (det3(U) * det3(V) < 0.0f) ? -1.0f : 1.0f;
        float US[3][3];
#pragma unroll
        for (int i = 0; i < 3; i++) {
            // (U*S)(i,j) = U(i,0)S(0,j) + (U(i,1)S(1,j) + U(i,2)S(2,j)), S diagonal
            US[i][0] = sum3f(U[i][0] * 1.f, U[i][1] * 0.f, U[i][2] * 0.f);
            US[i][1] = sum3f(U[i][0] * 0.f, U[i][1] * 1.f, U[i][2] * 0.f);
            US[i][2] = sum3f(U[i][0] * 0.f, U[i][1] * 0.f, U[i][2] * s22);
        }
        float R[3][3];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) R[i][j] = sum3f(US[i][0] * V[j][0], US[i][1] * V[j][1], US[i][2] * V[j][2]);
#pragma unroll
        for (int i = 0; i < 3; i++) {
            float t = m2[i] - sum3f(R[i][0] * m1[0], R[i][1] * m1[1], R[i][2] * m1[2]);
            T[i * 4 + 0] = R[i][0];
            T[i * 4 + 1] = R[i][1];
            T[i * 4 + 2] = R[i][2];
            T[i * 4 + 3] = t;
        }
    }
};

// ---------------------------------- Ransac::ErrorFunction2 (ransac.cpp:350)
// Returns DBL_MAX for rejected points (shortcut / NaN / non-PD), like the reference.
struct MahalConst {
    double raster_cov_x, raster_cov_y;
    double depth_cov;  // latched DepthCovariance value
};

#define ODO_DBL_MAX 1.7976931348623157e308

ODO_INLINE double error_function2(const float x1[3], const float x2[3], const double T[12], const MahalConst& K) {
    if (__builtin_isnan(x1[2]) || __builtin_isnan(x2[2])) return ODO_DBL_MAX;
    const double a0 = x1[0], a1 = x1[1], a2 = x1[2];
    const double mu0 = x2[0], mu1 = x2[1], mu2 = x2[2];
    double m0 = ((T[0] * a0 + T[1] * a1) + T[2] * a2) + T[3] * 1.0;
    double m1 = ((T[4] * a0 + T[5] * a1) + T[6] * a2) + T[7] * 1.0;
    double m2 = ((T[8] * a0 + T[9] * a1) + T[10] * a2) + T[11] * 1.0;
    double d0 = m0 - mu0, d1 = m1 - mu1, d2 = m2 - mu2;
    {
        double dsq = sum3d(d0 * d0, d1 * d1, d2 * d2);
        double s1 = fmax(K.raster_cov_x, K.depth_cov);
        double s2 = fmax(K.raster_cov_x, K.depth_cov);
        if (dsq > 2.0 * (s1 + s2)) return ODO_DBL_MAX;
    }
    const double R00 = T[0], R01 = T[1], R02 = T[2];
    const double R10 = T[4], R11 = T[5], R12 = T[6];
    const double R20 = T[8], R21 = T[9], R22 = T[10];
    const double c00 = K.raster_cov_x * a2, c11 = K.raster_cov_y * a2, c22 = K.depth_cov;
    // Eigen's RtC[i][j] = R[0][i]*C[0][j] + (R[1][i]*C[1][j] + R[2][i]*C[2][j])
    // with C diagonal is R[j][i]*C[j][j] plus two exact zeros. Adding them
    // changes at most the sign of an exact-zero RtC entry, and every A below
    // adds +0.0 or a positive covariance after the products, so A (and the
    // result) is bit-identical; for a non-finite R the point is rejected either
    // way (its delta is not finite). 9 products instead of 27 + 18 adds.
    const double R[3][3] = {{R00, R01, R02}, {R10, R11, R12}, {R20, R21, R22}};
    const double Cd[3] = {c00, c11, c22};
    double RtC[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) RtC[i][j] = R[j][i] * Cd[j];
    // lower triangle of C1 = RtC * R, plus cov2 (diagonal)
    const double cov2_0 = K.raster_cov_x * mu2, cov2_1 = K.raster_cov_y * mu2, cov2_2 = K.depth_cov;
    double A00 = sum3d(RtC[0][0] * R00, RtC[0][1] * R10, RtC[0][2] * R20) + cov2_0;
    double A10 = sum3d(RtC[1][0] * R00, RtC[1][1] * R10, RtC[1][2] * R20) + 0.0;
    double A11 = sum3d(RtC[1][0] * R01, RtC[1][1] * R11, RtC[1][2] * R21) + cov2_1;
    double A20 = sum3d(RtC[2][0] * R00, RtC[2][1] * R10, RtC[2][2] * R20) + 0.0;
    double A21 = sum3d(RtC[2][0] * R01, RtC[2][1] * R11, RtC[2][2] * R21) + 0.0;
    double A22 = sum3d(RtC[2][0] * R02, RtC[2][1] * R12, RtC[2][2] * R22) + cov2_2;
    if (__builtin_isnan(d2)) return ODO_DBL_MAX;
    // Eigen LLT<Matrix3d> (lower, unblocked); solve() ignores info()
    double L00 = A00, L10 = A10, L20 = A20, L11 = A11, L21 = A21, L22 = A22;
    {
        double x = L00;
        if (x > 0) {
            L00 = x = sqrt(x);
            L10 /= x;
            L20 /= x;
            x = L11 - L10 * L10;
            if (x > 0) {
                L11 = x = sqrt(x);
                L21 -= L20 * L10;
                L21 /= x;
                x = L22 - (L20 * L20 + L21 * L21);
                if (x > 0) L22 = sqrt(x);
            }
        }
    }
    double y0 = d0 / L00;
    double y1 = (d1 - L10 * y0) / L11;
    double y2 = (d2 - (L20 * y0 + L21 * y1)) / L22;
    double z2 = y2 / L22;
    double z1 = (y1 - L21 * z2) / L11;
    double z0 = (y0 - (L10 * z1 + L20 * z2)) / L00;
    double r = sum3d(d0 * z0, d1 * z1, d2 * z2);
    if (!(r >= 0.0)) return ODO_DBL_MAX;
    return r;
}

// a / b from y = RN(1 / b) (an IEEE division) by one Markstein correction:
// q = RN(a y), r = a - b q (exact with the fused multiply-add), RN(q + r y).
// Markstein's theorem makes that the correctly rounded quotient when q is
// within 1 ulp of a / b; RN(a y) can be up to ~1.5 ulp off (a's significand
// near 2), outside the theorem, so the equality with a / b rests on
// tests/test_markstein.py: the same operation sequence on the host over
// random and adversarial operands, no counterexample in 2 x 10^8 cases.
// Three operations instead of the ten of the IEEE division sequence (the
// IEEE form stays selectable: -DLN_MARKSTEIN=0 -DEV_MARKSTEIN=0). Zero /
// non-finite denominators give NaN where the division gives +-inf: the
// callers below reject the point either way.
ODO_INLINE double div_mk(double a, double b, double y) {
    const double q = a * y;
    const double r = __builtin_fma(-b, q, a);
    return __builtin_fma(r, y, q);
}
// ErrorFunction2 with the nine divisions of the LLT solve done as three
// reciprocals (L00, L11, L22) and Markstein-corrected quotients. Same value
// as error_function2 for every point it accepts as an inlier candidate (a
// finite non-negative result from normal quotients); points with a zero or
// non-finite pivot end rejected in both (DBL_MAX or a non-finite r).
// The point-independent terms of ErrorFunction2's A (the depth column of
// RtC = R^T C times R, C[2][2] = depth_cov): Z = {A00, A10, A11, A20, A21,
// A22}'s third products, (R[2][i] * c22) * R[2][j], the same operations as
// the per-point form, done once per hypothesis.
ODO_INLINE void hyp_cov_terms(const double T[12], const MahalConst& K, double Z[6]) {
    const double c22 = K.depth_cov;
    Z[0] = (T[8] * c22) * T[8];
    Z[1] = (T[9] * c22) * T[8];
    Z[2] = (T[9] * c22) * T[9];
    Z[3] = (T[10] * c22) * T[8];
    Z[4] = (T[10] * c22) * T[9];
    Z[5] = (T[10] * c22) * T[10];
}
#ifndef EF_FAST
// ErrorFunction2's three square roots and three reciprocals (error_function2_mk)
// as the cores of LLVM's correctly rounded AMDGPU f64 sequences without their
// range fix-ups, which are inactive on the ranges below (ef_sqrt / ef_rcp).
// 1: every evaluation in the fast form, redone with the IEEE sequences when an
// operand falls outside them (bit-identical; costs k_ransac_lanes registers:
// 187 VGPRs, which break its co-residency with k_pnp). 2 (default):
// k_ransac_lanes picks the fast form once per launch when every open pair
// passed k_ransac_prep's range guard (below), else the IEEE form;
// k_ransac_eval / _eval_list pick it per pair (EV_EFAST; a wave holds one
// pair, so the branch is uniform). Round 6, hard workload, 3 alternations each:
// 53.1k vs 51.4k frames/s (profiles/r06_ef2); 46 parity tests green on it.
#define EF_FAST 2
#endif
// sqrt: v_rsq_f64, then the Goldschmidt iteration and two corrections of
// LLVM's lowering (its ldexp scaling only acts below 2^-767, its class test
// only at 0 and +inf)
template <bool FAST>
ODO_INLINE double ef_sqrt(double x, bool& ok) {
    if (!FAST) return sqrt(x);
    ok = ok & (x >= 0x1p-767) & (x <= ODO_DBL_MAX);
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y, h = y * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
// 1 / b: v_rcp_f64 and the Newton steps of LLVM's f64 division with the
// numerator 1.0 (v_div_scale leaves 1.0 and b unscaled, v_div_fmas is a plain
// fma and v_div_fixup returns its input for 2^-500 <= |b| <= 2^500)
template <bool FAST>
ODO_INLINE double ef_rcp(double b, bool& ok) {
    if (!FAST) return 1.0 / b;
    const double ab = __builtin_fabs(b);
    ok = ok & (ab >= 0x1p-500) & (ab <= 0x1p500);
    double y = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-b, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-b, y, 1.0);
    return __builtin_fma(e, y, y);
}
template <bool FAST>
ODO_INLINE double error_function2_mk_t(const float x1[3], const float x2[3], const double T[12], const MahalConst& K,
                                       const double* Z, bool& ok) {
    if (__builtin_isnan(x1[2]) || __builtin_isnan(x2[2])) return ODO_DBL_MAX;
    const double a0 = x1[0], a1 = x1[1], a2 = x1[2];
    const double mu0 = x2[0], mu1 = x2[1], mu2 = x2[2];
    double m0 = ((T[0] * a0 + T[1] * a1) + T[2] * a2) + T[3] * 1.0;
    double m1 = ((T[4] * a0 + T[5] * a1) + T[6] * a2) + T[7] * 1.0;
    double m2 = ((T[8] * a0 + T[9] * a1) + T[10] * a2) + T[11] * 1.0;
    double d0 = m0 - mu0, d1 = m1 - mu1, d2 = m2 - mu2;
    {
        double dsq = sum3d(d0 * d0, d1 * d1, d2 * d2);
        double s1 = fmax(K.raster_cov_x, K.depth_cov);
        double s2 = fmax(K.raster_cov_x, K.depth_cov);
        if (dsq > 2.0 * (s1 + s2)) return ODO_DBL_MAX;
    }
    const double R00 = T[0], R01 = T[1], R02 = T[2];
    const double R10 = T[4], R11 = T[5], R12 = T[6];
    const double R20 = T[8], R21 = T[9], R22 = T[10];
    const double c00 = K.raster_cov_x * a2, c11 = K.raster_cov_y * a2, c22 = K.depth_cov;
    const double R[3][3] = {{R00, R01, R02}, {R10, R11, R12}, {R20, R21, R22}};
    const double Cd[3] = {c00, c11, c22};
    double RtC[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) RtC[i][j] = R[j][i] * Cd[j];
    const double cov2_0 = K.raster_cov_x * mu2, cov2_1 = K.raster_cov_y * mu2, cov2_2 = K.depth_cov;
    // the third products from Z when the caller has them (hyp_cov_terms)
    const double z00 = Z ? Z[0] : RtC[0][2] * R20, z10 = Z ? Z[1] : RtC[1][2] * R20, z11 = Z ? Z[2] : RtC[1][2] * R21;
    const double z20 = Z ? Z[3] : RtC[2][2] * R20, z21 = Z ? Z[4] : RtC[2][2] * R21, z22 = Z ? Z[5] : RtC[2][2] * R22;
    double A00 = sum3d(RtC[0][0] * R00, RtC[0][1] * R10, z00) + cov2_0;
    double A10 = sum3d(RtC[1][0] * R00, RtC[1][1] * R10, z10) + 0.0;
    double A11 = sum3d(RtC[1][0] * R01, RtC[1][1] * R11, z11) + cov2_1;
    double A20 = sum3d(RtC[2][0] * R00, RtC[2][1] * R10, z20) + 0.0;
    double A21 = sum3d(RtC[2][0] * R01, RtC[2][1] * R11, z21) + 0.0;
    double A22 = sum3d(RtC[2][0] * R02, RtC[2][1] * R12, z22) + cov2_2;
    if (__builtin_isnan(d2)) return ODO_DBL_MAX;
    double L00 = A00, L10 = A10, L20 = A20, L11 = A11, L21 = A21, L22 = A22;
    double i00, i11, i22;
    {
        double x = L00;
        if (x > 0) {
            L00 = x = ef_sqrt<FAST>(x, ok);
            i00 = ef_rcp<FAST>(x, ok);
            L10 = div_mk(L10, x, i00);
            L20 = div_mk(L20, x, i00);
            x = L11 - L10 * L10;
            if (x > 0) {
                L11 = x = ef_sqrt<FAST>(x, ok);
                i11 = ef_rcp<FAST>(x, ok);
                L21 -= L20 * L10;
                L21 = div_mk(L21, x, i11);
                x = L22 - (L20 * L20 + L21 * L21);
                if (x > 0) L22 = ef_sqrt<FAST>(x, ok);
            } else {
                i11 = ef_rcp<FAST>(L11, ok);
            }
        } else {
            i00 = ef_rcp<FAST>(L00, ok);
            i11 = ef_rcp<FAST>(L11, ok);
        }
    }
    i22 = ef_rcp<FAST>(L22, ok);
    double y0 = div_mk(d0, L00, i00);
    double y1 = div_mk(d1 - L10 * y0, L11, i11);
    double y2 = div_mk(d2 - (L20 * y0 + L21 * y1), L22, i22);
    double z2 = div_mk(y2, L22, i22);
    double z1 = div_mk(y1 - L21 * z2, L11, i11);
    double z0 = div_mk(y0 - (L10 * z1 + L20 * z2), L00, i00);
    double r = sum3d(d0 * z0, d1 * z1, d2 * z2);
    if (!(r >= 0.0)) return ODO_DBL_MAX;
    return r;
}

// EF_FAST == 2 (k_ransac_lanes, k_ransac_eval*): the fast form without the per-call
// check, for pairs whose evaluated points all have depths in [2^-20, 2^20]
// (ef_fast_pt, checked once per pair by k_ransac_prep: RState.efast) under a
// DepthCovariance latch in [2^-200, 2^200] (ef_fast_cov). There every operand
// lies in the ranges above whenever the result can be accepted: with C2 =
// diag(rcx mu2, rcy mu2, dcov) positive, A00 >= rcx mu2 > 2^-40, a positive
// Schur complement of entries >= 2^-200 is at least one of their ulps (above
// 2^-260), T comes from the float fit (|T| < 2^128, so A < 2^300), and a
// NaN / infinite delta rejects the point before its value is read.
ODO_INLINE bool ef_fast_pt(float sz, float tx, float sz2, float tz) {
    // points ComputeInliersAndError skips (origin.z == 0 || target.x == 0,
    // ransac.cpp:326) or rejects first (NaN depth) do not count
    if (sz == 0.0f || tx == 0.0f || __builtin_isnan(sz2) || __builtin_isnan(tz)) return true;
    return sz2 >= 0x1p-20f && sz2 <= 0x1p20f && tz >= 0x1p-20f && tz <= 0x1p20f;
}
ODO_INLINE bool ef_fast_cov(const MahalConst& K) {
    return K.depth_cov >= 0x1p-200 && K.depth_cov <= 0x1p200 && K.raster_cov_x > 0x1p-40 &&
           K.raster_cov_y > 0x1p-40 && K.raster_cov_x < 1.0 && K.raster_cov_y < 1.0;
}
ODO_INLINE double error_function2_mk(const float x1[3], const float x2[3], const double T[12], const MahalConst& K,
                                     const double* Z = nullptr, bool fast = false) {
    bool ok = true;
    if (EF_FAST == 2) return fast ? error_function2_mk_t<true>(x1, x2, T, K, Z, ok)
                                  : error_function2_mk_t<false>(x1, x2, T, K, Z, ok);
    double r = error_function2_mk_t<EF_FAST != 0>(x1, x2, T, K, Z, ok);
    if (EF_FAST == 1 && __builtin_expect(!ok, 0)) r = error_function2_mk_t<false>(x1, x2, T, K, Z, ok);
    return r;
}

// The shortcut of error_function2 (ransac.cpp:350-365): true when the point
// is rejected before the covariance solve (NaN depth, the squared residual
// beyond 2 (s1 + s2), NaN residual). The same expressions as the start of
// error_function2_bf, which tests them again: a pre-filter, never a second
// opinion.
ODO_INLINE bool error_function2_shortcut(const float x1[3], const float x2[3], const double T[12],
                                         const MahalConst& K) {
    const double a0 = x1[0], a1 = x1[1], a2 = x1[2];
    const double mu0 = x2[0], mu1 = x2[1], mu2 = x2[2];
    const double m0 = ((T[0] * a0 + T[1] * a1) + T[2] * a2) + T[3] * 1.0;
    const double m1 = ((T[4] * a0 + T[5] * a1) + T[6] * a2) + T[7] * 1.0;
    const double m2 = ((T[8] * a0 + T[9] * a1) + T[10] * a2) + T[11] * 1.0;
    const double d0 = m0 - mu0, d1 = m1 - mu1, d2 = m2 - mu2;
    const double dsq = sum3d(d0 * d0, d1 * d1, d2 * d2);
    const double s1 = fmax(K.raster_cov_x, K.depth_cov), s2 = fmax(K.raster_cov_x, K.depth_cov);
    return __builtin_isnan(x1[2]) | __builtin_isnan(x2[2]) | (dsq > 2.0 * (s1 + s2)) | __builtin_isnan(d2);
}

// error_function2_mk as straight-line code: every branch becomes a select
// between the values both sides compute, so the scheduler can interleave two
// evaluations (the pivots' square roots, reciprocals and quotients are one
// long dependency chain; a wave running one evaluation at a time waits on
// it). Same value as error_function2_mk for every point: each select takes
// what the branch error_function2_mk follows computes, from the same
// operations on the same operands; the values it drops are never read.
ODO_INLINE double error_function2_bf(const float x1[3], const float x2[3], const double T[12], const MahalConst& K) {
    const double a0 = x1[0], a1 = x1[1], a2 = x1[2];
    const double mu0 = x2[0], mu1 = x2[1], mu2 = x2[2];
    const double m0 = ((T[0] * a0 + T[1] * a1) + T[2] * a2) + T[3] * 1.0;
    const double m1 = ((T[4] * a0 + T[5] * a1) + T[6] * a2) + T[7] * 1.0;
    const double m2 = ((T[8] * a0 + T[9] * a1) + T[10] * a2) + T[11] * 1.0;
    const double d0 = m0 - mu0, d1 = m1 - mu1, d2 = m2 - mu2;
    const double dsq = sum3d(d0 * d0, d1 * d1, d2 * d2);
    const double s1 = fmax(K.raster_cov_x, K.depth_cov), s2 = fmax(K.raster_cov_x, K.depth_cov);
    // (non-short-circuit ors: no branch for the compiler to sink work into)
    bool rej = __builtin_isnan(x1[2]) | __builtin_isnan(x2[2]) | (dsq > 2.0 * (s1 + s2)) | __builtin_isnan(d2);
    const double R00 = T[0], R01 = T[1], R02 = T[2];
    const double R10 = T[4], R11 = T[5], R12 = T[6];
    const double R20 = T[8], R21 = T[9], R22 = T[10];
    const double c00 = K.raster_cov_x * a2, c11 = K.raster_cov_y * a2, c22 = K.depth_cov;
    const double R[3][3] = {{R00, R01, R02}, {R10, R11, R12}, {R20, R21, R22}};
    const double Cd[3] = {c00, c11, c22};
    double RtC[3][3];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
        for (int j = 0; j < 3; j++) RtC[i][j] = R[j][i] * Cd[j];
    const double cov2_0 = K.raster_cov_x * mu2, cov2_1 = K.raster_cov_y * mu2, cov2_2 = K.depth_cov;
    const double A00 = sum3d(RtC[0][0] * R00, RtC[0][1] * R10, RtC[0][2] * R20) + cov2_0;
    const double A10 = sum3d(RtC[1][0] * R00, RtC[1][1] * R10, RtC[1][2] * R20) + 0.0;
    const double A11 = sum3d(RtC[1][0] * R01, RtC[1][1] * R11, RtC[1][2] * R21) + cov2_1;
    const double A20 = sum3d(RtC[2][0] * R00, RtC[2][1] * R10, RtC[2][2] * R20) + 0.0;
    const double A21 = sum3d(RtC[2][0] * R01, RtC[2][1] * R11, RtC[2][2] * R21) + 0.0;
    const double A22 = sum3d(RtC[2][0] * R02, RtC[2][1] * R12, RtC[2][2] * R22) + cov2_2;
    // the LLT's three nested pivot tests (p0, p1, p2): a failed test leaves
    // the rest of the factor as A, and the reciprocals are of whatever pivot stands
    const bool p0 = A00 > 0;
    const double L00 = p0 ? sqrt(A00) : A00;
    const double i00 = 1.0 / L00;
    const double L10 = p0 ? div_mk(A10, L00, i00) : A10;
    const double L20 = p0 ? div_mk(A20, L00, i00) : A20;
    const double x11 = A11 - L10 * L10;
    const bool p1 = p0 & (x11 > 0);
    const double L11 = p1 ? sqrt(x11) : A11;
    const double i11 = 1.0 / L11;
    const double L21 = p1 ? div_mk(A21 - L20 * L10, L11, i11) : A21;
    const double x22 = A22 - (L20 * L20 + L21 * L21);
    const bool p2 = p1 & (x22 > 0);
    const double L22 = p2 ? sqrt(x22) : A22;
    const double i22 = 1.0 / L22;
    const double y0 = div_mk(d0, L00, i00);
    const double y1 = div_mk(d1 - L10 * y0, L11, i11);
    const double y2 = div_mk(d2 - (L20 * y0 + L21 * y1), L22, i22);
    const double z2 = div_mk(y2, L22, i22);
    const double z1 = div_mk(y1 - L21 * z2, L11, i11);
    const double z0 = div_mk(y0 - (L10 * z1 + L20 * z2), L00, i00);
    const double r = sum3d(d0 * z0, d1 * z1, d2 * z2);
    rej = rej | !(r >= 0.0);
    return rej ? ODO_DBL_MAX : r;
}

// error_function2_bf twice, written in lockstep (each statement for both)
// so the two dependency chains issue interleaved: e[k] ==
// error_function2_bf(x1[k], x2[k], T[k], K). The callers pass one point under
// two transforms (k_ransac_lanes) or two points under one transform
// (k_ransac_eval); the shared terms fold together.
#define EF2(stmt) _Pragma("unroll") for (int k = 0; k < 2; k++) { stmt; }
ODO_INLINE void error_function2_bf2(const float x1[2][3], const float x2[2][3], const double T[2][12],
                                    const MahalConst& K, double e[2]) {
    const double s1 = fmax(K.raster_cov_x, K.depth_cov), s2 = fmax(K.raster_cov_x, K.depth_cov);
    double a0[2], a1[2], a2[2], mu2[2], c00[2], c11[2], cov2_0[2], cov2_1[2];
    const double c22 = K.depth_cov, cov2_2 = K.depth_cov;
    EF2(a0[k] = x1[k][0]; a1[k] = x1[k][1]; a2[k] = x1[k][2]; mu2[k] = x2[k][2])
    EF2(c00[k] = K.raster_cov_x * a2[k]; c11[k] = K.raster_cov_y * a2[k])
    EF2(cov2_0[k] = K.raster_cov_x * mu2[k]; cov2_1[k] = K.raster_cov_y * mu2[k])
    double d0[2], d1[2], d2[2];
    bool rej[2];
    EF2(d0[k] = (((T[k][0] * a0[k] + T[k][1] * a1[k]) + T[k][2] * a2[k]) + T[k][3] * 1.0) - (double)x2[k][0])
    EF2(d1[k] = (((T[k][4] * a0[k] + T[k][5] * a1[k]) + T[k][6] * a2[k]) + T[k][7] * 1.0) - (double)x2[k][1])
    EF2(d2[k] = (((T[k][8] * a0[k] + T[k][9] * a1[k]) + T[k][10] * a2[k]) + T[k][11] * 1.0) - mu2[k])
    EF2(rej[k] = __builtin_isnan(x1[k][2]) | __builtin_isnan(x2[k][2]) |
                 (sum3d(d0[k] * d0[k], d1[k] * d1[k], d2[k] * d2[k]) > 2.0 * (s1 + s2)) | __builtin_isnan(d2[k]))
    // RtC[i][j] = R[j][i] * Cd[j]; A's lower triangle (error_function2_bf)
    double A00[2], A10[2], A11[2], A20[2], A21[2], A22[2];
    EF2(A00[k] = sum3d((T[k][0] * c00[k]) * T[k][0], (T[k][4] * c11[k]) * T[k][4], (T[k][8] * c22) * T[k][8]) +
                 cov2_0[k])
    EF2(A10[k] = sum3d((T[k][1] * c00[k]) * T[k][0], (T[k][5] * c11[k]) * T[k][4], (T[k][9] * c22) * T[k][8]) + 0.0)
    EF2(A11[k] = sum3d((T[k][1] * c00[k]) * T[k][1], (T[k][5] * c11[k]) * T[k][5], (T[k][9] * c22) * T[k][9]) +
                 cov2_1[k])
    EF2(A20[k] = sum3d((T[k][2] * c00[k]) * T[k][0], (T[k][6] * c11[k]) * T[k][4], (T[k][10] * c22) * T[k][8]) + 0.0)
    EF2(A21[k] = sum3d((T[k][2] * c00[k]) * T[k][1], (T[k][6] * c11[k]) * T[k][5], (T[k][10] * c22) * T[k][9]) + 0.0)
    EF2(A22[k] = sum3d((T[k][2] * c00[k]) * T[k][2], (T[k][6] * c11[k]) * T[k][6], (T[k][10] * c22) * T[k][10]) +
                 cov2_2)
    bool p0[2], p1[2], p2[2];
    double L00[2], i00[2], L10[2], L20[2], x11[2], L11[2], i11[2], L21[2], x22[2], L22[2], i22[2];
    EF2(p0[k] = A00[k] > 0)
    EF2(L00[k] = p0[k] ? sqrt(A00[k]) : A00[k])
    EF2(i00[k] = 1.0 / L00[k])
    EF2(L10[k] = p0[k] ? div_mk(A10[k], L00[k], i00[k]) : A10[k])
    EF2(L20[k] = p0[k] ? div_mk(A20[k], L00[k], i00[k]) : A20[k])
    EF2(x11[k] = A11[k] - L10[k] * L10[k])
    EF2(p1[k] = p0[k] & (x11[k] > 0))
    EF2(L11[k] = p1[k] ? sqrt(x11[k]) : A11[k])
    EF2(i11[k] = 1.0 / L11[k])
    EF2(L21[k] = p1[k] ? div_mk(A21[k] - L20[k] * L10[k], L11[k], i11[k]) : A21[k])
    EF2(x22[k] = A22[k] - (L20[k] * L20[k] + L21[k] * L21[k]))
    EF2(p2[k] = p1[k] & (x22[k] > 0))
    EF2(L22[k] = p2[k] ? sqrt(x22[k]) : A22[k])
    EF2(i22[k] = 1.0 / L22[k])
    double y0[2], y1[2], y2[2], z0[2], z1[2], z2[2];
    EF2(y0[k] = div_mk(d0[k], L00[k], i00[k]))
    EF2(y1[k] = div_mk(d1[k] - L10[k] * y0[k], L11[k], i11[k]))
    EF2(y2[k] = div_mk(d2[k] - (L20[k] * y0[k] + L21[k] * y1[k]), L22[k], i22[k]))
    EF2(z2[k] = div_mk(y2[k], L22[k], i22[k]))
    EF2(z1[k] = div_mk(y1[k] - L21[k] * z2[k], L11[k], i11[k]))
    EF2(z0[k] = div_mk(y0[k] - (L10[k] * z1[k] + L20[k] * z2[k]), L00[k], i00[k]))
    EF2(const double r = sum3d(d0[k] * z0[k], d1[k] * z1[k], d2[k] * z2[k]);
        e[k] = (rej[k] | !(r >= 0.0)) ? ODO_DBL_MAX : r)
}
#undef EF2

// ---------------------------------------- glibc TYPE_3 random_r (A.12)
struct Rng {
    int32_t s[31];
    int f, r;
    ODO_INLINE void seed(uint32_t seedv) {
        // __srandom_r: word is int32_t, Schrage's method, 310 discards
        if (seedv == 0) seedv = 1;
        s[0] = (int32_t)seedv;
        int32_t word = (int32_t)seedv;
        for (int i = 1; i < 31; ++i) {
            long hi = word / 127773;
            long lo = word % 127773;
            long w2 = 16807 * lo - 2836 * hi;
            if (w2 < 0) w2 += 2147483647;
            word = (int32_t)w2;
            s[i] = word;
        }
        f = 3;
        r = 0;
        for (int k = 0; k < 310; k++) next();
    }
    ODO_INLINE int32_t next() {
        uint32_t val = (uint32_t)s[f] + (uint32_t)s[r];
        s[f] = (int32_t)val;
        int32_t out = (int32_t)(val >> 1);
        ++f;
        if (f >= 31) {
            f = 0;
            ++r;
        } else {
            ++r;
            if (r >= 31) r = 0;
        }
        return out;
    }
};

// Per-pair seed of the batched contract: splitmix64(seed ^ pair index), low
// 32 bits (SURVEY.md §8d "Seeds").
ODO_INLINE __host__ uint32_t pair_seed(uint64_t base, uint64_t pair) {
    uint64_t z = (base ^ pair) + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    return (uint32_t)z;
}

}  // namespace odo
