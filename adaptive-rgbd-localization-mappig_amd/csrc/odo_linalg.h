// Small dense linear algebra shared by the pose back-ends (k_pnpransac.hip,
// k_gicp.hip): a one-sided Jacobi SVD in double whose sizes are template
// parameters, so 3x3 / 6xN systems stay in registers. Rotation order, the
// convergence test and the descending sort match oracle/pnpransac_ref.cpp's
// svdj (and gicp_ref.cpp's svd3_v).
#pragma once

#include <hip/hip_runtime.h>

#include <cfloat>

namespace odo {

// ------------------------------------------- one-sided Jacobi SVD (double)
// A (M x N, M >= N, row-major) = U diag(w) V^T, w descending (first maximum
// first); U M x N, V N x N by columns. Sizes are template parameters so the
// small systems (3x3, 6xN) live in registers.
template <int M, int N>
__device__ inline void svdj(const double* A, double* w, double* U, double* V) {
    double a[M * N], v[N * N];
#pragma unroll
    for (int i = 0; i < M * N; i++) a[i] = A[i];
#pragma unroll
    for (int i = 0; i < N; i++)
#pragma unroll
        for (int j = 0; j < N; j++) v[i * N + j] = i == j ? 1.0 : 0.0;
    for (int sweep = 0; sweep < 60; sweep++) {
        int changed = 0;
#pragma unroll
        for (int p = 0; p < N - 1; p++)
#pragma unroll
            for (int q = p + 1; q < N; q++) {
                double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
                for (int i = 0; i < M; i++) {
                    const double ap = a[i * N + p], aq = a[i * N + q];
                    alpha += ap * ap;
                    beta += aq * aq;
                    gamma += ap * aq;
                }
                if (gamma == 0.0 || fabs(gamma) <= DBL_EPSILON * sqrt(alpha * beta)) continue;
                changed = 1;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
                for (int i = 0; i < M; i++) {
                    const double ap = a[i * N + p], aq = a[i * N + q];
                    a[i * N + p] = c * ap - s * aq;
                    a[i * N + q] = s * ap + c * aq;
                }
#pragma unroll
                for (int i = 0; i < N; i++) {
                    const double vp = v[i * N + p], vq = v[i * N + q];
                    v[i * N + p] = c * vp - s * vq;
                    v[i * N + q] = s * vp + c * vq;
                }
            }
        if (!changed) break;
    }
    double ww[N];
    int ord[N];
#pragma unroll
    for (int j = 0; j < N; j++) {
        double s = 0;
#pragma unroll
        for (int i = 0; i < M; i++) s += a[i * N + j] * a[i * N + j];
        ww[j] = sqrt(s);
        ord[j] = j;
    }
    // selection sort (descending, first maximum wins) on the values, ord follows
#pragma unroll
    for (int j = 0; j < N; j++) {
        int b = j;
        double wb = ww[j];
#pragma unroll
        for (int k = j + 1; k < N; k++)
            if (ww[k] > wb) {
                b = k;
                wb = ww[k];
            }
#pragma unroll
        for (int k = j + 1; k < N; k++)
            if (k == b) {
                const double tw = ww[j];
                ww[j] = ww[k];
                ww[k] = tw;
                const int to = ord[j];
                ord[j] = ord[k];
                ord[k] = to;
            }
    }
#pragma unroll
    for (int j = 0; j < N; j++) {
        w[j] = ww[j];
        const double inv = ww[j] > 0 ? 1.0 / ww[j] : 0.0;
#pragma unroll
        for (int c = 0; c < N; c++)
            if (ord[j] == c) {
                if (U)
#pragma unroll
                    for (int i = 0; i < M; i++) U[i * N + j] = a[i * N + c] * inv;
#pragma unroll
                for (int i = 0; i < N; i++) V[i * N + j] = v[i * N + c];
            }
    }
}

}  // namespace odo
