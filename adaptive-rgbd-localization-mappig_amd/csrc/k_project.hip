// Tracking::SearchLocalLMs for gfx950 (System/tracking.cpp:368-405): the
// local-map landmarks' Frame::isInFrustum (Core/frame.cpp:100-133) and
// Matcher(0.8f)::ProjectionMatch (Features/matcher.cpp:90-145) with
// GetFeaturesInArea's window (frame.cpp:258-274). SURVEY.md §8(f) rank 1.
//
//   k_proj_cands    one thread per landmark: the folded gemm Rcw*P + tcw
//                   (double accumulation, one rounding), projection, bounds,
//                   then the frame keypoints inside the +-th window in index
//                   order (the frame's undistorted points staged in LDS), each
//                   packed with its Hamming distance and octave
//   k_proj_resolve  the reference visits landmarks in order and a landmark's
//                   candidates skip slots already holding a landmark with
//                   observations - including slots earlier landmarks of this
//                   call took - so the stable best / second-best and the
//                   same-level ratio test run in landmark order on lane 0,
//                   over candidate lists prefetched into LDS 256 landmarks at
//                   a time; lists longer than PJ_CAP rescan the frame exactly
#include "odo_device.h"
#include "odo_internal.h"

namespace odo {

#define PJ_CAP 16  // candidates kept per landmark (more: exact rescan on the resolver)

struct PjCalib {
    float fx, fy, cx, cy, mbf;
    float minX, maxX, minY, maxY;
};

ODO_INLINE int hamming32d(const uint32_t* a, const uint8_t* b8) {
    const uint4* b = reinterpret_cast<const uint4*>(b8);
    const uint4 x = b[0], y = b[1];
    return __popc(a[0] ^ x.x) + __popc(a[1] ^ x.y) + __popc(a[2] ^ x.z) + __popc(a[3] ^ x.w) + __popc(a[4] ^ y.x) +
           __popc(a[5] ^ y.y) + __popc(a[6] ^ y.z) + __popc(a[7] ^ y.w);
}

// candidate = idx (13 bits) | octave (5 bits) << 13 | distance (9 bits) << 18
ODO_INLINE uint32_t pj_pack(int idx, int oct, int d) {
    return (uint32_t)idx | ((uint32_t)(oct & 31) << 13) | ((uint32_t)d << 18);
}

__global__ void __launch_bounds__(256) k_proj_cands(const float* __restrict__ Tcw, const odo_landmark* __restrict__ lms,
                                                    int nL, const float* __restrict__ kun,
                                                    const int32_t* __restrict__ octave,
                                                    const uint8_t* __restrict__ desc, int n, PjCalib C, float th,
                                                    float* __restrict__ proj, uint8_t* __restrict__ inview,
                                                    int* __restrict__ ccount, uint32_t* __restrict__ cand) {
    extern __shared__ float2 s_kun[];
    for (int j = threadIdx.x; j < n; j += blockDim.x) s_kun[j] = make_float2(kun[2 * j], kun[2 * j + 1]);
    __syncthreads();
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nL) return;
    const odo_landmark L = lms[i];
    const float nan = __builtin_nanf("");
    float u = nan, v = nan, ur = nan;
    bool in = false;
    if (!(L.flags & (ODO_LM_BAD | ODO_LM_SEEN))) {
        float Pc[3];
#pragma unroll
        for (int k = 0; k < 3; k++)
            Pc[k] = (float)((((double)Tcw[4 * k] * L.X[0] + (double)Tcw[4 * k + 1] * L.X[1]) +
                             (double)Tcw[4 * k + 2] * L.X[2]) + (double)Tcw[4 * k + 3]);
        if (!(Pc[2] < 0.0f)) {
            const float invz = 1.0f / Pc[2];
            const float uu = C.fx * Pc[0] * invz + C.cx;
            const float vv = C.fy * Pc[1] * invz + C.cy;
            if (!(uu < C.minX || uu > C.maxX) && !(vv < C.minY || vv > C.maxY)) {
                in = true;
                u = uu;
                v = vv;
                ur = uu - C.mbf * invz;
            }
        }
    }
    proj[3 * i] = u;
    proj[3 * i + 1] = v;
    proj[3 * i + 2] = ur;
    inview[i] = in ? 1 : 0;
    int c = 0;
    if (in) {
        uint32_t ld[8];
#pragma unroll
        for (int k = 0; k < 8; k++) ld[k] = reinterpret_cast<const uint32_t*>(L.desc)[k];
        uint32_t* out = cand + (size_t)i * PJ_CAP;
        for (int j = 0; j < n; j++) {
            const float2 q = s_kun[j];
            const float dx = q.x - u, dy = q.y - v;
            if (fabsf(dx) < th && fabsf(dy) < th) {
                if (c < PJ_CAP) out[c] = pj_pack(j, octave[j], hamming32d(ld, desc + 32 * (size_t)j));
                c++;
            }
        }
    }
    ccount[i] = c;
}

#define PJ_CHUNK 256
__global__ void __launch_bounds__(256) k_proj_resolve(const odo_landmark* __restrict__ lms, int nL,
                                                      const float* __restrict__ proj,
                                                      const uint8_t* __restrict__ inview,
                                                      const int* __restrict__ ccount, const uint32_t* __restrict__ cand,
                                                      const float* __restrict__ kun,
                                                      const int32_t* __restrict__ octave,
                                                      const uint8_t* __restrict__ desc, int n,
                                                      const uint8_t* __restrict__ slot_taken, float th, float nnratio,
                                                      int32_t* __restrict__ slot_lm, int* __restrict__ nmatches) {
    extern __shared__ uint8_t s_dyn[];
    uint8_t* taken = s_dyn;                                          // n
    int32_t* sl = reinterpret_cast<int32_t*>(s_dyn + ((n + 15) & ~15));  // n
    __shared__ uint32_t s_c[PJ_CHUNK][PJ_CAP];
    __shared__ int s_n[PJ_CHUNK];
    __shared__ int s_fl[PJ_CHUNK];
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
        taken[j] = slot_taken[j];
        sl[j] = -1;
    }
    int nm = 0;
    const double TH_HIGH = 100.0;  // Matcher::Matcher, NORM_HAMMING (matcher.cpp:15-17)
    for (int i0 = 0; i0 < nL; i0 += PJ_CHUNK) {
        __syncthreads();
        {
            const int i = i0 + threadIdx.x;
            int cnt = 0, fl = 0;
            if (i < nL) {
                fl = inview[i] ? lms[i].flags : -1;
                cnt = fl >= 0 ? ccount[i] : 0;
                const int m = cnt < PJ_CAP ? cnt : PJ_CAP;
                for (int k = 0; k < m; k++) s_c[threadIdx.x][k] = cand[(size_t)i * PJ_CAP + k];
            }
            s_n[threadIdx.x] = cnt;
            s_fl[threadIdx.x] = i < nL ? fl : -1;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const int m = min(PJ_CHUNK, nL - i0);
            for (int q = 0; q < m; q++) {
                const int fl = s_fl[q];
                if (fl < 0 || (fl & ODO_LM_BAD) || s_n[q] == 0) continue;  // !mbTrackInView, isBad, empty area
                const int i = i0 + q;
                double best1 = 1.7976931348623157e308, best2 = best1;
                int lvl1 = -1, lvl2 = -1, bidx = -1;
                auto visit = [&](int j, int oct, int d) {
                    if (taken[j]) return;
                    const double dd = (double)d;
                    if (dd < best1) {
                        best2 = best1;
                        best1 = dd;
                        lvl2 = lvl1;
                        lvl1 = oct;
                        bidx = j;
                    } else if (dd < best2) {
                        lvl2 = oct;
                        best2 = dd;
                    }
                };
                if (s_n[q] <= PJ_CAP) {
                    for (int k = 0; k < s_n[q]; k++) {
                        const uint32_t e = s_c[q][k];
                        visit((int)(e & 0x1fff), (int)((e >> 13) & 31), (int)(e >> 18));
                    }
                } else {
                    // more than PJ_CAP keypoints in the window: the exact scan
                    const float x = proj[3 * i], y = proj[3 * i + 1];
                    uint32_t ld[8];
                    for (int k = 0; k < 8; k++) ld[k] = reinterpret_cast<const uint32_t*>(lms[i].desc)[k];
                    for (int j = 0; j < n; j++) {
                        const float dx = kun[2 * j] - x, dy = kun[2 * j + 1] - y;
                        if (fabsf(dx) < th && fabsf(dy) < th) visit(j, octave[j], hamming32d(ld, desc + 32 * (size_t)j));
                    }
                }
                if (best1 <= TH_HIGH) {
                    if (lvl1 == lvl2 && best1 > (double)nnratio * best2) continue;
                    sl[bidx] = i;  // Frame::AddLandmark
                    taken[bidx] = (fl & ODO_LM_HAS_OBS) ? 1 : 0;
                    nm++;
                }
            }
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += blockDim.x) slot_lm[j] = sl[j];
    if (threadIdx.x == 0) *nmatches = nm;
}

int launch_projection_match(hipStream_t st, const float* Tcw, const odo_landmark* lms, int nL, const float* kun,
                            const int32_t* octave, const uint8_t* desc, int n, const uint8_t* slot_taken,
                            const float* calib5, const float* bounds, float th, float nnratio, float* proj,
                            uint8_t* inview, int* ccount, uint32_t* cand, int32_t* slot_lm, int* nmatches) {
    if (n > 8191) return -1;  // 13-bit candidate index
    PjCalib C{calib5[0], calib5[1], calib5[2], calib5[3], calib5[4], bounds[0], bounds[1], bounds[2], bounds[3]};
    const size_t lds1 = (size_t)n * sizeof(float2);
    const size_t lds2 = (size_t)((n + 15) & ~15) + (size_t)n * 4;
    if (lds1 > 64 * 1024)
        (void)hipFuncSetAttribute((const void*)k_proj_cands, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds1);
    if (lds2 > 40 * 1024)
        (void)hipFuncSetAttribute((const void*)k_proj_resolve, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds2);
    if (nL > 0)
        hipLaunchKernelGGL(k_proj_cands, dim3((nL + 255) / 256), dim3(256), lds1, st, Tcw, lms, nL, kun, octave, desc,
                           n, C, th, proj, inview, ccount, cand);
    hipLaunchKernelGGL(k_proj_resolve, dim3(1), dim3(256), lds2, st, lms, nL, proj, inview, ccount, cand, kun, octave,
                       desc, n, slot_taken, th, nnratio, slot_lm, nmatches);
    return 0;
}

size_t projection_cand_cap() { return PJ_CAP; }

}  // namespace odo
