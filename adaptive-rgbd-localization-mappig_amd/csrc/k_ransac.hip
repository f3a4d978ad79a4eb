// Ransac::Iterate(Frame*,Frame*,m12) for gfx950 (Odometry/ransac.cpp:155-267).
//
// One workgroup per frame pair. Visited iterations are evaluated
// speculatively, one per lane, RB at a time: lane v draws the v-th sample of
// the pair's glibc rand() stream (SampleMatches, ransac.cpp:269-293), then runs
// the refinement loop exactly as the reference does for that iteration — PCL
// TFC fit over the current inlier set in sorted-good order, Mahalanobis sweep
// over all good matches with the sequential double meanError sum (the sweep
// order is the reference's, so every lane reproduces it bit for bit).
// Thread 0 then replays the ordered running-best fold with its skip (n+=10)
// and break rules (ransac.cpp:233-249); if the fold needs more iterations than
// were evaluated, the next RB are evaluated from the advanced RNG state.
// Inlier sets are bitmasks over the sorted good matches, [word][lane] layout.
#include "odo_device.h"
#include "odo_internal.h"

namespace odo {

struct SortElR {
    uint32_t key;
    uint32_t val;
};

struct GoodPt {
    float sx, sy, sz, tx, ty, tz, w, pad;
};

#define RB 256
#define MAX_SAMPLE 8

__global__ void __launch_bounds__(RB) k_ransac(const SortElR* __restrict__ good, const int* __restrict__ n_good,
                                               const int* __restrict__ n_matches, const odo_dmatch* __restrict__ matches,
                                               const float* __restrict__ xyz, int kp_cap, int slot0, int match_cap,
                                               RansacCfg cfg, const double* __restrict__ latch,
                                               uint64_t seed_base, uint64_t pair_base, const int* __restrict__ pair_valid,
                                               int min_matches, odo_rng* __restrict__ rng_io,
                                               GoodPt* __restrict__ gpts, uint32_t* __restrict__ masks,
                                               uint32_t* __restrict__ best_mask, int mask_words_cap,
                                               odo_pair_result* __restrict__ res, float* __restrict__ T12_out) {
    const int p = blockIdx.x;
    const int t = threadIdx.x;
    __shared__ int s_samp[RB * MAX_SAMPLE];
    __shared__ int s_ns[RB];
    __shared__ double s_err[RB];
    __shared__ int s_cnt[RB];
    __shared__ float s_T[RB][12];
    __shared__ int s_mbuf[RB];
    __shared__ Rng s_rng;
    __shared__ int s_done, s_n, s_valid, s_visited, s_best_v, s_best_cnt, s_copy, s_copy_v, s_copy_buf;
    __shared__ float s_rmse;
    __shared__ float s_bestT[12];

    odo_pair_result* R = res + p;
    float* T12o = T12_out + (size_t)p * 16;
    const int ng = n_good[p];
    const int nm = n_matches[p];
    if (t == 0) {
        R->rmse = 1e6f;
        R->n_good = 0;
        R->n_inliers = 0;
        R->ransac_ok = 0;
        R->visited = 0;
        for (int i = 0; i < 16; i++) R->T12[i] = T12o[i] = (i % 5 == 0) ? 1.f : 0.f;
    }
    if (!pair_valid[p]) return;
    if (nm < min_matches) return;  // TrackFrame: nmatches < 20 -> no Odometry::Compute (tracking.cpp:201)
    if (nm < cfg.min_inlier_th) return;
    if (t == 0) R->n_good = ng;
    if (ng < cfg.min_inlier_th) return;

    const SortElR* G = good + (size_t)p * match_cap;
    const odo_dmatch* M = matches + (size_t)p * match_cap;
    const float* X1 = xyz + (size_t)(slot0 + p) * kp_cap * 3;
    const float* X2 = xyz + (size_t)(slot0 + p + 1) * kp_cap * 3;
    GoodPt* P = gpts + (size_t)p * match_cap;
    for (int k = t; k < ng; k += RB) {
        const odo_dmatch m = M[G[k].val];
        GoodPt g;
        g.sx = X1[3 * m.queryIdx];
        g.sy = X1[3 * m.queryIdx + 1];
        g.sz = X1[3 * m.queryIdx + 2];
        g.tx = X2[3 * m.trainIdx];
        g.ty = X2[3 * m.trainIdx + 1];
        g.tz = X2[3 * m.trainIdx + 2];
        g.w = 1.0f / (g.sz * g.tz);
        g.pad = 0.f;
        P[k] = g;
    }
    const int words = (ng + 31) >> 5;
    uint32_t* MK = masks + (size_t)p * 2 * mask_words_cap * RB;  // [buf][word][lane]
    uint32_t* BM = best_mask + (size_t)p * mask_words_cap;
    MahalConst K;
    K.raster_cov_x = cfg.raster_cov_x;
    K.raster_cov_y = cfg.raster_cov_y;
    K.depth_cov = *latch;
    const float th = cfg.max_mahal * cfg.max_mahal;
    const int H = cfg.iterations;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    const int S = cfg.sample_size < MAX_SAMPLE ? cfg.sample_size : MAX_SAMPLE;
    if (t == 0) {
        if (rng_io) {
            for (int i = 0; i < 31; i++) s_rng.s[i] = rng_io->state[i];
            s_rng.f = rng_io->fpos;
            s_rng.r = rng_io->rpos;
        } else {
            s_rng.seed(pair_seed(seed_base, pair_base + (uint64_t)p));
        }
        s_done = (H <= 0 || ng < S) ? 1 : 0;
        s_n = 0;
        s_valid = 0;
        s_visited = 0;
        s_best_v = -1;
        s_best_cnt = 0;
        s_rmse = 1e6f;
        for (int i = 0; i < 12; i++) s_bestT[i] = (i % 5 == 0) ? 1.f : 0.f;
    }
    __syncthreads();

    int round = 0;
    while (!s_done) {
        // ---- samples for visited iterations [round*RB, round*RB+RB)
        if (t == 0) {
            for (int v = 0; v < RB; v++) {
                int cnt = 0;
                int ids[MAX_SAMPLE];
                int safety = 0;
                while (cnt < S) {
                    int id1 = (int)((uint32_t)s_rng.next() % (uint32_t)ng);
                    int id2 = (int)((uint32_t)s_rng.next() % (uint32_t)ng);
                    if (id1 > id2) id1 = id2;
                    bool dup = false;
                    for (int q = 0; q < cnt; q++) dup |= ids[q] == id1;
                    if (!dup) {
                        int pos = cnt;  // keep ascending (std::set order)
                        while (pos > 0 && ids[pos - 1] > id1) {
                            ids[pos] = ids[pos - 1];
                            pos--;
                        }
                        ids[pos] = id1;
                        cnt++;
                    }
                    if (++safety > 10000) break;
                }
                s_ns[v] = cnt;
                for (int q = 0; q < cnt; q++) s_samp[v * MAX_SAMPLE + q] = ids[q];
            }
        }
        __syncthreads();
        // ---- one refinement loop per lane (ransac.cpp:201-231)
        {
            double refinedError = 1e6;
            unsigned refinedCnt = 0;
            float refinedT[12];
            for (int i = 0; i < 12; i++) refinedT[i] = (i % 5 == 0) ? 1.f : 0.f;
            int cur = -1;  // mask buffer holding the current inlier set (-1: sample)
            int nb = 0;    // buffer the next sweep writes
            for (int refinements = 1; refinements < 20; refinements++) {
                TFC tfc;
                tfc.reset();
                if (cur < 0) {
                    for (int q = 0; q < s_ns[t]; q++) {
                        const GoodPt g = P[s_samp[t * MAX_SAMPLE + q]];
                        if (__builtin_isnan(g.sz) || __builtin_isnan(g.tz)) continue;
                        tfc.add(g.sx, g.sy, g.sz, g.tx, g.ty, g.tz, g.w);
                    }
                } else {
                    const uint32_t* mk = MK + (size_t)cur * mask_words_cap * RB;
                    for (int w = 0; w < words; w++) {
                        uint32_t bits = mk[(size_t)w * RB + t];
                        while (bits) {
                            const int b = __builtin_ctz(bits);
                            bits &= bits - 1;
                            const GoodPt g = P[w * 32 + b];
                            if (__builtin_isnan(g.sz) || __builtin_isnan(g.tz)) continue;
                            tfc.add(g.sx, g.sy, g.sz, g.tx, g.ty, g.tz, g.w);
                        }
                    }
                }
                float T[12];
                tfc.get(T);
                double Td[12];
                for (int i = 0; i < 12; i++) Td[i] = (double)T[i];
                // ComputeInliersAndError (ransac.cpp:315-348)
                double meanError = 0.0;
                unsigned cnt = 0;
                uint32_t* mo = MK + (size_t)nb * mask_words_cap * RB;
                for (int w = 0; w < words; w++) {
                    uint32_t bits = 0;
                    const int kend = min(32, ng - w * 32);
                    for (int b = 0; b < kend; b++) {
                        const GoodPt g = P[w * 32 + b];
                        if (g.sz == 0.0f || g.tx == 0.0f) continue;
                        const float x1[3] = {g.sx, g.sy, g.sz}, x2[3] = {g.tx, g.ty, g.tz};
                        const double d = error_function2(x1, x2, Td, K);
                        if (d > th) continue;
                        if (!(d >= 0.0)) continue;
                        meanError += d;
                        cnt++;
                        bits |= 1u << b;
                    }
                    mo[(size_t)w * RB + t] = bits;
                }
                if (cnt < 3) meanError = 1e9;
                else {
                    meanError /= (double)cnt;
                    meanError = sqrt(meanError);
                }
                if (cnt < minInl || meanError > (double)cfg.max_mahal) break;
                if (cnt >= refinedCnt && meanError <= refinedError) {
                    const unsigned prev = refinedCnt;
                    for (int i = 0; i < 12; i++) refinedT[i] = T[i];
                    refinedError = meanError;
                    refinedCnt = cnt;
                    cur = nb;
                    nb ^= 1;
                    if (cnt == prev) break;
                } else break;
            }
            s_err[t] = refinedError;
            s_cnt[t] = (int)refinedCnt;
            s_mbuf[t] = cur;
            for (int i = 0; i < 12; i++) s_T[t][i] = refinedT[i];
        }
        __syncthreads();
        // ---- ordered fold over visited iterations (ransac.cpp:233-249)
        if (t == 0) {
            s_copy = 0;
            int n = s_n;
            int v = 0;
            for (; v < RB && n < H; v++) {
                s_visited++;
                const unsigned rc = (unsigned)s_cnt[v];
                const double re = s_err[v];
                bool brk = false;
                if (rc > 0) {
                    s_valid++;
                    if (re <= (double)s_rmse && rc >= (unsigned)s_best_cnt && rc >= minInl) {
                        s_rmse = (float)re;
                        s_best_cnt = (int)rc;
                        s_best_v = round * RB + v;
                        for (int i = 0; i < 12; i++) s_bestT[i] = s_T[v][i];
                        s_copy = 1;
                        s_copy_v = v;
                        s_copy_buf = s_mbuf[v];
                        if (rc > ng * 0.5) n += 10;
                        if (rc > ng * 0.75) n += 10;
                        if (rc > ng * 0.8) brk = true;
                    }
                }
                n++;
                if (brk) {
                    n = H;  // loop exits
                    s_done = 1;
                    break;
                }
            }
            s_n = n;
            if (n >= H) s_done = 1;
        }
        __syncthreads();
        if (s_copy) {
            const uint32_t* src = MK + (size_t)s_copy_buf * mask_words_cap * RB;
            for (int w = t; w < words; w += RB) BM[w] = src[(size_t)w * RB + s_copy_v];
        }
        __syncthreads();
        round++;
    }
    // ---- identity fallback when no iteration was valid (ransac.cpp:252-264)
    if (s_valid == 0) {
        // one lane evaluates T = I
        if (t == 0) {
            double Td[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
            double meanError = 0.0;
            unsigned cnt = 0;
            for (int w = 0; w < words; w++) {
                uint32_t bits = 0;
                const int kend = min(32, ng - w * 32);
                for (int b = 0; b < kend; b++) {
                    const GoodPt g = P[w * 32 + b];
                    if (g.sz == 0.0f || g.tx == 0.0f) continue;
                    const float x1[3] = {g.sx, g.sy, g.sz}, x2[3] = {g.tx, g.ty, g.tz};
                    const double d = error_function2(x1, x2, Td, K);
                    if (d > th) continue;
                    if (!(d >= 0.0)) continue;
                    meanError += d;
                    cnt++;
                    bits |= 1u << b;
                }
                BM[w] = bits;
            }
            if (cnt < 3) meanError = 1e9;
            else {
                meanError /= (double)cnt;
                meanError = sqrt(meanError);
            }
            if (cnt > minInl && meanError < (double)cfg.max_mahal) {
                s_best_cnt = (int)cnt;
                s_rmse = (float)((double)s_rmse + meanError);
                for (int i = 0; i < 12; i++) s_bestT[i] = (i % 5 == 0) ? 1.f : 0.f;
            } else {
                s_best_cnt = 0;
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        R->rmse = s_rmse;
        R->n_inliers = s_best_cnt;
        R->ransac_ok = (unsigned)s_best_cnt >= minInl ? 1 : 0;
        R->visited = s_visited;
        for (int i = 0; i < 12; i++) R->T12[i] = T12o[i] = s_bestT[i];
        R->T12[12] = R->T12[13] = R->T12[14] = 0.f;
        R->T12[15] = 1.f;
        T12o[12] = T12o[13] = T12o[14] = 0.f;
        T12o[15] = 1.f;
    }
    if (s_best_cnt == 0)
        for (int w = t; w < words; w += RB) BM[w] = 0;
    // in/out rand() stream: advance the caller's state by exactly the samples
    // of the visited iterations (speculative draws are not consumed)
    if (rng_io && t == 0) {
        Rng r;
        for (int i = 0; i < 31; i++) r.s[i] = rng_io->state[i];
        r.f = rng_io->fpos;
        r.r = rng_io->rpos;
        for (int v = 0; v < s_visited; v++) {
            int cnt = 0, ids[MAX_SAMPLE], safety = 0;
            while (cnt < S) {
                int id1 = (int)((uint32_t)r.next() % (uint32_t)ng);
                int id2 = (int)((uint32_t)r.next() % (uint32_t)ng);
                if (id1 > id2) id1 = id2;
                bool dup = false;
                for (int q = 0; q < cnt; q++) dup |= ids[q] == id1;
                if (!dup) ids[cnt++] = id1;
                if (++safety > 10000) break;
            }
        }
        for (int i = 0; i < 31; i++) rng_io->state[i] = r.s[i];
        rng_io->fpos = r.f;
        rng_io->rpos = r.r;
    }
}

}  // namespace odo

namespace odo {
size_t ransac_gpt_bytes() { return sizeof(GoodPt); }
void launch_ransac(hipStream_t st, const void* good, const int* n_good, const int* n_matches, const odo_dmatch* matches,
                   const float* xyz, int kp_cap, int slot0, int match_cap, RansacCfg cfg, const double* latch,
                   uint64_t seed_base, uint64_t pair_base, const int* pair_valid, int min_matches, odo_rng* rng_io,
                   void* gpts, uint32_t* masks, uint32_t* best_mask, int mask_words_cap, odo_pair_result* res,
                   float* T12, int npairs) {
    hipLaunchKernelGGL(k_ransac, dim3(npairs), dim3(RB), 0, st, (const SortElR*)good, n_good, n_matches, matches, xyz,
                       kp_cap, slot0, match_cap, cfg, latch, seed_base, pair_base, pair_valid, min_matches, rng_io,
                       (GoodPt*)gpts, masks, best_mask, mask_words_cap, res, T12);
}
}  // namespace odo
