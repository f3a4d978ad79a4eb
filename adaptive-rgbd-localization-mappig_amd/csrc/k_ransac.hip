// Ransac::Iterate(Frame*,Frame*,m12) for gfx950 (Odometry/ransac.cpp:155-267).
//
// Visited iterations ("hypotheses") are evaluated speculatively in rounds of
// growing size (16, 48, 448, 512, ... — most pairs stop after the first, see
// ransac.cpp:246-247). One wave evaluates one hypothesis: the 64 lanes split
// the Mahalanobis sweep over the sorted good matches (ErrorFunction2, double),
// ballots build the ordered inlier bitmask, and lane 0 folds the meanError sum
// sequentially in match order and runs the PCL TFC recurrence over the inlier
// set (both order-dependent, so they stay serial and bit-identical to the
// reference). Hypothesis v uses the v-th SampleMatches draw of the pair's
// glibc rand() stream. Between rounds a one-wave scan replays the reference's
// ordered running-best fold with its n+=10 skips and >80% break, keeps the
// winner's mask and draws the next round's samples.
//
//   k_ransac_prep   per pair: early-outs, GoodPt table, RNG seed, round-0 samples
//   k_ransac_eval   per (pair, hypothesis): refinement loop (ransac.cpp:204-231)
//   k_ransac_scan   per pair: ordered fold (ransac.cpp:233-249), next samples
//   k_ransac_final  per pair: identity fallback (ransac.cpp:252-264), outputs
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

#define MAX_SAMPLE 8
#define RS_BMAX 512

struct RState {
    int32_t rng_s[31];
    int32_t rng_f, rng_r;
    int32_t rng0_s[31];  // stream position at entry (for the in/out API)
    int32_t rng0_f, rng0_r;
    int active, done, n, visited, valid, best_cnt, ng, S, round_base, round_count, words, pad;
    float rmse;
    float bestT[12];
};

struct HypRes {
    double err;
    int cnt;
    int pad;
    float T[12];
};

struct RansacBufs {
    const SortElR* good;
    const int* n_good;
    const int* n_matches;
    const odo_dmatch* matches;
    const float* xyz;
    int kp_cap, slot0, match_cap;
    const double* latch;
    uint64_t seed_base, pair_base;
    const int* pair_valid;
    int min_matches;
    odo_rng* rng_io;
    GoodPt* gpts;
    RState* st;
    HypRes* hyp;      // [pair][RS_BMAX]
    int* samples;     // [pair][RS_BMAX][MAX_SAMPLE+1] (count first)
    uint32_t* masks;  // [pair][RS_BMAX][mask_words]
    uint32_t* best_mask;
    int mask_words;
    odo_pair_result* res;
    float* T12;
};

// SampleMatches (ransac.cpp:269-293) for `count` consecutive visited
// iterations, state in LDS (dynamic indexing), one lane.
ODO_INLINE void draw_samples(Rng& r, int ng, int S, int count, int* out) {
    for (int v = 0; v < count; v++) {
        int cnt = 0;
        int ids[MAX_SAMPLE];
        int safety = 0;
        while (cnt < S) {
            int id1 = (int)((uint32_t)r.next() % (uint32_t)ng);
            int id2 = (int)((uint32_t)r.next() % (uint32_t)ng);
            if (id1 > id2) id1 = id2;
            bool dup = false;
            for (int q = 0; q < cnt; q++) dup |= ids[q] == id1;
            if (!dup) {
                int pos = cnt;  // std::set keeps them ascending
                while (pos > 0 && ids[pos - 1] > id1) {
                    ids[pos] = ids[pos - 1];
                    pos--;
                }
                ids[pos] = id1;
                cnt++;
            }
            if (++safety > 10000) break;
        }
        int* o = out + v * (MAX_SAMPLE + 1);
        o[0] = cnt;
        for (int q = 0; q < cnt; q++) o[1 + q] = ids[q];
    }
}

ODO_INLINE void rng_load(Rng& r, const int32_t* s, int f, int rr) {
    for (int i = 0; i < 31; i++) r.s[i] = s[i];
    r.f = f;
    r.r = rr;
}

// ---- fast SampleMatches for a whole round, one wave --------------------------
// (1) the glibc TYPE_3 stream is generated with the 31-word ring held in
//     registers (statically indexed after rotating to phase 0),
// (2) all lanes reduce draws to min(rand()%ng, rand()%ng) in parallel,
// (3) every draw position d speculatively forms "the sample that starts at d"
//     (S distinct ids, ascending = std::set order) and its length in draws,
// (4) lane 0 chases d -> d + len(d) for the round's visited iterations,
// (5) the stream is re-advanced by exactly the draws consumed.
// Bit-identical to draw_samples(); overflow of the LDS window falls back to it.
#define DRAW_MAX 2816

struct SampLds {
    uint32_t raw[2 * DRAW_MAX];
    uint16_t mval[DRAW_MAX];
    uint16_t len[DRAW_MAX];
    uint16_t ids[DRAW_MAX][MAX_SAMPLE];
};

ODO_INLINE void gen_raw(int32_t* st, int32_t& f, int32_t& r, uint32_t* out, int n) {
    uint32_t reg[31];
#pragma unroll
    for (int j = 0; j < 31; j++) {
        int q = r + j;
        q = q >= 31 ? q - 31 : q;
        reg[j] = (uint32_t)st[q];
    }
    int produced = 0;
    while (produced + 31 <= n) {
#pragma unroll
        for (int j = 0; j < 31; j++) {
            reg[(j + 3) % 31] += reg[j];
            if (out) out[produced + j] = reg[(j + 3) % 31] >> 1;
        }
        produced += 31;
    }
    const int rem = n - produced;
#pragma unroll
    for (int j = 0; j < 31; j++)
        if (j < rem) {
            reg[(j + 3) % 31] += reg[j];
            if (out) out[produced + j] = reg[(j + 3) % 31] >> 1;
        }
    // physical index of logical j is (r + j) % 31; after rem extra steps the
    // logical origin moved by rem
#pragma unroll
    for (int j = 0; j < 31; j++) {
        int q = r + j;
        q = q >= 31 ? q - 31 : q;
        st[q] = (int32_t)reg[j];
    }
    r = (r + (n % 31)) % 31;
    f = (r + 3) % 31;
}

// state: 31 ints + f + r in LDS (st), shared by the wave; count <= RS_BMAX.
ODO_INLINE void round_samples(int lane, int32_t* st, int32_t* fr, int ng, int S, int count, int* out, SampLds& L) {
    if (count <= 0) return;
    const int D = min(DRAW_MAX, 6 * count + 64);
    __shared__ int32_t save[33];
    __shared__ int s_pos, s_ok;
    if (lane == 0) {
        for (int i = 0; i < 31; i++) save[i] = st[i];
        save[31] = fr[0];
        save[32] = fr[1];
        int32_t f = fr[0], r = fr[1];
        gen_raw(st, f, r, L.raw, 2 * D);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int d = lane; d < D; d += 64) {
        uint32_t a = L.raw[2 * d] % (uint32_t)ng, b = L.raw[2 * d + 1] % (uint32_t)ng;
        L.mval[d] = (uint16_t)(a > b ? b : a);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (int d = lane; d < D; d += 64) {
        int ids[MAX_SAMPLE];
        int cnt = 0, k = d;
        while (cnt < S && k < D) {
            const int id1 = L.mval[k++];
            bool dup = false;
            for (int q = 0; q < cnt; q++) dup |= ids[q] == id1;
            if (!dup) {
                int pos = cnt;
                while (pos > 0 && ids[pos - 1] > id1) {
                    ids[pos] = ids[pos - 1];
                    pos--;
                }
                ids[pos] = id1;
                cnt++;
            }
        }
        L.len[d] = (uint16_t)(cnt == S ? k - d : 0);
        for (int q = 0; q < S; q++) L.ids[d][q] = (uint16_t)(q < cnt ? ids[q] : 0);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (lane == 0) {
        int pos = 0, ok = 1;
        for (int v = 0; v < count; v++) {
            if (pos >= D || L.len[pos] == 0) {
                ok = 0;
                break;
            }
            int* o = out + v * (MAX_SAMPLE + 1);
            o[0] = S;
            for (int q = 0; q < S; q++) o[1 + q] = L.ids[pos][q];
            pos += L.len[pos];
        }
        // restore the round-start state and advance by exactly the consumed draws
        for (int i = 0; i < 31; i++) st[i] = save[i];
        int32_t f = save[31], r = save[32];
        if (ok) {
            gen_raw(st, f, r, nullptr, 2 * pos);
        } else {
            Rng rr;
            rng_load(rr, st, f, r);
            draw_samples(rr, ng, S, count, out);
            for (int i = 0; i < 31; i++) st[i] = rr.s[i];
            f = rr.f;
            r = rr.r;
        }
        fr[0] = f;
        fr[1] = r;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__global__ void __launch_bounds__(256) k_ransac_prep(RansacBufs B, RansacCfg cfg, int round0) {
    const int p = blockIdx.x;
    const int t = threadIdx.x;
    __shared__ Rng s_rng;
    RState* S = B.st + p;
    odo_pair_result* R = B.res + p;
    float* T12o = B.T12 + (size_t)p * 16;
    const int ng = B.n_good[p];
    const int nm = B.n_matches[p];
    const int Ssz = cfg.sample_size < MAX_SAMPLE ? cfg.sample_size : MAX_SAMPLE;
    bool active = B.pair_valid[p] && nm >= B.min_matches && nm >= cfg.min_inlier_th;
    if (t == 0) {
        R->rmse = 1e6f;
        R->n_good = active ? ng : 0;
        R->n_inliers = 0;
        R->ransac_ok = 0;
        R->visited = 0;
        for (int i = 0; i < 16; i++) R->T12[i] = T12o[i] = (i % 5 == 0) ? 1.f : 0.f;
    }
    active = active && ng >= cfg.min_inlier_th;
    const int words = (ng + 31) >> 5;
    if (active) {
        const SortElR* G = B.good + (size_t)p * B.match_cap;
        const odo_dmatch* M = B.matches + (size_t)p * B.match_cap;
        const float* X1 = B.xyz + (size_t)(B.slot0 + p) * B.kp_cap * 3;
        const float* X2 = B.xyz + (size_t)(B.slot0 + p + 1) * B.kp_cap * 3;
        GoodPt* P = B.gpts + (size_t)p * B.match_cap;
        for (int k = t; k < ng; k += 256) {
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
        uint32_t* BM = B.best_mask + (size_t)p * B.mask_words;
        for (int w = t; w < words; w += 256) BM[w] = 0;
    }
    if (t == 0) {
        if (B.rng_io) {
            for (int i = 0; i < 31; i++) s_rng.s[i] = B.rng_io->state[i];
            s_rng.f = B.rng_io->fpos;
            s_rng.r = B.rng_io->rpos;
        } else {
            s_rng.seed(pair_seed(B.seed_base, B.pair_base + (uint64_t)p));
        }
        for (int i = 0; i < 31; i++) S->rng0_s[i] = s_rng.s[i];
        S->rng0_f = s_rng.f;
        S->rng0_r = s_rng.r;
        S->active = active ? 1 : 0;
        S->ng = ng;
        S->S = Ssz;
        S->words = words;
        S->n = 0;
        S->visited = 0;
        S->valid = 0;
        S->best_cnt = 0;
        S->rmse = 1e6f;
        for (int i = 0; i < 12; i++) S->bestT[i] = (i % 5 == 0) ? 1.f : 0.f;
        S->round_base = 0;
        const int H = cfg.iterations;
        S->done = (!active || H <= 0 || ng < Ssz) ? 1 : 0;
        S->round_count = S->done ? 0 : min(round0, H);
    }
    __syncthreads();
    __shared__ SampLds s_L;
    __shared__ int32_t s_st[31], s_fr[2];
    const int cnt = S->round_count;
    if (t < 64 && cnt > 0) {
        if (t == 0) {
            for (int i = 0; i < 31; i++) s_st[i] = s_rng.s[i];
            s_fr[0] = s_rng.f;
            s_fr[1] = s_rng.r;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        round_samples(t, s_st, s_fr, ng, Ssz, cnt, B.samples + (size_t)p * RS_BMAX * (MAX_SAMPLE + 1), s_L);
        if (t == 0) {
            for (int i = 0; i < 31; i++) S->rng_s[i] = s_st[i];
            S->rng_f = s_fr[0];
            S->rng_r = s_fr[1];
        }
    } else if (t == 0 && cnt == 0) {
        for (int i = 0; i < 31; i++) S->rng_s[i] = s_rng.s[i];
        S->rng_f = s_rng.f;
        S->rng_r = s_rng.r;
    }
}

// ---------------------------------------------------------------- eval
#define EV_WAVES 4

ODO_INLINE void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__global__ void __launch_bounds__(64 * EV_WAVES) k_ransac_eval(RansacBufs B, RansacCfg cfg) {
    const int p = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ uint32_t s_cur[EV_WAVES][256];   // current inlier set (refined), bit k = good match k
    __shared__ uint32_t s_new[EV_WAVES][256];   // set produced by the sweep
    __shared__ GoodPt s_pts[EV_WAVES][64];
    __shared__ double s_d2[EV_WAVES][64];
    const RState* S = B.st + p;
    if (S->done) return;
    const int count = S->round_count;
    const int ng = S->ng, words = S->words;
    const GoodPt* P = B.gpts + (size_t)p * B.match_cap;
    MahalConst K;
    K.raster_cov_x = cfg.raster_cov_x;
    K.raster_cov_y = cfg.raster_cov_y;
    K.depth_cov = *B.latch;
    const float th = cfg.max_mahal * cfg.max_mahal;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    uint32_t* cur = s_cur[wave];
    uint32_t* nw = s_new[wave];
    GoodPt* pts = s_pts[wave];
    double* d2s = s_d2[wave];
    for (int h = blockIdx.y * EV_WAVES + wave; h < count; h += gridDim.y * EV_WAVES) {
        const int* smp = B.samples + ((size_t)p * RS_BMAX + h) * (MAX_SAMPLE + 1);
        double refinedError = 1e6;
        unsigned refinedCnt = 0;
        float refinedT[12];
        for (int i = 0; i < 12; i++) refinedT[i] = (i % 5 == 0) ? 1.f : 0.f;
        bool useSample = true;
        for (int refinements = 1; refinements < 20; refinements++) {
            // ---- GetTransformFromMatches (ransac.cpp:295-313): lane 0, in set order
            TFC tfc;
            tfc.reset();
            if (useSample) {
                if (lane == 0) {
                    const int ns = smp[0];
                    for (int q = 0; q < ns; q++) {
                        const GoodPt g = P[smp[1 + q]];
                        if (__builtin_isnan(g.sz) || __builtin_isnan(g.tz)) continue;
                        tfc.add(g.sx, g.sy, g.sz, g.tx, g.ty, g.tz, g.w);
                    }
                }
            } else {
                for (int c0 = 0; c0 < ng; c0 += 64) {
                    const int k = c0 + lane;
                    const bool in = k < ng && ((cur[k >> 5] >> (k & 31)) & 1);
                    const uint64_t bal = __ballot(in);
                    if (in) {
                        const int pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
                        pts[pos] = P[k];
                    }
                    wave_sync();
                    if (lane == 0) {
                        const int nin = __popcll(bal);
                        for (int q = 0; q < nin; q++) {
                            const GoodPt g = pts[q];
                            if (__builtin_isnan(g.sz) || __builtin_isnan(g.tz)) continue;
                            tfc.add(g.sx, g.sy, g.sz, g.tx, g.ty, g.tz, g.w);
                        }
                    }
                    wave_sync();
                }
            }
            float Tl[12];
            for (int i = 0; i < 12; i++) Tl[i] = 0.f;
            if (lane == 0) tfc.get(Tl);
            float T[12];
#pragma unroll
            for (int i = 0; i < 12; i++) T[i] = __shfl(Tl[i], 0);
            double Td[12];
#pragma unroll
            for (int i = 0; i < 12; i++) Td[i] = (double)T[i];
            // ---- ComputeInliersAndError (ransac.cpp:315-348)
            double meanError = 0.0;
            unsigned cnt = 0;
            for (int c0 = 0; c0 < ng; c0 += 64) {
                const int k = c0 + lane;
                bool in = false;
                double d = 0.0;
                if (k < ng) {
                    const GoodPt g = P[k];
                    if (!(g.sz == 0.0f || g.tx == 0.0f)) {
                        const float x1[3] = {g.sx, g.sy, g.sz}, x2[3] = {g.tx, g.ty, g.tz};
                        d = error_function2(x1, x2, Td, K);
                        in = !(d > th) && (d >= 0.0);
                    }
                }
                const uint64_t bal = __ballot(in);
                d2s[lane] = d;
                if (lane == 0) {
                    nw[c0 >> 5] = (uint32_t)bal;
                    if (c0 + 32 < ng) nw[(c0 >> 5) + 1] = (uint32_t)(bal >> 32);
                }
                wave_sync();
                if (lane == 0) {
                    uint64_t b = bal;
                    while (b) {
                        const int q = __builtin_ctzll(b);
                        b &= b - 1;
                        meanError += d2s[q];
                    }
                }
                cnt += (unsigned)__popcll(bal);
                wave_sync();
            }
            meanError = __shfl(meanError, 0);
            if (cnt < 3) meanError = 1e9;
            else {
                meanError /= (double)cnt;
                meanError = sqrt(meanError);
            }
            if (cnt < minInl || meanError > (double)cfg.max_mahal) break;
            if (cnt >= refinedCnt && meanError <= refinedError) {
                const unsigned prev = refinedCnt;
#pragma unroll
                for (int i = 0; i < 12; i++) refinedT[i] = T[i];
                refinedError = meanError;
                refinedCnt = cnt;
                for (int w = lane; w < words; w += 64) cur[w] = nw[w];
                wave_sync();
                useSample = false;
                if (cnt == prev) break;
            } else break;
        }
        HypRes* hr = B.hyp + (size_t)p * RS_BMAX + h;
        if (lane == 0) {
            hr->err = refinedError;
            hr->cnt = (int)refinedCnt;
        }
        if (lane < 12) {
            float v = refinedT[0];
#pragma unroll
            for (int i = 1; i < 12; i++)
                if (lane == i) v = refinedT[i];
            hr->T[lane] = v;
        }
        uint32_t* mo = B.masks + ((size_t)p * RS_BMAX + h) * B.mask_words;
        if (refinedCnt > 0)
            for (int w = lane; w < words; w += 64) mo[w] = cur[w];
        wave_sync();
    }
}

// ---------------------------------------------------------------- scan
__global__ void __launch_bounds__(64) k_ransac_scan(RansacBufs B, RansacCfg cfg, int next_count) {
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    __shared__ Rng s_rng;
    __shared__ int s_copy_h;
    RState* S = B.st + p;
    if (S->done) return;
    const int ng = S->ng, words = S->words;
    const int H = cfg.iterations;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    __shared__ double s_err[RS_BMAX];
    __shared__ int s_hc[RS_BMAX];
    __shared__ int s_next;
    const int count0 = S->round_count;
    for (int v = lane; v < count0; v += 64) {
        const HypRes* hr = B.hyp + (size_t)p * RS_BMAX + v;
        s_err[v] = hr->err;
        s_hc[v] = hr->cnt;
    }
    __syncthreads();
    if (lane == 0) {
        s_copy_h = -1;
        s_next = 0;
        int n = S->n;
        const int count = S->round_count;
        for (int v = 0; v < count && n < H; v++) {
            S->visited++;
            const HypRes* hr = B.hyp + (size_t)p * RS_BMAX + v;
            const unsigned rc = (unsigned)s_hc[v];
            const double re = s_err[v];
            bool brk = false;
            if (rc > 0) {
                S->valid++;
                if (re <= (double)S->rmse && rc >= (unsigned)S->best_cnt && rc >= minInl) {
                    S->rmse = (float)re;
                    S->best_cnt = (int)rc;
                    for (int i = 0; i < 12; i++) S->bestT[i] = hr->T[i];
                    s_copy_h = v;
                    if (rc > ng * 0.5) n += 10;
                    if (rc > ng * 0.75) n += 10;
                    if (rc > ng * 0.8) brk = true;
                }
            }
            n++;
            if (brk) {
                n = H;
                break;
            }
        }
        S->n = n;
        S->round_base += count;
        if (n >= H) S->done = 1;
        if (!S->done && next_count > 0) {
            const int cnt = min(next_count, H - n);
            S->round_count = cnt;
            s_next = cnt;
        } else {
            S->done = 1;
            S->round_count = 0;
        }
    }
    __syncthreads();
    if (s_next > 0) {
        __shared__ SampLds s_L;
        __shared__ int32_t s_st[31], s_fr[2];
        if (lane == 0) {
            for (int i = 0; i < 31; i++) s_st[i] = S->rng_s[i];
            s_fr[0] = S->rng_f;
            s_fr[1] = S->rng_r;
        }
        __syncthreads();
        round_samples(lane, s_st, s_fr, ng, S->S, s_next, B.samples + (size_t)p * RS_BMAX * (MAX_SAMPLE + 1), s_L);
        if (lane == 0) {
            for (int i = 0; i < 31; i++) S->rng_s[i] = s_st[i];
            S->rng_f = s_fr[0];
            S->rng_r = s_fr[1];
        }
    }
    __syncthreads();
    const int h = s_copy_h;
    if (h >= 0) {
        const uint32_t* src = B.masks + ((size_t)p * RS_BMAX + h) * B.mask_words;
        uint32_t* BM = B.best_mask + (size_t)p * B.mask_words;
        for (int w = lane; w < words; w += 64) BM[w] = src[w];
    }
}

// ---------------------------------------------------------------- final
__global__ void __launch_bounds__(64) k_ransac_final(RansacBufs B, RansacCfg cfg) {
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    __shared__ Rng s_rng;
    __shared__ double s_d2[64];
    __shared__ int s_ok;
    RState* S = B.st + p;
    odo_pair_result* R = B.res + p;
    float* T12o = B.T12 + (size_t)p * 16;
    if (!S->active) return;
    const int ng = S->ng, words = S->words;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    if (S->valid == 0) {
        // identity fallback: one sweep with T = I, same lane split as the eval kernel
        const GoodPt* P = B.gpts + (size_t)p * B.match_cap;
        MahalConst K;
        K.raster_cov_x = cfg.raster_cov_x;
        K.raster_cov_y = cfg.raster_cov_y;
        K.depth_cov = *B.latch;
        const float th = cfg.max_mahal * cfg.max_mahal;
        const double Td[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
        uint32_t* BM = B.best_mask + (size_t)p * B.mask_words;
        double meanError = 0.0;
        unsigned cnt = 0;
        for (int c0 = 0; c0 < ng; c0 += 64) {
            const int k = c0 + lane;
            bool in = false;
            double d = 0.0;
            if (k < ng) {
                const GoodPt g = P[k];
                if (!(g.sz == 0.0f || g.tx == 0.0f)) {
                    const float x1[3] = {g.sx, g.sy, g.sz}, x2[3] = {g.tx, g.ty, g.tz};
                    d = error_function2(x1, x2, Td, K);
                    in = !(d > th) && (d >= 0.0);
                }
            }
            const uint64_t bal = __ballot(in);
            s_d2[lane] = d;
            if (lane == 0) {
                BM[c0 >> 5] = (uint32_t)bal;
                if (c0 + 32 < ng) BM[(c0 >> 5) + 1] = (uint32_t)(bal >> 32);
            }
            __syncthreads();
            if (lane == 0) {
                uint64_t b = bal;
                while (b) {
                    const int q = __builtin_ctzll(b);
                    b &= b - 1;
                    meanError += s_d2[q];
                }
            }
            cnt += (unsigned)__popcll(bal);
            __syncthreads();
        }
        if (lane == 0) {
            if (cnt < 3) meanError = 1e9;
            else {
                meanError /= (double)cnt;
                meanError = sqrt(meanError);
            }
            s_ok = (cnt > minInl && meanError < (double)cfg.max_mahal) ? 1 : 0;
            if (s_ok) {
                S->best_cnt = (int)cnt;
                S->rmse = (float)((double)S->rmse + meanError);
                for (int i = 0; i < 12; i++) S->bestT[i] = (i % 5 == 0) ? 1.f : 0.f;
            } else {
                S->best_cnt = 0;
            }
        }
        __syncthreads();
        if (!s_ok)
            for (int w = lane; w < words; w += 64) BM[w] = 0;
    }
    if (lane == 0) {
        R->rmse = S->rmse;
        R->n_inliers = S->best_cnt;
        R->ransac_ok = (unsigned)S->best_cnt >= minInl ? 1 : 0;
        R->visited = S->visited;
        for (int i = 0; i < 12; i++) R->T12[i] = T12o[i] = S->bestT[i];
        R->T12[12] = R->T12[13] = R->T12[14] = 0.f;
        R->T12[15] = 1.f;
        T12o[12] = T12o[13] = T12o[14] = 0.f;
        T12o[15] = 1.f;
        if (B.rng_io) {
            // advance the caller's rand() stream by the visited iterations' draws only
            rng_load(s_rng, S->rng0_s, S->rng0_f, S->rng0_r);
            for (int v = 0; v < S->visited; v++) {
                int cntv = 0, ids[MAX_SAMPLE], safety = 0;
                while (cntv < S->S) {
                    int id1 = (int)((uint32_t)s_rng.next() % (uint32_t)ng);
                    int id2 = (int)((uint32_t)s_rng.next() % (uint32_t)ng);
                    if (id1 > id2) id1 = id2;
                    bool dup = false;
                    for (int q = 0; q < cntv; q++) dup |= ids[q] == id1;
                    if (!dup) ids[cntv++] = id1;
                    if (++safety > 10000) break;
                }
            }
            for (int i = 0; i < 31; i++) B.rng_io->state[i] = s_rng.s[i];
            B.rng_io->fpos = s_rng.f;
            B.rng_io->rpos = s_rng.r;
        }
    }
}

// ---------------------------------------------------------------- host side
size_t ransac_gpt_bytes() { return sizeof(GoodPt); }

size_t ransac_scratch_bytes(int npairs, int match_cap, int mask_words) {
    size_t s = (size_t)npairs * match_cap * sizeof(GoodPt) + (size_t)npairs * sizeof(RState) + 16;
    s += (size_t)npairs * RS_BMAX * sizeof(HypRes);
    s += (size_t)npairs * RS_BMAX * (MAX_SAMPLE + 1) * sizeof(int) + 16;
    s += (size_t)npairs * RS_BMAX * (size_t)mask_words * 4;
    return s;
}

void launch_ransac(hipStream_t st, const void* good, const int* n_good, const int* n_matches, const odo_dmatch* matches,
                   const float* xyz, int kp_cap, int slot0, int match_cap, RansacCfg cfg, const double* latch,
                   uint64_t seed_base, uint64_t pair_base, const int* pair_valid, int min_matches, odo_rng* rng_io,
                   void* scratch, uint32_t* best_mask, int mask_words, odo_pair_result* res, float* T12, int npairs) {
    RansacBufs B;
    B.good = (const SortElR*)good;
    B.n_good = n_good;
    B.n_matches = n_matches;
    B.matches = matches;
    B.xyz = xyz;
    B.kp_cap = kp_cap;
    B.slot0 = slot0;
    B.match_cap = match_cap;
    B.latch = latch;
    B.seed_base = seed_base;
    B.pair_base = pair_base;
    B.pair_valid = pair_valid;
    B.min_matches = min_matches;
    B.rng_io = rng_io;
    B.mask_words = mask_words;
    B.best_mask = best_mask;
    B.res = res;
    B.T12 = T12;
    // carve the per-call scratch: gpts | state | hyp | samples | masks
    char* s = (char*)scratch;
    B.gpts = (GoodPt*)s;
    s += (size_t)npairs * match_cap * sizeof(GoodPt);
    B.st = (RState*)s;
    s += (size_t)npairs * sizeof(RState);
    s = (char*)(((uintptr_t)s + 15) & ~(uintptr_t)15);
    B.hyp = (HypRes*)s;
    s += (size_t)npairs * RS_BMAX * sizeof(HypRes);
    B.samples = (int*)s;
    s += (size_t)npairs * RS_BMAX * (MAX_SAMPLE + 1) * sizeof(int);
    s = (char*)(((uintptr_t)s + 15) & ~(uintptr_t)15);
    B.masks = (uint32_t*)s;
    // round schedule: 16, 48, 448, then 512 until H is covered
    int sizes[64];
    int nr = 0, cum = 0;
    const int H = cfg.iterations;
    const int sched[3] = {16, 48, 448};
    while (cum < H && nr < 64) {
        const int b = nr < 3 ? sched[nr] : RS_BMAX;
        sizes[nr++] = b;
        cum += b;
    }
    if (nr == 0) sizes[nr++] = 16;
    hipLaunchKernelGGL(k_ransac_prep, dim3(npairs), dim3(256), 0, st, B, cfg, sizes[0]);
    for (int r = 0; r < nr; r++) {
        const int b = sizes[r];
        dim3 g(npairs, (b + EV_WAVES - 1) / EV_WAVES);
        hipLaunchKernelGGL(k_ransac_eval, g, dim3(64 * EV_WAVES), 0, st, B, cfg);
        const int next = r + 1 < nr ? sizes[r + 1] : 0;
        hipLaunchKernelGGL(k_ransac_scan, dim3(npairs), dim3(64), 0, st, B, cfg, next);
    }
    hipLaunchKernelGGL(k_ransac_final, dim3(npairs), dim3(64), 0, st, B, cfg);
}

}  // namespace odo
