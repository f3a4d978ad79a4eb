// Ransac::Iterate(Frame*,Frame*,m12) for gfx950 (Odometry/ransac.cpp:155-267).
//
// The reference visits iterations one after another: SampleMatches draws a
// minimal set from the glibc rand() stream, the refinement loop re-fits PCL's
// TransformationFromCorrespondences to the Mahalanobis inlier set, and a
// running best with n+=10 skips / >80% break decides when to stop. Here:
//
//   k_ransac_raw    side stream, at batch start: each pair's rand() words are
//                   data independent (seed only), generated while frames are
//                   still being extracted
//   k_ransac_prep   per pair: early-outs, GoodPt table, and the minimal sets of
//                   ALL iterations at once (parallel mod, speculative sample
//                   lengths, ballot scan over sample starts)
//   k_ransac_eval   one launch, one wave per iteration (hypothesis); whichever
//                   wave completes the prefix runs the reference's ordered fold
//                   under a lock; once it breaks, in-flight hypotheses abort
//   k_ransac_final  per pair: identity fallback (ransac.cpp:252-264), outputs,
//                   the caller's rand() state after exactly the visited draws
//
// The TFC recurrence and the meanError sum are order-dependent float/double
// folds; they run in match order, bit-identical to the reference.
#include <algorithm>
#include <map>
#include <mutex>
#include <cstdlib>
#include <vector>

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

#define EV_WAVES_C 4   // waves per k_ransac_eval workgroup (EV_WAVES below)
#ifndef EV2_FOLD_WAVE
#define EV2_FOLD_WAVE 1  // the second launch's ordered fold by the whole wave (0: lane 0)
#endif
#ifndef EV_H0
// hypotheses per pair in the first eval launch of a batch (round 5: 2; a row
// of 4 until round 4). In the bench's sequence 52 of 64 pairs break at
// hypothesis 0 and 10 at hypothesis 1 (oracle, the 80 % break of
// ransac.cpp:247), so the 2 further waves of a row of 4 ran for nothing
// beside the extraction kernels
#define EV_H0 2
#endif
#define MAX_SAMPLE 8
#define SREC (MAX_SAMPLE + 2)  // sample record: count, ids[MAX_SAMPLE], end (draw pairs consumed after it)

struct RState {
    int32_t rng0_s[31];  // rand() state at entry (written by k_ransac_raw)
    int32_t rng0_f, rng0_r;
    int active, done, ng, S, words, H;
    // ordered fold (ransac.cpp:233-249), updated under `lock`
    int lock, fold_pos, n, visited, valid, best_cnt, best_h;
    int efast;  // every evaluated point's depths in ef_fast_range (k_ransac_prep): ErrorFunction2's fast form is exact
    float rmse;
    int sweeps, fitpts;  // work of the visited prefix (odo_pair_result.n_sweeps / n_fit_points)
    int nexth;           // k_ransac_lanes: the next hypothesis a lane takes up
};

struct HypRes {
    double err;
    int cnt;
    int pad;  // work: ComputeInliersAndError sweeps | TFC points added << 5
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
    const int* pair_valid;
    int min_matches;
    odo_rng* rng_io;
    GoodPt* gpts;      // [pair][match_cap]
    RState* st;        // [pair]
    HypRes* hyp;       // [pair][hcap]
    int* samples;      // [pair][hcap][SREC], by visited index
    int* ready;        // [pair][hcap]
    uint32_t* masks;   // [pair][hcap][mask_words]
    uint32_t* raw;     // [pair][rawcap] full 32-bit generator words (rand() = word >> 1)
    int hcap, rawcap;
    uint32_t* best_mask;
    int mask_words;
    odo_pair_result* res;
    float* T12;
    // hypotheses mode: evaluate only [h_lo, h_hi), no fold
    int h_lo, h_hi, no_fold;
    int* open_list;  // [pair] pairs still folding after the first launch
    int* open_cnt;   // [0] their count, [1] the second launch's work counter, [2] all passed the EF guard
    uint32_t* lslab;  // k_ransac_lanes: [wave][2][mask_words][64] inlier sets
};

ODO_INLINE int ld_relaxed(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
ODO_INLINE void st_relaxed(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// One std::set insertion (ascending order) with statically indexed registers.
ODO_INLINE bool set_insert(int (&ids)[MAX_SAMPLE], int& cnt, int id1) {
    bool dup = false;
    int less = 0;
#pragma unroll
    for (int q = 0; q < MAX_SAMPLE; q++) {
        const bool v = q < cnt;
        dup |= v && ids[q] == id1;
        less += (v && ids[q] < id1) ? 1 : 0;
    }
    if (dup) return false;
#pragma unroll
    for (int q = MAX_SAMPLE - 1; q >= 1; q--) ids[q] = q > less ? ids[q - 1] : (q == less ? id1 : ids[q]);
    if (less == 0) ids[0] = id1;
    cnt++;
    return true;
}

// SampleMatches (ransac.cpp:269-293) for one visited iteration: pairs of
// rand() draws reduced to min(rand()%M, rand()%M) until S distinct ids.
ODO_INLINE int draw_one(Rng& r, int ng, int S, int (&ids)[MAX_SAMPLE], int& used) {
#pragma unroll
    for (int q = 0; q < MAX_SAMPLE; q++) ids[q] = 0;
    int cnt = 0, safety = 0;
    while (cnt < S) {
        int id1 = (int)((uint32_t)r.next() % (uint32_t)ng);
        const int id2 = (int)((uint32_t)r.next() % (uint32_t)ng);
        if (id1 > id2) id1 = id2;
        set_insert(ids, cnt, id1);
        if (++safety > 10000) break;
    }
    used = safety > 10000 ? 10001 : safety;
    return cnt;
}


ODO_INLINE void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

ODO_INLINE void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

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
            if (out) out[produced + j] = reg[(j + 3) % 31];
        }
        produced += 31;
    }
    const int rem = n - produced;
#pragma unroll
    for (int j = 0; j < 31; j++)
        if (j < rem) {
            reg[(j + 3) % 31] += reg[j];
            if (out) out[produced + j] = reg[(j + 3) % 31];
        }
#pragma unroll
    for (int j = 0; j < 31; j++) {
        int q = r + j;
        q = q >= 31 ? q - 31 : q;
        st[q] = (int32_t)reg[j];
    }
    r = (r + (n % 31)) % 31;
    f = (r + 3) % 31;
}

// Sample starting at draw d of the window; returns its length in draw pairs
// (0 if the window ends first).
ODO_INLINE int form_sample(const uint16_t* mval, int d, int D, int S, int (&ids)[MAX_SAMPLE]) {
#pragma unroll
    for (int q = 0; q < MAX_SAMPLE; q++) ids[q] = 0;
    int cnt = 0, k = d;
    while (cnt < S && k < D) set_insert(ids, cnt, (int)mval[k++]);
    return cnt == S ? k - d : 0;
}

// glibc __srandom_r into LDS: Schrage LCG fill, then 310 discards in registers.
ODO_INLINE void seed_ring(uint32_t seedv, int32_t* st, int32_t* fr) {
    if (seedv == 0) seedv = 1;
    st[0] = (int32_t)seedv;
    int32_t word = (int32_t)seedv;
    for (int i = 1; i < 31; ++i) {
        const long hi = word / 127773;
        const long lo = word % 127773;
        long w2 = 16807 * lo - 2836 * hi;
        if (w2 < 0) w2 += 2147483647;
        word = (int32_t)w2;
        st[i] = word;
    }
    int32_t f = 3, r = 0;
    gen_raw(st, f, r, nullptr, 310);
    fr[0] = f;
    fr[1] = r;
}


// rand() state after N generator words from the entry state (the ring holds
// the last 31 words; the word of step k sits at logical slot (k+3)%31).
ODO_INLINE void ring_at(const uint32_t* raw, const RState* S, int N, Rng& R) {
    const int r0 = S->rng0_r;
    for (int L = 0; L < 31; L++) {
        const int k0 = (L + 28) % 31;
        int32_t val = S->rng0_s[(r0 + L) % 31];
        if (k0 < N) val = (int32_t)raw[k0 + 31 * ((N - 1 - k0) / 31)];
        R.s[(r0 + L) % 31] = val;
    }
    R.r = (r0 + N) % 31;
    R.f = (R.r + 3) % 31;
}

// The generator words x_n = x_{n-31} + x_{n-3} (mod 2^32) are a linear map of
// the 31-word state, so instead of one lane producing all rawcap words in
// sequence, lane k jumps to word k*L with a host-built matrix A^(kL) and
// produces its own L words (the 310 seeding discards jump too: A^310).
// Same words, bit for bit; ~150 us of serial generation becomes a 31x31
// matrix-vector product plus L steps per lane.
#define RAW_LANES 64

// state vector, oldest word first, from / to the ring (slot r = x_{n-3})
ODO_INLINE void ring_to_vec(const int32_t* st, int r, uint32_t* v) {
    for (int m = 0; m < 28; m++) v[m] = (uint32_t)st[(r + 3 + m) % 31];
    for (int m = 0; m < 3; m++) v[28 + m] = (uint32_t)st[(r + m) % 31];
}
ODO_INLINE void vec_to_ring(const uint32_t* v, int r, int32_t* st) {
    for (int m = 0; m < 28; m++) st[(r + 3 + m) % 31] = (int32_t)v[m];
    for (int m = 0; m < 3; m++) st[(r + m) % 31] = (int32_t)v[28 + m];
}

// jump: [RAW_LANES][31][31] stored as [i][j][lane] (lane k: A^(k*L)), then
// A^310 as [31][31]
__global__ void __launch_bounds__(64) k_ransac_raw(RansacBufs B, uint64_t seed_base, uint64_t pair_base,
                                                   const uint32_t* __restrict__ jump, int L) {
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    __shared__ int32_t s_st[31], s_fr[2];
    __shared__ uint32_t s_v[31], s_w[31];
    if (lane == 0) {
        if (B.rng_io) {
            for (int i = 0; i < 31; i++) s_st[i] = B.rng_io->state[i];
            s_fr[0] = B.rng_io->fpos;
            s_fr[1] = B.rng_io->rpos;
        } else {
            // __srandom_r: Schrage fill (f = 3, r = 0), discards below
            uint32_t seedv = pair_seed(seed_base, pair_base + (uint64_t)p);
            if (seedv == 0) seedv = 1;
            s_st[0] = (int32_t)seedv;
            int32_t word = (int32_t)seedv;
            for (int i = 1; i < 31; ++i) {
                const long hi = word / 127773;
                const long lo = word % 127773;
                long w2 = 16807 * lo - 2836 * hi;
                if (w2 < 0) w2 += 2147483647;
                word = (int32_t)w2;
                s_st[i] = word;
            }
            s_fr[0] = 3;
            s_fr[1] = 0;
        }
        ring_to_vec(s_st, s_fr[1], s_v);
    }
    lds_sync();
    if (!B.rng_io) {
        // 310 discards: v <- A^310 v (row `lane` per lane); r advances 310 % 31 = 0
        const uint32_t* D = jump + (size_t)RAW_LANES * 31 * 31;
        if (lane < 31) {
            uint32_t a = 0;
            for (int j = 0; j < 31; j++) a += D[lane * 31 + j] * s_v[j];
            s_w[lane] = a;
        }
        lds_sync();
        if (lane < 31) s_v[lane] = s_w[lane];
        lds_sync();
        if (lane == 0) vec_to_ring(s_v, s_fr[1], s_st);
        lds_sync();
    }
    RState* S = B.st + p;
    if (lane < 31) S->rng0_s[lane] = s_st[lane];
    if (lane == 0) {
        S->rng0_f = s_fr[0];
        S->rng0_r = s_fr[1];
    }
    // lane k: state at word k*L, then words [kL, kL + L)
    uint32_t reg[31];
    {
        uint32_t v[31];
#pragma unroll
        for (int i = 0; i < 31; i++) {
            uint32_t a = 0;
            if (lane == 0) a = s_v[i];
            else
                for (int j = 0; j < 31; j++) a += jump[((size_t)i * 31 + j) * RAW_LANES + lane] * s_v[j];
            v[i] = a;
        }
        // ring registers as gen_raw holds them: reg[0..2] = x_{n-3..n-1}, reg[3..30] = x_{n-31..n-4}
#pragma unroll
        for (int m = 0; m < 28; m++) reg[3 + m] = v[m];
#pragma unroll
        for (int m = 0; m < 3; m++) reg[m] = v[28 + m];
    }
    uint32_t* out = B.raw + (size_t)p * B.rawcap;
    const int k0 = lane * L;
    const int n = max(0, min(L, B.rawcap - k0));
    int produced = 0;
    while (produced + 31 <= n) {
#pragma unroll
        for (int j = 0; j < 31; j++) {
            reg[(j + 3) % 31] += reg[j];
            out[k0 + produced + j] = reg[(j + 3) % 31];
        }
        produced += 31;
    }
#pragma unroll
    for (int j = 0; j < 31; j++)
        if (produced + j < n) {
            reg[(j + 3) % 31] += reg[j];
            out[k0 + produced + j] = reg[(j + 3) % 31];
        }
}

// ---------------------------------------------------------------- sampling
// SampleMatches for every iteration of a pair (ransac.cpp:269-293): each draw
// pair d reduces to mval[d] = min(rand()%ng, rand()%ng); the sample starting at
// d takes S draw pairs unless an id repeats (rare), so lengths are formed
// speculatively for every d and a ballot scan walks the chain of sample starts.
#define SWIN 4096

struct SampWin {
    uint16_t mval[SWIN];
    uint16_t len[SWIN];
    uint16_t posv[SWIN];
    int nv, e;
};

template <int S>
ODO_INLINE int sample_len_fast(const uint16_t* mval, int d, int D) {
    if (d + S > D) return -1;
    int w[S];
#pragma unroll
    for (int q = 0; q < S; q++) w[q] = mval[d + q];
    bool dup = false;
#pragma unroll
    for (int i = 0; i < S; i++)
#pragma unroll
        for (int j = i + 1; j < S; j++) dup |= w[i] == w[j];
    return dup ? -1 : S;
}

ODO_INLINE int sample_len(const uint16_t* mval, int d, int D, int S) {
    int l = -1;
    if (S == 4) l = sample_len_fast<4>(mval, d, D);
    else if (S == 3) l = sample_len_fast<3>(mval, d, D);
    if (l > 0) return l;
    int ids[MAX_SAMPLE];
    return form_sample(mval, d, D, S, ids);
}

// ids of the sample at d (length ln): sorted window when duplicate-free.
ODO_INLINE void sample_ids(const uint16_t* mval, int d, int D, int S, int ln, int (&ids)[MAX_SAMPLE]) {
    if (ln == S) {
#pragma unroll
        for (int q = 0; q < MAX_SAMPLE; q++) ids[q] = q < S ? (int)mval[min(d + q, SWIN - 1)] : 0x7fffffff;
#pragma unroll
        for (int i = 0; i < MAX_SAMPLE; i++)
#pragma unroll
            for (int j = 0; j < MAX_SAMPLE - 1 - i; j++) {
                const int a = ids[j], b = ids[j + 1];
                ids[j] = a < b ? a : b;
                ids[j + 1] = a < b ? b : a;
            }
    } else {
        form_sample(mval, d, D, S, ids);
    }
}

// One wave: chain of sample starts through the window (0, len[0], ...). Lane j
// guesses "start of sample v+j" = base + S*j, valid up to the first irregular
// sample; that one is resolved through its stored length.
ODO_INLINE void chase_window(int lane, SampWin& L, int D, int S, int want) {
    int v = 0, base = 0;
    while (v < want) {
        const int vv = v + lane;
        const int pos = base + S * lane;
        const bool inr = vv < want;
        const int ln = (inr && pos < D) ? (int)L.len[pos] : 0;
        const uint64_t irr = __ballot(inr && ln != S);
        if (!irr) {
            const int nin = __popcll(__ballot(inr));
            if (inr) L.posv[vv] = (uint16_t)pos;
            v += nin;
            base += S * nin;
            continue;
        }
        const int f = __builtin_ctzll(irr);
        const int lnf = __shfl(ln, f);
        if (lane < f || (lane == f && lnf > 0)) L.posv[vv] = (uint16_t)pos;
        if (lnf == 0) {
            v += f;
            base += S * f;
            break;
        }
        v += f + 1;
        base += S * f + lnf;
    }
    if (lane == 0) {
        L.nv = v;
        L.e = base;
    }
}

ODO_INLINE void write_rec(int* o, int cnt, const int (&ids)[MAX_SAMPLE], int end) {
    o[0] = cnt;
#pragma unroll
    for (int q = 0; q < MAX_SAMPLE; q++)
        if (q < cnt) o[1 + q] = ids[q];
    o[SREC - 1] = end;
}

// All H samples of pair p (256 threads). Falls back to the serial draw when
// the generated words run out (only with extreme duplicate rates).
ODO_INLINE void pair_samples(const RansacBufs& B, int p, int ng, int S, int H, SampWin& L, Rng& R) {
    const int t = threadIdx.x;
    const uint32_t* raw = B.raw + (size_t)p * B.rawcap;
    int* rec = B.samples + (size_t)p * B.hcap * SREC;
    const int total = B.rawcap / 2;
    int v = 0, pos = 0;
    while (v < H) {
        const int D = min(SWIN, total - pos);
        if (D <= 0) break;
        for (int d = t; d < D; d += blockDim.x) {
            const uint2 w = *reinterpret_cast<const uint2*>(raw + 2 * (size_t)(pos + d));
            const uint32_t a = (w.x >> 1) % (uint32_t)ng, b = (w.y >> 1) % (uint32_t)ng;
            L.mval[d] = (uint16_t)(a > b ? b : a);
        }
        __syncthreads();
        for (int d = t; d < D; d += blockDim.x) L.len[d] = (uint16_t)sample_len(L.mval, d, D, S);
        __syncthreads();
        if (t < 64) chase_window(t, L, D, S, H - v);
        __syncthreads();
        const int nv = L.nv, e = L.e;
        for (int i = t; i < nv; i += blockDim.x) {
            const int d = L.posv[i];
            const int ln = L.len[d];
            int ids[MAX_SAMPLE];
            sample_ids(L.mval, d, D, S, ln, ids);
            write_rec(rec + (size_t)(v + i) * SREC, S, ids, pos + d + ln);
        }
        __syncthreads();
        const bool last = pos + D >= total;
        v += nv;
        pos += e;
        if (last && v < H) break;
    }
    if (v < H && t == 0) {
        // serial continuation from the generator state after 2*pos words
        ring_at(raw, B.st + p, 2 * pos, R);
        for (; v < H; v++) {
            int ids[MAX_SAMPLE];
            int used = 0;
            const int cnt = draw_one(R, ng, S, ids, used);
            pos += used;
            write_rec(rec + (size_t)v * SREC, cnt, ids, pos);
        }
    }
}


__global__ void __launch_bounds__(256) k_ransac_prep(RansacBufs B, RansacCfg cfg) {
    __builtin_amdgcn_s_setprio(ODO_WAVE_PRIO);  // latency-bound: issue ahead of co-resident extraction waves
    const int p = blockIdx.x;
    const int t = threadIdx.x;
    RState* S = B.st + p;
    odo_pair_result* R = B.res + p;
    float* T12o = B.T12 + (size_t)p * 16;
    const int ng = B.n_good[p];
    const int nm = B.n_matches[p];
    const int Ssz = min(max(cfg.sample_size, 1), MAX_SAMPLE);
    const int H = cfg.iterations;
    bool active = B.pair_valid[p] && nm >= B.min_matches && nm >= cfg.min_inlier_th;
    __shared__ int s_efast_ok;
    if (t == 0) {
        R->rmse = 1e6f;
        R->n_good = active ? ng : 0;
        R->n_inliers = 0;
        R->ransac_ok = 0;
        R->visited = 0;
        R->n_sweeps = 0;
        R->n_fit_points = 0;
        for (int i = 0; i < 16; i++) R->T12[i] = T12o[i] = (i % 5 == 0) ? 1.f : 0.f;
    }
    active = active && ng >= cfg.min_inlier_th;
    const int words = (ng + 31) >> 5;
    const bool done = !active || H <= 0 || ng < Ssz;
    if (active) {
        const SortElR* G = B.good + (size_t)p * B.match_cap;
        const odo_dmatch* M = B.matches + (size_t)p * B.match_cap;
        const float* X1 = B.xyz + (size_t)(B.slot0 + p) * B.kp_cap * 3;
        const float* X2 = B.xyz + (size_t)(B.slot0 + p + 1) * B.kp_cap * 3;
        GoodPt* P = B.gpts + (size_t)p * B.match_cap;
        bool zok = true;  // ErrorFunction2's fast form (ef_fast_pt)
        for (int k = t; k < ng; k += 256) {
            // defensive: an index outside the match list (never produced by a
            // correct sort) yields an excluded NaN point instead of a stray read
            const uint32_t gi = G[k].val;
            const odo_dmatch m = gi < (uint32_t)nm ? M[gi] : odo_dmatch{0, 0, 0, __builtin_nanf("")};
            if (gi >= (uint32_t)nm) {
                P[k] = GoodPt{0.f, 0.f, __builtin_nanf(""), 0.f, 0.f, __builtin_nanf(""), 0.f, 0.f};
                continue;
            }
            GoodPt g;
            g.sx = X1[3 * m.queryIdx];
            g.sy = X1[3 * m.queryIdx + 1];
            g.sz = X1[3 * m.queryIdx + 2];
            g.tx = X2[3 * m.trainIdx];
            g.ty = X2[3 * m.trainIdx + 1];
            g.tz = X2[3 * m.trainIdx + 2];
            g.w = 1.0f / (g.sz * g.tz);  // ransac.cpp:305
            g.pad = 0.f;
            P[k] = g;
            zok = zok && ef_fast_pt(g.sz, g.tx, g.sz, g.tz);
            // the TFC weights (tfc_div's range): every point the TFC adds
            if (!__builtin_isnan(g.sz) && !__builtin_isnan(g.tz) && g.w != 0.0f)  // tfc_point_ok
                zok = zok && g.w >= 0x1p-20f && g.w <= 0x1p20f;
        }
        s_efast_ok = 1;
        __syncthreads();
        if (!zok) s_efast_ok = 0;  // benign race: every writer stores 0
        uint32_t* BM = B.best_mask + (size_t)p * B.mask_words;
        for (int w = t; w < words; w += 256) BM[w] = 0;
        if (!done) {
            int* rd = B.ready + (size_t)p * B.hcap;
            for (int h = t; h < H; h += 256) rd[h] = 0;
        }
    }
    __syncthreads();
    if (t == 0) {
        S->efast = active && EF_FAST == 2 && s_efast_ok;
        S->active = active ? 1 : 0;
        S->ng = ng;
        S->S = Ssz;
        S->words = words;
        S->H = H;
        S->done = done ? 1 : 0;
        S->lock = 0;
        S->fold_pos = 0;
        S->n = 0;
        S->visited = 0;
        S->valid = 0;
        S->best_cnt = 0;
        S->best_h = -1;
        S->rmse = 1e6f;
        S->sweeps = 0;
        S->fitpts = 0;
        S->nexth = cfg.h0;  // the first eval launch covers [0, h0)
    }
    if (done) return;
    __shared__ SampWin s_win;
    __shared__ Rng s_rng;
    pair_samples(B, p, ng, Ssz, H, s_win, s_rng);
}

// ---------------------------------------------------------------- eval
#define EV_WAVES EV_WAVES_C

struct EvalLds {
    uint32_t cur[256];  // current inlier set (refined), bit k = good match k
    uint32_t nw[256];   // set produced by the sweep
    double dv[64];      // compacted Mahalanobis terms of one sweep chunk
};

// TFC input slab of one wave (dynamic LDS after the good-point cache): the
// current set's points compacted in set order, SoA rows sx sy sz tx ty tz
// w->alpha acc->(1-alpha); up to TFC_CAP points per fold pass.
#ifndef TFC_CAP
#define TFC_CAP 256  // 256 vs 512: +1.4% frames/s (less LDS per eval workgroup)
#endif
struct TfcSlab {
    float* v;  // 8 rows of TFC_CAP floats
    ODO_INLINE float* row(int r) const { return v + r * TFC_CAP; }
};

ODO_INLINE bool tfc_point_ok(const GoodPt& g) {
    return !__builtin_isnan(g.sz) && !__builtin_isnan(g.tz) && g.w != 0.0f;  // ransac.cpp:303, TFC::add
}

ODO_INLINE void stage_pt(const TfcSlab& L, int q, const GoodPt& g) {
    L.row(0)[q] = g.sx;
    L.row(1)[q] = g.sy;
    L.row(2)[q] = g.sz;
    L.row(3)[q] = g.tx;
    L.row(4)[q] = g.ty;
    L.row(5)[q] = g.tz;
    L.row(6)[q] = g.w;
}

ODO_INLINE uint32_t lane_rank(uint64_t bal) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
}

// PCL TransformationFromCorrespondences::add over the slab's n points,
// bit-identical to the serial add(): lane 0 runs the accumulated-weight
// prefix, all lanes form alpha = w/acc in parallel, then lane (i,j) < 9 runs
// three independent chains per point - m1[j], m2[i] (recomputed redundantly,
// same operations) and cov[i][j] - so the wave issues them interleaved
// instead of waiting on one dependent chain. Chains carry over passes.
ODO_INLINE void tfc_fold(const TfcSlab& L, int nin, int lane, float& acc, float& m1, float& m2, float& c,
                         uint64_t* tp = nullptr) {
    if (nin <= 0) return;
#ifdef ODO_RANSAC_PROFILE
    uint64_t q = wall_clock64();
#define TP(i) if (tp) { const uint64_t n_ = wall_clock64(); tp[i] += n_ - q; q = n_; }
#else
#define TP(i)
#endif
    if (lane == 0) {
        float a = acc;
        const float* W = L.row(6);
        float* A = L.row(7);
        for (int q0 = 0; q0 < nin; q0 += 16) {
            float wv[16];
#pragma unroll
            for (int u = 0; u < 16; u += 4) {
                const float4 v = *reinterpret_cast<const float4*>(W + q0 + u);
                wv[u] = v.x;
                wv[u + 1] = v.y;
                wv[u + 2] = v.z;
                wv[u + 3] = v.w;
            }
            if (q0 + 16 <= nin) {
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    a += wv[u];
                    A[q0 + u] = a;
                }
            } else {
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    a = (q0 + u < nin) ? a + wv[u] : a;
                    A[q0 + u] = a;
                }
            }
        }
        acc = a;
    }
    wave_sync();
    TP(0)
    for (int k = lane; k < nin; k += 64) {
        const float al = L.row(6)[k] / L.row(7)[k];
        L.row(6)[k] = al;
        L.row(7)[k] = 1.0f - al;
    }
    wave_sync();
    TP(1)
    if (lane < 9) {
        const int i = lane / 3, j = lane - 3 * (lane / 3);
        const float* s1 = L.row(j);
        const float* s2 = L.row(3 + i);
        const float* sa = L.row(6);
        const float* so = L.row(7);
        float a1 = m1, a2 = m2, cc = c;
        for (int q0 = 0; q0 < nin; q0 += 16) {
            float P1[16], P2[16], AL[16], OM[16];
#pragma unroll
            for (int u = 0; u < 16; u += 4) {
                const float4 a = *reinterpret_cast<const float4*>(s1 + q0 + u);
                const float4 b = *reinterpret_cast<const float4*>(s2 + q0 + u);
                const float4 e = *reinterpret_cast<const float4*>(sa + q0 + u);
                const float4 o = *reinterpret_cast<const float4*>(so + q0 + u);
                P1[u] = a.x, P1[u + 1] = a.y, P1[u + 2] = a.z, P1[u + 3] = a.w;
                P2[u] = b.x, P2[u + 1] = b.y, P2[u + 2] = b.z, P2[u + 3] = b.w;
                AL[u] = e.x, AL[u + 1] = e.y, AL[u + 2] = e.z, AL[u + 3] = e.w;
                OM[u] = o.x, OM[u + 1] = o.y, OM[u + 2] = o.z, OM[u + 3] = o.w;
            }
            if (q0 + 16 <= nin) {
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const float d1 = P1[u] - a1;
                    const float d2 = P2[u] - a2;
                    const float ad2 = AL[u] * d2;
                    cc = OM[u] * (cc + ad2 * d1);
                    a1 = a1 + AL[u] * d1;
                    a2 = a2 + ad2;
                }
            } else {
#pragma unroll
                for (int u = 0; u < 16; u++) {
                    const bool on = q0 + u < nin;
                    const float d1 = P1[u] - a1;
                    const float d2 = P2[u] - a2;
                    const float ad2 = AL[u] * d2;
                    cc = on ? OM[u] * (cc + ad2 * d1) : cc;
                    a1 = on ? a1 + AL[u] * d1 : a1;
                    a2 = on ? a2 + ad2 : a2;
                }
            }
        }
        m1 = a1;
        m2 = a2;
        c = cc;
    }
    wave_sync();
    TP(2)
#undef TP
}

// Ordered sum of dv[0..nin) (lane 0), 16 loads ahead.
ODO_INLINE double fold_dv(const EvalLds& L, int nin, double s) {
    for (int q0 = 0; q0 < nin; q0 += 16) {
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; u++) v[u] = L.dv[q0 + u];
        if (q0 + 16 <= nin) {
#pragma unroll
            for (int u = 0; u < 16; u++) s += v[u];
        } else {
#pragma unroll
            for (int u = 0; u < 16; u++) s = (q0 + u < nin) ? s + v[u] : s;
        }
    }
    return s;
}


// The pair's good-match table is staged in LDS (shared by the workgroup's
// waves) when it fits; every refinement sweeps it twice.
#ifndef PCACHE
#define PCACHE 0
#endif
// dynamic LDS of k_ransac_eval: good-point cache + one TFC slab per wave
#define EV_LDS (PCACHE * sizeof(GoodPt) + (size_t)EV_WAVES * 8 * TFC_CAP * sizeof(float))
extern __shared__ __align__(16) uint8_t ev_dyn[];

template <bool CACHED>
ODO_INLINE GoodPt load_pt(const GoodPt* P, int k) {
    if (CACHED) return reinterpret_cast<const GoodPt*>(ev_dyn)[k];
    return P[k];
}

#ifdef ODO_RANSAC_PROFILE
#define RPROF_MAX 4096
__device__ uint64_t g_rprof[RPROF_MAX * 8];
__device__ uint64_t g_rprof_done;
#endif

// Ordered fold of finished hypotheses (ransac.cpp:233-249), lane 0 only.
// Whoever completes the visited prefix folds it; a wave that finds the lock
// taken leaves, the holder re-checks after releasing it.
ODO_INLINE void try_fold(const RansacBufs& B, const RansacCfg& cfg, int p) {
    RState* S = B.st + p;
    int* ready = B.ready + (size_t)p * B.hcap;
    const HypRes* hyp = B.hyp + (size_t)p * B.hcap;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    while (true) {
        if (atomicCAS(&S->lock, 0, 1) != 0) return;
        __threadfence();
        const int H = S->H, ng = S->ng;
        int pos = ld_relaxed(&S->fold_pos), n = ld_relaxed(&S->n), visited = ld_relaxed(&S->visited);
        int valid = ld_relaxed(&S->valid), best = ld_relaxed(&S->best_cnt), best_h = ld_relaxed(&S->best_h);
        float rmse = __int_as_float(ld_relaxed(reinterpret_cast<const int*>(&S->rmse)));
        int sweeps = ld_relaxed(&S->sweeps), fitpts = ld_relaxed(&S->fitpts);
        bool fin = n >= H;
        while (!fin && pos < H) {
            if (!__hip_atomic_load(&ready[pos], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) break;
            const unsigned rc = (unsigned)ld_relaxed(&hyp[pos].cnt);
            const double re = __longlong_as_double(__hip_atomic_load(
                reinterpret_cast<const long long*>(&hyp[pos].err), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            visited++;
            const int work = ld_relaxed(&hyp[pos].pad);
            sweeps += work & 31;
            fitpts += work >> 5;
            bool brk = false;
            if (rc > 0) {
                valid++;
                if (re <= (double)rmse && rc >= (unsigned)best && rc >= minInl) {
                    rmse = (float)re;
                    best = (int)rc;
                    best_h = pos;
                    if (rc > ng * 0.5) n += 10;
                    if (rc > ng * 0.75) n += 10;
                    if (rc > ng * 0.8) brk = true;
                }
            }
            n++;
            if (brk) n = H;
            pos++;
            fin = n >= H;
        }
        st_relaxed(&S->fold_pos, pos);
        st_relaxed(&S->n, n);
        st_relaxed(&S->visited, visited);
        st_relaxed(&S->sweeps, sweeps);
        st_relaxed(&S->fitpts, fitpts);
        st_relaxed(&S->valid, valid);
        st_relaxed(&S->best_cnt, best);
        st_relaxed(&S->best_h, best_h);
        st_relaxed(reinterpret_cast<int*>(&S->rmse), __float_as_int(rmse));
        if (fin) st_relaxed(&S->done, 1);
#ifdef ODO_RANSAC_PROFILE
        if (fin) g_rprof_done = wall_clock64();
#endif
        __threadfence();
        atomicExch(&S->lock, 0);
        __threadfence();
        if (fin) return;
        if (!__hip_atomic_load(&ready[pos], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
}

// The same fold run by a whole wave (uniform control flow): the ready flags
// and results of the next 64 hypotheses are loaded at once, one vector load
// each, and the serial fold steps over the ready run read them with
// v_readlane — instead of four dependent coherent loads per hypothesis (a
// visited-to-the-end pair folds 500 of them: 215 us of serial loads at ~0.43
// us each, longer than every hypothesis' evaluation). A holder re-checks the
// next ready flag after releasing the lock; a finisher whose flag it still
// missed leaves the rest to k_ransac_final, which completes the fold.
ODO_INLINE int rdl(int v, int i) { return __builtin_amdgcn_readlane(v, i); }
ODO_INLINE void try_fold_wave(const RansacBufs& B, const RansacCfg& cfg, int p, int lane) {
    RState* S = B.st + p;
    int* ready = B.ready + (size_t)p * B.hcap;
    const HypRes* hyp = B.hyp + (size_t)p * B.hcap;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    while (true) {
        int got = 0;
        if (lane == 0) got = atomicCAS(&S->lock, 0, 1) == 0;
        if (!__builtin_amdgcn_readfirstlane(got)) return;
        __threadfence();
        const int H = __builtin_amdgcn_readfirstlane(S->H), ng = __builtin_amdgcn_readfirstlane(S->ng);
        int pos = __builtin_amdgcn_readfirstlane(ld_relaxed(&S->fold_pos));
        int n = __builtin_amdgcn_readfirstlane(ld_relaxed(&S->n));
        int visited = __builtin_amdgcn_readfirstlane(ld_relaxed(&S->visited));
        int valid = __builtin_amdgcn_readfirstlane(ld_relaxed(&S->valid));
        int best = __builtin_amdgcn_readfirstlane(ld_relaxed(&S->best_cnt));
        int best_h = __builtin_amdgcn_readfirstlane(ld_relaxed(&S->best_h));
        float rmse = __int_as_float(__builtin_amdgcn_readfirstlane(ld_relaxed(reinterpret_cast<const int*>(&S->rmse))));
        int sweeps = __builtin_amdgcn_readfirstlane(ld_relaxed(&S->sweeps));
        int fitpts = __builtin_amdgcn_readfirstlane(ld_relaxed(&S->fitpts));
        bool fin = n >= H;
        while (!fin && pos < H) {
            const int q = pos + lane;
            int rd = 0;
            if (q < H) rd = __hip_atomic_load(&ready[q], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            const uint64_t stop = __ballot(rd == 0);
            const int m = stop ? (int)__builtin_ctzll(stop) : 64;  // ready run from pos
            if (m == 0) break;
            int rc = 0, work = 0, elo = 0, ehi = 0;
            if (lane < m) {
                rc = ld_relaxed(&hyp[q].cnt);
                const long long e = __hip_atomic_load(reinterpret_cast<const long long*>(&hyp[q].err), __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
                elo = (int)(uint32_t)e;
                ehi = (int)(uint32_t)((unsigned long long)e >> 32);
                work = ld_relaxed(&hyp[q].pad);
            }
            // Only a hypothesis that beats the state at the run's start can
            // be accepted (rmse only falls, best only grows along the run), so
            // the serial steps visit those candidates alone; the entries
            // between them just count (n++), and n crossing H ends the fold
            // at the crossing entry.
            uint64_t cand = __ballot(lane < m && rc > 0 && __hiloint2double(ehi, elo) <= (double)rmse &&
                                     (unsigned)rc >= (unsigned)best && (unsigned)rc >= minInl);
            int i = 0;  // entries of this run folded so far
            while (i < m && !fin) {
                const int c = cand ? (int)__builtin_ctzll(cand) : m;  // next candidate (or the run's end)
                if (c - i >= H - n) {  // n reaches H before the candidate
                    i += H - n;
                    n = H;
                    fin = true;
                    break;
                }
                n += c - i;
                i = c;
                if (c == m) break;
                cand &= cand - 1;
                const unsigned rci = (unsigned)rdl(rc, c);
                const double re = __hiloint2double(rdl(ehi, c), rdl(elo, c));
                bool brk = false;
                if (re <= (double)rmse && rci >= (unsigned)best) {  // rci >= minInl and > 0 already
                    rmse = (float)re;
                    best = (int)rci;
                    best_h = pos + c;
                    if (rci > ng * 0.5) n += 10;
                    if (rci > ng * 0.75) n += 10;
                    if (rci > ng * 0.8) brk = true;
                }
                n++;
                i++;
                if (brk) n = H;
                fin = n >= H;
            }
            // the folded entries' counters, summed over the wave
            const bool in = lane < i;
            visited += i;
            valid += __popcll(__ballot(in && rc > 0));
            int sw = in ? (work & 31) : 0, fp = in ? (work >> 5) : 0;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) {
                sw += __shfl_xor(sw, o);
                fp += __shfl_xor(fp, o);
            }
            sweeps += __builtin_amdgcn_readfirstlane(sw);
            fitpts += __builtin_amdgcn_readfirstlane(fp);
            pos += i;
            if (m < 64) break;
        }
        if (lane == 0) {
            st_relaxed(&S->fold_pos, pos);
            st_relaxed(&S->n, n);
            st_relaxed(&S->visited, visited);
            st_relaxed(&S->sweeps, sweeps);
            st_relaxed(&S->fitpts, fitpts);
            st_relaxed(&S->valid, valid);
            st_relaxed(&S->best_cnt, best);
            st_relaxed(&S->best_h, best_h);
            st_relaxed(reinterpret_cast<int*>(&S->rmse), __float_as_int(rmse));
            if (fin) st_relaxed(&S->done, 1);
#ifdef ODO_RANSAC_PROFILE
            if (fin) g_rprof_done = wall_clock64();
#endif
            __threadfence();
            atomicExch(&S->lock, 0);
            __threadfence();
        }
        if (fin) return;
        int rd = 0;
        if (lane == 0) rd = __hip_atomic_load(&ready[pos], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (!__builtin_amdgcn_readfirstlane(rd)) return;
    }
}

#ifndef EV_EFAST
#define EV_EFAST 1  // the evaluation kernels take the fast ErrorFunction2 form for guarded pairs
#endif
#ifndef EV_Z
#define EV_Z 1  // ... and the per-hypothesis covariance products (hyp_cov_terms)
#endif
template <bool CACHED>
ODO_INLINE void eval_hyps(const RansacBufs& B, const RansacCfg& cfg, int p, int wave, int lane, EvalLds& L,
                          const GoodPt* P, int ng, int words, int H, int hofs, int y0, int hlim, int yrow,
                          int ystride) {
    RState* S = B.st + p;
    const int* smp0 = B.samples + (size_t)p * B.hcap * SREC;
    const TfcSlab TS{reinterpret_cast<float*>(ev_dyn + PCACHE * sizeof(GoodPt)) + (size_t)wave * 8 * TFC_CAP};
    MahalConst K;
    K.raster_cov_x = cfg.raster_cov_x;
    K.raster_cov_y = cfg.raster_cov_y;
    K.depth_cov = *B.latch;
    const float th = cfg.max_mahal * cfg.max_mahal;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    // the pair's points passed k_ransac_prep's range guard (RState.efast):
    // ErrorFunction2's fast form, the same bits (odo_device.h); wave-uniform
    const bool efast = EV_EFAST && EF_FAST == 2 && __builtin_amdgcn_readfirstlane(S->efast) && ef_fast_cov(K);
    // this launch's waves stride over hypotheses [hofs + y0*EV_WAVES, hlim)
    const int hend = min(H, hlim);
    for (int h = hofs + (y0 + yrow) * EV_WAVES + wave; h < hend; h += ystride * EV_WAVES) {
        if (h < B.h_lo || h >= B.h_hi) continue;  // hypotheses mode: another rank's range
        const int* smp = smp0 + (size_t)h * SREC;
        double refinedError = 1e6;
        unsigned refinedCnt = 0;
        float refinedT[12];
        for (int i = 0; i < 12; i++) refinedT[i] = (i % 5 == 0) ? 1.f : 0.f;
        bool useSample = true, aborted = false;
        int nsweep = 0, nfit = 0;  // algorithmic work of this hypothesis
#ifdef ODO_RANSAC_PROFILE
        // -DODO_RANSAC_PROFILE: per-hypothesis phase times (10 ns ticks) via printf
        uint64_t t_tfc = 0, t_get = 0, t_sweep = 0, t0 = 0, t_start = wall_clock64();
        uint64_t tpp[3] = {0, 0, 0};
        int nref = 0, npass = 0;
#define TPP (npass++, tpp)
#define RP_T0() t0 = wall_clock64()
#define RP_ACC(x) x += wall_clock64() - t0
#else
#define RP_T0()
#define RP_ACC(x)
#define TPP nullptr
#endif
        for (int refinements = 1; refinements < 20; refinements++) {
            // ---- GetTransformFromMatches (ransac.cpp:295-313), in set order
            float tacc = 0.f, tm1 = 0.f, tm2 = 0.f, tc = 0.f;
            RP_T0();
            if (useSample) {
                const int ns = smp[0];
                bool in = false;
                GoodPt g;
                if (lane < ns) {
                    g = load_pt<CACHED>(P, smp[1 + lane]);
                    in = tfc_point_ok(g);
                }
                const uint64_t bal = __ballot(in);
                if (in) stage_pt(TS, lane_rank(bal), g);
                wave_sync();
                nfit += __popcll(bal);
                tfc_fold(TS, __popcll(bal), lane, tacc, tm1, tm2, tc, TPP);
            } else {
                // the whole set compacted into the slab in set order, folded
                // once per TFC_CAP points (no per-chunk fold overhead)
                int nfill = 0;
                for (int c0 = 0; c0 < ng; c0 += 64) {
                    const int k = c0 + lane;
                    bool in = false;
                    GoodPt g;
                    if (k < ng && ((L.cur[k >> 5] >> (k & 31)) & 1)) {
                        g = load_pt<CACHED>(P, k);
                        in = tfc_point_ok(g);
                    }
                    const uint64_t bal = __ballot(in);
                    const int cnt = __popcll(bal);
                    nfit += cnt;
                    if (nfill + cnt > TFC_CAP) {
                        wave_sync();
                        tfc_fold(TS, nfill, lane, tacc, tm1, tm2, tc, TPP);
                        nfill = 0;
                    }
                    if (in) stage_pt(TS, nfill + lane_rank(bal), g);
                    nfill += cnt;
                }
                wave_sync();
                tfc_fold(TS, nfill, lane, tacc, tm1, tm2, tc, TPP);
            }
            RP_ACC(t_tfc);
            RP_T0();
            TFC tf;
            tf.accW = __shfl(tacc, 0);
#pragma unroll
            for (int i = 0; i < 3; i++) {
                tf.m1[i] = __shfl(tm1, i);
                tf.m2[i] = __shfl(tm2, 3 * i);
#pragma unroll
                for (int j = 0; j < 3; j++) tf.cov[i][j] = __shfl(tc, 3 * i + j);
            }
            float T[12];
            tf.get(T);
            double Td[12];
#pragma unroll
            for (int i = 0; i < 12; i++) Td[i] = (double)T[i];
            double Zd[6];  // the covariance's point-independent products, once per sweep
            if (EV_Z) hyp_cov_terms(Td, K, Zd);
            RP_ACC(t_get);
            RP_T0();
            // poll the fold's stop flag once per refinement: issued here, read
            // after the sweep (one memory-coherent load per wave per refinement;
            // polling per chunk hot-spots the flag's line)
            const int dn = ld_relaxed(&S->done);
            // ---- ComputeInliersAndError (ransac.cpp:315-348)
            double meanError = 0.0;
            unsigned cnt = 0;
            for (int c0 = 0; c0 < ng; c0 += 64) {
                const int k = c0 + lane;
                bool in = false;
                double d = 0.0;
                if (k < ng) {
                    const GoodPt g = load_pt<CACHED>(P, k);
                    if (!(g.sz == 0.0f || g.tx == 0.0f)) {
                        const float x1[3] = {g.sx, g.sy, g.sz}, x2[3] = {g.tx, g.ty, g.tz};
                        d = error_function2_mk(x1, x2, Td, K, EV_Z ? Zd : nullptr, efast);
                        in = !(d > th) && (d >= 0.0);
                    }
                }
                const uint64_t bal = __ballot(in);
                if (in) L.dv[lane_rank(bal)] = d;
                if (lane == 0) {
                    L.nw[c0 >> 5] = (uint32_t)bal;
                    if (c0 + 32 < ng) L.nw[(c0 >> 5) + 1] = (uint32_t)(bal >> 32);
                }
                wave_sync();
                const int nin = __popcll(bal);
                if (lane == 0) meanError = fold_dv(L, nin, meanError);
                cnt += (unsigned)nin;
                wave_sync();
            }
            meanError = __shfl(meanError, 0);
            RP_ACC(t_sweep);
            // the fold already stopped before this hypothesis: nothing will read it
            if (__builtin_amdgcn_readfirstlane(dn)) {
                aborted = true;
                break;
            }
            nsweep++;
#ifdef ODO_RANSAC_PROFILE
            nref++;
#endif
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
                for (int w = lane; w < words; w += 64) L.cur[w] = L.nw[w];
                wave_sync();
                useSample = false;
                if (cnt == prev) break;
            } else break;
        }
#ifdef ODO_RANSAC_PROFILE
        // per-hypothesis record in g_rprof (read by odo_ransac_prof_read; a
        // device printf stalls co-resident waves and delays the fold)
        if (lane == 0 && h < RPROF_MAX) {
            uint64_t* r = g_rprof + (size_t)h * 8;
            r[0] = t_start;
            r[1] = wall_clock64();
            r[2] = (uint64_t)nref | ((uint64_t)aborted << 8) | ((uint64_t)refinedCnt << 16) | ((uint64_t)ng << 40);
            r[3] = t_tfc;
            r[4] = t_get;
            r[5] = t_sweep;
            r[6] = (uint64_t)npass;
            r[7] = 0;
        }
#endif
        if (aborted) continue;
        HypRes* hr = B.hyp + (size_t)p * B.hcap + h;
        if (lane == 0) {
            hr->err = refinedError;
            hr->cnt = (int)refinedCnt;
            hr->pad = nsweep | (nfit << 5);
        }
        if (lane < 12) {
            float v = refinedT[0];
#pragma unroll
            for (int i = 1; i < 12; i++)
                if (lane == i) v = refinedT[i];
            hr->T[lane] = v;
        }
        uint32_t* mo = B.masks + ((size_t)p * B.hcap + h) * B.mask_words;
        if (refinedCnt > 0)
            for (int w = lane; w < words; w += 64) mo[w] = L.cur[w];
        __threadfence();
        // a lone pair folds with the whole wave (its fold is on the latency
        // path: 500 visited hypotheses cost ~100 us of serial lane-0 loads);
        // batches keep the lane-0 fold (the wave form measured 2.3 % slower
        // there, where folds are short and overlap the extraction)
        if (cfg.fold_wave) {
            if (lane == 0)
                __hip_atomic_store(B.ready + (size_t)p * B.hcap + h, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if (!B.no_fold) try_fold_wave(B, cfg, p, lane);
        } else if (lane == 0) {
            __hip_atomic_store(B.ready + (size_t)p * B.hcap + h, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if (!B.no_fold) try_fold(B, cfg, p);
        }
        wave_sync();
#ifdef ODO_RANSAC_PROFILE
        if (lane == 0 && h < RPROF_MAX) g_rprof[(size_t)h * 8 + 7] = wall_clock64();  // after ready + fold
#endif
    }
}

#ifndef EV_MIN_BLOCKS
#define EV_MIN_BLOCKS 2
#endif
__global__ void __launch_bounds__(64 * EV_WAVES, EV_MIN_BLOCKS) k_ransac_eval(RansacBufs B, RansacCfg cfg, int hofs, int y0,
                                                                                  int hlim) {
    __builtin_amdgcn_s_setprio(ODO_WAVE_PRIO);  // latency-bound: issue ahead of co-resident extraction waves
    const int p = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ EvalLds s_w[EV_WAVES];
    RState* S = B.st + p;
    const int H = S->H;
    if (hofs + (y0 + (int)blockIdx.y) * EV_WAVES >= min(H, hlim)) return;
    __shared__ int s_done;
    if (threadIdx.x == 0) s_done = ld_relaxed(&S->done);
    __syncthreads();
    if (s_done) return;  // uniform over the workgroup
    const int ng = S->ng, words = S->words;
    const GoodPt* P = B.gpts + (size_t)p * B.match_cap;
    if (PCACHE > 0 && ng <= PCACHE) {
        GoodPt* pc = reinterpret_cast<GoodPt*>(ev_dyn);
        for (int k = threadIdx.x; k < ng; k += blockDim.x) pc[k] = P[k];
        __syncthreads();
        eval_hyps<true>(B, cfg, p, wave, lane, s_w[wave], P, ng, words, H, hofs, y0, hlim, blockIdx.y, gridDim.y);
    } else {
        eval_hyps<false>(B, cfg, p, wave, lane, s_w[wave], P, ng, words, H, hofs, y0, hlim, blockIdx.y, gridDim.y);
    }
}

// The pairs still folding after the first launch, in pair order, and a work
// counter for the second launch (one workgroup).
__global__ void __launch_bounds__(256) k_ransac_open(RansacBufs B, int npairs) {
    __shared__ int s_base, s_fast;
    if (threadIdx.x == 0) s_base = 0, s_fast = 1;
    __syncthreads();
    for (int p0 = 0; p0 < npairs; p0 += 256) {
        const int p = p0 + (int)threadIdx.x;
        const bool open = p < npairs && !ld_relaxed(&B.st[p].done);
        if (open && !B.st[p].efast) s_fast = 0;  // benign race: every writer stores 0
        const uint64_t bal = __ballot(open);
        __shared__ int s_cnt[4];
        if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = __popcll(bal);
        __syncthreads();
        int before = 0, tot = 0;
        for (int w = 0; w < 4; w++) {
            if (w < (int)(threadIdx.x >> 6)) before += s_cnt[w];
            tot += s_cnt[w];
        }
        if (open) B.open_list[s_base + before + (int)lane_rank(bal)] = p;
        __syncthreads();
        if (threadIdx.x == 0) s_base += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        B.open_cnt[0] = s_base;
        B.open_cnt[1] = 0;  // work counter
        B.open_cnt[2] = s_fast;  // every open pair passed the fast-form guard (k_ransac_lanes)
    }
}

// Second launch as a work list: a fixed grid of workgroups takes (row, open
// pair) items in row-major order (lower hypotheses first) from an atomic
// counter, 4 hypotheses per item - no launch-sized crowd of early-exit
// workgroups for the pairs that already broke.
__global__ void __launch_bounds__(64 * EV_WAVES, EV_MIN_BLOCKS) k_ransac_eval_list(RansacBufs B, RansacCfg cfg, int hofs,
                                                                                   int rows, int max_open) {
    __builtin_amdgcn_s_setprio(ODO_WAVE_PRIO);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    __shared__ EvalLds s_w[EV_WAVES];
    __shared__ int s_item;
    const int cnt = B.open_cnt[0];
    if (cnt > max_open) return;  // many open pairs: k_ransac_lanes takes them
    const int total = cnt * rows;
    while (true) {
        __syncthreads();
        if (threadIdx.x == 0) s_item = atomicAdd(&B.open_cnt[1], 1);
        __syncthreads();
        const int item = s_item;
        if (item >= total) break;
        const int row = item / cnt, p = B.open_list[item - row * cnt];
        RState* S = B.st + p;
        const int H = S->H;
        if (hofs + row * EV_WAVES >= H || ld_relaxed(&S->done)) continue;  // uniform per item
        const GoodPt* P = B.gpts + (size_t)p * B.match_cap;
        eval_hyps<false>(B, cfg, p, wave, lane, s_w[wave], P, S->ng, S->words, H, hofs, row,
                         hofs + (row + 1) * EV_WAVES, 0, 1);
    }
}

// ---------------------------------------------------------------- lanes
// The hypotheses after the first launch, one per LANE (the throughput form;
// k_ransac_eval keeps one per wave for the latency of the first rows).
// Ransac::Iterate's inner loop (ransac.cpp:201-231) is sequential per
// hypothesis: PCL's TFC recurrence over the inlier set in set order, then
// ComputeInliersAndError's ordered double sum. With a hypothesis per lane both
// run in their natural order in that lane, with no cross-lane folds, and the
// wave-uniform good points (one 32-B record per step) are shared by all 64
// lanes. A round is one refinement of every lane's hypothesis: pass A (the TFC
// over the lane's current inlier set; a fresh hypothesis fits its minimal
// sample instead), the SVD, pass B (the Mahalanobis sweep over all good
// points: new inlier set, mean error). A lane whose hypothesis ends writes its
// result, marks it ready, runs the ordered fold and takes the next hypothesis
// of the pair from the pair's counter, so lanes never idle while the pair has
// hypotheses left. Inlier sets live in a per-wave global slab ([2][words][64],
// coalesced), swapped on accept.
ODO_INLINE double readlane_d(double v, int l) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
#define LN_WAVES 4
#define LN_RS 33  // LDS row stride (doubles) of the parked terms
#ifndef LN_TFAST
#define LN_TFAST 1  // the fast-form launch also takes the TFC division's fast form (tfc_div)
#endif
#ifndef LN_TD
// 1: the active slots' transforms parked in LDS as doubles, with their
// point-independent covariance terms (hyp_cov_terms), so the sweep's
// evaluations read them instead of converting twelve floats and forming six
// products each time (the same values: the conversions are exact and Z's
// products are the ones error_function2_mk forms without it)
#define LN_TD 1
#endif
// LDS words per slot: 12 + 6 doubles (1), 12 doubles without the covariance
// terms (2), or 12 floats (0)
#define LN_TW (LN_TD == 1 ? 18 : 12)
#ifndef LN_SLOTS
#define LN_SLOTS 32  // lanes per wave that take up hypotheses (rows of parked terms per wave)
#endif
#ifndef LN_PRIO
#define LN_PRIO ODO_WAVE_PRIO  // k_ransac_lanes' wave priority
#endif
#ifndef LN_BAL_EXP
#define LN_BAL_EXP 1  // LN_BAL weight: (good matches + 1) ^ LN_BAL_EXP (1 or 2)
#endif
ODO_INLINE int ln_weight(int ng) { return LN_BAL_EXP == 2 ? ((ng + 1) * (ng + 1) + 63) >> 6 : ng + 1; }
#ifdef ODO_LANES_PROFILE
// -DODO_LANES_PROFILE: per wave of the last k_ransac_lanes launch: start, end,
// loop rounds, sum of active lanes over the rounds, TFC / sweep ticks and the
// sweep's evaluation / ordered-sum parts (10 ns wall-clock ticks; read by
// odo_lanes_prof_read, tools/lanes_probe.py)
#define LPROF_MAX 4096
__device__ uint64_t g_lprof[LPROF_MAX * 10];
#define LP(...) __VA_ARGS__
#else
#define LP(...)
#endif
static_assert(LN_SLOTS <= 64, "a wave's hypothesis slots are its lanes");
// EFAST: every open pair's points passed k_ransac_prep's guard (RState.efast)
// under a latch in ef_fast_cov's range: ErrorFunction2 in its fast form, which
// gives the same bits there (odo_device.h). Two instantiations, chosen once per
// launch, so neither carries the other's registers.
template <bool EFAST>
ODO_INLINE void lanes_body(const RansacBufs& B, const RansacCfg& cfg, uint32_t* lane_slab, int waves_total,
                           int min_open, int lane, int wv, int gw, GoodPt* lp, double* lres, int* la, double* lTd) {
    float* const lT = reinterpret_cast<float*>(lTd);
    const int cnt = B.open_cnt[0];
    if (cnt < min_open || cnt <= 0) return;  // few open pairs: latency matters, k_ransac_eval_list takes them
    uint32_t* slab = lane_slab + (size_t)gw * 2 * B.mask_words * 64;
    MahalConst K;
    K.raster_cov_x = cfg.raster_cov_x;
    K.raster_cov_y = cfg.raster_cov_y;
    K.depth_cov = *B.latch;
    const float th = cfg.max_mahal * cfg.max_mahal;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    // waves_total >= open pairs: several waves per pair share its counter;
    // fewer: each wave walks its pairs in turn
    LP(uint64_t lp_t0 = wall_clock64(); uint64_t lp_rounds = 0, lp_nact = 0, lp_tfc = 0, lp_sweep = 0, lp_fold = 0;
       uint64_t lp_q = 0; int lp_pair = -1; uint64_t lp_inner = 0, lp_sum = 0, lp_p1 = 0, lp_p2 = 0;)
    // open-list slots: gw, gw + waves_total, ... (the pairs this wave owns; a
    // wave leaves a pair once every lane is idle: the pair's counter is
    // exhausted or its fold has stopped)
    int slot = cnt > waves_total ? gw : gw % cnt;
    int lane_lim = LN_SLOTS;  // lanes that take up hypotheses
    // Waves in proportion to the pairs' work: pair i of the open list gets
    // 1 + spare * w_i / sum(w) waves (w = good matches + 1: a sweep and a
    // refinement fit walk them all), and each of its waves takes up to
    // ceil(remaining hypotheses / its waves) at a time. With an even split
    // the pairs with the most matches set the launch's length (their waves
    // carry 64 hypotheses each, the small pairs' finish early).
    if (cnt <= waves_total) {
        const int spare = waves_total - cnt;
        int tot = 0;
        for (int i0 = 0; i0 < cnt; i0 += 64) {
            const int i = i0 + lane;
            tot += i < cnt ? ln_weight(B.st[B.open_list[i]].ng) : 0;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        int carry = 0, mine = -1, wn = 1;
        for (int i0 = 0; i0 < cnt && mine < 0; i0 += 64) {
            const int i = i0 + lane;
            const int w = i < cnt ? ln_weight(B.st[B.open_list[i]].ng) : 0;
            int incl = w;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o);
                if (lane >= o) incl += t;
            }
            const int c0 = carry + incl - w, c1 = carry + incl;
            const int st = i + (int)((long long)spare * c0 / tot), en = i + 1 + (int)((long long)spare * c1 / tot);
            const uint64_t hit = __ballot(i < cnt && st <= gw && gw < en);
            if (hit) {
                const int src = (int)__builtin_ctzll(hit);
                mine = i0 + src;
                wn = __shfl(en - st, src);
            }
            carry += __shfl(incl, 63);
        }
        if (mine >= 0) {
            slot = mine;
            const int rem = max(1, cfg.iterations - cfg.h0);
            lane_lim = min(LN_SLOTS, (rem + wn - 1) / wn);
        }
    }
    for (;;) {
        if (slot < 0) break;
        const int p = __builtin_amdgcn_readfirstlane(B.open_list[slot]);
        RState* S = B.st + p;
        const int H = S->H, ng = S->ng, words = S->words;
        const GoodPt* P = B.gpts + (size_t)p * B.match_cap;
        const int* smp0 = B.samples + (size_t)p * B.hcap * SREC;
        // lane state: hypothesis h (-1 idle), inlier set buffer, refinement bookkeeping
        int h = -1, cur = 0, nref = 0, nsweep = 0, nfit = 0;
        bool sample = false, exhausted = lane >= lane_lim;
        unsigned refinedCnt = 0;
        double refinedError = 1e6;
        float refinedT[12];
        while (true) {
            if (h < 0 && !exhausted) {
                const int nh = atomicAdd(&S->nexth, 1);
                if (nh < H) {
                    h = nh;
                    sample = true;
                    nref = nsweep = nfit = 0;
                    refinedCnt = 0;
                    refinedError = 1e6;
#pragma unroll
                    for (int i = 0; i < 12; i++) refinedT[i] = (i % 5 == 0) ? 1.f : 0.f;
                } else {
                    exhausted = true;
                }
            }
            if (__ballot(h >= 0) == 0) break;
            if (ld_relaxed(&S->done)) break;  // the fold has stopped: nothing will read these
            const bool act = h >= 0;
            LP(lp_rounds++; lp_nact += __popcll(__ballot(act)); lp_pair = p; lp_q = wall_clock64();)
            // ---- GetTransformFromMatches (ransac.cpp:295-313) in set order
            TFC tf;
            tf.reset();
            if (act && sample) {
                const int* smp = smp0 + (size_t)h * SREC;
                const int ns = smp[0];
#pragma unroll
                for (int j = 0; j < MAX_SAMPLE; j++) {
                    if (j < ns) {
                        const GoodPt g = P[smp[1 + j]];
                        if (tfc_point_ok(g)) {
                            tf.add<EFAST && LN_TFAST>(g.sx, g.sy, g.sz, g.tx, g.ty, g.tz, g.w);
                            nfit++;
                        }
                    }
                }
            }
            const bool inset = act && !sample;
            if (__ballot(inset) != 0) {
                const uint32_t* cw = slab + (size_t)cur * B.mask_words * 64;
                // the next 64-point chunk (its points and this lane's two set
                // words) is loaded into registers while this one is folded
                GoodPt gq = lane < ng ? P[lane] : GoodPt{};
                uint32_t q0 = inset ? cw[lane] : 0u, q1 = inset && 32 < ng ? cw[64 + lane] : 0u;
                for (int c0 = 0; c0 < ng; c0 += 64) {
                    wave_sync();  // the previous chunk has been read
                    lp[lane] = gq;
                    wave_sync();
                    const uint32_t b0 = q0, b1 = q1;
                    if (c0 + 64 < ng) {
                        const int c1 = c0 + 64, w1 = c1 >> 5;
                        if (c1 + lane < ng) gq = P[c1 + lane];
                        q0 = inset ? cw[(size_t)w1 * 64 + lane] : 0u;
                        q1 = inset && c1 + 32 < ng ? cw[(size_t)(w1 + 1) * 64 + lane] : 0u;
                    }
                    const int n = min(64, ng - c0);
                    // only the points some lane's set holds (the union of the
                    // chunk's set words over the wave, valid points only: a
                    // point no lane adds changes no lane's state), in order,
                    // four per step: their LDS reads first, the adds
                    // branch-free (the next point's division overlaps)
                    const uint64_t mine = ((uint64_t)b1 << 32) | b0;
                    uint32_t u0 = b0, u1 = b1;
#pragma unroll
                    for (int o = 32; o > 0; o >>= 1) {
                        u0 |= (uint32_t)__shfl_xor((int)u0, o);
                        u1 |= (uint32_t)__shfl_xor((int)u1, o);
                    }
                    uint64_t U = (((uint64_t)u1 << 32) | u0) & __ballot(lane < n && tfc_point_ok(lp[min(lane, n - 1)]));
                    U = ((uint64_t)__builtin_amdgcn_readfirstlane((int)(U >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)U);
                    while (U) {
                        int js[4];
                        bool vj[4];
#pragma unroll
                        for (int t = 0; t < 4; t++) {
                            vj[t] = U != 0;
                            // a step past the union's end re-reads its first
                            // point (in U: finite, so the guarded alpha = 0
                            // no-op of add_sel stays exact)
                            js[t] = vj[t] ? (int)__builtin_ctzll(U) : js[0];
                            U &= U - 1;
                        }
                        GoodPt g4[4];
#pragma unroll
                        for (int t = 0; t < 4; t++) g4[t] = lp[js[t]];
#pragma unroll
                        for (int t = 0; t < 4; t++) {
                            const bool in = vj[t] && ((mine >> js[t]) & 1u);
                            tf.add_sel<EFAST && LN_TFAST>(g4[t].sx, g4[t].sy, g4[t].sz, g4[t].tx, g4[t].ty, g4[t].tz,
                                                          g4[t].w, in);
                            nfit += in;
                        }
                    }
                }
            }
            float T[12];
            tf.get(T);
            LP(lp_tfc += wall_clock64() - lp_q; lp_q = wall_clock64();)
            double Td[12];
#pragma unroll
            for (int i = 0; i < 12; i++) Td[i] = (double)T[i];
            // ---- ComputeInliersAndError (ransac.cpp:315-348): the new set into the other buffer
            // Evaluations are spread over the lanes, not over the hypotheses:
            // per 32-point chunk, lanes (point j, half hf) evaluate point j for
            // the active hypotheses 2i + hf, i = 0.. (T broadcast by readlane),
            // and park d in LDS; then every active lane sums its own 32 values
            // in point order (the reference's sequential double sum) and forms
            // the chunk's inlier word. Work is proportional to the active
            // hypotheses, so lanes whose hypothesis already ended cost nothing.
            uint32_t* nw = slab + (size_t)(cur ^ 1) * B.mask_words * 64;
            const uint64_t actm = __ballot(act);
            const int nact = __popcll(actm);
            const int rank = (int)lane_rank(actm);  // this lane's slot among the active ones
            if (act) la[rank] = lane;
            // the active hypotheses' transforms in slot order, read back by the
            // sweep as three broadcast 16-byte loads per slot instead of 12 permutes
            if (act) {
                if (LN_TD) {
                    double* tw = lTd + rank * LN_TW;
                    double Z[6];
#pragma unroll
                    for (int i = 0; i < 12; i += 2) *reinterpret_cast<double2*>(tw + i) = double2{Td[i], Td[i + 1]};
                    if (LN_TD == 1) {
                        hyp_cov_terms(Td, K, Z);
#pragma unroll
                        for (int i = 0; i < 6; i += 2) *reinterpret_cast<double2*>(tw + 12 + i) = double2{Z[i], Z[i + 1]};
                    }
                } else {
                    float4* tw = reinterpret_cast<float4*>(lT + rank * 12);
                    tw[0] = make_float4(T[0], T[1], T[2], T[3]);
                    tw[1] = make_float4(T[4], T[5], T[6], T[7]);
                    tw[2] = make_float4(T[8], T[9], T[10], T[11]);
                }
            }
            wave_sync();
            double meanError = 0.0;
            unsigned c = 0;
            const int pj = lane & 31, hf = lane >> 5;
            GoodPt gn = pj < ng ? P[pj] : GoodPt{};  // the next chunk's point, loaded a chunk ahead
            for (int c0 = 0; c0 < ng; c0 += 32) {
                LP(const uint64_t lp_ca = wall_clock64();)
                const int k = c0 + pj;
                const GoodPt g = gn;
                if (k + 32 < ng) gn = P[k + 32];
                const bool skip = k >= ng || g.sz == 0.0f || g.tx == 0.0f;  // sic: target.x (ransac.cpp:326)
                const float x1[3] = {g.sx, g.sy, g.sz}, x2[3] = {g.tx, g.ty, g.tz};
                for (int i = 0; i < nact; i += 2) {
                    const int a = i + hf;  // this half's hypothesis slot
                    double Ta[12];
                    const double* Za = nullptr;
                    if (LN_TD) {
                        const double* tr = lTd + min(a, nact - 1) * LN_TW;
#pragma unroll
                        for (int q = 0; q < 12; q += 2) {
                            const double2 v = *reinterpret_cast<const double2*>(tr + q);
                            Ta[q] = v.x, Ta[q + 1] = v.y;
                        }
                        if (LN_TD == 1) Za = tr + 12;
                    } else {
                        const float4* tr = reinterpret_cast<const float4*>(lT + min(a, nact - 1) * 12);
                        const float4 t0 = tr[0], t1 = tr[1], t2 = tr[2];
                        const float tf[12] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w, t2.x, t2.y, t2.z, t2.w};
#pragma unroll
                        for (int q = 0; q < 12; q++) Ta[q] = tf[q];
                    }
                    double d = -1.0;  // not an inlier
                    if (a < nact && !skip) {
                        const double e = error_function2_mk(x1, x2, Ta, K, Za, EFAST);
                        if (!(e > th) && (e >= 0.0)) d = e;
                    }
                    if (a < nact) lres[a * LN_RS + pj] = d;
                }
                LP(const uint64_t lp_cb = wall_clock64(); lp_inner += lp_cb - lp_ca;)
                wave_sync();
                uint32_t word = 0;
                if (act) {
                    const int nj = min(32, ng - c0);
                    // a full chunk: the 32 terms read 8 at a time ahead of
                    // the (sequential, in point order) sum
                    if (nj == 32) {
#pragma unroll
                        for (int j0 = 0; j0 < 32; j0 += 8) {
                            double v[8];
#pragma unroll
                            for (int t = 0; t < 8; t++) v[t] = lres[rank * LN_RS + j0 + t];
#pragma unroll
                            for (int t = 0; t < 8; t++) {
                                if (v[t] >= 0.0) {
                                    meanError += v[t];
                                    c++;
                                    word |= 1u << (j0 + t);
                                }
                            }
                        }
                    } else
                    for (int j = 0; j < nj; j++) {
                        const double v = lres[rank * LN_RS + j];
                        if (v >= 0.0) {
                            meanError += v;
                            c++;
                            word |= 1u << j;
                        }
                    }
                    nw[(size_t)(c0 >> 5) * 64 + lane] = word;
                }
                wave_sync();
                LP(lp_sum += wall_clock64() - lp_cb;)
            }
            LP(lp_sweep += wall_clock64() - lp_q; lp_q = wall_clock64();)
            if (!act) continue;
            nsweep++;
            nref++;
            if (c < 3) meanError = 1e9;
            else {
                meanError /= (double)c;
                meanError = sqrt(meanError);
            }
            bool fin;
            if (c < minInl || meanError > (double)cfg.max_mahal) {
                fin = true;
            } else if (c >= refinedCnt && meanError <= refinedError) {
                const unsigned prev = refinedCnt;
#pragma unroll
                for (int i = 0; i < 12; i++) refinedT[i] = T[i];
                refinedError = meanError;
                refinedCnt = c;
                cur ^= 1;  // the new set becomes the current one
                sample = false;
                fin = c == prev || nref >= 19;
            } else {
                fin = true;
            }
            if (fin) {
                HypRes* hr = B.hyp + (size_t)p * B.hcap + h;
                hr->err = refinedError;
                hr->cnt = (int)refinedCnt;
                hr->pad = nsweep | (nfit << 5);
#pragma unroll
                for (int i = 0; i < 12; i++) hr->T[i] = refinedT[i];
                uint32_t* mo = B.masks + ((size_t)p * B.hcap + h) * B.mask_words;
                if (refinedCnt > 0) {
                    const uint32_t* cw = slab + (size_t)cur * B.mask_words * 64;
                    for (int w = 0; w < words; w++) mo[w] = cw[(size_t)w * 64 + lane];
                }
                __threadfence();
                __hip_atomic_store(B.ready + (size_t)p * B.hcap + h, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                try_fold(B, cfg, p);
                h = -1;
            }
            LP(lp_fold += wall_clock64() - lp_q;)
        }
        // the next pair
        if (cnt <= waves_total) break;  // one pair per wave
        if (cnt > waves_total && slot + waves_total < cnt) {
            slot += waves_total;
            continue;
        }
        slot = -1;
    }
#ifdef ODO_LANES_PROFILE
    if (lane == 0 && gw < LPROF_MAX) {
        uint64_t* r = g_lprof + (size_t)gw * 10;
        r[0] = lp_t0, r[1] = wall_clock64(), r[2] = lp_rounds, r[3] = lp_nact, r[4] = lp_tfc, r[5] = lp_sweep,
        r[6] = lp_inner, r[7] = lp_sum, r[8] = lp_p1, r[9] = lp_p2;  // (fold time and pair: lp_fold, lp_pair)
    }
#endif
}

__global__ void __launch_bounds__(64 * LN_WAVES, 2) k_ransac_lanes(RansacBufs B, RansacCfg cfg, uint32_t* lane_slab,
                                                                   int waves_total, int min_open) {
    // a throughput kernel (ms of FP64 issue): at LN_PRIO its waves do not
    // starve the co-resident extraction waves of the next batch
    __builtin_amdgcn_s_setprio(LN_PRIO);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int gw = (int)blockIdx.x * LN_WAVES + wv;
    // the good points stream through a per-wave LDS chunk: one coalesced load
    // per lane, then wave-uniform broadcast reads in point order
    __shared__ GoodPt s_pts[LN_WAVES][64];
    // the sweep's parked Mahalanobis terms: [active slot][32 points, row
    // stride LN_RS], and the active lanes in slot order. Every active lane then
    // reads its own row in point order: with a 32-double stride all 64 lanes
    // would hit one bank pair (a 32-way conflict per ds_read_b64 half); 33
    // puts lane r's row on banks 2r, 2r + 1
    __shared__ double s_res[LN_WAVES][LN_SLOTS * LN_RS];
    __shared__ int s_la[LN_WAVES][64];
    __shared__ __attribute__((aligned(16))) double s_T[LN_WAVES][LN_SLOTS * LN_TW / (LN_TD ? 1 : 2)];  // active slots' transforms
    MahalConst K;
    K.raster_cov_x = cfg.raster_cov_x;
    K.raster_cov_y = cfg.raster_cov_y;
    K.depth_cov = *B.latch;
    if (EF_FAST == 2 && __builtin_amdgcn_readfirstlane(B.open_cnt[2]) && ef_fast_cov(K))
        lanes_body<true>(B, cfg, lane_slab, waves_total, min_open, lane, wv, gw, s_pts[wv], s_res[wv], s_la[wv],
                         s_T[wv]);
    else
        lanes_body<false>(B, cfg, lane_slab, waves_total, min_open, lane, wv, gw, s_pts[wv], s_res[wv], s_la[wv],
                          s_T[wv]);
}

// ---------------------------------------------------------------- final
// mode 0: every pair. mode 1: after the first eval launch — record which pairs
// are finished (phase[p] = 1) and finalize those. mode 2: finalize the others.
__global__ void __launch_bounds__(64) k_ransac_final(RansacBufs B, RansacCfg cfg, int mode, int* phase) {
    __builtin_amdgcn_s_setprio(ODO_WAVE_PRIO);  // latency-bound: issue ahead of co-resident extraction waves
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    if (mode == 1) {
        const int dn = B.st[p].done;
        if (lane == 0) phase[p] = dn ? 1 : 0;
        if (!dn) return;
    } else if (mode == 2 && phase[p] == 1) {
        return;
    }

    __shared__ Rng s_rng;
    __shared__ double s_d2[64];
    __shared__ int s_ok;
    RState* S = B.st + p;
    odo_pair_result* R = B.res + p;
    float* T12o = B.T12 + (size_t)p * 16;
    const bool active = S->active;
    // every hypothesis has been evaluated by now (the eval launches are
    // ordered before this one); a fold that did not finish there - the last
    // finisher's lock attempt raced a holder's release and re-check (the
    // ready store and the lock CAS are not ordered with each other without a
    // full fence, which measured 4 % of the batch step) - is completed here
    if (active && mode != 1 && !B.no_fold && !ld_relaxed(&S->done)) try_fold_wave(B, cfg, p, lane);
    const int ng = S->ng, words = S->words;
    const unsigned minInl = (unsigned)cfg.min_inlier_th;
    uint32_t* BM = B.best_mask + (size_t)p * B.mask_words;
    float bestT[12];
    for (int i = 0; i < 12; i++) bestT[i] = (i % 5 == 0) ? 1.f : 0.f;
    int best_cnt = S->best_cnt;
    float rmse = S->rmse;
    const int best_h = S->best_h;
    if (active && S->valid == 0) {
        // identity fallback (ransac.cpp:252-264): one sweep with T = I
        const GoodPt* P = B.gpts + (size_t)p * B.match_cap;
        MahalConst K;
        K.raster_cov_x = cfg.raster_cov_x;
        K.raster_cov_y = cfg.raster_cov_y;
        K.depth_cov = *B.latch;
        const float th = cfg.max_mahal * cfg.max_mahal;
        const double Td[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
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
            if (in) s_d2[lane_rank(bal)] = d;
            if (lane == 0) {
                BM[c0 >> 5] = (uint32_t)bal;
                if (c0 + 32 < ng) BM[(c0 >> 5) + 1] = (uint32_t)(bal >> 32);
            }
            __syncthreads();
            const int nin = __popcll(bal);
            if (lane == 0)
                for (int q = 0; q < nin; q++) meanError += s_d2[q];
            cnt += (unsigned)nin;
            __syncthreads();
        }
        if (lane == 0) {
            if (cnt < 3) meanError = 1e9;
            else {
                meanError /= (double)cnt;
                meanError = sqrt(meanError);
            }
            s_ok = (cnt > minInl && meanError < (double)cfg.max_mahal) ? 1 : 0;
        }
        __syncthreads();
        if (s_ok) {
            best_cnt = (int)cnt;
            rmse = (float)((double)rmse + meanError);
        } else {
            best_cnt = 0;
            for (int w = lane; w < words; w += 64) BM[w] = 0;
        }
    } else if (active && best_h >= 0) {
        const HypRes* hr = B.hyp + (size_t)p * B.hcap + best_h;
        for (int i = 0; i < 12; i++) bestT[i] = hr->T[i];
        const uint32_t* src = B.masks + ((size_t)p * B.hcap + best_h) * B.mask_words;
        for (int w = lane; w < words; w += 64) BM[w] = src[w];
    }
    if (lane == 0 && active) {
        R->rmse = rmse;
        R->n_inliers = best_cnt;
        R->ransac_ok = (unsigned)best_cnt >= minInl ? 1 : 0;
        R->visited = S->visited;
        R->n_sweeps = S->sweeps + (S->valid == 0 ? 1 : 0);  // + the identity fallback's sweep
        R->n_fit_points = S->fitpts;
        for (int i = 0; i < 12; i++) R->T12[i] = T12o[i] = bestT[i];
        R->T12[12] = R->T12[13] = R->T12[14] = 0.f;
        R->T12[15] = 1.f;
        T12o[12] = T12o[13] = T12o[14] = 0.f;
        T12o[15] = 1.f;
    }
    if (lane == 0 && B.rng_io) {
        // the caller's rand() stream advances by the visited iterations' draws only
        const int vis = active ? S->visited : 0;
        const int pairs = vis > 0 ? B.samples[((size_t)p * B.hcap + vis - 1) * SREC + SREC - 1] : 0;
        const uint32_t* raw = B.raw + (size_t)p * B.rawcap;
        const int N = min(2 * pairs, B.rawcap);
        ring_at(raw, S, N, s_rng);
        for (int k = N; k < 2 * pairs; k++) s_rng.next();
        for (int i = 0; i < 31; i++) B.rng_io->state[i] = s_rng.s[i];
        B.rng_io->fpos = s_rng.f;
        B.rng_io->rpos = s_rng.r;
    }
}

// hypotheses mode: the ordered fold ran on the host over every rank's
// summaries; install its outcome so k_ransac_final produces the outputs
__global__ void k_ransac_install(RansacBufs B, int best_h, int visited, int valid, int best_cnt, float rmse) {
    RState* S = B.st;
    S->visited = visited;
    S->valid = valid;
    S->best_cnt = best_cnt;
    S->best_h = best_h;
    S->rmse = rmse;
    S->done = 1;
}

// ---------------------------------------------------------------- hypotheses mode on the device
// The exchange of SURVEY §8(e)'s hypotheses mode without host staging: every
// rank's per-hypothesis summaries stay in HBM (a device copy of its HypRes
// range), the ranks all_gather them over RCCL, every rank folds the gathered
// array here, and the owner of the winner packs (T12, rmse, ok, inliers) into
// a payload the ranks sum-reduce (the other ranks contribute zeros).

// The ordered running-best fold of ransac.cpp:233-249 over the gathered
// summaries (hypothesis order), by one wave, as try_fold_wave: only entries
// that beat the state at the start of a 64-entry run can be accepted (rmse
// only falls and best only grows along the run), so the serial steps visit
// those candidates alone and the entries between them just count n++. The
// same record as the host odo_ransac_fold.
__global__ void __launch_bounds__(64) k_hyp_fold(const HypRes* __restrict__ all, int H, int iterations, int ng,
                                                 int min_inl, int sample_size,
                                                 odo_ransac_fold_result* __restrict__ out) {
    const int lane = threadIdx.x;
    int best_h = -1, visited = 0, valid = 0, best = 0;
    float rmse = 1e6f;
    if (ng >= min_inl && ng >= sample_size) {
        const unsigned minInl = (unsigned)min_inl;
        int n = 0, pos = 0;
        bool fin = n >= iterations;
        while (!fin && pos < H) {
            const int m = min(64, H - pos);
            const int q = pos + lane;
            int rc = 0, elo = 0, ehi = 0;
            if (lane < m) {
                rc = all[q].cnt;
                const long long e = __double_as_longlong(all[q].err);
                elo = (int)(uint32_t)e;
                ehi = (int)(uint32_t)((unsigned long long)e >> 32);
            }
            uint64_t cand = __ballot(lane < m && rc > 0 && __hiloint2double(ehi, elo) <= (double)rmse &&
                                     (unsigned)rc >= (unsigned)best && (unsigned)rc >= minInl);
            int i = 0;  // entries of this run visited so far
            while (i < m && !fin) {
                const int c = cand ? (int)__builtin_ctzll(cand) : m;
                if (c - i >= iterations - n) {  // n reaches the limit before the candidate
                    i += iterations - n;
                    n = iterations;
                    fin = true;
                    break;
                }
                n += c - i;
                i = c;
                if (c == m) break;
                cand &= cand - 1;
                const unsigned rci = (unsigned)rdl(rc, c);
                const double re = __hiloint2double(rdl(ehi, c), rdl(elo, c));
                bool brk = false;
                if (re <= (double)rmse && rci >= (unsigned)best) {
                    rmse = (float)re;
                    best = (int)rci;
                    best_h = pos + c;
                    if (rci > ng * 0.5) n += 10;
                    if (rci > ng * 0.75) n += 10;
                    if (rci > ng * 0.8) brk = true;
                }
                n++;
                i++;
                if (brk) n = iterations;
                fin = n >= iterations;
            }
            visited += i;
            valid += __popcll(__ballot(lane < i && rc > 0));
            pos += i;
            if (i < m) break;
        }
    }
    if (lane == 0) *out = odo_ransac_fold_result{best_h, visited, valid, best, rmse, ng, {0, 0}};
}

// the fold's outcome into the pair state, read from device memory
__global__ void k_hyp_install_dev(RansacBufs B, const odo_ransac_fold_result* __restrict__ fr) {
    RState* S = B.st;
    S->visited = fr->visited;
    S->valid = fr->valid;
    S->best_cnt = fr->n_inliers;
    S->best_h = fr->best_h;
    S->rmse = fr->rmse;
    S->done = 1;
}

// The winner's owner packs the payload (HYP_PAYLOAD_HDR header words: T12 bits,
// rmse bits, ok, n_inliers, visited; then the inlier list as DMatch records in
// good-list order, the RANSAC mask compacted); every other rank writes zeros,
// so a sum over the ranks delivers the owner's words exactly. Owner: the rank
// whose range [h0, h1) holds best_h; rank 0 for the identity fallback and for
// a pair that never sampled. One 256-thread workgroup.
#define HYP_PAYLOAD_HDR 32
__global__ void __launch_bounds__(256) k_hyp_payload(RansacBufs B, const odo_ransac_fold_result* __restrict__ fr,
                                                     int h0, int h1, int rank0, const odo_dmatch* __restrict__ good,
                                                     int ng, int* __restrict__ payload, int words) {
    __shared__ int s_wc[4];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int active = B.st->active;
    const int bh = fr->best_h;
    const bool owner = (active && bh >= 0) ? (bh >= h0 && bh < h1) : rank0 != 0;
    if (!owner) {
        for (int w = t; w < words; w += 256) payload[w] = 0;
        return;
    }
    const odo_pair_result* R = B.res;
    if (t < HYP_PAYLOAD_HDR) {
        int v = 0;
        if (t < 16) v = active ? __float_as_int(R->T12[t]) : __float_as_int((t % 5 == 0) ? 1.f : 0.f);
        else if (t == 16) v = __float_as_int(active ? R->rmse : 1e6f);
        else if (t == 17) v = active ? R->ransac_ok : 0;
        else if (t == 18) v = active ? R->n_inliers : 0;
        else if (t == 19) v = active ? fr->visited : 0;
        payload[t] = v;
    }
    const uint32_t* BM = B.best_mask;
    int base = 0;
    if (active) {
        for (int c0 = 0; c0 < ng; c0 += 256) {
            const int k = c0 + t;
            const bool in = k < ng && ((BM[k >> 5] >> (k & 31)) & 1u);
            const uint64_t bal = __ballot(in);
            if (lane == 0) s_wc[wave] = __popcll(bal);
            __syncthreads();
            int before = base, tot = 0;
            for (int w = 0; w < 4; w++) {
                before += w < wave ? s_wc[w] : 0;
                tot += s_wc[w];
            }
            if (in) {
                const int r = before + (int)lane_rank(bal);
                const odo_dmatch m = good[k];
                int* o = payload + HYP_PAYLOAD_HDR + 4 * r;
                o[0] = m.queryIdx;
                o[1] = m.trainIdx;
                o[2] = m.imgIdx;
                o[3] = __float_as_int(m.distance);
            }
            base += tot;
            __syncthreads();
        }
    }
    for (int w = HYP_PAYLOAD_HDR + 4 * base + t; w < words; w += 256) payload[w] = 0;
}

// ---------------------------------------------------------------- host side
size_t ransac_gpt_bytes() { return sizeof(GoodPt); }

static int ransac_hcap(const RansacCfg& cfg) { return std::max(cfg.iterations, 1); }

// generator words per pair: twice the duplicate-free need, plus slack
static int ransac_rawcap(const RansacCfg& cfg) {
    const int S = std::min(std::max(cfg.sample_size, 1), MAX_SAMPLE);
    const long w = 4L * S * ransac_hcap(cfg) + 512;
    return (int)((w + 63) / 64 * 64);
}

struct Layout {
    size_t gpts, st, hyp, samples, ready, masks, raw, open, lslab, total;
};

// k_ransac_lanes grid: workgroups of LN_WAVES waves (ODO_RANSAC_LANES, 0 = the
// wave-per-hypothesis work list k_ransac_eval_list instead). 384 = 1.5 per CU
// of the 256: alone the launch is faster at 2 per CU (512), but in the
// pipelined step the half-empty CUs run the other pair stream's PnP and the
// next batch's extraction beside it (hard workload +5 %)
#ifndef LN_GROUPS
#define LN_GROUPS 384
#endif
static int ln_groups() {
    static int r = [] {
        const char* e = odo_knob("ODO_RANSAC_LANES");
        return e ? std::max(0, atoi(e)) : LN_GROUPS;
    }();
    return r;
}
// Open pairs from which the second RANSAC launch switches from the
// wave-per-hypothesis work list (latency: a few long pairs, as in the default
// workload) to k_ransac_lanes (throughput: most pairs run most of their
// hypotheses, as in the hard workload). Both are launched; the other exits.
static int ln_min_open() {
    static int r = [] {
        const char* e = odo_knob("ODO_LANES_MIN_OPEN");
        return e ? std::max(1, atoi(e)) : 32;
    }();
    return r;
}

static Layout layout(int npairs, int match_cap, int mask_words, const RansacCfg& cfg) {
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    const size_t hc = ransac_hcap(cfg);
    Layout L;
    size_t o = 0;
    L.gpts = o;
    o = al(o + (size_t)npairs * match_cap * sizeof(GoodPt));
    L.st = o;
    o = al(o + (size_t)npairs * sizeof(RState));
    L.hyp = o;
    o = al(o + (size_t)npairs * hc * sizeof(HypRes));
    L.samples = o;
    o = al(o + (size_t)npairs * hc * SREC * sizeof(int));
    L.ready = o;
    o = al(o + (size_t)npairs * hc * sizeof(int));
    L.masks = o;
    o = al(o + (size_t)npairs * hc * mask_words * 4);
    L.raw = o;
    o = al(o + (size_t)npairs * ransac_rawcap(cfg) * 4);
    L.open = o;
    o = al(o + (size_t)(npairs + 4) * 4);
    L.lslab = o;  // per-wave inlier-set buffers of k_ransac_lanes (never launched for one pair:
                  // a lone pair starts every hypothesis row in the first launch)
    if (npairs > 1) o = al(o + (size_t)ln_groups() * LN_WAVES * 2 * mask_words * 64 * 4);
    L.total = o;
    return L;
}

size_t ransac_scratch_bytes(int npairs, int match_cap, int mask_words, const RansacCfg& cfg) {
    return layout(npairs, match_cap, mask_words, cfg).total;
}

static RansacBufs carve(void* scratch, int npairs, int match_cap, int mask_words, const RansacCfg& cfg) {
    const Layout L = layout(npairs, match_cap, mask_words, cfg);
    char* s = (char*)scratch;
    RansacBufs B{};
    B.gpts = (GoodPt*)(s + L.gpts);
    B.st = (RState*)(s + L.st);
    B.hyp = (HypRes*)(s + L.hyp);
    B.samples = (int*)(s + L.samples);
    B.ready = (int*)(s + L.ready);
    B.masks = (uint32_t*)(s + L.masks);
    B.open_list = (int*)(s + L.open);
    B.open_cnt = B.open_list + npairs;
    B.lslab = (uint32_t*)(s + L.lslab);
    B.raw = (uint32_t*)(s + L.raw);
    B.hcap = ransac_hcap(cfg);
    B.rawcap = ransac_rawcap(cfg);
    B.match_cap = match_cap;
    B.mask_words = mask_words;
    return B;
}

// A^k of the generator's 31x31 transition (mod 2^32), host side
typedef std::vector<uint32_t> Mat31;
static Mat31 mat_mul31(const Mat31& X, const Mat31& Y) {
    Mat31 Z(31 * 31, 0);
    for (int i = 0; i < 31; i++)
        for (int k = 0; k < 31; k++) {
            const uint32_t x = X[i * 31 + k];
            if (!x) continue;
            for (int j = 0; j < 31; j++) Z[i * 31 + j] += x * Y[k * 31 + j];
        }
    return Z;
}
static Mat31 mat_pow31(long e) {
    Mat31 A(31 * 31, 0), R(31 * 31, 0);
    for (int i = 0; i < 30; i++) A[i * 31 + i + 1] = 1;  // shift
    A[30 * 31 + 0] = 1;                                  // x_n = x_{n-31} + x_{n-3}
    A[30 * 31 + 28] = 1;
    for (int i = 0; i < 31; i++) R[i * 31 + i] = 1;
    while (e > 0) {
        if (e & 1) R = mat_mul31(R, A);
        A = mat_mul31(A, A);
        e >>= 1;
    }
    return R;
}

// device jump tables per (device, L): [i][j][lane] A^(lane*L), then A^310
static const uint32_t* raw_jump_tables(int L) {
    static std::mutex mu;
    static std::map<std::pair<int, int>, uint32_t*> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find({dev, L});
    if (it != cache.end()) return it->second;
    std::vector<uint32_t> h((size_t)RAW_LANES * 961 + 961);
    const Mat31 AL = mat_pow31(L);
    Mat31 M(31 * 31, 0);
    for (int i = 0; i < 31; i++) M[i * 31 + i] = 1;
    for (int k = 0; k < RAW_LANES; k++) {
        for (int i = 0; i < 31; i++)
            for (int j = 0; j < 31; j++) h[((size_t)i * 31 + j) * RAW_LANES + k] = M[i * 31 + j];
        M = mat_mul31(AL, M);
    }
    const Mat31 D = mat_pow31(310);
    std::copy(D.begin(), D.end(), h.begin() + (size_t)RAW_LANES * 961);
    uint32_t* d = nullptr;
    if (hipMalloc(&d, h.size() * 4) != hipSuccess) return nullptr;
    (void)hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    cache[{dev, L}] = d;
    return d;
}

void launch_ransac_raw(hipStream_t st, void* scratch, int npairs, int match_cap, int mask_words, RansacCfg cfg,
                       uint64_t seed_base, uint64_t pair_base, odo_rng* rng_io) {
    RansacBufs B = carve(scratch, npairs, match_cap, mask_words, cfg);
    B.rng_io = rng_io;
    const int L = (B.rawcap + RAW_LANES - 1) / RAW_LANES;
    hipLaunchKernelGGL(k_ransac_raw, dim3(npairs), dim3(64), 0, st, B, seed_base, pair_base, raw_jump_tables(L), L);
}

static int ev2_rows() {
    static int r = [] {
        const char* e = odo_knob("ODO_EV2_ROWS");
        // default: every remaining hypothesis row in flight. A pair whose best
        // inlier ratio stays just under the 80 % break visits ~all H
        // hypotheses; fewer rows make it take several rounds (measured at
        // 64-frame batches: 1.366 ms per step with all rows, 1.39 with 16)
        return e ? std::max(1, atoi(e)) : 1 << 30;
    }();
    return r;
}

// workgroups of the work-list second launch (ODO_EV2_LIST; 0 = the
// (pairs x rows) grid instead)
static int ev2_list() {
    static int r = [] {
        const char* e = odo_knob("ODO_EV2_LIST");
        return e ? std::max(0, atoi(e)) : 512;
    }();
    return r;
}

static void ransac_eval_lds_attr() {
    static bool done = false;
    if (!done) {
        (void)hipFuncSetAttribute((const void*)k_ransac_eval, hipFuncAttributeMaxDynamicSharedMemorySize, (int)EV_LDS);
        (void)hipFuncSetAttribute((const void*)k_ransac_eval_list, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)EV_LDS);
        done = true;
    }
}

void launch_ransac(hipStream_t st, const void* good, const int* n_good, const int* n_matches,
                   const odo_dmatch* matches, const float* xyz, int kp_cap, int slot0, int match_cap, RansacCfg cfg,
                   const double* latch, const int* pair_valid, int min_matches, odo_rng* rng_io, void* scratch,
                   uint32_t* best_mask, int mask_words, odo_pair_result* res, float* T12, int npairs, int part,
                   int* phase, int* open_hint) {
    ransac_eval_lds_attr();
    cfg.h0 = EV_H0;
    cfg.fold_wave = 0;
    RansacBufs B = carve(scratch, npairs, match_cap, mask_words, cfg);
    B.good = (const SortElR*)good;
    B.n_good = n_good;
    B.n_matches = n_matches;
    B.matches = matches;
    B.xyz = xyz;
    B.kp_cap = kp_cap;
    B.slot0 = slot0;
    B.latch = latch;
    B.pair_valid = pair_valid;
    B.min_matches = min_matches;
    B.rng_io = rng_io;
    B.best_mask = best_mask;
    B.res = res;
    B.T12 = T12;
    const int H = std::max(cfg.iterations, 0);
    B.h_lo = 0;
    B.h_hi = H;
    B.no_fold = 0;
    if (part == 3) {
        // hypotheses mode, one pair: samples of all H, evaluation of [h0, h1)
        // only (h0/h1 passed in phase[0..1]), no fold and no outputs
        B.h_lo = std::max(0, phase[0]);
        B.h_hi = std::min(H, phase[1]);
        B.no_fold = 1;
        hipLaunchKernelGGL(k_ransac_prep, dim3(npairs), dim3(256), 0, st, B, cfg);
        if (B.h_hi > B.h_lo) {
            const int ya = B.h_lo / EV_WAVES, yb = (B.h_hi + EV_WAVES - 1) / EV_WAVES;
            hipLaunchKernelGGL(k_ransac_eval, dim3(npairs, yb - ya), dim3(64 * EV_WAVES), EV_LDS, st,
                               B, cfg, 0, ya, yb * EV_WAVES);
        }
        return;
    }
    // Two eval launches: the first h0 hypotheses of every pair (the >80% break
    // usually ends a pair within them), then the rest, which only pairs still
    // folding take up — so the speculative hypotheses of finished pairs do
    // not compete with the long ones. part 1 = prep, first launch and the
    // finished pairs' outputs (phase[] marks them); part 2 = the rest; part 0
    // = both.
    // hypotheses of the first launch: odo_kernel_forms.ransac_first_hyps, else
    // ODO_EV_H0 (tuning), else EV_H0
    static const int h0env = [] {
        const char* e = odo_knob("ODO_EV_H0");
        return e ? std::max(1, atoi(e)) : EV_H0;
    }();
    const int h0k = cfg.first_hyps > 0 ? cfg.first_hyps : h0env;
    // a lone pair (the per-stage odo_ransac, a one-frame batch) starts every
    // hypothesis at once: the device is otherwise idle, and the visited
    // hypotheses beyond the first row no longer wait for the first launch
    // (the fold and the aborts make the result independent of the schedule)
    const int h0 = npairs == 1 ? H : std::min(H, h0k);
    cfg.h0 = h0;
    cfg.fold_wave = npairs == 1;
    if (part != 2) {
        hipLaunchKernelGGL(k_ransac_prep, dim3(npairs), dim3(256), 0, st, B, cfg);
        if (h0 > 0) {
            // rows of EV_WAVES hypotheses; a first launch of fewer runs that many waves
            const int r0 = (h0 + EV_WAVES - 1) / EV_WAVES, nw = std::min(h0, EV_WAVES);
            hipLaunchKernelGGL(k_ransac_eval, dim3(npairs, r0), dim3(64 * nw), EV_LDS, st, B, cfg, 0, 0, h0);
        }
        if (part == 1) hipLaunchKernelGGL(k_ransac_final, dim3(npairs), dim3(64), 0, st, B, cfg, 1, phase);
    }
    if (part != 1) {
        // the second launch's waves stride over the remaining hypotheses
        // [h0, H): ev2_rows() rows of EV_WAVES per pair in flight (ODO_EV2_ROWS)
        const int rows = (H - h0 + EV_WAVES - 1) / EV_WAVES;
        if (rows > 0) {
            if (ev2_list()) {
                hipLaunchKernelGGL(k_ransac_open, dim3(1), dim3(256), 0, st, B, npairs);
                // which of the two kernels takes the open pairs: decided on the
                // host from the previous batch's open count on this frame set
                // (open_hint, page-locked, copied back asynchronously), so
                // only one of them is launched; both give the same results
                // (no hint yet, -1: the first batch of a set: both are
                // launched and the open count on the device picks one)
                const int lanes = ln_groups();
                const int tmin = cfg.lanes_min_open > 0 ? cfg.lanes_min_open : ln_min_open();
                const int hint = open_hint ? *reinterpret_cast<volatile int*>(open_hint) : 0;
                const bool use_lanes = lanes && open_hint && hint >= tmin;
                // the pairs still open after the first launch are the long
                // ones (the bench's sequence: 2 of 64, visiting 36 and 380
                // hypotheses): the work list folds them with the whole wave
                // (64 ready flags per load, try_fold_wave) instead of lane
                // 0's serial coherent loads, ~0.4 us per visited hypothesis
                RansacCfg cfg2 = cfg;
                cfg2.fold_wave = EV2_FOLD_WAVE;
                if (lanes && hint < 0) {
                    hipLaunchKernelGGL(k_ransac_eval_list, dim3(ev2_list()), dim3(64 * EV_WAVES), EV_LDS, st, B, cfg2,
                                       h0, rows, tmin - 1);
                    hipLaunchKernelGGL(k_ransac_lanes, dim3(lanes), dim3(64 * LN_WAVES), 0, st, B, cfg, B.lslab,
                                       lanes * LN_WAVES, tmin);
                } else if (use_lanes)
                    hipLaunchKernelGGL(k_ransac_lanes, dim3(lanes), dim3(64 * LN_WAVES), 0, st, B, cfg, B.lslab,
                                       lanes * LN_WAVES, 1);
                else
                    hipLaunchKernelGGL(k_ransac_eval_list, dim3(ev2_list()), dim3(64 * EV_WAVES), EV_LDS, st, B, cfg2,
                                       h0, rows, 1 << 30);
                if (open_hint) (void)hipMemcpyAsync(open_hint, B.open_cnt, sizeof(int), hipMemcpyDeviceToHost, st);
            } else {
                hipLaunchKernelGGL(k_ransac_eval, dim3(npairs, std::min(rows, ev2_rows())), dim3(64 * EV_WAVES),
                                   EV_LDS, st, B, cfg, h0, 0, H);
            }
        }
        hipLaunchKernelGGL(k_ransac_final, dim3(npairs), dim3(64), 0, st, B, cfg, part == 2 ? 2 : 0, phase);
    }
}

// Hypotheses mode readback / finish over the scratch of a part-3 launch
// (one pair): per-hypothesis (err, cnt, T) of [h0, h1), then the outputs of
// the folded run (k_ransac_final mode 0: T12 / inlier mask of best_h when this
// process evaluated it, identity fallback when nothing was valid, and the
// caller's rand() state after exactly the visited draws).
void ransac_read_hyps(hipStream_t st, void* scratch, int match_cap, int mask_words, RansacCfg cfg, int h0, int h1,
                      double* err, int* cnt, float* T) {
    RansacBufs B = carve(scratch, 1, match_cap, mask_words, cfg);
    std::vector<HypRes> h(std::max(h1 - h0, 0));
    if (h.empty()) return;
    (void)hipMemcpyAsync(h.data(), B.hyp + h0, h.size() * sizeof(HypRes), hipMemcpyDeviceToHost, st);
    (void)hipStreamSynchronize(st);
    for (size_t i = 0; i < h.size(); i++) {
        err[i] = h[i].err;
        cnt[i] = h[i].cnt;
        for (int k = 0; k < 12; k++) T[i * 12 + k] = h[i].T[k];
    }
}

void launch_ransac_finish(hipStream_t st, void* scratch, int match_cap, int mask_words, RansacCfg cfg,
                          const double* latch, odo_rng* rng_io, uint32_t* best_mask, odo_pair_result* res, float* T12,
                          int best_h, int visited, int valid, int best_cnt, float rmse) {
    RansacBufs B = carve(scratch, 1, match_cap, mask_words, cfg);
    B.latch = latch;
    B.rng_io = rng_io;
    B.best_mask = best_mask;
    B.res = res;
    B.T12 = T12;
    hipLaunchKernelGGL(k_ransac_install, dim3(1), dim3(1), 0, st, B, best_h, visited, valid, best_cnt, rmse);
    hipLaunchKernelGGL(k_ransac_final, dim3(1), dim3(64), 0, st, B, cfg, 0, (int*)nullptr);
}

// hypotheses mode on the device: this rank's summaries [h0, h1) into d_block
// (HypRes = odo_hyp_summary layout, 64 B each)
void ransac_export_hyps(hipStream_t st, void* scratch, int match_cap, int mask_words, RansacCfg cfg, int h0, int h1,
                        void* d_block) {
    RansacBufs B = carve(scratch, 1, match_cap, mask_words, cfg);
    if (h1 > h0)
        (void)hipMemcpyAsync(d_block, B.hyp + h0, (size_t)(h1 - h0) * sizeof(HypRes), hipMemcpyDeviceToDevice, st);
}
void launch_hyp_fold(hipStream_t st, const void* d_all, int H, int iterations, int ng, int min_inl, int sample_size,
                     odo_ransac_fold_result* d_out) {
    static_assert(sizeof(HypRes) == sizeof(odo_hyp_summary), "summary layout");
    hipLaunchKernelGGL(k_hyp_fold, dim3(1), dim3(64), 0, st, (const HypRes*)d_all, H, iterations, ng, min_inl,
                       sample_size, d_out);
}
void launch_hyp_finish(hipStream_t st, void* scratch, int match_cap, int mask_words, RansacCfg cfg,
                       const double* latch, odo_rng* rng_io, uint32_t* best_mask, odo_pair_result* res, float* T12,
                       const odo_ransac_fold_result* d_fold, int h0, int h1, int rank0, const odo_dmatch* good, int ng,
                       int* payload, int words) {
    RansacBufs B = carve(scratch, 1, match_cap, mask_words, cfg);
    B.latch = latch;
    B.rng_io = rng_io;
    B.best_mask = best_mask;
    B.res = res;
    B.T12 = T12;
    hipLaunchKernelGGL(k_hyp_install_dev, dim3(1), dim3(1), 0, st, B, d_fold);
    hipLaunchKernelGGL(k_ransac_final, dim3(1), dim3(64), 0, st, B, cfg, 0, (int*)nullptr);
    hipLaunchKernelGGL(k_hyp_payload, dim3(1), dim3(256), 0, st, B, d_fold, h0, h1, rank0, good, ng, payload, words);
}
int hyp_payload_words(int ng) { return HYP_PAYLOAD_HDR + 4 * std::max(ng, 0); }

}  // namespace odo
#ifdef ODO_LANES_PROFILE
// profile builds only: the per-wave records of the last k_ransac_lanes launch
extern "C" int odo_lanes_prof_read(uint64_t* out, int n) {
    n = std::min(n, LPROF_MAX);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(odo::g_lprof), (size_t)n * 10 * sizeof(uint64_t)) != hipSuccess) return -1;
    return n;
}
#endif
#ifdef ODO_RANSAC_PROFILE
// profile builds only: the per-hypothesis records of the last launch
extern "C" int odo_ransac_prof_read(uint64_t* out, int n, uint64_t* done_t) {
    n = std::min(n, RPROF_MAX);
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(odo::g_rprof), (size_t)n * 8 * sizeof(uint64_t)) != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(done_t, HIP_SYMBOL(odo::g_rprof_done), sizeof(uint64_t)) != hipSuccess) return -1;
    std::vector<uint64_t> z((size_t)n * 8, 0);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(odo::g_rprof), z.data(), z.size() * sizeof(uint64_t));
    return n;
}
#endif
