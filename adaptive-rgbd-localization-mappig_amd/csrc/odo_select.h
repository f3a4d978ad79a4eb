// Workgroup-wide helpers shared by the ADAPTIVE grid extractors
// (k_adaptive.hip: FAST inner detector; k_adaptive_orb.hip: cv::ORB inner
// detector): ordered ranks and scans over the workgroup, the threshold-free
// FAST S map of one 128 x 8 tile, and libstdc++'s std::nth_element /
// std::partition restated as workgroup-parallel code over any element type
// with a 32-bit ascending key.
#pragma once

#include "odo_device.h"

namespace odo {

// ============================================================ block helpers
// ordered rank of `keep` among the workgroup's threads (thread order) and the
// total; ws: >= 16 ints of LDS
ODO_INLINE int block_rank(bool keep, int* ws, int* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    const uint64_t b = __ballot(keep);
    const int in_wave = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) ws[wv] = __popcll(b);
    __syncthreads();
    int base = 0, tot = 0;
    for (int k = 0; k < nw; k++) {
        const int c = ws[k];
        if (k < wv) base += c;
        tot += c;
    }
    __syncthreads();
    *total = tot;
    return base + in_wave;
}

// exclusive scan of two per-thread counts over the workgroup
ODO_INLINE int2 block_scan2i(int a, int b, int (*ws)[2], int2* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
    int ia = a, ib = b;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int x = __shfl_up(ia, o), y = __shfl_up(ib, o);
        if (lane >= o) {
            ia += x;
            ib += y;
        }
    }
    if (lane == 63) {
        ws[wv][0] = ia;
        ws[wv][1] = ib;
    }
    __syncthreads();
    int ba = 0, bb = 0, ta = 0, tb = 0;
    for (int k = 0; k < nw; k++) {
        if (k < wv) {
            ba += ws[k][0];
            bb += ws[k][1];
        }
        ta += ws[k][0];
        tb += ws[k][1];
    }
    __syncthreads();
    *total = make_int2(ta, tb);
    return make_int2(ba + ia - a, bb + ib - b);
}

// ============================================================ S map tile
// S(p) = the best 9-arc contrast of p (FAST at threshold t keeps p iff
// S(p) > t; its cornerScore is S(p) - 1). One 128 x 8 tile of one image,
// 4 pixels per thread (256 threads); the window (columns tx0-4 .. tx0+131,
// rows ty0-3 .. ty0+10) staged in LDS with dword loads of the pitched image.
// Pixels within 3 of the image border get S = 0 (FAST never tests them), so
// out-of-image words are clamped reads whose values are unused.
#define SM_TW 128
#define SM_TH 8
#define SM_LW (SM_TW + 8)            // bytes per LDS row
#define SM_LR (SM_TH + 6)            // LDS rows

typedef short short2v __attribute__((ext_vector_type(2)));

ODO_INLINE short2v pk_min(short2v a, short2v b) { return __builtin_elementwise_min(a, b); }
ODO_INLINE short2v pk_max(short2v a, short2v b) { return __builtin_elementwise_max(a, b); }

// S of the 4 pixels x..x+3 of one row from W, the 7 rows (dy = -3..3) x 3
// aligned dwords (columns x-4 .. x+7) their circles touch; byte e of the
// result = S(x + e), no border masking. A circle pixel pair (columns c, c+1
// of a row) is one v_perm into the two 16-bit halves; two pixels per packed
// 16-bit op.
ODO_INLINE uint32_t smap4(const uint32_t (&W)[7][3]) {
    // bytes i, i+1 (i = 0..10 over the row's 12 bytes) -> 16-bit lanes (lo, hi)
    auto pair16 = [&](int dy, int i) -> short2v {
        const uint32_t lo = W[dy][i >> 2], hi = W[dy][(i >> 2) + 1 < 3 ? (i >> 2) + 1 : 2];
        const int o = i & 3;  // byte offset within lo; o + 1 may spill into hi
        const uint32_t sel = (uint32_t)o | 0x0c00u | ((uint32_t)(o + 1) << 16) | 0x0c000000u;
        const uint32_t v = __builtin_amdgcn_perm(hi, lo, sel);
        return *reinterpret_cast<const short2v*>(&v);
    };
    // circle offsets (x, y) of FAST_t<16> (App. A.3)
    constexpr int cxo[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    constexpr int cyo[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    uint32_t out = 0;
#pragma unroll
    for (int pp = 0; pp < 4; pp += 2) {
        short2v d[16];
        const short2v v = pair16(3, 4 + pp);
#pragma unroll
        for (int k = 0; k < 16; k++) d[k] = v - pair16(3 + cyo[k], 4 + pp + cxo[k]);
        // dark = max over the 16 circular 9-arcs of their min d. Arcs k and
        // k+1 (k even) share M = min d[k+1 .. k+8], so their larger min is
        // min(M, max(d[k], d[k+9])): only the 8-runs starting at odd j are
        // needed (built from odd 2- and 4-runs). bright is the same with min
        // and max exchanged. 96 packed ops instead of 160.
        short2v mn2[8], mx2[8], mn4[8], mx4[8];
#pragma unroll
        for (int i = 0; i < 8; i++) {  // runs starting at j = 2i + 1
            const int j = 2 * i + 1;
            mn2[i] = pk_min(d[j], d[(j + 1) & 15]);
            mx2[i] = pk_max(d[j], d[(j + 1) & 15]);
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            mn4[i] = pk_min(mn2[i], mn2[(i + 1) & 7]);
            mx4[i] = pk_max(mx2[i], mx2[(i + 1) & 7]);
        }
        short2v dark = short2v{0, 0}, bright = short2v{0, 0};  // max(arc min), min(arc max)
#pragma unroll
        for (int i = 0; i < 8; i++) {  // arcs k = 2i, 2i + 1
            const int k = 2 * i;
            const short2v m8 = pk_min(mn4[i], mn4[(i + 2) & 7]);
            const short2v x8 = pk_max(mx4[i], mx4[(i + 2) & 7]);
            dark = pk_max(dark, pk_min(m8, pk_max(d[k], d[(k + 9) & 15])));
            bright = pk_min(bright, pk_max(x8, pk_min(d[k], d[(k + 9) & 15])));
        }
        const short2v sv = pk_max(dark, -bright);
        out |= ((uint32_t)(uint16_t)sv.x << (8 * pp)) | ((uint32_t)(uint16_t)sv.y << (8 * (pp + 1)));
    }
    return out;
}

ODO_INLINE void smap_tile(const uint8_t* __restrict__ img, int w, int h, int pitch, int tx0, int ty0,
                          uint8_t* __restrict__ smap, uint32_t* lds) {
    for (int i = threadIdx.x; i < SM_LR * (SM_LW / 4); i += 256) {
        const int r = i / (SM_LW / 4), q = i % (SM_LW / 4);
        int gy = ty0 - 3 + r;
        gy = gy < 0 ? 0 : (gy >= h ? h - 1 : gy);
        int gx = tx0 - 4 + 4 * q;
        gx = gx < 0 ? 0 : (gx + 4 > pitch ? pitch - 4 : gx);
        lds[i] = *reinterpret_cast<const uint32_t*>(img + (size_t)gy * pitch + gx);
    }
    __syncthreads();
    const int r = threadIdx.x >> 5, q = threadIdx.x & 31;
    const int y = ty0 + r, x = tx0 + 4 * q;
    if (y >= h || x >= pitch) return;
    const int ly = r + 3;
    uint32_t W[7][3];
#pragma unroll
    for (int dy = 0; dy < 7; dy++)
#pragma unroll
        for (int j = 0; j < 3; j++) W[dy][j] = lds[(ly - 3 + dy) * (SM_LW / 4) + q + j];
    uint32_t out = smap4(W);
    const bool yin = y >= 3 && y < h - 3;
#pragma unroll
    for (int e = 0; e < 4; e++) {
        const int xx = x + e;
        if (!(yin && xx >= 3 && xx < w - 3)) out &= ~(0xffu << (8 * e));
    }
    *reinterpret_cast<uint32_t*>(smap + (size_t)y * pitch + x) = out;
}

// ============================================================ std::nth_element
// libstdc++ __introselect over elements of type T ordered by an ascending
// 32-bit key K::key(e) (comp(a, b) = key(a) < key(b)). Every partition runs
// on the whole workgroup: the Hoare scan pairs the k-th left stop
// (key >= pk) with the k-th right stop (key <= pk) while they have not
// crossed (k < k*), and cuts at min(L[k*], R[k*-1]) (the model checked
// against the real std::nth_element in tests/test_adaptive_model.py).
struct SelState {
    int first, last, depth, pk, ks, nl, nr, done;
    int ws[16][2];
};

template <typename T>
ODO_INLINE void sel_swap(T* A, int i, int j) {
    const T t = A[i];
    A[i] = A[j];
    A[j] = t;
}

template <typename T, typename K>
ODO_INLINE void sel_adjust_heap(T* A, int first, int hole, int len, T value) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (K::key(A[first + child]) < K::key(A[first + child - 1])) child--;
        A[first + hole] = A[first + child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        A[first + hole] = A[first + child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && K::key(A[first + parent]) < K::key(value)) {
        A[first + hole] = A[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    A[first + hole] = value;
}

// std::__heap_select(first, middle, last) (depth-limit fallback; one lane)
template <typename T, typename K>
ODO_INLINE void sel_heap_select(T* A, int first, int middle, int last) {
    const int len = middle - first;
    if (len >= 2)
        for (int parent = (len - 2) / 2;; parent--) {
            sel_adjust_heap<T, K>(A, first, parent, len, A[first + parent]);
            if (parent == 0) break;
        }
    for (int i = middle; i < last; ++i)
        if (K::key(A[i]) < K::key(A[first])) {  // __pop_heap(first, middle, i)
            const T v = A[i];
            A[i] = A[first];
            sel_adjust_heap<T, K>(A, first, 0, len, v);
        }
}

template <typename T, typename K>
ODO_INLINE void sel_insertion_sort(T* A, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        const T v = A[i];
        if (K::key(v) < K::key(A[first])) {
            for (int k = i; k > first; --k) A[k] = A[k - 1];
            A[first] = v;
        } else {
            int cur = i, next = i - 1;
            while (K::key(v) < K::key(A[next])) {
                A[cur] = A[next];
                cur = next;
                --next;
            }
            A[cur] = v;
        }
    }
}

// comp(a, b) = score(a) > score(b) (ResponseComparator /
// KeypointResponseGreater) on packed FAST keypoints (score << 24 | y << 12 |
// x): key = 255 - score ascending.
struct ScoreKey {
    static ODO_INLINE uint32_t key(uint32_t e) { return 255u - (e >> 24); }
};

// A: n elements (LDS or global); posL/posR: n ints of scratch; every thread of
// the workgroup calls this.
template <typename T, typename K>
ODO_INLINE void block_nth_element(T* A, int n, int nth, int* posL, int* posR, SelState& S) {
    if (n <= 0 || nth >= n) return;
    const int t = threadIdx.x, NT = blockDim.x;
    if (t == 0) {
        S.first = 0;
        S.last = n;
        S.depth = 2 * (31 - __builtin_clz((unsigned)n));
        S.done = 0;
    }
    __syncthreads();
    while (S.last - S.first > 3 && !S.done) {
        const int first = S.first, last = S.last;
        if (S.depth == 0) {
            if (t == 0) {
                sel_heap_select<T, K>(A, first, nth + 1, last);
                sel_swap(A, first, nth);
                S.done = 1;
            }
            __syncthreads();
            break;
        }
        if (t == 0) {
            S.depth--;
            // __move_median_to_first(first, first + 1, mid, last - 1)
            const int a = first + 1, b = first + (last - first) / 2, c = last - 1;
            const uint32_t ka = K::key(A[a]), kb = K::key(A[b]), kc = K::key(A[c]);
            int m;
            if (ka < kb) m = kb < kc ? b : (ka < kc ? c : a);
            else m = ka < kc ? a : (kb < kc ? c : b);
            sel_swap(A, first, m);
            S.pk = (int)K::key(A[first]);
        }
        __syncthreads();
        const uint32_t pk = (uint32_t)S.pk;
        const int m = last - first - 1;
        const int chunk = (m + NT - 1) / NT;
        const int j0 = first + 1 + min(m, t * chunk), j1 = first + 1 + min(m, t * chunk + chunk);
        int cg = 0, cl = 0;
        for (int j = j0; j < j1; j++) {
            const uint32_t k = K::key(A[j]);
            cg += k >= pk;
            cl += k <= pk;
        }
        int2 tot;
        const int2 base = block_scan2i(cg, cl, S.ws, &tot);
        int rg = base.x, rl = base.y;
        for (int j = j0; j < j1; j++) {
            const uint32_t k = K::key(A[j]);
            if (k >= pk) posL[rg++] = j;
            if (k <= pk) posR[tot.y - 1 - rl++] = j;  // posR[0] = the rightmost right stop
        }
        __syncthreads();
        if (t == 0) {
            // k* = #{k < min(nL, nR) : posL[k] < posR[k]} (monotone in k)
            int lo = 0, hi = min(tot.x, tot.y);
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (posL[mid] < posR[mid]) lo = mid + 1;
                else hi = mid;
            }
            S.ks = lo;
        }
        __syncthreads();
        const int ks = S.ks;
        for (int k = t; k < ks; k += NT) sel_swap(A, posL[k], posR[k]);
        __syncthreads();
        if (t == 0) {
            int cut = ks < tot.x ? posL[ks] : last;
            if (ks > 0) cut = min(cut, posR[ks - 1]);
            if (cut <= nth) S.first = cut;
            else S.last = cut;
        }
        __syncthreads();
    }
    if (t == 0 && !S.done) sel_insertion_sort<T, K>(A, S.first, S.last);
    __syncthreads();
}

// std::partition(A + first, A + last, key <= amb) (libstdc++ bidirectional
// __partition; one lane): the tail step of KeyPointsFilter::retainBest, whose
// predicate response >= ambiguous is key <= key(ambiguous) for a key that
// orders by response descending. Returns the partition point.
template <typename T, typename K>
ODO_INLINE int sel_partition_le(T* A, int first, int last, uint32_t amb) {
    while (true) {
        while (first != last && K::key(A[first]) <= amb) ++first;
        if (first == last) break;
        --last;
        while (first != last && !(K::key(A[last]) <= amb)) --last;
        if (first == last) break;
        sel_swap(A, first, last);
        ++first;
    }
    return first;
}

}  // namespace odo
