// Extractor(FAST, ORB, ADAPTIVE) for gfx950:
// Features/extractor.cpp:39-77, videogridadaptedfeaturedetector.cpp:24-84,
// videodynamicadaptedfeaturedetector.cpp:24-44, detectoradjuster.cpp:22-65,
// then KeyPointsFilter::retainBest and cv::ORB::compute on the kept keypoints.
//
// The reference runs, per grid cell, up to five dependent cv::FAST passes
// whose threshold is a per-cell state carried from frame to frame. Here the
// threshold never touches the pixel work (DESIGN.md §4 "ADAPTIVE grid"):
//
//   k_adapt_smap    S(p) = the best 9-arc contrast of every pixel. FAST at
//                   threshold t keeps p iff S(p) > t, its cornerScore is
//                   S(p) - 1, and the strict 3x3 NMS becomes "S(p) >= 2 and
//                   S(p) > S(q) for every neighbour q inside the cell ROI's
//                   detection region" - independent of t.
//   k_adapt_cand    per (frame, cell, band of rows): the NMS survivors in
//                   row-major order + a per-cell histogram of S. The keypoint
//                   count of every threshold is a suffix sum of the histogram.
//   k_adapt_chain   per cell: the tooFew/tooMany/good threshold chain over the
//                   batch's frames in order, on the count tables (no pixels).
//   k_adapt_select  per (frame, cell): survivors with S > t*, then
//                   keepStrongest = std::nth_element (exact libstdc++
//                   introselect, workgroup-parallel partitions).
//   k_adapt_assemble per frame: cells in grid order, retainBest (nth_element +
//                   std::partition of the ties), ORB's runByImageBorder(31).
//   k_adapt_finalize rBRIEF at angle -1 (ORB does not orient provided
//                   keypoints) on the blurred image, undistort, depth.
#include "odo_device.h"
#include "odo_internal.h"
#include "../../include/odo_orb_pattern.h"

namespace odo {

__constant__ int8_t c_apattern[1024];

// ============================================================ S map
// Tile: 128 x 8 output pixels, 4 per thread; input window staged in LDS with
// dword loads of the pitched level 0 (columns tx0-4 .. tx0+131, rows ty0-3 ..
// ty0+10). Pixels within 3 of the image border get S = 0 (FAST never tests
// them), so out-of-image words are clamped reads whose values are unused.
#define SM_TW 128
#define SM_TH 8
#define SM_LW (SM_TW + 8)            // bytes per LDS row
#define SM_LR (SM_TH + 6)            // LDS rows

typedef short short2v __attribute__((ext_vector_type(2)));

ODO_INLINE short2v pk_min(short2v a, short2v b) { return __builtin_elementwise_min(a, b); }
ODO_INLINE short2v pk_max(short2v a, short2v b) { return __builtin_elementwise_max(a, b); }

__global__ void __launch_bounds__(256) k_adapt_smap(const uint8_t* __restrict__ pyr, size_t pyr_stride, int w, int h,
                                                    int pitch, int tiles_x, uint8_t* __restrict__ smap,
                                                    size_t smap_stride) {
    __shared__ uint32_t lds[SM_LR * SM_LW / 4];
    const int f = blockIdx.y;
    const int tx0 = (blockIdx.x % tiles_x) * SM_TW, ty0 = (blockIdx.x / tiles_x) * SM_TH;
    const uint8_t* img = pyr + (size_t)f * pyr_stride;
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
    // the 7 rows x 12 columns (x-4 .. x+7) the 4 pixels' circles touch: three
    // aligned dwords per row; a circle pixel pair (columns c, c+1 of a row) is
    // one v_perm into the two 16-bit halves
    const int ly = r + 3;
    uint32_t W[7][3];
#pragma unroll
    for (int dy = 0; dy < 7; dy++)
#pragma unroll
        for (int j = 0; j < 3; j++) W[dy][j] = lds[(ly - 3 + dy) * (SM_LW / 4) + q + j];
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
        // two pixels per packed 16-bit lane pair
        short2v d[16];
        const short2v v = pair16(3, 4 + pp);
#pragma unroll
        for (int k = 0; k < 16; k++) d[k] = v - pair16(3 + cyo[k], 4 + pp + cxo[k]);
        short2v mn[16], mx[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            mn[k] = pk_min(d[k], d[(k + 1) & 15]);
            mx[k] = pk_max(d[k], d[(k + 1) & 15]);
        }
        short2v mn4[16], mx4[16];
#pragma unroll
        for (int k = 0; k < 16; k++) {
            mn4[k] = pk_min(mn[k], mn[(k + 2) & 15]);
            mx4[k] = pk_max(mx[k], mx[(k + 2) & 15]);
        }
        short2v dark = short2v{0, 0}, bright = short2v{0, 0};  // max(arc min), min(arc max)
#pragma unroll
        for (int k = 0; k < 16; k++) {
            const short2v a = pk_min(pk_min(mn4[k], mn4[(k + 4) & 15]), d[(k + 8) & 15]);
            const short2v b = pk_max(pk_max(mx4[k], mx4[(k + 4) & 15]), d[(k + 8) & 15]);
            dark = pk_max(dark, a);
            bright = pk_min(bright, b);
        }
        const short2v s = pk_max(dark, -bright);
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const int xx = x + pp + e;
            const int sv = e ? s.y : s.x;
            const bool in = xx >= 3 && xx < w - 3 && y >= 3 && y < h - 3;
            out |= (uint32_t)(in ? sv : 0) << (8 * (pp + e));
        }
    }
    *reinterpret_cast<uint32_t*>(smap + (size_t)f * smap_stride + (size_t)y * pitch + x) = out;
}

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

// ============================================================ candidates
// One workgroup per (band, frame). The band's S rows (plus one row/column of
// halo, zeroed outside the cell's detection region, where FAST has no score)
// are staged in LDS; survivors of the threshold-free NMS are written in
// row-major order and counted into the cell's S histogram.
__global__ void __launch_bounds__(256) k_adapt_cand(const uint8_t* __restrict__ smap, size_t smap_stride, int pitch,
                                                    const AdBand* __restrict__ bands, const AdCell* __restrict__ cells,
                                                    int ncells, uint32_t* __restrict__ cand, size_t cand_stride,
                                                    int* __restrict__ band_cnt, int nbands, int* __restrict__ hist) {
    __shared__ uint8_t s[(AD_BH + 2) * (AD_MAXW + 2)];
    __shared__ int sh[256];
    __shared__ int ws[16];
    const int f = blockIdx.y;
    const AdBand B = bands[blockIdx.x];
    const AdCell C = cells[B.cell];
    const int cw = C.c1 - C.c0, lw = cw + 2;
    const int rows = B.y1 - B.y0;
    const uint8_t* S = smap + (size_t)f * smap_stride;
    sh[threadIdx.x] = 0;
    // rows outer, columns across the threads: no division per staged byte
    for (int r = 0; r < rows + 2; r++) {
        const int y = B.y0 - 1 + r;
        const bool yin = y >= C.r0 && y < C.r1;
        for (int q = threadIdx.x; q < lw; q += 256) {
            const int x = C.c0 - 1 + q;
            s[r * lw + q] = (yin && x >= C.c0 && x < C.c1) ? S[(size_t)y * pitch + x] : 0;
        }
    }
    __syncthreads();
    // each thread a contiguous run of the band's pixels (row-major order is
    // kept by the scan below); (row, col) stepped, not divided, per pixel;
    // survivors of the first pass remembered in a bit mask (runs <= 32 px)
    const int npx = rows * cw;
    const int chunk = (npx + 255) / 256;
    const int i0 = min(npx, (int)threadIdx.x * chunk), i1 = min(npx, i0 + chunk);
    const int r0 = cw > 0 ? i0 / cw : 0, q0 = i0 - r0 * cw;
    auto survivor = [&](int r, int q, int* sv) -> bool {
        const uint8_t* p = s + (r + 1) * lw + (q + 1);
        const int v = p[0];
        *sv = v;
        if (v < 2) return false;
        int m = max(max(p[-lw - 1], p[-lw]), max(p[-lw + 1], p[-1]));
        m = max(m, max(max(p[1], p[lw - 1]), max(p[lw], p[lw + 1])));
        return v > m;
    };
    int cnt = 0;
    uint32_t smask = 0;
    {
        int r = r0, q = q0;
        for (int i = i0; i < i1; i++) {
            int sv;
            if (survivor(r, q, &sv)) {
                cnt++;
                atomicAdd(&sh[sv], 1);
                if (i - i0 < 32) smask |= 1u << (i - i0);
            }
            if (++q == cw) {
                q = 0;
                r++;
            }
        }
    }
    int2 tot;
    const int2 base = block_scan2i(cnt, 0, reinterpret_cast<int(*)[2]>(ws), &tot);
    uint32_t* out = cand + (size_t)f * cand_stride + B.cand_off;
    int o = base.x;
    {
        int r = r0, q = q0;
        for (int i = i0; i < i1; i++) {
            int sv = s[(r + 1) * lw + (q + 1)];
            const bool keep = (i - i0 < 32) ? ((smask >> (i - i0)) & 1u) != 0 : survivor(r, q, &sv);
            if (keep) out[o++] = ((uint32_t)sv << 24) | ((uint32_t)(B.y0 + r) << 12) | (uint32_t)(C.c0 + q);
            if (++q == cw) {
                q = 0;
                r++;
            }
        }
    }
    if (threadIdx.x == 0) band_cnt[(size_t)f * nbands + blockIdx.x] = tot.x;
    __syncthreads();
    const int hv = sh[threadIdx.x];
    if (hv) atomicAdd(&hist[((size_t)f * ncells + B.cell) * 256 + threadIdx.x], hv);
}

// ============================================================ threshold chain
// One workgroup per cell: count-above-threshold tables of FCH frames at a
// time (one wave per frame: 4 bins per lane, reverse wave scan), then the
// DetectorAdjuster chain in frame order on lane 0 (double arithmetic, as
// detectoradjuster.cpp:52-65; FastFeatureDetector::create(int) truncates).
#define AD_FCH 16
__global__ void __launch_bounds__(256) k_adapt_chain(const int* __restrict__ hist, int ncells, int nframes, AdParams P,
                                                     double* __restrict__ thresh, int* __restrict__ tsel,
                                                     int* __restrict__ nsel) {
    __shared__ int above[AD_FCH][256];
    const int c = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double th = thresh[c];
    for (int f0 = 0; f0 < nframes; f0 += AD_FCH) {
        const int nf = min(AD_FCH, nframes - f0);
        for (int fi = wv; fi < nf; fi += 4) {
            const int4 hv = reinterpret_cast<const int4*>(hist + ((size_t)(f0 + fi) * ncells + c) * 256)[lane];
            const int s3 = hv.w, s2 = hv.z + s3, s1 = hv.y + s2, s0 = hv.x + s1;
            int x = s0;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_down(x, o);
                if (lane + o < 64) x += y;
            }
            const int after = x - s0;  // bins >= 4*lane + 4
            // above[t] = #{S > t}
            above[fi][4 * lane + 0] = s1 + after;
            above[fi][4 * lane + 1] = s2 + after;
            above[fi][4 * lane + 2] = s3 + after;
            above[fi][4 * lane + 3] = after;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int fi = 0; fi < nf; fi++) {
                int it = P.escape_iters, t = 0, n = 0;
                do {
                    const int ti = (int)th;
                    t = ti < 0 ? 0 : (ti > 255 ? 255 : ti);
                    n = above[fi][t];
                    if (n < P.cell_min) {
                        th *= P.decrease_factor;  // tooFew
                        if (th < P.min_thresh) th = P.min_thresh;
                    } else if (n > P.cell_max) {
                        th *= P.increase_factor;  // tooMany
                        if (th > P.max_thresh) th = P.max_thresh;
                        break;
                    } else
                        break;
                    it--;
                } while (it > 0 && th > P.min_thresh && th < P.max_thresh);
                tsel[(size_t)(f0 + fi) * ncells + c] = t;
                nsel[(size_t)(f0 + fi) * ncells + c] = n;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) thresh[c] = th;
}

// ============================================================ std::nth_element
// libstdc++ __introselect on packed keypoints (score << 24 | y << 12 | x),
// comp(a, b) = score(a) > score(b) (ResponseComparator /
// KeypointResponseGreater): key = 255 - score ascending. Every partition runs
// on the whole workgroup: the Hoare scan pairs the k-th left stop (key >= pk)
// with the k-th right stop (key <= pk) while they have not crossed (k < k*),
// and cuts at min(L[k*], R[k*-1]) (the model checked against the real
// std::nth_element in tests/test_adaptive_model.py).
ODO_INLINE uint32_t sel_key(uint32_t e) { return 255u - (e >> 24); }

struct SelState {
    int first, last, depth, pk, ks, nl, nr, done;
    int ws[16][2];
};

ODO_INLINE void sel_swap(uint32_t* A, int i, int j) {
    const uint32_t t = A[i];
    A[i] = A[j];
    A[j] = t;
}

ODO_INLINE void sel_adjust_heap(uint32_t* A, int first, int hole, int len, uint32_t value) {
    const int top = hole;
    int child = hole;
    while (child < (len - 1) / 2) {
        child = 2 * (child + 1);
        if (sel_key(A[first + child]) < sel_key(A[first + child - 1])) child--;
        A[first + hole] = A[first + child];
        hole = child;
    }
    if ((len & 1) == 0 && child == (len - 2) / 2) {
        child = 2 * (child + 1);
        A[first + hole] = A[first + child - 1];
        hole = child - 1;
    }
    int parent = (hole - 1) / 2;
    while (hole > top && sel_key(A[first + parent]) < sel_key(value)) {
        A[first + hole] = A[first + parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    A[first + hole] = value;
}

// std::__heap_select(first, middle, last) (depth-limit fallback; one lane)
ODO_INLINE void sel_heap_select(uint32_t* A, int first, int middle, int last) {
    const int len = middle - first;
    if (len >= 2)
        for (int parent = (len - 2) / 2;; parent--) {
            sel_adjust_heap(A, first, parent, len, A[first + parent]);
            if (parent == 0) break;
        }
    for (int i = middle; i < last; ++i)
        if (sel_key(A[i]) < sel_key(A[first])) {  // __pop_heap(first, middle, i)
            const uint32_t v = A[i];
            A[i] = A[first];
            sel_adjust_heap(A, first, 0, len, v);
        }
}

ODO_INLINE void sel_insertion_sort(uint32_t* A, int first, int last) {
    if (first == last) return;
    for (int i = first + 1; i != last; ++i) {
        const uint32_t v = A[i];
        if (sel_key(v) < sel_key(A[first])) {
            for (int k = i; k > first; --k) A[k] = A[k - 1];
            A[first] = v;
        } else {
            int cur = i, next = i - 1;
            while (sel_key(v) < sel_key(A[next])) {
                A[cur] = A[next];
                cur = next;
                --next;
            }
            A[cur] = v;
        }
    }
}

// A: n elements (LDS or global); posL/posR: n ints of scratch; every thread of
// the workgroup calls this.
ODO_INLINE void block_nth_element(uint32_t* A, int n, int nth, int* posL, int* posR, SelState& S) {
    if (n <= 0 || nth >= n) return;
    const int t = threadIdx.x, T = blockDim.x;
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
                sel_heap_select(A, first, nth + 1, last);
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
            const uint32_t ka = sel_key(A[a]), kb = sel_key(A[b]), kc = sel_key(A[c]);
            int m;
            if (ka < kb) m = kb < kc ? b : (ka < kc ? c : a);
            else m = ka < kc ? a : (kb < kc ? c : b);
            sel_swap(A, first, m);
            S.pk = (int)sel_key(A[first]);
        }
        __syncthreads();
        const uint32_t pk = (uint32_t)S.pk;
        const int m = last - first - 1;
        const int chunk = (m + T - 1) / T;
        const int j0 = first + 1 + min(m, t * chunk), j1 = first + 1 + min(m, t * chunk + chunk);
        int cg = 0, cl = 0;
        for (int j = j0; j < j1; j++) {
            const uint32_t k = sel_key(A[j]);
            cg += k >= pk;
            cl += k <= pk;
        }
        int2 tot;
        const int2 base = block_scan2i(cg, cl, S.ws, &tot);
        int rg = base.x, rl = base.y;
        for (int j = j0; j < j1; j++) {
            const uint32_t k = sel_key(A[j]);
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
        for (int k = t; k < ks; k += T) sel_swap(A, posL[k], posR[k]);
        __syncthreads();
        if (t == 0) {
            int cut = ks < tot.x ? posL[ks] : last;
            if (ks > 0) cut = min(cut, posR[ks - 1]);
            if (cut <= nth) S.first = cut;
            else S.last = cut;
        }
        __syncthreads();
    }
    if (t == 0 && !S.done) sel_insertion_sort(A, S.first, S.last);
    __syncthreads();
}

// ============================================================ per-cell select
// One workgroup per (cell, frame): gather the survivors with S > t* from the
// cell's bands in order (= cv::FAST's row-major emission), keepStrongest.
__global__ void __launch_bounds__(256) k_adapt_select(const uint32_t* __restrict__ cand, size_t cand_stride,
                                                      const int* __restrict__ band_cnt, int nbands,
                                                      const AdBand* __restrict__ bands,
                                                      const AdCell* __restrict__ cells, int ncells,
                                                      const int* __restrict__ tsel, const int* __restrict__ nsel,
                                                      int max_per_cell, uint32_t* __restrict__ big,
                                                      size_t big_stride, uint32_t* __restrict__ cell_out,
                                                      int* __restrict__ cell_cnt) {
    extern __shared__ uint32_t dyn[];
    __shared__ SelState S;
    __shared__ int ws[16];
    const int c = blockIdx.x, f = blockIdx.y;
    const AdCell C = cells[c];
    const int ts = tsel[(size_t)f * ncells + c];
    const int n = nsel[(size_t)f * ncells + c];
    const bool in_lds = n <= AD_SEL_LDS;
    uint32_t* A = in_lds ? dyn : big + ((size_t)f * ncells + c) * big_stride;
    int* posL = in_lds ? reinterpret_cast<int*>(dyn + AD_SEL_LDS) : reinterpret_cast<int*>(A + C.cand_cap);
    int* posR = in_lds ? posL + AD_SEL_LDS : posL + C.cand_cap;
    int pos = 0;
    const uint32_t* fc = cand + (size_t)f * cand_stride;
    for (int b = C.band0; b < C.band1; b++) {
        const int cnt = band_cnt[(size_t)f * nbands + b];
        const uint32_t* src = fc + bands[b].cand_off;
        for (int i0 = 0; i0 < cnt; i0 += blockDim.x) {
            const int i = i0 + threadIdx.x;
            const uint32_t e = i < cnt ? src[i] : 0u;
            const bool keep = i < cnt && (int)(e >> 24) > ts;
            int tot;
            const int r = block_rank(keep, ws, &tot);
            if (keep && pos + r < n) A[pos + r] = e;
            pos += tot;
        }
    }
    const int m = min(pos, n);
    __syncthreads();
    if (m > max_per_cell) block_nth_element(A, m, max_per_cell, posL, posR, S);
    const int k = min(m, max_per_cell);
    uint32_t* out = cell_out + ((size_t)f * ncells + c) * max_per_cell;
    for (int i = threadIdx.x; i < k; i += blockDim.x) out[i] = A[i];
    if (threadIdx.x == 0) cell_cnt[(size_t)f * ncells + c] = k;
}

// ============================================================ per-frame assemble
// aggregateKeypointsPerGridCell (coordinates are already image coordinates),
// Extractor::Extract's retainBest(nFeatures) (extractor.cpp:45-46), then
// cv::ORB::compute's KeyPointsFilter::runByImageBorder(edgeThreshold=31).
__global__ void __launch_bounds__(256) k_adapt_assemble(const uint32_t* __restrict__ cell_out,
                                                        const int* __restrict__ cell_cnt, int ncells,
                                                        int max_per_cell, int retain, int w, int h,
                                                        uint32_t* __restrict__ akp, int akp_stride,
                                                        int* __restrict__ nkp, int kp_cap) {
    extern __shared__ uint32_t dyn[];
    __shared__ SelState S;
    __shared__ int ws[16];
    __shared__ int s_off[65];
    const int f = blockIdx.x;
    const int cap = ncells * max_per_cell;
    uint32_t* A = dyn;
    int* posL = reinterpret_cast<int*>(dyn + cap);
    int* posR = posL + cap;
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int c = 0; c < ncells; c++) {
            s_off[c] = acc;
            acc += cell_cnt[(size_t)f * ncells + c];
        }
        s_off[ncells] = acc;
    }
    __syncthreads();
    int n = s_off[ncells];
    for (int c = 0; c < ncells; c++) {
        const int cnt = s_off[c + 1] - s_off[c];
        const uint32_t* src = cell_out + ((size_t)f * ncells + c) * max_per_cell;
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) A[s_off[c] + i] = src[i];
    }
    __syncthreads();
    if (retain >= 0 && n > retain) {
        if (retain == 0) n = 0;
        else {
            block_nth_element(A, n, retain, posL, posR, S);
            if (threadIdx.x == 0) {
                // std::partition(begin + n_points, end, response >= ambiguous)
                // (libstdc++ bidirectional __partition)
                const uint32_t amb = A[retain - 1] >> 24;
                int first = retain, last = n;
                while (true) {
                    while (first != last && (A[first] >> 24) >= amb) ++first;
                    if (first == last) break;
                    --last;
                    while (first != last && !((A[last] >> 24) >= amb)) --last;
                    if (first == last) break;
                    sel_swap(A, first, last);
                    ++first;
                }
                S.nl = first;
            }
            __syncthreads();
            n = S.nl;
        }
    }
    // runByImageBorder: keep 31 <= x < w-31 and 31 <= y < h-31 (stable)
    const int B = 31;
    const bool ok_img = h > 2 * B && w > 2 * B;
    int o = 0;
    for (int i0 = 0; i0 < n; i0 += blockDim.x) {
        const int i = i0 + threadIdx.x;
        bool keep = false;
        uint32_t e = 0;
        if (i < n && ok_img) {
            e = A[i];
            const int x = (int)(e & 0xfff), y = (int)((e >> 12) & 0xfff);
            keep = x >= B && x < w - B && y >= B && y < h - B;
        }
        int tot;
        const int r = block_rank(keep, ws, &tot);
        if (keep && o + r < kp_cap) akp[(size_t)f * akp_stride + o + r] = e;
        o += tot;
    }
    if (threadIdx.x == 0) nkp[f] = min(o, kp_cap);
}

// ============================================================ finalize
// Four keypoints per wave, 16 lanes each: rBRIEF (16 tests per lane, one
// ballot per test group) at the fixed angle -1 deg (cos/sin precomputed on the
// host in the reference's float arithmetic); undistort + depth follow in
// k_kp_geometry (k_finalize.hip).
#define AF_KPW 4
#define AF_KPB (4 * AF_KPW)
__global__ void __launch_bounds__(256) k_adapt_finalize(const uint8_t* __restrict__ blur, size_t pyr_stride, int pitch,
                                                        const uint32_t* __restrict__ akp, int akp_stride,
                                                        const int* __restrict__ nkp, float ca, float sb,
                                                        orb_kp* __restrict__ kps, uint8_t* __restrict__ desc,
                                                        int kp_cap) {
    __shared__ uint64_t s_bal[4][16];
    const int f = blockIdx.y;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, sub = lane & 15;
    const int n = nkp[f];
    if (blockIdx.x * AF_KPB >= n) return;  // whole workgroup idle
    const int idx = blockIdx.x * AF_KPB + wave * AF_KPW + g;
    const bool valid = idx < n;
    const uint32_t key = valid ? akp[(size_t)f * akp_stride + idx] : (40u | (40u << 12));
    const int kx = (int)(key & 0xfff), ky = (int)((key >> 12) & 0xfff);
    const float a = ca, b = sb;
    const uint8_t* center = blur + (size_t)f * pyr_stride + (size_t)ky * pitch + kx;
    int tv0[16], tv1[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
        const int bit = w * 16 + sub;
        const float x0 = (float)c_apattern[4 * bit + 0], y0 = (float)c_apattern[4 * bit + 1];
        const float x1 = (float)c_apattern[4 * bit + 2], y1 = (float)c_apattern[4 * bit + 3];
        tv0[w] = center[cv_round(x0 * b + y0 * a) * pitch + cv_round(x0 * a - y0 * b)];
        tv1[w] = center[cv_round(x1 * b + y1 * a) * pitch + cv_round(x1 * a - y1 * b)];
    }
#pragma unroll
    for (int w = 0; w < 16; w++) {
        const uint64_t bal = __ballot(tv0[w] < tv1[w]);
        if (lane == 0) s_bal[wave][w] = bal;
    }
    __syncthreads();
    if (valid && sub < 8) {
        const uint32_t lo = (uint32_t)(s_bal[wave][2 * sub] >> (16 * g)) & 0xffffu;
        const uint32_t hi = (uint32_t)(s_bal[wave][2 * sub + 1] >> (16 * g)) & 0xffffu;
        reinterpret_cast<uint32_t*>(desc + ((size_t)f * kp_cap + idx) * 32)[sub] = lo | (hi << 16);
    }
    if (valid && sub == 0) {
        orb_kp* kp = kps + (size_t)f * kp_cap + idx;
        const float px = (float)kx, py = (float)ky;
        kp->x = px;
        kp->y = py;
        kp->size = 7.f;
        kp->angle = -1.f;
        kp->response = (float)((int)(key >> 24) - 1);  // cornerScore = S - 1
        kp->octave = 0;
        kp->class_id = -1;
    }
}

// ============================================================ debug: selection
// mode 0: std::nth_element(a, a + nth, a + n); mode 1: retainBest(a, nth).
__global__ void __launch_bounds__(256) k_adapt_select_dbg(uint32_t* A, int n, int nth, int mode, int* posL, int* posR,
                                                          int* n_out) {
    __shared__ SelState S;
    block_nth_element(A, n, nth, posL, posR, S);
    if (threadIdx.x == 0) {
        int m = n;
        if (mode == 1 && n > nth) {
            const uint32_t amb = A[nth - 1] >> 24;
            int first = nth, last = n;
            while (true) {
                while (first != last && (A[first] >> 24) >= amb) ++first;
                if (first == last) break;
                --last;
                while (first != last && !((A[last] >> 24) >= amb)) --last;
                if (first == last) break;
                sel_swap(A, first, last);
                ++first;
            }
            m = first;
        }
        *n_out = m;
    }
}

// ============================================================ launch wrappers
void upload_adaptive_constants() {
    hipMemcpyToSymbol(HIP_SYMBOL(c_apattern), ODO_ORB_PATTERN, sizeof(ODO_ORB_PATTERN));
}

void launch_adapt_smap(hipStream_t st, const uint8_t* pyr, size_t pyr_stride, int w, int h, int pitch, uint8_t* smap,
                       size_t smap_stride, int nframes) {
    const int tx = (pitch + SM_TW - 1) / SM_TW, ty = (h + SM_TH - 1) / SM_TH;
    hipLaunchKernelGGL(k_adapt_smap, dim3(tx * ty, nframes), dim3(256), 0, st, pyr, pyr_stride, w, h, pitch, tx, smap,
                       smap_stride);
}

void launch_adapt_cand(hipStream_t st, const uint8_t* smap, size_t smap_stride, int pitch, const AdBand* bands,
                       int nbands, const AdCell* cells, int ncells, uint32_t* cand, size_t cand_stride, int* band_cnt,
                       int* hist, int nframes) {
    hipLaunchKernelGGL(k_adapt_cand, dim3(nbands, nframes), dim3(256), 0, st, smap, smap_stride, pitch, bands, cells,
                       ncells, cand, cand_stride, band_cnt, nbands, hist);
}

void launch_adapt_chain(hipStream_t st, const int* hist, int ncells, int nframes, AdParams P, double* thresh,
                        int* tsel, int* nsel) {
    hipLaunchKernelGGL(k_adapt_chain, dim3(ncells), dim3(256), 0, st, hist, ncells, nframes, P, thresh, tsel, nsel);
}

size_t adapt_select_lds_bytes() { return (size_t)AD_SEL_LDS * 12; }

void launch_adapt_select(hipStream_t st, const uint32_t* cand, size_t cand_stride, const int* band_cnt, int nbands,
                         const AdBand* bands, const AdCell* cells, int ncells, const int* tsel, const int* nsel,
                         int max_per_cell, uint32_t* big, size_t big_stride, uint32_t* cell_out, int* cell_cnt,
                         int nframes) {
    hipLaunchKernelGGL(k_adapt_select, dim3(ncells, nframes), dim3(256), adapt_select_lds_bytes(), st, cand,
                       cand_stride, band_cnt, nbands, bands, cells, ncells, tsel, nsel, max_per_cell, big, big_stride,
                       cell_out, cell_cnt);
}

size_t adapt_assemble_lds_bytes(int ncells, int max_per_cell) { return (size_t)ncells * max_per_cell * 12; }

void launch_adapt_assemble(hipStream_t st, const uint32_t* cell_out, const int* cell_cnt, int ncells, int max_per_cell,
                           int retain, int w, int h, uint32_t* akp, int akp_stride, int* nkp, int kp_cap,
                           int nframes) {
    const size_t lds = adapt_assemble_lds_bytes(ncells, max_per_cell);
    if (lds > 64 * 1024)
        hipFuncSetAttribute((const void*)k_adapt_assemble, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_adapt_assemble, dim3(nframes), dim3(256), lds, st, cell_out, cell_cnt, ncells, max_per_cell,
                       retain, w, h, akp, akp_stride, nkp, kp_cap);
}

void launch_adapt_finalize(hipStream_t st, const uint8_t* blur, size_t pyr_stride, int pitch, const uint32_t* akp,
                           int akp_stride, const int* nkp, float ca, float sb, const uint16_t* depth,
                           size_t depth_stride, int img_w, FrameCalib cal, orb_kp* kps, uint8_t* desc, float* kun,
                           float* xyz, float* ur, int kp_cap, int nframes) {
    dim3 g((kp_cap + AF_KPB - 1) / AF_KPB, nframes);
    hipLaunchKernelGGL(k_adapt_finalize, g, dim3(256), 0, st, blur, pyr_stride, pitch, akp, akp_stride, nkp, ca, sb,
                       kps, desc, kp_cap);
    launch_kp_geometry(st, kps, nkp, depth, depth_stride, img_w, cal, kun, xyz, ur, kp_cap, nframes);
}

void launch_adapt_select_dbg(hipStream_t st, uint32_t* a, int n, int nth, int mode, int* posL, int* posR,
                             int* n_out) {
    hipLaunchKernelGGL(k_adapt_select_dbg, dim3(1), dim3(256), 0, st, a, n, nth, mode, posL, posR, n_out);
}

}  // namespace odo
