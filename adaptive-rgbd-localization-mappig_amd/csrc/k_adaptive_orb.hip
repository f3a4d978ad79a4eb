// Extractor(ORB, ORB, ADAPTIVE) for gfx950: the
// grid-adapted detector of k_adaptive.hip with the cv::ORB inner detector of
// Features/detectoradjuster.cpp:29 - cv::ORB::create(10000, 1.2f, 8, 15, 0,
// 2, HARRIS_SCORE, 31, (int)thresh)->detect(cell sub-image) - then
// Extractor::Extract's retainBest(1000) and cv::ORB::compute on the kept
// keypoints, which carry the detector's octaves (extractor.cpp:39-50).
// OpenCV 3.4 orb.cpp is restated in oracle/orb_ref.cpp (orbcv_detect,
// orb_compute_provided_levels); DESIGN.md §4 "ADAPTIVE, cv::ORB inner".
//
// As in the FAST-inner path, the threshold never touches the pixels: FAST at
// threshold t on a cell level keeps p iff S(p) > t and p passes the
// threshold-free NMS, so one S map per cell level gives the candidates of
// every threshold. Each level then keeps retainBest(2 * quota) by FAST score
// and retainBest(quota) by Harris response; quota >= 606 > gridMax 113, so a
// level that binds makes the cell's count exceed gridMax whatever the exact
// count is, and the DetectorAdjuster chain runs on sum_l min(count_l, quota_l)
// (the host checks the quota bound).
//
//   k_oa_pyr       per (frame, cell): the cell's 8-level pyramid (INTER_LINEAR,
//                  App. A.2), levels ping-ponged in LDS, written to HBM
//   k_oa_scand     per (frame, band of a cell level): S (smap4) of the band
//                  in LDS, NMS survivors in [15, w-15) x [15, h-15) in
//                  row-major order + per-level S histogram
//   k_oa_count     per (frame, cell): the chain's count table for every t
//   (k_adapt_chain) the tooFew/tooMany/good chain over the batch, in frame order
//   k_oa_select    per (frame, cell): survivors with S > t*, retainBest by FAST
//                  score, Harris responses, retainBest by Harris, keepStrongest
//                  by |response| (libstdc++ introselect, odo_select.h)
//   k_oa_assemble  per frame: cells in grid order, retainBest(1000),
//                  runByImageBorder(31), stable regroup by octave
//   k_oa_finalize  IC angle on the cell level, rBRIEF on the blurred level of
//                  the frame pyramid (samples past the level edge read the
//                  unblurred REFLECT_101 border), keypoint record
#include "odo_device.h"
#include "odo_internal.h"
#include "odo_select.h"
#include "../../include/odo_orb_pattern.h"

namespace odo {

// ============================================================ cell pyramids
// One 1024-thread workgroup per (frame, cell). Level 0 = the cell's ROI of the frame's
// gray level 0; level l = cv::resize(level l-1, INTER_LINEAR) to the getScale
// size (host). Source and destination levels alternate between two LDS
// buffers; every level is also written to the frame's cell-pyramid buffer
// (pitched rows, zero padding). Resize tables are made in LDS with the
// generic-path rules of App. A.2 (the host rules of odo_capi.cpp
// build_geometry).
// LDS = false (cells too large for the two LDS level buffers, e.g. 1280x960
// frames): every level reads its source level back from the cell-pyramid
// buffer the same workgroup wrote (L2), through the same code.
template <bool LDS>
__global__ void __launch_bounds__(1024) k_oa_pyr(const uint8_t* __restrict__ pyr, size_t pyr_stride, int gpitch,
                                                const OaCell* __restrict__ cells, const OaImg* __restrict__ imgs,
                                                int buf0, uint8_t* __restrict__ cpyr, size_t cp_stride) {
    extern __shared__ __attribute__((aligned(16))) uint8_t op_lds[];
    __shared__ ResizeX xt[1024];
    __shared__ ResizeY yt[1024];
    const int c = blockIdx.x, f = blockIdx.y;
    const OaCell C = cells[c];
    uint8_t* buf[2] = {op_lds, op_lds + buf0};
    uint8_t* out = cpyr + (size_t)f * cp_stride;
    {
        // level 0: aligned dword pairs of the frame row realigned to the cell's
        // first column (rows are pitch-aligned), bytes past the cell width zeroed
        const OaImg I = imgs[C.img0];
        const uint32_t* g = reinterpret_cast<const uint32_t*>(pyr + (size_t)f * pyr_stride + (size_t)C.rs * gpitch +
                                                              (C.cs & ~3));
        const int sh = C.cs & 3, gq = gpitch >> 2;
        const int nq = I.pitch >> 2;
        for (int i = threadIdx.x; i < I.h * nq; i += blockDim.x) {
            const int r = i / nq, q = i - r * nq;
            const uint32_t* row = g + (size_t)r * gq + q;
            uint32_t v = __builtin_amdgcn_alignbyte(row[1], row[0], sh);
            const int valid = I.w - 4 * q;  // bytes of this dword inside the cell
            if (valid < 4) v = valid <= 0 ? 0u : v & ((1u << (8 * valid)) - 1u);
            if (LDS) reinterpret_cast<uint32_t*>(buf[0])[i] = v;
            reinterpret_cast<uint32_t*>(out + I.off)[i] = v;
        }
    }
    for (int l = 1; l < OA_NLEV; l++) {
        const OaImg S = imgs[C.img0 + l - 1], D = imgs[C.img0 + l];
        const uint8_t* src = LDS ? buf[(l - 1) & 1] : out + S.off;
        uint8_t* dst = buf[l & 1];
        const double scale_x = 1. / ((double)D.w / S.w), scale_y = 1. / ((double)D.h / S.h);
        for (int dx = threadIdx.x; dx < D.w; dx += blockDim.x) {
            float fx = (float)((dx + 0.5) * scale_x - 0.5);
            int sx = cv_floor(fx);
            fx -= sx;
            if (sx < 0) {
                fx = 0;
                sx = 0;
            }
            ResizeX X;
            if (sx + 1 >= S.w) {  // past xmax: S[w-1] * 2048
                X.sx0 = X.sx1 = S.w - 1;
                X.a0 = 2048;
                X.a1 = 0;
            } else {
                X.sx0 = sx;
                X.sx1 = sx + 1;
                X.a0 = cv_round((1.f - fx) * 2048);
                X.a1 = cv_round(fx * 2048);
            }
            xt[dx] = X;
        }
        for (int dy = threadIdx.x; dy < D.h; dy += blockDim.x) {
            float fy = (float)((dy + 0.5) * scale_y - 0.5);
            const int sy = cv_floor(fy);
            fy -= sy;
            ResizeY Y;
            Y.b0 = cv_round((1.f - fy) * 2048);
            Y.b1 = cv_round(fy * 2048);
            Y.sy0 = min(max(sy, 0), S.h - 1);
            Y.sy1 = min(max(sy + 1, 0), S.h - 1);
            yt[dy] = Y;
        }
        __syncthreads();
        const int nq = D.pitch >> 2;
        for (int i = threadIdx.x; i < D.h * nq; i += blockDim.x) {
            const int r = i / nq, q = i - r * nq;
            const ResizeY Y = yt[r];
            const uint8_t* r0 = src + Y.sy0 * S.pitch;
            const uint8_t* r1 = src + Y.sy1 * S.pitch;
            uint32_t packed = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int dx = 4 * q + j;
                if (dx < D.w) {
                    const ResizeX X = xt[dx];
                    const int h0 = r0[X.sx0] * X.a0 + r0[X.sx1] * X.a1;
                    const int h1 = r1[X.sx0] * X.a0 + r1[X.sx1] * X.a1;
                    int v = (h0 * Y.b0 + h1 * Y.b1 + (1 << 21)) >> 22;
                    v = v < 0 ? 0 : (v > 255 ? 255 : v);
                    packed |= (uint32_t)v << (8 * j);
                }
            }
            if (LDS) reinterpret_cast<uint32_t*>(dst)[i] = packed;
            reinterpret_cast<uint32_t*>(out + D.off)[i] = packed;
        }
        __syncthreads();
    }
}

// ============================================================ S + candidates
// One workgroup per (band, frame). The band's image rows y0-4 .. y1+3 are
// staged in LDS (aligned dwords); S (smap4) is computed for the band's rows
// and one halo row / column on each side (rows y0-1 .. y1, columns 12 ..
// w-14: inside FAST's detection region [3, h-3), so every value is the real
// S), kept in LDS; then the survivors of the threshold-free NMS (S >= 2,
// S > all 8 neighbours) inside runByImageBorder's [15, w-15) x [15, h-15),
// in row-major order, + the level's S histogram. The S map never goes to HBM.
#define OA_X0 12  // first S column (dword aligned, <= 15 - 1)
__global__ void __launch_bounds__(256) k_oa_scand(const uint8_t* __restrict__ cpyr, size_t cp_stride,
                                                  const OaImg* __restrict__ imgs, const OaBand* __restrict__ bands,
                                                  int nimgs, uint32_t* __restrict__ cand, size_t cand_stride,
                                                  int* __restrict__ band_cnt, int nbands, int* __restrict__ hist,
                                                  int maxpitch) {
    // dynamic LDS sized for the widest cell level (maxpitch): the image rows,
    // then the S rows
    extern __shared__ __attribute__((aligned(16))) uint32_t img_l[];
    uint8_t* s = reinterpret_cast<uint8_t*>(img_l + (OA_BH + 8) * (maxpitch >> 2));
    __shared__ int sh[256];
    __shared__ int ws[16];
    const int f = blockIdx.y;
    const OaBand B = bands[blockIdx.x];
    const OaImg I = imgs[B.img];
    const int c0 = OA_EDGE, c1 = I.w - OA_EDGE;
    const int cw = c1 - c0;
    const int rows = B.y1 - B.y0;
    const int pq = I.pitch >> 2;                       // dwords per image row
    const int nq = (c1 + 1 - OA_X0 + 3) >> 2;          // S dwords per row (columns OA_X0 .. c1)
    const int lw = nq * 4;                             // S bytes per LDS row
    sh[threadIdx.x] = 0;
    {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(cpyr + (size_t)f * cp_stride + I.off +
                                                                (size_t)(B.y0 - 4) * I.pitch);
        for (int i = threadIdx.x; i < (rows + 8) * pq; i += 256) img_l[i] = src[i];
    }
    __syncthreads();
    for (int it = threadIdx.x; it < (rows + 2) * nq; it += 256) {
        const int r = it / nq, q = it - r * nq;         // S row y0-1+r, columns OA_X0 + 4q ..
        const int k = (OA_X0 >> 2) + q;                 // image dword of the 4 pixels
        uint32_t W[7][3];
#pragma unroll
        for (int dy = 0; dy < 7; dy++)
#pragma unroll
            for (int j = 0; j < 3; j++) W[dy][j] = img_l[(r + dy) * pq + min(k - 1 + j, pq - 1)];
        reinterpret_cast<uint32_t*>(s)[r * nq + q] = smap4(W);
    }
    __syncthreads();
#ifdef OA_SCAND_NO_NMS  // measurement only (wrong results): the S part alone
    if (threadIdx.x == 0) band_cnt[(size_t)f * nbands + blockIdx.x] = s[threadIdx.x] & 0;
    return;
#endif
    // NMS four pixels at a time: item (r, k) = the S dword of band row r at
    // columns OA_X0 + 4k .. +3. The 3x3 neighbourhood max of its four bytes
    // comes from byte-shifted dwords (v_alignbyte) split into (b0, b2) / (b1,
    // b3) u16 pairs and packed max; survivors are bytes with S >= 2, S > max,
    // inside [c0, c1). Contiguous runs of items per thread keep row-major order.
    const int nitem = rows * nq;
    const int chunk = (nitem + 255) / 256;
    const int i0 = min(nitem, (int)threadIdx.x * chunk), i1 = min(nitem, i0 + chunk);
    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(s);
    auto lo16 = [](uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c020c00u); };  // (b0, b2)
    auto hi16 = [](uint32_t x) { return __builtin_amdgcn_perm(0u, x, 0x0c030c01u); };  // (b1, b3)
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    auto pmax = [](uint32_t x, uint32_t y) -> uint32_t {
        const u16x2 r = __builtin_elementwise_max(*reinterpret_cast<const u16x2*>(&x), *reinterpret_cast<const u16x2*>(&y));
        return *reinterpret_cast<const uint32_t*>(&r);
    };
    // survivor mask (bit e = byte e) of item (r, k)
    auto survivors = [&](int r, int k) -> uint32_t {
        const int km = max(k - 1, 0), kp = min(k + 1, nq - 1);
        uint32_t L[3], C[3], R[3];
#pragma unroll
        for (int d = 0; d < 3; d++) {  // S rows r-1, r, r+1 = LDS rows r .. r+2
            const uint32_t* row = s32 + (r + d) * nq;
            const uint32_t a0 = row[km], a1 = row[k], a2 = row[kp];
            C[d] = a1;
            L[d] = __builtin_amdgcn_alignbyte(a1, a0, 3);  // bytes x-1 .. x+2
            R[d] = __builtin_amdgcn_alignbyte(a2, a1, 1);  // bytes x+1 .. x+4
        }
        const uint32_t mL = pmax(pmax(lo16(L[0]), lo16(L[2])), pmax(lo16(C[0]), lo16(C[2])));
        const uint32_t mlo = pmax(pmax(mL, pmax(lo16(R[0]), lo16(R[2]))), pmax(lo16(L[1]), lo16(R[1])));
        const uint32_t mH = pmax(pmax(hi16(L[0]), hi16(L[2])), pmax(hi16(C[0]), hi16(C[2])));
        const uint32_t mhi = pmax(pmax(mH, pmax(hi16(R[0]), hi16(R[2]))), pmax(hi16(L[1]), hi16(R[1])));
        const uint32_t v = C[1];
        uint32_t m = 0;
#pragma unroll
        for (int e = 0; e < 4; e++) {
            const uint32_t ve = (v >> (8 * e)) & 0xffu;
            const uint32_t me = ((e & 1 ? mhi : mlo) >> (16 * (e >> 1))) & 0xffffu;
            const int x = OA_X0 + 4 * k + e;
            m |= (uint32_t)(ve >= 2u && ve > me && x >= c0 && x < c1) << e;
        }
        return m;
    };
    int cnt = 0;
    uint64_t smask = 0;  // 4 bits per item, first 16 items of the run
    {
        int r = i0 / max(nq, 1), k = i0 - r * nq;
        for (int i = i0; i < i1; i++) {
            const uint32_t m = survivors(r, k);
            if (m) {
                cnt += __popc(m);
                const uint32_t v = s32[(r + 1) * nq + k];
#pragma unroll
                for (int e = 0; e < 4; e++)
                    if ((m >> e) & 1u) atomicAdd(&sh[(v >> (8 * e)) & 0xffu], 1);
            }
            if (i - i0 < 16) smask |= (uint64_t)m << (4 * (i - i0));
            if (++k == nq) {
                k = 0;
                r++;
            }
        }
    }
    int2 tot;
    const int2 base = block_scan2i(cnt, 0, reinterpret_cast<int(*)[2]>(ws), &tot);
    uint32_t* out = cand + (size_t)f * cand_stride + B.cand_off;
    int o = base.x;
    {
        int r = i0 / max(nq, 1), k = i0 - r * nq;
        for (int i = i0; i < i1; i++) {
            const uint32_t m = (i - i0 < 16) ? (uint32_t)(smask >> (4 * (i - i0))) & 0xfu : survivors(r, k);
            if (m) {
                const uint32_t v = s32[(r + 1) * nq + k];
#pragma unroll
                for (int e = 0; e < 4; e++)
                    if ((m >> e) & 1u)
                        out[o++] = (((v >> (8 * e)) & 0xffu) << 24) | ((uint32_t)(B.y0 + r) << 12) |
                                   (uint32_t)(OA_X0 + 4 * k + e);
            }
            if (++k == nq) {
                k = 0;
                r++;
            }
        }
    }
    if (threadIdx.x == 0) band_cnt[(size_t)f * nbands + blockIdx.x] = tot.x;
    __syncthreads();
    const int hv = sh[threadIdx.x];
    if (hv) atomicAdd(&hist[((size_t)f * nimgs + B.img) * 256 + threadIdx.x], hv);
}

// ============================================================ count tables
// Per (frame, cell): n(t) = sum_l min(#{S_l > t}, quota_l), written as a
// pseudo-histogram ph[t] = n(t-1) - n(t) (ph[0] = 0), so k_adapt_chain's
// suffix sums give back n(t) (n(255) = 0).
__global__ void __launch_bounds__(256) k_oa_count(const int* __restrict__ hist, const OaCell* __restrict__ cells,
                                                  const OaImg* __restrict__ imgs, int nimgs, int ncells,
                                                  int* __restrict__ phist) {
    __shared__ int hv[OA_NLEV][256];
    __shared__ int nt[256];
    const int c = blockIdx.x, f = blockIdx.y, t = threadIdx.x;
    const OaCell C = cells[c];
    for (int l = 0; l < OA_NLEV; l++) hv[l][t] = hist[((size_t)f * nimgs + C.img0 + l) * 256 + t];
    __syncthreads();
    int n = 0;
    for (int l = 0; l < OA_NLEV; l++) {
        int above = 0;
        for (int s2 = t + 1; s2 < 256; s2++) above += hv[l][s2];
        n += min(above, imgs[C.img0 + l].quota);
    }
    nt[t] = n;
    __syncthreads();
    phist[((size_t)f * ncells + c) * 256 + t] = t ? nt[t - 1] - n : 0;
}

// ============================================================ per-cell select
// Float responses as ascending 32-bit keys: comp(a, b) = a.response >
// b.response is key(a) < key(b) for key = ~ord(response), ord the
// order-preserving map of IEEE floats (no response is -0 or NaN).
ODO_INLINE uint32_t f_ord(float v) {
    const uint32_t u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
ODO_INLINE float f_unord(uint32_t o) { return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o); }
ODO_INLINE uint32_t key_greater(float r) { return ~f_ord(r); }
ODO_INLINE float resp_of_key(uint32_t k) { return f_unord(~k); }

struct HiKey {  // 64-bit elements ordered by their high word
    static ODO_INLINE uint32_t key(uint64_t e) { return (uint32_t)(e >> 32); }
};

// HarrisResponses (orb.cpp): 7x7 block of the 3x3 Sobel-like gradients around
// (x0, y0), integer sums, float response (-ffp-contract=off keeps the order).
ODO_INLINE float harris_at(const uint8_t* img, int pitch, int x0, int y0) {
    int a = 0, b = 0, c = 0;
    for (int i = 0; i < 7; i++) {
        const uint8_t* r0 = img + (y0 - 4 + i) * pitch;
        const uint8_t* r1 = r0 + pitch;
        const uint8_t* r2 = r1 + pitch;
#pragma unroll
        for (int j = 0; j < 7; j++) {
            const int x = x0 - 3 + j;
            const int Ix = (r1[x + 1] - r1[x - 1]) * 2 + (r0[x + 1] - r0[x - 1]) + (r2[x + 1] - r2[x - 1]);
            const int Iy = (r2[x] - r0[x]) * 2 + (r2[x - 1] - r0[x - 1]) + (r2[x + 1] - r0[x + 1]);
            a += Ix * Ix;
            b += Iy * Iy;
            c += Ix * Iy;
        }
    }
    const float scale = 1.f / ((1 << 2) * 7 * 255.f);
    const float scale_sq_sq = scale * scale * scale * scale;
    const float fa = (float)a, fb = (float)b, fc = (float)c;
    return (fa * fb - fc * fc - 0.04f * (fa + fb) * (fa + fb)) * scale_sq_sq;
}

// One workgroup per (cell, frame); its arrays live in a global scratch slice
// (sizes up to the cell's candidate capacity): A32 (level survivors), posL /
// posR (selection scratch), A64 (Harris-keyed level list, then the
// keepStrongest list), rec (the cell's keypoints, level-major). Record =
// key_greater(response) << 32 | level << 24 | y << 12 | x (level coords).
__global__ void __launch_bounds__(256) k_oa_select(const uint32_t* __restrict__ cand, size_t cand_stride,
                                                   const int* __restrict__ band_cnt, int nbands,
                                                   const OaBand* __restrict__ bands, const OaImg* __restrict__ imgs,
                                                   const OaCell* __restrict__ cells, int ncells,
                                                   const int* __restrict__ tsel, const uint8_t* __restrict__ cpyr,
                                                   size_t cp_stride, int max_per_cell, uint8_t* __restrict__ scr,
                                                   size_t scr_stride, int ncap, uint64_t* __restrict__ cell_out,
                                                   int* __restrict__ cell_cnt) {
    __shared__ SelState S;
    __shared__ int ws[16];
    __shared__ int s_n;
    const int c = blockIdx.x, f = blockIdx.y;
    const OaCell C = cells[c];
    const int ts = tsel[(size_t)f * ncells + c];
    uint8_t* base = scr + ((size_t)f * ncells + c) * scr_stride;
    uint64_t* A64 = reinterpret_cast<uint64_t*>(base);
    uint64_t* rec = A64 + ncap;
    uint32_t* A32 = reinterpret_cast<uint32_t*>(rec + ncap);
    int* posL = reinterpret_cast<int*>(A32 + ncap);
    int* posR = posL + ncap;
    const uint32_t* fc = cand + (size_t)f * cand_stride;
    const uint8_t* fp = cpyr + (size_t)f * cp_stride;
    int cnt = 0;
    for (int l = 0; l < OA_NLEV; l++) {
        const OaImg I = imgs[C.img0 + l];
        // FAST(t*) + runByImageBorder: the level's survivors with S > t*, in order
        int m = 0;
        for (int b = I.band0; b < I.band1; b++) {
            const int bc = band_cnt[(size_t)f * nbands + b];
            const uint32_t* src = fc + bands[b].cand_off;
            for (int i0 = 0; i0 < bc; i0 += blockDim.x) {
                const int i = i0 + threadIdx.x;
                const uint32_t e = i < bc ? src[i] : 0u;
                const bool keep = i < bc && (int)(e >> 24) > ts;
                int tot;
                const int r = block_rank(keep, ws, &tot);
                if (keep) A32[m + r] = e;
                m += tot;
            }
        }
        __syncthreads();
        // retainBest(2 * quota) by FAST score
        if (m > 2 * I.quota) {
            block_nth_element<uint32_t, ScoreKey>(A32, m, 2 * I.quota, posL, posR, S);
            if (threadIdx.x == 0)
                s_n = sel_partition_le<uint32_t, ScoreKey>(A32, 2 * I.quota, m, ScoreKey::key(A32[2 * I.quota - 1]));
            __syncthreads();
            m = s_n;
        }
        // Harris responses on the unblurred cell level
        const uint8_t* img = fp + I.off;
        for (int i = threadIdx.x; i < m; i += blockDim.x) {
            const uint32_t e = A32[i];
            const int x = (int)(e & 0xfff), y = (int)((e >> 12) & 0xfff);
            const float h = harris_at(img, I.pitch, x, y);
            A64[i] = ((uint64_t)key_greater(h) << 32) | ((uint32_t)l << 24) | (e & 0xffffffu);
        }
        __syncthreads();
        // retainBest(quota) by Harris response
        if (m > I.quota) {
            block_nth_element<uint64_t, HiKey>(A64, m, I.quota, posL, posR, S);
            if (threadIdx.x == 0) s_n = sel_partition_le<uint64_t, HiKey>(A64, I.quota, m, HiKey::key(A64[I.quota - 1]));
            __syncthreads();
            m = s_n;
        }
        for (int i = threadIdx.x; i < m; i += blockDim.x) rec[cnt + i] = A64[i];
        cnt += m;
        __syncthreads();
    }
    uint64_t* out = cell_out + ((size_t)f * ncells + c) * max_per_cell;
    if (cnt > max_per_cell) {
        // keepStrongest: nth_element at begin + N by |response|, erase the tail
        for (int i = threadIdx.x; i < cnt; i += blockDim.x)
            A64[i] = ((uint64_t)key_greater(fabsf(resp_of_key((uint32_t)(rec[i] >> 32)))) << 32) | (uint32_t)i;
        __syncthreads();
        block_nth_element<uint64_t, HiKey>(A64, cnt, max_per_cell, posL, posR, S);
        for (int i = threadIdx.x; i < max_per_cell; i += blockDim.x) out[i] = rec[(uint32_t)A64[i]];
    } else {
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) out[i] = rec[i];
    }
    if (threadIdx.x == 0) cell_cnt[(size_t)f * ncells + c] = min(cnt, max_per_cell);
}

// ============================================================ per-frame assemble
// aggregateKeypointsPerGridCell, retainBest(retain) by response, cv::ORB::
// compute's runByImageBorder(31) and its stable regroup by octave. Output per
// keypoint: key_greater(response) << 32 | cell << 27 | level << 24 | y << 12 | x.
__global__ void __launch_bounds__(256) k_oa_assemble(const uint64_t* __restrict__ cell_out,
                                                     const int* __restrict__ cell_cnt, const OaCell* __restrict__ cells,
                                                     int ncells, int max_per_cell, int retain, int w, int h,
                                                     OaScales sc, uint64_t* __restrict__ akp, int akp_stride,
                                                     int* __restrict__ nkp, int kp_cap) {
    extern __shared__ __attribute__((aligned(16))) uint64_t oa_dyn[];
    __shared__ SelState S;
    __shared__ int ws[16];
    __shared__ int s_off[65];
    __shared__ int s_n;
    const int f = blockIdx.x;
    const int cap = ncells * max_per_cell;
    uint64_t* rec = oa_dyn;
    uint64_t* A = rec + cap;
    int* posL = reinterpret_cast<int*>(A + cap);
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
        const uint64_t* src = cell_out + ((size_t)f * ncells + c) * max_per_cell;
        for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
            rec[s_off[c] + i] = src[i] | ((uint64_t)c << 27);
            A[s_off[c] + i] = (src[i] & 0xffffffff00000000ull) | (uint32_t)(s_off[c] + i);
        }
    }
    __syncthreads();
    if (retain >= 0 && n > retain) {
        if (retain == 0) n = 0;
        else {
            block_nth_element<uint64_t, HiKey>(A, n, retain, posL, posR, S);
            if (threadIdx.x == 0) s_n = sel_partition_le<uint64_t, HiKey>(A, retain, n, HiKey::key(A[retain - 1]));
            __syncthreads();
            n = s_n;
        }
    }
    // runByImageBorder(31) on the image coordinates, then octave-major (stable)
    const float B = 31.f;
    const bool ok_img = h > 62 && w > 62;
    int o = 0;
    for (int lv = 0; lv < OA_NLEV; lv++) {
        for (int i0 = 0; i0 < n; i0 += blockDim.x) {
            const int i = i0 + threadIdx.x;
            bool keep = false;
            uint64_t e = 0;
            if (i < n && ok_img) {
                e = rec[(uint32_t)A[i]];
                const int l = (int)((e >> 24) & 7), cc = (int)((e >> 27) & 15);
                if (l == lv) {
                    const OaCell C = cells[cc];
                    const float x = (float)(int)(e & 0xfff) * sc.s[l] + (float)C.cs;
                    const float y = (float)(int)((e >> 12) & 0xfff) * sc.s[l] + (float)C.rs;
                    keep = x >= B && x < (float)(w - 31) && y >= B && y < (float)(h - 31);
                }
            }
            int tot;
            const int r = block_rank(keep, ws, &tot);
            if (keep && o + r < kp_cap) akp[(size_t)f * akp_stride + o + r] = e;
            o += tot;
        }
    }
    if (threadIdx.x == 0) nkp[f] = min(o, kp_cap);
}

// ============================================================ finalize
// Four keypoints per wave, 16 lanes each, OF_NW waves per workgroup (the
// k_finalize_lds scheme, k_finalize.hip): each keypoint's two patches are
// staged in LDS by its 16 lanes with row-contiguous dword loads -
//   the IC disc, rows y-15..y+15 of the keypoint's cell level (always inside:
//   runByImageBorder(15)), 9 dwords each;
//   the rBRIEF window, rows cy-18..cy+18 of the frame pyramid's blurred level
//   around the centre cvRound(pt / scale), 10 dwords each, written over the
//   disc once the angle is known (its loads in flight meanwhile). A window that
//   leaves the level is staged byte by byte with computeOrbDescriptors'
//   border: the unblurred level at the REFLECT_101 position (the bordered
//   pyramid's border, which the in-place ROI blur leaves untouched).
// IC angle (ICAngles, orb.cpp): lane s sums disc rows s-15 and s+1 with
// v_dot4 against the column weights and the |v| masks; 16-lane butterfly.
// rBRIEF (computeOrbDescriptors): 16 tests per lane read as LDS bytes at the
// magic-rounded offsets (cvRound half to even), one ballot per test group.
__constant__ int c_oumax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
__constant__ float4 c_opatf[256];  // pattern test t: (x0, y0, x1, y1)

ODO_INLINE int refl101(int i, int n) {
    while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
    return i;
}

typedef float f32x2o __attribute__((ext_vector_type(2)));
#define OF_RND_MAGIC 12582912.0f  // 1.5 * 2^23
#define OF_RND_BITS 0x4B400000u
#define OF_IC_W 9
#define OF_IC_N (31 * OF_IC_W)
#define OF_BR_W 10
#define OF_BR_N (37 * OF_BR_W)
#define OF_KP_DW OF_BR_N  // the rBRIEF window overlays the IC disc
#define OF_NW 2
#define OF_KPB (4 * OF_NW)
__global__ void __launch_bounds__(64 * OF_NW) k_oa_finalize(const uint8_t* __restrict__ pyr,
                                                            const uint8_t* __restrict__ blur, size_t pyr_stride,
                                                            const LevelDesc* __restrict__ lv,
                                                            const uint8_t* __restrict__ cpyr, size_t cp_stride,
                                                            const OaImg* __restrict__ imgs,
                                                            const OaCell* __restrict__ cells, OaScales sc,
                                                            const uint64_t* __restrict__ akp, int akp_stride,
                                                            const int* __restrict__ nkp, orb_kp* __restrict__ kps,
                                                            uint8_t* __restrict__ desc, int kp_cap) {
    __shared__ uint64_t s_bal[OF_NW][16];
    __shared__ __attribute__((aligned(16))) uint32_t s_disc[16][8];
    __shared__ __attribute__((aligned(16))) uint32_t s_patch[OF_NW * 4][OF_KP_DW];
    for (int d = threadIdx.x; d < 128; d += 64 * OF_NW) {
        const int av = d >> 3, i = d & 7;
        const int um = c_oumax[av];
        uint32_t m = 0;
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int u = 4 * i + bb - 15;
            if (u >= -um && u <= um) m |= 0xffu << (8 * bb);
        }
        s_disc[av][i] = m;
    }
    const int f = blockIdx.y;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 4, sub = lane & 15;
    const int n = nkp[f];
    if (blockIdx.x * OF_KPB >= n) return;  // uniform over the workgroup
    const int kslot = wave * 4 + g;
    const int idx = blockIdx.x * OF_KPB + kslot;
    const bool valid = idx < n;
    // an invalid slot stages a dummy in-level patch (keypoint 0) and writes nothing
    const uint64_t e = akp[(size_t)f * akp_stride + (valid ? idx : 0)];
    const int cc = (int)((e >> 27) & 15), l = (int)((e >> 24) & 7);
    const int kx = (int)(e & 0xfff), ky = (int)((e >> 12) & 0xfff);
    const OaCell C = cells[cc];
    const OaImg I = imgs[C.img0 + l];
    const LevelDesc L = lv[l];
    const float s = sc.s[l];
    const float px = (float)kx * s + (float)C.cs, py = (float)ky * s + (float)C.rs;
    const float inv = 1.f / s;
    const int cy = cv_round(py * inv), cx = cv_round(px * inv);
    uint32_t* P = s_patch[kslot];
    const int sh = (kx - 15) & 3, sh2 = (cx - 18) & 3;
    const bool inside = cy >= 18 && cy + 18 < L.h && cx >= 18 && cx + 18 < L.w;  // uniform per keypoint
    {
        const uint8_t* img = cpyr + (size_t)f * cp_stride + I.off + (size_t)(ky - 15) * I.pitch + (kx - 15 - sh);
        uint32_t v[18];
#pragma unroll
        for (int j = 0; j < 18; j++) {
            const int i = min(sub + 16 * j, OF_IC_N - 1);
            const int r = i / OF_IC_W, c = i - r * OF_IC_W;
            v[j] = *reinterpret_cast<const uint32_t*>(img + (size_t)r * I.pitch + 4 * c);
        }
#pragma unroll
        for (int j = 0; j < 18; j++)
            if (sub + 16 * j < OF_IC_N) P[sub + 16 * j] = v[j];
    }
    // the rBRIEF window overlays the IC disc once the angle is known (the
    // k_finalize_lds FIN_OVERLAY scheme): its in-level dwords are loaded now and
    // held in registers, a window past the level edge is staged afterwards
    const uint8_t* bim = blur + (size_t)f * pyr_stride + L.off;
    uint32_t vbr[24];
    if (inside) {
        const uint8_t* b0 = bim + (size_t)(cy - 18) * L.pitch + (cx - 18 - sh2);
#pragma unroll
        for (int j = 0; j < 24; j++) {
            const int i = min(sub + 16 * j, OF_BR_N - 1);
            const int r = i / OF_BR_W, c = i - r * OF_BR_W;
            vbr[j] = *reinterpret_cast<const uint32_t*>(b0 + (size_t)r * L.pitch + 4 * c);
        }
    }
    __syncthreads();  // s_disc, the patches
    int m10, m01;
    {
        const bool has1 = sub < 15;
        const int v0 = sub - 15, v1 = has1 ? sub + 1 : 0;
        const uint32_t* r0 = P + (v0 + 15) * OF_IC_W;
        const uint32_t* r1 = P + (v1 + 15) * OF_IC_W;
        uint32_t w0[9], w1[9];
#pragma unroll
        for (int i = 0; i < 9; i++) {
            w0[i] = r0[i];
            w1[i] = r1[i];
        }
        const uint4* M0 = reinterpret_cast<const uint4*>(s_disc[-v0]);
        const uint4* M1 = reinterpret_cast<const uint4*>(s_disc[v1]);
        const uint4 a0 = M0[0], a1 = M0[1], b0 = M1[0], b1 = M1[1];
        const uint32_t z = has1 ? 0xffffffffu : 0u;
        const uint32_t mk0[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        const uint32_t mk1[8] = {b0.x & z, b0.y & z, b0.z & z, b0.w & z, b1.x & z, b1.y & z, b1.z & z, b1.w & z};
        uint32_t s0 = 0, s1 = 0, t = 0;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t U = (uint32_t)(4 * i + 1) | ((uint32_t)(4 * i + 2) << 8) | ((uint32_t)(4 * i + 3) << 16) |
                               ((uint32_t)(4 * i + 4) << 24);
            const uint32_t d0 = __builtin_amdgcn_alignbyte(w0[i + 1], w0[i], sh) & mk0[i];
            const uint32_t d1 = __builtin_amdgcn_alignbyte(w1[i + 1], w1[i], sh) & mk1[i];
            s0 = __builtin_amdgcn_udot4(d0, 0x01010101u, s0, false);
            s1 = __builtin_amdgcn_udot4(d1, 0x01010101u, s1, false);
            t = __builtin_amdgcn_udot4(d0, U, t, false);
            t = __builtin_amdgcn_udot4(d1, U, t, false);
        }
        m10 = (int)t - 16 * (int)(s0 + s1);
        m01 = v0 * (int)s0 + v1 * (int)s1;
    }
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
        m10 += __shfl_xor(m10, off);
        m01 += __shfl_xor(m01, off);
    }
    const float angle = fast_atan2((float)m01, (float)m10);
    __syncthreads();  // every IC disc read
    if (inside) {
#pragma unroll
        for (int j = 0; j < 24; j++)
            if (sub + 16 * j < OF_BR_N) P[sub + 16 * j] = vbr[j];
    } else {
        const uint8_t* un = pyr + (size_t)f * pyr_stride + L.off;
        uint8_t* PBw = reinterpret_cast<uint8_t*>(P);
        for (int i = sub; i < 4 * OF_BR_N; i += 16) {
            const int r = i / (4 * OF_BR_W), c = i - r * (4 * OF_BR_W);
            const int yy = cy - 18 + r, xx = cx - 18 - sh2 + c;
            PBw[i] = (yy >= 0 && yy < L.h && xx >= 0 && xx < L.w)
                         ? bim[(size_t)yy * L.pitch + xx]
                         : un[(size_t)refl101(yy, L.h) * L.pitch + refl101(xx, L.w)];
        }
    }
    __syncthreads();
    const float ang = angle * (float)(3.14159265358979323846 / 180.f);
    double sd, cd;
    sincos((double)ang, &sd, &cd);
    const float a = (float)cd, b = (float)sd;
    const f32x2o BA = {b, a}, AB = {a, b}, MAG = {OF_RND_MAGIC, OF_RND_MAGIC};
    const uint8_t* PB = reinterpret_cast<const uint8_t*>(P);
    const uint32_t cofs = (uint32_t)(18 * 4 * OF_BR_W + 18 + sh2) - OF_RND_BITS * (uint32_t)(4 * OF_BR_W + 1);
    int tv0[16], tv1[16];
#pragma unroll
    for (int w = 0; w < 16; w++) {
        const float4 Pt = c_opatf[w * 16 + sub];
        f32x2o q0 = (f32x2o){Pt.x, Pt.x} * BA + (f32x2o){Pt.y, -Pt.y} * AB;
        f32x2o q1 = (f32x2o){Pt.z, Pt.z} * BA + (f32x2o){Pt.w, -Pt.w} * AB;
        q0 = q0 + MAG;
        q1 = q1 + MAG;
        const uint32_t o0 = __float_as_uint(q0.x) * (uint32_t)(4 * OF_BR_W) + __float_as_uint(q0.y) + cofs;
        const uint32_t o1 = __float_as_uint(q1.x) * (uint32_t)(4 * OF_BR_W) + __float_as_uint(q1.y) + cofs;
        tv0[w] = PB[o0];
        tv1[w] = PB[o1];
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
        kp->x = px;
        kp->y = py;
        kp->size = (float)OA_PATCH * s;
        kp->angle = angle;
        kp->response = resp_of_key((uint32_t)(e >> 32));
        kp->octave = l;
        kp->class_id = -1;
    }
}

// ============================================================ launch wrappers
void upload_adaptive_orb_constants() {
    float4 pat[256];
    for (int t = 0; t < 256; t++)
        pat[t] = make_float4((float)ODO_ORB_PATTERN[4 * t], (float)ODO_ORB_PATTERN[4 * t + 1],
                             (float)ODO_ORB_PATTERN[4 * t + 2], (float)ODO_ORB_PATTERN[4 * t + 3]);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_opatf), pat, sizeof(pat));
}

void launch_oa_pyr(hipStream_t st, const uint8_t* pyr, size_t pyr_stride, int gpitch, const OaCell* cells, int ncells,
                   const OaImg* imgs, int buf0, int buf1, uint8_t* cpyr, size_t cp_stride, int nframes) {
    const size_t lds = (size_t)buf0 + buf1;
    if (lds + 32 * 1024 <= 160 * 1024) {
        hipFuncSetAttribute((const void*)k_oa_pyr<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k_oa_pyr<true>, dim3(ncells, nframes), dim3(1024), lds, st, pyr, pyr_stride, gpitch, cells,
                           imgs, buf0, cpyr, cp_stride);
    } else {
        hipLaunchKernelGGL(k_oa_pyr<false>, dim3(ncells, nframes), dim3(1024), 0, st, pyr, pyr_stride, gpitch, cells,
                           imgs, 0, cpyr, cp_stride);
    }
}

size_t oa_scand_lds_bytes(int maxpitch) { return (size_t)(OA_BH + 8) * maxpitch + (size_t)(OA_BH + 2) * maxpitch; }

void launch_oa_scand(hipStream_t st, const uint8_t* cpyr, size_t cp_stride, const OaImg* imgs, int nimgs,
                     const OaBand* bands, int nbands, uint32_t* cand, size_t cand_stride, int* band_cnt, int* hist,
                     int maxpitch, int nframes) {
    const size_t lds = oa_scand_lds_bytes(maxpitch);
    if (lds > 64 * 1024)
        hipFuncSetAttribute((const void*)k_oa_scand, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_oa_scand, dim3(nbands, nframes), dim3(256), lds, st, cpyr,
                       cp_stride, imgs, bands, nimgs, cand, cand_stride, band_cnt, nbands, hist, maxpitch);
}

void launch_oa_count(hipStream_t st, const int* hist, const OaCell* cells, const OaImg* imgs, int nimgs, int ncells,
                     int* phist, int nframes) {
    hipLaunchKernelGGL(k_oa_count, dim3(ncells, nframes), dim3(256), 0, st, hist, cells, imgs, nimgs, ncells, phist);
}

size_t oa_select_scratch_bytes(int ncap) { return (size_t)ncap * (8 + 8 + 4 + 4 + 4); }

void launch_oa_select(hipStream_t st, const uint32_t* cand, size_t cand_stride, const int* band_cnt, int nbands,
                      const OaBand* bands, const OaImg* imgs, const OaCell* cells, int ncells, const int* tsel,
                      const uint8_t* cpyr, size_t cp_stride, int max_per_cell, uint8_t* scr, size_t scr_stride,
                      int ncap, uint64_t* cell_out, int* cell_cnt, int nframes) {
    hipLaunchKernelGGL(k_oa_select, dim3(ncells, nframes), dim3(256), 0, st, cand, cand_stride, band_cnt, nbands, bands,
                       imgs, cells, ncells, tsel, cpyr, cp_stride, max_per_cell, scr, scr_stride, ncap, cell_out,
                       cell_cnt);
}

size_t oa_assemble_lds_bytes(int ncells, int max_per_cell) { return (size_t)ncells * max_per_cell * 24; }

void launch_oa_assemble(hipStream_t st, const uint64_t* cell_out, const int* cell_cnt, const OaCell* cells,
                        int ncells, int max_per_cell, int retain, int w, int h, OaScales sc, uint64_t* akp,
                        int akp_stride, int* nkp, int kp_cap, int nframes) {
    const size_t lds = oa_assemble_lds_bytes(ncells, max_per_cell);
    if (lds > 64 * 1024)
        hipFuncSetAttribute((const void*)k_oa_assemble, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_oa_assemble, dim3(nframes), dim3(256), lds, st, cell_out, cell_cnt, cells, ncells,
                       max_per_cell, retain, w, h, sc, akp, akp_stride, nkp, kp_cap);
}

void launch_oa_finalize(hipStream_t st, const uint8_t* pyr, const uint8_t* blur, size_t pyr_stride,
                        const LevelDesc* lv, const uint8_t* cpyr, size_t cp_stride, const OaImg* imgs,
                        const OaCell* cells, OaScales sc, const uint64_t* akp, int akp_stride, const int* nkp,
                        const uint16_t* depth, size_t depth_stride, int img_w, FrameCalib cal, orb_kp* kps,
                        uint8_t* desc, float* kun, float* xyz, float* ur, int kp_cap, int nframes) {
    dim3 g((kp_cap + OF_KPB - 1) / OF_KPB, nframes);
    hipLaunchKernelGGL(k_oa_finalize, g, dim3(64 * OF_NW), 0, st, pyr, blur, pyr_stride, lv, cpyr, cp_stride, imgs, cells, sc,
                       akp, akp_stride, nkp, kps, desc, kp_cap);
    launch_kp_geometry(st, kps, nkp, depth, depth_stride, img_w, cal, kun, xyz, ur, kp_cap, nframes);
}

}  // namespace odo
