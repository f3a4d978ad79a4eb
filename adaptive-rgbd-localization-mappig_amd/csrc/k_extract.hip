// ORB-SLAM2 extraction kernels for gfx950 (Features/orbextractor.cpp,
// Core/frame.cpp). One launch processes a batch of frames; all per-level
// geometry lives in device tables built once per image size (odo_capi.cpp).
//
//   k_gray        cvtColor(BGR2GRAY)                 frame.cpp:23
//   k_resize      ComputePyramid (INTER_LINEAR 8U)    orbextractor.cpp:833-857
//   k_fast_seg    FAST-9/16 + NMS per 30px cell       orbextractor.cpp:669-723
//   k_octree      DistributeOctTree                   orbextractor.cpp:466-663
//   k_blur        GaussianBlur 7x7 s=2 REFLECT_101    orbextractor.cpp:795-796
//   k_finalize    (k_finalize.hip) IC_Angle + rBRIEF + scale; k_kp_geometry undistort + depth
//                 orbextractor.cpp:14-85,805-811; frame.cpp:139-164,286-313
#include "odo_device.h"
#include "odo_internal.h"
#ifdef FS_STATS
#include <cstdio>
#endif

// wave priority of the extraction kernels (ODO_EXTRACT_PRIO, measurement
// builds): the pair stages' waves issue at ODO_WAVE_PRIO
#ifndef ODO_EXTRACT_PRIO
#define ODO_EXTRACT_PRIO 0
#endif
#define EXTRACT_PRIO() \
    if (ODO_EXTRACT_PRIO) __builtin_amdgcn_s_setprio(ODO_EXTRACT_PRIO)

namespace odo {

// ============================================================ gray
// gray = (B*1868 + G*9617 + R*4899 + 8192) >> 14, 4 pixels per thread; level 0
// rows are pitch-aligned (pitch = width rounded up to 16), so a quad never
// crosses a row when the width is a multiple of 4 (the generic tail handles
// the rest pixel by pixel).
__global__ void __launch_bounds__(256) k_gray(const uint8_t* __restrict__ bgr, uint8_t* __restrict__ pyr,
                                              int w, int h, int pitch, size_t in_stride, size_t pyr_stride) {
    EXTRACT_PRIO();
    const int f = blockIdx.y;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;  // quad index
    const uint8_t* src = bgr + (size_t)f * in_stride;
    uint8_t* dst = pyr + (size_t)f * pyr_stride;
    const int npix = w * h;
    const int p0 = q * 4;
    if (p0 >= npix) return;
    const int y = p0 / w, x = p0 - y * w;
    if ((w & 3) == 0) {
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + (size_t)p0 * 3);
        uint32_t w0 = s32[0], w1 = s32[1], w2 = s32[2];
        uint8_t b[12];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            b[i] = (w0 >> (8 * i)) & 0xff;
            b[4 + i] = (w1 >> (8 * i)) & 0xff;
            b[8 + i] = (w2 >> (8 * i)) & 0xff;
        }
        uint32_t out = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint32_t g = ((uint32_t)b[3 * i] * 1868u + (uint32_t)b[3 * i + 1] * 9617u + (uint32_t)b[3 * i + 2] * 4899u +
                          8192u) >> 14;
            out |= g << (8 * i);
        }
        *reinterpret_cast<uint32_t*>(dst + (size_t)y * pitch + x) = out;
    } else {
        for (int p = p0; p < p0 + 4 && p < npix; p++) {
            const uint8_t* s = src + (size_t)p * 3;
            const int yy = p / w, xx = p - yy * w;
            dst[(size_t)yy * pitch + xx] =
                (uint8_t)(((uint32_t)s[0] * 1868u + (uint32_t)s[1] * 9617u + (uint32_t)s[2] * 4899u + 8192u) >> 14);
        }
    }
}

// ============================================================ resize
// One workgroup per band of RB output rows of one frame: the source rows the
// band needs and the per-column x table are staged in LDS with 16-byte loads
// (rows are pitch-aligned), then each thread makes 4 adjacent output pixels
// from LDS byte reads and writes them as one aligned dword. Tables are
// precomputed on the host with the OpenCV generic-path rules (xmax rule
// folded into a0=2048, a1=0); bytes past the level width in the pitch are 0.
__global__ void __launch_bounds__(256) k_resize(uint8_t* __restrict__ pyr, size_t pyr_stride, int src_off,
                                                int spitch, int dst_off, int dpitch, int dw, int dh, int rb,
                                                const ResizeX* __restrict__ xt, const ResizeY* __restrict__ yt) {
    EXTRACT_PRIO();
    extern __shared__ __attribute__((aligned(16))) uint8_t rz_lds[];
    const int f = blockIdx.y;
    const int y0 = blockIdx.x * rb;
    const int nrow = min(rb, dh - y0);
    const int t = threadIdx.x;
    uint8_t* base = pyr + (size_t)f * pyr_stride;
    const int sy_lo = yt[y0].sy0, sy_hi = yt[y0 + nrow - 1].sy1;
    const int srows = sy_hi - sy_lo + 1;
    const int nq = (dw + 3) >> 2;
    ResizeX* xs = reinterpret_cast<ResizeX*>(rz_lds);
    uint8_t* rows = rz_lds + (size_t)nq * 4 * sizeof(ResizeX);
    for (int i = t; i < dw; i += 256) xs[i] = xt[i];
    {
        const uint4* src = reinterpret_cast<const uint4*>(base + src_off + (size_t)sy_lo * spitch);
        uint4* dstl = reinterpret_cast<uint4*>(rows);
        const int n16 = srows * (spitch >> 4);
        for (int i = t; i < n16; i += 256) dstl[i] = src[i];
    }
    __syncthreads();
    const float inv_nq = 1.0f / (float)nq;
    const int items = nrow * nq;
    for (int it = t; it < items; it += 256) {
        const int r = (int)(((float)it + 0.5f) * inv_nq);
        const int q = it - r * nq;
        const ResizeY Y = yt[y0 + r];
        // 32-bit LDS offsets and 24-bit multiplies (pixels <= 255, taps <= 2048,
        // h <= 522240): left to size_t / int the compiler emits quarter-rate
        // v_mad_u64_u32 / v_mul_lo_u32 for every tap
        const uint8_t* r0 = rows + (uint32_t)__umul24((uint32_t)(Y.sy0 - sy_lo), (uint32_t)spitch);
        const uint8_t* r1 = rows + (uint32_t)__umul24((uint32_t)(Y.sy1 - sy_lo), (uint32_t)spitch);
        const uint32_t b0 = (uint32_t)Y.b0, b1 = (uint32_t)Y.b1;
        uint32_t packed = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int dx = 4 * q + j;
            if (dx < dw) {
                const ResizeX X = xs[dx];
                const uint32_t a0 = (uint32_t)X.a0, a1 = (uint32_t)X.a1;
                const uint32_t h0 = __umul24(r0[X.sx0], a0) + __umul24(r0[X.sx1], a1);
                const uint32_t h1 = __umul24(r1[X.sx0], a0) + __umul24(r1[X.sx1], a1);
                const uint32_t v = (__umul24(h0, b0) + __umul24(h1, b1) + (1u << 21)) >> 22;
                packed |= min(v, 255u) << (8 * j);
            }
        }
        *reinterpret_cast<uint32_t*>(base + dst_off + (size_t)(y0 + r) * dpitch + 4 * q) = packed;
    }
}

// ============================================================ FAST per cell-row segment
// ComputeKeyPointsOctTree's FAST part (orbextractor.cpp:669-723): every cell
// ROI runs cv::FAST(th = iniThFAST, nonmax), and again at minThFAST when it
// kept nothing (FAST_t<16> + cornerScore<16>, NMS strictly greater than the 8
// neighbours inside the ROI's detection area).
//
// One 256-thread workgroup per segment: up to FS_NCM consecutive cells of one
// cell row of one level (FastSeg, host table). The cells' ROIs overlap only
// in their 3-pixel margins and their detection areas tile the row, so the
// segment stages the union of its ROIs in LDS once (16-byte loads) and runs
// each phase over the whole segment:
//   1. compass pre-filter on 4 pixels per item (pixels 0/4/8/12 of the circle:
//      any 9-arc holds two adjacent compass points of its sign), survivors
//      appended to a per-wave ring in LDS; every 128 survivors the wave runs
//   2. the segment test + cornerScore, two per lane in packed 16-bit lanes
//      (corner iff the threshold-free S > th; score = S - 1), scores into an
//      LDS map, corners appended to the segment's corner list;
//   3. NMS per corner against the 8 neighbours that lie in the corner's own
//      cell (a neighbour across a cell boundary is outside that cell's ROI
//      detection area, i.e. 0 in its FAST score buffer); kept corners set a
//      bit in a per-row bitmap and count per (row, cell);
//   4. per cell an exclusive scan of the row counts; a kept corner's slot in
//      its cell's list = the kept corners of its cell in earlier rows + the
//      bits left of it in its row inside the cell: the cell's row-major order,
//      with no ordered compaction anywhere.
// Cells that kept nothing run the four phases again at minThFAST over their
// own quads only. Scores do not depend on the threshold (S - 1 for any corner),
// so the map is not cleared for the second pass.
// (Until round 4: one wave per cell ROI, staged per cell with its halo, with
// per-cell setup and ordered compactions: 988 VALU + 510 SALU per cell.)
// the Bresenham circle of radius 3 (FAST_t<16>'s pixel order)
constexpr int kCircleDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
constexpr int kCircleDy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
#define FS_TH 256
#define FS_RING 512  // survivors per wave ring (u16 offsets): <= 127 pending + 256 per compass step
#define FS_RSTRIDE (FS_RING + 8)  // a wave's ring + its trash slot (entry FS_RING), 16-byte multiple
#ifndef FS_APPEND
#define FS_APPEND 1  // the ring append by per-pixel ballots (1) or a DPP prefix sum (0)
#endif
#define FS_CL 1024   // corner list (a level-0 segment of 7 cells: ~270); beyond it NMS and placement scan the score map

ODO_INLINE void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#ifdef FS_STATS
// measurement build only: work counters of k_fast_seg, printed per launch
__device__ unsigned long long fs_stats[8];
#define FS_STAT(i, v) atomicAdd(&fs_stats[i], (unsigned long long)(v))
#else
#define FS_STAT(i, v) ((void)0)
#endif
// a quad's 4-bit pixel mask in the compass's layout: pixel i at bit 8i + 7
ODO_INLINE uint32_t fs_msb_mask(uint32_t b4) {
    return ((b4 & 1u) << 7) | ((b4 & 2u) << 14) | ((b4 & 4u) << 21) | ((b4 & 8u) << 28);
}
// inclusive prefix sum over the wave's lanes (DPP: row shifts, then the row
// totals broadcast into the rows above)
ODO_INLINE int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}
struct FastMisc {
    int ncl, ovf, nl;
    int tot[FS_NCM], retry[FS_NCM];
};

__global__ void __launch_bounds__(FS_TH) k_fast_seg(const uint8_t* __restrict__ pyr, size_t pyr_stride,
                                                   const FastSeg* __restrict__ segs, const LevelDesc* __restrict__ lv,
                                                   uint32_t* __restrict__ cand, int* __restrict__ cand_cnt, int ncells,
                                                   int cell_cap, int ini_th, int min_th, FastLds LO) {
    EXTRACT_PRIO();
    extern __shared__ __attribute__((aligned(16))) uint8_t fs_lds[];
    const FastSeg G = segs[blockIdx.x];
    const int f = blockIdx.y;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint8_t* const roi = fs_lds;
    const uint32_t* const roi32 = reinterpret_cast<const uint32_t*>(fs_lds);
    uint8_t* const score = fs_lds + LO.img;
    uint16_t* const ring = reinterpret_cast<uint16_t*>(fs_lds + LO.ring) + wave * FS_RSTRIDE;
    uint16_t* const clist = reinterpret_cast<uint16_t*>(fs_lds + LO.clist);
    uint32_t* const bits = reinterpret_cast<uint32_t*>(fs_lds + LO.bits);
    int* const cnt = reinterpret_cast<int*>(fs_lds + LO.cnt);
    uint2* const qlist = reinterpret_cast<uint2*>(fs_lds + LO.qlist);  // (pixel mask, 4 m)
    FastMisc& M = *reinterpret_cast<FastMisc*>(fs_lds + LO.misc);
    const LevelDesc L = lv[G.level];
    const int R = G.rows, cols = G.cols, BW = G.bw, wcell = G.wcell, nc = G.ncell;
    constexpr int RS = FS_RS, RS4 = RS >> 2;
    const int sh = G.x0 & 15;  // staged from the 16-byte column below x0: pixel (r, x) at byte r*RS + sh + x
    {
        const uint4* src = reinterpret_cast<const uint4*>(pyr + (size_t)f * pyr_stride + L.off +
                                                          (size_t)G.y0 * L.pitch + (G.x0 & ~15));
        const int nw = (sh + cols + 15) >> 4, p16 = L.pitch >> 4;
        const int rstep = FS_TH / nw, k = t % nw, r0 = t / nw;
        if (r0 < rstep)
            for (int r = r0; r < R; r += rstep)
                reinterpret_cast<uint4*>(roi + r * RS)[k] = src[__umul24((uint32_t)r, (uint32_t)p16) + (uint32_t)k];
        for (int i = t; i < (R * RS) >> 4; i += FS_TH) reinterpret_cast<uint4*>(score)[i] = uint4{0, 0, 0, 0};
        for (int i = t; i < R * BW; i += FS_TH) bits[i] = 0;
        for (int i = t; i < R * FS_NCM; i += FS_TH) cnt[i] = 0;
        if (t == 0) M.ncl = 0, M.ovf = 0;
    }
    const int drows = R - 6;
    const int m0 = (sh + 3) >> 2, m1 = (sh + cols - 4) >> 2;
    {
        // the first pass's quads per detection row: (its detection pixels
        // (fs_msb_mask), byte column 4 m)
        const uint32_t mlo = (0xFu << (sh + 3 - 4 * m0)) & 0xFu, mhi = (1u << (sh + cols - 3 - 4 * m1)) - 1u;
        if (t <= m1 - m0) {
            const int m = m0 + t;
            qlist[t] = uint2{fs_msb_mask((t == 0 ? mlo : 0xFu) & (m == m1 ? mhi : 0xFu)), 4u * (uint32_t)m};
        }
    }
    __syncthreads();
    const float inv_w = 1.0f / (float)wcell;
    uint32_t* const out = cand + ((size_t)f * ncells + G.ci0) * cell_cap;
    typedef short s16x2 __attribute__((ext_vector_type(2)));
    for (int pass = 0; pass < 2; pass++) {
        const int th = pass == 0 ? ini_th : min_th;
        const int thc = th < 0 ? 0 : (th > 255 ? 255 : th);
        const int NL = pass == 0 ? m1 - m0 + 1 : M.nl;  // quads per detection row (qlist)
        const int items = drows > 0 && cols > 6 && NL > 0 ? drows * NL : 0;
        if (t == 0) FS_STAT(pass, items);
        // ---- 1 + 2: compass, ring, segment test
        {
            const s16x2 thv = {(short)thc, (short)thc};
            // item it = (detection row ii, quad kk): ii = (it + 0.5) / NL in
            // float (it < 2^13, so the error stays far below the 0.5 / NL margin)
            const float inl = NL > 0 ? 1.0f / (float)NL : 0.0f, inl_h = 0.5f * inl;
            int head = 0, tail = 0;
            // segment test + cornerScore of ring entries [h, h + n), two per lane
            auto seg_test = [&](int h, int n) {
                const int i0 = 2 * lane, i1 = i0 + 1;
                bool c0 = false, c1 = false;
                int o0 = 0, o1 = 0;
                if (i0 < n) {
                    o0 = ring[(h + i0) & (FS_RING - 1)];
                    o1 = i1 < n ? ring[(h + i1) & (FS_RING - 1)] : o0;
                    const s16x2 vv = {(short)roi[o0], (short)roi[o1]};
                    // from the circle's top-left corner: every offset a
                    // non-negative immediate of the LDS reads (the empty asm
                    // keeps the compiler from folding the corner back into them)
                    int a0 = o0 - 3 * RS - 3, a1 = o1 - 3 * RS - 3;
                    asm("" : "+v"(a0), "+v"(a1));
                    const uint8_t* const q0 = roi + a0;
                    const uint8_t* const q1 = roi + a1;
                    s16x2 d[16];
#pragma unroll
                    for (int k = 0; k < 16; k++) {
                        const int off = (kCircleDy[k] + 3) * RS + kCircleDx[k] + 3;
                        s16x2 c;
                        c.x = (short)q0[off];
                        c.y = (short)q1[off];
                        d[k] = vv - c;
                    }
                    // best 9-arc min / max: arcs k, k+1 (k even) share the run
                    // d[k+1 .. k+8] (odd 2-, 4-, 8-runs)
                    s16x2 mn2[8], mx2[8], mn4[8], mx4[8];
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const int j = 2 * q + 1;
                        mn2[q] = __builtin_elementwise_min(d[j], d[(j + 1) & 15]);
                        mx2[q] = __builtin_elementwise_max(d[j], d[(j + 1) & 15]);
                    }
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        mn4[q] = __builtin_elementwise_min(mn2[q], mn2[(q + 1) & 7]);
                        mx4[q] = __builtin_elementwise_max(mx2[q], mx2[(q + 1) & 7]);
                    }
                    s16x2 dk = s16x2{-32768, -32768}, br = s16x2{32767, 32767};
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const int k = 2 * q;
                        const s16x2 m8 = __builtin_elementwise_min(mn4[q], mn4[(q + 2) & 7]);
                        const s16x2 x8 = __builtin_elementwise_max(mx4[q], mx4[(q + 2) & 7]);
                        dk = __builtin_elementwise_max(
                            dk, __builtin_elementwise_min(m8, __builtin_elementwise_max(d[k], d[(k + 9) & 15])));
                        br = __builtin_elementwise_min(
                            br, __builtin_elementwise_max(x8, __builtin_elementwise_min(d[k], d[(k + 9) & 15])));
                    }
                    const s16x2 sc = __builtin_elementwise_max(dk, -br);
                    c0 = sc.x > thc;
                    c1 = i1 < n && sc.y > thc;
                    if (c0) score[o0] = (uint8_t)(sc.x - 1);
                    if (c1) score[o1] = (uint8_t)(sc.y - 1);
                }
                const uint64_t b0 = __ballot(c0), b1 = __ballot(c1);
                const int nco = __popcll(b0) + __popcll(b1);
                if (lane == 0) FS_STAT(3, 1);
                if (nco) {
                    int cb = 0;
                    if (lane == 0) cb = atomicAdd(&M.ncl, nco);
                    cb = __shfl(cb, 0);
                    const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b0, 0)) +
                                    (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(b1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b1, 0));
                    const int p0 = cb + pre, p1 = p0 + (c0 ? 1 : 0);
                    if (c0) { if (p0 < FS_CL) clist[p0] = (uint16_t)o0; else M.ovf = 1; }
                    if (c1) { if (p1 < FS_CL) clist[p1] = (uint16_t)o1; else M.ovf = 1; }
                }
            };
            for (int base = wave * 64; base < items; base += FS_TH) {
                uint32_t pass4 = 0;  // bit 8i + 7: pixel 4m+i survives
                int qoff = 0;
                const int it = base + lane;
                if (it < items) {
                    const int ii = (int)__builtin_fmaf((float)it, inl, inl_h);
                    const int kk = it - __mul24(ii, NL);
                    const uint2 e = qlist[kk];
                    int wb = (int)__umul24((uint32_t)ii, (uint32_t)RS) + (int)e.y;  // 3 rows above the quad: offsets >= 0
                    asm("" : "+v"(wb));
                    qoff = wb + 3 * RS;
                    const uint32_t* w = reinterpret_cast<const uint32_t*>(roi + wb);
                    const uint32_t Cw = w[3 * RS4], Uw = w[0], Dw = w[6 * RS4];
                    const uint32_t Lw = __builtin_amdgcn_alignbyte(Cw, w[3 * RS4 - 1], 1);
                    const uint32_t Rw = __builtin_amdgcn_alignbyte(w[3 * RS4 + 1], Cw, 3);
                    uint32_t hm[2];
#pragma unroll
                    for (int hh = 0; hh < 2; hh++) {
                        const uint32_t sel = hh ? 0x0c030c02u : 0x0c010c00u;
                        s16x2 v, a0, a4, a8, a12;
                        *reinterpret_cast<uint32_t*>(&v) = __builtin_amdgcn_perm(0u, Cw, sel);
                        *reinterpret_cast<uint32_t*>(&a0) = __builtin_amdgcn_perm(0u, Dw, sel);   // circle 0: +3 rows
                        *reinterpret_cast<uint32_t*>(&a4) = __builtin_amdgcn_perm(0u, Rw, sel);   // circle 4: +3 cols
                        *reinterpret_cast<uint32_t*>(&a8) = __builtin_amdgcn_perm(0u, Uw, sel);   // circle 8: -3 rows
                        *reinterpret_cast<uint32_t*>(&a12) = __builtin_amdgcn_perm(0u, Lw, sel);  // circle 12: -3 cols
                        // two adjacent compass points darker than v - th:
                        // max(min(a0, a8), min(a4, a12)) < v - th; brighter:
                        // min(max(a0, a8), max(a4, a12)) > v + th (sign bits)
                        const s16x2 dk = __builtin_elementwise_max(__builtin_elementwise_min(a0, a8),
                                                                   __builtin_elementwise_min(a4, a12));
                        const s16x2 bk = __builtin_elementwise_min(__builtin_elementwise_max(a0, a8),
                                                                   __builtin_elementwise_max(a4, a12));
                        const s16x2 t1 = dk - (v - thv), t2 = (v + thv) - bk;
                        hm[hh] = *reinterpret_cast<const uint32_t*>(&t1) | *reinterpret_cast<const uint32_t*>(&t2);
                    }
                    // pixel i's sign bit (bit 15 / 31 of half i / 2) to bit 8i + 7
                    pass4 = __builtin_amdgcn_perm(hm[1], hm[0], 0x07050301u) & e.x;
                }
#if FS_APPEND
                // append to the ring (any order): pixel 0 of every lane's quad
                // in lane order, then pixel 1, ...: a pixel's slot is the tail
                // plus the survivors before it in that order (one ballot per
                // pixel, mbcnt with the running tail as its addend). Every lane
                // writes four entries, a pixel that did not survive to the
                // wave's trash slot (no divergent branches). Until round 6:
                // a DPP prefix sum of the lanes' counts and per-lane popcounts
                // (the select takes the ballot itself as its lane mask: bit l
                // of the ballot is lane l's condition)
                uint32_t pos = (uint32_t)tail;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const bool sv = (pass4 >> (8 * k + 7)) & 1u;
                    const uint64_t bk = __ballot(sv);
                    const uint32_t slot =
                        __builtin_amdgcn_mbcnt_hi((uint32_t)(bk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bk, pos)) &
                        (FS_RING - 1);
                    uint32_t at;
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(at) : "v"((uint32_t)FS_RING), "v"(slot), "s"(bk));
                    ring[at] = (uint16_t)(qoff + k);
                    pos += (uint32_t)__popcll(bk);
                }
                tail = (int)pos;
#else
                // append to the ring (any order): this lane's survivors after
                // those of the lanes below (a DPP prefix sum of the counts)
                const int c = __builtin_popcount(pass4);
                const int incl = wave_incl_scan(c);
                const int pos = tail + incl - c;
                // every lane writes four entries: pixel k of the quad to its
                // ring slot if it survived, else to the wave's trash slot (no
                // divergent branches)
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const int slot = (pos + __builtin_popcount(pass4 & ((1u << (8 * k)) - 1u))) & (FS_RING - 1);
                    ring[(pass4 >> (8 * k + 7)) & 1u ? slot : FS_RING] = (uint16_t)(qoff + k);
                }
                tail += __builtin_amdgcn_readlane(incl, 63);
#endif
                if (tail - head >= 128) {
                    wave_lds_sync();
                    do {
                        seg_test(head, 128);
                        head += 128;
                    } while (tail - head >= 128);
                    wave_lds_sync();
                }
            }
            if (lane == 0) FS_STAT(2, tail);
            if (tail > head) {
                wave_lds_sync();
                seg_test(head, tail - head);
            }
        }
        __syncthreads();
        // ---- 3: NMS of this pass's corners (the list, or the score map over
        //         the pass's quads when the list overflowed)
        const bool ovf = M.ovf != 0;
        const int ncl = min(M.ncl, FS_CL);
        if (t == 0) FS_STAT(4, M.ncl), FS_STAT(5, ovf ? 1 : 0);
        // corner at ROI byte offset o -> (row, segment x, cell) and its cell's
        // detection columns [xl, xh) in segment x
        auto locate = [&](int o, int& r, int& xs, int& jl, int& xl, int& xh) {
            r = o / RS;
            xs = (o - r * RS) - sh;
            jl = (int)(((float)(xs - 3) + 0.5f) * inv_w);
            xl = 3 + jl * wcell;
            xh = min(xl + wcell, cols - 3);
        };
        auto nms = [&](int o) {
            int so = o - RS - 1;  // the 3x3 block's top-left
            asm("" : "+v"(so));
            const uint8_t* const sb = score + so;
            const int sc = sb[RS + 1];
            int r, xs, jl, xl, xh;
            locate(o, r, xs, jl, xl, xh);
            // all eight neighbours read; a side column counts only inside the cell
            const int nmid = max((int)sb[1], (int)sb[2 * RS + 1]);
            const int nl = max(max((int)sb[0], (int)sb[RS]), (int)sb[2 * RS]);
            const int nr = max(max((int)sb[2], (int)sb[RS + 2]), (int)sb[2 * RS + 2]);
            const int nb = max(nmid, max(xs - 1 >= xl ? nl : 0, xs + 1 < xh ? nr : 0));
            if (sc > nb) {
                atomicOr(&bits[r * BW + (xs >> 5)], 1u << (xs & 31));
                atomicAdd(&cnt[r * FS_NCM + jl], 1);
            }
        };
        // the pass's quads as (row, quad) items, for the overflow scans
        auto scan = [&](auto&& fn) {
            for (int it = t; it < items; it += FS_TH) {
                const int ii2 = it / NL, kk2 = it - ii2 * NL;
                const uint2 e = qlist[kk2];
                const uint32_t msk = e.x;
                const int qo = (3 + ii2) * RS + (int)e.y;
                for (int b = 0; b < 4; b++)
                    if (((msk >> (8 * b + 7)) & 1u) && score[qo + b]) fn(qo + b);
            }
        };
        if (!ovf)
            for (int i = t; i < ncl; i += FS_TH) nms(clist[i]);
        else
            scan(nms);
        __syncthreads();
        // ---- 4: per cell, exclusive scan of the kept counts over the rows:
        //         wave w takes cells w, w + 4, ..., a lane per detection row
        //         (drows <= 64: the host checks rows <= 70)
        for (int j = wave; j < nc; j += FS_TH / 64) {
            if (pass == 1 && !M.retry[j]) continue;  // uniform per wave
            const int r = 3 + lane;
            const int v = lane < drows ? cnt[r * FS_NCM + j] : 0;
            int incl = v;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(incl, o);
                if (lane >= o) incl += y;
            }
            if (lane < drows) cnt[r * FS_NCM + j] = incl - v;
            if (lane == 63) M.tot[j] = incl;
        }
        __syncthreads();
        auto place = [&](int o) {
            int r, xs, jl, xl, xh;
            locate(o, r, xs, jl, xl, xh);
            const uint32_t* row = bits + r * BW;
            if (!((row[xs >> 5] >> (xs & 31)) & 1u)) return;
            int rank = cnt[r * FS_NCM + jl];
            // kept corners of the cell left of xs in this row: words wl .. wl + nwd
            // (a cell spans at most four words; the words past it are masked off)
            const int wl = xl >> 5, nwd = (xs >> 5) - wl;
            const uint32_t hm = (1u << (xs & 31)) - 1u;
#pragma unroll
            for (int i = 0; i < 4; i++) {
                uint32_t v = row[wl + i];
                if (i == 0) v &= ~0u << (xl & 31);
                v &= i < nwd ? ~0u : (i == nwd ? hm : 0u);
                rank += __builtin_popcount(v);
            }
            if (rank < cell_cap)
                out[(size_t)jl * cell_cap + rank] = ((uint32_t)score[o] << 24) |
                                                    ((uint32_t)(r + G.y0 - 16) << 12) | (uint32_t)(xs + G.x0 - 16);
        };
        if (!ovf)
            for (int i = t; i < ncl; i += FS_TH) place(clist[i]);
        else
            scan(place);
        // ---- cells that kept nothing: their quads, for the minThFAST pass
        if (pass == 0) {
            if (t < nc) M.retry[t] = M.tot[t] == 0;
            __syncthreads();
            if (t < nc && M.retry[t]) FS_STAT(6, 1);
            if (t == 0) FS_STAT(7, nc);
            if (t < nc) {
                const int xa = sh + 3 + t * wcell, xe = sh + min(3 + (t + 1) * wcell, cols - 3);
                if (M.retry[t]) {
                    int at = 0;  // entries of the retry cells before this one
                    for (int j = 0; j < t; j++)
                        if (M.retry[j]) {
                            const int ja = sh + 3 + j * wcell, je = sh + min(3 + (j + 1) * wcell, cols - 3);
                            at += ((je - 1) >> 2) - (ja >> 2) + 1;
                        }
                    for (int m = xa >> 2; m <= (xe - 1) >> 2; m++) {
                        const int lo = max(xa - 4 * m, 0), hi = min(xe - 4 * m, 4);
                        qlist[at++] = uint2{fs_msb_mask((0xFu << lo) & ((1u << hi) - 1u)), 4u * (uint32_t)m};
                    }
                } else {
                    cand_cnt[(size_t)f * ncells + G.ci0 + t] = min(M.tot[t], cell_cap);
                }
            }
            if (t == 0) {
                int n = 0;
                for (int j = 0; j < nc; j++)
                    if (M.retry[j]) {
                        const int ja = sh + 3 + j * wcell, je = sh + min(3 + (j + 1) * wcell, cols - 3);
                        n += ((je - 1) >> 2) - (ja >> 2) + 1;
                    }
                M.nl = n;
                M.ncl = 0;
                M.ovf = 0;
            }
            __syncthreads();
            if (M.nl == 0) return;  // uniform: no cell to retry
        } else if (t < nc && M.retry[t]) {
            cand_cnt[(size_t)f * ncells + G.ci0 + t] = min(M.tot[t], cell_cap);
        }
    }
}

// ============================================================ octree
// DistributeOctTree as a parallel restatement: the std::list is an array in
// list order rebuilt every pass with scans; push_front order, creation order
// (the pinned tie-break for the (size, pointer) sort) and "first max wins"
// are reproduced exactly.
struct ONode {
    int16_t x0, y0, x1, y1;
    int32_t cnt;
    int32_t seq;
};

#ifndef OT_THREADS
#define OT_THREADS 256  // threads per (frame, level) workgroup
#endif

// The workgroup's keys k = t, t + OT_THREADS, ... in batches of OT_KB per
// thread: ld(k, u) issues a batch's global loads (keys / knode / kquad live in
// HBM scratch) before pr(k, u) consumes them, so a pass over the keys waits
// one memory latency per batch instead of one per key (round 5)
#ifndef OT_KB
#define OT_KB 8
#endif
#ifndef OT_RANK_MAX
#define OT_RANK_MAX 512  // phase 2's node ranks counted (not sorted) up to this many entries
#endif
template <typename Ld, typename Pr>
ODO_INLINE void ot_keys(int n, int t, Ld&& ld, Pr&& pr) {
    for (int k0 = t; k0 < n; k0 += OT_THREADS * OT_KB) {
#pragma unroll
        for (int u = 0; u < OT_KB; u++)
            if (k0 + u * OT_THREADS < n) ld(k0 + u * OT_THREADS, u);
#pragma unroll
        for (int u = 0; u < OT_KB; u++)
            if (k0 + u * OT_THREADS < n) pr(k0 + u * OT_THREADS, u);
    }
}

// vSizeAndPointerToNode entry: sorts by (size, creation seq); low 16 bits carry
// the node's list position (never compared: seq is unique).
ODO_INLINE uint64_t ot_key(int cnt, int seq, int pos) {
    return ((uint64_t)(uint32_t)cnt << 40) | ((uint64_t)(uint32_t)(seq & 0xFFFFFF) << 16) | (uint64_t)(pos & 0xFFFF);
}

// Block-wide exclusive scans in threadIdx order: DPP wave scans
// (wave_incl_scan), then the wave totals (tmp: OT_THREADS/64 ints per value)
// in one LDS step. (Until round 5 the wave scans were __shfl_up chains: six
// dependent ds_bpermute round trips per scan.)
ODO_INLINE int block_exclusive_scan(int v, int* tmp, int* total) {
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int x = wave_incl_scan(v);
    if (lane == 63) tmp[wave] = x;
    __syncthreads();
    int base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < OT_THREADS / 64; w++) {
        const int sw = tmp[w];
        if (w < wave) base += sw;
        tot += sw;
    }
    *total = tot;
    __syncthreads();
    return base + x - v;
}
// two values at once (tmp: 2 * OT_THREADS/64 ints)
ODO_INLINE int2 block_exclusive_scan2(int a, int b, int* tmp, int2* total) {
    constexpr int NWV = OT_THREADS / 64;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int xa = wave_incl_scan(a), xb = wave_incl_scan(b);
    if (lane == 63) tmp[wave] = xa, tmp[NWV + wave] = xb;
    __syncthreads();
    int ba = 0, bb = 0, ta = 0, tb = 0;
#pragma unroll
    for (int w = 0; w < NWV; w++) {
        const int sa = tmp[w], sb = tmp[NWV + w];
        if (w < wave) ba += sa, bb += sb;
        ta += sa;
        tb += sb;
    }
    *total = int2{ta, tb};
    __syncthreads();
    return int2{ba + xa - a, bb + xb - b};
}

__global__ void __launch_bounds__(OT_THREADS) k_octree(const uint32_t* __restrict__ cand,
                                                       const int* __restrict__ cand_cnt, const LevelDesc* __restrict__ lv,
                                                       int ncells, int cell_cap, int nlevels,
                                                       uint32_t* __restrict__ keys_g, int32_t* __restrict__ knode_g,
                                                       uint8_t* __restrict__ kquad_g, size_t keys_stride_frame,
                                                       uint32_t* __restrict__ okp, int* __restrict__ ocnt, int okp_stride,
                                                       int node_cap) {
    EXTRACT_PRIO();
#ifdef ODO_OCTREE_PRIO
    __builtin_amdgcn_s_setprio(ODO_OCTREE_PRIO);  // tuning: the barrier-bound octree's waves ahead of co-runners
#endif
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // grid (levels, frames). Measured and retired: (frames, levels), every
    // frame's level 0 (the longest workgroups) dispatched first: 129 vs
    // 190-206 us alone, but the step slower (110.8 k vs 113.5 k frames/s,
    // profiles/r02_octree_ab/): 256 level-0 workgroups at once crowd out the
    // co-running pair stages.
    const int f = blockIdx.y;
    const int l = blockIdx.x;
    const int t = threadIdx.x;
    const LevelDesc L = lv[l];
    // carve LDS
    ONode* nodesA = reinterpret_cast<ONode*>(smem);
    ONode* nodesB = nodesA + node_cap;
    int* cc = reinterpret_cast<int*>(nodesB + node_cap);          // node_cap*4 child counts / scratch
    int* npos = cc + 4 * node_cap;                                 // node_cap*4 child positions
    int* iscr = npos + 4 * node_cap;                               // node_cap ints scratch
    int* scan = iscr + node_cap;                                   // OT_THREADS
    uint64_t* sortk = reinterpret_cast<uint64_t*>(scan + OT_THREADS + 2);  // node_cap (pow2) sort keys
    __shared__ __attribute__((aligned(16))) int s_vars[16];
    int& s_J = s_vars[6];
    int& s_size = s_vars[0];
    int& s_prev = s_vars[1];
    int& s_seq = s_vars[2];
    int& s_phase = s_vars[3];
    int& s_finish = s_vars[4];
    int& s_vcnt = s_vars[5];

    const size_t kbase = (size_t)f * keys_stride_frame + (size_t)L.key_off;
    uint32_t* keys = keys_g + kbase;
    int32_t* knode = knode_g + kbase;
    uint8_t* kquad = kquad_g + kbase;
    uint32_t* out = okp + ((size_t)f * nlevels + l) * okp_stride;

    // ---- gather candidates of this level's cells in cell order
    const int c0 = L.cell_begin, nc = L.cell_end - L.cell_begin;
    int n = 0;
    for (int cb = 0; cb < nc; cb += OT_THREADS) {
        const int c = cb + t;
        const int cnt = c < nc ? cand_cnt[(size_t)f * ncells + c0 + c] : 0;
        int tot;
        const int ex = block_exclusive_scan(cnt, scan, &tot);
        if (c < nc) {
            // 32 candidates in flight per batch (cell rows are 16-byte aligned):
            // a load-then-store loop would wait out one memory latency per 4 keys
            const uint4* src = reinterpret_cast<const uint4*>(cand + ((size_t)f * ncells + c0 + c) * cell_cap);
            uint32_t* dst = keys + n + ex;
            for (int k0 = 0; k0 < cnt; k0 += 32) {
                uint4 v[8];
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (k0 + 4 * u < cnt) v[u] = src[(k0 >> 2) + u];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const int k = k0 + 4 * u;
                    if (k < cnt) dst[k] = v[u].x;
                    if (k + 1 < cnt) dst[k + 1] = v[u].y;
                    if (k + 2 < cnt) dst[k + 2] = v[u].z;
                    if (k + 3 < cnt) dst[k + 3] = v[u].w;
                }
            }
        }
        n += tot;
    }
    __syncthreads();
    if (n == 0) {
        if (t == 0) ocnt[f * nlevels + l] = 0;
        return;
    }
    const int minX = 16, maxX = L.w - 16, minY = 16, maxY = L.h - 16;
    const int N = L.quota;
    const int nIni = (int)roundf((float)(maxX - minX) / (float)(maxY - minY));
    const float hX = (float)(maxX - minX) / (float)nIni;

    // ---- initial nodes
    for (int i = t; i < nIni; i += OT_THREADS) {
        ONode nd;
        nd.x0 = (int16_t)(int)(hX * (float)i);
        nd.x1 = (int16_t)(int)(hX * (float)(i + 1));
        nd.y0 = 0;
        nd.y1 = (int16_t)(maxY - minY);
        nd.cnt = 0;
        nd.seq = i;
        nodesA[i] = nd;
    }
    __syncthreads();
    uint32_t ky[OT_KB];
    int nd[OT_KB];
    uint8_t kq[OT_KB];
    // the initial nodes' key counts: nIni is 1-2 for 4:3 frames, so every
    // key's atomic hit the same one or two LDS words (a 64-way serialised
    // atomic per key batch); the first four nodes are counted in registers
    // and added once per thread (the same integer counts)
    int ic0 = 0, ic1 = 0, ic2 = 0, ic3 = 0;
    ot_keys(
        n, t, [&](int k, int u) { ky[u] = keys[k]; },
        [&](int k, int u) {
            const float x = (float)(ky[u] & 0xfff);
            const int ni = (int)(x / hX);
            knode[k] = ni;
            ic0 += ni == 0;
            ic1 += ni == 1;
            ic2 += ni == 2;
            ic3 += ni == 3;
            if (ni > 3) atomicAdd(&nodesA[ni].cnt, 1);
        });
    if (ic0) atomicAdd(&nodesA[0].cnt, ic0);
    if (ic1) atomicAdd(&nodesA[1].cnt, ic1);
    if (ic2) atomicAdd(&nodesA[2].cnt, ic2);
    if (ic3) atomicAdd(&nodesA[3].cnt, ic3);
    __syncthreads();
    // erase empty initial nodes (keep order)
    if (t == 0) {
        int w = 0;
        for (int i = 0; i < nIni; i++) {
            iscr[i] = -1;
            if (nodesA[i].cnt > 0) {
                iscr[i] = w;
                nodesB[w++] = nodesA[i];
            }
        }
        s_size = w;
        s_seq = nIni;
        s_finish = 0;
        s_phase = 1;
    }
    __syncthreads();
    ot_keys(
        n, t, [&](int k, int u) { nd[u] = knode[k]; }, [&](int k, int u) { knode[k] = iscr[nd[u]]; });
    for (int i = t; i < s_size; i += OT_THREADS) nodesA[i] = nodesB[i];
    __syncthreads();

    ONode* cur = nodesA;
    ONode* nxt = nodesB;
    // vSizeAndPtr entries live in sortk as (cnt<<32 | seq); positions resolved by seq lookup
    int vcount = 0;

    while (!s_finish) {
        const int S = s_size;
        if (s_phase == 1) {
            // ---------------- phase 1: divide every node with >1 keys
            for (int i = t; i < 4 * S; i += OT_THREADS) cc[i] = 0;
            __syncthreads();
            ot_keys(
                n, t,
                [&](int k, int u) {
                    nd[u] = knode[k];
                    ky[u] = keys[k];
                },
                [&](int k, int u) {
                    const ONode N0 = cur[nd[u]];
                    if (N0.cnt > 1) {
                        const int x = ky[u] & 0xfff, y = (ky[u] >> 12) & 0xfff;
                        const int hx = (N0.x1 - N0.x0 + 1) >> 1;  // ceil((x1-x0)/2), x1>=x0
                        const int hy = (N0.y1 - N0.y0 + 1) >> 1;
                        const int q = (x < N0.x0 + hx) ? (y < N0.y0 + hy ? 0 : 2) : (y < N0.y0 + hy ? 1 : 3);
                        kquad[k] = (uint8_t)q;
                        atomicAdd(&cc[nd[u] * 4 + q], 1);
                    }
                });
            __syncthreads();
            // per-node children stats, scans over list order (chunks of OT_THREADS)
            int childBase = 0, survBase = 0, expBase = 0;
            int totalChildren = 0;
            // first: total children (for survivor offset) and reverse positions
            // pass A: e_i forward exclusive scan (seq, vSizeAndPtr order)
            for (int cb = 0; cb < S; cb += OT_THREADS) {
                const int i = cb + t;
                int e = 0, ne = 0, s = 0;
                if (i < S) {
                    if (cur[i].cnt > 1) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            e += cc[i * 4 + q] > 0;
                            ne += cc[i * 4 + q] > 1;
                        }
                    } else s = 1;
                }
                // one scan of the three counts: (e, ne) packed in 16-bit
                // fields (each <= 4 * node_cap <= 8192), s beside them
                int2 tp;
                const int2 ex = block_exclusive_scan2(e | (ne << 16), s, scan, &tp);
                const int ex_e = ex.x & 0xFFFF, ex_ne = ex.x >> 16, ex_s = ex.y;
                const int te = tp.x & 0xFFFF, tne = tp.x >> 16, ts = tp.y;
                if (i < S) {
                    iscr[i] = childBase + ex_e;          // forward children prefix
                    npos[i * 4 + 0] = e;                 // stash e
                    npos[i * 4 + 1] = ex_ne + expBase;   // vSizeAndPtr base
                    npos[i * 4 + 2] = survBase + ex_s;   // survivor rank
                    npos[i * 4 + 3] = s;
                }
                childBase += te;
                expBase += tne;
                survBase += ts;
                __syncthreads();
            }
            totalChildren = childBase;
            const int newSize = totalChildren + survBase;
            // build new list
            for (int i = t; i < S; i += OT_THREADS) {
                const ONode P = cur[i];
                const int e = npos[i * 4 + 0];
                const int vb = npos[i * 4 + 1];
                const int sr = npos[i * 4 + 2];
                if (npos[i * 4 + 3]) {
                    const int pos = totalChildren + sr;
                    nxt[pos] = P;
                    cc[i * 4 + 0] = pos;  // survivor mapping
                } else {
                    // reverse-chronological block start: children of later nodes come first
                    const int blockStart = totalChildren - (iscr[i] + e);
                    const int hx = (P.x1 - P.x0 + 1) >> 1, hy = (P.y1 - P.y0 + 1) >> 1;
                    int r = 0, v = vb;
                    int cpos[4];
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int c = cc[i * 4 + q];
                        cpos[q] = -1;
                        if (c > 0) {
                            ONode C;
                            const int qx = q & 1, qy = q >> 1;
                            C.x0 = (int16_t)(qx ? P.x0 + hx : P.x0);
                            C.x1 = (int16_t)(qx ? P.x1 : P.x0 + hx);
                            C.y0 = (int16_t)(qy ? P.y0 + hy : P.y0);
                            C.y1 = (int16_t)(qy ? P.y1 : P.y0 + hy);
                            C.cnt = c;
                            C.seq = s_seq + iscr[i] + r;
                            const int pos = blockStart + (e - 1 - r);
                            nxt[pos] = C;
                            cpos[q] = pos;
                            if (c > 1) {
                                sortk[v] = ot_key(c, C.seq, pos);
                                v++;
                            }
                            r++;
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; q++) cc[i * 4 + q] = cpos[q];
                }
            }
            __syncthreads();
            ot_keys(
                n, t,
                [&](int k, int u) {
                    nd[u] = knode[k];
                    kq[u] = kquad[k];
                },
                [&](int k, int u) { knode[k] = cc[nd[u] * 4 + (cur[nd[u]].cnt > 1 ? kq[u] : 0)]; });
            __syncthreads();
            if (t == 0) {
                s_prev = S;
                s_size = newSize;
                s_seq += totalChildren;
                s_vcnt = expBase;
                if (newSize >= N || newSize == S) s_finish = 1;
                else if (newSize + expBase * 3 > N) s_phase = 2;
            }
            vcount = expBase;
            __syncthreads();
            ONode* tmpp = cur;
            cur = nxt;
            nxt = tmpp;
        } else {
            // ---------------- phase 2: divide the largest nodes first
            vcount = s_vcnt;
            // processing rank per node: the entries of sortk[0..vcount)
            // descending by (cnt, seq), the node of the j-th one processed
            // j-th. The keys are unique (seq is), so an entry's place is the
            // number of larger entries: counted directly while vcount is
            // small (one barrier; round 5), a bitonic sort beyond
            for (int i = t; i < S; i += OT_THREADS) iscr[i] = -1;
            if (vcount <= OT_RANK_MAX) {
                __syncthreads();  // every iscr reset
                for (int i = t; i < vcount; i += OT_THREADS) {
                    const uint64_t ki = sortk[i];
                    int above = 0, j = 0;
                    // eight broadcast reads in flight per step
                    for (; j + 8 <= vcount; j += 8) {
                        uint64_t kj[8];
#pragma unroll
                        for (int u = 0; u < 8; u++) kj[u] = sortk[j + u];
#pragma unroll
                        for (int u = 0; u < 8; u++) above += kj[u] > ki;
                    }
                    for (; j < vcount; j++) above += sortk[j] > ki;
                    iscr[(int)(ki & 0xFFFF)] = above;
                }
                __syncthreads();
            } else {
                int pw = 1;
                while (pw < vcount) pw <<= 1;
                for (int i = vcount + t; i < pw; i += OT_THREADS) sortk[i] = ~0ull;
                __syncthreads();
                for (int kk = 2; kk <= pw; kk <<= 1) {
                    for (int jj = kk >> 1; jj > 0; jj >>= 1) {
                        for (int i = t; i < pw; i += OT_THREADS) {
                            const int ixj = i ^ jj;
                            if (ixj > i) {
                                const uint64_t a = sortk[i], b = sortk[ixj];
                                const bool up = (i & kk) == 0;
                                if ((a > b) == up) {
                                    sortk[i] = b;
                                    sortk[ixj] = a;
                                }
                            }
                        }
                        __syncthreads();
                    }
                }
                for (int j = t; j < vcount; j += OT_THREADS) iscr[(int)(sortk[vcount - 1 - j] & 0xFFFF)] = j;
                __syncthreads();
            }
            for (int i = t; i < 4 * S; i += OT_THREADS) cc[i] = 0;
            __syncthreads();
            ot_keys(
                n, t,
                [&](int k, int u) {
                    nd[u] = knode[k];
                    ky[u] = keys[k];
                },
                [&](int k, int u) {
                    if (iscr[nd[u]] >= 0) {
                        const ONode N0 = cur[nd[u]];
                        const int x = ky[u] & 0xfff, y = (ky[u] >> 12) & 0xfff;
                        const int hx = (N0.x1 - N0.x0 + 1) >> 1;
                        const int hy = (N0.y1 - N0.y0 + 1) >> 1;
                        const int q = (x < N0.x0 + hx) ? (y < N0.y0 + hy ? 0 : 2) : (y < N0.y0 + hy ? 1 : 3);
                        kquad[k] = (uint8_t)q;
                        atomicAdd(&cc[nd[u] * 4 + q], 1);
                    }
                });
            __syncthreads();
            // Node divisions in processing order j (largest first) until the
            // list reaches N: with e_j the non-empty children of node proc[j],
            // the list size after j is S + sum_{j'<=j}(e_j' - 1), so the break
            // point J, the children's seq numbers, their (reverse processing
            // order) block positions and the new vSizeAndPtr slots are all
            // prefix sums over j; survivors keep their order after the blocks.
            int* proc = npos;                  // [vcount] node of rank j
            int* eincl = npos + node_cap;      // inclusive prefix of e_j
            int* vexcl = npos + 2 * node_cap;  // exclusive prefix of #children with >1 keys
            for (int i = t; i < S; i += OT_THREADS)
                if (iscr[i] >= 0) proc[iscr[i]] = i;
            if (t == 0) s_J = vcount;
            __syncthreads();
            {
                int eb = 0, vb = 0;
                for (int cb = 0; cb < vcount; cb += OT_THREADS) {
                    const int j = cb + t;
                    int e = 0, v = 0;
                    if (j < vcount) {
                        const int i = proc[j];
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            e += cc[i * 4 + q] > 0;
                            v += cc[i * 4 + q] > 1;
                        }
                    }
                    int tot;
                    const int ex = block_exclusive_scan(e | (v << 16), scan, &tot);
                    if (j < vcount) {
                        const int ei = eb + (ex & 0xFFFF) + e;
                        eincl[j] = ei;
                        vexcl[j] = vb + (ex >> 16);
                        if (S + ei - (j + 1) >= N) atomicMin(&s_J, j + 1);
                    }
                    eb += tot & 0xFFFF;
                    vb += tot >> 16;
                }
            }
            __syncthreads();
            const int J = s_J;
            const int EJ = J > 0 ? eincl[J - 1] : 0;
            for (int j = t; j < J; j += OT_THREADS) {
                const int i = proc[j];
                const ONode P = cur[i];
                const int hx = (P.x1 - P.x0 + 1) >> 1, hy = (P.y1 - P.y0 + 1) >> 1;
                int e = 0;
#pragma unroll
                for (int q = 0; q < 4; q++) e += cc[i * 4 + q] > 0;
                const int blockStart = EJ - eincl[j];
                const int seqBase = s_seq + eincl[j] - e;
                int r = 0, v = vexcl[j];
                int cpos[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int c = cc[i * 4 + q];
                    cpos[q] = -1;
                    if (c > 0) {
                        ONode C;
                        const int qx = q & 1, qy = q >> 1;
                        C.x0 = (int16_t)(qx ? P.x0 + hx : P.x0);
                        C.x1 = (int16_t)(qx ? P.x1 : P.x0 + hx);
                        C.y0 = (int16_t)(qy ? P.y0 + hy : P.y0);
                        C.y1 = (int16_t)(qy ? P.y1 : P.y0 + hy);
                        C.cnt = c;
                        C.seq = seqBase + r;
                        const int pp = blockStart + (e - 1 - r);
                        nxt[pp] = C;
                        cpos[q] = pp;
                        if (c > 1) sortk[v++] = ot_key(c, C.seq, pp);
                        r++;
                    }
                }
#pragma unroll
                for (int q = 0; q < 4; q++) cc[i * 4 + q] = cpos[q];
                if (j == J - 1) s_vcnt = v;  // vSizeAndPtr entries of the new list
            }
            // survivors: every node not processed (rank >= J or not listed), list order
            int sb = 0;
            for (int cb = 0; cb < S; cb += OT_THREADS) {
                const int i = cb + t;
                int sv = 0;
                if (i < S) {
                    const int j = iscr[i];
                    sv = !(j >= 0 && j < J);
                }
                int tot;
                const int ex = block_exclusive_scan(sv, scan, &tot);
                if (sv) {
                    const int pp = EJ + sb + ex;
                    nxt[pp] = cur[i];
                    cc[i * 4 + 0] = pp;
                    iscr[i] = -2;
                }
                sb += tot;
            }
            if (t == 0) {
                const int size = EJ + sb;
                s_prev = S;
                s_size = size;
                s_seq += EJ;
                if (J == 0) s_vcnt = 0;
                if (size >= N || size == S) s_finish = 1;
            }
            __syncthreads();
            ot_keys(
                n, t,
                [&](int k, int u) {
                    nd[u] = knode[k];
                    kq[u] = kquad[k];
                },
                [&](int k, int u) {
                    const int is = iscr[nd[u]];
                    knode[k] = cc[nd[u] * 4 + (is == -2 || is == -1 ? 0 : kq[u])];
                });
            __syncthreads();
            ONode* tmpp = cur;
            cur = nxt;
            nxt = tmpp;
        }
        __syncthreads();
    }
    // ---- retain best key per node (max response, first in candidate order)
    const int S = s_size;
    unsigned* best = reinterpret_cast<unsigned*>(cc);
    for (int i = t; i < S; i += OT_THREADS) best[i] = 0;
    __syncthreads();
    ot_keys(
        n, t,
        [&](int k, int u) {
            ky[u] = keys[k];
            nd[u] = knode[k];
        },
        [&](int k, int u) { atomicMax(&best[nd[u]], ((ky[u] >> 24) << 23) | (0x7FFFFFu - (unsigned)k)); });
    __syncthreads();
    const int cap = okp_stride;
    for (int i = t; i < S && i < cap; i += OT_THREADS) {
        const int k = 0x7FFFFF - (int)(best[i] & 0x7FFFFF);
        out[i] = keys[k];
    }
    if (t == 0) ocnt[f * nlevels + l] = S < cap ? S : cap;
}

// ============================================================ blur
// Separable 7-tap Q8 kernel {18,34,48,56,48,34,18}, REFLECT_101, exact integer
// (GaussianBlur 7x7 sigma 2 on 8U). One 128x32 output tile per workgroup over
// a flattened (level, tile) grid. The 136x38 input window (x from tx0-4) is
// staged in LDS with aligned dword loads (rows are pitch-aligned; reflection
// only on border tiles). Horizontal pass: 4 outputs from three LDS dwords,
// two byte-aligned windows and two v_dot4_u32_u8 each, two rows per item,
// stored as (row 2i, row 2i+1) u16 pairs per column. Vertical pass: 4x4
// outputs per thread, odd row pairs formed with one v_perm, summed with
// v_dot2_u32_u16 (the rounding term as the first accumulator), output bytes
// gathered with v_perm, one aligned dword store per output row.
#define BLUR_TX 128
#define BLUR_TY 32
#define BLUR_IW (BLUR_TX + 8)  // staged row stride: x in [tx0-4, tx0+132)
#define BLUR_IH (BLUR_TY + 6)
ODO_INLINE int reflect101(int i, int n) {
    while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
    return i;
}
// one reflection (|overshoot| < n): branch-free
ODO_INLINE int reflect101_1(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

struct BlurTiles {
    int base[17];  // first tile of each level (prefix), base[nlevels] = total
    int tx[16];    // tiles across
};

typedef unsigned short blur_us2 __attribute__((ext_vector_type(2)));
ODO_INLINE uint32_t dot2u16(uint32_t a, uint32_t b, uint32_t c) {
    blur_us2 x, y;
    x.x = (unsigned short)(a & 0xffff), x.y = (unsigned short)(a >> 16);
    y.x = (unsigned short)(b & 0xffff), y.y = (unsigned short)(b >> 16);
    return __builtin_amdgcn_udot2(x, y, c, false);
}

__global__ void __launch_bounds__(256) k_blur(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                              size_t pyr_stride, const LevelDesc* __restrict__ lv, BlurTiles TT,
                                              int nlevels) {
    __shared__ __attribute__((aligned(16))) uint8_t tile[BLUR_IH * BLUR_IW];
    __shared__ __attribute__((aligned(16))) uint32_t hrow[(BLUR_IH / 2) * BLUR_TX];
    const int f = blockIdx.y;
    const int tid = blockIdx.x;
    int l = 0;
    while (l + 1 < nlevels && tid >= TT.base[l + 1]) l++;
    const LevelDesc L = lv[l];
    const int ti = tid - TT.base[l];
    const int tx0 = (ti % TT.tx[l]) * BLUR_TX, ty0 = (ti / TT.tx[l]) * BLUR_TY;
    const uint8_t* src = pyr + (size_t)f * pyr_stride + L.off;
    uint8_t* dst = blur + (size_t)f * pyr_stride + L.off;
    const int t = threadIdx.x;
    const bool interior = tx0 >= 4 && ty0 >= 3 && tx0 + BLUR_TX + 4 <= L.w && ty0 + BLUR_TY + 3 <= L.h;
    if (interior) {
        constexpr int NW = BLUR_IW / 4;  // dwords per staged row
        for (int it = t; it < BLUR_IH * NW; it += 256) {
            const int r = it / NW, c = it - r * NW;
            const uint32_t* srow = reinterpret_cast<const uint32_t*>(src + (size_t)(ty0 + r - 3) * L.pitch + tx0 - 4);
            reinterpret_cast<uint32_t*>(tile + r * BLUR_IW)[c] = srow[c];
        }
    } else {
        // border tile: rows reflected once per dword, in-row dwords loaded whole,
        // only the dwords straddling a left/right edge assembled bytewise
        constexpr int NW = BLUR_IW / 4;
        for (int it = t; it < BLUR_IH * NW; it += 256) {
            const int r = it / NW, c = it - r * NW;
            const uint8_t* srow = src + (size_t)reflect101(ty0 + r - 3, L.h) * L.pitch;
            const int x = tx0 - 4 + 4 * c;
            uint32_t v;
            if (x >= 0 && x + 3 < L.w) {
                v = *reinterpret_cast<const uint32_t*>(srow + x);
            } else {
                v = 0;
#pragma unroll
                for (int b = 0; b < 4; b++) v |= (uint32_t)srow[reflect101(x + b, L.w)] << (8 * b);
            }
            reinterpret_cast<uint32_t*>(tile + r * BLUR_IW)[c] = v;
        }
    }
    __syncthreads();
    // horizontal: row r, outputs 4q+o take staged bytes 4q+1+o .. 4q+7+o. An
    // item is two rows (2rp, 2rp+1) x 4 columns; hrow holds per (row pair,
    // column) the dword (h[2rp], h[2rp+1]), the vertical pass's even row pairs
    constexpr uint32_t C0 = 18u | (34u << 8) | (48u << 16) | (56u << 24);
    constexpr uint32_t C1 = 48u | (34u << 8) | (18u << 16);
    for (int it = t; it < (BLUR_IH / 2) * (BLUR_TX / 4); it += 256) {
        const int rp = it / (BLUR_TX / 4), q = it % (BLUR_TX / 4);
        uint32_t h[2][4];
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(&tile[(2 * rp + e) * BLUR_IW + 4 * q]);
            const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
            h[e][0] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 1), C1,
                                             __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 1), C0, 0u, false),
                                             false);
            h[e][1] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 2), C1,
                                             __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 2), C0, 0u, false),
                                             false);
            h[e][2] = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 3), C1,
                                             __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 3), C0, 0u, false),
                                             false);
            h[e][3] = __builtin_amdgcn_udot4(w2, C1, __builtin_amdgcn_udot4(w1, C0, 0u, false), false);
        }
        uint4 pk;
        pk.x = h[0][0] | (h[1][0] << 16);
        pk.y = h[0][1] | (h[1][1] << 16);
        pk.z = h[0][2] | (h[1][2] << 16);
        pk.w = h[0][3] | (h[1][3] << 16);
        *reinterpret_cast<uint4*>(&hrow[rp * BLUR_TX + 4 * q]) = pk;
    }
    __syncthreads();
    // vertical: 4 columns x 4 rows per thread
    {
        const int q = t % (BLUR_TX / 4), rb = (t / (BLUR_TX / 4)) * 4;  // 32 x 8 threads
        uint4 pk[5];  // row pairs (rb + 2i, rb + 2i + 1), columns 4q .. 4q+3
#pragma unroll
        for (int i = 0; i < 5; i++) pk[i] = *reinterpret_cast<const uint4*>(&hrow[(rb / 2 + i) * BLUR_TX + 4 * q]);
        constexpr uint32_t K01 = 18u | (34u << 16), K23 = 48u | (56u << 16), K45 = 48u | (34u << 16), K6 = 18u;
        // sums start at the rounding term 32768: (S + 32768) >> 16 is then byte 2
        // of the sum (S < 2^24), gathered four columns at a time with v_perm
        uint32_t sum4[4][4];  // [output row][column]
#pragma unroll
        for (int cI = 0; cI < 4; cI++) {
            uint32_t E[5];
#pragma unroll
            for (int i = 0; i < 5; i++) E[i] = cI == 0 ? pk[i].x : cI == 1 ? pk[i].y : cI == 2 ? pk[i].z : pk[i].w;
            // P[j] = (row j, row j+1): even j straight from hrow, odd j = (high
            // half of pair j-1, low half of pair j+1); P[9] = row 9 alone
            uint32_t P[10];
#pragma unroll
            for (int j = 0; j < 9; j++)
                P[j] = (j & 1) ? __builtin_amdgcn_perm(E[(j + 1) / 2], E[(j - 1) / 2], 0x05040302u) : E[j / 2];
            P[9] = E[4] >> 16;
#pragma unroll
            for (int o = 0; o < 4; o++) {
                uint32_t sum = dot2u16(P[o], K01, 32768u);
                sum = dot2u16(P[o + 2], K23, sum);
                sum = dot2u16(P[o + 4], K45, sum);
                sum4[o][cI] = dot2u16(P[o + 6], K6, sum);
            }
        }
        uint32_t out[4];
#pragma unroll
        for (int o = 0; o < 4; o++) {
            // bytes 2 of columns (0, 1) and (2, 3) into the low / high halves
            const uint32_t lo = __builtin_amdgcn_perm(sum4[o][1], sum4[o][0], 0x0c0c0602u);
            const uint32_t hi = __builtin_amdgcn_perm(sum4[o][3], sum4[o][2], 0x06020c0cu);
            out[o] = lo | hi;
        }
        const int x = tx0 + 4 * q;
        if (x < L.w) {
#pragma unroll
            for (int o = 0; o < 4; o++) {
                const int y = ty0 + rb + o;
                if (y < L.h) *reinterpret_cast<uint32_t*>(dst + (size_t)y * L.pitch + x) = out[o];
            }
        }
    }
}

// ---------------------------------------------------------------- k_blur_rows
// The same 7x7 GaussianBlur (exact Q8 taps, (S + 32768) >> 16) with no LDS:
// a 16-lane group owns a strip of 16 four-pixel quads and walks BR_R output
// rows down it. Per input row a lane loads the three aligned dwords around its
// quad, forms the 4 horizontal sums with 8 v_dot4 (packed as u16 pairs), pairs
// each column with the previous row's value (one v_perm per column) and adds
// the pair into the three output rows it belongs to with v_dot2_u32_u16; the
// row's own single tap closes the output three rows up, which is stored. The
// six accumulators rotate with the row index mod 6 (the row loop is unrolled
// by 6) and rows are loaded a block of 6 ahead, so nothing is staged or
// re-read: ~10 lane-ops per pixel against 31 for the LDS-tiled k_blur.
// Strips cover quads 1 .. nq[l] (x - 3 >= 0 and x + 7 <= w - 1: no column
// reflection, the three dwords inside the row) and every row; the first and
// last chunk reflect their halo rows (reflect101). The quads left of quad 1
// and right of quad nq run the same walk one lane each (a lane per (level,
// chunk, edge quad), packed 64 to a wave at the end of the grid): per-lane
// row reflection, and the row's 12 bytes rebuilt with reflect101 columns by
// two v_perm per dword from per-lane selectors. Widths that are not a
// multiple of 4 leave garbage in the row padding past w, never read.
#define BR_R 30  // output rows per chunk (a multiple of 6; levels are >= 40 rows)
#ifndef BW_ROLL
#define BW_ROLL 1  // blur walk rows loaded as a rolling 6-row queue (see blur_walk)
#endif
#ifndef PYR_NT
// nontemporal (streaming) accesses for the pyramid's data that is not read
// again soon: bit 0 the BGR loads, bit 1 the blurred-level stores (finalize
// reads them a millisecond later), so they do not evict from L2 the levels the
// next resize and blur walks read back
#define PYR_NT 0
#endif
struct BlurRows {
    int base[17];   // first strip item of each level (prefix); base[nlevels] = items
    int nst[16];    // strips of 16 quads across the interior
    int nq[16];     // interior quads (q = 1 .. nq)
    int nch[16];    // row chunks
    int ebase[17];  // first edge lane of each level (prefix); ebase[nlevels] = edge lanes
};

ODO_INLINE uint32_t pair_lo(uint32_t cur, uint32_t prev) { return __builtin_amdgcn_perm(cur, prev, 0x05040100u); }
ODO_INLINE uint32_t pair_hi(uint32_t cur, uint32_t prev) { return __builtin_amdgcn_perm(cur, prev, 0x07060302u); }

// the last chunk of a level overlaps its predecessor instead of running past
// the last row (both write the same bytes)
template <int R>
ODO_INLINE int chunk_y0(int chunk, int h) { return min(chunk * R, h - R); }
#define BR_RE 6  // output rows per edge-lane chunk

// One quad's walk down rows y0 - 3 .. y0 + R + 2. s0: the level's row 0 at
// byte x - 4 (interior) / the level's row 0 (EDGE); dp: row y0 at byte x.
template <bool EDGE, int R>
ODO_INLINE void blur_walk(const uint8_t* s0, uint8_t* dp, size_t pitch, int h, int y0, bool top, bool bottom,
                          bool store, int o0, int o1, int o2, const uint32_t (&selA)[3], const uint32_t (&selB)[3]) {
    constexpr uint32_t C0 = 18u | (34u << 8) | (48u << 16) | (56u << 24);
    constexpr uint32_t C1 = 48u | (34u << 8) | (18u << 16);
    constexpr uint32_t K01 = 18u | (34u << 16), K23 = 48u | (56u << 16), K45 = 48u | (34u << 16);
    constexpr uint32_t KLO = 18u, KHI = 18u << 16;
    uint32_t acc[6][4];
#pragma unroll
    for (int a = 0; a < 6; a++)
#pragma unroll
        for (int c = 0; c < 4; c++) acc[a][c] = 32768u;
    uint32_t hp0 = 0, hp1 = 0;  // the previous row's (h0, h1), (h2, h3)
    // rows are loaded a block of 6 ahead (the loads of block b + 1 are in
    // flight while block b is computed); the first and the last block of an
    // edge chunk address their rows through reflect101
    static_assert(R % 6 == 0, "the accumulators rotate over 6 rows");
    constexpr int NB = (R + 6) / 6;
    uint32_t cw[6][3];
#if !BW_ROLL
    uint32_t nw[6][3];
#endif
    const uint8_t* sp = s0 + (size_t)(y0 - 3) * pitch;
    // input row 6b + j of the walk (rows y0 - 3 ...) into d
    auto load_row = [&](uint32_t(&d)[3], int b, int j, bool refl) {
        if (EDGE) {
            const uint8_t* rp = s0 + (size_t)reflect101_1(y0 - 3 + 6 * b + j, h) * pitch;
            d[0] = *reinterpret_cast<const uint32_t*>(rp + o0);
            d[1] = *reinterpret_cast<const uint32_t*>(rp + o1);
            d[2] = *reinterpret_cast<const uint32_t*>(rp + o2);
        } else {
            const uint8_t* rp = refl ? s0 + (size_t)reflect101_1(y0 - 3 + 6 * b + j, h) * pitch : sp + j * pitch;
            const uint32_t* w = reinterpret_cast<const uint32_t*>(rp);
            d[0] = w[0], d[1] = w[1], d[2] = w[2];
        }
    };
    auto load_block = [&](uint32_t(&d)[6][3], int b, bool refl) {
#pragma unroll
        for (int j = 0; j < 6; j++) load_row(d[j], b, j, refl);
        sp += 6 * pitch;
    };
    load_block(cw, 0, top);
    for (int b = 0; b < NB; b++) {
#if !BW_ROLL
        if (b + 1 < NB) load_block(nw, b + 1, b + 1 == NB - 1 && bottom);
#else
        // BW_ROLL: a 6-row queue instead of two 6-row blocks: row j of block b
        // + 1 is loaded into row j's registers as soon as row j of block b has
        // been consumed (6 rows in flight, 18 registers fewer)
        const bool nref = b + 1 == NB - 1 && bottom;
#endif
#pragma unroll
        for (int j = 0; j < 6; j++) {
            // input row r = y0 - 3 + 6b + j
            uint32_t w0 = cw[j][0], w1 = cw[j][1], w2 = cw[j][2];
#if BW_ROLL
            if (b + 1 < NB) load_row(cw[j], b + 1, j, nref);
#endif
            if (EDGE) {
                // the row's bytes x-4 .. x+7 with reflected columns
                const uint32_t e0 = __builtin_amdgcn_perm(w1, w0, selA[0]) | __builtin_amdgcn_perm(w2, w2, selB[0]);
                const uint32_t e1 = __builtin_amdgcn_perm(w1, w0, selA[1]) | __builtin_amdgcn_perm(w2, w2, selB[1]);
                const uint32_t e2 = __builtin_amdgcn_perm(w1, w0, selA[2]) | __builtin_amdgcn_perm(w2, w2, selB[2]);
                w0 = e0, w1 = e1, w2 = e2;
            }
            const uint32_t h0 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 1), C1,
                                                       __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 1), C0, 0u, false), false);
            const uint32_t h1 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 2), C1,
                                                       __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 2), C0, 0u, false), false);
            const uint32_t h2 = __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w2, w1, 3), C1,
                                                       __builtin_amdgcn_udot4(__builtin_amdgcn_alignbyte(w1, w0, 3), C0, 0u, false), false);
            const uint32_t h3 = __builtin_amdgcn_udot4(w2, C1, __builtin_amdgcn_udot4(w1, C0, 0u, false), false);
            const uint32_t hc0 = h0 | (h1 << 16), hc1 = h2 | (h3 << 16);
            // pairs (h[r-1], h[r]) per column
            const uint32_t P0 = pair_lo(hc0, hp0), P1 = pair_hi(hc0, hp0), P2 = pair_lo(hc1, hp1), P3 = pair_hi(hc1, hp1);
            hp0 = hc0;
            hp1 = hc1;
            const int sa = (j + 5) % 6, sb = (j + 3) % 6, sc = (j + 1) % 6, sd = j;
            // output r + 2: its first pair (taps 18, 34) opens the accumulator
            acc[sa][0] = dot2u16(P0, K01, 32768u);
            acc[sa][1] = dot2u16(P1, K01, 32768u);
            acc[sa][2] = dot2u16(P2, K01, 32768u);
            acc[sa][3] = dot2u16(P3, K01, 32768u);
            // output r: taps 48, 56; output r - 2: taps 48, 34
            acc[sb][0] = dot2u16(P0, K23, acc[sb][0]);
            acc[sb][1] = dot2u16(P1, K23, acc[sb][1]);
            acc[sb][2] = dot2u16(P2, K23, acc[sb][2]);
            acc[sb][3] = dot2u16(P3, K23, acc[sb][3]);
            acc[sc][0] = dot2u16(P0, K45, acc[sc][0]);
            acc[sc][1] = dot2u16(P1, K45, acc[sc][1]);
            acc[sc][2] = dot2u16(P2, K45, acc[sc][2]);
            acc[sc][3] = dot2u16(P3, K45, acc[sc][3]);
            // output r - 3: the last tap (18) closes it
            const uint32_t s0v = dot2u16(hc0, KLO, acc[sd][0]), s1v = dot2u16(hc0, KHI, acc[sd][1]);
            const uint32_t s2v = dot2u16(hc1, KLO, acc[sd][2]), s3v = dot2u16(hc1, KHI, acc[sd][3]);
            if (b > 0 && store) {
                const uint32_t lo = __builtin_amdgcn_perm(s1v, s0v, 0x0c0c0602u);
                const uint32_t hi = __builtin_amdgcn_perm(s3v, s2v, 0x06020c0cu);
                if (PYR_NT & 2)
                    __builtin_nontemporal_store(lo | hi, reinterpret_cast<uint32_t*>(dp));
                else
                    *reinterpret_cast<uint32_t*>(dp) = lo | hi;
                dp += pitch;
            }
        }
#if BW_ROLL
        sp += 6 * pitch;
#else
#pragma unroll
        for (int j = 0; j < 6; j++) cw[j][0] = nw[j][0], cw[j][1] = nw[j][1], cw[j][2] = nw[j][2];
#endif
    }
}

// Edge quads: one lane per (level, 6-row chunk, quad left of 1 / right of nq).
// srcL: the level's row 0 (rows outside the ones the walk reads need not exist:
// k_pyramid's level-0 bands pass an LDS band as "row 0" minus its first row)
ODO_INLINE void blur_edge_lane(const uint8_t* srcL, uint8_t* __restrict__ blur, size_t pyr_stride,
                                const LevelDesc* __restrict__ lv, const BlurRows& S, int nlevels, int f, int k) {
    if (k >= S.ebase[nlevels]) return;
    int l = 0;
    while (l + 1 < nlevels && k >= S.ebase[l + 1]) l++;
    const LevelDesc L = lv[l];
    const int nqa = (L.w + 3) >> 2, ne = 1 + nqa - (S.nq[l] + 1);  // quad 0 and quads nq+1 .. nqa-1
    const int i = k - S.ebase[l], chunk = i / ne, e = i - chunk * ne;
    const int q = e == 0 ? 0 : S.nq[l] + e;
    const int x = 4 * q;
    const int y0 = chunk_y0<BR_RE>(chunk, L.h);
    // selectors: byte b of dword d is position P = x - 4 + 4d + b, taken from
    // reflect101(P) - (x - 4) of the loaded window (w0, w1, w2); a window
    // dword that would lie outside the row is loaded from x instead and never
    // selected
    uint32_t selA[3], selB[3];
#pragma unroll
    for (int d = 0; d < 3; d++) {
        uint32_t a = 0, bsel = 0;
#pragma unroll
        for (int bb = 0; bb < 4; bb++) {
            const int src = reflect101_1(x - 4 + 4 * d + bb, L.w) - (x - 4);
            const int sd = src >> 2, sb = src & 3;
            a |= (uint32_t)(sd == 0 ? sb : sd == 1 ? 4 + sb : 0x0c) << (8 * bb);
            bsel |= (uint32_t)(sd == 2 ? sb : 0x0c) << (8 * bb);
        }
        selA[d] = a;
        selB[d] = bsel;
    }
    const int o0 = x >= 4 ? x - 4 : x, o2 = x + 8 <= L.pitch ? x + 4 : x;
    const uint8_t* s0 = srcL;
    uint8_t* dp = blur + (size_t)f * pyr_stride + L.off + (size_t)y0 * L.pitch + x;
    blur_walk<true, BR_RE>(s0, dp, (size_t)L.pitch, L.h, y0, true, true, true, o0, x, o2, selA, selB);
}

// Strips (quads 1 .. nq, every row) and, in the first eblocks workgroups of
// the grid, the edge quads (blur_edge_lane, 256 lanes per workgroup): one
// launch, so the edge lanes' latency-bound walks overlap the strips instead of
// running as a separate launch ahead of them (72-109 us of the extraction
// stream in the pipelined step, profiles/r03_b).
__global__ void __launch_bounds__(256) k_blur_rows(const uint8_t* __restrict__ pyr, uint8_t* __restrict__ blur,
                                                   size_t pyr_stride, const LevelDesc* __restrict__ lv, BlurRows S,
                                                   int nlevels, int eblocks) {
    EXTRACT_PRIO();
    const int f = blockIdx.y;
    if ((int)blockIdx.x < eblocks) {
        const int k = (int)blockIdx.x * 256 + (int)threadIdx.x;
        if (k >= S.ebase[nlevels]) return;
        int l = 0;
        while (l + 1 < nlevels && k >= S.ebase[l + 1]) l++;
        blur_edge_lane(pyr + (size_t)f * pyr_stride + lv[l].off, blur, pyr_stride, lv, S, nlevels, f, k);
        return;
    }
    const uint32_t none[3] = {0, 0, 0};
    const int item = ((int)blockIdx.x - eblocks) * 16 + ((int)threadIdx.x >> 4);
    if (item >= S.base[nlevels]) return;
    int l = 0;
    while (l + 1 < nlevels && item >= S.base[l + 1]) l++;
    const LevelDesc L = lv[l];
    const int it = item - S.base[l];
    const int chunk = it / S.nst[l], strip = it - chunk * S.nst[l];
    const int q = 1 + strip * 16 + ((int)threadIdx.x & 15);
    const bool store = q <= S.nq[l];
    const int x = 4 * (store ? q : S.nq[l]);  // idle lanes shadow the last quad (loads stay in the row)
    const int y0 = chunk_y0<BR_R>(chunk, L.h);
    const bool top = y0 < 3, bottom = y0 + BR_R + 3 > L.h;  // halo rows to reflect (uniform per group)
    const uint8_t* s0 = pyr + (size_t)f * pyr_stride + L.off + (x - 4);
    uint8_t* dp = blur + (size_t)f * pyr_stride + L.off + (size_t)y0 * L.pitch + x;
    blur_walk<false, BR_R>(s0, dp, (size_t)L.pitch, L.h, y0, top, bottom, store, 0, 0, 0, none, none);
}

// ============================================================ fused pyramid
// k_pyramid: one 1024-thread workgroup per frame builds the whole pyramid,
// gray (level 0) and then each level from the one before it, with a
// workgroup barrier between levels instead of eight dependent launches (the
// chain's per-level drain and launch latency were most of its 0.28 ms alone
// and 0.35-0.6 ms pipelined per 256 frames, profiles/r03_b). Levels >= 1 are
// read back through the CU's own L1 / L2 (every wave of the workgroup is on
// one CU, so workgroup-scope ordering is all the barrier needs).
// (Round 5 tried level 0 band by band in LDS, gray + 3-row halos, its blur
// and level 1 made from the band so that level 0 is never read back: 356 vs
// 329 us alone per 256 frames, step unchanged, profiles/r05_e; not kept.)
// Resize: thread t owns quad q = t mod nq of the level (4 output pixels) and
// walks the rows ph, ph + P, ... (ph = t / nq, P = 1024 / nq), so its x taps
// are loaded once per level into registers: the quad's source bytes lie in
// the 8-byte window starting at sx0(4q) (host-checked), one v_alignbyte pair
// per source row brings the window into two registers, and per pixel one
// v_perm picks (s[sx0], s[sx1]) as a u16 pair for v_dot2 with (a0, a1).
// Same integer arithmetic as k_resize: h = a0 s0 + a1 s1, out = (b0 h0 +
// b1 h1 + 2^21) >> 22.
// BLUR: the workgroup also blurs each level (k_blur_rows' strip walks and
// edge lanes) once the level is complete, beside the resize that reads it,
// so no separate blur launch follows (uint8 blur pyramid written to `blur`).
#ifndef PYR_TH
// threads per frame workgroup. 512 (round 6): 2 waves per SIMD at <= 80
// VGPRs (BW_ROLL) = 160 registers, so a frame's workgroup fits on a CU that
// holds a k_pnp workgroup (328 per SIMD); at 1024 (352) it waited for PnP
// to drain off the CU on every other step (DESIGN §4 Pipelining)
#define PYR_TH 512
#endif
#ifndef PYR_VGPR
#define PYR_ATTR
#else
// a VGPR cap (PYR_VGPR registers) on the fused pyramid, so that its
// workgroups fit beside the pair kernels' register footprints
#define PYR_ATTR __attribute__((amdgpu_waves_per_eu(PYR_VGPR)))
#endif
#ifndef PYR_RU
#define PYR_RU 4  // output rows in flight per thread (resize; 2 until round 5, at 1024 threads)
#endif
#ifndef PYR_GU
#define PYR_GU 8  // gray quads in flight per thread (4 until round 5, at 1024 threads)
#endif
struct PyrLevels {
    int rx_off[16], ry_off[16];
};
#ifndef PYR_PARTS
#define PYR_PARTS 1  // workgroups per frame (PyrSplit; the host falls back to 1 where a split does not fit)
#endif
// k_pyramid's split of a frame over `parts` workgroups (pyramid_split_plan):
// part p builds rows [lo, hi) of level l and blurs its strip chunks [ca, cb)
// and 6-row edge chunks [ea, eb)
struct PyrSplit {
    int parts;
    int lo[2][16], hi[2][16], ca[2][16], cb[2][16], ea[2][16], eb[2][16];
};
// the 7x7 blur of level l of frame f by the whole workgroup (PYR_TH threads:
// 64 strip groups of 16 lanes, then the edge lanes), read from srcL (the
// level's row 0)
ODO_INLINE void pyr_blur_level(const uint8_t* srcL, uint8_t* __restrict__ blur, size_t pyr_stride,
                               const LevelDesc* __restrict__ lv, const BlurRows& S, int nlevels, int f, int l,
                               const LevelDesc& L, int t, int ca, int cb, int ea, int eb) {
    // strip chunks [ca, cb) and edge chunks [ea, eb) of the level: this
    // workgroup's part of the frame (PyrSplit)
    const uint32_t none[3] = {0, 0, 0};
    const int items = cb * S.nst[l];
    const int g = t >> 4;
    for (int it = ca * S.nst[l] + g; it < items; it += PYR_TH / 16) {
        const int chunk = it / S.nst[l], strip = it - chunk * S.nst[l];
        const int q = 1 + strip * 16 + (t & 15);
        const bool store = q <= S.nq[l];
        const int x = 4 * (store ? q : S.nq[l]);
        const int y0 = chunk_y0<BR_R>(chunk, L.h);
        const bool top = y0 < 3, bottom = y0 + BR_R + 3 > L.h;
        const uint8_t* s0 = srcL + (x - 4);
        uint8_t* dp = blur + (size_t)f * pyr_stride + L.off + (size_t)y0 * L.pitch + x;
        blur_walk<false, BR_R>(s0, dp, (size_t)L.pitch, L.h, y0, top, bottom, store, 0, 0, 0, none, none);
    }
    const int ne = (S.ebase[l + 1] - S.ebase[l]) / ((L.h + BR_RE - 1) / BR_RE);  // edge quads per chunk
    for (int k = S.ebase[l] + ea * ne + t; k < S.ebase[l] + eb * ne; k += PYR_TH)
        blur_edge_lane(srcL, blur, pyr_stride, lv, S, nlevels, f, k);
}
// level D's rows [ylo, yhi) from level S (whose row 0 is srcS), thread t's quad
ODO_INLINE void pyr_resize_rows(const uint8_t* srcS, uint8_t* dstD, const LevelDesc& S, const LevelDesc& D,
                                const ResizeX* __restrict__ X, const ResizeY* __restrict__ Y, int t, int ylo, int yhi) {
    const int nq = (D.w + 3) >> 2;
    const int P = PYR_TH / nq;  // row phases (the host checks nq <= PYR_TH)
    if (t >= P * nq) return;
    const int ph = t / nq, q = t - ph * nq;
    // the quad's taps: window origin sx0(4q), per-pixel selectors and weights
    const int x00 = X[4 * q].sx0;
    const int wb = x00 & ~3, sh = x00 & 3;
    uint32_t sel[4], wt[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const int dx = 4 * q + j;
        if (dx < D.w) {
            const ResizeX xj = X[dx];
            const uint32_t r0 = (uint32_t)(xj.sx0 - x00), r1 = (uint32_t)(xj.sx1 - x00);  // 0..7
            sel[j] = r0 | (0x0cu << 8) | (r1 << 16) | (0x0cu << 24);
            wt[j] = (uint32_t)xj.a0 | ((uint32_t)xj.a1 << 16);
        } else {
            sel[j] = 0x0c0c0c0cu;  // past the level width: 0 (the row padding)
            wt[j] = 0;
        }
    }
    const uint8_t* sbase = srcS + wb;
    uint8_t* dbase = dstD + 4 * q;
    auto hsum = [&](const uint8_t* row, uint32_t (&h)[4]) {
        const uint32_t* w32 = reinterpret_cast<const uint32_t*>(row);
        const uint32_t w0 = w32[0], w1 = w32[1], w2 = w32[2];
        const uint32_t A = __builtin_amdgcn_alignbyte(w1, w0, sh), B = __builtin_amdgcn_alignbyte(w2, w1, sh);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
            h[j] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, __builtin_amdgcn_perm(B, A, sel[j])),
                                          __builtin_bit_cast(u16x2, wt[j]), 0u, false);
        }
    };
    for (int y = ylo + ph; y < yhi; y += PYR_RU * P) {
        ResizeY Yr[PYR_RU];
#pragma unroll
        for (int u = 0; u < PYR_RU; u++) Yr[u] = Y[min(y + u * P, yhi - 1)];
        uint32_t h0[PYR_RU][4], h1[PYR_RU][4];
#pragma unroll
        for (int u = 0; u < PYR_RU; u++) {
            hsum(sbase + Yr[u].sy0 * S.pitch, h0[u]);
            hsum(sbase + Yr[u].sy1 * S.pitch, h1[u]);
        }
#pragma unroll
        for (int u = 0; u < PYR_RU; u++) {
            uint32_t pk = 0;
#pragma unroll
            for (int j = 0; j < 4; j++)
                pk |= min((__umul24(h0[u][j], (uint32_t)Yr[u].b0) + __umul24(h1[u][j], (uint32_t)Yr[u].b1) + (1u << 21)) >> 22,
                          255u) << (8 * j);
            if (y + u * P < yhi) *reinterpret_cast<uint32_t*>(dbase + (size_t)(y + u * P) * D.pitch) = pk;
        }
    }
}
// gray of level-0 rows [r0, r1) (k_gray's arithmetic, PYR_GU quads of 4
// pixels in flight per thread): row y to gdst + y * pitch
ODO_INLINE void pyr_gray_rows(const uint8_t* __restrict__ src, uint8_t* gdst, int w, int pitch, int r0, int r1,
                              int t) {
    if ((w & 3) == 0) {
        const int nq4 = (r1 * w) >> 2;
        // (row, column) of the thread's next quad, stepped by PYR_TH quads
        // (4 PYR_TH pixels) without a division per quad
        const int q00 = ((r0 * w) >> 2) + t;
        int cy = (4 * q00) / w, cx = 4 * q00 - cy * w;
        const int dy = (4 * PYR_TH) / w, dx = 4 * PYR_TH - dy * w;
        for (int q0 = q00; q0 < nq4; q0 += PYR_GU * PYR_TH) {
            uint32_t wv[PYR_GU][3];
#pragma unroll
            for (int u = 0; u < PYR_GU; u++) {
                const int q = q0 + u * PYR_TH;
                if (q < nq4) {
                    const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + (size_t)q * 12);
                    if (PYR_NT & 1) {
                        wv[u][0] = __builtin_nontemporal_load(s32);
                        wv[u][1] = __builtin_nontemporal_load(s32 + 1);
                        wv[u][2] = __builtin_nontemporal_load(s32 + 2);
                    } else {
                        wv[u][0] = s32[0], wv[u][1] = s32[1], wv[u][2] = s32[2];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < PYR_GU; u++) {
                const int q = q0 + u * PYR_TH;
                const int y = cy, x = cx;
                cx += dx;
                cy += dy;
                if (cx >= w) cx -= w, cy++;
                if (q < nq4) {
                    uint32_t out = 0;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const int b = 3 * i;
                        const uint32_t B = (wv[u][b >> 2] >> (8 * (b & 3))) & 0xffu;
                        const uint32_t G = (wv[u][(b + 1) >> 2] >> (8 * ((b + 1) & 3))) & 0xffu;
                        const uint32_t R = (wv[u][(b + 2) >> 2] >> (8 * ((b + 2) & 3))) & 0xffu;
                        out |= ((B * 1868u + G * 9617u + R * 4899u + 8192u) >> 14) << (8 * i);
                    }
                    *reinterpret_cast<uint32_t*>(gdst + (size_t)y * pitch + x) = out;
                }
            }
        }
    } else {
        for (int p = r0 * w + t; p < r1 * w; p += PYR_TH) {
            const uint8_t* s = src + (size_t)p * 3;
            const int yy = p / w, xx = p - yy * w;
            gdst[(size_t)yy * pitch + xx] =
                (uint8_t)(((uint32_t)s[0] * 1868u + (uint32_t)s[1] * 9617u + (uint32_t)s[2] * 4899u + 8192u) >> 14);
        }
    }
}
template <bool BLUR>
__global__ void __launch_bounds__(PYR_TH) PYR_ATTR k_pyramid(const uint8_t* __restrict__ bgr, uint8_t* __restrict__ pyr,
                                                    size_t in_stride, size_t pyr_stride,
                                                    const LevelDesc* __restrict__ lv, const ResizeX* __restrict__ xt,
                                                    const ResizeY* __restrict__ yt, PyrLevels PL, int nlevels,
                                                    uint8_t* __restrict__ blur, BlurRows BR, PyrSplit SP) {
    EXTRACT_PRIO();
    // SP.parts == 2: two workgroups per frame, the top and the bottom part;
    // each builds every row it reads itself (rows both build are the same
    // bytes), so the parts never wait for each other
    const int part = SP.parts == 2 ? (int)(blockIdx.x & 1) : 0;
    const int f = SP.parts == 2 ? (int)(blockIdx.x >> 1) : (int)blockIdx.x;
    const int t = threadIdx.x;
    uint8_t* base = pyr + (size_t)f * pyr_stride;
    if (bgr) {
        const LevelDesc L0 = lv[0];
        pyr_gray_rows(bgr + (size_t)f * in_stride, base + L0.off, L0.w, L0.pitch, SP.lo[part][0], SP.hi[part][0], t);
    }
    for (int l = 1; l < nlevels; l++) {
        __syncthreads();  // level l - 1 is complete (this part's rows)
        const LevelDesc S = lv[l - 1], D = lv[l];
        if (BLUR)
            pyr_blur_level(base + S.off, blur, pyr_stride, lv, BR, nlevels, f, l - 1, S, t, SP.ca[part][l - 1],
                           SP.cb[part][l - 1], SP.ea[part][l - 1], SP.eb[part][l - 1]);
        pyr_resize_rows(base + S.off, base + D.off, S, D, xt + PL.rx_off[l], yt + PL.ry_off[l], t, SP.lo[part][l],
                        SP.hi[part][l]);
    }
    if (BLUR) {
        __syncthreads();  // the last level is complete
        const int ll = nlevels - 1;
        const LevelDesc L = lv[ll];
        pyr_blur_level(base + L.off, blur, pyr_stride, lv, BR, nlevels, f, ll, L, t, SP.ca[part][ll], SP.cb[part][ll],
                       SP.ea[part][ll], SP.eb[part][ll]);
    }
    __syncthreads();
}

// ============================================================ host-side launch helpers
void upload_extract_constants() { upload_finalize_constants(); }

}  // namespace odo

// ============================================================ launch wrappers
namespace odo {
void launch_gray(hipStream_t st, const uint8_t* bgr, uint8_t* pyr, int w, int h, int pitch, size_t in_stride,
                 size_t pyr_stride, int nframes) {
    dim3 g((w * h / 4 + 255) / 256 + 1, nframes);
    hipLaunchKernelGGL(k_gray, g, dim3(256), 0, st, bgr, pyr, w, h, pitch, in_stride, pyr_stride);
}
// k_blur_rows' work plan (strip items and edge lanes per level); false when a
// level is too small for its strips (the LDS-tiled k_blur then)
static bool blur_rows_plan(const LevelDesc* lv_host, int nlevels, BlurRows& R) {
    bool rows = nlevels <= 16;
    for (int l = 0; l < nlevels; l++) rows = rows && lv_host[l].h >= BR_R && lv_host[l].w >= 12;
    if (!rows) return false;
    R = BlurRows{};
    int acc = 0, eacc = 0;
    for (int l = 0; l < nlevels; l++) {
        const LevelDesc& L = lv_host[l];
        R.base[l] = acc;
        R.ebase[l] = eacc;
        R.nq[l] = (L.w - 8) / 4;  // x + 7 <= w - 1: the lane's three dwords stay inside the row
        R.nst[l] = (R.nq[l] + 15) / 16;
        R.nch[l] = (L.h + BR_R - 1) / BR_R;
        acc += R.nst[l] * R.nch[l];
        eacc += (1 + (L.w + 3) / 4 - (R.nq[l] + 1)) * ((L.h + BR_RE - 1) / BR_RE);
    }
    R.base[nlevels] = acc;
    R.ebase[nlevels] = eacc;
    return true;
}
bool pyramid_blur_fusable(const LevelDesc* lv_host, int nlevels) {
    BlurRows R;
    return blur_rows_plan(lv_host, nlevels, R);
}
// The part ranges of k_pyramid (PyrSplit). parts == 1: everything. parts == 2:
// level l's blur rows split at s_l (a multiple of BR_R = 30, so the 30-row
// strip chunks and 6-row edge chunks split with it; a level under 60 rows is
// blurred by the top part alone); each part builds the rows its blur reads
// (3-row halo) and the source rows of the next level's rows it builds, from
// the top level down. Every row keeps its one arithmetic, so rows both parts
// build are the same bytes. ry_h: the host copy of the vertical resize table.
static void pyramid_split_plan(const LevelDesc* lv_host, const ResizeY* ry_h, const int* ry_off, int nlevels,
                               int parts, PyrSplit& S) {
    S = PyrSplit{};
    S.parts = parts;
    for (int l = 0; l < nlevels && l < 16; l++) {
        const int h = lv_host[l].h, nch = (h + BR_R - 1) / BR_R, nch6 = (h + BR_RE - 1) / BR_RE;
        for (int p = 0; p < 2; p++) {
            S.lo[p][l] = 0, S.hi[p][l] = h;
            S.ca[p][l] = 0, S.cb[p][l] = nch, S.ea[p][l] = 0, S.eb[p][l] = nch6;
        }
    }
    if (parts != 2 || nlevels > 16 || !ry_h) {
        S.parts = 1;
        return;
    }
    int sp[16];
    for (int l = 0; l < nlevels; l++) {
        const int h = lv_host[l].h;
        int s = ((h / 2 + BR_R / 2) / BR_R) * BR_R;  // the multiple of 30 nearest h / 2
        if (h < 2 * BR_R) s = h;                       // too small to split: the top part blurs it all
        s = std::min(s, h < 2 * BR_R ? h : h - BR_R);
        sp[l] = s;
        const int nch = (h + BR_R - 1) / BR_R, nch6 = (h + BR_RE - 1) / BR_RE;
        S.ca[0][l] = 0, S.cb[0][l] = s == h ? nch : s / BR_R;
        S.ca[1][l] = S.cb[0][l], S.cb[1][l] = nch;
        S.ea[0][l] = 0, S.eb[0][l] = s == h ? nch6 : s / BR_RE;
        S.ea[1][l] = S.eb[0][l], S.eb[1][l] = nch6;
    }
    // rows built per part, from the top level down
    for (int l = nlevels - 1; l >= 0; l--) {
        const int h = lv_host[l].h;
        int thi = std::min(h, sp[l] + 3), blo = std::max(0, sp[l] - 3);
        if (sp[l] == h) blo = h;  // the bottom part blurs none of this level
        if (l + 1 < nlevels) {
            const ResizeY* Y = ry_h + ry_off[l + 1];
            if (S.hi[0][l + 1] > 0) thi = std::max(thi, Y[S.hi[0][l + 1] - 1].sy1 + 1);
            if (S.lo[1][l + 1] < lv_host[l + 1].h) blo = std::min(blo, Y[S.lo[1][l + 1]].sy0);
        }
        S.lo[0][l] = 0, S.hi[0][l] = std::min(h, thi);
        S.lo[1][l] = std::max(0, blo), S.hi[1][l] = h;
        if (S.lo[1][l] >= h) S.lo[1][l] = h;  // nothing to build
    }
}
void launch_pyramid(hipStream_t st, const uint8_t* bgr, uint8_t* pyr, size_t in_stride, size_t pyr_stride,
                    const LevelDesc* lv, const ResizeX* rx, const ResizeY* ry, const int* rx_off, const int* ry_off,
                    int nlevels, int nframes, uint8_t* blur, const LevelDesc* lv_host, const ResizeY* ry_h) {
    PyrLevels PL{};
    for (int l = 0; l < nlevels && l < 16; l++) PL.rx_off[l] = rx_off[l], PL.ry_off[l] = ry_off[l];
    PyrSplit SP;
    pyramid_split_plan(lv_host, ry_h, ry_off, nlevels, PYR_PARTS, SP);
    const dim3 g(nframes * SP.parts);
    BlurRows BR{};
    if (blur && blur_rows_plan(lv_host, nlevels, BR)) {
        hipLaunchKernelGGL(k_pyramid<true>, g, dim3(PYR_TH), 0, st, bgr, pyr, in_stride, pyr_stride, lv, rx, ry, PL,
                           nlevels, blur, BR, SP);
        return;
    }
    hipLaunchKernelGGL(k_pyramid<false>, g, dim3(PYR_TH), 0, st, bgr, pyr, in_stride, pyr_stride, lv, rx, ry, PL,
                       nlevels, (uint8_t*)nullptr, BR, SP);
}
bool pyramid_fusable(const LevelDesc* lv_host, const ResizeX* rx, const int* rx_off, int nlevels) {
    if (nlevels > 16) return false;
    for (int l = 1; l < nlevels; l++) {
        const LevelDesc& D = lv_host[l];
        const int nq = (D.w + 3) / 4;
        if (nq > PYR_TH) return false;
        const ResizeX* X = rx + rx_off[l];
        for (int q = 0; q < nq; q++) {
            const int x00 = X[4 * q].sx0;
            for (int j = 0; j < 4 && 4 * q + j < D.w; j++) {
                const ResizeX& xj = X[4 * q + j];
                if (xj.sx0 < x00 || xj.sx1 < x00 || xj.sx0 - x00 > 7 || xj.sx1 - x00 > 7) return false;
                if (xj.a0 < 0 || xj.a0 > 65535 || xj.a1 < 0 || xj.a1 > 65535) return false;
            }
        }
    }
    return true;
}
size_t resize_lds_bytes(int spitch, int dw, int max_src_rows) {
    return (size_t)((dw + 3) & ~3) * sizeof(ResizeX) + (size_t)max_src_rows * spitch;
}
void launch_resize(hipStream_t st, uint8_t* pyr, size_t pyr_stride, int src_off, int spitch, int dst_off, int dpitch,
                   int dw, int dh, int rb, int max_src_rows, const ResizeX* xt, const ResizeY* yt, int nframes) {
    dim3 g((dh + rb - 1) / rb, nframes);
    const size_t lds = resize_lds_bytes(spitch, dw, max_src_rows);
    hipLaunchKernelGGL(k_resize, g, dim3(256), lds, st, pyr, pyr_stride, src_off, spitch, dst_off, dpitch, dw, dh, rb,
                       xt, yt);
}
bool fast_lds_plan(const FastSeg* segs, int nsegs, FastLds& L) {
    int img = 16, bw = 1, rows = 1, nl = 1;
    for (int k = 0; k < nsegs; k++) {
        img = std::max(img, (int)segs[k].rows * FS_RS);
        bw = std::max(bw, (int)segs[k].rows * (int)segs[k].bw);
        rows = std::max(rows, (int)segs[k].rows);
        nl = std::max(nl, FS_RS / 4 + FS_NCM);
        if ((int)segs[k].ncell > FS_NCM || (int)segs[k].rows * FS_RS > 65536 || ((segs[k].x0 & 15) + segs[k].cols) > FS_RS)
            return false;
    }
    auto al = [](int x) { return (x + 15) & ~15; };
    L.img = al(img);
    L.ring = 2 * L.img;
    L.clist = L.ring + (FS_TH / 64) * FS_RSTRIDE * 2;
    L.bits = al(L.clist + FS_CL * 2);
    L.cnt = al(L.bits + bw * 4);
    L.qlist = al(L.cnt + rows * FS_NCM * 4);
    L.misc = al(L.qlist + nl * 8);
    L.total = al(L.misc + (int)sizeof(FastMisc));
    return L.total <= 160 * 1024;
}
void launch_fast(hipStream_t st, const uint8_t* pyr, size_t pyr_stride, const FastSeg* segs, int nsegs,
                 const LevelDesc* lv, uint32_t* cand, int* cand_cnt, int ncells, int cell_cap, int ini_th, int min_th,
                 const FastLds& lds, int nframes) {
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k_fast_seg, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    hipLaunchKernelGGL(k_fast_seg, dim3(nsegs, nframes), dim3(FS_TH), lds.total, st, pyr, pyr_stride, segs, lv, cand,
                       cand_cnt, ncells, cell_cap, ini_th, min_th, lds);
#ifdef FS_STATS
    unsigned long long h[8];
    (void)hipStreamSynchronize(st);
    (void)hipMemcpyFromSymbol(h, HIP_SYMBOL(fs_stats), sizeof(h));
    fprintf(stderr, "fs_stats frames %d segs %d items0 %llu items1 %llu survivors %llu segtest_calls %llu corners %llu ovf %llu retry_cells %llu cells %llu\n",
            nframes, nsegs, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
    static const unsigned long long z[8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(fs_stats), z, sizeof(z));
#endif
}
size_t octree_lds_bytes(int node_cap) { return (size_t)76 * node_cap + 1032; }
void launch_octree(hipStream_t st, const uint32_t* cand, const int* cand_cnt, const LevelDesc* lv, int ncells,
                   int cell_cap, int nlevels, uint32_t* keys, int32_t* knode, uint8_t* kquad, size_t keys_stride,
                   uint32_t* okp, int* ocnt, int okp_stride, int node_cap, int nframes) {
    const dim3 g(nlevels, nframes);
    hipLaunchKernelGGL(k_octree, g, dim3(OT_THREADS), octree_lds_bytes(node_cap), st, cand, cand_cnt, lv, ncells,
                       cell_cap, nlevels, keys, knode, kquad, keys_stride, okp, ocnt, okp_stride, node_cap);
}
void launch_blur(hipStream_t st, const uint8_t* pyr, uint8_t* blur, size_t pyr_stride, const LevelDesc* lv,
                 const LevelDesc* lv_host, int nlevels, int nframes) {
    // k_blur_rows needs BR_R interior rows and one interior quad per level;
    // smaller levels take the LDS-tiled kernel (ODO_BLUR_TILES=1 forces it)
    static const bool tiles = [] {
        const char* e = odo_knob("ODO_BLUR_TILES");
        return e && e[0] == '1';
    }();
    BlurRows R{};
    if (!tiles && blur_rows_plan(lv_host, nlevels, R)) {
        const int acc = R.base[nlevels], eacc = R.ebase[nlevels];
        const int eblocks = (eacc + 255) / 256;
        hipLaunchKernelGGL(k_blur_rows, dim3(eblocks + (acc + 15) / 16, nframes), dim3(256), 0, st, pyr, blur,
                           pyr_stride, lv, R, nlevels, eblocks);
        return;
    }
    BlurTiles T{};
    int acc = 0;
    for (int l = 0; l < nlevels; l++) {
        T.base[l] = acc;
        T.tx[l] = (lv_host[l].w + BLUR_TX - 1) / BLUR_TX;
        acc += T.tx[l] * ((lv_host[l].h + BLUR_TY - 1) / BLUR_TY);
    }
    T.base[nlevels] = acc;
    hipLaunchKernelGGL(k_blur, dim3(acc, nframes), dim3(256), 0, st, pyr, blur, pyr_stride, lv, T, nlevels);
}
// Frame roll: the last frame of a batch becomes slot 0 (Tracking::mLastFrame)
// of the next batch's frame set. One launch for all per-frame feature arrays
// (16-byte moves; every array is kp_cap-sized, kp_cap a multiple of 64).
struct FrameCopy {
    const uint4* src[5];
    uint4* dst[5];
    int n16[5];
    const int* nsrc;
    int* ndst;
};

__global__ void __launch_bounds__(256) k_copy_frame(FrameCopy F) {
    const int a = blockIdx.y;
    const uint4* s = F.src[a];
    uint4* d = F.dst[a];
    for (int i = blockIdx.x * 256 + threadIdx.x; i < F.n16[a]; i += gridDim.x * 256) d[i] = s[i];
    if (a == 0 && blockIdx.x == 0 && threadIdx.x == 0) *F.ndst = *F.nsrc;
}

void launch_copy_frame(hipStream_t st, const orb_kp* kps_s, const uint8_t* desc_s, const float* kun_s,
                       const float* xyz_s, const float* ur_s, const int* n_s, orb_kp* kps_d, uint8_t* desc_d,
                       float* kun_d, float* xyz_d, float* ur_d, int* n_d, int kp_cap) {
    FrameCopy F;
    const size_t bytes[5] = {(size_t)kp_cap * sizeof(orb_kp), (size_t)kp_cap * 32, (size_t)kp_cap * 8,
                             (size_t)kp_cap * 12, (size_t)kp_cap * 4};
    const void* s[5] = {kps_s, desc_s, kun_s, xyz_s, ur_s};
    void* d[5] = {kps_d, desc_d, kun_d, xyz_d, ur_d};
    for (int i = 0; i < 5; i++) {
        F.src[i] = (const uint4*)s[i];
        F.dst[i] = (uint4*)d[i];
        F.n16[i] = (int)(bytes[i] / 16);
    }
    F.nsrc = n_s;
    F.ndst = n_d;
    hipLaunchKernelGGL(k_copy_frame, dim3(8, 5), dim3(256), 0, st, F);
}

__global__ void k_pair_valid(int* pv, int n, int first_valid) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) pv[i] = (i > 0 || first_valid) ? 1 : 0;
}

void launch_pair_valid(hipStream_t st, int* pv, int n, int first_valid) {
    hipLaunchKernelGGL(k_pair_valid, dim3((n + 255) / 256), dim3(256), 0, st, pv, n, first_valid);
}
}  // namespace odo
