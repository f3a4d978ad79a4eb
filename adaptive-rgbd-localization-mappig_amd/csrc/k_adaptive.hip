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
#include "odo_select.h"
#include "../../include/odo_orb_pattern.h"

namespace odo {

__constant__ int8_t c_apattern[1024];

// ============================================================ S map
// Tile: 128 x 8 output pixels of the pitched level 0 (smap_tile, odo_select.h).
__global__ void __launch_bounds__(256) k_adapt_smap(const uint8_t* __restrict__ pyr, size_t pyr_stride, int w, int h,
                                                    int pitch, int tiles_x, uint8_t* __restrict__ smap,
                                                    size_t smap_stride) {
    __shared__ uint32_t lds[SM_LR * SM_LW / 4];
    const int f = blockIdx.y;
    const int tx0 = (blockIdx.x % tiles_x) * SM_TW, ty0 = (blockIdx.x / tiles_x) * SM_TH;
    smap_tile(pyr + (size_t)f * pyr_stride, w, h, pitch, tx0, ty0, smap + (size_t)f * smap_stride, lds);
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
    if (m > max_per_cell) block_nth_element<uint32_t, ScoreKey>(A, m, max_per_cell, posL, posR, S);
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
            block_nth_element<uint32_t, ScoreKey>(A, n, retain, posL, posR, S);
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
    block_nth_element<uint32_t, ScoreKey>(A, n, nth, posL, posR, S);
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
