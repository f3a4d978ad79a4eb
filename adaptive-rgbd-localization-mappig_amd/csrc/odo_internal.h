// Internal (non-ABI) structures shared by the HIP kernels and the host
// orchestration in odo_capi.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/odo_types.h"

namespace odo {

// Measurement / A-B knobs (stream schedules, stage skipping, retired kernel
// forms, grid sizes). Only the tuning build (make tuning: -DODO_TUNING,
// build_tuning/libodo_hip.so, selected with ODO_LIB) reads them from the
// environment; the production library ignores the environment entirely, so a
// stray variable cannot change (or invalidate) a production context.
static inline const char* odo_knob(const char* name) {
#ifdef ODO_TUNING
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}

#define FAST_ROI_MAX 72  // largest FAST cell ROI side (a level narrower than 2 cells: up to 65)

// One pyramid level of one frame (all frames share the geometry).
struct LevelDesc {
    int off;          // byte offset of the level inside a frame's pyramid buffer
    int w, h;
    int pitch;        // row stride in bytes (w rounded up to 16)
    float scale;      // mvScaleFactor[level] (float, orbextractor.cpp:358)
    int quota;        // mnFeaturesPerLevel[level]
    int cell_begin;   // range in the global cell table
    int cell_end;
    int key_off;      // offset of this level's key scratch inside a frame's key buffer
};

// One FAST cell ROI (orbextractor.cpp:688-711).
struct CellDesc {
    int16_t level;
    int16_t rows, cols;
    int16_t x0, y0;   // ROI origin in level pixels
    int16_t offx, offy;  // j*wCell, i*hCell (added to ROI coords, relative to the 16px border)
    int16_t pad;
};

// A FAST segment (k_fast_seg): cells [ja, ja + ncell) of one cell row of one
// level, whose ROIs (orbextractor.cpp:688-703) are staged in LDS as one union:
// rows [y0, y0 + rows), cols [x0, x0 + cols) of the level; cell jl of the
// segment is cells_h[ci0 + jl] (ROI x0 + jl*wcell).
#ifndef FS_SEGC
#define FS_SEGC 8  // cells per segment (at most; the host splits a cell row evenly)
#endif
#define FS_NCM FS_SEGC
// LDS row stride of a staged segment (bytes): a compile-time constant, so the
// kernel's neighbour offsets (the 16 circle pixels, the compass points, the
// NMS neighbours) are instruction immediates; the host sizes segments to fit
// it. 272 = 68 dwords, a 16-byte multiple (the staging stores) that moves each
// row 4 banks over: with 256 every row of a column fell in the same bank, and
// the segment test's scattered circle reads of candidates from different rows
// conflicted (profiles/r05_rs)
#ifndef FS_RS
#define FS_RS 272
#endif
struct FastSeg {
    int level, ci0;
    int16_t y0, x0, rows, cols, ncell, wcell;
    int16_t bw, pad;  // kept-bitmap words per row
};
// k_fast_seg's dynamic LDS: byte offsets of its regions
struct FastLds {
    int img;  // bytes of the staged ROI union (the score map follows at img)
    int ring, clist, bits, cnt, qlist, misc, total;
};

// cv::resize INTER_LINEAR tables (per output column / row).
struct ResizeX {
    int sx0, sx1;
    int a0, a1;
};
struct ResizeY {
    int sy0, sy1;
    int b0, b1;
};

struct FrameCalib {
    float fx, fy, cx, cy;
    float k1, k2, p1, p2, k3;
    float depth_factor, mbf;
    float invfx, invfy;
};

// Frame::ExtractFeatures tail for one keypoint (frame.cpp:139-164, 286-313):
// cv::undistortPoints (5 iterations in double; skipped when k1 == 0,
// frame.cpp:288), then the depth at the truncated distorted pixel and the
// back-projection of the undistorted point.
__device__ inline void kp_geometry(float uu, float vv, const FrameCalib& cal, const uint16_t* depth, int img_w,
                                   float* ku, float* p3, float* urp) {
    float ux = uu, uy = vv;
    if (cal.k1 != 0.0f) {
        const double fx = cal.fx, fy = cal.fy, cx = cal.cx, cy = cal.cy;
        const double ifx = 1. / fx, ify = 1. / fy;
        const double k0 = cal.k1, k1 = cal.k2, k2 = cal.p1, k3 = cal.p2, k4 = cal.k3;
        double x = uu, y = vv;
        x = (x - cx) * ifx;
        y = (y - cy) * ify;
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {
            double r2 = x * x + y * y;
            double icdist = 1 / (1 + ((k4 * r2 + k1) * r2 + k0) * r2);
            double deltaX = 2 * k2 * x * y + k3 * (r2 + 2 * x * x);
            double deltaY = k2 * (r2 + 2 * y * y) + 2 * k3 * x * y;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
        ux = (float)(fx * x + cx);
        uy = (float)(fy * y + cy);
    }
    ku[0] = ux;
    ku[1] = uy;
    float urv = -1.f, X = 0.f, Y = 0.f, Z = 0.f;
    const uint16_t d16 = depth[(size_t)((int)vv) * img_w + (int)uu];
    const float z = (float)d16 * cal.depth_factor + 0.0f;
    if (z > 0) {
        urv = ux - cal.mbf / z;
        X = (ux - cal.cx) * z * cal.invfx;
        Y = (uy - cal.cy) * z * cal.invfy;
        Z = z;
    }
    p3[0] = X;
    p3[1] = Y;
    p3[2] = Z;
    *urp = urv;
}

// ---- ADAPTIVE grid extractor (k_adaptive.hip)
#define AD_BH 16          // rows per candidate band
#define AD_MAXW 1024      // widest cell detection region (LDS staging)
#define AD_SEL_LDS 4096   // survivors a cell selects in LDS (more: global scratch)
using AdParams = odo_adaptive_params;

// One grid cell of VideoGridAdaptedFeatureDetector (videogridadaptedfeature
// detector.cpp:62-71): ROI [rs,re) x [cs,ce); FAST's detection region is the
// ROI minus 3 pixels on every side: rows [r0,r1), cols [c0,c1).
struct AdCell {
    int rs, re, cs, ce;
    int r0, r1, c0, c1;
    int band0, band1;  // its bands in the band table
    int cand_cap;      // survivor capacity over all its bands
    int pad;
};
// AD_BH rows [y0,y1) of one cell's detection region; its survivors land at
// cand_off of the frame's candidate buffer
struct AdBand {
    int cell, y0, y1, cand_off;
};

// ---- ADAPTIVE grid with the cv::ORB inner detector (k_adaptive_orb.hip):
// cv::ORB::create(10000, 1.2f, 8, 15, 0, 2, HARRIS_SCORE, 31, t) per grid
// cell (detectoradjuster.cpp:29)
#define OA_NLEV 8     // nlevels
#define OA_EDGE 15    // edgeThreshold (runByImageBorder of each level)
#define OA_PATCH 31   // patchSize
#ifndef OA_BH
#define OA_BH 64      // rows per candidate band of a cell level (k_oa_scand; 32: -1 %, profiles/r02_oa_bands_ab)
#endif
// one pyramid level of one grid cell, inside a frame's cell-pyramid buffer
struct OaImg {
    int off, w, h, pitch;
    int quota;         // nfeaturesPerLevel[level] of nfeatures 10000
    int band0, band1;  // its candidate bands (rows [15, h-15))
    int cand_cap;      // survivors over its bands
};
// one grid cell: ROI origin / size in the frame, its 8 level images
struct OaCell {
    int rs, cs, cw, ch;
    int img0;
    int pad[3];
};
struct OaBand {
    int img, y0, y1, cand_off;
};
struct OaScales {
    float s[OA_NLEV];  // getScale(level) = (float)pow((double)1.2f, level)
};

// RANSAC per-pair constants.
struct RansacCfg {
    int iterations;
    int min_inlier_th;
    float max_mahal;
    int sample_size;
    int check_depth;
    double raster_cov_x, raster_cov_y;
    int h0;     // hypotheses of the first eval launch ([0, h0)); set by launch_ransac
    int lanes_min_open;  // odo_kernel_forms.ransac_lanes_min_open (0 = default)
    int fold_wave;       // ordered fold by the whole wave (a lone pair); set by launch_ransac
    int first_hyps;      // odo_kernel_forms.ransac_first_hyps (0 = EV_H0)
};

// ---- launch wrappers (defined next to their kernels)
void upload_extract_constants();
void upload_finalize_constants();
void launch_kp_geometry(hipStream_t st, const orb_kp* kps, const int* nkp, const uint16_t* depth, size_t depth_stride,
                        int img_w, FrameCalib cal, float* kun, float* xyz, float* ur, int kp_cap, int nframes);
void launch_gray(hipStream_t st, const uint8_t* bgr, uint8_t* pyr, int w, int h, int pitch, size_t in_stride,
                 size_t pyr_stride, int nframes);
size_t resize_lds_bytes(int spitch, int dw, int max_src_rows);
// gray + every pyramid level in one launch (one workgroup per frame); bgr may be
// null (level 0 already in place). pyramid_fusable: the host check of its
// assumptions (<= 16 levels, <= 4096 px wide, each quad's taps inside 8 bytes)
void launch_pyramid(hipStream_t st, const uint8_t* bgr, uint8_t* pyr, size_t in_stride, size_t pyr_stride,
                    const LevelDesc* lv, const ResizeX* rx, const ResizeY* ry, const int* rx_off, const int* ry_off,
                    int nlevels, int nframes, uint8_t* blur, const LevelDesc* lv_host,
                    const ResizeY* ry_h);
// blur: the blurred pyramid is written by the same launch (null: not);
// pyramid_blur_fusable: every level is large enough for the strip walks
bool pyramid_blur_fusable(const LevelDesc* lv_host, int nlevels);
bool pyramid_fusable(const LevelDesc* lv_host, const ResizeX* rx, const int* rx_off, int nlevels);
void launch_resize(hipStream_t st, uint8_t* pyr, size_t pyr_stride, int src_off, int spitch, int dst_off, int dpitch,
                   int dw, int dh, int rb, int max_src_rows, const ResizeX* xt, const ResizeY* yt, int nframes);
void launch_fast(hipStream_t st, const uint8_t* pyr, size_t pyr_stride, const FastSeg* segs, int nsegs,
                 const LevelDesc* lv, uint32_t* cand, int* cand_cnt, int ncells, int cell_cap, int ini_th, int min_th,
                 const FastLds& lds, int nframes);
// LDS layout of k_fast_seg for the context's largest segment (false: too large)
bool fast_lds_plan(const FastSeg* segs, int nsegs, FastLds& L);
size_t octree_lds_bytes(int node_cap);
void launch_octree(hipStream_t st, const uint32_t* cand, const int* cand_cnt, const LevelDesc* lv, int ncells,
                   int cell_cap, int nlevels, uint32_t* keys, int32_t* knode, uint8_t* kquad, size_t keys_stride,
                   uint32_t* okp, int* ocnt, int okp_stride, int node_cap, int nframes);
void launch_blur(hipStream_t st, const uint8_t* pyr, uint8_t* blur, size_t pyr_stride, const LevelDesc* lv,
                 const LevelDesc* lv_host, int nlevels, int nframes);
void launch_finalize(hipStream_t st, const uint8_t* pyr, const uint8_t* blur, size_t pyr_stride, const LevelDesc* lv,
                     int nlevels, const uint32_t* okp, const int* ocnt, int okp_stride, const uint16_t* depth,
                     size_t depth_stride, int img_w, FrameCalib cal, orb_kp* kps, uint8_t* desc, float* kun, float* xyz,
                     float* ur, int* nkp, int kp_cap, int nframes, bool geometry = true);
void launch_pair_valid(hipStream_t st, int* pv, int n, int first_valid);
void launch_copy_frame(hipStream_t st, const orb_kp* kps_s, const uint8_t* desc_s, const float* kun_s,
                       const float* xyz_s, const float* ur_s, const int* n_s, orb_kp* kps_d, uint8_t* desc_d,
                       float* kun_d, float* xyz_d, float* ur_d, int* n_d, int kp_cap);
void launch_knn2(hipStream_t st, const uint8_t* q, const int* qn, size_t q_stride, const uint8_t* t, const int* tn,
                 size_t t_stride, int2* idx, int2* dist, size_t out_stride, int max_q, int npairs,
                 const int32_t* qlist = nullptr, const int* qcnt = nullptr, size_t ql_stride = 0, int nsplit = 1,
                 size_t split_stride = 0);
// the same top-2 on the matrix cores (exact int8 sign-vector formulation); one
// split slot, all trains (k_knn2_mx)
// kNN-2 kernel forms (ODO_KNN_MFMA): VALU xor/popcount, int8 MFMA, FP4 MFMA
enum { KNN_FMT_VALU = 0, KNN_FMT_I8 = 1, KNN_FMT_F4 = 2 };
void launch_knn2_mx(hipStream_t st, const uint8_t* q, const int* qn, size_t q_stride, const uint8_t* t, const int* tn,
                    size_t t_stride, int2* idx, int2* dist, size_t out_stride, int max_q, int npairs,
                    const int32_t* qlist = nullptr, const int* qcnt = nullptr, size_t ql_stride = 0,
                    int fmt = KNN_FMT_I8);
void launch_vo_lm(hipStream_t st, const float* xyz, const int* nkp, int kp_cap, int slot0, float th_depth_m,
                  uint32_t* lm_bits, int lm_words, int32_t* qlist, int* qcnt, int npairs);
void launch_pair_match(hipStream_t st, const int2* knn_idx, const int2* knn_dist, size_t knn_stride, const float* xyz,
                       const int* nkp, int kp_cap, int slot0, float ratio, const uint32_t* lm_bits, int lm_words,
                       int nsplit, size_t split_stride, int check_depth,
                       odo_dmatch* matches, int* n_matches, void* good, int* n_good, int32_t* f2_src,
                       uint64_t* sort_scratch, int match_cap, int npairs);
int launch_sort_dbg(hipStream_t st, void* a, int n);
void launch_latch(hipStream_t st, double* latch, const void* good, const int* n_good, const int* n_matches,
                  const odo_dmatch* matches, const float* xyz, int kp_cap, int slot0, int npairs, int match_cap,
                  int min_inl, int sample_size, int iterations, const int* pair_valid, int* set_flag = nullptr);
size_t ransac_gpt_bytes();
// rand() words for every pair (data independent): launched at batch start on
// a side stream; launch_ransac's stream must wait for it.
void launch_ransac_raw(hipStream_t st, void* scratch, int npairs, int match_cap, int mask_words, RansacCfg cfg,
                       uint64_t seed_base, uint64_t pair_base, odo_rng* rng_io);
void launch_ransac(hipStream_t st, const void* good, const int* n_good, const int* n_matches,
                   const odo_dmatch* matches, const float* xyz, int kp_cap, int slot0, int match_cap, RansacCfg cfg,
                   const double* latch, const int* pair_valid, int min_matches, odo_rng* rng_io, void* scratch,
                   uint32_t* best_mask, int mask_words, odo_pair_result* res, float* T12, int npairs, int part = 0,
                   int* phase = nullptr, int* open_hint = nullptr);
size_t ransac_scratch_bytes(int npairs, int match_cap, int mask_words, const RansacCfg& cfg);
void ransac_read_hyps(hipStream_t st, void* scratch, int match_cap, int mask_words, RansacCfg cfg, int h0, int h1,
                      double* err, int* cnt, float* T);
void launch_ransac_finish(hipStream_t st, void* scratch, int match_cap, int mask_words, RansacCfg cfg,
                          const double* latch, odo_rng* rng_io, uint32_t* best_mask, odo_pair_result* res, float* T12,
                          int best_h, int visited, int valid, int best_cnt, float rmse);
// hypotheses mode with the exchange on the device (odo_ransac_hyps_dev ...)
void ransac_export_hyps(hipStream_t st, void* scratch, int match_cap, int mask_words, RansacCfg cfg, int h0, int h1,
                        void* d_block);
void launch_hyp_fold(hipStream_t st, const void* d_all, int H, int iterations, int ng, int min_inl, int sample_size,
                     odo_ransac_fold_result* d_out);
void launch_hyp_finish(hipStream_t st, void* scratch, int match_cap, int mask_words, RansacCfg cfg,
                       const double* latch, odo_rng* rng_io, uint32_t* best_mask, odo_pair_result* res, float* T12,
                       const odo_ransac_fold_result* d_fold, int h0, int h1, int rank0, const odo_dmatch* good, int ng,
                       int* payload, int words);
int hyp_payload_words(int ng);
size_t pnp_edge_bytes();
void launch_pnp(hipStream_t st, const int32_t* f2_src, const float* xyz, const float* kun, const float* ur,
                const int* nkp, int kp_cap, int slot0, FrameCalib cal, const float* T12, const int* pair_valid,
                const int* n_matches, int min_matches, void* edges, odo_pair_result* res, uint8_t* inlier_mask,
                int npairs, const int* sel = nullptr, int sel_val = 0);
void launch_kabsch(hipStream_t st, const float* A, const float* B, int n, float* T);
// GICP (k_gicp.hip), nprob problems: source p = points [soffs[p], soffs[p+1]) of
// src, target p = [toffs[p], toffs[p+1]) of tgt. Cs sum(ns)*9, Ct sum(nt)*9,
// outp sum(ns)*3, Mah sum(ns)*9, is / it sum(ns); T12 16 and outi 4 per problem.
struct GicpArgs {
    const float* guess;  // 16 per problem (device)
    const int* soffs;    // nprob + 1 (device)
    const int* toffs;
    double max_corr_dist;
    int max_iterations;
    int max_inner;
};
void launch_gicp(hipStream_t st, const float* src, const float* tgt, int nprob, int max_ns, int max_nt, double* Cs,
                 double* Ct, float* outp, double* Mah, int* is, int* it, GicpArgs args, float* T12, int* outi);
// PnPRansac (k_pnpransac.hip), nprob problems, problem p = points [offs[p], offs[p+1]):
// idx P*H*5, model P*H*6, Rproj P*H*9, mask H*sum(n), good P*H, state P*4, res P, mask_out sum(n)
int pnp_ransac_max_points();
void launch_pnp_ransac(hipStream_t st, const float* Xw, const float* uv, const int* offs, int nprob,
                       const float K4[4], int H, float reproj_err, double confidence, int* idx, double* model,
                       double* Rproj, uint8_t* mask, int* good, int* state, odo_pnp_ransac_result* res,
                       uint8_t* mask_out);
int launch_projection_match(hipStream_t st, const float* Tcw, const odo_landmark* lms, int nL, const float* kun,
                            const int32_t* octave, const uint8_t* desc, int n, const uint8_t* slot_taken,
                            const float* calib5, const float* bounds, float th, float nnratio, float* proj,
                            uint8_t* inview, int* ccount, uint32_t* cand, int32_t* slot_lm, int* nmatches);
size_t projection_cand_cap();
void upload_adaptive_constants();
void launch_adapt_smap(hipStream_t st, const uint8_t* pyr, size_t pyr_stride, int w, int h, int pitch, uint8_t* smap,
                       size_t smap_stride, int nframes);
void launch_adapt_cand(hipStream_t st, const uint8_t* smap, size_t smap_stride, int pitch, const AdBand* bands,
                       int nbands, const AdCell* cells, int ncells, uint32_t* cand, size_t cand_stride, int* band_cnt,
                       int* hist, int nframes);
void launch_adapt_chain(hipStream_t st, const int* hist, int ncells, int nframes, AdParams P, double* thresh,
                        int* tsel, int* nsel);
size_t adapt_select_lds_bytes();
void launch_adapt_select(hipStream_t st, const uint32_t* cand, size_t cand_stride, const int* band_cnt, int nbands,
                         const AdBand* bands, const AdCell* cells, int ncells, const int* tsel, const int* nsel,
                         int max_per_cell, uint32_t* big, size_t big_stride, uint32_t* cell_out, int* cell_cnt,
                         int nframes);
size_t adapt_assemble_lds_bytes(int ncells, int max_per_cell);
void launch_adapt_assemble(hipStream_t st, const uint32_t* cell_out, const int* cell_cnt, int ncells, int max_per_cell,
                           int retain, int w, int h, uint32_t* akp, int akp_stride, int* nkp, int kp_cap,
                           int nframes);
void launch_adapt_finalize(hipStream_t st, const uint8_t* blur, size_t pyr_stride, int pitch, const uint32_t* akp,
                           int akp_stride, const int* nkp, float ca, float sb, const uint16_t* depth,
                           size_t depth_stride, int img_w, FrameCalib cal, orb_kp* kps, uint8_t* desc, float* kun,
                           float* xyz, float* ur, int kp_cap, int nframes);
void upload_adaptive_orb_constants();
void launch_oa_pyr(hipStream_t st, const uint8_t* pyr, size_t pyr_stride, int gpitch, const OaCell* cells, int ncells,
                   const OaImg* imgs, int buf0, int buf1, uint8_t* cpyr, size_t cp_stride, int nframes);
size_t oa_scand_lds_bytes(int maxpitch);
void launch_oa_scand(hipStream_t st, const uint8_t* cpyr, size_t cp_stride, const OaImg* imgs, int nimgs,
                     const OaBand* bands, int nbands, uint32_t* cand, size_t cand_stride, int* band_cnt, int* hist,
                     int maxpitch, int nframes);
void launch_oa_count(hipStream_t st, const int* hist, const OaCell* cells, const OaImg* imgs, int nimgs, int ncells,
                     int* phist, int nframes);
size_t oa_select_scratch_bytes(int ncap);
void launch_oa_select(hipStream_t st, const uint32_t* cand, size_t cand_stride, const int* band_cnt, int nbands,
                      const OaBand* bands, const OaImg* imgs, const OaCell* cells, int ncells, const int* tsel,
                      const uint8_t* cpyr, size_t cp_stride, int max_per_cell, uint8_t* scr, size_t scr_stride,
                      int ncap, uint64_t* cell_out, int* cell_cnt, int nframes);
size_t oa_assemble_lds_bytes(int ncells, int max_per_cell);
void launch_oa_assemble(hipStream_t st, const uint64_t* cell_out, const int* cell_cnt, const OaCell* cells,
                        int ncells, int max_per_cell, int retain, int w, int h, OaScales sc, uint64_t* akp,
                        int akp_stride, int* nkp, int kp_cap, int nframes);
void launch_oa_finalize(hipStream_t st, const uint8_t* pyr, const uint8_t* blur, size_t pyr_stride,
                        const LevelDesc* lv, const uint8_t* cpyr, size_t cp_stride, const OaImg* imgs,
                        const OaCell* cells, OaScales sc, const uint64_t* akp, int akp_stride, const int* nkp,
                        const uint16_t* depth, size_t depth_stride, int img_w, FrameCalib cal, orb_kp* kps,
                        uint8_t* desc, float* kun, float* xyz, float* ur, int kp_cap, int nframes);
void launch_adapt_select_dbg(hipStream_t st, uint32_t* a, int n, int nth, int mode, int* posL, int* posR,
                             int* n_out);

}  // namespace odo
