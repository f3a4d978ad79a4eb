// Internal (non-ABI) structures shared by the HIP kernels and the host
// orchestration in odo_capi.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/odo_types.h"

namespace odo {

#define FAST_ROI_MAX 48

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

// RANSAC per-pair constants.
struct RansacCfg {
    int iterations;
    int min_inlier_th;
    float max_mahal;
    int sample_size;
    int check_depth;
    double raster_cov_x, raster_cov_y;
};

// ---- launch wrappers (defined next to their kernels)
void upload_extract_constants();
void launch_gray(hipStream_t st, const uint8_t* bgr, uint8_t* pyr, int w, int h, int pitch, size_t in_stride,
                 size_t pyr_stride, int nframes);
size_t resize_lds_bytes(int spitch, int dw, int max_src_rows);
void launch_resize(hipStream_t st, uint8_t* pyr, size_t pyr_stride, int src_off, int spitch, int dst_off, int dpitch,
                   int dw, int dh, int rb, int max_src_rows, const ResizeX* xt, const ResizeY* yt, int nframes);
void launch_fast(hipStream_t st, const uint8_t* pyr, size_t pyr_stride, const CellDesc* cells, const LevelDesc* lv,
                 uint32_t* cand, int* cand_cnt, int ncells, int cell_cap, int ini_th, int min_th, int nframes);
size_t octree_lds_bytes(int node_cap);
void launch_octree(hipStream_t st, const uint32_t* cand, const int* cand_cnt, const LevelDesc* lv, int ncells,
                   int cell_cap, int nlevels, uint32_t* keys, int32_t* knode, uint8_t* kquad, size_t keys_stride,
                   uint32_t* okp, int* ocnt, int okp_stride, int node_cap, int nframes);
void launch_blur(hipStream_t st, const uint8_t* pyr, uint8_t* blur, size_t pyr_stride, const LevelDesc* lv,
                 const LevelDesc* lv_host, int nlevels, int nframes);
void launch_finalize(hipStream_t st, const uint8_t* pyr, const uint8_t* blur, size_t pyr_stride, const LevelDesc* lv,
                     int nlevels, const uint32_t* okp, const int* ocnt, int okp_stride, const uint16_t* depth,
                     size_t depth_stride, int img_w, FrameCalib cal, orb_kp* kps, uint8_t* desc, float* kun, float* xyz,
                     float* ur, int* nkp, int kp_cap, int nframes);
void launch_pair_valid(hipStream_t st, int* pv, int n, int first_valid);
void launch_copy_frame(hipStream_t st, const orb_kp* kps_s, const uint8_t* desc_s, const float* kun_s,
                       const float* xyz_s, const float* ur_s, const int* n_s, orb_kp* kps_d, uint8_t* desc_d,
                       float* kun_d, float* xyz_d, float* ur_d, int* n_d, int kp_cap);
void launch_knn2(hipStream_t st, const uint8_t* q, const int* qn, size_t q_stride, const uint8_t* t, const int* tn,
                 size_t t_stride, int2* idx, int2* dist, size_t out_stride, int max_q, int npairs);
void launch_pair_match(hipStream_t st, const int2* knn_idx, const int2* knn_dist, size_t knn_stride, const float* xyz,
                       const int* nkp, int kp_cap, int slot0, float ratio, float th_depth_m, int check_depth,
                       odo_dmatch* matches, int* n_matches, void* good, int* n_good, int32_t* f2_src,
                       uint64_t* sort_scratch, int match_cap, int npairs);
int launch_sort_dbg(hipStream_t st, void* a, int n);
void launch_latch(hipStream_t st, double* latch, const void* good, const int* n_good, const int* n_matches,
                  const odo_dmatch* matches, const float* xyz, int kp_cap, int slot0, int npairs, int match_cap,
                  int min_inl, int sample_size, int iterations, const int* pair_valid);
size_t ransac_gpt_bytes();
// rand() words for every pair (data independent): launched at batch start on
// a side stream; launch_ransac's stream must wait for it.
void launch_ransac_raw(hipStream_t st, void* scratch, int npairs, int match_cap, int mask_words, RansacCfg cfg,
                       uint64_t seed_base, uint64_t pair_base, odo_rng* rng_io);
void launch_ransac(hipStream_t st, const void* good, const int* n_good, const int* n_matches,
                   const odo_dmatch* matches, const float* xyz, int kp_cap, int slot0, int match_cap, RansacCfg cfg,
                   const double* latch, const int* pair_valid, int min_matches, odo_rng* rng_io, void* scratch,
                   uint32_t* best_mask, int mask_words, odo_pair_result* res, float* T12, int npairs, int part = 0,
                   int* phase = nullptr);
size_t ransac_scratch_bytes(int npairs, int match_cap, int mask_words, const RansacCfg& cfg);
size_t pnp_edge_bytes();
void launch_pnp(hipStream_t st, const int32_t* f2_src, const float* xyz, const float* kun, const float* ur,
                const int* nkp, int kp_cap, int slot0, FrameCalib cal, const float* T12, const int* pair_valid,
                const int* n_matches, int min_matches, void* edges, odo_pair_result* res, uint8_t* inlier_mask,
                int npairs, const int* sel = nullptr, int sel_val = 0);
void launch_kabsch(hipStream_t st, const float* A, const float* B, int n, float* T);

}  // namespace odo
