/*
 * odo.h — C-ABI of the MI355X-native per-frame odometry hot path
 * (ORB extraction + Hamming kNN matching + RANSAC-wrapped PnP), the drop-in
 * boundary for ttwang0303/Adaptive-RGBD-Localization-Mappig.
 *
 * Implemented by libodo_hip.so (hand-written HIP for gfx950). Plain pointers
 * and sizes only; every function returns an int status (ODO_OK = 0, < 0 on
 * error, message via odo_last_error()). The library never falls back to a CPU
 * implementation: without a usable gfx950 device odo_create() fails.
 *
 * Each entry point names the reference interface it replaces (file:line in
 * the reference tree). INTEGRATION.md shows the reference-side bindings.
 */
#ifndef ODO_H
#define ODO_H

#include <stddef.h>
#include <stdint.h>

#include "odo_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ODO_OK 0
#define ODO_ERR_ARG (-1)
#define ODO_ERR_DEVICE (-2)
#define ODO_ERR_CAPACITY (-3)
#define ODO_ERR_STATE (-4)

/* odo_config.detector: Extractor(detector, descriptor, mode) (extractor.cpp:14) */
#define ODO_DETECTOR_ORB_SLAM2 0      /* ORB_SLAM2 / ORB_SLAM2 / NORMAL (main.cpp:19-21, the reference default) */
#define ODO_DETECTOR_ADAPTIVE_FAST 1  /* FAST / ORB / ADAPTIVE: 3x3 grid-adapted FAST + cv::ORB descriptor */
#define ODO_DETECTOR_ADAPTIVE_ORB 2   /* ORB / ORB / ADAPTIVE: 3x3 grid-adapted cv::ORB detector (Harris,
                                         8 levels; detectoradjuster.cpp:29) + cv::ORB descriptor */

/* odo_config.forms: which of several bit-identical kernel forms runs (all
 * produce the same results; the parity tests run each). 0 everywhere = the
 * defaults. These are explicit per-context settings: the library reads no
 * environment variables (measurement knobs exist only in the separate
 * tuning build, make -C ... tuning). */
#define ODO_KNN_FORM_FP4 0   /* default: exact sign-vector products on the matrix cores (FP4 operands) */
#define ODO_KNN_FORM_VALU 1  /* xor + popcount on the VALUs (also taken for train sets above 8192) */
#define ODO_PYRAMID_FORM_AUTO 0   /* default: FUSED for batches of >= 128 frames, CHAIN below */
#define ODO_PYRAMID_FORM_CHAIN 1  /* k_gray + one k_resize launch per level, then the blur launch */
#define ODO_PYRAMID_FORM_FUSED_NOBLUR 2  /* one launch, a workgroup per frame builds every level;
                                            the blur as its own launch */
#define ODO_PYRAMID_FORM_FUSED 3  /* one launch: every level and its 7x7 blur (falls back to the
                                     chain / a separate blur launch where its host checks fail) */
typedef struct odo_kernel_forms {
    int32_t knn;                    /* ODO_KNN_FORM_* */
    int32_t knn_split;              /* VALU form: train splits per query block, 1..8 (0 = 2) */
    int32_t ransac_lanes_min_open;  /* open pairs from which the second RANSAC launch takes the
                                       lane-per-hypothesis kernel (0 = 32) */
    int32_t pyramid;                /* ODO_PYRAMID_FORM_*: gray + pyramid levels */
    int32_t ransac_first_hyps;      /* batched path: hypotheses per pair in the first RANSAC
                                       evaluation launch, 1..64 (0 = 2) */
} odo_kernel_forms;

/* Layout version of the structs below. odo_config starts with its own size,
 * which odo_default_config fills and odo_create checks, so a caller built
 * against a header with a different odo_config fails with ODO_ERR_ARG instead
 * of reading past its struct. */
#define ODO_ABI_VERSION 5
int odo_abi_version(void);  /* ODO_ABI_VERSION of the library */

typedef struct odo_config {
    uint32_t struct_size;       /* sizeof(odo_config): set by odo_default_config */
    int32_t width, height;      /* frame size (all frames of a context share it) */
    int32_t max_batch;          /* frames per odo_track_batch() call */
    odo_orb_params orb;         /* ORBextractor(nFeatures,1.2,8,20,7) extractor.cpp:86 */
    odo_calib calib;            /* Utils/common.h Calibration */
    float nn_ratio;             /* Matcher(0.9f) tracking.cpp:197 */
    odo_ransac_params ransac;   /* Ransac(200,20,3.0,4) odometry.cpp:28 */
    uint32_t seed;              /* per-pair RNG seed base (replaces srand(clock()), main.cpp:27) */
    int32_t detector;           /* ODO_DETECTOR_* */
    odo_adaptive_params adaptive; /* ADAPTIVE grid (Extractor::CreateAdaptiveDetector, extractor.cpp:55-77) */
    odo_kernel_forms forms;     /* bit-identical kernel alternatives (tests / A-B); zero = defaults */
} odo_config;

typedef struct odo_ctx odo_ctx;

/* Fill cfg with the reference's defaults (FR1 calibration, nfeatures=1000)
 * and its struct_size. */
void odo_default_config(odo_config* cfg, int width, int height, int max_batch);

/* Context: owns the HIP stream, HBM scratch and the cross-frame state the
 * reference keeps in globals or detector objects (previous frame,
 * DepthCovariance latch, the ADAPTIVE grid's per-cell FAST thresholds). */
odo_ctx* odo_create(const odo_config* cfg, int device);
void odo_destroy(odo_ctx* ctx);
const char* odo_last_error(void);
void* odo_stream(odo_ctx* ctx);               /* hipStream_t, for callers that share streams */
int odo_reset(odo_ctx* ctx);                  /* forget previous frame, latch, adaptive thresholds */
int odo_set_latch(odo_ctx* ctx, double cov);  /* NaN = unlatched */
double odo_get_latch(odo_ctx* ctx);

/* ---- Batched hot path: Tracking::Track for n frames (tracking.cpp:38-78 minus
 * map bookkeeping): Frame::Frame + ExtractFeatures (frame.cpp:18,135), then for
 * every frame t with a predecessor: UpdateLastFrame VO landmarks
 * (tracking.cpp:136), Matcher::KnnMatch (matcher.cpp:55), Odometry::Compute
 * ADAPTIVE_RBA = Ransac::Iterate + PnPSolver::Compute (odometry.cpp:105-116),
 * with F1 pose = identity (DESIGN.md §3 batched contract).
 * d_bgr: device [n][H][W][3] u8, d_depth: device [n][H][W] u16 (x5000).
 * results[n] (host): results[i] is the pair (frame i-1 -> frame i); frame -1
 * is the last frame of the previous call. When h_results is NULL the call is
 * asynchronous: the work runs on the library's streams (extraction =
 * odo_stream(), plus pair / PnP / side streams), d_bgr is read by the
 * extraction stream and d_depth by the batch's pair stream (the keypoint
 * geometry), and odo_synchronize() waits for all of them. */
int odo_track_batch(odo_ctx* ctx, const uint8_t* d_bgr, const uint16_t* d_depth, int n,
                    odo_pair_result* h_results);
/* Same with host inputs, as Tracking::Track receives them (main.cpp:93-102).
 * The H2D upload runs on the context's copy stream into one of two device
 * staging buffers and overlaps the compute of the batches already queued; the
 * call returns once the host buffers have been consumed (the caller may refill
 * them) and the batch is queued. Pinned buffers (odo_host_alloc) are read by
 * the DMA engines directly; pageable ones are staged by the HIP runtime. With
 * h_results non-null it waits for the batch and fills the results. */
int odo_track_batch_host(odo_ctx* ctx, const uint8_t* bgr, const uint16_t* depth, int n,
                         odo_pair_result* h_results);
/* odo_track_batch_host with the depth frames read in place: depth must be
 * page-locked host memory from odo_host_alloc (else ODO_ERR_ARG). Only the BGR
 * frames are uploaded; the keypoint geometry kernel reads each keypoint's depth
 * pixel through the mapped pointer, so about 2000 small reads per frame cross
 * PCIe instead of the 614 kB depth image. The BGR buffer is consumed when the
 * call returns; the DEPTH buffer must stay valid and unchanged until the batch
 * has read it: odo_host_depth_query() returns 0 / odo_host_depth_wait() returns
 * (or odo_synchronize(), or the call itself when h_results is set). */
int odo_track_batch_host_sparse_depth(odo_ctx* ctx, const uint8_t* bgr, const uint16_t* depth, int n,
                                      odo_pair_result* h_results);
/* Whether the last odo_track_batch_host_sparse_depth batch may still read its
 * depth buffer: 1 = in use (do not refill it), 0 = released (< 0 on error).
 * odo_host_depth_wait blocks until it is released (odo_synchronize too). */
int odo_host_depth_query(odo_ctx* ctx);
int odo_host_depth_wait(odo_ctx* ctx);
/* odo_track_batch_host with the result records streamed to PAGE-LOCKED host
 * memory as odo_track_batch_async does (no host sync for the results; the host
 * input buffers are consumed when the call returns): the from-host form of the
 * SURVEY §8(e) frames mode, one PCIe upload per rank. */
int odo_track_batch_host_async(odo_ctx* ctx, const uint8_t* bgr, const uint16_t* depth, int n,
                               odo_pair_result* h_results);
/* odo_track_batch with the n result records copied into PAGE-LOCKED host memory
 * (odo_host_alloc) asynchronously after the batch's PnP: no host sync, the
 * records are valid after odo_synchronize(). Used to stream results. */
int odo_track_batch_async(odo_ctx* ctx, const uint8_t* d_bgr, const uint16_t* d_depth, int n,
                          odo_pair_result* h_results);
/* Sequence position (SURVEY §8(e) frames mode, replaces the implicit global
 * frame counter of Tracking): the next batch's pair p uses global pair index
 * pair_index + p for its RANSAC seed; keep_prev = 0 makes the next batch's
 * first frame a segment start (a rank's halo frame: extracted, no pair with
 * the previous call). The DepthCovariance latch and ADAPTIVE thresholds stay. */
int odo_seek(odo_ctx* ctx, uint64_t pair_index, int keep_prev);
/* Page-locked host memory for input frames (decode straight into it so the
 * upload needs no extra host copy). NULL on failure; free with odo_host_free. */
void* odo_host_alloc(size_t bytes);
int odo_host_free(void* p);
/* Extraction only (frames land in the batch slots; no pairs). Device inputs. */
int odo_extract_batch(odo_ctx* ctx, const uint8_t* d_bgr, const uint16_t* d_depth, int n);
int odo_synchronize(odo_ctx* ctx);

/* Read back frame features of batch slot i (0 <= i < n of the last call). */
int odo_get_frame(odo_ctx* ctx, int i, orb_kp* kps, uint8_t* desc, float* kps_un, float* xyz,
                  float* u_right, int cap, int* n);
/* Read back pair i's matches (KnnMatch output), RANSAC inlier mask over the
 * sorted good matches, and PnP inlier mask over frame-i keypoints. */
int odo_get_pair(odo_ctx* ctx, int i, odo_dmatch* matches, int match_cap, int* n_matches,
                 odo_dmatch* good_sorted, int* n_good, uint8_t* ransac_inliers /* n_good */,
                 uint8_t* pnp_inliers /* frame kps */, int32_t* f2_src);

/* ---- Per-stage entry points (host buffers, synchronous) ---- */

/* Extractor::Extract + Frame::ExtractFeatures (extractor.cpp:39, frame.cpp:135):
 * BGR8 (or gray when channels==1) + optional depth16 -> keypoints,
 * 32-byte descriptors, undistorted points, camera xyz and right coordinate.
 * With ODO_DETECTOR_ADAPTIVE_FAST / _ORB every call advances the cell thresholds. */
int odo_extract(odo_ctx* ctx, const uint8_t* img, int channels, const uint16_t* depth,
                orb_kp* kps, uint8_t* desc, float* kps_un, float* xyz, float* u_right, int cap,
                int* n);

/* cv::BFMatcher(NORM_HAMMING).knnMatch(k=2) as used by Matcher::KnnMatch
 * (matcher.cpp:60). idx/dist: nq x 2 (trainIdx -1 / INT_MAX when absent). */
int odo_knn2_hamming(odo_ctx* ctx, const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx,
                     int32_t* dist);

/* Ransac::Iterate(Frame*,Frame*,m12) (ransac.cpp:155). xyz1/xyz2: mvKeys3Dc of
 * both frames (n1/n2 points). rng: in/out glibc rand() state; latch: in/out
 * DepthCovariance static (NaN = unlatched). inliers: capacity n12. Returns the
 * bool result (1/0) in *ok. */
int odo_ransac(odo_ctx* ctx, const odo_dmatch* m12, int n12, const float* xyz1, int n1,
               const float* xyz2, int n2, const odo_ransac_params* p, odo_rng* rng, double* latch,
               float T12[16], float* rmse, odo_dmatch* inliers, int* n_inliers, int* ok);

/* ---- Hypotheses mode of Ransac::Iterate: the
 * hypotheses of one pair are sharded over ranks; each rank evaluates
 * [h0, h1) from the same rand() stream, the per-hypothesis summaries are
 * all-gathered (16..64 B each), every rank replays the ordered fold, and the
 * rank that owns the winner supplies T12 and the inlier list.
 * 1) odo_ransac_hyps: same inputs as odo_ransac (rng and latch are read, the
 *    latch is set if unlatched, rng is NOT advanced); writes summaries of
 *    [h0, h1) to out[0 .. h1-h0) and keeps the range's inlier masks in ctx. */
int odo_ransac_hyps(odo_ctx* ctx, const odo_dmatch* m12, int n12, const float* xyz1, int n1,
                    const float* xyz2, int n2, const odo_ransac_params* p, const odo_rng* rng,
                    double* latch, int h0, int h1, odo_hyp_summary* out, int* n_good);
/* 2) the ordered fold over all H = p->iterations summaries (host only, no
 *    device needed): identical on every rank. */
int odo_ransac_fold(const odo_hyp_summary* all, int H, int n_good, const odo_ransac_params* p,
                    odo_ransac_fold_result* r);
/* 3) outputs of the folded run from the last odo_ransac_hyps of this ctx:
 *    rng advanced by exactly the visited draws (every rank); T12, rmse,
 *    inliers and ok are valid when *owner = 1 (best_h in this rank's range,
 *    or no valid hypothesis: identity fallback), otherwise they come from the
 *    owner rank (broadcast). */
int odo_ransac_hyps_finish(odo_ctx* ctx, const odo_ransac_fold_result* r, odo_rng* rng, float T12[16],
                           float* rmse, odo_dmatch* inliers, int* n_inliers, int* ok, int* owner);

/* ---- The same hypotheses mode with the exchange in device memory (RCCL
 * collectives on device buffers, no host staging; ransac.cpp:233-249 is the
 * ordered fold it feeds). All work is queued on odo_stream(ctx); a caller
 * orders its collectives after it on that stream.
 * 1) odo_ransac_hyps_dev: as odo_ransac_hyps, the summaries of [h0, h1) into
 *    the DEVICE buffer d_block ((h1-h0) x 64 B, odo_hyp_summary layout); no
 *    host synchronisation. The gathered array must hold all H summaries in
 *    hypothesis order (contiguous rank ranges). When the pair never samples
 *    (Iterate returns before its loop: too few matches) the default summaries
 *    are copied on odo_stream(ctx) and this call synchronises that stream
 *    before it returns (step 4 does the same for its payload). */
int odo_ransac_hyps_dev(odo_ctx* ctx, const odo_dmatch* m12, int n12, const float* xyz1, int n1,
                        const float* xyz2, int n2, const odo_ransac_params* p, const odo_rng* rng,
                        double* latch, int h0, int h1, void* d_block, int* n_good);
/* 2) the ordered fold over the gathered device array d_all (H summaries) on
 *    the GPU; the odo_ransac_fold_result record is written to device memory
 *    d_fold (same values as odo_ransac_fold). */
int odo_ransac_fold_dev(odo_ctx* ctx, const void* d_all, int H, void* d_fold);
/* 3) size in int32 words of the payload buffer of step 4 (32 header words +
 *    4 per good match). */
int odo_ransac_hyps_payload_words(odo_ctx* ctx);
/* 4) the folded run's outputs: this rank's rand() state advanced on the
 *    device by exactly the visited draws; the owner of the winner (its range
 *    holds best_h; rank 0 when rank0 != 0 for the identity fallback or a pair
 *    that never sampled) writes the payload [T12 bits x16, rmse bits, ok,
 *    n_inliers, visited, 12 x 0, inliers as odo_dmatch...] to d_payload and
 *    every other rank writes zeros, so an int32 SUM all-reduce over the ranks
 *    leaves the owner's payload everywhere. */
int odo_ransac_hyps_finish_dev(odo_ctx* ctx, const void* d_fold, int rank0, void* d_payload, int payload_words);
/* 5) synchronise and unpack a (reduced) payload and this rank's rand() state. */
int odo_ransac_hyps_result(odo_ctx* ctx, const void* d_payload, odo_rng* rng, float T12[16], float* rmse,
                           odo_dmatch* inliers, int* n_inliers, int* ok, int* visited);

/* PnPSolver::Compute (pnpsolver.cpp:17): Xw n x 3 (world), obs n x 3 (u,v,uR;
 * uR<0 = mono edge). outlier: out, per edge. Returns inliers in *n_inliers. */
int odo_pnp_motion_ba(odo_ctx* ctx, const float* Xw, const float* obs, int n, const odo_calib* calib,
                      const float Tcw_init[16], float Tcw_out[16], uint8_t* outlier, int* n_inliers);

/* PnPRansac::Compute (pnpransac.cpp:11-51), the RANSAC
 * PnP back-end: cv::solvePnPRansac(v3D, v2D, mK, noDist, r, t, false,
 * iterations = 500, reproj_err = 3.0f, confidence = 0.85, inliers) over the
 * frame's landmark observations. Xw: n x 3 world points (Landmark::GetWorldPos),
 * uv: n x 2 undistorted keypoints (mvKeysUn), in index order. n < 10 returns
 * res->ok = 0 without running (pnpransac.cpp:30); no model with more than 4
 * inliers gives ok = 0; a best model with exactly 5 non-planar inliers gives
 * ok = ODO_PNP_RANSAC_THROW (-1: OpenCV's final solvePnP asserts count >= 6
 * in its DLT start and throws; Tcw and rvec/tvec are then zero, the model,
 * mask and n_inliers are set). Test ok == 1 for success, never truthiness. inlier_mask (n, optional):
 * the RANSAC inliers (Frame::SetInlier); good_counts (iterations, optional):
 * inliers of every hypothesis, of which the first res->iterations_visited are
 * the ones RANSAC visited. Hypotheses, EPnP, counts, the ordered fold and the
 * Levenberg-Marquardt refinement all run on the GPU (k_pnpransac.hip). */
#define ODO_PNP_RANSAC_THROW (-1)
int odo_pnp_ransac(odo_ctx* ctx, const float* Xw, const float* uv, int n, const odo_calib* calib, int iterations,
                   float reproj_err, double confidence, odo_pnp_ransac_result* res, uint8_t* inlier_mask,
                   int32_t* good_counts);

/* PnPRansac::Compute for a batch of frames in one launch chain (the batched
 * contract of odo_track_batch): problem p = observations [offs[p], offs[p+1])
 * of Xw / uv (offs[0] = 0, nprob + 1 entries); res[p] as odo_pnp_ransac
 * (problems with fewer than 10 observations: ok = 0, best_iter = -1);
 * inlier_mask (optional) over all offs[nprob] observations. */
int odo_pnp_ransac_batch(odo_ctx* ctx, const float* Xw, const float* uv, const int32_t* offs, int nprob,
                         const odo_calib* calib, int iterations, float reproj_err, double confidence,
                         odo_pnp_ransac_result* res, uint8_t* inlier_mask);

/* GeneralizedICP(max_iterations, max_corr_dist)::Compute(source, target, guess)
 * (generalizedicp.cpp:11-22, 30-39, 65-89): the PCL
 * GICP refinement Odometry::Compute's ADAPTIVE_RICP mode runs on RANSAC's
 * matched clouds (odometry.cpp:46-78; the reference builds it with 10
 * iterations and 0.07 m). src/tgt: n x 3 (Ransac::mpSourceCloud /
 * mpTargetCloud). Fewer than 20 points in either cloud: *converged = 0 without
 * running (generalizedicp.cpp:33). T12 = the final transformation when
 * converged, identity otherwise (generalizedicp.cpp:76-88); iterations = ICP
 * iterations run, n_corr = correspondences of the last one. Covariances,
 * correspondences and the BFGS all run on the GPU (k_gicp.hip); neighbour
 * searches are brute force, so clouds hold at most 16384 points
 * (ODO_ERR_CAPACITY; RANSAC's matched clouds are a few hundred). */
int odo_gicp(odo_ctx* ctx, const float* src, int ns, const float* tgt, int nt, const float guess[16],
             int max_iterations, double max_corr_dist, float T12[16], int* converged, int* iterations, int* n_corr);

/* GeneralizedICP::Compute for a batch of pairs in one launch chain: pair p =
 * source points [soffs[p], soffs[p+1]) of src, target points [toffs[p],
 * toffs[p+1]) of tgt (offsets start at 0, nprob + 1 entries), guesses 16 per
 * pair (NULL: identity); T12 16 per pair, converged / iterations / n_corr one
 * per pair, as odo_gicp. */
int odo_gicp_batch(odo_ctx* ctx, const float* src, const int32_t* soffs, const float* tgt, const int32_t* toffs,
                   const float* guesses, int nprob, int max_iterations, double max_corr_dist, float* T12,
                   int32_t* converged, int32_t* iterations, int32_t* n_corr);

/* ---- Trajectory (host only) ----
 * Relative-pose chain of the batched contract: results[i].Tcw is frame i's
 * pose in frame i-1's camera coordinates, so Tcw(i) = Tcw_rel(i) * Tcw(i-1)
 * (Odometry::Compute's Tcw2 = T12 * Tcw1, odometry.cpp:110-112), starting
 * from Tcw_prev (the last pose of the previous batch; identity for a new
 * sequence). Pairs without a predecessor (n_matches == 0 at i == 0 of a
 * sequence) keep Tcw_prev. 4x4 row-major floats; products in double. */
int odo_chain_poses(const odo_pair_result* results, int n, const float Tcw_prev[16], float* Tcw_out);
/* Tracking::SaveTrajectory's line format (tracking.cpp:544-582): "timestamp
 * tx ty tz qx qy qz qw" of the camera centre twc = -Rcw^T tcw and
 * Converter::toQuaternion(Rwc) (Eigen Quaterniond from the double matrix,
 * converter.cpp:149-161), std::fixed with 6 / 9 decimals. append: 0 = new
 * file. */
int odo_write_tum_trajectory(const char* path, const double* timestamps, const float* Tcw, int n, int append);

/* Frame::ComputeImageBounds (frame.cpp:315-349) for the context's calibration
 * and image size: undistorted corners -> minX, maxX, minY, maxY. Host only. */
int odo_image_bounds(odo_ctx* ctx, float bounds[4]);

/* Tracking::SearchLocalLMs (tracking.cpp:368-405): Frame::isInFrustum
 * (frame.cpp:100-133) for every landmark neither ODO_LM_BAD nor ODO_LM_SEEN,
 * then Matcher(nn_ratio)::ProjectionMatch(frame, landmarks, th)
 * (matcher.cpp:90-145; the reference passes 0.8f and 8.0f). Frame: n
 * undistorted keypoints (mvKeysUn), their octaves and descriptors;
 * slot_taken[j] = slot j holds a landmark with Observations() > 0. Outputs:
 * slot_lm[j] = index of the landmark AddLandmark put in slot j, or -1;
 * proj[3*i..] = (mTrackProjX, mTrackProjY, mTrackProjXR) of in-view
 * landmarks, NaN otherwise; *n_matches = ProjectionMatch's return. Then
 * TrackLocalMap's second PnPSolver::Compute is odo_pnp_motion_ba over every
 * slot holding a landmark. */
int odo_projection_match(odo_ctx* ctx, const float Tcw[16], const odo_landmark* lms, int n_lms,
                         const float* kps_un, const int32_t* octave, const uint8_t* desc, int n,
                         const uint8_t* slot_taken, float th, float nn_ratio, int32_t* slot_lm, float* proj,
                         int* n_matches);

/* Kabsch::Compute (kabsch.cpp:14): one GPU workgroup (k_kabsch: centroids, A^T B
 * with a fixed-order block reduction, 3x3 Jacobi SVD). A,B: n x 3 host arrays. */
int odo_kabsch(const float* A, const float* B, int n, float T[16]);

/* glibc rand() stream helpers (srand/rand of main.cpp:27, ransac.cpp:275). */
void odo_rng_seed(odo_rng* r, uint32_t seed);
int32_t odo_rng_next(odo_rng* r);

/* ---- Introspection for parity tests ---- */
int odo_debug_pyramid(odo_ctx* ctx, int i, uint8_t* out, size_t cap);
int odo_debug_fast(odo_ctx* ctx, int i, int level, orb_kp* out, int cap, int* n);
int odo_debug_octree(odo_ctx* ctx, int i, int level, orb_kp* out, int cap, int* n);
int odo_debug_blur(odo_ctx* ctx, int i, uint8_t* out, size_t cap);
/* std::sort(vGoodMatches) of Ransac::Iterate (ransac.cpp:199) as the pair
 * stage runs it on the GPU (workgroup-parallel introsort): in -> out sorted by
 * distance in libstdc++'s exact (unstable) order; distances must be >= 0. */
int odo_debug_sort(odo_ctx* ctx, const odo_dmatch* in, int n, odo_dmatch* out);

/* Measurement only (no reference counterpart): re-runs the most recent
 * batch's kNN-2 launch `reps` times on an idle device and returns its mean
 * duration in ms (HIP events). The bench's roofline "alone" figure. */
int odo_knn_replay_time(odo_ctx* ctx, int reps, float* avg_ms);
/* ADAPTIVE detector state. The per-cell DetectorAdjuster thresholds persist
 * across frames and calls (detectoradjuster.cpp:52-65, App. B.13); they
 * advance with every extracted frame, in frame order within a batch.
 * odo_debug_adaptive: FAST threshold each cell used for frame i of the last
 * batch (t_used, grid cells; NULL skips) and the current thresholds (thresh;
 * NULL skips). Returns the number of grid cells (< 0 on error). */
int odo_debug_adaptive(odo_ctx* ctx, int i, int32_t* t_used, double* thresh);
int odo_set_adaptive_thresholds(odo_ctx* ctx, const double* thresh, int n);
/* std::nth_element(a, a + nth, a + n) by score (mode 0; keepStrongest,
 * videogridadaptedfeaturedetector.cpp:24-31) or KeyPointsFilter::retainBest
 * (mode 1) exactly as the ADAPTIVE stages run them on the GPU, over packed
 * keys (score << 24 | y << 12 | x). out: n keys, *n_out kept. */
int odo_debug_select(odo_ctx* ctx, const uint32_t* in, int n, int nth, int mode, uint32_t* out, int* n_out);
/* Timing (off by default; mode 0). Mode 1: odo_track_batch records HIP events
 * between stages and odo_last_timings reports the last batch (ms); these
 * events serialise the streams they sit on. Mode 2: an event pair brackets the
 * Hamming-match (kNN-2) launch of every batch on the extraction stream, and
 * odo_kernel_timing reports the mean launch duration since the mode was set. */
int odo_set_timing(odo_ctx* ctx, int mode);
int odo_kernel_timing(odo_ctx* ctx, double* avg_ms, long* launches);
/* Measurement only (mode 2): the start of every batch's kNN-2 launch since the
 * mode was set, in ms after odo_set_timing, batch order. A batch's kNN-2 starts
 * when its extraction has finished, so consecutive differences are the
 * pipeline's per-step times. Copies up to cap marks; returns how many exist. */
int odo_step_marks(odo_ctx* ctx, double* ms, int cap);
/* Per-stage device time of the last odo_track_batch (ms), via HIP events. */
int odo_last_timings(odo_ctx* ctx, float* ms, int cap, const char** names);

#ifdef __cplusplus
}
#endif

#endif /* ODO_H */
