/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A single-threaded C++ CPU restatement of the reference's per-frame
 * odometry hot path (ttwang0303/Adaptive-RGBD-Localization-Mappig), used as
 * the checker for the HIP product path and as the `cpu_baseline` leg of
 * bench.py. Nothing in the product (adaptive-rgbd-localization-mappig_amd/)
 * links, loads or calls this code; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may.
 *
 * Parity status: PARTIALLY PINNED. The reference needs OpenCV/PCL/Eigen/g2o,
 * none of which exist in this image, so it cannot be built here and ships no
 * golden vectors. This restatement follows the reference
 * files cited per function plus the third-party semantics fixed in SURVEY.md
 * Appendix A. Pinned against the real thing: glibc rand() stream (the real
 * libc is called), libstdc++ std::sort / std::nth_element / std::list (the
 * same library algorithms are used), IEEE arithmetic. Unpinned: OpenCV /
 * Eigen / PCL / g2o internals (restated from App. A).
 *
 * Every entry point is extern "C" so tests can drive it through ctypes.
 */
#ifndef ODO_ORACLE_H
#define ODO_ORACLE_H

#include <stddef.h>
#include <stdint.h>
#include "../include/odo_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* A.1 cvtColor(BGR2GRAY) + A.1b depth convertTo (frame.cpp:23-24). */
void oracle_bgr2gray(const uint8_t* bgr, int w, int h, int stride, uint8_t* gray);
void oracle_depth_to_f32(const uint16_t* d, int n, float factor, float* z);

/* ORBextractor tables (orbextractor.cpp:346-404). */
int oracle_level_sizes(const odo_orb_params* p, int w, int h, int* lw, int* lh,
                       float* scale, int* quota);
int oracle_umax(int* umax16);

/* ComputePyramid (orbextractor.cpp:833-857): levels written back to back. */
int oracle_pyramid(const uint8_t* gray, int w, int h, const odo_orb_params* p, uint8_t* out);

/* FAST part of ComputeKeyPointsOctTree (orbextractor.cpp:669-723) for one
 * level: candidates in vToDistributeKeys order (relative to the 16px border). */
int oracle_fast_level(const uint8_t* img, int w, int h, int ini_th, int min_th,
                      orb_kp* out, int cap);

/* DistributeOctTree (orbextractor.cpp:466-663). */
int oracle_octree(const orb_kp* keys, int n, int minX, int maxX, int minY, int maxY,
                  int N, orb_kp* out, int cap);

/* GaussianBlur 7x7 sigma 2 REFLECT_101 fixed point (App. A.4). */
void oracle_blur(const uint8_t* img, int w, int h, uint8_t* out);

/* fastAtan2 (App. A.5). */
float oracle_fast_atan2(float y, float x);

/* ORBextractor::operator() (orbextractor.cpp:756-815): returns N. */
int oracle_orb_extract(const uint8_t* gray, int w, int h, const odo_orb_params* p,
                       orb_kp* kps, uint8_t* desc, int cap);

/* ---- Extractor(FAST, ORB, ADAPTIVE) (extractor.cpp:14-77, a10). thresh:
 * in/out per-cell DetectorAdjuster thresholds (grid_rows*grid_cols doubles,
 * start at init_thresh); t_used (optional): FAST threshold of each cell's last
 * detect call. */
void oracle_adaptive_default(odo_adaptive_params* p);
/* VideoGridAdaptedFeatureDetector::detect (before retainBest). Returns N. */
int oracle_adaptive_detect(const uint8_t* gray, int w, int h, const odo_adaptive_params* p,
                           double* thresh, orb_kp* out, int cap, int* t_used);
/* cv::FAST(roi, thr, nonmax) on an ROI given by pointer/stride/size. */
int oracle_fast_roi(const uint8_t* gray, int stride, int rows, int cols, int threshold,
                    orb_kp* out, int cap);
/* Extractor::Extract: detect + retainBest(nFeatures) + cv::ORB::compute. */
int oracle_adaptive_extract(const uint8_t* gray, int w, int h, const odo_adaptive_params* p,
                            double* thresh, orb_kp* kps, uint8_t* desc, int cap, int* t_used);
/* libstdc++ std::nth_element / retainBest on packed (score<<24|y<<12|x). */
void oracle_nth_element_score(uint32_t* a, int n, int nth);
int oracle_retain_best_score(uint32_t* a, int n, int n_points);
/* Full Frame construction in ADAPTIVE mode. Returns N. */
int oracle_extract_frame_adaptive(const uint8_t* bgr, const uint16_t* depth, int w, int h,
                                  const odo_adaptive_params* p, double* thresh, const odo_calib* c,
                                  orb_kp* kps, uint8_t* desc, float* kps_un, float* xyz,
                                  float* u_right, int cap);

/* ---- Extractor(ORB, ORB, ADAPTIVE): the same grid / threshold chain with
 * the cv::ORB inner detector of detectoradjuster.cpp:29 (SURVEY §8(f) rank 2;
 * OpenCV 3.4 orb.cpp restated). */
int oracle_adaptive_orb_extract(const uint8_t* gray, int w, int h, const odo_adaptive_params* p,
                                double* thresh, orb_kp* kps, uint8_t* desc, int cap, int* t_used);
int oracle_adaptive_orb_detect(const uint8_t* gray, int w, int h, const odo_adaptive_params* p,
                               double* thresh, orb_kp* out, int cap, int* t_used);
/* cv::ORB(10000, 1.2, 8, 15, 0, 2, HARRIS, 31, threshold)::detect on one image. */
int oracle_orbcv_detect(const uint8_t* img, int stride, int rows, int cols, int threshold,
                        orb_kp* out, int cap);
/* HarrisResponses (blockSize 7, k 0.04) at (x, y) of a w x h image. */
float oracle_harris(const uint8_t* img, int w, int h, int x, int y);
/* cv::ORB pyramid sizes / getScale / nfeaturesPerLevel for nfeatures 10000. */
int oracle_orbcv_levels(int w, int h, int* lw, int* lh, float* scale, int* quota);
int oracle_extract_frame_adaptive_orb(const uint8_t* bgr, const uint16_t* depth, int w, int h,
                                      const odo_adaptive_params* p, double* thresh, const odo_calib* c,
                                      orb_kp* kps, uint8_t* desc, float* kps_un, float* xyz,
                                      float* u_right, int cap);

/* Frame::ExtractFeatures tail + UndistortKeyPoints (frame.cpp:139-169, 286-313). */
void oracle_frame_geometry(const orb_kp* kps, int n, const float* depth, int w, int h,
                           const odo_calib* c, float* kps_un, float* xyz, float* u_right);

/* Full Frame construction + extraction from BGR8 + depth16. Returns N. */
int oracle_extract_frame(const uint8_t* bgr, const uint16_t* depth, int w, int h,
                         const odo_orb_params* p, const odo_calib* c,
                         orb_kp* kps, uint8_t* desc, float* kps_un, float* xyz,
                         float* u_right, int cap);

/* Hypotheses mode: per-hypothesis summaries of visited iterations [h0, h1)
 * of Ransac::Iterate (no fold; rng_in is not advanced). Returns n_good. */
int oracle_ransac_hyps(const odo_dmatch* m12, int n12, const float* xyz1, const float* xyz2,
                       const odo_ransac_params* p, const odo_rng* rng_in, double* latch, int h0, int h1,
                       odo_hyp_summary* out);

/* Frame::ComputeImageBounds (frame.cpp:315-349): minX maxX minY maxY. */
void oracle_image_bounds(const odo_calib* c, int w, int h, float* bounds);
/* SearchLocalLMs' isInFrustum + Matcher(0.8)::ProjectionMatch (tracking.cpp:368-405,
 * matcher.cpp:90-145). Returns nmatches. */
int oracle_projection_match(const float* Tcw, const odo_landmark* lms, int nL, const float* kun,
                            const int32_t* octave, const uint8_t* desc, int n, const uint8_t* slot_taken,
                            const odo_calib* c, const float* bounds, float th, float nnratio,
                            int32_t* slot_lm, float* proj);

/* BFMatcher(NORM_HAMMING).knnMatch(k=2) (App. A.6). */
void oracle_knn2(const uint8_t* q, int nq, const uint8_t* t, int nt, int32_t* idx, int32_t* dist);

/* Matcher::KnnMatch(Frame&,Frame&) (matcher.cpp:55-88). f1_has_lm/f1_outlier:
 * per F1 keypoint; f2_lm_obs: per F2 slot, -1 = no landmark, else the
 * landmark's Observations(). On return f2_lm_src[i2] = F1 index whose landmark
 * now sits in F2 slot i2 (or -1), f2_outlier set per matcher.cpp:82. */
int oracle_knn_match(const uint8_t* d1, int n1, const uint8_t* d2, int n2, float ratio,
                     const uint8_t* f1_has_lm, const uint8_t* f1_outlier,
                     const int32_t* f1_lm_obs, int32_t* f2_lm_obs, int32_t* f2_lm_src,
                     uint8_t* f2_outlier, odo_dmatch* out, int cap);

/* Tracking::UpdateLastFrame VO-landmark rule (tracking.cpp:146-190) for a
 * frame with no prior landmarks: marks has_lm. Returns count. */
int oracle_vo_landmarks(const float* xyz, int n, float th_depth_m, uint8_t* has_lm);

/* glibc rand() stream (the real libc). */
void oracle_rng_seed(odo_rng* r, uint32_t seed);
int32_t oracle_rng_next(odo_rng* r);
void oracle_libc_rand_stream(uint32_t seed, int n, int32_t* out);

/* Ransac::Iterate(Frame*,Frame*,m12) (ransac.cpp:155-267). xyz1/xyz2:
 * mvKeys3Dc of both frames. inliers receives mvInliers (ransac.cpp:240, 258)
 * as DMatch copies in list order. latch: in/out DepthCovariance static
 * (NaN = not yet latched). */
void oracle_last_ransac_work(int* sweeps, int* fit_points);
int oracle_ransac(const odo_dmatch* m12, int n12, const float* xyz1, const float* xyz2,
                  const odo_ransac_params* p, odo_rng* rng, double* latch,
                  float* T12, float* rmse, odo_dmatch* inliers, int* n_inliers,
                  int* visited, int* n_good);

/* PCL TransformationFromCorrespondences + Eigen JacobiSVD<3x3f> (App. A.7/A.8). */
void oracle_tfc(const float* src, const float* tgt, const float* w, int n, float* T);
void oracle_svd3(const float* A, float* U, float* S, float* V);

/* PnPSolver::Compute (pnpsolver.cpp:17-214). Xw/obs: per F2 keypoint with a
 * landmark in index order; obs = (u,v,uR) with uR<0 => mono edge.
 * outlier: in/out per edge. Returns nInitial - nBad. */
int oracle_pnp(const float* Xw, const float* obs, int n, const odo_calib* c,
               const float* Tcw_init, float* Tcw_out, uint8_t* outlier);

/* ---- PnPRansac::Compute (pnpransac.cpp:11-51):
 * cv::solvePnPRansac(v3D, v2D, K, noDist, r, t, false, iterations, reproj_err,
 * confidence, inliers) of OpenCV 3.4 restated in pnpransac_ref.cpp. Xw n x 3,
 * uv n x 2 (mvKeysUn). model_out: best RANSAC model (rvec, tvec); rt_out: the
 * refined (rvec, tvec); Tcw: Converter::toHomogeneous(r, t); mask: RANSAC
 * inlier mask (n); good_counts (optional, >= iterations): inliers of every
 * visited hypothesis. Returns 1 (bOK), 0 when n < 10 or no model, -1 when
 * the refinement's cvFindExtrinsicCameraParams2 would throw (non-planar
 * inliers, only 5 of them: its DLT branch asserts count >= 6; model, mask and
 * n_inliers are set, rt_out and Tcw are zero). */
int oracle_pnp_ransac(const float* Xw, const float* uv, int n, const odo_calib* c, int iterations, float reproj_err,
                      double confidence, double model_out[6], double rt_out[6], float* Tcw, uint8_t* mask,
                      int* n_inliers, int* best_iter, int* niters_out, int* good_counts);
/* Pieces of it, for known-answer tests: cv::RNG(state).uniform(a, b) x n,
 * RANSACUpdateNumIters, cvRodrigues2 both ways (dRdr 3x9, optional), the EPnP
 * model of n points, the LM refinement from param (in/out). */
void oracle_cvrng_stream(uint64_t state, int a, int b, int n, int32_t* out);
int oracle_ransac_update_num_iters(double p, double ep, int model_points, int max_iters);
void oracle_rodrigues(const double r[3], double R[9], double* dRdr);
void oracle_rodrigues_inv(const double R[9], double r[3]);
void oracle_epnp(const double* pw, const double* uv, int n, const double K[4], double model[6]);
void oracle_pnp_refine(const double* M, const double* m, int n, const double K[4], double param[6]);
/* cvFindExtrinsicCameraParams2's start without an extrinsic guess (DLT /
 * homography; pnpransac.cpp:34 passes useExtrinsicGuess = false) */
int oracle_pnp_extrinsic_init(const double* M, const double* m, int n, const double K[4], double param[6]);

/* ---- GeneralizedICP::Compute(source, target, guess) (generalizedicp.cpp:30-39,
 * 65-89; SURVEY §8(f) rank 4, the ADAPTIVE_RICP fallback of odometry.cpp:46-78):
 * PCL 1.8 GICP restated in gicp_ref.cpp. src/tgt: n x 3. Returns 1 when
 * hasConverged (T12 = final transformation), 0 otherwise (T12 = identity,
 * generalizedicp.cpp:84-87). iterations: outer ICP iterations run; n_corr:
 * correspondences of the last one. */
int oracle_gicp(const float* src, int ns, const float* tgt, int nt, const float* guess, int max_iterations,
                double max_corr_dist, float* T12, int* converged, int* iterations, int* n_corr);
/* computeCovariances (k 20, epsilon 1e-3): n x 9 doubles. */
void oracle_gicp_covariances(const float* P, int n, double* C);

/* Kabsch::Compute (kabsch.cpp:14-57). */
void oracle_kabsch(const float* A, const float* B, int n, float* T);

/* One frame pair through the whole path (batched contract):
 * F1 pose = identity, F1 VO landmarks per UpdateLastFrame. matches and
 * ransac_inliers (Ransac::mvInliers, in list order; optional) hold up to cap
 * entries; n_ransac_inliers receives the list length. */
int oracle_track_pair(const orb_kp* k1, const uint8_t* d1, const float* xyz1, int n1,
                      const orb_kp* k2, const uint8_t* d2, const float* kun2,
                      const float* xyz2, const float* ur2, int n2,
                      const odo_calib* c, float ratio, const odo_ransac_params* rp,
                      uint32_t seed, double* latch, odo_pair_result* res,
                      uint8_t* inlier_mask /* n2 */, odo_dmatch* matches, int cap,
                      odo_dmatch* ransac_inliers, int* n_ransac_inliers);

#ifdef __cplusplus
}
#endif

#endif
