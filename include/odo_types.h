/*
 * odo_types.h — plain-old-data types crossing the C-ABI of the MI355X
 * odometry hot path. Layouts mirror the OpenCV / reference types they
 * replace so a caller can memcpy between them.
 *
 *   orb_kp      <-> cv::KeyPoint  {pt.x, pt.y, size, angle, response, octave, class_id}
 *                   (produced by ORBextractor::operator(), Features/orbextractor.cpp:756)
 *   odo_dmatch  <-> cv::DMatch    {queryIdx, trainIdx, imgIdx, distance}
 *                   (Matcher::KnnMatch, Features/matcher.cpp:55)
 *   odo_calib   <-> Calibration namespace constants, Utils/common.h:32-74
 */
#ifndef ODO_TYPES_H
#define ODO_TYPES_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orb_kp {
    float x, y;       /* pt (level-0 pixel coordinates after scaling, orbextractor.cpp:805-811) */
    float size;       /* PATCH_SIZE * scale, int-truncated (orbextractor.cpp:731) */
    float angle;      /* IC angle in degrees [0,360) (orbextractor.cpp:14-39) */
    float response;   /* FAST score (cornerScore<16>) */
    int32_t octave;   /* pyramid level */
    int32_t class_id; /* always -1 */
} orb_kp;

typedef struct odo_dmatch {
    int32_t queryIdx;
    int32_t trainIdx;
    int32_t imgIdx;
    float distance;
} odo_dmatch;

typedef struct odo_calib {
    float fx, fy, cx, cy;      /* common.h:35-38 (FR1 active) */
    float k1, k2, p1, p2, k3;  /* common.h:40-44; k1 == 0 disables undistortion (frame.cpp:288) */
    float depth_factor;        /* common.h:67, 1/5000 */
    float mbf;                 /* common.h:71, 40 */
    float th_depth;            /* common.h:72, 40 (mThDepth = mbf*thDepth/fx) */
} odo_calib;

typedef struct odo_orb_params {
    int32_t nfeatures;    /* ORBextractor(nFeatures=1000,...) extractor.cpp:86 */
    float scale_factor;   /* 1.2 */
    int32_t nlevels;      /* 8 */
    int32_t ini_th_fast;  /* 20 */
    int32_t min_th_fast;  /* 7 */
} odo_orb_params;

typedef struct odo_ransac_params {
    int32_t iterations;        /* Ransac(200,...) odometry.cpp:28 */
    int32_t min_inlier_th;     /* 20 */
    float max_mahalanobis;     /* 3.0 */
    int32_t sample_size;       /* 4 */
    int32_t check_depth;       /* mCheckDepth, true (ransac.cpp:20) */
} odo_ransac_params;

/* Grid-adapted detector (Extractor::ADAPTIVE with FAST inner detector),
 * extractor.cpp:52-77: DetectorAdjuster(FAST, 20, 2, 10000, 1.3, 0.7),
 * VideoDynamicAdaptedFeatureDetector(gridMin=67, gridMax=113, iters=5),
 * VideoGridAdaptedFeatureDetector(maxTotal=1020, 3x3, edge=31), then
 * retainBest(nFeatures=1000) and cv::ORB::compute (extractor.cpp:39-50). */
typedef struct odo_adaptive_params {
    int32_t grid_rows, grid_cols;
    int32_t edge_threshold;
    int32_t max_total_keypoints;
    int32_t cell_min, cell_max;
    int32_t escape_iters;
    double init_thresh, min_thresh, max_thresh;
    double increase_factor, decrease_factor;
    int32_t retain_best;       /* Extract: retainBest(nFeatures) extractor.cpp:45-46 */
} odo_adaptive_params;

/* glibc TYPE_3 additive-feedback generator state (random_r), the
 * process-global rand() stream used by Ransac::SampleMatches
 * (ransac.cpp:275-276) made explicit. */
typedef struct odo_rng {
    int32_t state[31];
    int32_t fpos;   /* index of fptr into state */
    int32_t rpos;   /* index of rptr into state */
} odo_rng;

/* Hypotheses mode: one evaluated RANSAC hypothesis (the
 * visited iteration of that index: its sample, refinement loop and refined
 * transform, ransac.cpp:201-231). cnt = |refined inliers| (0 = no valid
 * refinement); err = refinedError; T = refined T12 rows 0..2. 64 bytes. */
typedef struct odo_hyp_summary {
    double err;
    int32_t cnt;
    int32_t pad;
    float T[12];
} odo_hyp_summary;

/* Outcome of Ransac::Iterate's ordered running-best fold over all
 * hypotheses (ransac.cpp:233-249): best_h = index of the accepted hypothesis
 * (-1: none), visited = iterations run, valid = validIters. */
typedef struct odo_ransac_fold_result {
    int32_t best_h, visited, valid, n_inliers;
    float rmse;
    int32_t n_good;
    int32_t pad[2];
} odo_ransac_fold_result;

/* Result of PnPRansac::Compute's cv::solvePnPRansac (pnpransac.cpp:34-50):
 * (rvec, tvec) refined by solvePnP(ITERATIVE) on the RANSAC inliers, the best
 * RANSAC model, T = Converter::toHomogeneous(r, t) (row-major float), bOK,
 * inliers.rows, the index of the winning hypothesis and the RANSAC
 * iterations run (niters after RANSACUpdateNumIters). 176 bytes. */
typedef struct odo_pnp_ransac_result {
    double rvec[3], tvec[3];
    double model_rvec[3], model_tvec[3];
    float Tcw[16];
    int32_t ok, n_inliers, best_iter, iterations_visited;
} odo_pnp_ransac_result;

/* One local-map landmark for Matcher::ProjectionMatch (matcher.cpp:90-145):
 * world position (Landmark::GetWorldPos), distinctive descriptor
 * (GetDescriptor) and state flags. 48 bytes. */
#define ODO_LM_BAD 1       /* Landmark::isBad() */
#define ODO_LM_SEEN 2      /* mnLastFrameSeen == current frame (already matched; SearchLocalLMs skips it) */
#define ODO_LM_HAS_OBS 4   /* Observations() > 0 (a slot holding it is skipped by later landmarks) */
typedef struct odo_landmark {
    float X[3];
    int32_t flags;
    uint8_t desc[32];
} odo_landmark;

/* Per-frame-pair odometry result. */
typedef struct odo_pair_result {
    float T12[16];        /* RANSAC transform F1->F2 (row-major 4x4) */
    float Tcw[16];        /* PnP-refined pose of F2 (row-major 4x4) */
    float rmse;           /* Ransac::rmse */
    int32_t n_matches;    /* KnnMatch result size */
    int32_t n_good;       /* depth-valid matches entering RANSAC */
    int32_t n_inliers;    /* |Ransac::mvInliers| */
    int32_t ransac_ok;    /* Ransac::Iterate return */
    int32_t pnp_inliers;  /* PnPSolver::Compute return */
    int32_t visited;      /* RANSAC iterations actually run (realIters) */
    int32_t n_queries;    /* kNN-2 queries: F1 keypoints holding a VO landmark (the only ones KnnMatch keeps) */
    int32_t n_sweeps;     /* ComputeInliersAndError calls in the visited iterations (+1 for the identity
                             fallback): the RANSAC work E of SURVEY §8(d) is n_sweeps * n_good evaluations */
    int32_t n_fit_points; /* points added to TransformationFromCorrespondences fits (F of SURVEY §8(d)) */
} odo_pair_result;

#ifdef __cplusplus
}
#endif

#endif /* ODO_TYPES_H */
