// Per-frame latency of the drop-in path: one
// Tracking::Track frame at a time through the reference-shaped C++ classes of
// include/odo_frontend.hpp, in TrackFrame order (tracking.cpp:38-78, 193-208):
//
//   Frame(bgr, depth) + ExtractFeatures   -> odo_extract
//   UpdateLastFrame VO landmarks          -> host
//   Matcher(0.9).KnnMatch                 -> odo_knn2_hamming + host ratio/bookkeeping
//   Ransac(iters, 20, 3, 4).Iterate       -> odo_ransac
//   SetPose(T12 * Tcw1); PnPSolver        -> odo_pnp_motion_ba
//
// Usage: frontend_latency FRAMES.bin W H F [ITERS] [WARMUP]   (FRAMES.bin = F BGR8 frames
// then F depth16 frames). Prints one JSON object: per-frame wall time p50 /
// p90 / p99 / mean (ms) after WARMUP frames, and each stage's median.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <vector>

#include "../include/odo_frontend.hpp"

using Clock = std::chrono::steady_clock;

static double pct(std::vector<double> v, double q) {
    if (v.empty()) return 0.0;
    std::sort(v.begin(), v.end());
    const size_t i = std::min(v.size() - 1, (size_t)(q * (double)(v.size() - 1) + 0.5));
    return v[i];
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s FRAMES.bin W H F [ITERS] [WARMUP]\n", argv[0]);
        return 2;
    }
    const int W = atoi(argv[2]), H = atoi(argv[3]), F = atoi(argv[4]);
    const int iters = argc > 5 ? atoi(argv[5]) : 500;
    const int warm = argc > 6 ? atoi(argv[6]) : 8;
    const size_t npx = (size_t)W * H;
    std::vector<uint8_t> bgr(npx * 3 * F);
    std::vector<uint16_t> dep(npx * F);
    FILE* fp = fopen(argv[1], "rb");
    if (!fp || fread(bgr.data(), 1, bgr.size(), fp) != bgr.size() || fread(dep.data(), 2, dep.size(), fp) != dep.size()) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    fclose(fp);
    try {
        odo_hip::Extractor extractor(odo_hip::Extractor::ORB_SLAM2, odo_hip::Extractor::ORB_SLAM2,
                                     odo_hip::Extractor::NORMAL);
        odo_hip::Srand(12345);
        odo_hip::ResetDepthCovarianceLatch();
        std::unique_ptr<odo_hip::Frame> last;
        std::vector<double> tot, t_ext, t_lm, t_knn, t_ran, t_pnp;
        long matches = 0, inliers = 0, pairs = 0;
        for (int k = 0; k < F; k++) {
            const auto t0 = Clock::now();
            auto cur = std::make_unique<odo_hip::Frame>(odo_hip::kBorrowImages, &bgr[npx * 3 * k], &dep[npx * k], W, H,
                                                        0.033 * k);  // the buffers outlive the loop
            cur->ExtractFeatures(&extractor);
            const auto t1 = Clock::now();
            auto t2 = t1, t3 = t1, t4 = t1, t5 = t1;
            if (last) {
                // Tracking::UpdateLastFrame (tracking.cpp:136-191): F1 at its pose, fresh VO landmarks
                last->mvpLandmarks.assign(last->N, nullptr);
                last->mvbOutlier.assign(last->N, false);
                last->SetPose(odo_hip::Identity());
                odo_hip::CreateVOLandmarks(*last);
                t2 = Clock::now();
                odo_hip::Matcher matcher(0.9f);
                std::vector<odo_hip::DMatch> m12;
                const size_t nm = matcher.KnnMatch(*last, *cur, m12);
                t3 = t4 = t5 = Clock::now();
                if (nm >= 20) {
                    odo_hip::Ransac ransac(iters, 20, 3.0f, 4);
                    ransac.Iterate(last.get(), cur.get(), m12);
                    t4 = Clock::now();
                    cur->SetPose(odo_hip::Mul(ransac.mT12, last->GetPose()));  // Tcw2 = T12 * Tcw1
                    odo_hip::PnPSolver::Compute(cur.get());
                    t5 = Clock::now();
                    inliers += (long)ransac.mvInliers.size();
                }
                matches += (long)nm;
                pairs++;
            }
            auto ms = [](Clock::time_point a, Clock::time_point b) {
                return std::chrono::duration<double, std::milli>(b - a).count();
            };
            if (k >= warm) {
                tot.push_back(ms(t0, t5));
                t_ext.push_back(ms(t0, t1));
                t_lm.push_back(ms(t1, t2));
                t_knn.push_back(ms(t2, t3));
                t_ran.push_back(ms(t3, t4));
                t_pnp.push_back(ms(t4, t5));
            }
            last = std::move(cur);
        }
        double mean = 0;
        for (double v : tot) mean += v;
        mean /= std::max<size_t>(tot.size(), 1);
        printf("{\"frames\": %zu, \"warmup\": %d, \"p50_ms\": %.4f, \"p90_ms\": %.4f, \"p99_ms\": %.4f, "
               "\"mean_ms\": %.4f, \"max_ms\": %.4f, \"stage_median_ms\": {\"extract\": %.4f, \"vo_landmarks\": %.4f, "
               "\"knn_match\": %.4f, \"ransac\": %.4f, \"pnp\": %.4f}, \"mean_matches\": %.1f, "
               "\"mean_ransac_inliers\": %.1f}\n",
               tot.size(), warm, pct(tot, 0.5), pct(tot, 0.9), pct(tot, 0.99), mean, pct(tot, 1.0), pct(t_ext, 0.5),
               pct(t_lm, 0.5), pct(t_knn, 0.5), pct(t_ran, 0.5), pct(t_pnp, 0.5),
               pairs ? (double)matches / pairs : 0.0, pairs ? (double)inliers / pairs : 0.0);
    } catch (const odo_hip::Error& e) {
        fprintf(stderr, "odo_hip::Error(%d): %s\n", e.status, e.what());
        return 3;
    }
    return 0;
}
