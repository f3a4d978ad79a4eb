// Parity test of the C++ reference-interface mirror (include/odo_frontend.hpp)
// against the CPU oracle. TEST INFRASTRUCTURE: links liboracle.so as the checker.
//
// Drives the hot path the way the reference does — Tracking::TrackFrame
// (System/tracking.cpp:193-232) around Odometry::Compute ADAPTIVE_RBA
// (Odometry/odometry.cpp:105-116), in the shape of Tests/Ransac-mahal.cpp's
// frame loop — through odo_hip::Extractor / Frame / Matcher / Ransac /
// PnPSolver on the GPU, and checks every stage against the oracle on the same
// frames:
//   keypoints + descriptors        bit-exact   (oracle_extract_frame[_adaptive])
//   KnnMatch list                  bit-exact   (oracle_track_pair)
//   Ransac mT12, inliers, rmse     bit-exact
//   PnPSolver pose                 |dT| < 1e-4, inlier count and outlier flags equal
//   GeneralizedICP on RANSAC's clouds from T12 (ADAPTIVE_RICP)   converged, |dT| < 1e-5
//   PnPRansac on the frame's landmarks                           inlier count, |dT| < 1e-5
//
// usage: frontend_parity FRAMES.bin W H F SEED [adaptive|adaptive_orb]
//   FRAMES.bin = F x H x W x 3 BGR8, then F x H x W depth16 (x5000)
// Prints one summary line; exit 0 = parity.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/odo_frontend.hpp"
#include "../../oracle/oracle.h"

using namespace std;

static int g_fail = 0;
#define EXPECT(c, ...)                                   \
    do {                                                 \
        if (!(c)) {                                      \
            fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);                \
            fprintf(stderr, "\n");                       \
            g_fail++;                                    \
        }                                                \
    } while (0)

struct OracleFrame {
    vector<orb_kp> kps;
    vector<uint8_t> desc;
    vector<float> kun, xyz, ur;
};

static int run(int argc, char** argv);

// Tracking::SearchLocalLMs' ProjectionMatch on the current frame at its PnP
// pose against the previous frame's landmarks (some with observations, some
// bad, the ones already matched into the frame skipped), through the mirror
// and through the oracle on the same inputs. Returns the match count.
static int check_projection(odo_hip::Frame& last, odo_hip::Frame& cur, const OracleFrame& o, const odo_calib& cal,
                            int W, int H) {
    std::vector<odo_hip::LandmarkPtr> lms;
    for (size_t i = 0; i < last.N; i++)
        if (last.mvpLandmarks[i]) lms.push_back(last.mvpLandmarks[i]);
    for (size_t i = 0; i < lms.size(); i++) {
        lms[i]->nObs = (i % 3 == 0) ? 1 : 0;
        lms[i]->mbBad = (i % 17 == 5);
    }
    const int n = (int)cur.N, nL = (int)lms.size();
    // oracle inputs from the frame state before the call
    std::vector<odo_landmark> ol(std::max(nL, 1));
    for (int i = 0; i < nL; i++) {
        memcpy(ol[i].X, lms[i]->mWorldPos, 12);
        memcpy(ol[i].desc, lms[i]->mDescriptor, 32);
        ol[i].flags = (lms[i]->mbBad ? ODO_LM_BAD : 0) | (lms[i]->nObs > 0 ? ODO_LM_HAS_OBS : 0);
        for (int j = 0; j < n; j++)
            if (cur.mvpLandmarks[j] == lms[i]) ol[i].flags |= ODO_LM_SEEN;
    }
    std::vector<uint8_t> taken(std::max(n, 1));
    std::vector<int32_t> oct(std::max(n, 1)), slot_lm(std::max(n, 1));
    for (int j = 0; j < n; j++) {
        taken[j] = cur.mvpLandmarks[j] && cur.mvpLandmarks[j]->nObs > 0;
        oct[j] = o.kps[j].octave;
    }
    std::vector<odo_hip::LandmarkPtr> before = cur.mvpLandmarks;
    float bounds[4];
    oracle_image_bounds(&cal, W, H, bounds);
    std::vector<float> proj(3 * (size_t)std::max(nL, 1));
    const int onm = oracle_projection_match(cur.mTcw.data(), ol.data(), nL, o.kun.data(), oct.data(), o.desc.data(), n,
                                            taken.data(), &cal, bounds, 8.0f, 0.8f, slot_lm.data(), proj.data());
    odo_hip::Matcher matcher(0.8f);
    const int nm = (int)matcher.ProjectionMatch(&cur, lms, 8.0f);
    EXPECT(nm == onm, "ProjectionMatch: %d matches vs oracle %d", nm, onm);
    int slot_diff = 0, view_diff = 0;
    for (int j = 0; j < n; j++) {
        const odo_hip::LandmarkPtr want = slot_lm[j] >= 0 ? lms[slot_lm[j]] : before[j];
        slot_diff += cur.mvpLandmarks[j] != want;
    }
    for (int i = 0; i < nL; i++) {
        if (ol[i].flags & ODO_LM_SEEN) continue;
        const bool in = !std::isnan(proj[3 * i]);
        view_diff += in != lms[i]->mbTrackInView;
        if (in && lms[i]->mbTrackInView)
            view_diff += memcmp(&proj[3 * i], &lms[i]->mTrackProjX, 4) != 0 ||
                         memcmp(&proj[3 * i + 1], &lms[i]->mTrackProjY, 4) != 0 ||
                         memcmp(&proj[3 * i + 2], &lms[i]->mTrackProjXR, 4) != 0;
    }
    EXPECT(slot_diff == 0, "ProjectionMatch: %d frame slots differ", slot_diff);
    EXPECT(view_diff == 0, "ProjectionMatch: %d landmarks' isInFrustum projections differ", view_diff);
    return nm;
}

int main(int argc, char** argv) {
    // the library never falls back to the CPU: without a gfx950 device the
    // first call that needs one throws odo_hip::Error
    try {
        return run(argc, argv);
    } catch (const odo_hip::Error& e) {
        fprintf(stderr, "odo_hip::Error(%d): %s\n", e.status, e.what());
        return 3;
    }
}

static int run(int argc, char** argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s FRAMES.bin W H F SEED [adaptive|adaptive_orb]\n", argv[0]);
        return 2;
    }
    const int W = atoi(argv[2]), H = atoi(argv[3]), F = atoi(argv[4]);
    const uint32_t seed = (uint32_t)strtoul(argv[5], nullptr, 0);
    const bool adaptive_orb = argc > 6 && strcmp(argv[6], "adaptive_orb") == 0;
    const bool adaptive = adaptive_orb || (argc > 6 && strcmp(argv[6], "adaptive") == 0);
    const size_t npx = (size_t)W * H;
    vector<uint8_t> bgr(npx * 3 * F);
    vector<uint16_t> dep(npx * F);
    FILE* fp = fopen(argv[1], "rb");
    if (!fp || fread(bgr.data(), 1, bgr.size(), fp) != bgr.size() ||
        fread(dep.data(), 2, dep.size(), fp) != dep.size()) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    fclose(fp);

    // unsupported detector combinations fail loudly
    bool threw = false;
    try {
        odo_hip::Extractor bad(odo_hip::Extractor::SURF, odo_hip::Extractor::BRIEF, odo_hip::Extractor::ADAPTIVE);
    } catch (const std::invalid_argument&) {
        threw = true;
    }
    EXPECT(threw, "Extractor(SURF, BRIEF, ADAPTIVE) must throw");

    odo_hip::Extractor extractor =
        adaptive_orb ? odo_hip::Extractor(odo_hip::Extractor::ORB, odo_hip::Extractor::ORB, odo_hip::Extractor::ADAPTIVE)
        : adaptive   ? odo_hip::Extractor(odo_hip::Extractor::FAST, odo_hip::Extractor::ORB, odo_hip::Extractor::ADAPTIVE)
                     : odo_hip::Extractor(odo_hip::Extractor::ORB_SLAM2, odo_hip::Extractor::ORB_SLAM2,
                                      odo_hip::Extractor::NORMAL);
    const odo_calib cal = odo_hip::Calibration();
    odo_orb_params orb;
    {
        odo_config cfg;
        odo_default_config(&cfg, W, H, 2);
        orb = cfg.orb;
    }
    odo_adaptive_params ap;
    oracle_adaptive_default(&ap);
    vector<double> thresh(ap.grid_rows * ap.grid_cols, ap.init_thresh);
    const int cap = 2048;
    odo_ransac_params rp{200, 20, 3.0f, 4, 1};
    double latch = nan("");
    odo_hip::ResetDepthCovarianceLatch();

    std::unique_ptr<odo_hip::Frame> last;
    OracleFrame olast;
    long total_matches = 0, total_inliers = 0, total_pnp = 0;
    int proj_checked = -1, gicp_checked = 0, pnpransac_checked = 0;
    double max_dT = 0;
    for (int t = 0; t < F; t++) {
        // the frame keeps its own images: built from scratch
        // buffers that are overwritten before ExtractFeatures
        vector<uint8_t> sb(&bgr[npx * 3 * t], &bgr[npx * 3 * (t + 1)]);
        vector<uint16_t> sd(&dep[npx * t], &dep[npx * (t + 1)]);
        auto cur = std::make_unique<odo_hip::Frame>(sb.data(), sd.data(), W, H, 0.033 * t);
        std::fill(sb.begin(), sb.end(), (uint8_t)0x5A);
        std::fill(sd.begin(), sd.end(), (uint16_t)0);
        cur->ExtractFeatures(&extractor);
        if (t == 0 && !adaptive && !adaptive_orb) {
            // a copy of the frame shares the images and extracts again
            odo_hip::Frame cp = *cur;
            cp.ExtractFeatures(&extractor);
            EXPECT(cp.mvKeys.size() == cur->N && cp.mDescriptors == cur->mDescriptors &&
                       cp.mvKeys3Dc.size() == cur->N,
                   "frame 0: re-extraction from a copy of the frame differs");
        }

        OracleFrame o;
        o.kps.resize(cap);
        o.desc.resize(32 * cap);
        o.kun.resize(2 * cap);
        o.xyz.resize(3 * cap);
        o.ur.resize(cap);
        const int n = adaptive_orb
                          ? oracle_extract_frame_adaptive_orb(&bgr[npx * 3 * t], &dep[npx * t], W, H, &ap,
                                                              thresh.data(), &cal, o.kps.data(), o.desc.data(),
                                                              o.kun.data(), o.xyz.data(), o.ur.data(), cap)
                      : adaptive ? oracle_extract_frame_adaptive(&bgr[npx * 3 * t], &dep[npx * t], W, H, &ap,
                                                               thresh.data(), &cal, o.kps.data(), o.desc.data(),
                                                               o.kun.data(), o.xyz.data(), o.ur.data(), cap)
                               : oracle_extract_frame(&bgr[npx * 3 * t], &dep[npx * t], W, H, &orb, &cal,
                                                      o.kps.data(), o.desc.data(), o.kun.data(), o.xyz.data(),
                                                      o.ur.data(), cap);
        o.kps.resize(n);
        o.desc.resize(32 * (size_t)n);
        EXPECT((int)cur->N == n, "frame %d: N %zu vs oracle %d", t, cur->N, n);
        if ((int)cur->N == n) {
            EXPECT(memcmp(cur->mvKeys.data(), o.kps.data(), n * sizeof(orb_kp)) == 0, "frame %d: keypoints", t);
            EXPECT(cur->mDescriptors == o.desc, "frame %d: descriptors", t);
            bool geo = true;
            for (int i = 0; i < n; i++)
                geo = geo && cur->mvKeysUn[i].x == o.kun[2 * i] && cur->mvKeysUn[i].y == o.kun[2 * i + 1] &&
                      memcmp(&cur->mvKeys3Dc[i], &o.xyz[3 * i], 12) == 0 && memcmp(&cur->mvuRight[i], &o.ur[i], 4) == 0;
            EXPECT(geo, "frame %d: mvKeysUn / mvKeys3Dc / mvuRight", t);
        }

        if (last) {
            // Batched contract: F1 at identity with fresh VO landmarks.
            last->mvpLandmarks.assign(last->N, nullptr);
            last->mvbOutlier.assign(last->N, false);
            last->SetPose(odo_hip::Identity());
            odo_hip::CreateVOLandmarks(*last);

            // Tracking::TrackFrame
            odo_hip::Matcher matcher(0.9f);
            vector<odo_hip::DMatch> vMatches12;
            const size_t nmatches = matcher.KnnMatch(*last, *cur, vMatches12);
            const uint32_t pseed = seed + (uint32_t)t;
            int pnp = 0;
            odo_hip::Ransac ransac(200, 20, 3.0f, 4);
            bool ok = false;
            odo_hip::Pose T12 = odo_hip::Identity();
            if (nmatches >= 20) {
                odo_hip::Srand(pseed);
                ok = ransac.Iterate(last.get(), cur.get(), vMatches12);
                T12 = ransac.mT12;
                cur->SetPose(odo_hip::Mul(T12, last->GetPose()));  // Tcw2 = T12 * Tcw1
                pnp = odo_hip::PnPSolver::Compute(cur.get());
            }

            odo_pair_result r;
            vector<uint8_t> mask(std::max(n, 1));
            vector<odo_dmatch> om(std::max((int)olast.kps.size(), 1)), oinl(om.size());
            int noinl = 0;
            const int onm = oracle_track_pair(olast.kps.data(), olast.desc.data(), olast.xyz.data(),
                                              (int)olast.kps.size(), o.kps.data(), o.desc.data(), o.kun.data(),
                                              o.xyz.data(), o.ur.data(), n, &cal, 0.9f, &rp, pseed, &latch, &r,
                                              mask.data(), om.data(), (int)om.size(), oinl.data(), &noinl);
            EXPECT((int)nmatches == onm, "pair %d: %zu matches vs oracle %d", t, nmatches, onm);
            if ((int)nmatches == onm)
                EXPECT(memcmp(vMatches12.data(), om.data(), onm * sizeof(odo_dmatch)) == 0, "pair %d: match list", t);
            total_matches += (long)nmatches;
            if (nmatches >= 20) {
                EXPECT(ok == (r.ransac_ok != 0), "pair %d: Iterate %d vs %d", t, ok, r.ransac_ok);
                EXPECT(memcmp(T12.data(), r.T12, 64) == 0, "pair %d: mT12", t);
                EXPECT((int)ransac.mvInliers.size() == r.n_inliers, "pair %d: inliers %zu vs %d", t,
                       ransac.mvInliers.size(), r.n_inliers);
                // Ransac::mvInliers entry for entry (ransac.cpp:240, 258)
                if ((int)ransac.mvInliers.size() == noinl)
                    EXPECT(memcmp(ransac.mvInliers.data(), oinl.data(), noinl * sizeof(odo_dmatch)) == 0,
                           "pair %d: mvInliers list", t);
                EXPECT(ransac.rmse == r.rmse, "pair %d: rmse %.9g vs %.9g", t, ransac.rmse, r.rmse);
                EXPECT(pnp == r.pnp_inliers, "pair %d: PnP inliers %d vs %d", t, pnp, r.pnp_inliers);
                double d = 0;
                for (int k = 0; k < 16; k++) d = std::max(d, (double)fabsf(cur->mTcw[k] - r.Tcw[k]));
                max_dT = std::max(max_dT, d);
                EXPECT(d < 1e-4, "pair %d: PnP pose |dT| = %g", t, d);
                int flag_diff = 0;
                for (int i = 0; i < n; i++) {
                    const int in = cur->GetLandmark(i) && !cur->IsOutlier(i);
                    flag_diff += in != mask[i];
                }
                EXPECT(flag_diff == 0, "pair %d: %d PnP outlier flags differ", t, flag_diff);
                total_inliers += r.n_inliers;
                total_pnp += pnp;
                // GeneralizedICP(10, 0.07) on RANSAC's matched clouds from T12
                // (ADAPTIVE_RICP, odometry.cpp:61) vs the oracle on the same clouds
                {
                    odo_hip::GeneralizedICP gicp(10, 0.07);
                    const bool gok = gicp.Compute(ransac.mvSourceCloud, ransac.mvTargetCloud, T12);
                    float Tg[16];
                    int conv = 0, it = 0, nc = 0;
                    oracle_gicp(ransac.mvSourceCloud.data(), (int)(ransac.mvSourceCloud.size() / 3),
                                ransac.mvTargetCloud.data(), (int)(ransac.mvTargetCloud.size() / 3), T12.data(), 10,
                                0.07, Tg, &conv, &it, &nc);
                    EXPECT(gok == (conv != 0), "pair %d: GICP converged %d vs %d", t, (int)gok, conv);
                    double dg = 0;
                    for (int k = 0; k < 16; k++) dg = std::max(dg, (double)fabsf(gicp.mT12[k] - Tg[k]));
                    EXPECT(dg < 1e-5, "pair %d: GICP |dT| = %g", t, dg);
                    gicp_checked++;
                }
                // PnPRansac::Compute on the frame's landmarks (a copy of the frame)
                {
                    odo_hip::Frame fr = *cur;
                    odo_hip::PnPRansac pr;
                    vector<float> Xw, uv;
                    for (size_t i = 0; i < fr.N; i++)
                        if (fr.GetLandmark(i)) {
                            const odo_hip::LandmarkPtr lm = fr.GetLandmark(i);
                            Xw.insert(Xw.end(), {lm->mWorldPos[0], lm->mWorldPos[1], lm->mWorldPos[2]});
                            uv.insert(uv.end(), {fr.mvKeysUn[i].x, fr.mvKeysUn[i].y});
                        }
                    const int nobs = (int)(uv.size() / 2);
                    if (nobs >= 10) {
                        const int ninl = pr.Compute(fr);
                        double model[6], rt[6];
                        float To[16];
                        vector<uint8_t> om2(nobs);
                        int oinl = 0, best = 0, nit = 0;
                        const int ook = oracle_pnp_ransac(Xw.data(), uv.data(), nobs, &cal, 500, 3.0f, 0.85, model, rt,
                                                          To, om2.data(), &oinl, &best, &nit, nullptr);
                        EXPECT(ook == 1 && ninl == oinl, "pair %d: PnPRansac inliers %d vs %d", t, ninl, oinl);
                        double dp = 0;
                        for (int k = 0; k < 16; k++) dp = std::max(dp, (double)fabsf(fr.mTcw[k] - To[k]));
                        EXPECT(dp < 1e-5, "pair %d: PnPRansac |dT| = %g", t, dp);
                        pnpransac_checked++;
                    }
                }
                if (t == F - 1) proj_checked = check_projection(*last, *cur, o, cal, W, H);
            }
        }
        last = std::move(cur);
        olast = std::move(o);
    }

    // Kabsch::Compute on a known rigid motion
    {
        vector<float> A, B;
        const float R[9] = {0.936293f, -0.275034f, 0.218351f, 0.289629f, 0.956425f, -0.036957f,
                            -0.198669f, 0.097843f, 0.975170f};
        for (int i = 0; i < 50; i++) {
            const float p[3] = {0.1f * (i % 7) - 0.3f, 0.05f * (i % 11) - 0.2f, 1.0f + 0.03f * i};
            A.insert(A.end(), p, p + 3);
            for (int r = 0; r < 3; r++) B.push_back(R[3 * r] * p[0] + R[3 * r + 1] * p[1] + R[3 * r + 2] * p[2] + 0.1f * (r + 1));
        }
        odo_hip::Kabsch k;
        const odo_hip::Pose T = k.Compute(A, B);
        float To[16];
        oracle_kabsch(A.data(), B.data(), 50, To);
        double d = 0;
        for (int q = 0; q < 16; q++) d = std::max(d, (double)fabsf(T[q] - To[q]));
        EXPECT(d < 1e-4, "Kabsch::Compute vs oracle: %g", d);
    }

    printf("frontend_parity %s frames=%d matches=%ld ransac_inliers=%ld pnp_inliers=%ld max_dT=%.3g "
           "projection_matches=%d gicp_checked=%d pnpransac_checked=%d failures=%d\n",
           adaptive_orb ? "adaptive_orb" : adaptive ? "adaptive" : "orb_slam2", F, total_matches, total_inliers, total_pnp, max_dT, proj_checked,
           gicp_checked, pnpransac_checked, g_fail);
    return g_fail ? 1 : 0;
}
