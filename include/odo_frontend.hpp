/*
 * odo_frontend.hpp — C++ mirror of the reference's hot-path classes over the
 * C-ABI of libodo_hip.so (header-only, C++17, no OpenCV / Eigen / g2o).
 *
 * A reference user keeps the call pattern of Tracking::TrackFrame
 * (System/tracking.cpp:193-232) and Odometry::Compute ADAPTIVE_RBA
 * (Odometry/odometry.cpp:105-116):
 *
 *     odo_hip::Extractor extractor(Extractor::ORB_SLAM2, Extractor::ORB_SLAM2, Extractor::NORMAL);
 *     odo_hip::Frame cur(bgr, depth, width, height, timestamp);
 *     cur.ExtractFeatures(&extractor);
 *     odo_hip::CreateVOLandmarks(last);                       // UpdateLastFrame
 *     odo_hip::Matcher matcher(0.9f);
 *     matcher.KnnMatch(last, cur, vMatches12);
 *     odo_hip::Ransac ransac(200, 20, 3.0f, 4);
 *     ransac.Iterate(&last, &cur, vMatches12);
 *     cur.SetPose(odo_hip::Mul(ransac.mT12, last.mTcw));
 *     odo_hip::PnPSolver::Compute(&cur);
 *
 * Each class names the reference interface it stands in for. The classes are
 * host bookkeeping only: every feature, match, hypothesis and pose comes from
 * the HIP kernels behind include/odo.h, and any failure of the library
 * (no gfx950 device, bad arguments) throws odo_hip::Error — there is no CPU
 * fallback. Types are plain structs with the memory layout of the OpenCV
 * types they replace (odo_types.h), so vectors of them can be memcpy'd into
 * std::vector<cv::KeyPoint> / std::vector<cv::DMatch>.
 *
 * Process-wide state mirrors the reference's globals: the rand() stream that
 * Ransac::SampleMatches draws from (srand(clock()) in main.cpp:27 -> Srand()),
 * the DepthCovariance static latch (ransac.cpp:303-312) and the Calibration
 * namespace (Utils/common.h:32-74 -> SetCalibration()).
 */
#ifndef ODO_FRONTEND_HPP
#define ODO_FRONTEND_HPP

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "odo.h"

namespace odo_hip {

using KeyPoint = orb_kp;   // cv::KeyPoint layout
using DMatch = odo_dmatch; // cv::DMatch layout
using Pose = std::array<float, 16>;  // row-major 4x4 (cv::Mat mTcw / Eigen::Matrix4f mT12)

struct Point3f {
    float x, y, z;
};

struct Error : std::runtime_error {
    int status;
    Error(int st, const std::string& what) : std::runtime_error(what), status(st) {}
};

inline void Check(int st, const char* what) {
    if (st != ODO_OK) throw Error(st, std::string(what) + ": " + odo_last_error());
}

inline Pose Identity() {
    Pose T{};
    T[0] = T[5] = T[10] = T[15] = 1.f;
    return T;
}

// A * B for row-major 4x4 (cv::Mat float product, accumulated in double).
inline Pose Mul(const Pose& A, const Pose& B) {
    Pose C{};
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) {
            double s = 0;
            for (int k = 0; k < 4; k++) s += (double)A[4 * r + k] * B[4 * k + c];
            C[4 * r + c] = (float)s;
        }
    return C;
}

namespace detail {
struct Globals {
    std::mutex mu;
    odo_rng rng;                 // rand() stream of Ransac::SampleMatches
    double latch = std::nan(""); // DepthCovariance static (ransac.cpp:303)
    odo_calib calib;             // Calibration namespace
    bool calib_set = false;
    std::shared_ptr<odo_ctx> ctx;  // scratch for Matcher / Ransac / PnPSolver
    int device = 0;
    Globals() { odo_rng_seed(&rng, 1); }  // glibc: rand() without srand() = srand(1)
};
inline Globals& G() {
    static Globals g;
    return g;
}
inline std::shared_ptr<odo_ctx> make_ctx(const odo_config& cfg, int device) {
    odo_ctx* c = odo_create(&cfg, device);
    if (!c) throw Error(ODO_ERR_DEVICE, std::string("odo_create: ") + odo_last_error());
    return std::shared_ptr<odo_ctx>(c, odo_destroy);
}
inline odo_config default_config(int width, int height) {
    odo_config cfg;
    odo_default_config(&cfg, width, height, 2);
    if (G().calib_set) cfg.calib = G().calib;
    return cfg;
}
// Matcher / Ransac / PnPSolver need device scratch but no image geometry.
inline odo_ctx* shared_ctx() {
    Globals& g = G();
    std::lock_guard<std::mutex> lk(g.mu);
    if (!g.ctx) g.ctx = make_ctx(default_config(640, 480), g.device);
    return g.ctx.get();
}
// ProjectionMatch needs the frame's image bounds: one context per image size.
inline odo_ctx* geometry_ctx(int width, int height) {
    Globals& g = G();
    std::lock_guard<std::mutex> lk(g.mu);
    static std::vector<std::pair<std::pair<int, int>, std::shared_ptr<odo_ctx>>> by_size;
    for (auto& e : by_size)
        if (e.first.first == width && e.first.second == height) return e.second.get();
    by_size.emplace_back(std::make_pair(width, height), make_ctx(default_config(width, height), g.device));
    return by_size.back().second.get();
}
}  // namespace detail

// srand(seed) for the stream Ransac::SampleMatches draws from (main.cpp:27).
inline void Srand(uint32_t seed) {
    std::lock_guard<std::mutex> lk(detail::G().mu);
    odo_rng_seed(&detail::G().rng, seed);
}
// Forget the DepthCovariance latch (a new process in the reference).
inline void ResetDepthCovarianceLatch() { detail::G().latch = std::nan(""); }
// Calibration namespace (common.h); default = FR1 as odo_default_config.
inline void SetCalibration(const odo_calib& c) {
    detail::G().calib = c;
    detail::G().calib_set = true;
}
inline odo_calib Calibration() { return detail::default_config(640, 480).calib; }
// Device used by objects created afterwards (the reference has no choice).
inline void SetDevice(int device) { detail::G().device = device; }

// Landmark (Core/landmark.h): the fields the hot path reads.
struct Landmark {
    float mWorldPos[3] = {0, 0, 0};
    int nObs = 0;  // Observations(): 0 for visual-odometry temporal points
    bool mbBad = false;
    uint8_t mDescriptor[32] = {};
    // set by Matcher::ProjectionMatch's isInFrustum (frame.cpp:100-133)
    bool mbTrackInView = false;
    float mTrackProjX = 0, mTrackProjY = 0, mTrackProjXR = 0;
    int Observations() const { return nObs; }
    bool isBad() const { return mbBad; }
};
using LandmarkPtr = std::shared_ptr<Landmark>;

class Frame;

// Features/extractor.h:6-42. The configurations of the hot path run on the
// GPU: (ORB_SLAM2, ORB_SLAM2, NORMAL), the reference default (main.cpp:19-21),
// and the grid-adapted detector (extractor.cpp:52-77) with the FAST inner
// detector, (FAST, ORB, ADAPTIVE), or the cv::ORB one, (ORB, ORB, ADAPTIVE)
// (detectoradjuster.cpp:29). Any other combination throws
// std::invalid_argument.
class Extractor {
public:
    enum eAlgorithm { ORB = 0, ORB_SLAM2, FAST, GFTT, STAR, BRISK, FREAK, BRIEF, LATCH, SURF, SIFT };
    enum eMode { NORMAL = 0, ADAPTIVE };

    eAlgorithm mDetectorAlgorithm;
    eAlgorithm mDescriptorAlgorithm;
    eMode mMode;
    static constexpr int mNorm = 6;  // cv::NORM_HAMMING (extractor.cpp:7, set by CreateDescriptor)

    Extractor(const eAlgorithm& detector = ORB_SLAM2, const eAlgorithm& descriptor = ORB_SLAM2,
              const eMode& mode = NORMAL)
        : mDetectorAlgorithm(detector), mDescriptorAlgorithm(descriptor), mMode(mode) {
        if (detector == ORB_SLAM2 && descriptor == ORB_SLAM2 && mode == NORMAL)
            mDetector = ODO_DETECTOR_ORB_SLAM2;
        else if (detector == FAST && descriptor == ORB && mode == ADAPTIVE)
            mDetector = ODO_DETECTOR_ADAPTIVE_FAST;
        else if (detector == ORB && descriptor == ORB && mode == ADAPTIVE)
            mDetector = ODO_DETECTOR_ADAPTIVE_ORB;
        else
            throw std::invalid_argument("odo_hip::Extractor: only (ORB_SLAM2, ORB_SLAM2, NORMAL), "
                                        "(FAST, ORB, ADAPTIVE) and (ORB, ORB, ADAPTIVE) run on the MI355X path");
    }

    // Extractor::Extract(image, mask, keypoints, descriptors) (extractor.cpp:39-50):
    // image = BGR8 (channels 3) or gray (channels 1), row-major width x height;
    // descriptors = N x 32 bytes. The mask argument of the reference is always
    // cv::noArray() on this path.
    void Extract(const uint8_t* image, int width, int height, int channels, std::vector<KeyPoint>& keypoints,
                 std::vector<uint8_t>& descriptors) {
        run(image, width, height, channels, nullptr, &keypoints, &descriptors, nullptr, nullptr, nullptr);
    }

    // The Frame::ExtractFeatures variant (frame.cpp:135-170): also the
    // undistorted keypoints, camera-frame points from depth and mvuRight.
    void ExtractFrame(const uint8_t* image, int width, int height, int channels, const uint16_t* depth,
                      std::vector<KeyPoint>& kps, std::vector<uint8_t>& desc, std::vector<float>& kps_un,
                      std::vector<float>& xyz, std::vector<float>& u_right) {
        run(image, width, height, channels, depth, &kps, &desc, &kps_un, &xyz, &u_right);
    }

    odo_ctx* context() const { return mCtx.get(); }

private:
    void run(const uint8_t* image, int width, int height, int channels, const uint16_t* depth,
             std::vector<KeyPoint>* kps, std::vector<uint8_t>* desc, std::vector<float>* kun,
             std::vector<float>* xyz, std::vector<float>* ur) {
        if (!image || width <= 0 || height <= 0 || (channels != 1 && channels != 3))
            throw std::invalid_argument("odo_hip::Extractor::Extract: empty or unsupported image");
        if (!mCtx || width != mW || height != mH) {
            odo_config cfg = detail::default_config(width, height);
            cfg.detector = mDetector;
            mCtx = detail::make_ctx(cfg, detail::G().device);
            mW = width;
            mH = height;
            mCap = std::max(cfg.orb.nfeatures + 4 * cfg.orb.nlevels + 64, cfg.adaptive.max_total_keypoints + 64);
        }
        std::vector<KeyPoint> k(mCap);
        std::vector<uint8_t> d((size_t)mCap * 32);
        std::vector<float> un((size_t)mCap * 2), p((size_t)mCap * 3), r(mCap);
        int n = 0;
        Check(odo_extract(mCtx.get(), image, channels, depth, k.data(), d.data(), un.data(), p.data(), r.data(), mCap,
                          &n),
              "Extractor::Extract");
        k.resize(n);
        d.resize((size_t)n * 32);
        un.resize((size_t)n * 2);
        p.resize((size_t)n * 3);
        r.resize(n);
        *kps = std::move(k);
        *desc = std::move(d);
        if (kun) *kun = std::move(un);
        if (xyz) *xyz = std::move(p);
        if (ur) *ur = std::move(r);
    }

    int mDetector = ODO_DETECTOR_ORB_SLAM2;
    std::shared_ptr<odo_ctx> mCtx;
    int mW = 0, mH = 0, mCap = 0;
};

// Tag of Frame's zero-copy constructor.
struct BorrowImages {};
constexpr BorrowImages kBorrowImages{};

// Core/frame.h: the members the hot path reads and writes.
class Frame {
public:
    // Frame(imColor, imDepth, timestamp) (frame.cpp:18-60): BGR8 + depth16
    // (x5000, Calibration::mDepthFactor; depth may be null). As the
    // reference's cv::Mat members (mImColor, mImGray and mImDepth stay with the
    // frame, keyframe.cpp:27, matcher.cpp:318), the frame keeps its own copies:
    // the caller may reuse its buffers at once, copies of the frame share
    // them, and ExtractFeatures may run again. The gray / float conversions
    // are the GPU's (odo_extract).
    Frame(const uint8_t* bgr, const uint16_t* depth, int width, int height, double timestamp)
        : mTimestamp(timestamp), mW(width), mH(height), mTcw(Identity()) {
        if (!bgr || width <= 0 || height <= 0) throw std::invalid_argument("odo_hip::Frame: empty image");
        const size_t npx = (size_t)width * height;
        auto c = std::make_shared<std::vector<uint8_t>>(bgr, bgr + 3 * npx);
        mImColor = c->data();
        mColorOwned = std::move(c);
        if (depth) {
            auto d = std::make_shared<std::vector<uint16_t>>(depth, depth + npx);
            mImDepth = d->data();
            mDepthOwned = std::move(d);
        }
    }

    // Zero-copy opt-in (not a reference constructor): the frame refers to the
    // caller's images, which must stay valid and unchanged for as long as any
    // copy of the frame may call ExtractFeatures. For a per-frame loop that
    // extracts right after construction (Tracking::Track, tracking.cpp:41) it
    // saves the 1.5 MB host copy.
    Frame(BorrowImages, const uint8_t* bgr, const uint16_t* depth, int width, int height, double timestamp)
        : mTimestamp(timestamp), mW(width), mH(height), mImColor(bgr), mImDepth(depth), mTcw(Identity()) {
        if (!bgr || width <= 0 || height <= 0) throw std::invalid_argument("odo_hip::Frame: empty image");
    }

    // Frame::ExtractFeatures (frame.cpp:135-170): Extract + UndistortKeyPoints +
    // depth backprojection (mvKeys3Dc, mvuRight), landmark slots reset.
    void ExtractFeatures(Extractor* pExtractor) {
        std::vector<float> kun, xyz;
        pExtractor->ExtractFrame(mImColor, mW, mH, 3, mImDepth, mvKeys, mDescriptors, kun, xyz, mvuRight);
        N = mvKeys.size();
        mvKeysUn = mvKeys;
        mvKeys3Dc.resize(N);
        for (size_t i = 0; i < N; i++) {
            mvKeysUn[i].x = kun[2 * i];
            mvKeysUn[i].y = kun[2 * i + 1];
            mvKeys3Dc[i] = Point3f{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
        }
        mvpLandmarks.assign(N, nullptr);
        mvbOutlier.assign(N, false);
    }

    int Width() const { return mW; }
    int Height() const { return mH; }
    void SetPose(const Pose& Tcw) { mTcw = Tcw; }
    Pose GetPose() const { return mTcw; }

    LandmarkPtr GetLandmark(size_t i) const { return mvpLandmarks[i]; }
    void AddLandmark(LandmarkPtr p, size_t i) { mvpLandmarks[i] = std::move(p); }
    void ReleaseLandmark(size_t i) { mvpLandmarks[i] = nullptr; }
    void SetOutlier(size_t i) { mvbOutlier[i] = true; }
    void SetInlier(size_t i) { mvbOutlier[i] = false; }
    bool IsOutlier(size_t i) const { return mvbOutlier[i]; }
    bool IsInlier(size_t i) const { return !mvbOutlier[i]; }

    // Frame::UnprojectWorld (frame.cpp:231-247) of a point already in camera
    // coordinates: Rwc * Xc + twc, in double.
    Point3f UnprojectWorld(size_t i) const {
        const Point3f& p = mvKeys3Dc[i];
        const Pose& T = mTcw;
        // Twc = [R^T | -R^T t]: Xw = R^T (Xc - t)
        const double d[3] = {(double)p.x - T[3], (double)p.y - T[7], (double)p.z - T[11]};
        double c[3];
        for (int r = 0; r < 3; r++) c[r] = (double)T[r] * d[0] + (double)T[4 + r] * d[1] + (double)T[8 + r] * d[2];
        return Point3f{(float)c[0], (float)c[1], (float)c[2]};
    }

    double mTimestamp;
    size_t N = 0;
    std::vector<KeyPoint> mvKeys, mvKeysUn;
    std::vector<Point3f> mvKeys3Dc;
    std::vector<float> mvuRight;
    std::vector<uint8_t> mDescriptors;  // N x 32
    std::vector<LandmarkPtr> mvpLandmarks;
    std::vector<bool> mvbOutlier;

    const uint8_t* ImColor() const { return mImColor; }
    const uint16_t* ImDepth() const { return mImDepth; }

private:
    int mW, mH;
    const uint8_t* mImColor = nullptr;   // BGR8: the frame's copy, or the caller's (BorrowImages)
    const uint16_t* mImDepth = nullptr;  // depth16 (or null), likewise
    std::shared_ptr<const std::vector<uint8_t>> mColorOwned;  // shared by copies of the frame
    std::shared_ptr<const std::vector<uint16_t>> mDepthOwned;

public:
    Pose mTcw;
};

// Tracking::UpdateLastFrame's "visual odometry" landmarks (tracking.cpp:146-190):
// points sorted by depth, all closer than Calibration::mThDepth, at least the
// 100 closest. Returns the number of points visited (nPoints).
inline int CreateVOLandmarks(Frame& F) {
    const odo_calib c = Calibration();
    const float thDepth = c.mbf * c.th_depth / c.fx;  // Calibration::mThDepth
    std::vector<std::pair<float, size_t>> v;
    for (size_t i = 0; i < F.N; i++)
        if (F.mvKeys3Dc[i].z > 0) v.push_back(std::make_pair(F.mvKeys3Dc[i].z, i));
    if (v.empty()) return 0;
    std::sort(v.begin(), v.end());
    int nPoints = 0;
    for (size_t j = 0; j < v.size(); j++) {
        const size_t i = v[j].second;
        LandmarkPtr lm = F.GetLandmark(i);
        if (!lm || lm->Observations() < 1) {
            auto p = std::make_shared<Landmark>();
            const Point3f X = F.UnprojectWorld(i);
            p->mWorldPos[0] = X.x;
            p->mWorldPos[1] = X.y;
            p->mWorldPos[2] = X.z;
            std::memcpy(p->mDescriptor, &F.mDescriptors[32 * i], 32);
            F.AddLandmark(p, i);
        }
        nPoints++;
        if (v[j].first > thDepth && nPoints > 100) break;
    }
    return nPoints;
}

// Features/matcher.h:9-45, the frame-to-frame path.
class Matcher {
public:
    explicit Matcher(float nnratio = 0.6f) : mfNNratio(nnratio) {}

    // Matcher::KnnMatch(Frame&, Frame&, vMatches12) (matcher.cpp:55-88): the
    // k=2 Hamming brute force on the GPU for the queries that can match, then
    // the ratio test and the landmark hand-over in query order on the host.
    size_t KnnMatch(Frame& F1, Frame& F2, std::vector<DMatch>& vMatches12) {
        vMatches12.clear();
        const int n2 = (int)F2.N;
        // only queries holding a landmark that is not an outlier can yield a
        // match (matcher.cpp:70-74): kNN-2 runs on those, in query order
        std::vector<int> qi;
        for (size_t i = 0; i < F1.N; i++)
            if (F1.GetLandmark(i) && !F1.IsOutlier(i)) qi.push_back((int)i);
        const int nq = (int)qi.size();
        std::vector<uint8_t> qd(32 * (size_t)std::max(nq, 1));
        for (int k = 0; k < nq; k++) std::memcpy(&qd[32 * (size_t)k], &F1.mDescriptors[32 * (size_t)qi[k]], 32);
        std::vector<int32_t> idx(2 * (size_t)std::max(nq, 1)), dist(2 * (size_t)std::max(nq, 1));
        Check(odo_knn2_hamming(detail::shared_ctx(), qd.data(), nq, F2.mDescriptors.data(), n2, idx.data(),
                               dist.data()),
              "Matcher::KnnMatch");
        for (int k = 0; k < nq; k++) {
            // a missing second neighbour counts as distance INT_MAX
            if (idx[2 * k] < 0) continue;
            const float d0 = (float)dist[2 * k], d1 = (float)dist[2 * k + 1];
            if (!(d0 < mfNNratio * d1)) continue;
            const size_t i1 = qi[k], i2 = idx[2 * k];
            LandmarkPtr lm = F1.GetLandmark(i1);
            if (F2.GetLandmark(i2) && F2.GetLandmark(i2)->Observations() > 0) continue;
            F2.AddLandmark(lm, i2);
            F2.SetOutlier(i2);
            vMatches12.push_back(DMatch{(int32_t)i1, (int32_t)i2, 0, d0});
        }
        return vMatches12.size();
    }

    // Tracking::SearchLocalLMs + Matcher::ProjectionMatch(pFrame, vpLandmarks, th)
    // (tracking.cpp:368-405, matcher.cpp:90-145): landmarks already in the
    // frame's slots are skipped (mnLastFrameSeen), the rest get isInFrustum at
    // the frame's pose (frame.cpp:100-133; mbTrackInView / mTrackProj* set),
    // then the windowed best / second-best search with the same-level ratio
    // test in landmark order on the GPU. Matches go into the frame's slots
    // (AddLandmark); returns their number.
    size_t ProjectionMatch(Frame* pFrame, const std::vector<LandmarkPtr>& vpLandmarks, const float th = 3.0f) {
        const int n = (int)pFrame->N, nL = (int)vpLandmarks.size();
        std::vector<odo_landmark> lms(std::max(nL, 1));
        for (int i = 0; i < nL; i++) {
            const Landmark& L = *vpLandmarks[i];
            odo_landmark& o = lms[i];
            std::memcpy(o.X, L.mWorldPos, sizeof(o.X));
            std::memcpy(o.desc, L.mDescriptor, 32);
            o.flags = (L.isBad() ? ODO_LM_BAD : 0) | (L.Observations() > 0 ? ODO_LM_HAS_OBS : 0);
            for (size_t j = 0; j < pFrame->N && !(o.flags & ODO_LM_SEEN); j++)
                if (pFrame->mvpLandmarks[j].get() == vpLandmarks[i].get()) o.flags |= ODO_LM_SEEN;
        }
        std::vector<float> kun(2 * (size_t)std::max(n, 1));
        std::vector<int32_t> oct(std::max(n, 1)), slot_lm(std::max(n, 1));
        std::vector<uint8_t> taken(std::max(n, 1));
        for (int j = 0; j < n; j++) {
            kun[2 * j] = pFrame->mvKeysUn[j].x;
            kun[2 * j + 1] = pFrame->mvKeysUn[j].y;
            oct[j] = pFrame->mvKeysUn[j].octave;
            const LandmarkPtr& lm = pFrame->mvpLandmarks[j];
            taken[j] = lm && lm->Observations() > 0;
        }
        std::vector<float> proj(3 * (size_t)std::max(nL, 1));
        int nm = 0;
        Check(odo_projection_match(detail::geometry_ctx(pFrame->Width(), pFrame->Height()), pFrame->mTcw.data(),
                                   lms.data(), nL, kun.data(), oct.data(), pFrame->mDescriptors.data(), n,
                                   taken.data(), th, mfNNratio, slot_lm.data(), proj.data(), &nm),
              "Matcher::ProjectionMatch");
        for (int i = 0; i < nL; i++) {
            Landmark& L = *vpLandmarks[i];
            if (lms[i].flags & ODO_LM_SEEN) continue;
            L.mbTrackInView = !std::isnan(proj[3 * i]);
            if (L.mbTrackInView) {
                L.mTrackProjX = proj[3 * i];
                L.mTrackProjY = proj[3 * i + 1];
                L.mTrackProjXR = proj[3 * i + 2];
            }
        }
        for (int j = 0; j < n; j++)
            if (slot_lm[j] >= 0) pFrame->AddLandmark(vpLandmarks[slot_lm[j]], j);
        return (size_t)nm;
    }

    // Matcher::DescriptorDistance (matcher.cpp:20-38): bit-count Hamming.
    static double DescriptorDistance(const uint8_t* a, const uint8_t* b) {
        int d = 0;
        for (int k = 0; k < 32; k++) d += __builtin_popcount((unsigned)(a[k] ^ b[k]));
        return d;
    }

    float mfNNratio;
};

// Odometry/ransac.h:13-73.
class Ransac {
public:
    Ransac() : Ransac(200, 20, 3.0f, 4) {}
    Ransac(int iters, unsigned minInlierTh, float maxMahalanobisDist, unsigned sampleSize) {
        SetParameters(iters, minInlierTh, maxMahalanobisDist, sampleSize);
        mP.check_depth = 1;
    }

    void SetParameters(int iters, unsigned minInlierTh, float maxMahalanobisDist, unsigned sampleSize) {
        mP.iterations = iters;
        mP.min_inlier_th = (int32_t)minInlierTh;
        mP.max_mahalanobis = maxMahalanobisDist;
        mP.sample_size = (int32_t)sampleSize;
    }
    void SetIterations(int iters) { mP.iterations = iters; }
    void SetMaxMahalanobisDistance(float dist) { mP.max_mahalanobis = dist; }
    void SetSampleSize(unsigned s) { mP.sample_size = (int32_t)s; }
    void SetInlierThreshold(unsigned th) { mP.min_inlier_th = (int32_t)th; }
    void CheckDepth(bool check) { mP.check_depth = check ? 1 : 0; }

    // Ransac::Iterate(pF1, pF2, m12) (ransac.cpp:155-258): hypotheses drawn
    // from the process rand() stream (advanced by exactly the draws made),
    // evaluated on the GPU; sets rmse, mvInliers, mT12.
    bool Iterate(Frame* pF1, Frame* pF2, const std::vector<DMatch>& m12) {
        // mpSourceCloud / mpTargetCloud (ransac.cpp:161-189): the depth-valid
        // matched points, kept for the GICP refinement of ADAPTIVE_RICP
        mvSourceCloud.clear();
        mvTargetCloud.clear();
        if (m12.size() >= (size_t)mP.min_inlier_th)
            for (const DMatch& m : m12) {
                const Point3f& s = pF1->mvKeys3Dc[m.queryIdx];
                const Point3f& t = pF2->mvKeys3Dc[m.trainIdx];
                if (mP.check_depth && (std::isnan(s.z) || std::isnan(t.z) || s.z <= 0 || t.z <= 0)) continue;
                mvSourceCloud.insert(mvSourceCloud.end(), {s.x, s.y, s.z});
                mvTargetCloud.insert(mvTargetCloud.end(), {t.x, t.y, t.z});
            }
        std::vector<float> x1 = xyz(*pF1), x2 = xyz(*pF2);
        std::vector<DMatch> inl(std::max<size_t>(m12.size(), 1));
        int ninl = 0, ok = 0;
        detail::Globals& g = detail::G();
        odo_ctx* c = detail::shared_ctx();
        std::lock_guard<std::mutex> lk(g.mu);
        Check(odo_ransac(c, m12.data(), (int)m12.size(), x1.data(), (int)pF1->N, x2.data(), (int)pF2->N, &mP, &g.rng,
                         &g.latch, mT12.data(), &rmse, inl.data(), &ninl, &ok),
              "Ransac::Iterate");
        inl.resize(ninl);
        mvInliers = std::move(inl);
        return ok != 0;
    }

    float rmse = 0.f;
    std::vector<DMatch> mvInliers;
    Pose mT12 = Identity();
    std::vector<float> mvSourceCloud, mvTargetCloud;  // n x 3

private:
    static std::vector<float> xyz(const Frame& F) {
        std::vector<float> v(3 * std::max<size_t>(F.N, 1));
        for (size_t i = 0; i < F.N; i++) {
            v[3 * i] = F.mvKeys3Dc[i].x;
            v[3 * i + 1] = F.mvKeys3Dc[i].y;
            v[3 * i + 2] = F.mvKeys3Dc[i].z;
        }
        return v;
    }
    odo_ransac_params mP{};
};

// Odometry/pnpsolver.h: motion-only bundle adjustment of a frame's pose
// against the landmarks in its slots (pnpsolver.cpp:17-190). Every slot with
// a landmark becomes an edge (stereo when mvuRight >= 0), marked inlier at
// edge creation, outlier per the final chi2 round; the pose is updated when
// at least 3 edges exist. Returns the inlier count.
class PnPSolver {
public:
    static int Compute(Frame* pFrame) {
        std::vector<float> Xw, obs;
        std::vector<size_t> idx;
        for (size_t i = 0; i < pFrame->N; i++) {
            LandmarkPtr lm = pFrame->GetLandmark(i);
            if (!lm) continue;
            Xw.insert(Xw.end(), {lm->mWorldPos[0], lm->mWorldPos[1], lm->mWorldPos[2]});
            obs.insert(obs.end(), {pFrame->mvKeysUn[i].x, pFrame->mvKeysUn[i].y, pFrame->mvuRight[i]});
            idx.push_back(i);
        }
        const int n = (int)idx.size();
        std::vector<uint8_t> out(std::max(n, 1), 0);
        Pose Tout = pFrame->mTcw;
        int nInliers = 0;
        const odo_calib cal = Calibration();
        if (n == 0) {
            Xw.resize(3);
            obs.resize(3);
        }
        Check(odo_pnp_motion_ba(detail::shared_ctx(), Xw.data(), obs.data(), n, &cal, pFrame->mTcw.data(),
                                Tout.data(), out.data(), &nInliers),
              "PnPSolver::Compute");
        for (int k = 0; k < n; k++) {
            if (out[k])
                pFrame->SetOutlier(idx[k]);
            else
                pFrame->SetInlier(idx[k]);
        }
        pFrame->SetPose(Tout);
        return nInliers;
    }
};

// Odometry/pnpransac.h: cv::solvePnPRansac over the frame's landmark
// observations (pnpransac.cpp:11-51): fewer than 10 returns 0; on success the
// pose is set and the RANSAC inliers are marked; a failed solve, where the
// reference prints "PnPRansac fail" and calls terminate(), throws.
class PnPRansac {
public:
    int Compute(Frame& frame) {
        std::vector<float> v3D, v2D;
        std::vector<size_t> vnIndex;
        for (size_t i = 0; i < frame.N; ++i) {
            LandmarkPtr lm = frame.GetLandmark(i);
            if (!lm) continue;
            v3D.insert(v3D.end(), {lm->mWorldPos[0], lm->mWorldPos[1], lm->mWorldPos[2]});
            v2D.insert(v2D.end(), {frame.mvKeysUn[i].x, frame.mvKeysUn[i].y});
            vnIndex.push_back(i);
        }
        const int n = (int)vnIndex.size();
        if (n < 10) return 0;
        const odo_calib cal = Calibration();
        odo_pnp_ransac_result r;
        std::vector<uint8_t> inl(n, 0);
        Check(odo_pnp_ransac(detail::shared_ctx(), v3D.data(), v2D.data(), n, &cal, 500, 3.0f, 0.85, &r, inl.data(),
                             nullptr),
              "PnPRansac::Compute");
        // ok = -1: cv::solvePnP's DLT start throws (CV_Assert(count >= 6)),
        // uncaught in PnPRansac::Compute; ok = 0: "PnPRansac fail" + terminate()
        if (r.ok < 0) throw std::runtime_error("cv::solvePnP: CV_Assert(count >= 6) in cvFindExtrinsicCameraParams2");
        if (!r.ok) throw std::runtime_error("PnPRansac fail");
        Pose T;
        std::copy(r.Tcw, r.Tcw + 16, T.begin());
        frame.SetPose(T);
        for (int k = 0; k < n; ++k)
            if (inl[k]) frame.SetInlier(vnIndex[k]);
        return r.n_inliers;
    }
};

// Odometry/generalizedicp.h: GeneralizedICP(iters, maxCorrespondenceDist)
// (generalizedicp.cpp:11-22; Odometry builds it with (10, 0.07)) and
// Compute(source, target, guess) (generalizedicp.cpp:30-39, 65-89) over n x 3
// clouds: mT12 = the final transformation when converged, identity otherwise.
class GeneralizedICP {
public:
    GeneralizedICP() : GeneralizedICP(15, 0.05) {}
    GeneralizedICP(int iters, double maxCorrespondenceDist) : mIters(iters), mDist(maxCorrespondenceDist) {}
    bool Compute(const std::vector<float>& source, const std::vector<float>& target, const Pose& guess) {
        if (source.size() % 3 || target.size() % 3) throw std::invalid_argument("GeneralizedICP::Compute: sizes");
        int converged = 0, iters = 0, ncorr = 0;
        Check(odo_gicp(detail::shared_ctx(), source.data(), (int)(source.size() / 3), target.data(),
                       (int)(target.size() / 3), guess.data(), mIters, mDist, mT12.data(), &converged, &iters, &ncorr),
              "GeneralizedICP::Compute");
        return converged != 0;
    }
    void SetMaximumIterations(int iters) { mIters = iters; }
    void SetMaxCorrespondenceDistance(double dist) { mDist = dist; }

    Pose mT12 = Identity();

private:
    int mIters;
    double mDist;
};

// Odometry/odometry.h: the pose back-end dispatcher (odometry.cpp:10-117).
// ADAPTIVE_RBA is the reference's (System/tracking.cpp); ADAPTIVE_RICP refines
// a weak RANSAC with GICP on RANSAC's matched clouds; ICP is "not implemented
// yet" in the reference and does nothing here either.
class Odometry {
public:
    enum eAlgorithm { RANSAC = 0, ICP, MOTION_ONLY_BA, ADAPTIVE_RICP, ADAPTIVE_RBA };

    explicit Odometry(eAlgorithm algorithm)
        : mRansac(200, 20, 3.0f, 4), mGicp(10, 0.07), mOdometryAlgorithm(algorithm) {}

    void Compute(Frame* pF1, Frame* pF2, const std::vector<DMatch>& vMatches12) {
        switch (mOdometryAlgorithm) {
        case ADAPTIVE_RICP: {  // odometry.cpp:46-78
            mRansac.Iterate(pF1, pF2, vMatches12);
            Pose T12 = mRansac.mT12;
            if (mRansac.mvInliers.size() < 20 || mRansac.rmse * 10.0f >= 7.0f) {
                if (mRansac.rmse * 10.0f >= 20)
                    T12 = mGicp.Compute(mRansac.mvSourceCloud, mRansac.mvTargetCloud, Identity()) ? mGicp.mT12
                                                                                                 : Identity();
                else
                    T12 = mGicp.Compute(mRansac.mvSourceCloud, mRansac.mvTargetCloud, mRansac.mT12) ? mGicp.mT12
                                                                                                   : mRansac.mT12;
            }
            pF2->SetPose(Mul(T12, pF1->GetPose()));
            for (const DMatch& m : mRansac.mvInliers) pF2->SetInlier((size_t)m.trainIdx);
            break;
        }
        case RANSAC:  // odometry.cpp:81-92
            mRansac.Iterate(pF1, pF2, vMatches12);
            pF2->SetPose(Mul(mRansac.mT12, pF1->GetPose()));
            for (const DMatch& m : mRansac.mvInliers) pF2->SetInlier((size_t)m.trainIdx);
            break;
        case ICP:  // odometry.cpp:95-97
            break;
        case MOTION_ONLY_BA:  // odometry.cpp:100-102
            PnPSolver::Compute(pF2);
            break;
        case ADAPTIVE_RBA:  // odometry.cpp:105-116
            mRansac.Iterate(pF1, pF2, vMatches12);
            pF2->SetPose(Mul(mRansac.mT12, pF1->GetPose()));
            PnPSolver::Compute(pF2);
            break;
        }
    }

    Ransac mRansac;
    GeneralizedICP mGicp;

private:
    eAlgorithm mOdometryAlgorithm;
};

// Odometry/kabsch.h: Compute(setA, setB) for n x 3 row-major point sets.
class Kabsch {
public:
    Pose Compute(const std::vector<float>& setA, const std::vector<float>& setB) {
        if (setA.size() != setB.size() || setA.size() % 3) throw std::invalid_argument("Kabsch::Compute: sizes");
        Check(odo_kabsch(setA.data(), setB.data(), (int)(setA.size() / 3), mTransformation.data()), "Kabsch::Compute");
        return mTransformation;
    }

private:
    Pose mTransformation = Identity();
};

}  // namespace odo_hip

#endif  // ODO_FRONTEND_HPP
