// orbslam2_amd_shim.hpp — header-only C++ layer between the reference's class surfaces and the
// C-ABI of liborbslam2_amd (include/orbslam2_amd.h).
//
// The reference's hot-path methods become one-line calls into these templates; they are written
// against the member names the reference's own types expose (cv::Mat / cv::KeyPoint, Frame,
// KeyFrame, MapPoint, Map), so the same code compiles against the real OpenCV / ORB-SLAM2 types
// (include/dropin/*.h) and against the mock types of tests/cpp/shim_caller.cpp, which is how it is
// tested here (OpenCV is not installed in this container).
//
//   Extractor                 ORBextractor (R/include/ORBextractor.h:45-123): ctor, operator()
//                             (R/src/ORBextractor.cpp:1120-1188), the inline getters, mvImagePyramid
//   Matcher                   ORBmatcher (R/include/ORBmatcher.h:37-143): DescriptorDistance
//                             (R/src/ORBmatcher.cpp:1901-1917), SearchForInitialization (:499-617),
//                             SearchByProjection(Frame&, const Frame&, th, bMono) (:1564-1718) and
//                             SearchByProjection(Frame&, const vector<MapPoint*>&, th) (:63-163),
//                             SearchForTriangulation (:785-983), Fuse(pKF, vpMapPoints, th)
//                             (:995-1154), SearchByBoW(pKF, F, ...) (:220-372) and
//                             SearchByBoW(pKF1, pKF2, ...) (:632-760)
//   ComputeStereoMatches      Frame::ComputeStereoMatches (R/src/Frame.cpp:551-770)
//   PoseOptimization          Optimizer::PoseOptimization (R/src/Optimizer.cpp:306-535)
//   LocalBundleAdjustment     Optimizer::LocalBundleAdjustment (R/include/Optimizer.h:45,
//                             R/src/Optimizer.cpp:564-918): graph gathering, lba_solve (or, given a
//                             device list, lba_group_solve over several GPUs), write-back
//
// Errors: the reference's methods have no error returns, so a negative ORB_E* status becomes a
// std::runtime_error here (there is no CPU fallback: without a gfx950 device the constructors
// throw).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <utility>
#include <vector>

#include "orbslam2_amd.h"

namespace orbslam2_amd {

inline int check(int rc, const char* what) {
    if (rc < 0) throw std::runtime_error(std::string("liborbslam2_amd: ") + what + " failed (" + std::to_string(rc) + ")");
    return rc;
}

constexpr int kCV_8U = 0, kCV_32F = 5;   // OpenCV type codes (stable since OpenCV 2.x)

// ======================================================================= ORBextractor
class Extractor {
public:
    Extractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST, int device = 0,
              int max_w = 2048, int max_h = 2048)
        : nlevels_(nlevels), scaleFactor_(scaleFactor) {
        orb_extractor_params p{nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST};
        check(orb_extractor_create(&p, device, max_w, max_h, 1, &h_), "orb_extractor_create");
        scale_.resize(nlevels);
        inv_.resize(nlevels);
        sig2_.resize(nlevels);
        invSig2_.resize(nlevels);
        check(orb_extractor_scale_tables(h_, scale_.data(), inv_.data(), sig2_.data(), invSig2_.data()),
              "orb_extractor_scale_tables");
    }
    ~Extractor() { orb_extractor_destroy(h_); }
    Extractor(const Extractor&) = delete;
    Extractor& operator=(const Extractor&) = delete;

    orb_extractor* handle() const { return h_; }
    int GetLevels() const { return nlevels_; }
    float GetScaleFactor() const { return scaleFactor_; }
    std::vector<float> GetScaleFactors() const { return scale_; }
    std::vector<float> GetInverseScaleFactors() const { return inv_; }
    std::vector<float> GetScaleSigmaSquares() const { return sig2_; }
    std::vector<float> GetInverseScaleSigmaSquares() const { return invSig2_; }

    // operator()(image, mask (ignored, as in the reference), keypoints, descriptors).  Image: 8-bit
    // single channel with .data / .cols / .rows / .step; KeyPoint: the 28-byte cv::KeyPoint layout;
    // Desc: .create(rows, cols, type) / .release() / .data.  An empty image returns leaving the
    // outputs untouched (R/src/ORBextractor.cpp:1123-1124).
    template <class Img, class KP, class Desc>
    void extract(const Img& image, std::vector<KP>& keypoints, Desc& descriptors) {
        static_assert(sizeof(KP) == sizeof(orb_keypoint), "KeyPoint must have the cv::KeyPoint layout");
        if (image.data == nullptr || image.cols <= 0 || image.rows <= 0) return;
        int cap = 0, n = 0;
        check(orb_extractor_geometry(h_, image.cols, image.rows, nullptr, nullptr, nullptr, &cap), "orb_extractor_geometry");
        std::vector<orb_keypoint> k((size_t)cap);
        std::vector<uint8_t> d((size_t)cap * 32);
        const int rc = orb_extract(h_, image.data, image.cols, image.rows, static_cast<size_t>(image.step), k.data(),
                                   d.data(), cap, &n);
        check(rc, "orb_extract");
        keypoints.resize((size_t)n);
        if (n) std::memcpy(static_cast<void*>(keypoints.data()), k.data(), (size_t)n * sizeof(orb_keypoint));
        if (n == 0) {
            descriptors.release();
        } else {
            descriptors.create(n, 32, kCV_8U);
            std::memcpy(descriptors.data, d.data(), (size_t)n * 32);
        }
        pyramidValid_ = false;
    }

    // mvImagePyramid (R/include/ORBextractor.h:88): host views of the last call's levels, valid
    // until the next extraction (Frame::ComputeStereoMatches reads them, R/src/Frame.cpp:558-695;
    // the on-device orb_compute_stereo_matches avoids the download altogether).
    struct Level {
        const uint8_t* data;
        int cols, rows;
        size_t step;
    };
    const std::vector<Level>& pyramid() {
        if (!pyramidValid_) {
            levels_.assign((size_t)nlevels_, Level{nullptr, 0, 0, 0});
            for (int l = 0; l < nlevels_; l++) {
                Level& L = levels_[(size_t)l];
                check(orb_pyramid_level(h_, 0, l, &L.data, &L.cols, &L.rows, &L.step), "orb_pyramid_level");
            }
            pyramidValid_ = true;
        }
        return levels_;
    }

private:
    orb_extractor* h_ = nullptr;
    int nlevels_;
    float scaleFactor_;
    std::vector<float> scale_, inv_, sig2_, invSig2_;
    std::vector<Level> levels_;
    bool pyramidValid_ = false;
};

// ======================================================================= ORBmatcher
// A Frame's (or KeyFrame's) matcher view: mvKeysUn split into arrays (built once per call),
// mDescriptors, mvuRight and the grid bounds (R/include/Frame.h: mnMinX .. mfGridElementHeightInv;
// R/include/KeyFrame.h:199-206 keeps the same names as const members).
template <class FrameT>
struct FrameView {
    std::vector<float> x, y, ang;
    std::vector<int32_t> oct;
    orb_frame_view v{};
    explicit FrameView(const FrameT& F) {
        const size_t n = F.mvKeysUn.size();
        x.resize(n); y.resize(n); ang.resize(n); oct.resize(n);
        for (size_t i = 0; i < n; i++) {
            const auto& k = F.mvKeysUn[i];
            x[i] = k.pt.x; y[i] = k.pt.y; ang[i] = k.angle; oct[i] = k.octave;
        }
        v.n = (int)n;
        v.x = x.data(); v.y = y.data(); v.angle = ang.data(); v.octave = oct.data();
        v.desc = F.mDescriptors.data;
        v.uright = F.mvuRight.empty() ? nullptr : F.mvuRight.data();
        // static members of Frame, const members of KeyFrame: both read through the object
        v.min_x = (float)F.mnMinX; v.min_y = (float)F.mnMinY; v.max_x = (float)F.mnMaxX; v.max_y = (float)F.mnMaxY;
        v.grid_w_inv = F.mfGridElementWidthInv; v.grid_h_inv = F.mfGridElementHeightInv;
    }
};

// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned int>>) as the C-ABI's arrays: node
// ids ascending (map order), CSR starts, feature indices in insertion order.
template <class FV>
struct FeatVecArrays {
    std::vector<uint32_t> nodes;
    std::vector<int32_t> start{0}, fidx;
    explicit FeatVecArrays(const FV& fv) {
        for (const auto& kv : fv) {
            nodes.push_back((uint32_t)kv.first);
            for (const auto i : kv.second) fidx.push_back((int32_t)i);
            start.push_back((int32_t)fidx.size());
        }
    }
    int n() const { return (int)nodes.size(); }
};

namespace detail {
template <class MatT>
inline void read_Tcw(const MatT& T, float out[16]) {
    for (int r = 0; r < 4; r++)
        for (int k = 0; k < 4; k++) out[4 * r + k] = T.template at<float>(r, k);
}
template <class MatT>
inline MatT make_mat(int rows, int cols, const float* v) {   // cv::Mat(rows, cols, CV_32F)
    MatT m(rows, cols, kCV_32F);
    for (int r = 0; r < rows; r++)
        for (int k = 0; k < cols; k++) m.template at<float>(r, k) = v[cols * r + k];
    return m;
}
// cv::Mat float products R*x + t (3x3 * 3x1 + 3x1) as OpenCV's GEMM evaluates CV_32F: dot products
// accumulated in double, rounded to float once (the oracle's convention, oracle/orb_oracle.c)
inline void rx_plus_t(const float R[9], const float x[3], const float t[3], float out[3]) {
    for (int r = 0; r < 3; r++)
        out[r] = (float)((double)R[3 * r] * x[0] + (double)R[3 * r + 1] * x[1] + (double)R[3 * r + 2] * x[2] +
                         (double)t[r]);
}
template <class MatT>
inline void read_vec3(const MatT& m, float out[3]) {
    for (int k = 0; k < 3; k++) out[k] = m.template at<float>(k, 0);
}
template <class MatT>
inline void read_mat33(const MatT& m, float out[9]) {
    for (int r = 0; r < 3; r++)
        for (int k = 0; k < 3; k++) out[3 * r + k] = m.template at<float>(r, k);
}
// Ow = -Rcw^T tcw of rows 0..2 of a pose (OpenCV float GEMM: double accumulation, one rounding)
inline void camera_center(const float T[12], float Ow[3]) {
    for (int k = 0; k < 3; k++)
        Ow[k] = (float)(-((double)T[k] * T[3] + (double)T[4 + k] * T[7] + (double)T[8 + k] * T[11]));
}
// Scw = [sR | st] -> Tcw = [R | t] and Ow = -R^T t as R/src/ORBmatcher.cpp:382-386 / :1172-1176 derive
// them: scw = sqrt(row 0 . row 0) (dot accumulated in double, the root rounded to float), every
// element x / scw as x * (1.0 / scw) rounded once, then the camera centre
template <class MatT>
inline void decompose_scw(const MatT& Scw, float Tcw[12], float Ow[3]) {
    double ss = 0.0;
    for (int k = 0; k < 3; k++) {
        const double v = Scw.template at<float>(0, k);
        ss += v * v;
    }
    const float scw = (float)std::sqrt(ss);
    const double inv = 1.0 / (double)scw;
    for (int r = 0; r < 3; r++)
        for (int k = 0; k < 4; k++) Tcw[4 * r + k] = (float)((double)Scw.template at<float>(r, k) * inv);
    camera_center(Tcw, Ow);
}
// orb_kf_params of a keyframe (ORBmatcher::Fuse reads GetPose, GetCameraCenter, the intrinsics
// and the scale tables, R/src/ORBmatcher.cpp:997-1006)
template <class KeyFrameT>
struct KfParams {
    orb_kf_params p{};
    std::vector<float> sf, isg;
    explicit KfParams(KeyFrameT* pKF) {
        const auto T = pKF->GetPose();
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 4; k++) p.Tcw[4 * r + k] = T.template at<float>(r, k);
        read_vec3(pKF->GetCameraCenter(), p.Ow);
        p.fx = pKF->fx; p.fy = pKF->fy; p.cx = pKF->cx; p.cy = pKF->cy; p.bf = pKF->mbf;
        p.log_scale_factor = pKF->mfLogScaleFactor;
        p.n_levels = pKF->mnScaleLevels;
        sf.assign(pKF->mvScaleFactors.begin(), pKF->mvScaleFactors.end());
        isg.assign(pKF->mvInvLevelSigma2.begin(), pKF->mvInvLevelSigma2.end());
        p.scale_factors = sf.data();
        p.inv_level_sigma2 = isg.data();
    }
};
}  // namespace detail

class Matcher {
public:
    explicit Matcher(float nnratio = 0.6f, bool checkOri = true, int device = 0)
        : nnratio_(nnratio), checkOri_(checkOri), device_(device) {
        check(orb_matcher_create(device, nnratio, checkOri ? 1 : 0, &h_), "orb_matcher_create");
    }
    ~Matcher() { orb_matcher_destroy(h_); }
    Matcher(const Matcher&) = delete;
    Matcher& operator=(const Matcher&) = delete;
    orb_matcher* handle() const { return h_; }

    static int DescriptorDistance(const uint8_t* a, const uint8_t* b) { return orb_descriptor_distance(a, b); }

    // SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize): vbPrevMatched holds
    // cv::Point2f (two floats) per F1 keypoint and is updated with the matched positions.
    template <class FrameT, class P2f>
    int SearchForInitialization(FrameT& F1, FrameT& F2, std::vector<P2f>& vbPrevMatched, std::vector<int>& vnMatches12,
                                int windowSize = 10) {
        static_assert(sizeof(P2f) == 2 * sizeof(float), "Point2f layout");
        FrameView<FrameT> a(F1), b(F2);
        vnMatches12.assign(F1.mvKeysUn.size(), -1);
        vbPrevMatched.resize(F1.mvKeysUn.size());
        return check(orb_search_for_initialization(h_, &a.v, &b.v, reinterpret_cast<float*>(vbPrevMatched.data()),
                                                   vnMatches12.data(), windowSize),
                     "orb_search_for_initialization");
    }

    // SearchByProjection(CurrentFrame, LastFrame, th, bMono) (R :1564-1718, Tracking::TrackWithMotionModel):
    // reads both frames' mTcw, the last frame's mvpMapPoints / mvbOutlier and their GetWorldPos /
    // GetDescriptor / Observations, the current frame's fx..cy, mbf, mb, mvScaleFactors, mvuRight and
    // mvpMapPoints; writes CurrentFrame.mvpMapPoints as the reference does (a slot holding a point
    // without observations may be taken over; the rotation check clears the slots it rejects).
    template <class FrameT>
    int SearchByProjection(FrameT& CurrentFrame, const FrameT& LastFrame, float th, bool bMono) {
        FrameView<FrameT> cur(CurrentFrame), last(LastFrame);
        const size_t nc = CurrentFrame.mvKeysUn.size(), nl = LastFrame.mvKeysUn.size();
        float Tc[12], Tl[12];
        detail_read_T34(CurrentFrame.mTcw, Tc);
        detail_read_T34(LastFrame.mTcw, Tl);
        std::vector<int32_t> has(nl, 0), slots(nc, -1);
        std::vector<uint8_t> outl(nl, 0), desc(nl * 32, 0);
        std::vector<float> xyz(nl * 3, 0.f);
        for (size_t i = 0; i < nl; i++) {
            auto mp = LastFrame.mvpMapPoints[i];   // MapPoint* (the vector is const, the points are not)
            if (!mp) continue;
            has[i] = mp->Observations() > 0 ? 1 : 2;
            outl[i] = LastFrame.mvbOutlier[i] ? 1 : 0;
            const auto X = mp->GetWorldPos();
            for (int k = 0; k < 3; k++) xyz[3 * i + (size_t)k] = X.template at<float>(k, 0);
            const auto d = mp->GetDescriptor();
            std::memcpy(&desc[32 * i], d.data, 32);
        }
        for (size_t i = 0; i < nc; i++)
            if (CurrentFrame.mvpMapPoints[i]) slots[i] = CurrentFrame.mvpMapPoints[i]->Observations() > 0 ? -2 : -3;
        const float cam[6] = {FrameT::fx, FrameT::fy, FrameT::cx, FrameT::cy, CurrentFrame.mbf, CurrentFrame.mb};
        const int n = check(orb_search_by_projection_frame(h_, &cur.v, Tc, &last.v, Tl, has.data(), outl.data(), xyz.data(),
                                                           desc.data(), CurrentFrame.mvScaleFactors.data(), cam, th,
                                                           bMono ? 1 : 0, slots.data()),
                            "orb_search_by_projection_frame");
        for (size_t i = 0; i < nc; i++) {
            if (slots[i] >= 0) CurrentFrame.mvpMapPoints[i] = LastFrame.mvpMapPoints[(size_t)slots[i]];
            else if (slots[i] == -1) CurrentFrame.mvpMapPoints[i] = nullptr;
        }
        return n;
    }

    // SearchByProjection(F, vpMapPoints, th) (R :63-163, Tracking::SearchLocalPoints): reads every
    // point's mbTrackInView / isBad / mTrackProjX / mTrackProjY / mTrackProjXR / mnTrackScaleLevel /
    // mTrackViewCos / GetDescriptor / Observations and F's mvScaleFactors, mvuRight, mvpMapPoints;
    // writes F.mvpMapPoints (later points overwrite earlier ones, as in the reference).
    template <class FrameT, class MapPointT>
    int SearchByProjection(FrameT& F, const std::vector<MapPointT*>& vpMapPoints, float th = 3) {
        FrameView<FrameT> f(F);
        const size_t nm = vpMapPoints.size(), nf = F.mvKeysUn.size();
        std::vector<uint8_t> inView(nm, 0), hasObs(nm, 0), desc(nm * 32, 0);
        std::vector<float> proj(nm * 3, 0.f), vcos(nm, 0.f);
        std::vector<int32_t> level(nm, 0), slots(nf, -1);
        for (size_t i = 0; i < nm; i++) {
            MapPointT* pMP = vpMapPoints[i];
            if (!pMP->mbTrackInView || pMP->isBad()) continue;
            inView[i] = 1;
            proj[3 * i] = pMP->mTrackProjX;
            proj[3 * i + 1] = pMP->mTrackProjY;
            proj[3 * i + 2] = pMP->mTrackProjXR;
            level[i] = pMP->mnTrackScaleLevel;
            vcos[i] = pMP->mTrackViewCos;
            hasObs[i] = pMP->Observations() > 0 ? 1 : 0;
            const auto d = pMP->GetDescriptor();
            std::memcpy(&desc[32 * i], d.data, 32);
        }
        for (size_t i = 0; i < nf; i++)
            if (F.mvpMapPoints[i]) slots[i] = F.mvpMapPoints[i]->Observations() > 0 ? -2 : -3;
        const int n = check(orb_search_by_projection_local(h_, &f.v, (int)nm, inView.data(), proj.data(), level.data(),
                                                           vcos.data(), desc.data(), hasObs.data(),
                                                           F.mvScaleFactors.data(), th, slots.data()),
                            "orb_search_by_projection_local");
        for (size_t i = 0; i < nf; i++)
            if (slots[i] >= 0) F.mvpMapPoints[i] = vpMapPoints[(size_t)slots[i]];
        return n;
    }

    // SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo) (R :785-983,
    // LocalMapping::CreateNewMapPoints, R/src/LocalMapping.cpp:374): the epipole (:791-797) from
    // pKF1->GetCameraCenter() and pKF2's GetRotation / GetTranslation / intrinsics, both keyframes'
    // mFeatVec, GetMapPoint(i) occupancy, pKF2's mvScaleFactors / mvLevelSigma2; vMatchedPairs in
    // KF1 index order (:975-981).
    template <class KeyFrameT, class MatT>
    int SearchForTriangulation(KeyFrameT* pKF1, KeyFrameT* pKF2, const MatT& F12,
                               std::vector<std::pair<size_t, size_t>>& vMatchedPairs, bool bOnlyStereo) {
        FrameView<KeyFrameT> a(*pKF1), b(*pKF2);
        FeatVecArrays<decltype(pKF1->mFeatVec)> fv1(pKF1->mFeatVec), fv2(pKF2->mFeatVec);
        const size_t n1 = pKF1->mvKeysUn.size(), n2 = pKF2->mvKeysUn.size();
        std::vector<uint8_t> has1(n1), has2(n2);
        for (size_t i = 0; i < n1; i++) has1[i] = pKF1->GetMapPoint(i) ? 1 : 0;
        for (size_t i = 0; i < n2; i++) has2[i] = pKF2->GetMapPoint(i) ? 1 : 0;
        float Cw[3], R2w[9], t2w[3], C2[3], F[9];
        detail::read_vec3(pKF1->GetCameraCenter(), Cw);
        detail::read_mat33(pKF2->GetRotation(), R2w);
        detail::read_vec3(pKF2->GetTranslation(), t2w);
        detail::rx_plus_t(R2w, Cw, t2w, C2);   // C2 = R2w*Cw + t2w
        const float invz = 1.0f / C2[2];
        const float ex = pKF2->fx * C2[0] * invz + pKF2->cx;
        const float ey = pKF2->fy * C2[1] * invz + pKF2->cy;
        detail::read_mat33(F12, F);
        const std::vector<float> sf2(pKF2->mvScaleFactors.begin(), pKF2->mvScaleFactors.end());
        const std::vector<float> s2(pKF2->mvLevelSigma2.begin(), pKF2->mvLevelSigma2.end());
        std::vector<int32_t> m12(n1, -1);
        const int n = check(orb_search_for_triangulation(device_, &a.v, &b.v, has1.data(), has2.data(), fv1.n(),
                                                         fv1.nodes.data(), fv1.start.data(), fv1.fidx.data(), fv2.n(),
                                                         fv2.nodes.data(), fv2.start.data(), fv2.fidx.data(), F, ex, ey,
                                                         sf2.data(), s2.data(), (int)sf2.size(), bOnlyStereo ? 1 : 0,
                                                         checkOri_ ? 1 : 0, m12.data()),
                            "orb_search_for_triangulation");
        vMatchedPairs.clear();
        vMatchedPairs.reserve((size_t)n);
        for (size_t i = 0; i < n1; i++)
            if (m12[i] >= 0) vMatchedPairs.push_back(std::make_pair(i, (size_t)m12[i]));
        return n;
    }

    // Fuse(pKF, vpMapPoints, th) (R :995-1154, LocalMapping::SearchInNeighbors): the matching step of
    // every point on the GPU (orb_fuse), then the replace / add step in vector order on the host.  A
    // point is re-checked there (isBad, IsInKeyFrame) because an earlier iteration of the reference
    // loop may have replaced it or added it to pKF, which makes the reference skip it (:1011-1014);
    // pKF->GetMapPoint(bestIdx) is likewise read at that point of the loop.  The distances are the
    // raw mfMinDistance / mfMaxDistance, read through MapPoint::GetDistances (a
    // one-line accessor the drop-in adds to MapPoint; the kernel applies the 0.8 / 1.2 invariance).
    template <class KeyFrameT, class MapPointT>
    int Fuse(KeyFrameT* pKF, const std::vector<MapPointT*>& vpMapPoints, const float th = 3.0f) {
        FrameView<KeyFrameT> kv(*pKF);
        detail::KfParams<KeyFrameT> kp(pKF);
        const size_t n = vpMapPoints.size();
        std::vector<uint8_t> valid(n, 0), desc(n * 32, 0);
        std::vector<float> xyz(3 * n, 0.f), nrm(3 * n, 0.f), mind(n, 0.f), maxd(n, 0.f);
        for (size_t i = 0; i < n; i++) {
            MapPointT* pMP = vpMapPoints[i];
            if (!pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
            valid[i] = 1;
            detail::read_vec3(pMP->GetWorldPos(), &xyz[3 * i]);
            detail::read_vec3(pMP->GetNormal(), &nrm[3 * i]);
            pMP->GetDistances(mind[i], maxd[i]);
            const auto d = pMP->GetDescriptor();
            std::memcpy(&desc[32 * i], d.data, 32);
        }
        std::vector<int32_t> bi(n, -1), bd(n, 256);
        if (n)
            check(orb_fuse(device_, &kv.v, &kp.p, (int)n, valid.data(), xyz.data(), nrm.data(), mind.data(), maxd.data(),
                           desc.data(), th, bi.data(), bd.data()),
                  "orb_fuse");
        int nFused = 0;
        for (size_t i = 0; i < n; i++) {
            if (bi[i] < 0) continue;   // bestDist > TH_LOW (or no candidate)
            MapPointT* pMP = vpMapPoints[i];
            if (pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
            const size_t bestIdx = (size_t)bi[i];
            MapPointT* pMPinKF = pKF->GetMapPoint(bestIdx);
            if (pMPinKF) {   // :1123-1136
                if (!pMPinKF->isBad()) {
                    if (pMPinKF->Observations() > pMP->Observations()) pMP->Replace(pMPinKF);
                    else pMPinKF->Replace(pMP);
                }
            } else {         // :1137-1141
                pMP->AddObservation(pKF, bestIdx);
                pKF->AddMapPoint(pMP, bestIdx);
            }
            nFused++;
        }
        return nFused;
    }

    // SearchByBoW(pKF, F, vpMapPointMatches) (R :220-372, Tracking::TrackReferenceKeyFrame /
    // Relocalization): vpMapPointMatches = F.N NULLs, then the keyframe's map point for every match.
    template <class KeyFrameT, class FrameT, class MapPointT>
    int SearchByBoW(KeyFrameT* pKF, FrameT& F, std::vector<MapPointT*>& vpMapPointMatches) {
        const std::vector<MapPointT*> vpMapPointsKF = pKF->GetMapPointMatches();
        FrameView<KeyFrameT> kv(*pKF);
        FrameView<FrameT> fv(F);
        FeatVecArrays<decltype(pKF->mFeatVec)> a(pKF->mFeatVec);
        FeatVecArrays<decltype(F.mFeatVec)> b(F.mFeatVec);
        std::vector<uint8_t> ok(vpMapPointsKF.size());
        for (size_t i = 0; i < ok.size(); i++) ok[i] = vpMapPointsKF[i] && !vpMapPointsKF[i]->isBad() ? 1 : 0;
        const size_t nf = F.mvKeysUn.size();
        vpMapPointMatches = std::vector<MapPointT*>(nf, static_cast<MapPointT*>(nullptr));
        std::vector<int32_t> mf(nf, -1);
        const int n = check(orb_search_by_bow_frame(device_, &kv.v, ok.data(), a.n(), a.nodes.data(), a.start.data(),
                                                    a.fidx.data(), &fv.v, b.n(), b.nodes.data(), b.start.data(),
                                                    b.fidx.data(), nnratio_, checkOri_ ? 1 : 0, mf.data()),
                            "orb_search_by_bow_frame");
        for (size_t j = 0; j < nf; j++)
            if (mf[j] >= 0) vpMapPointMatches[j] = vpMapPointsKF[(size_t)mf[j]];
        return n;
    }

    // SearchByBoW(pKF1, pKF2, vpMatches12) (R :632-760, LoopClosing::ComputeSim3).
    template <class KeyFrameT, class MapPointT>
    int SearchByBoW(KeyFrameT* pKF1, KeyFrameT* pKF2, std::vector<MapPointT*>& vpMatches12) {
        const std::vector<MapPointT*> vp1 = pKF1->GetMapPointMatches(), vp2 = pKF2->GetMapPointMatches();
        FrameView<KeyFrameT> k1(*pKF1), k2(*pKF2);
        FeatVecArrays<decltype(pKF1->mFeatVec)> a(pKF1->mFeatVec), b(pKF2->mFeatVec);
        std::vector<uint8_t> ok1(vp1.size()), ok2(vp2.size());
        for (size_t i = 0; i < vp1.size(); i++) ok1[i] = vp1[i] && !vp1[i]->isBad() ? 1 : 0;
        for (size_t i = 0; i < vp2.size(); i++) ok2[i] = vp2[i] && !vp2[i]->isBad() ? 1 : 0;
        vpMatches12 = std::vector<MapPointT*>(vp1.size(), static_cast<MapPointT*>(nullptr));
        std::vector<int32_t> m12(vp1.size(), -1);
        const int n = check(orb_search_by_bow_kf(device_, &k1.v, ok1.data(), a.n(), a.nodes.data(), a.start.data(),
                                                 a.fidx.data(), &k2.v, ok2.data(), b.n(), b.nodes.data(), b.start.data(),
                                                 b.fidx.data(), nnratio_, checkOri_ ? 1 : 0, m12.data()),
                            "orb_search_by_bow_kf");
        for (size_t i = 0; i < vp1.size(); i++)
            if (m12[i] >= 0) vpMatches12[i] = vp2[(size_t)m12[i]];
        return n;
    }

    // SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (R :1719-1800,
    // Tracking::Relocalization): pKF->GetMapPointMatches() minus NULL, bad and sAlreadyFound points;
    // the frame's mTcw (Ow = -Rcw^T tcw, :1723-1725), fx .. cy, mfLogScaleFactor, mnScaleLevels,
    // mvScaleFactors; CurrentFrame.mvpMapPoints gains the keyframe's point in every slot this call
    // matched (slots already set are never taken; the rotation check's rejects stay NULL).
    template <class FrameT, class KeyFrameT, class MapPointT>
    int SearchByProjection(FrameT& CurrentFrame, KeyFrameT* pKF, const std::set<MapPointT*>& sAlreadyFound,
                           const float th, const int ORBdist) {
        const std::vector<MapPointT*> vpMPs = pKF->GetMapPointMatches();
        FrameView<FrameT> cur(CurrentFrame);
        FrameView<KeyFrameT> kv(*pKF);
        const size_t n = vpMPs.size(), nc = CurrentFrame.mvKeysUn.size();
        std::vector<uint8_t> valid(n, 0), desc(n * 32, 0);
        std::vector<float> xyz(3 * n, 0.f), mind(n, 0.f), maxd(n, 0.f);
        for (size_t i = 0; i < n; i++) {
            MapPointT* pMP = vpMPs[i];
            if (!pMP || pMP->isBad() || sAlreadyFound.count(pMP)) continue;
            valid[i] = 1;
            detail::read_vec3(pMP->GetWorldPos(), &xyz[3 * i]);
            pMP->GetDistances(mind[i], maxd[i]);
            const auto d = pMP->GetDescriptor();
            std::memcpy(&desc[32 * i], d.data, 32);
        }
        float Tc[12], Ow[3];
        detail_read_T34(CurrentFrame.mTcw, Tc);
        detail::camera_center(Tc, Ow);
        std::vector<int32_t> slots(nc, -1);
        for (size_t i = 0; i < nc; i++)
            if (CurrentFrame.mvpMapPoints[i]) slots[i] = -2;
        const float cam[4] = {CurrentFrame.fx, CurrentFrame.fy, CurrentFrame.cx, CurrentFrame.cy};
        const int nm = check(orb_search_by_projection_kf(h_, &cur.v, Tc, Ow, &kv.v, valid.data(), xyz.data(), mind.data(),
                                                         maxd.data(), desc.data(), cam, CurrentFrame.mfLogScaleFactor,
                                                         CurrentFrame.mnScaleLevels, CurrentFrame.mvScaleFactors.data(),
                                                         th, ORBdist, slots.data()),
                             "orb_search_by_projection_kf");
        for (size_t i = 0; i < nc; i++)
            if (slots[i] >= 0) CurrentFrame.mvpMapPoints[i] = vpMPs[(size_t)slots[i]];
        return nm;
    }

    // SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (R :370-497, LoopClosing::ComputeSim3):
    // Tcw / Ow from Scw as :382-386 (detail::decompose_scw); a point is skipped when bad or already
    // in vpMatched (:390-391); vpMatched[bestIdx] = vpPoints[iMP] for every match (:488-492).
    template <class KeyFrameT, class MatT, class MapPointT>
    int SearchByProjection(KeyFrameT* pKF, const MatT& Scw, const std::vector<MapPointT*>& vpPoints,
                           std::vector<MapPointT*>& vpMatched, int th) {
        FrameView<KeyFrameT> kv(*pKF);
        detail::KfParams<KeyFrameT> kp(pKF);
        detail::decompose_scw(Scw, kp.p.Tcw, kp.p.Ow);
        std::set<MapPointT*> found(vpMatched.begin(), vpMatched.end());
        found.erase(static_cast<MapPointT*>(nullptr));
        const size_t n = vpPoints.size(), nk = vpMatched.size();
        std::vector<uint8_t> valid(n, 0), desc(n * 32, 0);
        std::vector<float> xyz(3 * n, 0.f), nrm(3 * n, 0.f), mind(n, 0.f), maxd(n, 0.f);
        read_points(vpPoints, found, valid, xyz, nrm, mind, maxd, desc);
        std::vector<int32_t> matched(nk, -1);
        for (size_t i = 0; i < nk; i++)
            if (vpMatched[i]) matched[i] = -2;
        const int nm = check(orb_search_by_projection_sim3(h_, &kv.v, &kp.p, (int)n, valid.data(), xyz.data(), nrm.data(),
                                                           mind.data(), maxd.data(), desc.data(), (float)th,
                                                           matched.data()),
                             "orb_search_by_projection_sim3");
        for (size_t i = 0; i < nk; i++)
            if (matched[i] >= 0) vpMatched[i] = vpPoints[(size_t)matched[i]];
        return nm;
    }

    // SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (R :1305-1503): sR12 = s12 R12,
    // sR21 = (1/s12) R12^T, t21 = -sR21 t12 (:1315-1318; scaled elements rounded to float, the product
    // accumulated in double); vbAlreadyMatched1 / 2 from vpMatches12 and GetIndexInKeyFrame(pKF2)
    // (:1327-1349); both keyframes' GetRotation / GetTranslation, scale tables and pKF1's intrinsics;
    // vpMatches12[i1] = pKF2's point for every mutual pair found (:1525-1540).
    template <class KeyFrameT, class MapPointT, class MatT>
    int SearchBySim3(KeyFrameT* pKF1, KeyFrameT* pKF2, std::vector<MapPointT*>& vpMatches12, const float& s12,
                     const MatT& R12, const MatT& t12, const float th) {
        const std::vector<MapPointT*> vp1 = pKF1->GetMapPointMatches(), vp2 = pKF2->GetMapPointMatches();
        const size_t N1 = vp1.size(), N2 = vp2.size();
        std::vector<uint8_t> am1(N1, 0), am2(N2, 0);
        for (size_t i = 0; i < N1; i++) {
            MapPointT* pMP = vpMatches12[i];
            if (!pMP) continue;
            am1[i] = 1;
            const int idx2 = pMP->GetIndexInKeyFrame(pKF2);
            if (idx2 >= 0 && idx2 < (int)N2) am2[(size_t)idx2] = 1;
        }
        float R[9], t[3];
        detail::read_mat33(R12, R);
        detail::read_vec3(t12, t);
        orb_sim3_points p1{}, p2{};
        for (int r = 0; r < 3; r++) {
            double acc = 0.0;
            for (int k = 0; k < 3; k++) {
                const float sr21 = (float)((double)R[3 * k + r] * (1.0 / (double)s12));
                p1.S[4 * r + k] = sr21;
                p2.S[4 * r + k] = (float)((double)R[3 * r + k] * (double)s12);
                acc += (double)sr21 * t[k];
            }
            p1.S[4 * r + 3] = (float)(-acc);
            p2.S[4 * r + 3] = t[r];
        }
        Sim3Side s1(pKF1, vp1, am1, p1), s2(pKF2, vp2, am2, p2);
        FrameView<KeyFrameT> k1(*pKF1), k2(*pKF2);
        const float cam1[4] = {pKF1->fx, pKF1->fy, pKF1->cx, pKF1->cy};
        const orb_scale_params sc1{pKF1->mfLogScaleFactor, pKF1->mnScaleLevels, pKF1->mvScaleFactors.data()};
        const orb_scale_params sc2{pKF2->mfLogScaleFactor, pKF2->mnScaleLevels, pKF2->mvScaleFactors.data()};
        std::vector<int32_t> m12(N1, -1);
        const int n = check(orb_search_by_sim3(device_, &k1.v, &k2.v, &p1, &p2, cam1, &sc1, &sc2, th, m12.data()),
                            "orb_search_by_sim3");
        for (size_t i = 0; i < N1; i++)
            if (m12[i] >= 0) vpMatches12[i] = vp2[(size_t)m12[i]];
        return n;
    }

    // Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (R :1164-1290, LoopClosing::SearchAndFuse): Tcw /
    // Ow from Scw (:1172-1176); a point is skipped when bad or among pKF->GetMapPoints() at entry
    // (:1178, :1190); the matching step on the GPU (orb_fuse_sim3), then in vector order: the
    // keyframe's point in the matched slot, read at that point of the loop, becomes
    // vpReplacePoint[iMP] unless bad, an empty slot receives the point (AddObservation /
    // AddMapPoint); nFused counts both (:1270-1283).
    template <class KeyFrameT, class MatT, class MapPointT>
    int Fuse(KeyFrameT* pKF, const MatT& Scw, const std::vector<MapPointT*>& vpPoints, float th,
             std::vector<MapPointT*>& vpReplacePoint) {
        FrameView<KeyFrameT> kv(*pKF);
        detail::KfParams<KeyFrameT> kp(pKF);
        detail::decompose_scw(Scw, kp.p.Tcw, kp.p.Ow);
        const std::set<MapPointT*> spAlreadyFound = pKF->GetMapPoints();
        const size_t n = vpPoints.size();
        std::vector<uint8_t> valid(n, 0), desc(n * 32, 0);
        std::vector<float> xyz(3 * n, 0.f), nrm(3 * n, 0.f), mind(n, 0.f), maxd(n, 0.f);
        read_points(vpPoints, spAlreadyFound, valid, xyz, nrm, mind, maxd, desc);
        std::vector<int32_t> bi(n, -1), bd(n, 256);
        if (n)
            check(orb_fuse_sim3(device_, &kv.v, &kp.p, (int)n, valid.data(), xyz.data(), nrm.data(), mind.data(),
                                maxd.data(), desc.data(), th, bi.data(), bd.data()),
                  "orb_fuse_sim3");
        int nFused = 0;
        for (size_t i = 0; i < n; i++) {
            if (bi[i] < 0) continue;
            MapPointT* pMP = vpPoints[i];
            const size_t bestIdx = (size_t)bi[i];
            MapPointT* pMPinKF = pKF->GetMapPoint(bestIdx);
            if (pMPinKF) {
                if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
            } else {
                pMP->AddObservation(pKF, bestIdx);
                pKF->AddMapPoint(pMP, bestIdx);
            }
            nFused++;
        }
        return nFused;
    }

private:
    // the per-point arrays of the Scw forms: valid = set, not bad, not in `skip`
    template <class MapPointT>
    static void read_points(const std::vector<MapPointT*>& vp, const std::set<MapPointT*>& skip, std::vector<uint8_t>& valid,
                            std::vector<float>& xyz, std::vector<float>& nrm, std::vector<float>& mind,
                            std::vector<float>& maxd, std::vector<uint8_t>& desc) {
        for (size_t i = 0; i < vp.size(); i++) {
            MapPointT* pMP = vp[i];
            if (!pMP || pMP->isBad() || skip.count(pMP)) continue;
            valid[i] = 1;
            detail::read_vec3(pMP->GetWorldPos(), &xyz[3 * i]);
            detail::read_vec3(pMP->GetNormal(), &nrm[3 * i]);
            pMP->GetDistances(mind[i], maxd[i]);
            const auto d = pMP->GetDescriptor();
            std::memcpy(&desc[32 * i], d.data, 32);
        }
    }
    // one keyframe's side of SearchBySim3 (orb_sim3_points): Tcw, and per slot the point's arrays
    // when set, not bad and not already matched (:1355-1361, :1430-1436)
    struct Sim3Side {
        std::vector<uint8_t> valid, desc;
        std::vector<float> xyz, mind, maxd;
        template <class KeyFrameT, class MapPointT>
        Sim3Side(KeyFrameT* pKF, const std::vector<MapPointT*>& vp, const std::vector<uint8_t>& already, orb_sim3_points& p)
            : valid(vp.size(), 0), desc(vp.size() * 32, 0), xyz(vp.size() * 3, 0.f), mind(vp.size(), 0.f),
              maxd(vp.size(), 0.f) {
            float R[9], t[3];
            detail::read_mat33(pKF->GetRotation(), R);
            detail::read_vec3(pKF->GetTranslation(), t);
            for (int r = 0; r < 3; r++) {
                for (int k = 0; k < 3; k++) p.Tcw[4 * r + k] = R[3 * r + k];
                p.Tcw[4 * r + 3] = t[r];
            }
            for (size_t i = 0; i < vp.size(); i++) {
                MapPointT* pMP = vp[i];
                if (!pMP || already[i] || pMP->isBad()) continue;
                valid[i] = 1;
                detail::read_vec3(pMP->GetWorldPos(), &xyz[3 * i]);
                pMP->GetDistances(mind[i], maxd[i]);
                const auto d = pMP->GetDescriptor();
                std::memcpy(&desc[32 * i], d.data, 32);
            }
            p.n = (int)vp.size();
            p.valid = valid.data(); p.xyz = xyz.data(); p.min_dist = mind.data(); p.max_dist = maxd.data();
            p.desc = desc.data();
        }
    };
    template <class MatT>
    static void detail_read_T34(const MatT& T, float out[12]) {   // rows 0..2 of a 4x4 float cv::Mat
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 4; k++) out[4 * r + k] = T.template at<float>(r, k);
    }
    orb_matcher* h_ = nullptr;
    float nnratio_;
    bool checkOri_;
    int device_;
};

// ======================================================================= Frame::ComputeStereoMatches
// R/src/Frame.cpp:551-770 on the device: reads the two extractors' device pyramids in place (no
// mvImagePyramid download) and F.mvKeys / mvKeysRight / mDescriptors / mDescriptorsRight / mbf /
// mb; writes F.mvuRight and F.mvDepth (N entries, -1 = no stereo match) as :555-556 initialise them.
// left / right = the handles that extracted this frame's images (their last call).
template <class FrameT>
void ComputeStereoMatches(FrameT& F, orb_extractor* left, orb_extractor* right) {
    const size_t N = F.mvKeys.size(), Nr = F.mvKeysRight.size();
    F.mvuRight = std::vector<float>(N, -1.0f);
    F.mvDepth = std::vector<float>(N, -1.0f);
    if (N == 0 || Nr == 0) return;
    static_assert(sizeof(F.mvKeys[0]) == sizeof(orb_keypoint), "KeyPoint must have the cv::KeyPoint layout");
    check(orb_compute_stereo_matches(left, right, reinterpret_cast<const orb_keypoint*>(F.mvKeys.data()),
                                     F.mDescriptors.data, (int)N,
                                     reinterpret_cast<const orb_keypoint*>(F.mvKeysRight.data()),
                                     F.mDescriptorsRight.data, (int)Nr, F.mbf, F.mb, F.mvuRight.data(),
                                     F.mvDepth.data()),
          "orb_compute_stereo_matches");
}

// ======================================================================= Optimizer::PoseOptimization
// R/src/Optimizer.cpp:306-535 (Tracking: every tracked frame, R/src/Tracking.cpp:1030, 1203, 1262,
// 1908): one edge per keypoint with a map point, in keypoint order, gathered under
// MapPoint::mGlobalMutex (:343-429; mvbOutlier[i] = false for each), the four optimize(10) rounds on
// the GPU (pose_optimize_batch, one frame), then mvbOutlier, SetPose and the return value
// nInitialCorrespondences - nBad.  Below 3 edges: return 0, pose untouched (:431-432).
template <class FrameT>
int PoseOptimization(FrameT* pFrame, int device = 0) {
    using MapPointT = typename std::remove_pointer<typename std::decay<decltype(pFrame->mvpMapPoints[0])>::type>::type;
    using MatT = typename std::decay<decltype(pFrame->mTcw)>::type;
    const size_t N = pFrame->mvKeysUn.size();
    std::vector<size_t> idx;
    std::vector<double> obs, xw, info;
    {
        std::unique_lock<std::mutex> lock(MapPointT::mGlobalMutex);
        for (size_t i = 0; i < N; i++) {
            MapPointT* pMP = pFrame->mvpMapPoints[i];
            if (!pMP) continue;
            pFrame->mvbOutlier[i] = false;
            const auto& kp = pFrame->mvKeysUn[i];
            obs.push_back(kp.pt.x);
            obs.push_back(kp.pt.y);
            obs.push_back(pFrame->mvuRight[i]);   // < 0: monocular edge
            float X[3];
            detail::read_vec3(pMP->GetWorldPos(), X);
            xw.insert(xw.end(), {(double)X[0], (double)X[1], (double)X[2]});
            info.push_back((double)pFrame->mvInvLevelSigma2[(size_t)kp.octave]);
            idx.push_back(i);
        }
    }
    const int E = (int)idx.size();
    if (E < 3) return 0;
    float T[16];
    detail::read_Tcw(pFrame->mTcw, T);
    double q[4], t[3], oq[4], ot[3];
    lba_pose_from_Tcw(T, q, t);   // Converter::toSE3Quat
    const double cam[5] = {pFrame->fx, pFrame->fy, pFrame->cx, pFrame->cy, pFrame->mbf};
    const int32_t start[2] = {0, E};
    pose_batch b{1, E, q, t, cam, start, obs.data(), xw.data(), info.data()};
    std::vector<uint8_t> outl((size_t)E, 0);
    int32_t ninl = 0;
    pose_batch_result r{oq, ot, outl.data(), &ninl};
    check(pose_optimize_batch(device, &b, &r, nullptr), "pose_optimize_batch");
    for (int e = 0; e < E; e++) pFrame->mvbOutlier[idx[(size_t)e]] = outl[(size_t)e] != 0;
    lba_pose_to_Tcw(oq, ot, T);   // Converter::toCvMat
    pFrame->SetPose(detail::make_mat<MatT>(4, 4, T));
    return ninl;
}

// ======================================================================= LocalBundleAdjustment
// Per-thread solver context (LocalMapping runs the local BA on its own thread).
inline lba_context* thread_lba(int device = 0) {
    thread_local lba_context* c = nullptr;
    if (!c) check(lba_create(device, &c), "lba_create");
    return c;
}

// Optimizer::LocalBundleAdjustment(pKF, pbStopFlag, pMap): the local window and its fixed
// observers gathered exactly as R/src/Optimizer.cpp:567-625 does (covisible keyframes in
// GetVectorCovisibleKeyFrames order, map points in first-seen order, fixed cameras from the points'
// observations), one lba_problem, lba_solve (optimize(5), outlier pass, optimize(10), final check;
// *pbStopFlag is read like g2o's terminate()), then the write-back of :883-917 under
// pMap->mMutexMapUpdate.  `dump`, when given, receives the problem and result arrays (tests).
struct LbaDump {
    std::vector<double> pose_q, pose_t, point_xyz, edge_obs, edge_info, edge_cam;
    std::vector<uint8_t> pose_fixed, point_bad, edge_stereo, edge_erase;
    std::vector<int64_t> pose_id, point_id;
    std::vector<int32_t> edge_point, edge_pose;
    std::vector<double> out_q, out_t, out_xyz;
    int iterations[2] = {0, 0}, trials = 0, aborted = 0;
    // host wall time of the call's phases (steady_clock): 0 gather of the window (R :567-625),
    // 1 the problem arrays (R :636-782), 2 lba_solve, 3 vToErase + write-back (R :850-917)
    double phase_us[4] = {0.0, 0.0, 0.0, 0.0};
    void clear() {   // keeps the capacity: a reused dump neither allocates nor faults pages in
        for (auto* v : {&pose_q, &pose_t, &point_xyz, &edge_obs, &edge_info, &edge_cam, &out_q, &out_t, &out_xyz})
            v->clear();
        for (auto* v : {&pose_fixed, &point_bad, &edge_stereo, &edge_erase}) v->clear();
        pose_id.clear(); point_id.clear(); edge_point.clear(); edge_pose.clear();
        iterations[0] = iterations[1] = trials = aborted = 0;
    }
};

// The phases (LbaDump::phase_us) of this thread's last LocalBundleAdjustment call.
inline double* lba_last_phases() {
    thread_local double ph[4] = {0.0, 0.0, 0.0, 0.0};
    return ph;
}

namespace detail {
// A small pool of host threads for the per-point loops of LocalBundleAdjustment's gather and
// write-back (one pool per calling thread, created on first use; ORB_SHIM_THREADS workers, default
// 4, 0 = run inline).  parallel_for(n, grain, fn) calls fn(begin, end) over [0, n) in chunks of
// `grain`, the caller taking chunks too, and returns when every chunk has run; an exception in a
// chunk is rethrown in the caller.  Every worker checks in once per call, so no worker can miss one.
class HostPool {
public:
    explicit HostPool(int n) {
        for (int i = 0; i < n; i++) th_.emplace_back([this] { run(); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    template <class F>
    void parallel_for(size_t n, size_t grain, F&& fn) {
        if (grain == 0) grain = 1;
        if (th_.empty() || n <= grain) {
            if (n) fn((size_t)0, n);
            return;
        }
        std::function<void(size_t, size_t)> f(std::forward<F>(fn));
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &f;
            n_ = n;
            grain_ = grain;
            err_ = nullptr;
            next_.store(0, std::memory_order_relaxed);
            pending_.store((int)th_.size(), std::memory_order_relaxed);
            ++gen_;
        }
        cv_.notify_all();
        work();
        while (pending_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
        job_ = nullptr;
        if (err_) std::rethrow_exception(err_);
    }

private:
    void work() {
        for (;;) {
            const size_t b = next_.fetch_add(grain_, std::memory_order_relaxed);
            if (b >= n_) break;
            try {
                (*job_)(b, std::min(n_, b + grain_));
            } catch (...) {
                std::lock_guard<std::mutex> lk(errM_);
                if (!err_) err_ = std::current_exception();
            }
        }
    }
    void run() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return gen_ != seen; });
                seen = gen_;
                if (stop_) return;
            }
            work();
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_, errM_;
    std::condition_variable cv_;
    uint64_t gen_ = 0;
    bool stop_ = false;
    const std::function<void(size_t, size_t)>* job_ = nullptr;
    size_t n_ = 0, grain_ = 1;
    std::atomic<size_t> next_{0};
    std::atomic<int> pending_{0};
    std::exception_ptr err_;
};

inline HostPool& thread_pool() {
    thread_local HostPool pool([] {
        const char* e = std::getenv("ORB_SHIM_THREADS");
        const int n = e ? std::atoi(e) : 4;
        return n < 0 ? 0 : (n > 64 ? 64 : n);
    }());
    return pool;
}

// Per-thread working set of local_ba, reused from call to call (LocalMapping calls it once per
// keyframe): the window lists, the problem / result arrays and the edge bookkeeping keep their
// capacity, so a steady-state call allocates only what the reference API returns by value.
template <class KeyFrameT, class MapPointT>
struct LbaScratch {
    struct Ob {   // one observation as read once from GetObservations(), with its observer's isBad()
        KeyFrameT* kf;
        size_t idx;
        bool bad;
    };
    LbaDump D;
    std::vector<KeyFrameT*> localKFs, fixedKFs, edgeKF;
    std::vector<MapPointT*> localMPs;
    std::vector<std::vector<Ob>> obs;   // per point (the inner vectors keep their capacity across calls)
    std::vector<std::pair<const KeyFrameT*, int>> poseIndex;
    std::vector<std::pair<KeyFrameT*, MapPointT*>> toErase;
    std::vector<int> nEdge;
    void clear() {
        D.clear();
        localKFs.clear(); fixedKFs.clear(); edgeKF.clear(); localMPs.clear(); poseIndex.clear();
        toErase.clear(); nEdge.clear();
    }
};

template <class KeyFrameT, class MapT, class Solve>
void local_ba(KeyFrameT* pKF, bool* pbStopFlag, MapT* pMap, LbaDump* dump, Solve&& solve) {
    using MapPointT = typename std::remove_pointer<typename decltype(pKF->GetMapPointMatches())::value_type>::type;
    using MatT = typename std::decay<decltype(pKF->GetPose())>::type;
    using Clock = std::chrono::steady_clock;
    auto tPhase = Clock::now();
    double* ph = lba_last_phases();
    auto lap = [&tPhase](double& acc) {
        const auto now = Clock::now();
        acc = std::chrono::duration<double, std::micro>(now - tPhase).count();
        tPhase = now;
    };
    ph[0] = ph[1] = ph[2] = ph[3] = 0.0;
    thread_local LbaScratch<KeyFrameT, MapPointT> sc;
    sc.clear();
    struct Out {   // the caller's dump (tests) receives a copy of the arrays, whatever the exit
        LbaScratch<KeyFrameT, MapPointT>& sc;
        LbaDump* dump;
        double* ph;
        ~Out() {
            std::copy(ph, ph + 4, sc.D.phase_us);
            if (dump) *dump = sc.D;
        }
    } out{sc, dump, ph};
    LbaDump& D = sc.D;
    // ---- local keyframes, local map points, fixed cameras (R :567-625; the reference's std::lists
    //      as arrays, same order)
    auto& lLocalKeyFrames = sc.localKFs;
    lLocalKeyFrames.push_back(pKF);
    pKF->mnBALocalForKF = pKF->mnId;
    const std::vector<KeyFrameT*> vNeighKFs = pKF->GetVectorCovisibleKeyFrames();
    for (KeyFrameT* pKFi : vNeighKFs) {
        pKFi->mnBALocalForKF = pKF->mnId;
        if (!pKFi->isBad()) lLocalKeyFrames.push_back(pKFi);
    }
    auto& lLocalMapPoints = sc.localMPs;
    for (KeyFrameT* k : lLocalKeyFrames)
        for (MapPointT* pMP : k->GetMapPointMatches())
            if (pMP && !pMP->isBad() && pMP->mnBALocalForKF != pKF->mnId) {
                lLocalMapPoints.push_back(pMP);
                pMP->mnBALocalForKF = pKF->mnId;
            }
    // (each point's observations are read once here, in parallel over the points, and reused for its
    // edges below; the reference calls GetObservations() again at :740 — both are snapshots of a map
    // other threads may grow).  Per point also the number of its edges (observers not bad).
    HostPool& pool = thread_pool();
    auto& vObs = sc.obs;
    auto& nEdge = sc.nEdge;
    const size_t nPts = lLocalMapPoints.size();
    vObs.resize(nPts);
    nEdge.assign(nPts + 1, 0);
    pool.parallel_for(nPts, 64, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; i++) {
            auto& v = vObs[i];
            v.clear();
            int n = 0;
            for (const auto& ob : lLocalMapPoints[i]->GetObservations()) {   // isBad() read once per observation
                const bool bad = ob.first->isBad();
                v.push_back({ob.first, (size_t)ob.second, bad});
                n += bad ? 0 : 1;
            }
            nEdge[i + 1] = n;
        }
    });
    auto& lFixedCameras = sc.fixedKFs;
    for (size_t i = 0; i < nPts; i++)   // first-seen order, as the reference's list
        for (const auto& ob : vObs[i]) {
            KeyFrameT* pKFi = ob.kf;
            if (pKFi->mnBALocalForKF != pKF->mnId && pKFi->mnBAFixedForKF != pKF->mnId) {
                pKFi->mnBAFixedForKF = pKF->mnId;
                if (!ob.bad) lFixedCameras.push_back(pKFi);
            }
        }
    for (size_t i = 0; i < nPts; i++) nEdge[i + 1] += nEdge[i];   // edge offsets per point
    const size_t nObs = (size_t)nEdge[nPts];
    lap(ph[0]);
    // ---- the graph as arrays (vertices: local poses (fixed iff mnId == 0), fixed cameras, points
    //      with id mnId + maxKFid + 1; edges per point in observation order, R :636-782)
    const size_t nPoses = lLocalKeyFrames.size() + lFixedCameras.size();
    D.pose_q.reserve(4 * nPoses); D.pose_t.reserve(3 * nPoses); D.pose_fixed.reserve(nPoses); D.pose_id.reserve(nPoses);
    D.point_xyz.resize(3 * nPts); D.point_id.resize(nPts); D.point_bad.resize(nPts);
    D.edge_point.resize(nObs); D.edge_pose.resize(nObs); D.edge_stereo.resize(nObs); D.edge_obs.resize(3 * nObs);
    D.edge_info.resize(nObs); D.edge_cam.resize(5 * nObs);
    // keyframe -> vertex index: a sorted array (a window holds tens of keyframes)
    auto& poseIndex = sc.poseIndex;
    unsigned long maxKFid = 0;
    auto addPose = [&](KeyFrameT* k, bool fixed) {
        poseIndex.emplace_back(k, (int)D.pose_fixed.size());
        float T[16];
        detail::read_Tcw(k->GetPose(), T);
        double q[4], t[3];
        lba_pose_from_Tcw(T, q, t);   // Converter::toSE3Quat
        D.pose_q.insert(D.pose_q.end(), q, q + 4);
        D.pose_t.insert(D.pose_t.end(), t, t + 3);
        D.pose_fixed.push_back(fixed ? 1 : 0);
        D.pose_id.push_back((int64_t)k->mnId);
        if (k->mnId > maxKFid) maxKFid = k->mnId;
    };
    for (KeyFrameT* k : lLocalKeyFrames) addPose(k, k->mnId == 0);
    for (KeyFrameT* k : lFixedCameras) addPose(k, true);
    std::sort(poseIndex.begin(), poseIndex.end());
    auto poseOf = [&poseIndex](const KeyFrameT* k) {
        const auto it = std::lower_bound(poseIndex.begin(), poseIndex.end(), std::make_pair(k, -1));
        if (it == poseIndex.end() || it->first != k) throw std::out_of_range("LocalBundleAdjustment: observer not in the window");
        return it->second;
    };
    auto& vpMP = lLocalMapPoints;   // vertex order = the local map points' order
    auto& vpEdgeKF = sc.edgeKF;
    vpEdgeKF.resize(nObs);
    // points and their edges, in parallel over the points: point pi's edges fill [nEdge[pi], nEdge[pi+1])
    pool.parallel_for(nPts, 64, [&](size_t b, size_t e) {
        for (size_t pi = b; pi < e; pi++) {
            MapPointT* pMP = vpMP[pi];
            const MatT X = pMP->GetWorldPos();
            for (int i = 0; i < 3; i++) D.point_xyz[3 * pi + (size_t)i] = (double)X.template at<float>(i, 0);   // Converter::toVector3d
            D.point_id[pi] = (int64_t)(pMP->mnId + maxKFid + 1);
            D.point_bad[pi] = pMP->isBad() ? 1 : 0;
            size_t k = (size_t)nEdge[pi];
            for (const auto& ob : vObs[pi]) {
                if (ob.bad) continue;
                KeyFrameT* pKFi = ob.kf;
                const auto& kpUn = pKFi->mvKeysUn[ob.idx];
                const float ur = pKFi->mvuRight[ob.idx];
                D.edge_point[k] = (int32_t)pi;
                D.edge_pose[k] = poseOf(pKFi);
                D.edge_stereo[k] = ur < 0 ? 0 : 1;
                D.edge_obs[3 * k] = kpUn.pt.x;
                D.edge_obs[3 * k + 1] = kpUn.pt.y;
                D.edge_obs[3 * k + 2] = ur < 0 ? 0.0 : (double)ur;
                D.edge_info[k] = (double)pKFi->mvInvLevelSigma2[kpUn.octave];   // I * invSigma2 (float)
                double* cam = &D.edge_cam[5 * k];
                cam[0] = pKFi->fx; cam[1] = pKFi->fy; cam[2] = pKFi->cx; cam[3] = pKFi->cy; cam[4] = pKFi->mbf;
                vpEdgeKF[k] = pKFi;
                k++;
            }
        }
    });
    const int NP = (int)D.pose_fixed.size(), NM = (int)vpMP.size(), NE = (int)D.edge_point.size();
    lba_problem p{NP, D.pose_q.data(), D.pose_t.data(), D.pose_fixed.data(), D.pose_id.data(),
                  NM, D.point_xyz.data(), D.point_id.data(), D.point_bad.data(),
                  NE, D.edge_point.data(), D.edge_pose.data(), D.edge_stereo.data(), D.edge_obs.data(),
                  D.edge_info.data(), D.edge_cam.data()};
    lba_options o{5, 10, 5.991, 7.815, 0, 0, 10, 0};
    o.huber_mono = (double)(float)std::sqrt(5.991);     // const float thHuberMono = sqrt(5.991) (R :696)
    o.huber_stereo = (double)(float)std::sqrt(7.815);
    D.out_q.assign(4 * (size_t)NP, 0.0);
    D.out_t.assign(3 * (size_t)NP, 0.0);
    D.out_xyz.assign(3 * (size_t)NM, 0.0);
    D.edge_erase.assign((size_t)NE, 0);
    lba_result r{D.out_q.data(), D.out_t.data(), D.out_xyz.data(), D.edge_erase.data(), nullptr, {0, 0}, 0,
                 nullptr, 0, 0};
    static_assert(sizeof(bool) == 1, "mbAbortBA is read as one byte");
    lap(ph[1]);
    check(solve(&p, &o, reinterpret_cast<const volatile uint8_t*>(pbStopFlag), &r), "lba_solve");
    lap(ph[2]);
    D.iterations[0] = r.iterations[0];
    D.iterations[1] = r.iterations[1];
    D.trials = r.trials;
    D.aborted = r.aborted;
    if (r.aborted) return;   // R :784-786: stopped before optimizing, nothing written back
    // ---- vToErase (R :850-880): the mono edges in insertion order, then the stereo edges, each
    //      skipping a point that became bad while the solve ran (isBad() read now, as R :855/:872
    //      do after optimize); the order matters to EraseObservation's choice of mpRefKF / SetBadFlag
    auto& vToErase = sc.toErase;
    for (int pass = 0; pass < 2; pass++)
        for (int e = 0; e < NE; e++) {
            if ((int)D.edge_stereo[(size_t)e] != pass || !D.edge_erase[(size_t)e]) continue;
            MapPointT* pMP = vpMP[(size_t)D.edge_point[(size_t)e]];
            if (pMP->isBad()) continue;
            vToErase.emplace_back(vpEdgeKF[(size_t)e], pMP);
        }
    // ---- write-back (R :883-917)
    std::unique_lock<std::mutex> lock(pMap->mMutexMapUpdate);
    for (auto& ke : vToErase) {
        ke.first->EraseMapPointMatch(ke.second);
        ke.second->EraseObservation(ke.first);
    }
    int i = 0;
    for (KeyFrameT* k : lLocalKeyFrames) {   // Converter::toCvMat(SE3Quat): 4x4 float
        float T[16];
        lba_pose_to_Tcw(&D.out_q[4 * (size_t)i], &D.out_t[3 * (size_t)i], T);
        k->SetPose(detail::make_mat<MatT>(4, 4, T));
        i++;
    }
    // the points in parallel: each SetWorldPos + UpdateNormalAndDepth touches its own point (and reads
    // the keyframe poses set above), as the reference's loop does one by one
    pool.parallel_for((size_t)NM, 64, [&](size_t b, size_t e) {
        for (size_t m = b; m < e; m++) {
            const float X[3] = {(float)D.out_xyz[3 * m], (float)D.out_xyz[3 * m + 1], (float)D.out_xyz[3 * m + 2]};
            vpMP[m]->SetWorldPos(detail::make_mat<MatT>(3, 1, X));
            vpMP[m]->UpdateNormalAndDepth();
        }
    });
    lap(ph[3]);
}
}  // namespace detail

template <class KeyFrameT, class MapT>
void LocalBundleAdjustment(KeyFrameT* pKF, bool* pbStopFlag, MapT* pMap, LbaDump* dump = nullptr,
                           lba_context* ctx = nullptr) {
    lba_context* c = ctx ? ctx : thread_lba();
    detail::local_ba(pKF, pbStopFlag, pMap, dump,
                     [c](const lba_problem* p, const lba_options* o, const volatile uint8_t* st, lba_result* r) {
                         return lba_solve(c, p, o, st, r);
                     });
}

// The same window sharded over several GPUs of this process (lba_group_*: landmark shards, the
// library's peer-to-peer all-reduce over xGMI, identical LM decisions on every device).  One group
// per calling thread and device list, created on first use.
inline lba_group* thread_lba_group(const std::vector<int>& devices) {
    thread_local std::map<std::vector<int>, lba_group*> groups;
    lba_group*& g = groups[devices];
    if (!g) check(lba_group_create(devices.data(), (int)devices.size(), &g), "lba_group_create");
    return g;
}
template <class KeyFrameT, class MapT>
void LocalBundleAdjustment(KeyFrameT* pKF, bool* pbStopFlag, MapT* pMap, const std::vector<int>& devices,
                           LbaDump* dump = nullptr) {
    lba_group* g = thread_lba_group(devices);
    detail::local_ba(pKF, pbStopFlag, pMap, dump,
                     [g](const lba_problem* p, const lba_options* o, const volatile uint8_t* st, lba_result* r) {
                         return lba_group_solve(g, p, o, st, r);
                     });
}

}  // namespace orbslam2_amd
