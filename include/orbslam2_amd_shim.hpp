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
//                             SearchByProjection(Frame&, const vector<MapPoint*>&, th) (:63-163)
//   LocalBundleAdjustment     Optimizer::LocalBundleAdjustment (R/include/Optimizer.h:45,
//                             R/src/Optimizer.cpp:564-918): graph gathering, lba_solve (or, given a
//                             device list, lba_group_solve over several GPUs), write-back
//
// Errors: the reference's methods have no error returns, so a negative ORB_E* status becomes a
// std::runtime_error here (there is no CPU fallback: without a gfx950 device the constructors
// throw).
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
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
// A Frame's matcher view: mvKeysUn split into arrays (built once per call), mDescriptors,
// mvuRight and the static grid bounds (R/include/Frame.h: mnMinX .. mfGridElementHeightInv).
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
        v.min_x = FrameT::mnMinX; v.min_y = FrameT::mnMinY; v.max_x = FrameT::mnMaxX; v.max_y = FrameT::mnMaxY;
        v.grid_w_inv = FrameT::mfGridElementWidthInv; v.grid_h_inv = FrameT::mfGridElementHeightInv;
    }
};

class Matcher {
public:
    explicit Matcher(float nnratio = 0.6f, bool checkOri = true, int device = 0) {
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

private:
    template <class MatT>
    static void detail_read_T34(const MatT& T, float out[12]) {   // rows 0..2 of a 4x4 float cv::Mat
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 4; k++) out[4 * r + k] = T.template at<float>(r, k);
    }
    orb_matcher* h_ = nullptr;
};

// ======================================================================= LocalBundleAdjustment
// Per-thread solver context (LocalMapping runs the local BA on its own thread).
inline lba_context* thread_lba(int device = 0) {
    thread_local lba_context* c = nullptr;
    if (!c) check(lba_create(device, &c), "lba_create");
    return c;
}

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
}  // namespace detail

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
};

namespace detail {
template <class KeyFrameT, class MapT, class Solve>
void local_ba(KeyFrameT* pKF, bool* pbStopFlag, MapT* pMap, LbaDump* dump, Solve&& solve) {
    using MapPointT = typename std::remove_pointer<typename decltype(pKF->GetMapPointMatches())::value_type>::type;
    using MatT = typename std::decay<decltype(pKF->GetPose())>::type;
    // ---- local keyframes, local map points, fixed cameras (R :567-625)
    std::list<KeyFrameT*> lLocalKeyFrames;
    lLocalKeyFrames.push_back(pKF);
    pKF->mnBALocalForKF = pKF->mnId;
    const std::vector<KeyFrameT*> vNeighKFs = pKF->GetVectorCovisibleKeyFrames();
    for (KeyFrameT* pKFi : vNeighKFs) {
        pKFi->mnBALocalForKF = pKF->mnId;
        if (!pKFi->isBad()) lLocalKeyFrames.push_back(pKFi);
    }
    std::list<MapPointT*> lLocalMapPoints;
    for (KeyFrameT* k : lLocalKeyFrames)
        for (MapPointT* pMP : k->GetMapPointMatches())
            if (pMP && !pMP->isBad() && pMP->mnBALocalForKF != pKF->mnId) {
                lLocalMapPoints.push_back(pMP);
                pMP->mnBALocalForKF = pKF->mnId;
            }
    std::list<KeyFrameT*> lFixedCameras;
    for (MapPointT* pMP : lLocalMapPoints)
        for (const auto& ob : pMP->GetObservations()) {
            KeyFrameT* pKFi = ob.first;
            if (pKFi->mnBALocalForKF != pKF->mnId && pKFi->mnBAFixedForKF != pKF->mnId) {
                pKFi->mnBAFixedForKF = pKF->mnId;
                if (!pKFi->isBad()) lFixedCameras.push_back(pKFi);
            }
        }
    // ---- the graph as arrays (vertices: local poses (fixed iff mnId == 0), fixed cameras, points
    //      with id mnId + maxKFid + 1; edges per point in observation order, R :636-782)
    LbaDump own;
    LbaDump& D = dump ? *dump : own;
    std::map<const KeyFrameT*, int> poseIndex;
    unsigned long maxKFid = 0;
    auto addPose = [&](KeyFrameT* k, bool fixed) {
        poseIndex[k] = (int)D.pose_fixed.size();
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
    std::vector<MapPointT*> vpMP;
    std::vector<KeyFrameT*> vpEdgeKF;
    for (MapPointT* pMP : lLocalMapPoints) {
        const int pi = (int)vpMP.size();
        vpMP.push_back(pMP);
        const MatT X = pMP->GetWorldPos();
        for (int i = 0; i < 3; i++) D.point_xyz.push_back((double)X.template at<float>(i, 0));   // Converter::toVector3d
        D.point_id.push_back((int64_t)(pMP->mnId + maxKFid + 1));
        D.point_bad.push_back(pMP->isBad() ? 1 : 0);
        for (const auto& ob : pMP->GetObservations()) {
            KeyFrameT* pKFi = ob.first;
            if (pKFi->isBad()) continue;
            const auto& kpUn = pKFi->mvKeysUn[ob.second];
            const float ur = pKFi->mvuRight[ob.second];
            D.edge_point.push_back(pi);
            D.edge_pose.push_back(poseIndex.at(pKFi));
            D.edge_stereo.push_back(ur < 0 ? 0 : 1);
            D.edge_obs.push_back(kpUn.pt.x);
            D.edge_obs.push_back(kpUn.pt.y);
            D.edge_obs.push_back(ur < 0 ? 0.0 : (double)ur);
            D.edge_info.push_back((double)pKFi->mvInvLevelSigma2[kpUn.octave]);   // I * invSigma2 (float)
            const double cam[5] = {pKFi->fx, pKFi->fy, pKFi->cx, pKFi->cy, pKFi->mbf};
            D.edge_cam.insert(D.edge_cam.end(), cam, cam + 5);
            vpEdgeKF.push_back(pKFi);
        }
    }
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
    check(solve(&p, &o, reinterpret_cast<const volatile uint8_t*>(pbStopFlag), &r), "lba_solve");
    D.iterations[0] = r.iterations[0];
    D.iterations[1] = r.iterations[1];
    D.trials = r.trials;
    D.aborted = r.aborted;
    if (r.aborted) return;   // R :784-786: stopped before optimizing, nothing written back
    // ---- vToErase (R :850-880): the mono edges in insertion order, then the stereo edges, each
    //      skipping a point that became bad while the solve ran (isBad() read now, as R :855/:872
    //      do after optimize); the order matters to EraseObservation's choice of mpRefKF / SetBadFlag
    std::vector<std::pair<KeyFrameT*, MapPointT*>> vToErase;
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
    for (int m = 0; m < NM; m++) {
        const float X[3] = {(float)D.out_xyz[3 * (size_t)m], (float)D.out_xyz[3 * (size_t)m + 1],
                            (float)D.out_xyz[3 * (size_t)m + 2]};
        vpMP[(size_t)m]->SetWorldPos(detail::make_mat<MatT>(3, 1, X));
        vpMP[(size_t)m]->UpdateNormalAndDepth();
    }
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
