// A C++ caller of liborbslam2_amd through include/orbslam2_amd_shim.hpp, with mock types that have
// the member names the shim reads from the reference's cv::Mat / cv::KeyPoint / Frame / KeyFrame /
// MapPoint / Map (OpenCV and the ORB-SLAM2 sources are not built here).  Driven by
// tests/test_cpp_shim.py:
//   shim_caller extract IN OUT   ORBextractor::operator() on one image
//   shim_caller sfi IN OUT       ORBmatcher::SearchForInitialization on two frames
//   shim_caller sbp IN OUT       ORBmatcher::SearchByProjection(Frame&, const Frame&, th, bMono)
//   shim_caller sbl IN OUT       ORBmatcher::SearchByProjection(Frame&, const vector<MapPoint*>&, th)
//   shim_caller lba IN OUT       Optimizer::LocalBundleAdjustment on a mock keyframe / map-point graph
//   shim_caller lbag IN OUT      the same through the device-list overload (lba_group, several GPUs)
//   shim_caller lbacpu IN OUT    the same gather / write-back around the CPU oracle's solve
//                                ($ORB_ORACLE_LIB; the routed row's like-for-like CPU column)
//   shim_caller pose IN OUT      Optimizer::PoseOptimization on a mock Frame
//   shim_caller stereo IN OUT    ORBextractor on a left / right image (two handles), then
//                                Frame::ComputeStereoMatches on the mock Frame
//   shim_caller fuse IN OUT      ORBmatcher::Fuse(pKF, vpMapPoints, th), replace / add on mock points
//   shim_caller sft IN OUT       ORBmatcher::SearchForTriangulation(pKF1, pKF2, F12, pairs, bOnlyStereo)
//   shim_caller sbbf IN OUT      ORBmatcher::SearchByBoW(pKF, F, vpMapPointMatches)
//   shim_caller sbbk IN OUT      ORBmatcher::SearchByBoW(pKF1, pKF2, vpMatches12)
//   shim_caller sbpk IN OUT      ORBmatcher::SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist)
//   shim_caller sbps IN OUT      ORBmatcher::SearchByProjection(pKF, Scw, vpPoints, vpMatched, th)
//   shim_caller sbs IN OUT       ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
//   shim_caller fuses IN OUT     ORBmatcher::Fuse(pKF, Scw, vpPoints, th, vpReplacePoint)
//   shim_caller timeit REPS lba IN   per-call wall time of Optimizer::LocalBundleAdjustment through the
//                                shim (graph gather + solve + write-back, the mock map rebuilt from IN
//                                before each call and not timed): prints "median_us N min_us M"
//   shim_caller threads IN OUT   the SURVEY 8b threading contract: two Extractor handles on two host
//                                threads at once (stereo L/R, R/src/Frame.cpp:86-89), SearchForInitialization
//                                and PoseOptimization on a third and fourth (Tracking), LocalBundleAdjustment
//                                on a fifth (LocalMapping), each repeated; results must not change
// IN / OUT: little-endian arrays, each written as int64 element count + raw elements.
// Exit status: 0 ok, 3 the library reported an error (e.g. no gfx950 device), 2 bad usage.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <utility>
#include <stdexcept>
#include <vector>

#include "orbslam2_amd_shim.hpp"

namespace mock {

struct Mat {   // the cv::Mat members the shim uses
    int rows = 0, cols = 0, type = 0;
    size_t step = 0;
    uint8_t* data = nullptr;
    std::vector<uint8_t> buf;
    Mat() = default;
    Mat(int r, int c, int t) { create(r, c, t); }
    Mat(const Mat& o) : rows(o.rows), cols(o.cols), type(o.type), step(o.step), buf(o.buf) { data = buf.empty() ? nullptr : buf.data(); }
    Mat& operator=(const Mat& o) {
        rows = o.rows; cols = o.cols; type = o.type; step = o.step; buf = o.buf;
        data = buf.empty() ? nullptr : buf.data();
        return *this;
    }
    void create(int r, int c, int t) {
        rows = r; cols = c; type = t;
        step = (size_t)c * (t == orbslam2_amd::kCV_32F ? 4 : 1);
        buf.assign((size_t)r * step, 0);
        data = buf.data();
    }
    void release() { buf.clear(); data = nullptr; rows = cols = 0; step = 0; }
    template <class T> T& at(int r, int c) { return *reinterpret_cast<T*>(data + (size_t)r * step + (size_t)c * sizeof(T)); }
    template <class T> const T& at(int r, int c) const {
        return *reinterpret_cast<const T*>(data + (size_t)r * step + (size_t)c * sizeof(T));
    }
};
struct Point2f { float x, y; };
struct KeyPoint { Point2f pt; float size, angle, response; int octave, class_id; };

using FeatureVector = std::map<unsigned int, std::vector<unsigned int>>;   // DBoW2::FeatureVector

struct MapPoint;
struct Frame {
    std::vector<KeyPoint> mvKeys, mvKeysRight, mvKeysUn;
    Mat mDescriptors, mDescriptorsRight;
    std::vector<float> mvuRight, mvDepth;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    std::vector<float> mvScaleFactors, mvInvLevelSigma2;
    float mfLogScaleFactor = 0;
    int mnScaleLevels = 8;
    FeatureVector mFeatVec;
    Mat mTcw;
    float mbf = 0, mb = 0;
    static float mnMinX, mnMinY, mnMaxX, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv;
    static float fx, fy, cx, cy;
    void SetPose(const Mat& T) { mTcw = T; }
};
float Frame::mnMinX, Frame::mnMinY, Frame::mnMaxX, Frame::mnMaxY, Frame::mfGridElementWidthInv,
    Frame::mfGridElementHeightInv, Frame::fx, Frame::fy, Frame::cx, Frame::cy;

// the order of KeyFrame::EraseMapPointMatch calls (keyframe mnId, map point mnId)
thread_local std::vector<std::pair<unsigned long, unsigned long>> g_erase_log;
struct KeyFrame {
    unsigned long mnId = 0, mnBALocalForKF = 0, mnBAFixedForKF = 0;
    bool bad = false;
    std::vector<KeyFrame*> covis;
    std::vector<MapPoint*> matches;   // mvpMapPoints
    Mat Tcw, Ow;
    std::vector<KeyPoint> mvKeysUn;
    Mat mDescriptors;
    std::vector<float> mvuRight, mvInvLevelSigma2, mvLevelSigma2, mvScaleFactors;
    FeatureVector mFeatVec;
    float fx = 0, fy = 0, cx = 0, cy = 0, mbf = 0;
    float mfLogScaleFactor = 0;
    int mnScaleLevels = 8;
    int mnMinX = 0, mnMinY = 0, mnMaxX = 640, mnMaxY = 480;   // const int members in the reference
    float mfGridElementWidthInv = 0, mfGridElementHeightInv = 0;
    std::vector<KeyFrame*> GetVectorCovisibleKeyFrames() { return covis; }
    std::vector<MapPoint*> GetMapPointMatches() { return matches; }
    MapPoint* GetMapPoint(size_t i) { return matches[i]; }
    std::set<MapPoint*> GetMapPoints();
    void AddMapPoint(MapPoint* p, size_t i) { matches[i] = p; }
    void ReplaceMapPointMatch(size_t i, MapPoint* p) { matches[i] = p; }
    bool isBad() const { return bad; }
    Mat GetPose() { return Tcw; }
    void SetPose(const Mat& T) { Tcw = T; }
    Mat GetCameraCenter() { return Ow; }
    Mat GetRotation() {
        Mat R(3, 3, orbslam2_amd::kCV_32F);
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 3; k++) R.at<float>(r, k) = Tcw.at<float>(r, k);
        return R;
    }
    Mat GetTranslation() {
        Mat t(3, 1, orbslam2_amd::kCV_32F);
        for (int r = 0; r < 3; r++) t.at<float>(r, 0) = Tcw.at<float>(r, 3);
        return t;
    }
    void EraseMapPointMatch(MapPoint* p);
    void EraseMapPointMatch(size_t i) { matches[i] = nullptr; }
};
struct MapPoint {
    unsigned long mnId = 0, mnBALocalForKF = 0;
    bool bad = false;
    Mat X;
    std::map<KeyFrame*, size_t> obs;
    int updates = 0;
    bool isBad() const { return bad; }
    Mat GetWorldPos() { return X; }
    void SetWorldPos(const Mat& P) { X = P; }
    std::map<KeyFrame*, size_t> GetObservations() { return obs; }
    void EraseObservation(KeyFrame* k) { obs.erase(k); }
    void UpdateNormalAndDepth() { updates++; }
    // tracking members read by SearchByProjection
    int extraObs = 0;   // observations beyond `obs` (the matcher tests keep `obs` empty)
    int Observations() { return (int)obs.size() + extraObs; }
    Mat desc;
    Mat GetDescriptor() { return desc; }
    bool mbTrackInView = false;
    float mTrackProjX = 0, mTrackProjY = 0, mTrackProjXR = 0, mTrackViewCos = 0;
    int mnTrackScaleLevel = 0;
    // Fuse / PoseOptimization members
    static std::mutex mGlobalMutex;
    Mat normal;
    float mfMinDistance = 0, mfMaxDistance = 0;
    Mat GetNormal() { return normal; }
    void GetDistances(float& mn, float& mx) { mn = mfMinDistance; mx = mfMaxDistance; }
    bool IsInKeyFrame(KeyFrame* k) { return obs.count(k) > 0; }
    int GetIndexInKeyFrame(KeyFrame* k) {
        const auto it = obs.find(k);
        return it == obs.end() ? -1 : (int)it->second;
    }
    void AddObservation(KeyFrame* k, size_t i) { obs[k] = i; }
    MapPoint* replacedBy = nullptr;
    // MapPoint::Replace (R/src/MapPoint.cpp:177-219): observations move to pMP unless it is in that
    // keyframe already (then the keyframe's slot is erased); this point becomes bad
    void Replace(MapPoint* p) {
        if (p == this) return;
        const auto o = obs;
        obs.clear();
        bad = true;
        replacedBy = p;
        for (const auto& kv : o) {
            if (!p->IsInKeyFrame(kv.first)) {
                kv.first->ReplaceMapPointMatch(kv.second, p);
                p->AddObservation(kv.first, kv.second);
            } else {
                kv.first->EraseMapPointMatch(kv.second);
            }
        }
        p->extraObs += extraObs;
    }
};
std::mutex MapPoint::mGlobalMutex;
inline void KeyFrame::EraseMapPointMatch(MapPoint* p) {   // R/src/KeyFrame.cpp: by GetIndexInKeyFrame
    g_erase_log.emplace_back(mnId, p->mnId);
    const int idx = p->GetIndexInKeyFrame(this);
    if (idx >= 0) matches[(size_t)idx] = nullptr;
}
inline std::set<MapPoint*> KeyFrame::GetMapPoints() {   // R/src/KeyFrame.cpp: set, not bad
    std::set<MapPoint*> s;
    for (MapPoint* p : matches)
        if (p && !p->isBad()) s.insert(p);
    return s;
}
struct Map {
    std::mutex mMutexMapUpdate;
};

}  // namespace mock

template <class T>
static std::vector<T> rd(FILE* f) {
    long long n = 0;
    if (std::fread(&n, 8, 1, f) != 1 || n < 0) throw std::runtime_error("truncated input");
    std::vector<T> v((size_t)n);
    if (n && std::fread(v.data(), sizeof(T), (size_t)n, f) != (size_t)n) throw std::runtime_error("truncated input");
    return v;
}
template <class T>
static void wr(FILE* f, const T* p, size_t n) {
    const long long c = (long long)n;
    std::fwrite(&c, 8, 1, f);
    if (n) std::fwrite(p, sizeof(T), n, f);
}
template <class T>
static void wr(FILE* f, const std::vector<T>& v) { wr(f, v.data(), v.size()); }

static void run_extract(FILE* in, FILE* out) {
    const auto wh = rd<int32_t>(in);
    const auto img = rd<uint8_t>(in);
    mock::Mat image(wh[1], wh[0], orbslam2_amd::kCV_8U);
    std::copy(img.begin(), img.end(), image.data);
    orbslam2_amd::Extractor ex(wh[2], 1.2f, 8, 20, 7, 0, wh[0], wh[1]);
    std::vector<mock::KeyPoint> kps;
    mock::Mat desc;
    ex.extract(image, kps, desc);
    wr(out, reinterpret_cast<const uint8_t*>(kps.data()), kps.size() * sizeof(mock::KeyPoint));
    wr(out, desc.data, (size_t)desc.rows * 32);
    const auto& lv = ex.pyramid();   // mvImagePyramid: the level sizes the reference exposes
    std::vector<int32_t> sizes;
    for (const auto& L : lv) { sizes.push_back(L.cols); sizes.push_back(L.rows); }
    wr(out, sizes);
    const auto sf = ex.GetScaleFactors();
    wr(out, sf);
}

static void load_frame(FILE* in, mock::Frame& F) {
    const auto x = rd<float>(in), y = rd<float>(in), a = rd<float>(in);
    const auto o = rd<int32_t>(in);
    const auto d = rd<uint8_t>(in);
    F.mvKeysUn.resize(x.size());
    for (size_t i = 0; i < x.size(); i++) F.mvKeysUn[i] = mock::KeyPoint{{x[i], y[i]}, 31.f, a[i], 0.f, o[i], -1};
    F.mDescriptors.create((int)x.size(), 32, orbslam2_amd::kCV_8U);
    std::copy(d.begin(), d.end(), F.mDescriptors.data);
}

static void run_sfi(FILE* in, FILE* out) {
    mock::Frame F1, F2;
    load_frame(in, F1);
    load_frame(in, F2);
    const auto g = rd<float>(in);
    mock::Frame::mnMinX = g[0]; mock::Frame::mnMinY = g[1]; mock::Frame::mnMaxX = g[2]; mock::Frame::mnMaxY = g[3];
    mock::Frame::mfGridElementWidthInv = g[4]; mock::Frame::mfGridElementHeightInv = g[5];
    const auto prev = rd<float>(in);
    const auto win = rd<int32_t>(in);
    std::vector<mock::Point2f> vbPrev(prev.size() / 2);
    for (size_t i = 0; i < vbPrev.size(); i++) vbPrev[i] = {prev[2 * i], prev[2 * i + 1]};
    std::vector<int> m12;
    orbslam2_amd::Matcher matcher(0.9f, true);
    const int n = matcher.SearchForInitialization(F1, F2, vbPrev, m12, win[0]);
    const int32_t nn = n;
    wr(out, &nn, 1);
    wr(out, m12);
    wr(out, reinterpret_cast<const float*>(vbPrev.data()), 2 * vbPrev.size());
    const int32_t d01 = orbslam2_amd::Matcher::DescriptorDistance(F1.mDescriptors.data, F2.mDescriptors.data);
    wr(out, &d01, 1);
}

static void set_grid(const std::vector<float>& g) {
    mock::Frame::mnMinX = g[0]; mock::Frame::mnMinY = g[1]; mock::Frame::mnMaxX = g[2]; mock::Frame::mnMaxY = g[3];
    mock::Frame::mfGridElementWidthInv = g[4]; mock::Frame::mfGridElementHeightInv = g[5];
}

// current-frame slots on entry: -1 NULL, -2 a point with observations, -3 one without; on exit the
// index of the point a slot holds in `pts`, or the same codes
static void init_slots(mock::Frame& F, const std::vector<int32_t>& init, mock::MapPoint& withObs, mock::MapPoint& noObs) {
    F.mvpMapPoints.assign(init.size(), nullptr);
    for (size_t i = 0; i < init.size(); i++)
        F.mvpMapPoints[i] = init[i] == -2 ? &withObs : init[i] == -3 ? &noObs : nullptr;
}
static std::vector<int32_t> read_slots(const mock::Frame& F, const std::vector<mock::MapPoint*>& pts,
                                       const mock::MapPoint& withObs, const mock::MapPoint& noObs) {
    std::map<const mock::MapPoint*, int32_t> idx;
    for (size_t i = 0; i < pts.size(); i++) idx[pts[i]] = (int32_t)i;
    std::vector<int32_t> o(F.mvpMapPoints.size(), -1);
    for (size_t i = 0; i < o.size(); i++) {
        const mock::MapPoint* p = F.mvpMapPoints[i];
        o[i] = !p ? -1 : p == &withObs ? -2 : p == &noObs ? -3 : idx.at(p);
    }
    return o;
}

static void run_sbp(FILE* in, FILE* out) {
    mock::Frame C, L;
    load_frame(in, C);
    C.mvuRight = rd<float>(in);
    load_frame(in, L);
    L.mvuRight.assign(L.mvKeysUn.size(), -1.f);
    set_grid(rd<float>(in));
    const auto Tc = rd<float>(in), Tl = rd<float>(in);
    const auto has = rd<int32_t>(in);
    const auto outl = rd<uint8_t>(in);
    const auto xyz = rd<float>(in);
    const auto mpd = rd<uint8_t>(in);
    C.mvScaleFactors = rd<float>(in);
    const auto cam = rd<float>(in);
    const auto th = rd<float>(in);
    const auto mono = rd<int32_t>(in);
    const auto init = rd<int32_t>(in);
    C.mTcw.create(4, 4, orbslam2_amd::kCV_32F);
    L.mTcw.create(4, 4, orbslam2_amd::kCV_32F);
    for (int i = 0; i < 16; i++) {
        C.mTcw.at<float>(i / 4, i % 4) = Tc[(size_t)i];
        L.mTcw.at<float>(i / 4, i % 4) = Tl[(size_t)i];
    }
    mock::Frame::fx = cam[0]; mock::Frame::fy = cam[1]; mock::Frame::cx = cam[2]; mock::Frame::cy = cam[3];
    C.mbf = cam[4]; C.mb = cam[5];
    const size_t nl = L.mvKeysUn.size();
    std::vector<mock::MapPoint> pts(nl);
    std::vector<mock::MapPoint*> ptr(nl, nullptr);
    L.mvpMapPoints.assign(nl, nullptr);
    L.mvbOutlier.assign(nl, false);
    for (size_t i = 0; i < nl; i++) {
        ptr[i] = &pts[i];
        pts[i].X.create(3, 1, orbslam2_amd::kCV_32F);
        for (int k = 0; k < 3; k++) pts[i].X.at<float>(k, 0) = xyz[3 * i + (size_t)k];
        pts[i].desc.create(1, 32, orbslam2_amd::kCV_8U);
        std::copy(mpd.begin() + 32 * (long)i, mpd.begin() + 32 * (long)(i + 1), pts[i].desc.data);
        pts[i].extraObs = has[i] == 1 ? 1 : 0;   // 2: a point without observations (temporal)
        if (has[i]) L.mvpMapPoints[i] = &pts[i];
        L.mvbOutlier[i] = outl[i] != 0;
    }
    mock::MapPoint withObs, noObs;
    withObs.extraObs = 1;
    init_slots(C, init, withObs, noObs);
    orbslam2_amd::Matcher matcher(0.9f, true);
    const int32_t n = matcher.SearchByProjection(C, L, th[0], mono[0] != 0);
    wr(out, &n, 1);
    wr(out, read_slots(C, ptr, withObs, noObs));
}

static void run_sbl(FILE* in, FILE* out) {
    mock::Frame F;
    load_frame(in, F);
    F.mvuRight = rd<float>(in);
    set_grid(rd<float>(in));
    const auto inView = rd<uint8_t>(in), bad = rd<uint8_t>(in);
    const auto proj = rd<float>(in);
    const auto level = rd<int32_t>(in);
    const auto vcos = rd<float>(in);
    const auto mpd = rd<uint8_t>(in);
    const auto hasObs = rd<uint8_t>(in);
    F.mvScaleFactors = rd<float>(in);
    const auto th = rd<float>(in), nn = rd<float>(in);
    const auto init = rd<int32_t>(in);
    const size_t nm = inView.size();
    std::vector<mock::MapPoint> pts(nm);
    std::vector<mock::MapPoint*> ptr(nm);
    for (size_t i = 0; i < nm; i++) {
        mock::MapPoint& p = pts[i];
        ptr[i] = &p;
        p.bad = bad[i] != 0;
        p.mbTrackInView = inView[i] != 0;
        p.mTrackProjX = proj[3 * i]; p.mTrackProjY = proj[3 * i + 1]; p.mTrackProjXR = proj[3 * i + 2];
        p.mnTrackScaleLevel = level[i];
        p.mTrackViewCos = vcos[i];
        p.extraObs = hasObs[i] ? 1 : 0;
        p.desc.create(1, 32, orbslam2_amd::kCV_8U);
        std::copy(mpd.begin() + 32 * (long)i, mpd.begin() + 32 * (long)(i + 1), p.desc.data);
    }
    mock::MapPoint withObs, noObs;
    withObs.extraObs = 1;
    init_slots(F, init, withObs, noObs);
    orbslam2_amd::Matcher matcher(nn[0], true);
    const int32_t n = matcher.SearchByProjection(F, ptr, th[0]);
    wr(out, &n, 1);
    wr(out, read_slots(F, ptr, withObs, noObs));
}

static double g_call_us = 0.0;   // wall time of the last timed shim call (timeit mode)
static double g_phase_us[4] = {-1.0, 0.0, 0.0, 0.0};   // the last lba call's phases (LbaDump::phase_us)
static bool g_timing = false;   // timeit: the lba modes call without a dump, as LocalMapping does

// The CPU column of the routed LocalBundleAdjustment row: the same shim gather / write-back around
// the oracle's single-threaded solve (oracle/lba_oracle.h, loaded from $ORB_ORACLE_LIB: the
// reference's LocalMapping thread runs g2o without OpenMP), so GPU and CPU calls compare like for like.
static int oracle_solve(const lba_problem* p, const lba_options* o, const volatile uint8_t* st, lba_result* r) {
    using Fn = int (*)(const lba_problem*, const lba_options*, const volatile uint8_t*, lba_result*);
    static Fn fn = [] {
        const char* path = std::getenv("ORB_ORACLE_LIB");
        void* h = path ? dlopen(path, RTLD_NOW | RTLD_LOCAL) : nullptr;
        if (!h) throw std::runtime_error("lbacpu: set ORB_ORACLE_LIB to oracle/build/liborb_oracle.so");
        Fn f = reinterpret_cast<Fn>(dlsym(h, "oracle_lba_solve"));
        if (!f) throw std::runtime_error("lbacpu: oracle_lba_solve not found");
        return f;
    }();
    // lba_result_t (oracle) is lba_result without the trailing `aborted`, which it signals by returning 1
    const int rc = fn(p, o, st, r);
    if (rc == 1) { r->aborted = 1; return 0; }
    return rc;
}

static void run_lba(FILE* in, FILE* out, bool group, bool cpu = false) {
    mock::g_erase_log.clear();
    const auto Tcw = rd<float>(in);
    const auto fixedCam = rd<uint8_t>(in);
    const auto kfId = rd<int64_t>(in);
    const auto X = rd<float>(in);
    const auto mpId = rd<int64_t>(in);
    const auto ePt = rd<int32_t>(in), eKf = rd<int32_t>(in);
    const auto eObs = rd<float>(in);
    const auto eOct = rd<int32_t>(in);
    const auto cam = rd<float>(in);
    const auto invSig2 = rd<float>(in);
    const auto stopFlag = rd<uint8_t>(in);
    const std::vector<int32_t> devices = group ? rd<int32_t>(in) : std::vector<int32_t>();
    const size_t nk = fixedCam.size(), np = mpId.size(), ne = ePt.size();
    std::vector<mock::KeyFrame> kfs(nk);
    std::vector<mock::MapPoint> mps(np);
    for (size_t k = 0; k < nk; k++) {
        auto& K = kfs[k];
        K.mnId = (unsigned long)kfId[k];
        K.Tcw.create(4, 4, orbslam2_amd::kCV_32F);
        for (int i = 0; i < 16; i++) K.Tcw.at<float>(i / 4, i % 4) = Tcw[16 * k + (size_t)i];
        K.fx = cam[0]; K.fy = cam[1]; K.cx = cam[2]; K.cy = cam[3]; K.mbf = cam[4];
        K.mvInvLevelSigma2 = invSig2;
    }
    for (size_t m = 0; m < np; m++) {
        mps[m].mnId = (unsigned long)mpId[m];
        mps[m].X.create(3, 1, orbslam2_amd::kCV_32F);
        for (int i = 0; i < 3; i++) mps[m].X.at<float>(i, 0) = X[3 * m + (size_t)i];
    }
    for (size_t e = 0; e < ne; e++) {   // keypoint idx = the keyframe's running observation count
        auto& K = kfs[(size_t)eKf[e]];
        const size_t idx = K.mvKeysUn.size();
        K.mvKeysUn.push_back(mock::KeyPoint{{eObs[3 * e], eObs[3 * e + 1]}, 31.f, 0.f, 0.f, eOct[e], -1});
        K.mvuRight.push_back(eObs[3 * e + 2]);
        K.matches.push_back(&mps[(size_t)ePt[e]]);
        mps[(size_t)ePt[e]].obs[&K] = idx;
    }
    // the local window: the first local keyframe plus every other local one as its covisibles
    mock::KeyFrame* pKF = nullptr;
    for (size_t k = 0; k < nk; k++) {
        if (fixedCam[k]) continue;
        if (!pKF) pKF = &kfs[k];
        else pKF->covis.push_back(&kfs[k]);
    }
    if (!pKF) throw std::runtime_error("no local keyframe in the input");
    mock::Map map;
    bool stop = stopFlag[0] != 0;
    orbslam2_amd::LbaDump D;
    orbslam2_amd::LbaDump* dp = g_timing ? nullptr : &D;
    const auto t0 = std::chrono::steady_clock::now();
    if (group)   // the multi-GPU overload: landmarks sharded over the listed devices
        orbslam2_amd::LocalBundleAdjustment(pKF, &stop, &map, std::vector<int>(devices.begin(), devices.end()), dp);
    else if (cpu)
        orbslam2_amd::detail::local_ba(pKF, &stop, &map, dp, oracle_solve);
    else
        orbslam2_amd::LocalBundleAdjustment(pKF, &stop, &map, dp);
    g_call_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    const double* ph = orbslam2_amd::lba_last_phases();
    std::copy(ph, ph + 4, g_phase_us);
    wr(out, D.pose_q); wr(out, D.pose_t); wr(out, D.pose_fixed); wr(out, D.pose_id);
    wr(out, D.point_xyz); wr(out, D.point_id); wr(out, D.point_bad);
    wr(out, D.edge_point); wr(out, D.edge_pose); wr(out, D.edge_stereo); wr(out, D.edge_obs); wr(out, D.edge_info);
    wr(out, D.edge_cam);
    wr(out, D.edge_erase); wr(out, D.out_q); wr(out, D.out_t); wr(out, D.out_xyz);
    const int32_t st[4] = {D.iterations[0], D.iterations[1], D.trials, D.aborted};
    wr(out, st, 4);
    // the write-back as the mock map sees it: keyframe poses (Tcw, input order), point positions and
    // UpdateNormalAndDepth calls, remaining observations
    std::vector<float> Tout;
    for (auto& K : kfs)
        for (int i = 0; i < 16; i++) Tout.push_back(K.Tcw.at<float>(i / 4, i % 4));
    std::vector<float> Xout;
    std::vector<int32_t> upd, nobs;
    for (auto& M : mps) {
        for (int i = 0; i < 3; i++) Xout.push_back(M.X.at<float>(i, 0));
        upd.push_back(M.updates);
        nobs.push_back((int32_t)M.obs.size());
    }
    wr(out, Tout); wr(out, Xout); wr(out, upd); wr(out, nobs);
    std::vector<int64_t> elog;   // EraseMapPointMatch calls in order: keyframe mnId, map point mnId
    for (const auto& e : mock::g_erase_log) { elog.push_back((int64_t)e.first); elog.push_back((int64_t)e.second); }
    wr(out, elog);
}

// ---------------------------------------------------------------- PoseOptimization
// IN: Tcw (16), keypoint x, y, octave, uright, has_mp (uint8), map point xyz (3 per keypoint),
//     mvInvLevelSigma2, cam (fx, fy, cx, cy, bf).  OUT: return value, mvbOutlier (uint8 per
//     keypoint), Tcw after the call.
static void run_pose(FILE* in, FILE* out) {
    const auto T = rd<float>(in);
    const auto x = rd<float>(in), y = rd<float>(in);
    const auto oct = rd<int32_t>(in);
    mock::Frame F;
    F.mvuRight = rd<float>(in);
    const auto has = rd<uint8_t>(in);
    const auto xyz = rd<float>(in);
    F.mvInvLevelSigma2 = rd<float>(in);
    const auto cam = rd<float>(in);
    const size_t n = x.size();
    F.mvKeysUn.resize(n);
    for (size_t i = 0; i < n; i++) F.mvKeysUn[i] = mock::KeyPoint{{x[i], y[i]}, 31.f, 0.f, 0.f, oct[i], -1};
    std::vector<mock::MapPoint> pts(n);
    F.mvpMapPoints.assign(n, nullptr);
    F.mvbOutlier.assign(n, true);   // stale flags: the call resets every edge's
    for (size_t i = 0; i < n; i++) {
        pts[i].X.create(3, 1, orbslam2_amd::kCV_32F);
        for (int k = 0; k < 3; k++) pts[i].X.at<float>(k, 0) = xyz[3 * i + (size_t)k];
        if (has[i]) F.mvpMapPoints[i] = &pts[i];
    }
    F.mTcw.create(4, 4, orbslam2_amd::kCV_32F);
    for (int i = 0; i < 16; i++) F.mTcw.at<float>(i / 4, i % 4) = T[(size_t)i];
    mock::Frame::fx = cam[0]; mock::Frame::fy = cam[1]; mock::Frame::cx = cam[2]; mock::Frame::cy = cam[3];
    F.mbf = cam[4];
    const int32_t r = orbslam2_amd::PoseOptimization(&F);
    wr(out, &r, 1);
    std::vector<uint8_t> o(n);
    for (size_t i = 0; i < n; i++) o[i] = F.mvbOutlier[i] ? 1 : 0;
    wr(out, o);
    std::vector<float> To(16);
    for (int i = 0; i < 16; i++) To[(size_t)i] = F.mTcw.at<float>(i / 4, i % 4);
    wr(out, To);
}

// ---------------------------------------------------------------- stereo Frame
// IN: (w, h, nfeatures), left image, right image, (mbf, mb).  OUT: left keypoints (bytes), left
// descriptors, right keypoints, right descriptors, mvuRight, mvDepth.  The two extractions run on
// two host threads at once, as the stereo Frame constructor does (R/src/Frame.cpp:86-89); the
// extractors persist per calling thread, as Tracking's mpORBextractorLeft / Right do.
struct StereoExtractors {
    int w = 0, h = 0, nf = 0;
    std::unique_ptr<orbslam2_amd::Extractor> L, R;
};
static void run_stereo(FILE* in, FILE* out) {
    const auto whn = rd<int32_t>(in);
    const auto l = rd<uint8_t>(in), r = rd<uint8_t>(in);
    const auto mb = rd<float>(in);
    const int W = whn[0], H = whn[1], NF = whn[2];
    thread_local StereoExtractors tls;
    StereoExtractors& ex = tls;   // (a lambda on another thread must not name the thread_local itself)
    if (!ex.L || ex.w != W || ex.h != H || ex.nf != NF) {
        ex.L.reset(new orbslam2_amd::Extractor(NF, 1.2f, 8, 20, 7, 0, W, H));
        ex.R.reset(new orbslam2_amd::Extractor(NF, 1.2f, 8, 20, 7, 0, W, H));
        ex.w = W; ex.h = H; ex.nf = NF;
    }
    mock::Mat iL(H, W, orbslam2_amd::kCV_8U), iR(H, W, orbslam2_amd::kCV_8U);
    std::copy(l.begin(), l.end(), iL.data);
    std::copy(r.begin(), r.end(), iR.data);
    mock::Frame F;
    std::string errL;
    std::thread tl([&] {
        try { ex.L->extract(iL, F.mvKeys, F.mDescriptors); } catch (const std::exception& e) { errL = e.what(); }
    });
    ex.R->extract(iR, F.mvKeysRight, F.mDescriptorsRight);
    tl.join();
    if (!errL.empty()) throw std::runtime_error(errL);
    F.mbf = mb[0];
    F.mb = mb[1];
    orbslam2_amd::ComputeStereoMatches(F, ex.L->handle(), ex.R->handle());
    wr(out, reinterpret_cast<const uint8_t*>(F.mvKeys.data()), F.mvKeys.size() * sizeof(mock::KeyPoint));
    wr(out, F.mDescriptors.data, (size_t)F.mDescriptors.rows * 32);
    wr(out, reinterpret_cast<const uint8_t*>(F.mvKeysRight.data()), F.mvKeysRight.size() * sizeof(mock::KeyPoint));
    wr(out, F.mDescriptorsRight.data, (size_t)F.mDescriptorsRight.rows * 32);
    wr(out, F.mvuRight);
    wr(out, F.mvDepth);
}

// ---------------------------------------------------------------- keyframes for the LocalMapping /
// LoopClosing matchers.  IN: keypoint x, y, angle, octave, descriptors, mvuRight, grid bounds
// (minX, minY, maxX, maxY, 1/cell w, 1/cell h), Tcw (16), camera centre (3), (fx, fy, cx, cy, bf),
// mfLogScaleFactor, mvScaleFactors, mvInvLevelSigma2, mvLevelSigma2, mFeatVec (node ids, CSR
// starts, feature indices).
static void load_kf(FILE* in, mock::KeyFrame& K) {
    const auto x = rd<float>(in), y = rd<float>(in), a = rd<float>(in);
    const auto o = rd<int32_t>(in);
    const auto d = rd<uint8_t>(in);
    K.mvuRight = rd<float>(in);
    const auto g = rd<float>(in);
    const auto T = rd<float>(in), Ow = rd<float>(in), cam = rd<float>(in), lsf = rd<float>(in);
    K.mvScaleFactors = rd<float>(in);
    K.mvInvLevelSigma2 = rd<float>(in);
    K.mvLevelSigma2 = rd<float>(in);
    const auto nodes = rd<uint32_t>(in);
    const auto start = rd<int32_t>(in), fidx = rd<int32_t>(in);
    const size_t n = x.size();
    K.mvKeysUn.resize(n);
    for (size_t i = 0; i < n; i++) K.mvKeysUn[i] = mock::KeyPoint{{x[i], y[i]}, 31.f, a[i], 0.f, o[i], -1};
    K.mDescriptors.create((int)n, 32, orbslam2_amd::kCV_8U);
    std::copy(d.begin(), d.end(), K.mDescriptors.data);
    K.mnMinX = (int)g[0]; K.mnMinY = (int)g[1]; K.mnMaxX = (int)g[2]; K.mnMaxY = (int)g[3];
    K.mfGridElementWidthInv = g[4]; K.mfGridElementHeightInv = g[5];
    K.Tcw.create(4, 4, orbslam2_amd::kCV_32F);
    for (int i = 0; i < 16; i++) K.Tcw.at<float>(i / 4, i % 4) = T[(size_t)i];
    K.Ow.create(3, 1, orbslam2_amd::kCV_32F);
    for (int i = 0; i < 3; i++) K.Ow.at<float>(i, 0) = Ow[(size_t)i];
    K.fx = cam[0]; K.fy = cam[1]; K.cx = cam[2]; K.cy = cam[3]; K.mbf = cam[4];
    K.mfLogScaleFactor = lsf[0];
    K.mnScaleLevels = (int)K.mvScaleFactors.size();
    for (size_t k = 0; k < nodes.size(); k++)
        for (int j = start[k]; j < start[k + 1]; j++) K.mFeatVec[nodes[k]].push_back((unsigned)fidx[(size_t)j]);
    K.matches.assign(n, nullptr);
}

// map points of a keyframe's slots: IN per keypoint -1 none, 0 a good point, 1 a bad point;
// point i of `pts` sits in slot i (mnId = slot)
static void attach_points(mock::KeyFrame& K, const std::vector<int32_t>& kind, std::vector<mock::MapPoint>& pts) {
    pts.assign(kind.size(), mock::MapPoint());
    for (size_t i = 0; i < kind.size(); i++) {
        pts[i].mnId = i;
        pts[i].bad = kind[i] == 1;
        if (kind[i] >= 0) K.matches[i] = &pts[i];
    }
}

// IN: the keyframe, then per map point xyz, normal, mfMinDistance, mfMaxDistance, descriptor,
// bad flag, observations outside this keyframe, the keyframe slot it already occupies (-1: none),
// then vpMapPoints (point index or -1 = NULL) and th.  Points in a slot are the keyframe's.
// OUT: nFused, per keyframe slot the mnId of its point (-1), per point bad / replaced-by mnId (-1) /
// its slot in the keyframe (-1) / Observations().
static void run_fuse(FILE* in, FILE* out) {
    mock::KeyFrame K;
    load_kf(in, K);
    const auto xyz = rd<float>(in), nrm = rd<float>(in), mind = rd<float>(in), maxd = rd<float>(in);
    const auto desc = rd<uint8_t>(in);
    const auto bad = rd<uint8_t>(in);
    const auto extra = rd<int32_t>(in), slot = rd<int32_t>(in), vec = rd<int32_t>(in);
    const auto th = rd<float>(in);
    const size_t np = bad.size();
    std::vector<mock::MapPoint> pts(np);
    for (size_t i = 0; i < np; i++) {
        mock::MapPoint& P = pts[i];
        P.mnId = i;
        P.X.create(3, 1, orbslam2_amd::kCV_32F);
        P.normal.create(3, 1, orbslam2_amd::kCV_32F);
        for (int k = 0; k < 3; k++) {
            P.X.at<float>(k, 0) = xyz[3 * i + (size_t)k];
            P.normal.at<float>(k, 0) = nrm[3 * i + (size_t)k];
        }
        P.mfMinDistance = mind[i];
        P.mfMaxDistance = maxd[i];
        P.desc.create(1, 32, orbslam2_amd::kCV_8U);
        std::copy(desc.begin() + 32 * (long)i, desc.begin() + 32 * (long)(i + 1), P.desc.data);
        P.bad = bad[i] != 0;
        P.extraObs = extra[i];
        if (slot[i] >= 0) {
            P.obs[&K] = (size_t)slot[i];
            K.matches[(size_t)slot[i]] = &P;
        }
    }
    std::vector<mock::MapPoint*> vp;
    for (const int32_t v : vec) vp.push_back(v < 0 ? nullptr : &pts[(size_t)v]);
    orbslam2_amd::Matcher matcher(0.6f, true);
    const int32_t n = matcher.Fuse(&K, vp, th[0]);
    wr(out, &n, 1);
    std::vector<int32_t> slots;
    for (auto* p : K.matches) slots.push_back(p ? (int32_t)p->mnId : -1);
    wr(out, slots);
    std::vector<int32_t> st;
    for (auto& P : pts) {
        st.push_back(P.bad ? 1 : 0);
        st.push_back(P.replacedBy ? (int32_t)P.replacedBy->mnId : -1);
        st.push_back(P.obs.count(&K) ? (int32_t)P.obs[&K] : -1);
        st.push_back(P.Observations());
    }
    wr(out, st);
}

// IN: keyframe 1, keyframe 2, each followed by its slot kinds (attach_points), then F12 (9),
// bOnlyStereo, checkOri.  OUT: nmatches, vMatchedPairs flattened.
static void run_sft(FILE* in, FILE* out) {
    mock::KeyFrame K1, K2;
    std::vector<mock::MapPoint> p1, p2;
    load_kf(in, K1);
    attach_points(K1, rd<int32_t>(in), p1);
    load_kf(in, K2);
    attach_points(K2, rd<int32_t>(in), p2);
    const auto F = rd<float>(in);
    const auto flags = rd<int32_t>(in);
    mock::Mat F12(3, 3, orbslam2_amd::kCV_32F);
    for (int i = 0; i < 9; i++) F12.at<float>(i / 3, i % 3) = F[(size_t)i];
    orbslam2_amd::Matcher matcher(0.6f, flags[1] != 0);
    std::vector<std::pair<size_t, size_t>> pairs;
    const int32_t n = matcher.SearchForTriangulation(&K1, &K2, F12, pairs, flags[0] != 0);
    wr(out, &n, 1);
    std::vector<int32_t> pv;
    for (const auto& pr : pairs) { pv.push_back((int32_t)pr.first); pv.push_back((int32_t)pr.second); }
    wr(out, pv);
}

// IN: the keyframe + its slot kinds, then the frame's keypoint x, y, angle, octave, descriptors and
// mFeatVec (nodes, starts, indices), then (nnratio, checkOri).  OUT: nmatches, per frame feature
// the keyframe slot whose point it matched (-1).
static void run_sbbf(FILE* in, FILE* out) {
    mock::KeyFrame K;
    std::vector<mock::MapPoint> pk;
    load_kf(in, K);
    attach_points(K, rd<int32_t>(in), pk);
    mock::Frame F;
    load_frame(in, F);
    const auto nodes = rd<uint32_t>(in);
    const auto start = rd<int32_t>(in), fidx = rd<int32_t>(in);
    for (size_t k = 0; k < nodes.size(); k++)
        for (int j = start[k]; j < start[k + 1]; j++) F.mFeatVec[nodes[k]].push_back((unsigned)fidx[(size_t)j]);
    const auto par = rd<float>(in);
    orbslam2_amd::Matcher matcher(par[0], par[1] != 0);
    std::vector<mock::MapPoint*> vm;
    const int32_t n = matcher.SearchByBoW(&K, F, vm);
    wr(out, &n, 1);
    std::vector<int32_t> o;
    for (auto* p : vm) o.push_back(p ? (int32_t)p->mnId : -1);
    wr(out, o);
}

// IN: keyframe 1 + slot kinds, keyframe 2 + slot kinds, (nnratio, checkOri).  OUT: nmatches, per
// keyframe-1 slot the keyframe-2 slot of vpMatches12 (-1).
static void run_sbbk(FILE* in, FILE* out) {
    mock::KeyFrame K1, K2;
    std::vector<mock::MapPoint> p1, p2;
    load_kf(in, K1);
    attach_points(K1, rd<int32_t>(in), p1);
    load_kf(in, K2);
    attach_points(K2, rd<int32_t>(in), p2);
    const auto par = rd<float>(in);
    orbslam2_amd::Matcher matcher(par[0], par[1] != 0);
    std::vector<mock::MapPoint*> vm;
    const int32_t n = matcher.SearchByBoW(&K1, &K2, vm);
    wr(out, &n, 1);
    std::vector<int32_t> o;
    for (auto* p : vm) o.push_back(p ? (int32_t)p->mnId : -1);
    wr(out, o);
}

// map points of a keyframe's slots with their data: IN per slot xyz, normal, mfMinDistance,
// mfMaxDistance, descriptor; point i sits in slot i (mnId = i), observed there
static void point_data(FILE* in, mock::KeyFrame& K, std::vector<mock::MapPoint>& pts) {
    const auto xyz = rd<float>(in), nrm = rd<float>(in), mind = rd<float>(in), maxd = rd<float>(in);
    const auto desc = rd<uint8_t>(in);
    for (size_t i = 0; i < pts.size(); i++) {
        mock::MapPoint& P = pts[i];
        P.mnId = i;
        P.X.create(3, 1, orbslam2_amd::kCV_32F);
        P.normal.create(3, 1, orbslam2_amd::kCV_32F);
        for (int k = 0; k < 3; k++) {
            P.X.at<float>(k, 0) = xyz[3 * i + (size_t)k];
            P.normal.at<float>(k, 0) = nrm.empty() ? 0.f : nrm[3 * i + (size_t)k];
        }
        P.mfMinDistance = mind[i];
        P.mfMaxDistance = maxd[i];
        P.desc.create(1, 32, orbslam2_amd::kCV_8U);
        std::copy(desc.begin() + 32 * (long)i, desc.begin() + 32 * (long)(i + 1), P.desc.data);
        if (K.matches[i] == &P) P.obs[&K] = i;
    }
}
static mock::Mat read_mat(FILE* in, int rows, int cols) {
    const auto v = rd<float>(in);
    if (v.size() != (size_t)(rows * cols)) throw std::runtime_error("bad matrix size");
    mock::Mat m(rows, cols, orbslam2_amd::kCV_32F);
    for (int i = 0; i < rows * cols; i++) m.at<float>(i / cols, i % cols) = v[(size_t)i];
    return m;
}

// IN: the frame (keypoints, descriptors), grid, mTcw (16), (fx, fy, cx, cy), mfLogScaleFactor,
// mvScaleFactors, slot codes (-1 NULL, -2 set), then the keyframe, its slot kinds (-1 none, 0 good,
// 1 bad, 2 good but in sAlreadyFound), the points' data, (th, ORBdist, checkOri).
// OUT: nmatches, per frame slot the keyframe slot of its point (-2 set before, -1 NULL).
static void run_sbpk(FILE* in, FILE* out) {
    mock::Frame F;
    load_frame(in, F);
    set_grid(rd<float>(in));
    F.mTcw = read_mat(in, 4, 4);
    const auto cam = rd<float>(in), lsf = rd<float>(in);
    mock::Frame::fx = cam[0]; mock::Frame::fy = cam[1]; mock::Frame::cx = cam[2]; mock::Frame::cy = cam[3];
    F.mfLogScaleFactor = lsf[0];
    F.mvScaleFactors = rd<float>(in);
    F.mnScaleLevels = (int)F.mvScaleFactors.size();
    const auto init = rd<int32_t>(in);
    mock::KeyFrame K;
    load_kf(in, K);
    auto kind = rd<int32_t>(in);
    std::vector<mock::MapPoint> pts;
    std::vector<int32_t> k01(kind);
    for (auto& k : k01) if (k == 2) k = 0;
    attach_points(K, k01, pts);
    point_data(in, K, pts);
    std::set<mock::MapPoint*> found;
    for (size_t i = 0; i < kind.size(); i++)
        if (kind[i] == 2) found.insert(&pts[i]);
    const auto par = rd<float>(in);
    mock::MapPoint preset;
    F.mvpMapPoints.assign(init.size(), nullptr);
    for (size_t i = 0; i < init.size(); i++)
        if (init[i] == -2) F.mvpMapPoints[i] = &preset;
    orbslam2_amd::Matcher matcher(0.6f, par[2] != 0);
    const int32_t n = matcher.SearchByProjection(F, &K, found, par[0], (int)par[1]);
    wr(out, &n, 1);
    std::vector<int32_t> o;
    for (auto* p : F.mvpMapPoints) o.push_back(!p ? -1 : p == &preset ? -2 : (int32_t)p->mnId);
    wr(out, o);
}

// IN: the keyframe, Scw (16), the points' data (one per vpPoints entry), their bad flags, vpMatched
// on entry per keyframe slot (-1 NULL, -2 a point outside vpPoints, else a vpPoints index), th.
// OUT: nmatches, vpMatched per slot in the same codes.
static void run_sbps(FILE* in, FILE* out) {
    mock::KeyFrame K;
    load_kf(in, K);
    const mock::Mat Scw = read_mat(in, 4, 4);
    const auto bad = rd<uint8_t>(in);
    std::vector<mock::MapPoint> pts(bad.size());
    mock::KeyFrame none;   // the points' data loader attaches nothing to an empty keyframe
    none.matches.assign(pts.size(), nullptr);
    point_data(in, none, pts);
    for (size_t i = 0; i < pts.size(); i++) pts[i].bad = bad[i] != 0;
    const auto pre = rd<int32_t>(in);
    const auto th = rd<int32_t>(in);
    std::vector<mock::MapPoint*> vp;
    for (auto& P : pts) vp.push_back(&P);
    mock::MapPoint foreign;
    std::vector<mock::MapPoint*> vm(pre.size(), nullptr);
    for (size_t i = 0; i < pre.size(); i++) vm[i] = pre[i] == -2 ? &foreign : pre[i] >= 0 ? vp[(size_t)pre[i]] : nullptr;
    orbslam2_amd::Matcher matcher(0.75f, true);
    const int32_t n = matcher.SearchByProjection(&K, Scw, vp, vm, th[0]);
    wr(out, &n, 1);
    std::vector<int32_t> o;
    for (auto* p : vm) o.push_back(!p ? -1 : p == &foreign ? -2 : (int32_t)p->mnId);
    wr(out, o);
}

// IN: keyframe 1, its slot kinds (-1 none, 0 good, 1 bad), its points' data; the same for keyframe 2;
// vpMatches12 on entry per keyframe-1 slot (-1 NULL, -2 a point not in keyframe 2, else the
// keyframe-2 slot whose point it is); s12, R12 (9), t12 (3), th.
// OUT: nFound, vpMatches12 per keyframe-1 slot in the same codes.
static void run_sbs(FILE* in, FILE* out) {
    mock::KeyFrame K1, K2;
    std::vector<mock::MapPoint> p1, p2;
    load_kf(in, K1);
    attach_points(K1, rd<int32_t>(in), p1);
    point_data(in, K1, p1);
    load_kf(in, K2);
    attach_points(K2, rd<int32_t>(in), p2);
    point_data(in, K2, p2);
    const auto pre = rd<int32_t>(in);
    const auto s12 = rd<float>(in);
    const mock::Mat R12 = read_mat(in, 3, 3), t12 = read_mat(in, 3, 1);
    const auto th = rd<float>(in);
    mock::MapPoint foreign;
    std::vector<mock::MapPoint*> vm(pre.size(), nullptr);
    for (size_t i = 0; i < pre.size(); i++) vm[i] = pre[i] == -2 ? &foreign : pre[i] >= 0 ? &p2[(size_t)pre[i]] : nullptr;
    orbslam2_amd::Matcher matcher(0.75f, true);
    const int32_t n = matcher.SearchBySim3(&K1, &K2, vm, s12[0], R12, t12, th[0]);
    wr(out, &n, 1);
    std::vector<int32_t> o;
    for (auto* p : vm) o.push_back(!p ? -1 : p == &foreign ? -2 : (int32_t)p->mnId);
    wr(out, o);
}

// IN: the keyframe, Scw (16), the points' data, bad flags, the keyframe slot each point occupies on
// entry (-1 none; such points are the keyframe's), vpPoints (point indices), th.
// OUT: nFused, per keyframe slot the mnId of its point (-1), vpReplacePoint per vpPoints entry (mnId
// or -1), per point its slot in the keyframe (-1).
static void run_fuses(FILE* in, FILE* out) {
    mock::KeyFrame K;
    load_kf(in, K);
    const mock::Mat Scw = read_mat(in, 4, 4);
    const auto bad = rd<uint8_t>(in);
    std::vector<mock::MapPoint> pts(bad.size());
    mock::KeyFrame none;
    none.matches.assign(pts.size(), nullptr);
    point_data(in, none, pts);
    const auto slot = rd<int32_t>(in), vec = rd<int32_t>(in);
    const auto th = rd<float>(in);
    for (size_t i = 0; i < pts.size(); i++) {
        pts[i].bad = bad[i] != 0;
        if (slot[i] >= 0) {
            pts[i].obs[&K] = (size_t)slot[i];
            K.matches[(size_t)slot[i]] = &pts[i];
        }
    }
    std::vector<mock::MapPoint*> vp;
    for (const int32_t v : vec) vp.push_back(&pts[(size_t)v]);
    std::vector<mock::MapPoint*> repl(vp.size(), nullptr);
    orbslam2_amd::Matcher matcher(0.6f, true);
    const int32_t n = matcher.Fuse(&K, Scw, vp, th[0], repl);
    wr(out, &n, 1);
    std::vector<int32_t> slots, ro, po;
    for (auto* p : K.matches) slots.push_back(p ? (int32_t)p->mnId : -1);
    for (auto* p : repl) ro.push_back(p ? (int32_t)p->mnId : -1);
    for (auto& P : pts) po.push_back(P.obs.count(&K) ? (int32_t)P.obs[&K] : -1);
    wr(out, slots); wr(out, ro); wr(out, po);
}

static bool run_mode(const std::string& mode, FILE* in, FILE* out) {
    if (mode == "extract") run_extract(in, out);
    else if (mode == "sfi") run_sfi(in, out);
    else if (mode == "sbp") run_sbp(in, out);
    else if (mode == "sbl") run_sbl(in, out);
    else if (mode == "lba") run_lba(in, out, false);
    else if (mode == "lbag") run_lba(in, out, true);
    else if (mode == "lbacpu") run_lba(in, out, false, true);
    else if (mode == "pose") run_pose(in, out);
    else if (mode == "stereo") run_stereo(in, out);
    else if (mode == "fuse") run_fuse(in, out);
    else if (mode == "sft") run_sft(in, out);
    else if (mode == "sbbf") run_sbbf(in, out);
    else if (mode == "sbbk") run_sbbk(in, out);
    else if (mode == "sbpk") run_sbpk(in, out);
    else if (mode == "sbps") run_sbps(in, out);
    else if (mode == "sbs") run_sbs(in, out);
    else if (mode == "fuses") run_fuses(in, out);
    else return false;
    return true;
}

// threads OUT REPS MODE1 IN1 [MODE2 IN2 ...]: one host thread per job, released together; each
// runs its job REPS times (inputs re-read, so a mutated mock map starts afresh) and every result
// must equal its first; OUT.k receives job k's first result.  Exit 4 on a differing repetition.
// A mode written "fresh:MODE" runs every repetition on a new host thread, so each call of a
// handle-less entry point creates its per-thread scratch (stream + device buffer, common.h
// host_scratch) while the other jobs — the local BA's graph capture among them — are running.
static int run_threads(int argc, char** argv) {
    const std::string outp = argv[2];
    const int reps = std::atoi(argv[3]);
    struct Job {
        std::string mode, in, err;
        std::vector<uint8_t> first;
        int mismatches = 0;
    };
    std::vector<Job> jobs;
    for (int a = 4; a + 1 < argc; a += 2) jobs.push_back(Job{argv[a], argv[a + 1], "", {}, 0});
    std::atomic<int> ready{0};
    std::vector<std::thread> th;
    for (auto& J : jobs) {
        th.emplace_back([&J, &ready, reps, n = (int)jobs.size()] {
            ready.fetch_add(1);
            while (ready.load() < n) std::this_thread::yield();
            const bool fresh = J.mode.rfind("fresh:", 0) == 0;
            const std::string mode = fresh ? J.mode.substr(6) : J.mode;
            for (int r = 0; r < reps && J.err.empty(); r++) {
                FILE* in = std::fopen(J.in.c_str(), "rb");
                char* buf = nullptr;
                size_t len = 0;
                FILE* mem = open_memstream(&buf, &len);
                auto call = [&] {
                    try {
                        if (!in || !mem || !run_mode(mode, in, mem)) J.err = "bad job " + J.mode;
                    } catch (const std::exception& e) {
                        J.err = e.what();
                    }
                };
                if (fresh) std::thread(call).join();
                else call();
                if (in) std::fclose(in);
                if (mem) std::fclose(mem);
                std::vector<uint8_t> v(buf, buf + len);
                std::free(buf);
                if (!J.err.empty()) break;
                if (r == 0) J.first = v;
                else if (v != J.first) J.mismatches++;
            }
        });
    }
    for (auto& t : th) t.join();
    int rc = 0;
    for (size_t k = 0; k < jobs.size(); k++) {
        const Job& J = jobs[k];
        if (!J.err.empty()) {
            std::fprintf(stderr, "job %zu (%s): %s\n", k, J.mode.c_str(), J.err.c_str());
            rc = 3;
            continue;
        }
        if (J.mismatches) {
            std::fprintf(stderr, "job %zu (%s): %d repetitions differ from the first\n", k, J.mode.c_str(), J.mismatches);
            if (!rc) rc = 4;
        }
        FILE* f = std::fopen((outp + "." + std::to_string(k)).c_str(), "wb");
        if (!f) return 2;
        if (!J.first.empty()) std::fwrite(J.first.data(), 1, J.first.size(), f);
        std::fclose(f);
    }
    return rc;
}

// timeit REPS MODE IN: the mode REPS times (after 3 untimed calls), output discarded; the median and
// minimum of the per-call times the mode recorded
static int run_timeit(int argc, char** argv) {
    if (argc != 5) return 2;
    const int reps = std::atoi(argv[2]);
    const std::string mode = argv[3];
    std::vector<double> ts, ph[4];
    g_timing = true;
    for (int r = 0; r < reps + 3; r++) {
        FILE* in = std::fopen(argv[4], "rb");
        char* buf = nullptr;
        size_t len = 0;
        FILE* mem = open_memstream(&buf, &len);
        if (!in || !mem) return 2;
        g_call_us = -1.0;
        try {
            if (!run_mode(mode, in, mem)) return 2;
        } catch (const std::exception& e) {
            std::fprintf(stderr, "%s\n", e.what());
            return 3;
        }
        std::fclose(in);
        std::fclose(mem);
        std::free(buf);
        if (g_call_us < 0) return 2;   // the mode records no call time
        if (r >= 3) {
            ts.push_back(g_call_us);
            for (int i = 0; i < 4; i++) ph[i].push_back(g_phase_us[i]);
        }
    }
    std::sort(ts.begin(), ts.end());
    std::printf("median_us %.1f min_us %.1f", ts[ts.size() / 2], ts[0]);
    if ((mode == "lba" || mode == "lbacpu") && ph[0][0] >= 0) {   // medians of the phases: gather, arrays, lba_solve, write-back
        for (auto& v : ph) std::sort(v.begin(), v.end());
        std::printf(" phases_us %.1f %.1f %.1f %.1f", ph[0][ph[0].size() / 2], ph[1][ph[1].size() / 2],
                    ph[2][ph[2].size() / 2], ph[3][ph[3].size() / 2]);
    }
    std::printf("\n");
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 2 && std::string(argv[1]) == "timeit") return run_timeit(argc, argv);
    if (argc >= 6 && std::string(argv[1]) == "threads") return run_threads(argc, argv);
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s extract|sfi|sbp|sbl|lba|lbag|pose|stereo|fuse|sft|sbbf|sbbk|sbpk|sbps|sbs|fuses IN OUT\n"
                             "       %s threads OUT REPS MODE IN [MODE IN ...]\n", argv[0], argv[0]);
        return 2;
    }
    FILE* in = std::fopen(argv[2], "rb");
    FILE* out = std::fopen(argv[3], "wb");
    if (!in || !out) return 2;
    const std::string mode = argv[1];
    try {
        if (!run_mode(mode, in, out)) return 2;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        std::fclose(out);
        return 3;
    }
    std::fclose(in);
    std::fclose(out);
    return 0;
}
