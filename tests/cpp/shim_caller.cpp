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
// IN / OUT: little-endian arrays, each written as int64 element count + raw elements.
// Exit status: 0 ok, 3 the library reported an error (e.g. no gfx950 device), 2 bad usage.
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
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

struct MapPoint;
struct Frame {
    std::vector<KeyPoint> mvKeysUn;
    Mat mDescriptors;
    std::vector<float> mvuRight;
    std::vector<MapPoint*> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    std::vector<float> mvScaleFactors;
    Mat mTcw;
    float mbf = 0, mb = 0;
    static float mnMinX, mnMinY, mnMaxX, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv;
    static float fx, fy, cx, cy;
};
float Frame::mnMinX, Frame::mnMinY, Frame::mnMaxX, Frame::mnMaxY, Frame::mfGridElementWidthInv,
    Frame::mfGridElementHeightInv, Frame::fx, Frame::fy, Frame::cx, Frame::cy;

// the order of KeyFrame::EraseMapPointMatch calls (keyframe mnId, map point mnId)
std::vector<std::pair<unsigned long, unsigned long>> g_erase_log;
struct KeyFrame {
    unsigned long mnId = 0, mnBALocalForKF = 0, mnBAFixedForKF = 0;
    bool bad = false;
    std::vector<KeyFrame*> covis;
    std::vector<MapPoint*> matches;
    Mat Tcw;
    std::vector<KeyPoint> mvKeysUn;
    std::vector<float> mvuRight, mvInvLevelSigma2;
    float fx = 0, fy = 0, cx = 0, cy = 0, mbf = 0;
    std::vector<KeyFrame*> GetVectorCovisibleKeyFrames() { return covis; }
    std::vector<MapPoint*> GetMapPointMatches() { return matches; }
    bool isBad() const { return bad; }
    Mat GetPose() { return Tcw; }
    void SetPose(const Mat& T) { Tcw = T; }
    void EraseMapPointMatch(MapPoint* p);
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
};
inline void KeyFrame::EraseMapPointMatch(MapPoint* p) {
    g_erase_log.emplace_back(mnId, p->mnId);
    for (auto& m : matches)
        if (m == p) m = nullptr;
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

static void run_lba(FILE* in, FILE* out, bool group) {
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
    if (group)   // the multi-GPU overload: landmarks sharded over the listed devices
        orbslam2_amd::LocalBundleAdjustment(pKF, &stop, &map, std::vector<int>(devices.begin(), devices.end()), &D);
    else
        orbslam2_amd::LocalBundleAdjustment(pKF, &stop, &map, &D);
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

int main(int argc, char** argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s extract|sfi|sbp|sbl|lba|lbag IN OUT\n", argv[0]);
        return 2;
    }
    FILE* in = std::fopen(argv[2], "rb");
    FILE* out = std::fopen(argv[3], "wb");
    if (!in || !out) return 2;
    const std::string mode = argv[1];
    try {
        if (mode == "extract") run_extract(in, out);
        else if (mode == "sfi") run_sfi(in, out);
        else if (mode == "sbp") run_sbp(in, out);
        else if (mode == "sbl") run_sbl(in, out);
        else if (mode == "lba") run_lba(in, out, false);
        else if (mode == "lbag") run_lba(in, out, true);
        else return 2;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        std::fclose(out);
        return 3;
    }
    std::fclose(in);
    std::fclose(out);
    return 0;
}
