"""Host mirror of ORB_SLAM2::ORBmatcher (R/include/ORBmatcher.h:37-143) over
the HIP C-ABI: DescriptorDistance, SearchForInitialization,
SearchByProjection(Frame&, const Frame&, th, bMono),
SearchByProjection(Frame&, const vector<MapPoint*>&, th) and a brute-force 2-NN."""
import ctypes as C
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _abi

FRAME_GRID_COLS = 64
FRAME_GRID_ROWS = 48


@dataclass
class Frame:
    """The subset of ORB_SLAM2::Frame the matcher reads (R/include/Frame.h)."""
    mvKeysUn: np.ndarray                 # KEYPOINT_DTYPE
    mDescriptors: np.ndarray             # [N, 32] uint8
    width: int = 640
    height: int = 480
    mvuRight: Optional[np.ndarray] = None
    mnMinX: float = 0.0
    mnMinY: float = 0.0
    mnMaxX: Optional[float] = None
    mnMaxY: Optional[float] = None
    mTcw: Optional[np.ndarray] = None    # 4x4 float32
    mvScaleFactors: Optional[np.ndarray] = None
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        if self.mnMaxX is None:
            self.mnMaxX = float(self.width)
        if self.mnMaxY is None:
            self.mnMaxY = float(self.height)

    @property
    def N(self):
        return len(self.mvKeysUn)

    def view(self):
        """orb_frame_view; keeps the arrays alive on the returned object.  Built once per frame and
        reused while the frame's keypoint / descriptor / uRight arrays and bounds are the same objects
        and values (a Frame's keypoints do not change after construction, R/src/Frame.cpp:60-180);
        assigning new arrays rebuilds it."""
        key = (id(self.mvKeysUn), id(self.mDescriptors), id(self.mvuRight), self.mnMinX, self.mnMinY, self.mnMaxX,
               self.mnMaxY, self.N)
        cached = self.__dict__.get("_view")
        if cached is not None and cached[0] == key:
            return cached[1]
        v = self._build_view()
        self.__dict__["_view"] = (key, v)
        return v

    def _build_view(self):
        k = self.mvKeysUn
        x = np.ascontiguousarray(k["x"], np.float32)
        y = np.ascontiguousarray(k["y"], np.float32)
        a = np.ascontiguousarray(k["angle"], np.float32)
        o = np.ascontiguousarray(k["octave"], np.int32)
        d = np.ascontiguousarray(self.mDescriptors, np.uint8)
        ur = None if self.mvuRight is None else np.ascontiguousarray(self.mvuRight, np.float32)
        winv = np.float32(FRAME_GRID_COLS) / np.float32(self.mnMaxX - self.mnMinX)
        hinv = np.float32(FRAME_GRID_ROWS) / np.float32(self.mnMaxY - self.mnMinY)
        v = _abi.FrameView(len(x), _abi.ptr(x), _abi.ptr(y), _abi.ptr(a), _abi.ptr(o), _abi.ptr(d), _abi.ptr(ur),
                           self.mnMinX, self.mnMinY, self.mnMaxX, self.mnMaxY, float(winv), float(hinv))
        v._keep = (x, y, a, o, d, ur)
        return v


@dataclass
class LocalMapPoints:
    """What SearchByProjection(Frame&, vector<MapPoint*>, th) reads of each local map point
    after Frame::isInFrustum (R/src/Frame.cpp:307-376), in vector order."""
    in_view: np.ndarray      # mbTrackInView && !isBad()   [n] bool
    proj: np.ndarray         # mTrackProjX, mTrackProjY, mTrackProjXR   [n, 3] float32
    level: np.ndarray        # mnTrackScaleLevel   [n] int32
    view_cos: np.ndarray     # mTrackViewCos   [n] float32
    desc: np.ndarray         # GetDescriptor()   [n, 32] uint8
    has_obs: np.ndarray      # Observations() > 0   [n] bool

    def __len__(self):
        return len(self.in_view)


def _featvec(fv):
    """A DBoW2 FeatureVector as (node ids uint32 ascending, CSR start int32, feature indices int32):
    accepts that tuple or the node -> feature-list dict of ORBVocabulary.transform."""
    if isinstance(fv, dict):
        keys = sorted(fv)
        start = np.zeros(len(keys) + 1, np.int32)
        start[1:] = np.cumsum([len(fv[k]) for k in keys])
        idx = np.array([i for k in keys for i in fv[k]], np.int32)
        return np.array(keys, np.uint32), start, idx
    return tuple(np.ascontiguousarray(x, t) for x, t in zip(fv, (np.uint32, np.int32, np.int32)))


class ORBmatcher:
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0):
        self.mfNNratio, self.mbCheckOrientation = float(nnratio), bool(checkOri)
        self.device = device
        h = C.c_void_p()
        _abi.check("orb_matcher_create", _abi.lib().orb_matcher_create(device, C.c_float(nnratio), int(checkOri),
                                                                        C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _abi.lib().orb_matcher_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @staticmethod
    def DescriptorDistance(a, b) -> int:
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return _abi.check("orb_descriptor_distance", _abi.lib().orb_descriptor_distance(_abi.ptr(a), _abi.ptr(b)))

    def SearchForInitialization(self, F1: Frame, F2: Frame, vbPrevMatched: np.ndarray, windowSize: int = 10):
        """Returns (nmatches, vnMatches12); vbPrevMatched ([N1, 2] float32) is updated in place."""
        prev = np.ascontiguousarray(vbPrevMatched, np.float32)
        m12 = np.zeros(F1.N, np.int32)
        v1, v2 = F1.view(), F2.view()
        n = _abi.check("orb_search_for_initialization", _abi.lib().orb_search_for_initialization(
            self._h, C.byref(v1), C.byref(v2), _abi.ptr(prev), _abi.ptr(m12), int(windowSize)))
        if prev is not vbPrevMatched:
            vbPrevMatched[...] = prev
        return n, m12

    def SearchByProjection(self, CurrentFrame: Frame, LastFrame: Frame, th: float, bMono: bool,
                           last_has_mp, last_outlier, last_mp_xyz, last_mp_desc, cam, cur_mp=None):
        """SearchByProjection(Frame&, const Frame&, th, bMono).  Map points of the last
        frame are passed explicitly per last keypoint; returns (nmatches, cur_mp) where
        cur_mp[i2] = index of the last-frame keypoint whose map point was assigned."""
        if cur_mp is None:
            cur_mp = np.full(CurrentFrame.N, -1, np.int32)
        cur_mp = np.ascontiguousarray(cur_mp, np.int32).copy()
        vc, vl = CurrentFrame.view(), LastFrame.view()
        Tc = np.ascontiguousarray(np.asarray(CurrentFrame.mTcw, np.float32)[:3, :4])
        Tl = np.ascontiguousarray(np.asarray(LastFrame.mTcw, np.float32)[:3, :4])
        has = np.ascontiguousarray(last_has_mp, np.int32)
        out = np.ascontiguousarray(last_outlier, np.uint8)
        xyz = np.ascontiguousarray(last_mp_xyz, np.float32)
        md = np.ascontiguousarray(last_mp_desc, np.uint8)
        sf = np.ascontiguousarray(CurrentFrame.mvScaleFactors, np.float32)
        camv = np.ascontiguousarray(cam, np.float32)
        n = _abi.check("orb_search_by_projection_frame", _abi.lib().orb_search_by_projection_frame(
            self._h, C.byref(vc), _abi.ptr(Tc), C.byref(vl), _abi.ptr(Tl), _abi.ptr(has), _abi.ptr(out),
            _abi.ptr(xyz), _abi.ptr(md), _abi.ptr(sf), _abi.ptr(camv), C.c_float(th), int(bMono),
            _abi.ptr(cur_mp)))
        return n, cur_mp

    def SearchByProjectionKF(self, CurrentFrame: Frame, pKF: Frame, mp_valid, mp_xyz, mp_min_dist, mp_max_dist,
                             mp_desc, cam, Ow, log_scale_factor, th: float, ORBdist: int, cur_mp=None):
        """SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound,
        th, ORBdist) (R/src/ORBmatcher.cpp:1719-1800).  Keyframe map points per keyframe keypoint
        (mp_valid = set, not bad, not in sAlreadyFound; mfMinDistance / mfMaxDistance); cam =
        (fx, fy, cx, cy); Ow = the frame's camera centre.  cur_mp: -1 empty, -2 already set.
        Returns (nmatches, cur_mp) with cur_mp[i2] = the keyframe map point index assigned."""
        if cur_mp is None:
            cur_mp = np.full(CurrentFrame.N, -1, np.int32)
        cur_mp = np.ascontiguousarray(cur_mp, np.int32).copy()
        vc, vk = CurrentFrame.view(), pKF.view()
        Tc = np.ascontiguousarray(np.asarray(CurrentFrame.mTcw, np.float32)[:3, :4])
        a = [np.ascontiguousarray(x, t) for x, t in ((mp_valid, np.uint8), (mp_xyz, np.float32),
                                                      (mp_min_dist, np.float32), (mp_max_dist, np.float32),
                                                      (mp_desc, np.uint8))]
        sf = np.ascontiguousarray(CurrentFrame.mvScaleFactors, np.float32)
        camv = np.ascontiguousarray(np.asarray(cam, np.float32)[:4])
        ow = np.ascontiguousarray(Ow, np.float32)
        lib = _abi.lib()
        vp = C.c_void_p
        _abi.sig(lib.orb_search_by_projection_kf, [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, C.c_float, C.c_int, vp,
                                                    C.c_float, C.c_int, vp], C.c_int)
        n = _abi.check("orb_search_by_projection_kf", lib.orb_search_by_projection_kf(
            self._h, C.byref(vc), _abi.ptr(Tc), _abi.ptr(ow), C.byref(vk), *[_abi.ptr(x) for x in a], _abi.ptr(camv),
            float(np.float32(log_scale_factor)), len(sf), _abi.ptr(sf), float(th), int(ORBdist), _abi.ptr(cur_mp)))
        return n, cur_mp

    def SearchByProjectionSim3(self, pKF: Frame, Tcw, Ow, cam, log_scale_factor, scale_factors, mp_valid, mp_xyz,
                               mp_normal, mp_min_dist, mp_max_dist, mp_desc, th: float, matched=None):
        """SearchByProjection(KeyFrame* pKF, cv::Mat Scw, vpPoints, vpMatched, th)
        (R/src/ORBmatcher.cpp:370-497).  Tcw = [Rcw | tcw] with the Sim3 scale removed and Ow =
        -Rcw^T tcw as the reference derives them from Scw; cam = (fx, fy, cx, cy); points as for
        Fuse (mp_valid = not bad and not already matched).  matched: -1 empty, -2 set before.
        Returns (nmatches, matched) with matched[idx] = the vpPoints index assigned."""
        matched = np.full(pKF.N, -1, np.int32) if matched is None else np.ascontiguousarray(matched, np.int32).copy()
        sf = np.ascontiguousarray(scale_factors, np.float32)
        kp = KfParams((C.c_float * 12)(*np.asarray(Tcw, np.float32).reshape(-1)[:12]),
                      (C.c_float * 3)(*np.asarray(Ow, np.float32)), *[float(np.float32(v)) for v in cam[:4]], 0.0,
                      float(np.float32(log_scale_factor)), len(sf), _abi.ptr(sf), None)
        a = [np.ascontiguousarray(x, t) for x, t in ((mp_valid, np.uint8), (mp_xyz, np.float32), (mp_normal, np.float32),
                                                      (mp_min_dist, np.float32), (mp_max_dist, np.float32),
                                                      (mp_desc, np.uint8))]
        v = pKF.view()
        lib = _abi.lib()
        vp = C.c_void_p
        _abi.sig(lib.orb_search_by_projection_sim3, [vp, vp, vp, C.c_int, vp, vp, vp, vp, vp, vp, C.c_float, vp], C.c_int)
        n = _abi.check("orb_search_by_projection_sim3", lib.orb_search_by_projection_sim3(
            self._h, C.byref(v), C.byref(kp), len(a[0]), *[_abi.ptr(x) for x in a], float(th), _abi.ptr(matched)))
        return n, matched

    def SearchByProjectionLocal(self, F: Frame, vpMapPoints: LocalMapPoints, th: float = 3.0, cur_mp=None):
        """SearchByProjection(Frame&, const vector<MapPoint*>&, th).  cur_mp mirrors
        F.mvpMapPoints (-1 empty, -2 map point with observations, -3 without); returns
        (nmatches, cur_mp) with matched slots set to the map point index."""
        if cur_mp is None:
            cur_mp = np.full(F.N, -1, np.int32)
        cur_mp = np.ascontiguousarray(cur_mp, np.int32).copy()
        v = F.view()
        mp = vpMapPoints
        arrs = [np.ascontiguousarray(mp.in_view, np.uint8), np.ascontiguousarray(mp.proj, np.float32),
                np.ascontiguousarray(mp.level, np.int32), np.ascontiguousarray(mp.view_cos, np.float32),
                np.ascontiguousarray(mp.desc, np.uint8), np.ascontiguousarray(mp.has_obs, np.uint8),
                np.ascontiguousarray(F.mvScaleFactors, np.float32)]
        n = _abi.check("orb_search_by_projection_local", _abi.lib().orb_search_by_projection_local(
            self._h, C.byref(v), len(mp), *[_abi.ptr(a) for a in arrs], C.c_float(th), _abi.ptr(cur_mp)))
        return n, cur_mp

    def SearchByBoW(self, pKF: Frame, kf_ok, kf_featvec, F: Frame, f_featvec):
        """SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches)
        (R/src/ORBmatcher.cpp:220-372) on the GPU.  kf_ok[i]: the keyframe's map point i is set
        and not bad; featvecs as (node ids ascending, CSR start, feature indices) or the dict
        ORBVocabulary.transform returns.  Returns (nmatches, matches) — per frame feature the
        keyframe feature whose map point it takes, -1 for none."""
        fk, ff = _featvec(kf_featvec), _featvec(f_featvec)
        ok = np.ascontiguousarray(kf_ok, np.uint8)
        m = np.zeros(F.N, np.int32)
        v1, v2 = pKF.view(), F.view()
        lib = _abi.lib()
        vp = C.c_void_p
        _abi.sig(lib.orb_search_by_bow_frame, [C.c_int, vp, vp, C.c_int, vp, vp, vp, vp, C.c_int, vp, vp, vp,
                                                C.c_float, C.c_int, vp], C.c_int)
        n = _abi.check("orb_search_by_bow_frame", lib.orb_search_by_bow_frame(
            self.device, C.byref(v1), _abi.ptr(ok), len(fk[0]), *[_abi.ptr(x) for x in fk], C.byref(v2), len(ff[0]),
            *[_abi.ptr(x) for x in ff], self.mfNNratio, int(self.mbCheckOrientation), _abi.ptr(m)))
        return n, m

    def SearchByBoWKF(self, pKF1: Frame, ok1, featvec1, pKF2: Frame, ok2, featvec2):
        """SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12)
        (R/src/ORBmatcher.cpp:632-760) on the GPU.  okN[i]: keyframe N's map point i is set and
        not bad.  Returns (nmatches, matches12) — per keyframe-1 feature the keyframe-2 feature
        whose map point becomes vpMatches12[i], -1 for none."""
        f1, f2 = _featvec(featvec1), _featvec(featvec2)
        o1, o2 = np.ascontiguousarray(ok1, np.uint8), np.ascontiguousarray(ok2, np.uint8)
        m = np.zeros(pKF1.N, np.int32)
        v1, v2 = pKF1.view(), pKF2.view()
        lib = _abi.lib()
        vp = C.c_void_p
        _abi.sig(lib.orb_search_by_bow_kf, [C.c_int, vp, vp, C.c_int, vp, vp, vp, vp, vp, C.c_int, vp, vp, vp,
                                             C.c_float, C.c_int, vp], C.c_int)
        n = _abi.check("orb_search_by_bow_kf", lib.orb_search_by_bow_kf(
            self.device, C.byref(v1), _abi.ptr(o1), len(f1[0]), *[_abi.ptr(x) for x in f1], C.byref(v2),
            _abi.ptr(o2), len(f2[0]), *[_abi.ptr(x) for x in f2], self.mfNNratio, int(self.mbCheckOrientation),
            _abi.ptr(m)))
        return n, m

    def knn2(self, q, t):
        q = np.ascontiguousarray(q, np.uint8)
        t = np.ascontiguousarray(t, np.uint8)
        bi, bd, sd = (np.zeros(len(q), np.int32) for _ in range(3))
        _abi.check("orb_hamming_knn2", _abi.lib().orb_hamming_knn2(
            self._h, _abi.ptr(q), len(q), _abi.ptr(t), len(t), _abi.ptr(bi), _abi.ptr(bd), _abi.ptr(sd)))
        return bi, bd, sd


def ComputeDistinctiveDescriptors(descriptor_lists, device=0):
    """MapPoint::ComputeDistinctiveDescriptors (R/src/MapPoint.cpp:306-385) for a batch of map
    points on the GPU.  descriptor_lists: per map point an (N, 32) uint8 array of its observed
    descriptors (mObservations order, non-bad keyframes).  Returns (best index per point, -1 for
    an empty list; the chosen 32-byte descriptors, (M, 32))."""
    lists = [np.ascontiguousarray(np.asarray(d, np.uint8).reshape(-1, 32)) for d in descriptor_lists]
    M = len(lists)
    start = np.zeros(M + 1, np.int32)
    start[1:] = np.cumsum([len(d) for d in lists])
    desc = np.ascontiguousarray(np.concatenate(lists) if M and start[-1] else np.zeros((0, 32), np.uint8))
    best = np.zeros(M, np.int32)
    out = np.zeros((M, 32), np.uint8)
    lib = _abi.lib()
    _abi.sig(lib.orb_distinctive_descriptors, [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p], C.c_int)
    _abi.check("orb_distinctive_descriptors",
               lib.orb_distinctive_descriptors(device, _abi.ptr(desc), _abi.ptr(start), M, _abi.ptr(best), _abi.ptr(out)))
    return best, out


class KfParams(C.Structure):
    _fields_ = [("Tcw", C.c_float * 12), ("Ow", C.c_float * 3), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float), ("log_scale_factor", C.c_float),
                ("n_levels", C.c_int), ("scale_factors", C.c_void_p), ("inv_level_sigma2", C.c_void_p)]


def FuseSim3(kf: Frame, Tcw, Ow, cam, log_scale_factor, scale_factors, mp_valid, mp_xyz, mp_normal, mp_min_dist,
             mp_max_dist, mp_desc, th=4.0, device=0):
    """ORBmatcher::Fuse(KeyFrame* pKF, cv::Mat Scw, vpPoints, th, vpReplacePoint) matching step
    (R/src/ORBmatcher.cpp:1164-1261) on the GPU: Tcw = [Rcw | tcw] with the Sim3 scale removed,
    Ow = -Rcw^T tcw, cam = (fx, fy, cx, cy); mp_valid = not bad and not among the keyframe's map
    points.  Returns (best_idx, best_dist) per point; the replace / add step stays with the caller."""
    return _fuse("orb_fuse_sim3", kf, Tcw, Ow, tuple(cam[:4]) + (0.0,), log_scale_factor, scale_factors, None, mp_valid,
                 mp_xyz, mp_normal, mp_min_dist, mp_max_dist, mp_desc, th, device)


def Fuse(kf: Frame, Tcw, Ow, cam, log_scale_factor, scale_factors, inv_level_sigma2, mp_valid, mp_xyz, mp_normal,
         mp_min_dist, mp_max_dist, mp_desc, th=3.0, device=0):
    """ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, float th) matching step
    (R/src/ORBmatcher.cpp:995-1121) on the GPU: per map point the keyframe keypoint it fuses into
    (-1 = none) and the distance.  kf: the keyframe as a Frame (mvKeysUn, mDescriptors, mvuRight,
    bounds); Tcw 3x4 float, Ow = camera centre, cam = (fx, fy, cx, cy, mbf)."""
    return _fuse("orb_fuse", kf, Tcw, Ow, cam, log_scale_factor, scale_factors, inv_level_sigma2, mp_valid, mp_xyz,
                 mp_normal, mp_min_dist, mp_max_dist, mp_desc, th, device)


def _fuse(entry, kf, Tcw, Ow, cam, log_scale_factor, scale_factors, inv_level_sigma2, mp_valid, mp_xyz, mp_normal,
          mp_min_dist, mp_max_dist, mp_desc, th, device):
    sf = np.ascontiguousarray(scale_factors, np.float32)
    isg = None if inv_level_sigma2 is None else np.ascontiguousarray(inv_level_sigma2, np.float32)
    kp = KfParams((C.c_float * 12)(*np.asarray(Tcw, np.float32).reshape(-1)[:12]),
                  (C.c_float * 3)(*np.asarray(Ow, np.float32)), *[float(np.float32(v)) for v in cam],
                  float(np.float32(log_scale_factor)), len(sf), _abi.ptr(sf), _abi.ptr(isg))
    a = [np.ascontiguousarray(x, t) for x, t in ((mp_valid, np.uint8), (mp_xyz, np.float32), (mp_normal, np.float32),
                                                  (mp_min_dist, np.float32), (mp_max_dist, np.float32),
                                                  (mp_desc, np.uint8))]
    n = len(a[0])
    bi, bd = np.zeros(n, np.int32), np.zeros(n, np.int32)
    v = kf.view()
    lib = _abi.lib()
    fn = getattr(lib, entry)
    _abi.sig(fn, [C.c_int, C.c_void_p, C.c_void_p, C.c_int] + [C.c_void_p] * 6 + [C.c_float, C.c_void_p, C.c_void_p], C.c_int)
    _abi.check(entry, fn(device, C.byref(v), C.byref(kp), n, *[_abi.ptr(x) for x in a], th, _abi.ptr(bi),
                         _abi.ptr(bd)))
    return bi, bd


class Sim3Points(C.Structure):
    _fields_ = [("Tcw", C.c_float * 12), ("S", C.c_float * 12), ("n", C.c_int), ("valid", C.c_void_p),
                ("xyz", C.c_void_p), ("min_dist", C.c_void_p), ("max_dist", C.c_void_p), ("desc", C.c_void_p)]


class ScaleParams(C.Structure):
    _fields_ = [("log_scale_factor", C.c_float), ("n_levels", C.c_int), ("scale_factors", C.c_void_p)]


def SearchBySim3(kf1: Frame, kf2: Frame, pts1, pts2, cam1, scale1, scale2, th=7.5, device=0):
    """ORBmatcher::SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th)
    (R/src/ORBmatcher.cpp:1305-1503) on the GPU.  ptsN: dict with Tcw ([R|t] world -> camera N),
    S ([sR|t] camera N -> the other camera, as the reference computes sR21 / t21 and sR12 / t12) and
    per keypoint valid / xyz / min_dist / max_dist / desc of its map point; cam1 = pKF1's (fx, fy,
    cx, cy); scaleN = (mfLogScaleFactor, mvScaleFactors).  Returns (nFound, matches12)."""
    keep = []

    def side(p):
        a = [np.ascontiguousarray(p[f], t) for f, t in (("valid", np.uint8), ("xyz", np.float32),
                                                        ("min_dist", np.float32), ("max_dist", np.float32),
                                                        ("desc", np.uint8))]
        keep.extend(a)
        return Sim3Points((C.c_float * 12)(*np.asarray(p["Tcw"], np.float32).reshape(-1)[:12]),
                          (C.c_float * 12)(*np.asarray(p["S"], np.float32).reshape(-1)[:12]), len(a[0]),
                          *[_abi.ptr(x) for x in a])

    def scale(sc):
        sf = np.ascontiguousarray(sc[1], np.float32)
        keep.append(sf)
        return ScaleParams(float(np.float32(sc[0])), len(sf), _abi.ptr(sf))
    p1, p2 = side(pts1), side(pts2)
    s1, s2 = scale(scale1), scale(scale2)
    cam = np.ascontiguousarray(np.asarray(cam1, np.float32)[:4])
    m = np.zeros(kf1.N, np.int32)
    v1, v2 = kf1.view(), kf2.view()
    lib = _abi.lib()
    vp = C.c_void_p
    _abi.sig(lib.orb_search_by_sim3, [C.c_int, vp, vp, vp, vp, vp, vp, vp, C.c_float, vp], C.c_int)
    n = _abi.check("orb_search_by_sim3", lib.orb_search_by_sim3(
        device, C.byref(v1), C.byref(v2), C.byref(p1), C.byref(p2), _abi.ptr(cam), C.byref(s1), C.byref(s2),
        float(th), _abi.ptr(m)))
    return n, m


def SearchForTriangulation(kf1: Frame, kf2: Frame, has_mp1, has_mp2, featvec1, featvec2, F12, epipole,
                           scale_factors2, level_sigma2, bOnlyStereo=False, checkOri=True, device=0):
    """ORBmatcher::SearchForTriangulation (R/src/ORBmatcher.cpp:785-983) on the GPU.
    featvecN = (node ids ascending, CSR start, feature indices) of pKF->mFeatVec; F12 3x3 float;
    epipole = (ex, ey).  Returns (nmatches, matches12) — vMatchedPairs = [(i, matches12[i]) for
    matches12[i] >= 0]."""
    v1, v2 = kf1.view(), kf2.view()
    fv = [tuple(np.ascontiguousarray(x, t) for x, t in zip(f, (np.uint32, np.int32, np.int32))) for f in (featvec1, featvec2)]
    hm1, hm2 = np.ascontiguousarray(has_mp1, np.uint8), np.ascontiguousarray(has_mp2, np.uint8)
    F = np.ascontiguousarray(np.asarray(F12, np.float32).reshape(-1))
    sf = np.ascontiguousarray(scale_factors2, np.float32)
    s2 = np.ascontiguousarray(level_sigma2, np.float32)
    m = np.zeros(kf1.N, np.int32)
    lib = _abi.lib()
    vp = C.c_void_p
    _abi.sig(lib.orb_search_for_triangulation, [C.c_int, vp, vp, vp, vp, C.c_int, vp, vp, vp, C.c_int, vp, vp, vp, vp,
                                                 C.c_float, C.c_float, vp, vp, C.c_int, C.c_int, C.c_int, vp], C.c_int)
    n = _abi.check("orb_search_for_triangulation", lib.orb_search_for_triangulation(
        device, C.byref(v1), C.byref(v2), _abi.ptr(hm1), _abi.ptr(hm2), len(fv[0][0]), *[_abi.ptr(x) for x in fv[0]],
        len(fv[1][0]), *[_abi.ptr(x) for x in fv[1]], _abi.ptr(F), float(epipole[0]), float(epipole[1]), _abi.ptr(sf),
        _abi.ptr(s2), len(sf), int(bOnlyStereo), int(checkOri), _abi.ptr(m)))
    return n, m
