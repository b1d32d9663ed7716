"""Host mirror of ORB_SLAM2::ORBextractor (R/include/ORBextractor.h:45-123) over
the HIP C-ABI.  Same constructor arguments, same call semantics
(R/src/ORBextractor.cpp:1120-1188), same getters and the public image pyramid."""
import ctypes as C

import numpy as np

from . import _abi


class ORBextractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)."""

    def __init__(self, nfeatures: int, scaleFactor: float, nlevels: int, iniThFAST: int, minThFAST: int,
                 device: int = 0, max_w: int = 1280, max_h: int = 1024, max_batch: int = 1):
        self.nfeatures, self.scaleFactor, self.nlevels = int(nfeatures), float(scaleFactor), int(nlevels)
        self.iniThFAST, self.minThFAST = int(iniThFAST), int(minThFAST)
        p = _abi.ExtractorParams(self.nfeatures, self.scaleFactor, self.nlevels, self.iniThFAST, self.minThFAST)
        h = C.c_void_p()
        _abi.check("orb_extractor_create",
                   _abi.lib().orb_extractor_create(C.byref(p), device, max_w, max_h, max_batch, C.byref(h)))
        self._h = h
        self.last_shape = None

    def close(self):
        if getattr(self, "_h", None):
            _abi.lib().orb_extractor_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    # ---- getters (R/include/ORBextractor.h:66-86)
    def _tables(self):
        n = self.nlevels
        s, inv, s2, inv2 = (np.zeros(n, np.float32) for _ in range(4))
        _abi.check("orb_extractor_scale_tables", _abi.lib().orb_extractor_scale_tables(
            self._h, _abi.ptr(s), _abi.ptr(inv), _abi.ptr(s2), _abi.ptr(inv2)))
        return s, inv, s2, inv2

    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return self.scaleFactor

    def GetScaleFactors(self):
        return self._tables()[0]

    def GetInverseScaleFactors(self):
        return self._tables()[1]

    def GetScaleSigmaSquares(self):
        return self._tables()[2]

    def GetInverseScaleSigmaSquares(self):
        return self._tables()[3]

    def GetFeaturesPerLevel(self):
        out = np.zeros(self.nlevels, np.int32)
        _abi.check("orb_extractor_features_per_level",
                   _abi.lib().orb_extractor_features_per_level(self._h, _abi.ptr(out)))
        return out

    # ---- operator()
    def __call__(self, image, mask=None, keypoints=None, descriptors=None):
        """Returns (keypoints[N] structured array, descriptors[N, 32] uint8).
        An empty image returns (keypoints, descriptors) unchanged (None if not given)."""
        img = None if image is None else np.asarray(image)
        if img is None or img.size == 0:
            return keypoints, descriptors
        if img.dtype != np.uint8 or img.ndim != 2:
            raise ValueError("ORBextractor expects an 8-bit single-channel image (CV_8UC1)")
        img = np.ascontiguousarray(img)
        h, w = img.shape
        cap = max(4 * self.nfeatures + 64, 64)
        while True:
            kps = np.zeros(cap, _abi.KEYPOINT_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            n = C.c_int(0)
            rc = _abi.lib().orb_extract(self._h, _abi.ptr(img), w, h, img.strides[0], _abi.ptr(kps),
                                        _abi.ptr(desc), cap, C.byref(n))
            if rc == -7:
                cap = n.value
                continue
            _abi.check("orb_extract", rc)
            break
        self.last_shape = (h, w)
        return kps[:n.value], desc[:n.value]

    @property
    def mvImagePyramid(self):
        """List of the last frame's pyramid levels (host copies, downloaded lazily)."""
        out = []
        for lvl in range(self.nlevels):
            p = C.POINTER(C.c_uint8)()
            w, h, st = C.c_int(), C.c_int(), C.c_size_t()
            _abi.check("orb_pyramid_level", _abi.lib().orb_pyramid_level(
                self._h, 0, lvl, C.byref(p), C.byref(w), C.byref(h), C.byref(st)))
            a = np.ctypeslib.as_array(p, shape=(h.value, st.value))[:, :w.value].copy()
            out.append(a)
        return out

    # ---- batched device path (torch tensors on cuda)
    def extract_batch_device(self, imgs, kps_out, desc_out, counts_out, stream=None):
        """imgs: uint8 [B, H, W] device tensor; kps_out: [B, cap*7] int32/float32 storage
        (cv::KeyPoint rows); desc_out: uint8 [B, cap, 32]; counts_out: int32 [B]."""
        B, H, W = imgs.shape
        cap = desc_out.shape[1]
        _abi.check("orb_extract_batch_device", _abi.lib().orb_extract_batch_device(
            self._h, _abi.ptr(imgs), H * W, B, W, H, _abi.ptr(kps_out), _abi.ptr(desc_out), cap,
            _abi.ptr(counts_out), C.c_void_p(stream) if stream else None))

    def batch_status(self):
        """Status bits of the last extraction (include/orbslam2_amd.h orb_extractor_batch_status):
        0 when no internal table overflowed."""
        st = C.c_int32(0)
        rc = _abi.lib().orb_extractor_batch_status(self._h, C.byref(st))
        if rc not in (0, -75):
            _abi.check("orb_extractor_batch_status", rc)
        return int(st.value)
