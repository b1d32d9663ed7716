"""Host mirror of Frame::ComputeStereoMatches (R/src/Frame.cpp:551-770) over the HIP C-ABI:
the two ORBextractor handles' device pyramids are read in place."""
import ctypes as C

import numpy as np

from . import _abi


def ComputeStereoMatches(extractorLeft, extractorRight, mvKeys, mDescriptors, mvKeysRight, mDescriptorsRight,
                         mbf: float, mb: float = 0.0):
    """Returns (nmatches, mvuRight, mvDepth).  Both extractors must hold the extraction of
    the left / right image that produced the keypoints.  mb = 0 reproduces the reference,
    whose constructor assigns mb only after this call (maxD = +inf)."""
    kl = np.ascontiguousarray(mvKeys, _abi.KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(mvKeysRight, _abi.KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(mDescriptors, np.uint8)
    dr = np.ascontiguousarray(mDescriptorsRight, np.uint8)
    ur = np.zeros(len(kl), np.float32)
    dep = np.zeros(len(kl), np.float32)
    n = _abi.check("orb_compute_stereo_matches", _abi.lib().orb_compute_stereo_matches(
        extractorLeft._h, extractorRight._h, _abi.ptr(kl), _abi.ptr(dl), len(kl), _abi.ptr(kr), _abi.ptr(dr),
        len(kr), C.c_float(mbf), C.c_float(mb), _abi.ptr(ur), _abi.ptr(dep)))
    return n, ur, dep
