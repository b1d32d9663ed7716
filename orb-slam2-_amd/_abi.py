"""ctypes binding of liborbslam2_amd.so (include/orbslam2_amd.h).

The HIP library is the only compute path: if it is missing or no gfx950 GPU
is present, every entry point raises — there is no CPU fallback.
"""
import ctypes as C
import os
import pathlib

import numpy as np

# ORB_SLAM2_AMD_LIB selects an instrumented build of the same sources (tools/build_variant.py)
LIB_PATH = pathlib.Path(os.environ.get("ORB_SLAM2_AMD_LIB") or
                        pathlib.Path(__file__).resolve().parent / "lib" / "liborbslam2_amd.so")

ORB_OK = 0
ERRORS = {-22: "ORB_EINVAL", -7: "ORB_E2BIG", -12: "ORB_ENOMEM", -19: "ORB_ENODEV", -5: "ORB_EGPU",
          -75: "ORB_EOVERFLOW"}

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])


class OrbError(RuntimeError):
    def __init__(self, fn, code):
        super().__init__(f"{fn} failed with {ERRORS.get(code, code)}")
        self.code = code


class ExtractorParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int), ("scaleFactor", C.c_float), ("nlevels", C.c_int),
                ("iniThFAST", C.c_int), ("minThFAST", C.c_int)]


class FrameView(C.Structure):
    _fields_ = [("n", C.c_int), ("x", C.c_void_p), ("y", C.c_void_p), ("angle", C.c_void_p),
                ("octave", C.c_void_p), ("desc", C.c_void_p), ("uright", C.c_void_p),
                ("min_x", C.c_float), ("min_y", C.c_float), ("max_x", C.c_float), ("max_y", C.c_float),
                ("grid_w_inv", C.c_float), ("grid_h_inv", C.c_float)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
        _lib = C.CDLL(str(LIB_PATH))
        vp, i32, f32, sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
        sig = {
            "orb_extractor_create": [vp, i32, i32, i32, i32, vp],
            "orb_extractor_destroy": [vp],
            "orb_extractor_levels": [vp],
            "orb_extractor_scale_tables": [vp, vp, vp, vp, vp],
            "orb_extractor_features_per_level": [vp, vp],
            "orb_extract": [vp, vp, i32, i32, sz, vp, vp, i32, vp],
            "orb_extract_batch_device": [vp, vp, sz, i32, i32, i32, vp, vp, i32, vp, vp],
            "orb_pyramid_level": [vp, i32, i32, vp, vp, vp, vp],
            "orb_pyramid_level_device": [vp, i32, i32, i32, vp, vp, vp, vp],
            "orb_extractor_profile": [vp, i32],
            "orb_extractor_set_level0_copy": [vp, i32],
            "orb_extractor_stage_times": [vp, vp, i32, vp],
            "orb_extractor_geometry": [vp, i32, i32, vp, vp, vp, vp],
            "orb_extractor_last_counts": [vp, i32, vp, vp],
            "orb_extractor_batch_status": [vp, vp],
            "orb_matcher_create": [i32, f32, i32, vp],
            "orb_matcher_destroy": [vp],
            "orb_descriptor_distance": [vp, vp],
            "orb_search_for_initialization": [vp, vp, vp, vp, vp, i32],
            "orb_search_by_projection_frame": [vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, f32, i32, vp],
            "orb_search_by_projection_local": [vp, vp, i32, vp, vp, vp, vp, vp, vp, vp, f32, vp],
            "orb_compute_stereo_matches": [vp, vp, vp, vp, i32, vp, vp, i32, f32, f32, vp, vp],
            "orb_compute_stereo_matches_batch_device": [vp, vp, vp, vp, i32, i32, f32, f32, vp, vp, vp, vp],
            "orb_hamming_knn2": [vp, vp, i32, vp, i32, vp, vp, vp],
            "orb_hamming_knn2_batch_device": [vp, vp, vp, vp, vp, i32, i32, i32, vp, vp, vp, vp],
            "orb_search_for_initialization_batch_device": [vp, vp, vp, vp, vp, vp, vp, i32, i32, i32, i32, i32,
                                                           vp, vp, vp],
            "orb_matcher_batch_status": [vp, vp],
        }
        for name, args in sig.items():
            fn = getattr(_lib, name)
            fn.argtypes = args
            fn.restype = None if name.endswith("_destroy") else C.c_int
    return _lib


def sig(fn, argtypes, restype=C.c_int):
    """Declares a library function's signature once (ctypes re-converts an argtypes list on every
    assignment: ~3 us a call for the host-buffer entry points that declared theirs per call)."""
    if fn.argtypes is None:
        fn.argtypes = argtypes
        fn.restype = restype
    return fn


def check(fn: str, rc: int) -> int:
    if rc < 0:
        raise OrbError(fn, rc)
    return rc


def ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        # the address through the buffer protocol: ~1 us where ndarray.ctypes.data_as takes ~5 (a
        # host call passes a dozen arrays); read-only, empty or non-contiguous arrays take the
        # ndarray.ctypes route
        try:
            return C.c_void_p(C.addressof(C.c_char.from_buffer(a)))
        except (TypeError, ValueError, BufferError):
            return C.c_void_p(a.ctypes.data)
    if hasattr(a, "data_ptr"):          # torch tensor (device memory)
        return C.c_void_p(a.data_ptr())
    return a
