"""The bindings' array-address helper (orb_slam2_amd._abi.ptr) and the oracle's (oracle_ref.P): the
buffer-protocol fast path and the ndarray.ctypes fallback give the same address for every kind of
array a binding passes (contiguous, read-only, empty, strided views, structured keypoint rows)."""
import ctypes as C

import numpy as np
import pytest

import oracle_ref as O
import pkgload

_abi = pkgload.load()._abi


@pytest.mark.parametrize("make", [
    lambda: np.arange(10, dtype=np.int32),
    lambda: np.zeros(0, np.uint8),
    lambda: np.frombuffer(b"abcdefgh", np.uint8),                 # read-only
    lambda: np.zeros((6, 4))[:, ::2],                             # strided view
    lambda: np.zeros(3, dtype=[("x", "<f4"), ("octave", "<i4")]),  # structured rows
    lambda: np.zeros((4, 32), np.uint8)[1:],                      # offset view
])
def test_ptr_matches_ndarray_address(make):
    a = make()
    for fn in (_abi.ptr, O.P):
        p = fn(a)
        assert isinstance(p, C.c_void_p)
        assert (p.value or 0) == (a.ctypes.data or 0)


def test_ptr_passes_none_and_tensors_through():
    assert _abi.ptr(None) is None and O.P(None) is None

    class T:
        def data_ptr(self):
            return 0x1000
    assert _abi.ptr(T()).value == 0x1000


def test_sig_declares_once():
    lib = C.CDLL(None)
    fn = lib.strlen
    fn.argtypes = None
    _abi.sig(fn, [C.c_char_p], C.c_size_t)
    _abi.sig(fn, [C.c_void_p], C.c_int)   # a later declaration does not replace the first
    assert list(fn.argtypes) == [C.c_char_p] and fn.restype is C.c_size_t
    assert fn(b"abcd") == 4
