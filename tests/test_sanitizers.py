"""Sanitizer builds of the CPU side: the local-BA host structure build
(orb-slam2-_amd/csrc/lba_host.h) checked under -fsanitize=address,undefined with leak detection on,
and the compiled drop-in caller (include/orbslam2_amd_shim.hpp) built the same way, run on its
no-GPU path (ORB_ENODEV, exit 3, no CPU fallback).  `oracle/Makefile` target `sanitize` builds
them; tools/sanitize_cpu.sh runs the whole `pytest -m "not gpu"` suite against the sanitized
oracle and caller (its log: profiles/r05_sanitize_cpu.txt)."""
import os
import pathlib
import shutil
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
ASAN = ROOT / "oracle" / "build" / "asan"


@pytest.fixture(scope="module")
def built():
    if shutil.which("g++") is None or not (ROOT / "orb-slam2-_amd" / "lib" / "liborbslam2_amd.so").exists():
        pytest.skip("g++ or the built library is missing")
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "build/asan/lba_host_check", "build/asan/shim_caller"],
                   check=True, capture_output=True, text=True)
    return ASAN


def test_lba_host_structure_under_asan_ubsan(built):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(built / "lba_host_check")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "lba_host_check ok" in r.stdout, r.stderr[-2000:]


def test_shim_caller_under_asan_ubsan_no_gpu(built, tmp_path):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: the sanitized caller is a CPU-side check")
    from test_cpp_shim import _run
    img = np.zeros((480, 640), np.uint8)
    os.environ.setdefault("ASAN_OPTIONS", "detect_leaks=0")
    r, _ = _run(built / "shim_caller", "extract", tmp_path, np.array([640, 480, 1000], np.int32), img)
    assert r.returncode == 3 and "failed (-19)" in r.stderr, (r.returncode, r.stderr[-2000:])
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
