"""The C-ABI library loads without a GPU and exports every entry point that
include/orbslam2_amd.h declares; compute entry points refuse cleanly without a GPU."""
import ctypes as C
import pathlib
import re

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "orbslam2_amd.h"


def declared():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"\b(orb_[a-z0-9_]+|lba_[a-z0-9_]+|pose_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("orb_extractor_create", "orb_extract", "orb_extract_batch_device", "orb_pyramid_level",
                 "orb_search_for_initialization", "orb_search_by_projection_frame", "orb_hamming_knn2",
                 "orb_descriptor_distance"):
        assert must in names


def test_library_exports_all_declared(amd):
    lib = amd._abi.lib()
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, f"not exported: {missing}"


def test_descriptor_distance_host_helper(amd):
    a = (C.c_uint8 * 32)(*([0xFF] * 32))
    b = (C.c_uint8 * 32)(*([0x0F] * 32))
    assert amd._abi.lib().orb_descriptor_distance(a, b) == 128


def test_no_gpu_is_an_error_not_a_fallback(amd):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(amd._abi.OrbError) as e:
        amd.ORBextractor(1000, 1.2, 8, 20, 7)
    assert e.value.code == -19   # ORB_ENODEV


def test_no_exception_crosses_the_abi():
    """no C++ exception crosses the C-ABI.  Every definition of a declared entry point
    in orb-slam2-_amd/csrc/*.hip is a function-try-block whose handler is ORB_ABI_CATCH
    (std::bad_alloc -> ORB_ENOMEM, anything else -> ORB_EINTERNAL) or, for the void functions,
    ORB_ABI_CATCH_VOID."""
    names = set(declared())
    seen = {}
    for f in sorted((ROOT / "orb-slam2-_amd" / "csrc").glob("*.hip")):
        src = f.read_text()
        for m in re.finditer(r"^(int|void)\s+(\w+)\(", src, re.M):
            if m.group(2) not in names:
                continue
            brace = src.index("{", m.start())
            head = src[m.start(): brace]
            if ";" in head:
                continue   # a forward declaration
            assert head.rstrip().endswith("try"), (f.name, m.group(2))
            want = "ORB_ABI_CATCH_VOID" if m.group(1) == "void" else "ORB_ABI_CATCH"
            first_line = src[m.start(): src.index("\n", m.start())].rstrip()
            if first_line.endswith("}" + " " + want):
                end = first_line   # a one-line definition
            else:
                close = re.compile(r"^}.*$", re.M).search(src, brace)   # the body's closing brace (column 0)
                end = close.group(0).rstrip()
            assert end.split()[-1] == want, (f.name, m.group(2), end)
            seen[m.group(2)] = f.name
    assert set(seen) == names, sorted(names - set(seen))
