"""What a PMC / profile JSON was captured from: SHA-256 of the device sources (orb-slam2-_amd/csrc/*),
of the library the run loaded and of bench.py, so a committed capture can be matched to the code it
describes (a capture whose hashes differ from the tree's is stale and is recaptured)."""
import hashlib
import os
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _sha(paths):
    h = hashlib.sha256()
    for p in paths:
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def provenance():
    csrc = sorted((ROOT / "orb-slam2-_amd" / "csrc").glob("*"))
    lib = pathlib.Path(os.environ.get("ORB_SLAM2_AMD_LIB", ROOT / "orb-slam2-_amd" / "lib" / "liborbslam2_amd.so"))
    out = {"csrc_sha256": _sha([p for p in csrc if p.is_file()]), "bench_py_sha256": _sha([ROOT / "bench.py"])}
    if lib.exists():
        out["library_sha256"] = _sha([lib])
    return out


if __name__ == "__main__":
    import json
    print(json.dumps(provenance(), indent=1))
