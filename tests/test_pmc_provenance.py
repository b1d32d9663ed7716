"""The committed PMC captures name the code they were taken from (tools/pmc_provenance.py), and the
bench line reports per capture whether the tree's device sources still match (bench.pmc_capture_current).
CPU only: no counters are read here."""
import importlib.util
import json
import pathlib
import re

ROOT = pathlib.Path(__file__).resolve().parents[1]


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_provenance_hashes_are_sha256():
    prov = _load("_prov", ROOT / "tools" / "pmc_provenance.py").provenance()
    for k in ("csrc_sha256", "bench_py_sha256"):
        assert re.fullmatch(r"[0-9a-f]{64}", prov[k]), k


def test_committed_captures_carry_provenance_and_bench_reports_them():
    bench = _load("_bench", ROOT / "bench.py")
    files = (bench.PMC_TRAFFIC, bench.PMC_VALU, bench.PMC_LANES)
    for f in files:
        doc = json.loads(pathlib.Path(f).read_text())
        assert re.fullmatch(r"[0-9a-f]{64}", doc["provenance"]["csrc_sha256"]), f.name
    cur = bench.pmc_capture_current()
    assert set(cur) == {pathlib.Path(f).name for f in files}
    assert all(isinstance(v, bool) for v in cur.values())
