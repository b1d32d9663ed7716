"""Golden vectors (tests/golden/extract_match_golden.json, made by
tools/make_golden.py): the oracle must reproduce them on CPU, and the HIP path
must reproduce them on the GPU without consulting the oracle."""
import hashlib
import json
import pathlib

import numpy as np
import pytest

import oracle_ref as O

GOLD = json.loads((pathlib.Path(__file__).resolve().parent / "golden" / "extract_match_golden.json").read_text())


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _frames(amd, cfg):
    from orb_slam2_amd import synth
    cv = synth.canvas(cfg["seed"], cfg["W"], cfg["H"])
    fr = [synth.frame(cv, cfg["W"], cfg["H"], t) for t in range(2)]
    for f, g in zip(fr, cfg["frames"]):
        assert sha(f) == g["image_sha256"], "synthetic input drifted"
    return fr


@pytest.mark.parametrize("name", sorted(GOLD))
def test_oracle_reproduces_golden(amd, name):
    cfg = GOLD[name]
    fr = _frames(amd, cfg)
    p = O.params(cfg["nfeatures"])
    res = [O.extract(p, f) for f in fr]
    for r, g in zip(res, cfg["frames"]):
        assert len(r["kps"]) == g["n"]
        assert r["level_counts"].tolist() == g["level_counts"] and r["pre_counts"].tolist() == g["pre_counts"]
        assert sha(r["kps"]) == g["kps_sha256"] and sha(r["desc"]) == g["desc_sha256"]
    a, b = res
    fa = O.FrameView(a["kps"], a["desc"], cfg["W"], cfg["H"])
    fb = O.FrameView(b["kps"], b["desc"], cfg["W"], cfg["H"])
    prev = np.stack([a["kps"]["x"], a["kps"]["y"]], 1).astype(np.float32).reshape(-1)
    n, m12, prev2 = O.search_for_initialization(fa, fb, prev, nnratio=0.9, window=100)
    assert n == cfg["sfi"]["nmatches"] and sha(m12) == cfg["sfi"]["matches12_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(GOLD))
def test_gpu_reproduces_golden(amd, name):
    cfg = GOLD[name]
    fr = _frames(amd, cfg)
    ex = amd.ORBextractor(cfg["nfeatures"], 1.2, 8, 20, 7, max_w=cfg["W"], max_h=cfg["H"])
    outs = [ex(f) for f in fr]
    for (k, d), g in zip(outs, cfg["frames"]):
        assert len(k) == g["n"] and sha(k) == g["kps_sha256"] and sha(d) == g["desc_sha256"]
    (k0, d0), (k1, d1) = outs
    prev = np.stack([k0["x"], k0["y"]], 1).astype(np.float32)
    m = amd.ORBmatcher(0.9, True)
    n, m12 = m.SearchForInitialization(amd.Frame(k0, d0, cfg["W"], cfg["H"]), amd.Frame(k1, d1, cfg["W"], cfg["H"]),
                                       prev, 100)
    assert n == cfg["sfi"]["nmatches"] and sha(m12) == cfg["sfi"]["matches12_sha256"]
    assert sha(prev.reshape(-1)) == cfg["sfi"]["prev_sha256"]
