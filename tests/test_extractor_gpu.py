"""GPU extractor parity: HIP path (through the C-ABI) vs the CPU oracle,
bit-exact keypoints (all fields) and descriptors, on seeded synthetic frames."""
import numpy as np
import pytest

import oracle_ref as O
from orb_slam2_amd import synth

pytestmark = pytest.mark.gpu
# Camera.bf of R/Examples/Stereo/EuRoC.yaml / KITTI00-02.yaml as the float Frame::mbf
EUROC_BF, KITTI_BF = (float(np.float32(synth.CAMERAS[k]["bf"])) for k in ("EUROC", "KITTI00"))

CONFIGS = [
    # (W, H, nfeatures, seed)
    (640, 480, 1000, 0x5EED0001),
    (640, 480, 2000, 0x5EED0002),
    (1241, 376, 2000, 0x5EED0003),
    (752, 480, 1200, 0x5EED0005),
]


def _frames(W, H, seed, n):
    from orb_slam2_amd import synth
    cv = synth.canvas(seed, W, H)
    return [synth.frame(cv, W, H, t) for t in range(n)]


def _compare(ref, kps, desc):
    assert len(kps) == len(ref["kps"]), (len(kps), len(ref["kps"]))
    for f in ("x", "y", "size", "angle", "response", "octave", "class_id"):
        a, b = kps[f], ref["kps"][f]
        bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
        assert bad.size == 0, f"field {f}: {bad.size} mismatches, first {bad[:5]} gpu={a[bad[:5]]} ref={b[bad[:5]]}"
    bad = np.nonzero((desc != ref["desc"]).any(1))[0]
    assert bad.size == 0, f"descriptor mismatches at {bad[:10]}"


@pytest.mark.parametrize("W,H,nf,seed", CONFIGS)
def test_extract_matches_oracle(amd, W, H, nf, seed):
    ex = amd.ORBextractor(nf, 1.2, 8, 20, 7, max_w=W, max_h=H)
    p = O.params(nf)
    for img in _frames(W, H, seed, 2):
        ref = O.extract(p, img)
        kps, desc = ex(img)
        _compare(ref, kps, desc)


@pytest.mark.parametrize("W,H,nf,scale,nlev,ini,minth,seed", [
    (639, 479, 800, 1.25, 6, 15, 5, 0x5EED0011),     # odd sizes (level 0 copied into the slab), other pyramid
    (320, 240, 500, 1.2, 8, 20, 7, 0x5EED0012),      # small frame: few cells per level
    (1024, 768, 1500, 1.3, 5, 25, 9, 0x5EED0013),    # coarse pyramid, high thresholds
    (800, 600, 1200, 1.15, 10, 12, 4, 0x5EED0014),   # fine pyramid, ten levels, low thresholds
])
def test_extract_parameters_match_oracle(amd, W, H, nf, scale, nlev, ini, minth, seed):
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) away from the defaults
    (R/src/ORBextractor.cpp:421-485): every geometry-derived table (level sizes, cell grids, resize
    coefficients, per-level feature quotas) and both FAST thresholds, bit-exact against the oracle."""
    ex = amd.ORBextractor(nf, scale, nlev, ini, minth, max_w=W, max_h=H)
    p = O.params(nf, scale, nlev, ini, minth)
    for img in _frames(W, H, seed, 2):
        kps, desc = ex(img)
        _compare(O.extract(p, img), kps, desc)


def test_extract_geometry_changes_on_one_handle(amd):
    """One handle created for the default bound (1280 x 1024), then fed 640 x 480, KITTI and 640 x 480
    again: every geometry change rebuilds the resize tables and the pyramid band table (which an
    earlier build freed twice, leaving a sticky HIP error that failed the next call)."""
    ex = amd.ORBextractor(1000, 1.2, 8, 20, 7)
    p = O.params(1000)
    for W, H, seed in ((640, 480, 0x5EED0001), (1241, 376, 0x5EED0003), (640, 480, 0x5EED0002)):
        img = _frames(W, H, seed, 1)[0]
        kps, desc = ex(img)
        _compare(O.extract(p, img), kps, desc)


def test_pyramid_matches_oracle(amd):
    W, H = 640, 480
    img = _frames(W, H, 0x5EED0001, 1)[0]
    ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=W, max_h=H)
    ex(img)
    ref = O.extract(O.params(1000), img, want_pyramid=True)
    lw, lh = ref["sizes"]
    off = 0
    for lvl, a in enumerate(ex.mvImagePyramid):
        b = ref["pyramid"][off:off + lw[lvl] * lh[lvl]].reshape(lh[lvl], lw[lvl])
        off += lw[lvl] * lh[lvl]
        assert a.shape == b.shape
        assert np.array_equal(a, b), f"level {lvl}: {np.count_nonzero(a != b)} px differ"


def test_blurred_pyramid_on_demand_matches_oracle(amd):
    """orb_pyramid_level_device(blurred=1): the full GaussianBlur pyramid (k_blur, run on
    demand) equals the oracle's per-level blur (REFLECT_101, 8-bit kernel)."""
    import ctypes as C
    from orb_slam2_amd import _abi
    hip = C.CDLL("libamdhip64.so")
    W, H = 640, 480
    img = _frames(W, H, 0x5EED0003, 1)[0]
    ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=W, max_h=H)
    ex(img)
    ref = O.extract(O.params(1000), img, want_pyramid=True)
    lw, lh = ref["sizes"]
    off = 0
    for lvl in range(8):
        p, w, h, st = C.c_void_p(), C.c_int(), C.c_int(), C.c_size_t()
        _abi.check("orb_pyramid_level_device", _abi.lib().orb_pyramid_level_device(
            ex._h, 0, lvl, 1, C.byref(p), C.byref(w), C.byref(h), C.byref(st)))
        buf = np.zeros((h.value, st.value), np.uint8)
        assert hip.hipMemcpy(C.c_void_p(buf.ctypes.data), p, C.c_size_t(buf.nbytes), 2) == 0
        a = buf[:, :w.value]
        b = ref["blurred"][off:off + lw[lvl] * lh[lvl]].reshape(lh[lvl], lw[lvl])
        off += lw[lvl] * lh[lvl]
        assert np.array_equal(a, b), f"level {lvl}: {np.count_nonzero(a != b)} px differ"


@pytest.mark.parametrize("W,H,nf", [(640, 480, 1000), (1241, 376, 2000)])
def test_batch_pyramid_level0_is_the_input(amd, W, H, nf):
    """Level 0 of a batched extraction is the caller's frame (R/src/ORBextractor.cpp:1223 rebinds
    mvImagePyramid[0] to the input): dword-aligned frames (640 wide) are read in place — the raw
    level-0 device pointer is the input frame itself — and odd widths (KITTI 1241) are read from
    the slab's copy; either way the host level 0 equals the frame and every level equals the
    oracle's pyramid, for a middle frame of the batch."""
    import ctypes as C
    import torch
    from orb_slam2_amd import _abi
    B = 3
    frames = _frames(W, H, 0x5EED0007, B)
    dev = torch.device("cuda", 0)
    ex = amd.ORBextractor(nf, 1.2, 8, 20, 7, max_w=W, max_h=H, max_batch=B)
    cap = C.c_int()
    _abi.check("geom", _abi.lib().orb_extractor_geometry(ex._h, W, H, None, None, None, C.byref(cap)))
    ti = torch.from_numpy(np.stack(frames)).to(dev)
    kps = torch.zeros((B, cap.value, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((B, cap.value, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    ex.extract_batch_device(ti, kps, desc, cnt, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    assert ex.batch_status() == 0
    ref = O.extract(O.params(nf), frames[1], want_pyramid=True)
    lw, lh = ref["sizes"]
    off = 0
    for lvl in range(8):
        p = C.POINTER(C.c_uint8)()
        w, h, st = C.c_int(), C.c_int(), C.c_size_t()
        _abi.check("orb_pyramid_level", _abi.lib().orb_pyramid_level(ex._h, 1, lvl, C.byref(p), C.byref(w), C.byref(h),
                                                                     C.byref(st)))
        a = np.ctypeslib.as_array(p, shape=(h.value, st.value))[:, :w.value]
        b = ref["pyramid"][off:off + lw[lvl] * lh[lvl]].reshape(lh[lvl], lw[lvl])
        off += lw[lvl] * lh[lvl]
        assert np.array_equal(a, b), f"level {lvl}: {np.count_nonzero(a != b)} px differ"
        if lvl == 0:
            assert np.array_equal(a, frames[1])
    dp, w, h, st = C.c_void_p(), C.c_int(), C.c_int(), C.c_size_t()
    _abi.check("orb_pyramid_level_device", _abi.lib().orb_pyramid_level_device(ex._h, 1, 0, 0, C.byref(dp), C.byref(w),
                                                                               C.byref(h), C.byref(st)))
    if W % 4 == 0:
        assert dp.value == ti.data_ptr() + W * H and st.value == W   # in place: no level-0 copy
    else:
        assert dp.value != ti.data_ptr() + W * H


def test_empty_image_leaves_outputs(amd):
    ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=640, max_h=480)
    sentinel = (np.zeros(3, np.uint8), np.ones((3, 32), np.uint8))
    out = ex(np.zeros((0, 0), np.uint8), None, *sentinel)
    assert out[0] is sentinel[0] and out[1] is sentinel[1]


def test_flat_image_no_keypoints(amd):
    ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=640, max_h=480)
    kps, desc = ex(np.full((480, 640), 77, np.uint8))
    assert len(kps) == 0 and desc.shape == (0, 32)


def test_noise_image_retry_threshold(amd):
    """Low-contrast noise: most cells find nothing at iniThFAST=20 and retry at 7."""
    rng = np.random.default_rng(3)
    img = (128 + rng.integers(-9, 10, size=(480, 640))).astype(np.uint8)
    ex = amd.ORBextractor(1000, 1.2, 8, 20, 7, max_w=640, max_h=480)
    ref = O.extract(O.params(1000), img)
    kps, desc = ex(img)
    _compare(ref, kps, desc)


@pytest.mark.parametrize("W,H,nf,seed,mbf", [(752, 480, 1200, 0x5EED0005, EUROC_BF), (640, 480, 1000, 0x5EED0006, 40.0),
                                             (1241, 376, 2000, 0x5EED0003, KITTI_BF)])
def test_compute_stereo_matches(amd, W, H, nf, seed, mbf):
    """Frame::ComputeStereoMatches on the GPU (pyramids read in place) vs the oracle on a
    synthetic stereo pair with a smooth disparity field: EuRoC geometry,
    TUM geometry, and KITTI 00 geometry with the KITTI bf (config 3, R/Examples/Stereo/KITTI00-02.yaml)."""
    from orb_slam2_amd import synth
    cv = synth.canvas(seed, W, H)
    left, right = synth.stereo_pair(cv, W, H, 0)
    p = O.params(nf)
    a = O.extract(p, left, want_pyramid=True)
    b = O.extract(p, right, want_pyramid=True)
    n_ref, ur_ref, dep_ref = O.compute_stereo_matches(p, a, b, mbf)
    exL = amd.ORBextractor(nf, 1.2, 8, 20, 7, max_w=W, max_h=H)
    exR = amd.ORBextractor(nf, 1.2, 8, 20, 7, max_w=W, max_h=H)
    kl, dl = exL(left)
    kr, dr = exR(right)
    _compare(a, kl, dl)
    _compare(b, kr, dr)
    n, ur, dep = amd.ComputeStereoMatches(exL, exR, kl, dl, kr, dr, mbf)
    assert n == n_ref
    assert np.array_equal(ur, ur_ref) and np.array_equal(dep, dep_ref)
    assert n > 300


@pytest.mark.parametrize("refill", [False, True])
def test_compute_stereo_matches_batch_device(amd, refill):
    """Device batch form: 3 stereo pairs extracted as frames (2p, 2p+1) of one batch.  refill:
    level-0 copy on (orb_extractor_set_level0_copy), and the caller's frame buffer zeroed on the
    stream right after the extraction is enqueued — the stereo matcher (which reads level 0) must
    still see the extracted frames (include/orbslam2_amd.h, LEVEL-0 LIFETIME)."""
    import torch
    from orb_slam2_amd import synth, _abi
    import ctypes as C
    W, H, nf, mbf = 752, 480, 1200, EUROC_BF
    cv = synth.canvas(0x5EED0005, W, H)
    pairs = [synth.stereo_pair(cv, W, H, t) for t in range(3)]
    imgs = np.stack([im for pr in pairs for im in pr])
    dev = torch.device("cuda", 0)
    ex = amd.ORBextractor(nf, 1.2, 8, 20, 7, max_w=W, max_h=H, max_batch=6)
    cap = C.c_int()
    _abi.check("geom", _abi.lib().orb_extractor_geometry(ex._h, W, H, None, None, None, C.byref(cap)))
    cap = cap.value
    ti = torch.from_numpy(imgs).to(dev)
    kps = torch.zeros((6, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((6, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(6, dtype=torch.int32, device=dev)
    ur = torch.zeros((3, cap), dtype=torch.float32, device=dev)
    dep = torch.zeros((3, cap), dtype=torch.float32, device=dev)
    ns = torch.zeros(3, dtype=torch.int32, device=dev)
    ts = torch.cuda.Stream(dev)   # an explicit stream: 0 (the legacy default) would select the handle's own
    torch.cuda.synchronize(dev)
    s = ts.cuda_stream
    lib = _abi.lib()
    if refill:
        _abi.check("l0copy", lib.orb_extractor_set_level0_copy(ex._h, 1))
    _abi.check("x", lib.orb_extract_batch_device(ex._h, C.c_void_p(ti.data_ptr()), H * W, 6, W, H,
                                                  C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()), cap,
                                                  C.c_void_p(cnt.data_ptr()), C.c_void_p(s)))
    if refill:
        with torch.cuda.stream(ts):
            ti.zero_()   # the caller's next upload into the same buffer, same stream
    _abi.check("s", lib.orb_compute_stereo_matches_batch_device(
        ex._h, C.c_void_p(kps.data_ptr()), C.c_void_p(desc.data_ptr()), C.c_void_p(cnt.data_ptr()), cap, 3,
        C.c_float(mbf), C.c_float(0.0), C.c_void_p(ur.data_ptr()), C.c_void_p(dep.data_ptr()),
        C.c_void_p(ns.data_ptr()), C.c_void_p(s)))
    torch.cuda.synchronize(dev)
    p = O.params(nf)
    for i, (l, r) in enumerate(pairs):
        a = O.extract(p, l, want_pyramid=True)
        b = O.extract(p, r, want_pyramid=True)
        n_ref, ur_ref, dep_ref = O.compute_stereo_matches(p, a, b, mbf)
        nl = len(a["kps"])
        assert int(cnt[2 * i]) == nl
        assert int(ns[i]) == n_ref
        assert np.array_equal(ur[i, :nl].cpu().numpy(), ur_ref)
        assert np.array_equal(dep[i, :nl].cpu().numpy(), dep_ref)


def test_batch_device_status_dense_octree_hbm_path(amd):
    """Throughput path with a frame whose levels hold far more FAST keys than the octree's LDS
    key buffers (uniform noise: ~27,700 keys on level 0, so k_octree runs on its HBM key
    arrays): keypoints / descriptors bit-exact vs the oracle and the batch status (cell /
    octree table overflow bits, orb_extractor_batch_status) reads 0."""
    import torch
    from orb_slam2_amd import synth, _abi
    import ctypes as C
    W, H, nf = 640, 480, 1000
    noise = np.random.default_rng(5).integers(0, 256, (H, W)).astype(np.uint8)
    frame = synth.frame(synth.canvas(0x5EED0001, W, H), W, H, 0)
    imgs = np.stack([noise, frame, noise[::-1].copy()])
    B = len(imgs)
    dev = torch.device("cuda", 0)
    ex = amd.ORBextractor(nf, 1.2, 8, 20, 7, max_w=W, max_h=H, max_batch=B)
    cap = C.c_int()
    _abi.check("geom", _abi.lib().orb_extractor_geometry(ex._h, W, H, None, None, None, C.byref(cap)))
    cap = cap.value
    ti = torch.from_numpy(imgs).to(dev)
    kps = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    ex.extract_batch_device(ti, kps, desc, cnt, torch.cuda.current_stream(dev).cuda_stream)
    assert ex.batch_status() == 0
    pre = np.zeros(8, np.int32)
    _abi.check("counts", _abi.lib().orb_extractor_last_counts(ex._h, 0, _abi.ptr(pre), None))
    assert pre[0] > 20000
    p = O.params(nf)
    for b in range(B):
        ref = O.extract(p, imgs[b])
        n = int(cnt[b])
        assert n == len(ref["kps"])
        got_k = kps[b, :n].cpu().numpy().view(amd._abi.KEYPOINT_DTYPE).reshape(-1)
        assert got_k.tobytes() == ref["kps"].tobytes()
        assert np.array_equal(desc[b, :n].cpu().numpy(), ref["desc"])


@pytest.mark.parametrize("copy", [0, 1])
def test_level0_lifetime_contract(amd, copy):
    """LEVEL-0 LIFETIME (include/orbslam2_amd.h): without level-0 copy, raw level 0 of a device
    batch IS the caller's frame (orb_pyramid_level_device returns a pointer into d_imgs, so a refill
    of d_imgs is what a later level-0 read sees, as the reference's Mat header rebinding does);
    with copy on, level 0 lives in the handle's slab and survives the refill.  Keypoints and
    descriptors are identical either way."""
    import torch
    from orb_slam2_amd import synth, _abi
    import ctypes as C
    W, H, nf, B = 640, 480, 1000, 2
    cv = synth.canvas(0x5EED0001, W, H)
    imgs = np.stack([synth.frame(cv, W, H, t) for t in range(B)])
    dev = torch.device("cuda", 0)
    ex = amd.ORBextractor(nf, 1.2, 8, 20, 7, max_w=W, max_h=H, max_batch=B)
    lib = _abi.lib()
    _abi.check("l0copy", lib.orb_extractor_set_level0_copy(ex._h, copy))
    assert lib.orb_extractor_set_level0_copy(ex._h, 2) == -22   # ORB_EINVAL
    cap = C.c_int()
    _abi.check("geom", lib.orb_extractor_geometry(ex._h, W, H, None, None, None, C.byref(cap)))
    cap = cap.value
    ti = torch.from_numpy(imgs).to(dev)
    kps = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    cnt = torch.zeros(B, dtype=torch.int32, device=dev)
    ts = torch.cuda.Stream(dev)   # an explicit stream: 0 (the legacy default) would select the handle's own
    torch.cuda.synchronize(dev)
    ex.extract_batch_device(ti, kps, desc, cnt, ts.cuda_stream)
    with torch.cuda.stream(ts):
        ti.fill_(7)   # the caller refills its buffer on the extraction's stream
    torch.cuda.synchronize(dev)
    dp, w, h, pitch = C.c_void_p(), C.c_int(), C.c_int(), C.c_size_t()
    _abi.check("lvl", lib.orb_pyramid_level_device(ex._h, 1, 0, 0, C.byref(dp), C.byref(w), C.byref(h), C.byref(pitch)))
    hp = C.POINTER(C.c_uint8)()
    _abi.check("lvlh", lib.orb_pyramid_level(ex._h, 1, 0, C.byref(hp), None, None, C.byref(pitch)))
    l0 = np.ctypeslib.as_array(hp, shape=(H, pitch.value))[:, :W]
    if copy:
        assert dp.value != ti.data_ptr() + H * W
        assert np.array_equal(l0, imgs[1])
    else:
        assert dp.value == ti.data_ptr() + H * W
        assert (l0 == 7).all()
    p = O.params(nf)
    for b in range(B):
        ref = O.extract(p, imgs[b])
        n = int(cnt[b])
        assert n == len(ref["kps"])
        assert kps[b, :n].cpu().numpy().view(amd._abi.KEYPOINT_DTYPE).reshape(-1).tobytes() == ref["kps"].tobytes()
        assert np.array_equal(desc[b, :n].cpu().numpy(), ref["desc"])


@pytest.mark.gpu
@pytest.mark.parametrize("row_bytes,B,cap", [(28, 5, 40), (32, 64, 1062), (4, 1, 7), (4, 33, 300)])
def test_pack_rows_device(amd, row_bytes, B, cap):
    """orb_pack_rows_device: frame b's min(counts[b], cap) rows at a capacity stride, packed back
    to back at the exclusive prefix; offsets[B] = the total (counts past cap, zero and negative
    counts included)."""
    import ctypes as C
    import torch
    from orb_slam2_amd import _abi
    rng = np.random.default_rng(row_bytes * 1000 + B)
    src = rng.integers(0, 256, (B, cap, row_bytes), dtype=np.uint8)
    cnt = rng.integers(-2, cap + 5, B).astype(np.int32)
    cnt[0] = cap + 3 if B > 1 else cnt[0]
    dev = torch.device("cuda", 0)
    ds = torch.from_numpy(src).to(dev)
    dc = torch.from_numpy(cnt).to(dev)
    dd = torch.zeros(B * cap * row_bytes + 4, dtype=torch.uint8, device=dev)
    do = torch.full((B + 1,), -7, dtype=torch.int32, device=dev)
    _abi.check("pack", _abi.lib().orb_pack_rows_device(C.c_void_p(ds.data_ptr()), row_bytes, cap,
                                                       C.c_void_p(dc.data_ptr()), B, C.c_void_p(dd.data_ptr()),
                                                       C.c_void_p(do.data_ptr()), None))
    torch.cuda.synchronize(dev)
    n = np.clip(cnt, 0, cap)
    off = np.concatenate([[0], np.cumsum(n)]).astype(np.int32)
    assert np.array_equal(do.cpu().numpy(), off)
    want = np.concatenate([src[b, :n[b]].reshape(-1) for b in range(B)])
    got = dd.cpu().numpy()
    assert np.array_equal(got[:len(want)], want) and not got[len(want):].any()
