"""Deterministic synthetic inputs standing in for TUM / KITTI / EuRoC frames
(the datasets are not on disk).

A 2W x 2H canvas (background 128, 400 filled rectangles — half of them rotated
45 degrees — and 300 filled discs with random grey levels, plus i.i.d. integer
noise U[-6, 6]) is cropped at an integer offset that advances by (+2, +1) px per
frame, so consecutive frames differ by a pure translation.
"""
import numpy as np


def canvas(seed: int, W: int, H: int) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    CW, CH = 2 * W, 2 * H
    img = np.full((CH, CW), 128, np.int16)
    for k in range(400):
        a, b = rng.integers(8, 81, size=2)
        cx, cy = rng.integers(0, CW), rng.integers(0, CH)
        val = int(rng.integers(0, 256))
        if k % 2 == 0:
            x0, x1 = max(0, cx - a // 2), min(CW, cx + (a + 1) // 2)
            y0, y1 = max(0, cy - b // 2), min(CH, cy + (b + 1) // 2)
            img[y0:y1, x0:x1] = val
        else:
            r = int(max(a, b))
            x0, x1 = max(0, cx - r), min(CW, cx + r + 1)
            y0, y1 = max(0, cy - r), min(CH, cy + r + 1)
            yy, xx = np.mgrid[y0:y1, x0:x1]
            dx, dy = xx - cx, yy - cy
            u, v = (dx + dy) * 0.70710678, (dx - dy) * 0.70710678
            m = (np.abs(u) <= a / 2) & (np.abs(v) <= b / 2)
            img[y0:y1, x0:x1][m] = val
    for _ in range(300):
        r = int(rng.integers(4, 31))
        cx, cy = rng.integers(0, CW), rng.integers(0, CH)
        val = int(rng.integers(0, 256))
        x0, x1 = max(0, cx - r), min(CW, cx + r + 1)
        y0, y1 = max(0, cy - r), min(CH, cy + r + 1)
        yy, xx = np.mgrid[y0:y1, x0:x1]
        m = (xx - cx) ** 2 + (yy - cy) ** 2 <= r * r
        img[y0:y1, x0:x1][m] = val
    img += rng.integers(-6, 7, size=img.shape).astype(np.int16)
    return np.clip(img, 0, 255).astype(np.uint8)


def frame(cv: np.ndarray, W: int, H: int, t: int) -> np.ndarray:
    ox = (W // 2 + 2 * t) % W
    oy = (H // 2 + t) % H
    return np.ascontiguousarray(cv[oy:oy + H, ox:ox + W])


def disparity_field(W: int, H: int, lo: int = 5, hi: int = 60) -> np.ndarray:
    """Smooth integer disparity field d(x, y) in [lo, hi]."""
    y, x = np.mgrid[0:H, 0:W].astype(np.float64)
    f = 0.5 + 0.25 * np.sin(2 * np.pi * x / W * 1.3 + 0.7) + 0.25 * np.cos(2 * np.pi * y / H * 0.9 + 0.3)
    return np.rint(lo + (hi - lo) * f).astype(np.int32)


def stereo_pair(cv: np.ndarray, W: int, H: int, t: int):
    """Left = frame t of the canvas crop; right(x, y) = left(x + d(x, y), y) with the smooth
    disparity field, so a left point at u appears at u - d in the right image."""
    ox = (W // 2 + 2 * t) % W
    oy = (H // 2 + t) % H
    big = cv[oy:oy + H, ox:ox + W + 64]
    left = np.ascontiguousarray(big[:, :W])
    d = disparity_field(W, H)
    xs = np.minimum(np.arange(W)[None, :] + d, big.shape[1] - 1)
    right = np.ascontiguousarray(np.take_along_axis(big, xs, axis=1))
    return left, right


def stream(seed: int, W: int, H: int, n: int) -> np.ndarray:
    cv = canvas(seed, W, H)
    return np.stack([frame(cv, W, H, t) for t in range(n)])


# ---------------------------------------------------------------- local-BA problem

# The reference's camera / extractor settings for the BASELINE configs, as the example YAMLs hold
# them (data values; tests/test_reference_data.py parses the YAMLs and pins every entry):
#   TUM1      R/Examples/Monocular/TUM1.yaml       (config 1; configs 2 and 4 use its intrinsics)
#   KITTI00   R/Examples/Stereo/KITTI00-02.yaml    (config 3)
#   EUROC     R/Examples/Stereo/EuRoC.yaml         (config 5)
# bf is the YAML's Camera.bf (Frame::mbf, a float: the stereo Frame reads it through cv::FileStorage
# into the float Tracking::mbf, R/src/Tracking.cpp:95, include/Tracking.h:194); 0 for the monocular
# camera.
CAMERAS = {
    "TUM1": dict(fx=517.306408, fy=516.469215, cx=318.643040, cy=255.313989, bf=0.0, width=640, height=480,
                 nFeatures=1000, scaleFactor=1.2, nLevels=8, iniThFAST=20, minThFAST=7),
    "KITTI00": dict(fx=718.856, fy=718.856, cx=607.1928, cy=185.2157, bf=386.1448, width=1241, height=376,
                    nFeatures=2000, scaleFactor=1.2, nLevels=8, iniThFAST=20, minThFAST=7, ThDepth=35),
    "EUROC": dict(fx=435.2046959714599, fy=435.2046959714599, cx=367.4517211914062, cy=252.2008514404297,
                  bf=47.90639384423901, width=752, height=480,
                  nFeatures=1200, scaleFactor=1.2, nLevels=8, iniThFAST=20, minThFAST=7, ThDepth=35),
}
TUM1 = tuple(CAMERAS["TUM1"][k] for k in ("fx", "fy", "cx", "cy"))
KITTI_BF = CAMERAS["KITTI00"]["bf"]
EUROC_BF = CAMERAS["EUROC"]["bf"]


def _rot(axis_angle):
    th = float(np.linalg.norm(axis_angle))
    if th < 1e-12:
        return np.eye(3)
    k = axis_angle / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def ba_problem(seed=42, n_local=20, n_fixed=4, n_points=3000, stereo_frac=0.0, W=640, H=480,
               k_range=(2, 8), outlier_frac=0.05, arc=2.0):
    """Synthetic LocalBundleAdjustment graph: n_local optimised keyframes (id 0 fixed,
    as mnId==0 is in the reference) on an `arc`-metre arc facing a 4 x 3 x 3 m point
    volume, n_fixed fixed cameras (lFixedCameras), n_points points each observed by
    k ~ U{k_range} keyframes it projects into; octave ~ U{0..7} with the extractor's
    invSigma2, pixel noise N(0, 1.2^octave), outlier_frac outliers at +20 px, poses
    perturbed by 0.01 rad / 1 cm, points by 2 cm.  Poses are float32 Tcw (KeyFrame::GetPose)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    fx, fy, cx, cy = TUM1
    nk = n_local + n_fixed
    centre = np.array([0.0, 0.0, 5.0])
    radius = 5.0
    half = arc / radius / 2
    th = list(np.linspace(-half, half, n_local))
    for i in range(n_fixed):
        s = 1 if i % 2 == 0 else -1
        th.append(s * (half + 0.05 * (i // 2 + 1)))
    Rcw, tcw = [], []
    for t in th:
        C = centre + radius * np.array([np.sin(t), 0.0, -np.cos(t)])
        z = (centre - C) / np.linalg.norm(centre - C)
        x = np.array([np.cos(t), 0.0, np.sin(t)])
        y = np.cross(z, x)
        Rwc = np.stack([x, y, z], 1) @ _rot(rng.normal(0, 0.02, 3))
        R = Rwc.T
        Rcw.append(R)
        tcw.append(-R @ C)
    Rcw, tcw = np.array(Rcw), np.array(tcw)
    inv_sigma2 = (np.float32(1.0) / np.array([np.float32(1.2) ** (2 * l) for l in range(8)], np.float32))
    pts, e_pt, e_kf, e_st, e_obs, e_oct = [], [], [], [], [], []
    while len(pts) < n_points:
        X = np.array([rng.uniform(-2, 2), rng.uniform(-1.5, 1.5), rng.uniform(3.5, 6.5)])
        Xc = np.einsum("kij,j->ki", Rcw, X) + tcw
        u = fx * Xc[:, 0] / Xc[:, 2] + cx
        v = fy * Xc[:, 1] / Xc[:, 2] + cy
        vis = np.nonzero((Xc[:, 2] > 0.1) & (u >= 0) & (u < W) & (v >= 0) & (v < H))[0]
        if len(vis) < 2:
            continue
        k = min(int(rng.integers(k_range[0], k_range[1] + 1)), len(vis))
        obs_kf = np.sort(rng.choice(vis, size=k, replace=False))
        pi = len(pts)
        pts.append(X)
        for kf in obs_kf:
            lvl = int(rng.integers(0, 8))
            sig = 1.2 ** lvl
            uo = u[kf] + rng.normal(0, sig)
            vo = v[kf] + rng.normal(0, sig)
            if rng.random() < outlier_frac:
                uo += 20.0
            stereo = rng.random() < stereo_frac
            ur = uo - KITTI_BF / Xc[kf, 2] + rng.normal(0, sig) if stereo else -1.0
            e_pt.append(pi)
            e_kf.append(int(kf))
            e_st.append(1 if stereo else 0)
            e_obs.append([np.float32(uo), np.float32(vo), np.float32(ur)])
            e_oct.append(lvl)
    pts = np.array(pts)
    # perturb the optimised keyframes (not id 0) and the points
    Tcw = np.zeros((nk, 4, 4), np.float32)
    for i in range(nk):
        R, t = Rcw[i], tcw[i]
        if 0 < i < n_local:
            R = _rot(rng.normal(0, 0.01 / np.sqrt(3), 3)) @ R
            t = t + rng.normal(0, 0.01 / np.sqrt(3), 3)
        Tcw[i, :3, :3] = R
        Tcw[i, :3, 3] = t
        Tcw[i, 3, 3] = 1
    Xp = (pts + rng.normal(0, 0.02 / np.sqrt(3), pts.shape)).astype(np.float32).astype(np.float64)
    fixed = np.zeros(nk, np.uint8)
    fixed[0] = 1
    fixed[n_local:] = 1
    ne = len(e_pt)
    cam = np.tile(np.array([fx, fy, cx, cy, np.float32(KITTI_BF)], np.float64), (ne, 1))
    return {
        "Tcw": Tcw, "pose_fixed": fixed, "pose_id": np.arange(nk, dtype=np.int64),
        "point_xyz": Xp, "point_id": np.arange(n_points, dtype=np.int64) + nk,
        "point_bad": np.zeros(n_points, np.uint8),
        "edge_point": np.array(e_pt, np.int32), "edge_pose": np.array(e_kf, np.int32),
        "edge_stereo": np.array(e_st, np.uint8), "edge_obs": np.array(e_obs, np.float64),
        "edge_info": inv_sigma2[np.array(e_oct)].astype(np.float64), "edge_cam": cam,
        "edge_octave": np.array(e_oct, np.int32),
    }


def ba_problem_corridor(seed=42, n_local=60, n_fixed=4, n_points=8000, stereo_frac=0.0, W=640, H=480,
                        k_range=(2, 8), outlier_frac=0.05, spacing=0.5):
    """A scaled LocalBundleAdjustment window (SURVEY 8d's "scaled config"): n_local optimised
    keyframes (id 0 fixed) and n_fixed fixed cameras (half before, half after the window) along a
    straight path of `spacing`-metre steps, all looking at a wall of points 4-8 m ahead, so each
    point is visible from a contiguous run of keyframes and the covisibility (the reduced camera
    matrix's non-zero blocks) is banded, as along a real trajectory.  Each point is observed by
    k ~ U{k_range} of the keyframes it projects into; octaves, noise, outliers, stereo and the
    pose / point perturbations as ba_problem (vectorised: 100k points in seconds)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    fx, fy, cx, cy = TUM1
    nk = n_local + n_fixed
    nb = n_fixed // 2
    xs = np.concatenate([np.arange(n_local) * spacing,
                         -(np.arange(nb) + 1) * spacing,
                         n_local * spacing + np.arange(n_fixed - nb) * spacing])
    Rcw = np.stack([_rot(rng.normal(0, 0.01, 3)) for _ in range(nk)])
    C = np.stack([xs, rng.normal(0, 0.05, nk), np.zeros(nk)], 1)
    tcw = -np.einsum("kij,kj->ki", Rcw, C)
    inv_sigma2 = (np.float32(1.0) / np.array([np.float32(1.2) ** (2 * l) for l in range(8)], np.float32))
    x_lo, x_hi = xs.min() - 2.0, xs.max() + 2.0
    pts, obs_kf, cnt = [], [], []
    got = 0
    while got < n_points:
        B = 8192
        X = np.stack([rng.uniform(x_lo, x_hi, B), rng.uniform(-1.5, 1.5, B), rng.uniform(4.0, 8.0, B)], 1)
        Xc = np.einsum("kij,bj->bki", Rcw, X) + tcw[None]
        u = fx * Xc[..., 0] / Xc[..., 2] + cx
        v = fy * Xc[..., 1] / Xc[..., 2] + cy
        vis = (Xc[..., 2] > 0.1) & (u >= 0) & (u < W) & (v >= 0) & (v < H)
        nvis = vis.sum(1)
        k = np.minimum(rng.integers(k_range[0], k_range[1] + 1, B), nvis)
        keep = nvis >= 2
        keys = np.where(vis, rng.random((B, nk)), 2.0)
        order = np.argsort(keys, axis=1)
        for b in np.nonzero(keep)[0]:
            if got >= n_points:
                break
            sel = np.sort(order[b, :k[b]])
            pts.append(X[b])
            obs_kf.append(sel)
            got += 1
    pts = np.array(pts)
    cnt = np.array([len(o) for o in obs_kf])
    e_pt = np.repeat(np.arange(n_points), cnt).astype(np.int32)
    e_kf = np.concatenate(obs_kf).astype(np.int32)
    ne = len(e_pt)
    Xc = np.einsum("eij,ej->ei", Rcw[e_kf], pts[e_pt]) + tcw[e_kf]
    u = fx * Xc[:, 0] / Xc[:, 2] + cx
    v = fy * Xc[:, 1] / Xc[:, 2] + cy
    lvl = rng.integers(0, 8, ne)
    sig = 1.2 ** lvl
    uo = u + rng.normal(0, 1, ne) * sig
    vo = v + rng.normal(0, 1, ne) * sig
    uo = np.where(rng.random(ne) < outlier_frac, uo + 20.0, uo)
    st = rng.random(ne) < stereo_frac
    ur = np.where(st, uo - KITTI_BF / Xc[:, 2] + rng.normal(0, 1, ne) * sig, -1.0)
    e_obs = np.stack([uo, vo, ur], 1).astype(np.float32).astype(np.float64)
    Tcw = np.zeros((nk, 4, 4), np.float32)
    for i in range(nk):
        R, t = Rcw[i], tcw[i]
        if 0 < i < n_local:
            R = _rot(rng.normal(0, 0.01 / np.sqrt(3), 3)) @ R
            t = t + rng.normal(0, 0.01 / np.sqrt(3), 3)
        Tcw[i, :3, :3] = R
        Tcw[i, :3, 3] = t
        Tcw[i, 3, 3] = 1
    Xp = (pts + rng.normal(0, 0.02 / np.sqrt(3), pts.shape)).astype(np.float32).astype(np.float64)
    fixed = np.zeros(nk, np.uint8)
    fixed[0] = 1
    fixed[n_local:] = 1
    cam = np.tile(np.array([fx, fy, cx, cy, np.float32(KITTI_BF)], np.float64), (ne, 1))
    return {
        "Tcw": Tcw, "pose_fixed": fixed, "pose_id": np.arange(nk, dtype=np.int64),
        "point_xyz": Xp, "point_id": np.arange(n_points, dtype=np.int64) + nk,
        "point_bad": np.zeros(n_points, np.uint8),
        "edge_point": e_pt, "edge_pose": e_kf,
        "edge_stereo": st.astype(np.uint8), "edge_obs": e_obs,
        "edge_info": inv_sigma2[lvl].astype(np.float64), "edge_cam": cam,
        "edge_octave": lvl.astype(np.int32),
    }


def pose_problems(n_frames=8, seed=5, n_points=600, stereo_frac=0.0, outlier_frac=0.1, W=640, H=480,
                  rot_noise=0.01, trans_noise=0.02):
    """Synthetic Optimizer::PoseOptimization inputs (Tracking's motion-model / local-map step):
    per frame a true camera, n_points map points (float world positions) in view, keypoint
    observations = projection + N(0, 1.2^octave) px with octave ~ U{0..7}, outlier_frac of them
    displaced by +20 px, stereo_frac of them with a right coordinate ur = u - bf/z (+ noise),
    the others monocular (ur = -1, Frame::mvuRight); the initial pose (pFrame->mTcw, float) is
    the true one perturbed by rot_noise rad / trans_noise m.  TUM1 intrinsics, KITTI bf."""
    rng = np.random.Generator(np.random.PCG64(seed))
    fx, fy, cx, cy = TUM1
    inv_sigma2 = (np.float32(1.0) / np.array([np.float32(1.2) ** (2 * l) for l in range(8)], np.float32))
    frames = []
    for f in range(n_frames):
        R = _rot(rng.normal(0, 0.3, 3))
        t = rng.normal(0, 0.5, 3)
        X, obs, oct_ = [], [], []
        while len(X) < n_points:
            u, v = rng.uniform(0, W), rng.uniform(0, H)
            z = rng.uniform(1.0, 8.0)
            Xc = np.array([(u - cx) / fx * z, (v - cy) / fy * z, z])
            Xw = R.T @ (Xc - t)
            Xw32 = Xw.astype(np.float32).astype(np.float64)
            Xc2 = R @ Xw32 + t
            uu, vv = fx * Xc2[0] / Xc2[2] + cx, fy * Xc2[1] / Xc2[2] + cy
            lvl = int(rng.integers(0, 8))
            sig = 1.2 ** lvl
            uo, vo = uu + rng.normal(0, sig), vv + rng.normal(0, sig)
            if rng.random() < outlier_frac:
                uo += 20.0
            ur = uo - KITTI_BF / Xc2[2] + rng.normal(0, sig) if rng.random() < stereo_frac else -1.0
            X.append(Xw32)
            obs.append([np.float32(uo), np.float32(vo), np.float32(ur)])
            oct_.append(lvl)
        Rp = _rot(rng.normal(0, rot_noise / np.sqrt(3), 3)) @ R
        tp = t + rng.normal(0, trans_noise / np.sqrt(3), 3)
        T = np.eye(4, dtype=np.float32)
        T[:3, :3] = Rp
        T[:3, 3] = tp
        frames.append({"Tcw": T, "obs": np.array(obs, np.float64), "xw": np.array(X, np.float64),
                       "info": inv_sigma2[np.array(oct_)].astype(np.float64),
                       "cam": (fx, fy, cx, cy, float(np.float32(KITTI_BF))),
                       "true_R": R, "true_t": t})
    return frames


def fuse_problem(seed=3, n_kps=1000, n_mp=800, true_frac=0.6, stereo_frac=0.3, W=640, H=480, nlevels=8):
    """Synthetic ORBmatcher::Fuse input: a keyframe (identity-ish pose, TUM1 intrinsics, KITTI bf)
    with n_kps keypoints (octave U{0..7}, random descriptors, stereo_frac with a right
    coordinate), and n_mp map points — true_frac of them the back-projection of a keypoint at a
    random depth (plus < 1 px of projection noise, descriptor = the keypoint's with U{0..60} bits
    flipped), the rest random points in front of the camera.  Distance ranges follow
    MapPoint::UpdateNormalAndDepth (mfMaxDistance = dist * 1.2^octave, mfMinDistance =
    mfMaxDistance / 1.2^7); normals are the viewing ray plus noise."""
    rng = np.random.Generator(np.random.PCG64(seed))
    fx, fy, cx, cy = TUM1
    bf = float(np.float32(KITTI_BF))
    sf = np.array([np.float32(1.2) ** l for l in range(nlevels)], np.float32)
    isig2 = (np.float32(1.0) / (sf * sf)).astype(np.float32)
    R = _rot(rng.normal(0, 0.05, 3)).astype(np.float32)
    t = rng.normal(0, 0.1, 3).astype(np.float32)
    Tcw = np.zeros((3, 4), np.float32)
    Tcw[:, :3], Tcw[:, 3] = R, t
    Ow = (-R.T.astype(np.float64) @ t.astype(np.float64)).astype(np.float32)
    kx = rng.uniform(0, W, n_kps).astype(np.float32)
    ky = rng.uniform(0, H, n_kps).astype(np.float32)
    oct_ = rng.integers(0, nlevels, n_kps).astype(np.int32)
    desc = rng.integers(0, 256, (n_kps, 32), dtype=np.uint8)
    depth = rng.uniform(1.0, 8.0, n_kps)
    ur = np.where(rng.random(n_kps) < stereo_frac, kx - bf / depth, -1.0).astype(np.float32)
    xyz, nrm, mind, maxd, mdesc = [], [], [], [], []
    for i in range(n_mp):
        if rng.random() < true_frac:
            j = int(rng.integers(0, n_kps))
            z = depth[j]
            Xc = np.array([(kx[j] + rng.normal(0, 0.5) - cx) / fx * z, (ky[j] + rng.normal(0, 0.5) - cy) / fy * z, z])
            d = desc[j].copy()
            nb = int(rng.integers(0, 61))
            bits = np.unpackbits(d)
            bits[rng.choice(256, nb, replace=False)] ^= 1
            d = np.packbits(bits)
            lvl = int(oct_[j])
        else:
            Xc = np.array([rng.uniform(-3, 3), rng.uniform(-2, 2), rng.uniform(0.5, 9)])
            d = rng.integers(0, 256, 32, dtype=np.uint8)
            lvl = int(rng.integers(0, nlevels))
        Xw = (R.T.astype(np.float64) @ (Xc - t.astype(np.float64))).astype(np.float32)
        PO = Xw.astype(np.float64) - Ow
        dist = np.linalg.norm(PO)
        n = PO / dist + rng.normal(0, 0.1, 3)
        n /= np.linalg.norm(n)
        xyz.append(Xw)
        nrm.append(n.astype(np.float32))
        mx = np.float32(dist * float(sf[lvl]))
        maxd.append(mx)
        mind.append(np.float32(mx / sf[nlevels - 1]))
        mdesc.append(d)
    valid = (rng.random(n_mp) > 0.05).astype(np.uint8)
    return {"kf": {"x": kx, "y": ky, "octave": oct_, "desc": desc, "uright": ur, "angle": np.zeros(n_kps, np.float32),
                   "W": W, "H": H},
            "kp": {"Tcw": Tcw, "Ow": Ow, "cam": (fx, fy, cx, cy, bf), "log_scale_factor": float(np.log(np.float32(1.2))),
                   "n_levels": nlevels, "scale_factors": sf, "inv_level_sigma2": isig2},
            "mp_valid": valid, "mp_xyz": np.array(xyz, np.float32), "mp_normal": np.array(nrm, np.float32),
            "mp_min_dist": np.array(mind, np.float32), "mp_max_dist": np.array(maxd, np.float32),
            "mp_desc": np.array(mdesc, np.uint8)}


def triangulation_problem(seed=4, n_points=800, extra=150, stereo_frac=0.3, mp_frac=0.3, n_nodes=3000, W=640, H=480):
    """Synthetic ORBmatcher::SearchForTriangulation input: two keyframes 0.3 m apart viewing
    n_points 3-D points (each keyframe keeps ~85 % of them, plus `extra` unrelated keypoints);
    observations = projection + N(0, 0.7 px), octave U{0..7}, descriptors = the point's with
    U{0..30} bits flipped, angles = the point's plus N(0, 3 deg); vocabulary nodes: a point's
    features share node (id * 7919) mod n_nodes, extras take random nodes; mp_frac of the
    keypoints already carry a map point.  F12 = K1^-T [t12]x R12 K2^-1 (LocalMapping::ComputeF12),
    (ex, ey) = keyframe 1's centre projected into keyframe 2."""
    rng = np.random.Generator(np.random.PCG64(seed))
    fx, fy, cx, cy = TUM1
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float32)
    R1, t1 = np.eye(3), np.zeros(3)
    R2 = _rot(np.array([0.0, 0.05, 0.01]))
    t2 = np.array([-0.3, 0.02, 0.01])
    pts = np.stack([rng.uniform(-2, 2, n_points), rng.uniform(-1.5, 1.5, n_points), rng.uniform(2, 8, n_points)], 1)
    base = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    ang = rng.uniform(0, 360, n_points)
    sf = np.array([np.float32(1.2) ** l for l in range(8)], np.float32)
    sig2 = (sf * sf).astype(np.float32)

    def kf(R, t):
        xs, ys, os, ds, us, an, nodes = [], [], [], [], [], [], []
        keep = rng.random(n_points) < 0.85
        for i in np.nonzero(keep)[0]:
            Xc = R @ pts[i] + t
            u, v = fx * Xc[0] / Xc[2] + cx + rng.normal(0, 0.7), fy * Xc[1] / Xc[2] + cy + rng.normal(0, 0.7)
            if not (0 <= u < W and 0 <= v < H):
                continue
            bits = np.unpackbits(base[i])
            bits[rng.choice(256, int(rng.integers(0, 31)), replace=False)] ^= 1
            xs.append(u); ys.append(v); os.append(int(rng.integers(0, 8))); ds.append(np.packbits(bits))
            us.append(u - KITTI_BF / Xc[2] if rng.random() < stereo_frac else -1.0)
            an.append((ang[i] + rng.normal(0, 3)) % 360)
            nodes.append((i * 7919) % n_nodes)
        for _ in range(extra):
            xs.append(rng.uniform(0, W)); ys.append(rng.uniform(0, H)); os.append(int(rng.integers(0, 8)))
            ds.append(rng.integers(0, 256, 32, dtype=np.uint8)); us.append(-1.0); an.append(rng.uniform(0, 360))
            nodes.append(int(rng.integers(0, n_nodes)))
        nodes = np.array(nodes)
        order = np.argsort(nodes, kind="stable")
        un, starts = np.unique(nodes[order], return_index=True)
        start = np.append(starts, len(nodes)).astype(np.int32)
        n = len(xs)
        return {"x": np.array(xs, np.float32), "y": np.array(ys, np.float32), "octave": np.array(os, np.int32),
                "angle": np.array(an, np.float32), "desc": np.array(ds, np.uint8), "uright": np.array(us, np.float32),
                "has_mp": (rng.random(n) < mp_frac).astype(np.uint8), "nodes": un.astype(np.uint32),
                "start": start, "fidx": order.astype(np.int32), "W": W, "H": H}
    k1, k2 = kf(R1, t1), kf(R2, t2)
    R12 = (R1 @ R2.T).astype(np.float32)
    t12 = (-R1 @ R2.T @ t2 + t1).astype(np.float32)
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]], np.float32)
    Kinv = np.linalg.inv(K.astype(np.float64)).astype(np.float32)
    F12 = (Kinv.T @ tx @ R12 @ Kinv).astype(np.float32)
    C1 = -R1.T @ t1
    C2 = R2 @ C1 + t2
    ex, ey = np.float32(fx * C2[0] / C2[2] + cx), np.float32(fy * C2[1] / C2[2] + cy)
    return {"kf1": k1, "kf2": k2, "F12": F12, "ex": float(ex), "ey": float(ey), "scale_factors": sf,
            "level_sigma2": sig2, "R1": R1.astype(np.float32), "t1": t1.astype(np.float32),
            "R2": R2.astype(np.float32), "t2": t2.astype(np.float32)}


def vocabulary(k=10, L=4, seed=7, early_leaf=0.08, stop_frac=0.05, dup_frac=0.03):
    """A synthetic DBoW2 ORB vocabulary in loader node order (breadth first): (parent, is_leaf,
    desc, weight), entry 0 the root.  Children perturb their parent's descriptor (~1/8 of the
    bits flipped; the root's children are random), so descents are meaningful; a fraction of
    inner nodes stop early (leaves at uneven depth), duplicate their previous sibling's
    descriptor (ties: the first child wins) or carry weight 0 (stopped words).  k=10, L=6 has
    the 10^6-word shape of ORBvoc.txt."""
    rng = np.random.default_rng(seed)
    parent = [np.zeros(1, np.int64)]
    leaf = [np.zeros(1, bool)]
    desc = [np.zeros((1, 32), np.uint8)]
    frontier = np.zeros(1, np.int64)           # node ids expanded at the next level
    fdesc = np.zeros((1, 32), np.uint8)
    n = 1
    for depth in range(1, L + 1):
        m = len(frontier)
        if m == 0:
            break
        par = np.repeat(frontier, k)
        pd = np.repeat(fdesc, k, axis=0)
        if depth == 1:
            d = rng.integers(0, 256, (m * k, 32), dtype=np.uint8)
        else:
            flip = (rng.integers(0, 256, (m * k, 32), dtype=np.uint8) & rng.integers(0, 256, (m * k, 32), dtype=np.uint8)
                    & rng.integers(0, 256, (m * k, 32), dtype=np.uint8))
            d = pd ^ flip
        dup = rng.random(m * k) < dup_frac
        dup[::k] = False
        d[dup] = d[np.flatnonzero(dup) - 1]
        is_leaf = np.full(m * k, depth == L)
        if depth < L and depth >= 2:
            is_leaf |= rng.random(m * k) < early_leaf
        ids = np.arange(n, n + m * k, dtype=np.int64)
        parent.append(par)
        leaf.append(is_leaf)
        desc.append(d)
        n += m * k
        frontier = ids[~is_leaf]
        fdesc = d[~is_leaf]
    parent = np.concatenate(parent)
    leaf = np.concatenate(leaf)
    desc = np.concatenate(desc)
    weight = np.where(leaf, rng.uniform(0.5, 9.0, n), 0.0)
    weight[leaf & (rng.random(n) < stop_frac)] = 0.0
    return parent, leaf, desc, weight


def bow_features(voc_desc, voc_leaf, n, seed=11, random_frac=0.1):
    """n query descriptors: leaf descriptors with ~1/8 of the bits flipped, a fraction uniform
    random."""
    rng = np.random.default_rng(seed)
    leaves = np.flatnonzero(voc_leaf)
    f = voc_desc[rng.choice(leaves, n)].copy()
    f ^= (rng.integers(0, 256, (n, 32), dtype=np.uint8) & rng.integers(0, 256, (n, 32), dtype=np.uint8)
          & rng.integers(0, 256, (n, 32), dtype=np.uint8))
    r = rng.random(n) < random_frac
    f[r] = rng.integers(0, 256, (int(r.sum()), 32), dtype=np.uint8)
    return f


def bow_match_problem(voc, seed=9, n_land=900, keep=0.8, extra=200, mp_frac=0.75, rot_deg=25.0, W=640, H=480):
    """Synthetic ORBmatcher::SearchByBoW input over a vocabulary from vocabulary(): two views of
    n_land landmark descriptors (near vocabulary leaves); each view keeps ~keep of them with
    U{0..20} bits flipped, plus `extra` random features; angles = the landmark's + N(0, 3 deg),
    the second view turned by rot_deg; mp_frac of the features carry a good map point.  The
    feature vectors come from transforming each view's descriptors with the vocabulary."""
    rng = np.random.Generator(np.random.PCG64(seed))
    base = bow_features(voc[2], voc[1], n_land, seed=seed + 1)
    ang = rng.uniform(0, 360, n_land)

    def view(turn):
        sel = np.flatnonzero(rng.random(n_land) < keep)
        d = base[sel].copy()
        for r in range(len(sel)):
            bits = np.unpackbits(d[r])
            bits[rng.choice(256, int(rng.integers(0, 21)), replace=False)] ^= 1
            d[r] = np.packbits(bits)
        a = (ang[sel] + turn + rng.normal(0, 3, len(sel))) % 360
        d = np.concatenate([d, rng.integers(0, 256, (extra, 32), dtype=np.uint8)])
        a = np.concatenate([a, rng.uniform(0, 360, extra)])
        perm = rng.permutation(len(d))
        n = len(d)
        return {"x": rng.uniform(0, W, n).astype(np.float32), "y": rng.uniform(0, H, n).astype(np.float32),
                "octave": rng.integers(0, 8, n).astype(np.int32), "angle": a[perm].astype(np.float32),
                "desc": np.ascontiguousarray(d[perm]), "uright": None,
                "has_mp": (rng.random(n) < mp_frac).astype(np.uint8), "W": W, "H": H}
    return view(0.0), view(rot_deg)


def sim3_problem(seed=6, n_points=700, keep=0.85, extra=120, mp_frac=0.85, s12=1.0, W=640, H=480, nlevels=8):
    """Synthetic ORBmatcher::SearchBySim3 input: two keyframes 0.4 m apart viewing n_points
    3-D points; keypoint = projection + N(0, 0.7 px), octave = the point's level, descriptor = the
    point's with U{0..25} bits flipped; mp_frac of the point keypoints carry the map point (xyz,
    mfMinDistance / mfMaxDistance from the distance to camera 1, descriptor = the point's); the
    Sim3 is (s12, R12 = R1 R2^T, t12 = t1 - s12 R12 t2).  Returns per keyframe the keypoints, the
    map-point arrays (per keypoint) and [R|t]; plus s12, R12, t12 and the camera."""
    rng = np.random.Generator(np.random.PCG64(seed))
    fx, fy, cx, cy = TUM1
    sf = np.array([np.float32(1.2) ** l for l in range(nlevels)], np.float32)
    R1, t1 = np.eye(3), np.zeros(3)
    R2 = _rot(np.array([0.02, 0.08, -0.01]))
    t2 = np.array([-0.4, 0.03, 0.02])
    pts = np.stack([rng.uniform(-2, 2, n_points), rng.uniform(-1.5, 1.5, n_points), rng.uniform(2, 8, n_points)], 1)
    base = rng.integers(0, 256, (n_points, 32), dtype=np.uint8)
    lvl = rng.integers(0, nlevels, n_points)
    dist1 = np.linalg.norm(pts, axis=1)
    maxd = (dist1 * sf[lvl]).astype(np.float32)
    mind = (maxd / sf[nlevels - 1]).astype(np.float32)

    def kf(R, t):
        xs, ys, os, ds, an, mp = [], [], [], [], [], []
        for i in np.flatnonzero(rng.random(n_points) < keep):
            Xc = R @ pts[i] + t
            u, v = fx * Xc[0] / Xc[2] + cx + rng.normal(0, 0.7), fy * Xc[1] / Xc[2] + cy + rng.normal(0, 0.7)
            if not (0 <= u < W and 0 <= v < H):
                continue
            bits = np.unpackbits(base[i])
            bits[rng.choice(256, int(rng.integers(0, 26)), replace=False)] ^= 1
            xs.append(u); ys.append(v); os.append(int(lvl[i])); ds.append(np.packbits(bits)); an.append(0.0)
            mp.append(i if rng.random() < mp_frac else -1)
        for _ in range(extra):
            xs.append(rng.uniform(0, W)); ys.append(rng.uniform(0, H)); os.append(int(rng.integers(0, nlevels)))
            ds.append(rng.integers(0, 256, 32, dtype=np.uint8)); an.append(0.0); mp.append(-1)
        mp = np.array(mp)
        has = mp >= 0
        n = len(xs)
        xyz = np.zeros((n, 3), np.float32)
        xyz[has] = pts[mp[has]].astype(np.float32)
        md = np.zeros((n, 32), np.uint8)
        md[has] = base[mp[has]]
        mn, mx = np.zeros(n, np.float32), np.zeros(n, np.float32)
        mn[has], mx[has] = mind[mp[has]], maxd[mp[has]]
        T = np.zeros((3, 4), np.float32)
        T[:, :3], T[:, 3] = R, t
        return {"x": np.array(xs, np.float32), "y": np.array(ys, np.float32), "octave": np.array(os, np.int32),
                "angle": np.array(an, np.float32), "desc": np.array(ds, np.uint8), "uright": None, "W": W, "H": H,
                "mp_valid": has.astype(np.uint8), "mp_xyz": xyz, "mp_min_dist": mn, "mp_max_dist": mx, "mp_desc": md,
                "Tcw": T, "point": mp}
    k1, k2 = kf(R1, t1), kf(R2, t2)
    R12 = (R1 @ R2.T).astype(np.float32)
    t12 = (t1 - s12 * R12.astype(np.float64) @ t2).astype(np.float32)
    return {"kf1": k1, "kf2": k2, "s12": np.float32(s12), "R12": R12, "t12": t12, "cam": (fx, fy, cx, cy),
            "scale_factors": sf, "log_scale_factor": float(np.log(np.float32(1.2))), "n_levels": nlevels}


def sim3_side_transforms(p):
    """sR21 = (1/s12) R12^T, t21 = -sR21 t12 and sR12 = s12 R12 as R/src/ORBmatcher.cpp:1315-1318
    compute them (float Mats: scaled elements rounded to float, the product accumulated in double)."""
    s12 = float(p["s12"])
    R12 = np.asarray(p["R12"], np.float32)
    sR12 = (R12.astype(np.float64) * s12).astype(np.float32)
    sR21 = (R12.T.astype(np.float64) * (1.0 / s12)).astype(np.float32)
    t21 = (-(sR21.astype(np.float64) @ np.asarray(p["t12"], np.float32).astype(np.float64))).astype(np.float32)
    S1 = np.zeros((3, 4), np.float32)
    S1[:, :3], S1[:, 3] = sR21, t21
    S2 = np.zeros((3, 4), np.float32)
    S2[:, :3], S2[:, 3] = sR12, p["t12"]
    return S1, S2
