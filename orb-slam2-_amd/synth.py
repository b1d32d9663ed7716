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


def stream(seed: int, W: int, H: int, n: int) -> np.ndarray:
    cv = canvas(seed, W, H)
    return np.stack([frame(cv, W, H, t) for t in range(n)])
