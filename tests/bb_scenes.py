"""Frame sequences for the whole-video bounding-box pass.

The reference ships no video, so these are synthetic two-view scenes over
SyntheticConfig's background: a body blob per view that moves with the frame
index, small distractor discs (some removed by the median filter, some left
as separate components), low-amplitude noise, and optional edge cases: blobs
touching the image border (exercising medianBlur's carried border ring),
frames equal to the background (normalize of an all-zero difference), and
two equal-area blobs (largest-component tie order)."""
import numpy as np


def _disc(yy, xx, cy, cx, r):
    return (yy - cy) ** 2 + (xx - cx) ** 2 <= r * r


def _ellipse(yy, xx, cy, cx, a, b):
    return ((xx - cx) / a) ** 2 + ((yy - cy) / b) ** 2 <= 1.0


def bb_frames(cfg, n, first=0, noise=1, seed=0, border=False, empty_every=0, ties=False, side_h=None):
    rows, cols, s = cfg.rows, cfg.cols, cfg.scale
    bkg = cfg.background.astype(np.int32)
    yy, xx = np.mgrid[0:rows, 0:cols]
    side_h = 96 * s if side_h is None else side_h
    out = np.zeros((n, rows, cols), dtype=np.uint8)
    for i in range(n):
        f = first + i
        rng = np.random.default_rng(seed * 1000003 + f)
        v = bkg.copy()
        if empty_every and f % empty_every == empty_every - 1:
            out[i] = np.clip(v, 0, 255)
            continue
        if ties and f % 3 == 1:
            # two equal discs in the bottom view only, mirrored about the centre
            cy = side_h + (rows - side_h) // 2
            for cx in (cols // 4, 3 * cols // 4):
                v += np.where(_disc(yy, xx, cy, cx, 12 * s), 90, 0)
        else:
            cx = cols // 2 + int(0.3 * cols * np.sin(0.21 * f))
            v += np.where(_ellipse(yy, xx, side_h // 2, cx, 0.12 * cols, 0.3 * side_h), 70, 0)
            v += np.where(_ellipse(yy, xx, side_h + (rows - side_h) // 2, cx + 9 * s, 0.14 * cols,
                                   0.3 * (rows - side_h)), 80, 0)
            for _ in range(6):  # distractors: radius 2 vanish under an 11x11 median, 8 survive
                r = int(rng.choice([2, 3, 8])) * s
                v += np.where(_disc(yy, xx, int(rng.integers(0, rows)), int(rng.integers(0, cols)), r), 60, 0)
        if border and f % 2 == 0:
            v[: 3 * s, :] += 90                                  # top rows
            v[:, -4 * s:] += 90                                   # right columns
            v += np.where(_disc(yy, xx, rows - 1, 5 * s, 10 * s), 90, 0)  # bottom-left corner
        if noise:
            v += rng.integers(0, noise + 1, size=(rows, cols))
        out[i] = np.clip(v, 0, 255)
    return out
