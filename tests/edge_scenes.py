"""Scenes and configurations for the reference's edge paths (shared by the
CPU oracle tests and the GPU parity tests):

* blank frames (frame == background: sat(F - BKG) = 0 everywhere, so
  normalize's min == max, the LUT is all zero and no score is positive),
* frames whose bottom view is blank (empty bottom lists, so
  detectSideCandidates skips both side lists, LocoMouse_class.cpp:820-833),
* frames whose side view is blank (side lists with zero positives,
  peakClustering's N_detections == 0, :1652-1655, and P22D "no side" entries),
* detectors that never fire (zero-positive lists every frame),
* dense tail maps (the whole tail box foreground) and checkerboard tail maps
  (one run per two columns: more runs than k_tail's LDS holds),
* detectors wider / taller than the width-specialised correlation kernels,
* the CV_8U grey-level LUT of transform_gray_values.
"""
import numpy as np

from locomouse_cpp_amd import abi
from locomouse_cpp_amd import synthetic as S

SIDE_ROWS = 96  # view_box_side height of the synthetic scene (scale 1)


def blank(cfg):
    return cfg.background.copy()


def blank_rows(cfg, frame, r0, r1):
    f = frame.copy()
    f[r0:r1] = cfg.background[r0:r1]
    return f


def edge_video(cfg, first=0):
    """14 frames: 2 blank, 4 and 5 blank (a batch seam of max_batch 5 lies
    between them), 7 bottom-blank, 9 side-blank, 11 blank, 13 bottom-blank."""
    fr = cfg.frames(first, 14)
    for k in (2, 4, 5, 11):
        fr[k] = blank(cfg)
    s = cfg.scale
    for k in (7, 13):
        fr[k] = blank_rows(cfg, fr[k], SIDE_ROWS * s, cfg.rows)
    fr[9] = blank_rows(cfg, fr[9], 0, SIDE_ROWS * s)
    return fr


def silent_config(names):
    """Detectors in `names` get a bias no score reaches (zero positives)."""
    return S.SyntheticConfig(biases={n: 1e6 for n in names})


def dense_tail_config():
    """Tail detectors with -rho = +1e6: every tail score is positive, the
    tail boxes are one component each and TAIL_MASK covers the whole box."""
    return S.SyntheticConfig(biases={"tail_bottom": -1e6, "tail_side": -1e6})


def pixel_tail_config(connectivity=8):
    """1x1 tail detectors (weight 1, bias 127.5): a tail score is positive
    exactly where the corrected pixel is >= 128, so the frame's pixels draw
    the tail maps directly; 1x1 also runs the generic correlation kernel."""
    one = np.ones((1, 1))
    return S.SyntheticConfig(connectivity=connectivity, weights={"tail_bottom": one, "tail_side": one},
                             biases={"tail_bottom": 127.5, "tail_side": 127.5})


def checker_frames(cfg, n, first=0, period=2, seed=0):
    """Frames whose whole image is a checkerboard of bright (+200) and
    background pixels with the phase varying per frame, plus a few noise
    pixels: thousands of runs per tail map."""
    rng = np.random.default_rng(seed)
    out = []
    r = np.arange(cfg.rows)[:, None]
    c = np.arange(cfg.cols)[None, :]
    for k in range(n):
        pat = (((r // (period // 2 or 1)) + (c // (period // 2 or 1)) + k) & 1).astype(bool)
        pat ^= rng.random((cfg.rows, cfg.cols)) < 0.02
        f = cfg.background.astype(np.int32) + np.where(pat, 200, 0)
        out.append(np.minimum(f, 255).astype(np.uint8))
    return np.stack(out)


def _bias_for_rate(cfg, names, rate=0.02):
    """Biases putting about `rate` of the scores of the first frame above 0."""
    from oracle import oracle as O
    c0 = S.SyntheticConfig(rows=cfg.rows, cols=cfg.cols, weights=cfg.weights, biases={n: 0.0 for n in S.DETECTOR_SPECS})
    r0 = O.OracleRun(c0, c0.frames(0, 1), flags=O.KEEP_DEBUG)
    det = {n: i for i, n in enumerate(abi.DETECTORS)}
    out = dict(cfg.biases)
    for n in names:
        v = np.sort(r0.scores(0, det[n]).ravel())
        out[n] = float(v[int((1 - rate) * (len(v) - 1))])
    return out


def odd_size_config():
    """snout_bottom 70x70 (taller and wider than any specialised kernel: the
    generic kernel in two row chunks), paw_side 13x13 and tail_side 9x33
    (widths without an instantiation), paw_bottom 24x24 as usual."""
    w = {"snout_bottom": S.dog_detector(70, 70, 9.0, 21), "paw_side": S.dog_detector(13, 13, 4.0, 22),
         "tail_side": S.line_detector(9, 33, 1.5, 23)}
    base = S.SyntheticConfig(weights=w)
    return S.SyntheticConfig(weights=w, biases=_bias_for_rate(base, ["snout_bottom", "paw_side"]))


def wide_ring_config():
    """Ring-kernel widths above 32 (k_corr_rw<36..64>): snout_bottom 40x40,
    paw_side 20 rows x 64 columns, tail_side 16 x 36 and tail_bottom 16 x 48
    (rows x columns); paw_bottom 24x24 and the default scene otherwise."""
    w = {"snout_bottom": S.dog_detector(40, 40, 6.0, 31), "paw_side": S.dog_detector(20, 64, 5.0, 32),
         "tail_side": S.line_detector(16, 36, 1.5, 33), "tail_bottom": S.line_detector(16, 48, 1.5, 34)}
    base = S.SyntheticConfig(weights=w)
    return S.SyntheticConfig(weights=w, biases=_bias_for_rate(base, ["snout_bottom", "paw_side"]))


def big_tail_config():
    """2048x1024 frames with a 2000-wide, 700-row bottom box and
    tail_sub_bounding_box = 1: k_tail's bitmaps of the tail box exceed the
    LDS (k_tail<true> on its global workspace), and the 75 x 35 = 2,625-node
    occlusion grid exceeds k_post's LDS columns (global-scratch k_post for
    every block).  9x9 detectors keep the oracle fast."""
    w = {n: S.dog_detector(9, 9, 2.0, 40 + i) for i, n in enumerate(S.DETECTOR_SPECS) if "tail" not in n}
    w["tail_bottom"] = S.line_detector(9, 9, 1.5, 50)
    w["tail_side"] = S.line_detector(9, 9, 1.5, 51)
    boxes = {"side": (20, 5, 2000, 180), "bottom": (20, 310, 2000, 700)}
    base = S.SyntheticConfig(rows=1024, cols=2048, weights=w, bounding_boxes=boxes)
    b = _bias_for_rate(base, ["paw_bottom", "snout_bottom", "paw_side", "snout_side"])
    b.update({k: v for k, v in _bias_for_rate(base, ["tail_bottom", "tail_side"], rate=0.05).items()
              if k.startswith("tail")})
    cfg = S.SyntheticConfig(rows=1024, cols=2048, weights=w, bounding_boxes=boxes, biases=b)
    cfg.params.tail_sub_bounding_box = 1.0
    return cfg


def gamma_table(g=0.6):
    return np.round(255.0 * (np.arange(256) / 255.0) ** g)


def gray_lut_config(table=None, depth=abi.LM_DEPTH_8U, **kw):
    cfg = S.SyntheticConfig(**kw)
    t = gamma_table() if table is None else table
    cfg.params.transform_gray_values = 1
    for i in range(256):
        cfg.params.gray_value_transformation[i] = float(t[i])
    cfg.params.gray_value_transformation_depth = depth
    return cfg


def moving_corners(cfg, n, first=0, amp=6):
    """Per-frame bottom-right corners (bb of lm_detect_batch) that move the
    crops by a few pixels around the provided box."""
    p = cfg.params
    x0 = p.bounding_box_bottom.x + p.bounding_box_bottom.width
    yb0 = p.bounding_box_bottom.y + p.bounding_box_bottom.height
    ys0 = p.bounding_box_side.y + p.bounding_box_side.height
    k = np.arange(first, first + n)
    dx = (amp * np.sin(k * 0.9)).astype(np.int32)
    dy = (amp // 2 * np.cos(k * 1.3)).astype(np.int32)
    return np.stack([x0 + dx, yb0 + dy, ys0 - dy], 1).astype(np.int32)
