"""Synthetic LocoMouse configuration: video, background, calibration, config
and detector model.

The reference ships no video, model, calibration or config fixtures, so every
parity test and benchmark runs on this deterministic scene (include/lm_synth.h
holds the C/HIP twin of the frame generator; test_synthetic.py checks they
agree bit for bit).  Detector weights are float64 arrays like the MATLAB-
trained models the reference loads from model.yml (LocoMouse_class.cpp:3106-3148).
"""
import ctypes as C

import numpy as np

from .abi import lm_detector, lm_location_prior, lm_model, lm_params, lm_rect, lm_setup

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def tri(t, period, amp):
    p = t % period
    q = (4 * amp * p) // period
    if q <= amp:
        return q
    if q <= 3 * amp:
        return 2 * amp - q
    return q - 4 * amp


def scene(rows, cols):
    s = 2 if rows >= 512 else 1
    return {"rows": rows, "cols": cols, "scale": s, "cx0": (cols * 500) // 1024, "side_cy": 48 * s, "bottom_cy": 176 * s}


def synth_background(rows, cols):
    idx = np.arange(rows * cols, dtype=np.uint64)
    return (16 + splitmix64(np.uint64(0xB4C0000000000000) ^ idx) % np.uint64(16)).astype(np.uint8).reshape(rows, cols)


def synth_frame(rows, cols, f):
    """numpy twin of lm_synth_pixel for one frame (include/lm_synth.h)."""
    sc = scene(rows, cols)
    s = sc["scale"]
    idx = np.arange(rows * cols, dtype=np.uint64)
    v = synth_background(rows, cols).reshape(-1).astype(np.int32)
    seed = np.uint64(((0x5EED0000 + f) & 0xFFFFFFFF) << 32)
    v += (splitmix64(seed ^ idx) % np.uint64(6)).astype(np.int32)
    r = (idx // np.uint64(cols)).astype(np.int64)
    c = (idx % np.uint64(cols)).astype(np.int64)
    cx = sc["cx0"] + s * tri(f, 50, 40)
    side = r < 96 * s
    cy = np.where(side, sc["side_cy"], sc["bottom_cy"])
    a, b = 150 * s, np.where(side, 30 * s, 50 * s)
    dx, dy = c - cx, r - cy
    v += np.where(dx * dx * b * b + dy * dy * a * a <= a * a * b * b, 80, 0)
    for k in range(4):
        dxk = (-110, -40, 40, 110)[k] * s
        px = cx + dxk + s * tri(f + 5 * k, 20, 30)
        py = np.where(side, 86 * s, sc["bottom_cy"] + (58 if (k & 1) else -58) * s)
        ddx, ddy = c - px, r - py
        v += np.where(ddx * ddx + ddy * ddy <= 36 * s * s, 100, 0)
    ddx, ddy = c - (cx + 158 * s), r - cy
    v += np.where(ddx * ddx + ddy * ddy <= 25 * s * s, 110, 0)
    v += np.where((c >= cx - 330 * s) & (c <= cx - 150 * s) & (dy >= -s) & (dy <= s), 150, 0)
    return np.minimum(v, 255).astype(np.uint8).reshape(rows, cols)


def synth_frames(rows, cols, first, n):
    return np.stack([synth_frame(rows, cols, first + i) for i in range(n)])


# ---------------------------------------------------------------- detectors

def _uniform(seed, n):
    u = splitmix64(np.uint64(seed) * np.uint64(1000003) + np.arange(n, dtype=np.uint64))
    return (u >> np.uint64(11)).astype(np.float64) / float(1 << 53) - 0.5


def dog_detector(kh, kw, radius, seed):
    """Zero-mean centre-surround (difference of Gaussians) point detector,
    scaled by 1/(kh*kw), with a small seeded perturbation that breaks mirror
    symmetry (exact score ties would otherwise be common)."""
    yy = np.arange(kh, dtype=np.float64)[:, None] - (kh - 1) / 2.0
    xx = np.arange(kw, dtype=np.float64)[None, :] - (kw - 1) / 2.0
    d2 = yy * yy + xx * xx
    c = np.exp(-d2 / (2 * (0.8 * radius) ** 2))
    srd = np.exp(-d2 / (2 * (2.0 * radius) ** 2))
    w = c / c.sum() - srd / srd.sum()
    w = w / np.abs(w).max() + 0.02 * _uniform(seed, kh * kw).reshape(kh, kw)
    w -= w.mean()
    return w / (kh * kw)


def line_detector(kh, kw, half_thickness, seed):
    """Horizontal bar detector for the tail (positive band, negative flanks)."""
    yy = np.abs(np.arange(kh, dtype=np.float64) - (kh - 1) / 2.0)[:, None] * np.ones((1, kw))
    w = np.where(yy <= half_thickness, 1.0, -0.35) + 0.02 * _uniform(seed, kh * kw).reshape(kh, kw)
    w -= w.mean()
    return w / (kh * kw)


# Detector sizes (rows, cols) at scale 1 and frozen biases.
# Biases were tuned once on frames 0..15 so that ~2 % of the unmasked crop
# pixels score > 0 for the point detectors and the tail line dominates the
# tail detectors' largest connected component.  Scale-2 biases are provisional.
DETECTOR_SPECS = {
    # name: (rows, cols, kind, radius_or_halfthickness, seed, bias_scale1, bias_scale2)
    "paw_bottom": (24, 24, "dog", 6.0, 11, 6.0, 6.0),
    "snout_bottom": (30, 30, "dog", 5.0, 12, 3.5, 3.5),
    "tail_bottom": (16, 26, "line", 1.5, 13, 20.0, 20.0),
    "paw_side": (22, 22, "dog", 6.0, 14, 8.5, 8.5),
    "snout_side": (26, 26, "dog", 5.0, 15, 5.5, 5.5),
    "tail_side": (16, 26, "line", 1.5, 16, 22.0, 22.0),
}


def make_weights(name, scale=1):
    kh, kw, kind, r, seed, _, _ = DETECTOR_SPECS[name]
    kh, kw, r = kh * scale, kw * scale, r * scale
    if kind == "dog":
        return dog_detector(kh, kw, r, seed)
    return line_detector(kh, kw, r, seed)


def default_bias(name, scale=1):
    spec = DETECTOR_SPECS[name]
    return spec[5] if scale == 1 else spec[6]


class SyntheticConfig:
    """Holds every array the C structs point to (keep this object alive while
    the structs are in use)."""

    def __init__(self, rows=256, cols=1024, method=0, flip=False, connectivity=8, biases=None, weights=None,
                 bounding_boxes=None):
        self.rows, self.cols = rows, cols
        s = 2 if rows >= 512 else 1
        self.scale = s
        self.background = np.ascontiguousarray(synth_background(rows, cols))
        self.calib = np.ascontiguousarray(np.arange(rows * cols, dtype=np.int32).reshape(rows, cols))
        self.weights = {}
        self.biases = {}
        for name in DETECTOR_SPECS:
            w = weights[name] if weights and name in weights else make_weights(name, s)
            self.weights[name] = np.ascontiguousarray(w, dtype=np.float64)
            self.biases[name] = float(biases[name]) if biases and name in biases else default_bias(name, s)

        su = lm_setup()
        su.method = method
        su.flip = 1 if flip else 0
        su.video_rows, su.video_cols = rows, cols
        su.background = self.background.ctypes.data_as(C.POINTER(C.c_uint8))
        su.calib_rows, su.calib_cols = rows, cols
        su.ind_warp_mapping = self.calib.ctypes.data_as(C.POINTER(C.c_int32))
        su.view_box_side = lm_rect(0, 0, cols, 96 * s)
        su.view_box_bottom = lm_rect(0, 96 * s, cols, rows - 96 * s)
        self.setup = su

        p = lm_params()
        p.conn_comp_connectivity = connectivity
        p.max_displacement_bottom = 15 * s
        p.max_displacement_side = 15 * s
        p.occlusion_grid_spacing_pixels_side = 20 * s
        p.occlusion_grid_spacing_pixels_bottom = 20 * s
        p.use_provided_bounding_box = 1
        p.transform_gray_values = 0
        p.side_bottom_min_overlap = 0.7
        p.occlusion_grid_max_width = 0.75
        p.tail_sub_bounding_box = 0.6
        p.alpha_vel_bottom = 0.1
        p.alpha_vel_side = 100.0
        p.pairwise_occluded_cost = 0.01
        priors = [
            (0.25, 0.10, 0.60, 0.00, 0.70, 0.00, 0.60),
            (0.40, 0.90, 0.60, 0.00, 0.80, 0.40, 1.00),
            (0.60, 0.10, 0.60, 0.20, 1.00, 0.00, 0.60),
            (0.75, 0.90, 0.60, 0.30, 1.00, 0.40, 1.00),
            (0.90, 0.50, 0.50, 0.60, 1.00, 0.20, 0.80),
        ]
        for i, row in enumerate(priors):
            p.location_prior[i] = lm_location_prior(*row)
        if bounding_boxes is None:
            bounding_boxes = {"side": (300 * s, 3 * s, 400 * s, 90 * s), "bottom": (300 * s, 106 * s, 400 * s, 140 * s)}
        p.bounding_box_side = lm_rect(*bounding_boxes["side"])
        p.bounding_box_bottom = lm_rect(*bounding_boxes["bottom"])
        self.params = p

        m = lm_model()
        for name in DETECTOR_SPECS:
            w = self.weights[name]
            setattr(m, name, lm_detector(w.ctypes.data_as(C.POINTER(C.c_double)), w.shape[0], w.shape[1], self.biases[name]))
        self.model = m

    def frames(self, first, n):
        return synth_frames(self.rows, self.cols, first, n)
