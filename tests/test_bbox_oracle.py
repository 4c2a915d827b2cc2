"""CPU checks of the whole-video bounding-box pass restatement (oracle/,
SURVEY.md §8(f) row 1) and of the reformulation the gfx950 kernels use.

PARITY UNPINNED against the reference itself: it needs OpenCV (absent here)
and ships no BB fixtures.  These tests pin the oracle's pieces against
independent numpy models of the OpenCV primitives it restates (medianBlur
with BORDER_REPLICATE, the firstLastOverT bookkeeping, vecmovingaverage) and
check that the 0/1 box-count formulation of lm_bbox.hip reproduces the
oracle's literal in-place medianBlur, border ring included."""
import numpy as np
import pytest

from locomouse_cpp_amd import abi
from locomouse_cpp_amd.synthetic import SyntheticConfig
from oracle import oracle as O
from tests.bb_scenes import bb_frames


def np_median_replicate(img, k):
    p = k // 2
    P = np.pad(img, p, mode="edge")
    win = np.lib.stride_tricks.sliding_window_view(P, (k, k))
    return np.median(win.reshape(img.shape[0], img.shape[1], -1), axis=2).astype(np.uint8)


@pytest.mark.parametrize("k", [1, 3, 5, 11])
def test_median_blur_matches_replicate_border_median(k):
    rng = np.random.default_rng(k)
    for shape in [(7, 9), (23, 31), (40, 17)]:
        img = rng.integers(0, 256, size=shape).astype(np.uint8)
        img[rng.random(shape) < 0.3] = 0  # many equal values
        assert np.array_equal(O.median_blur(img, k), np_median_replicate(img, k))


def test_first_last_over_t_bookkeeping():
    v = np.array([0, 255, 0, 510, 255, 0], dtype=np.int32)
    # integer comparison
    assert O.first_last(v, 255, integer=True) == (1, 4)
    assert O.first_last(v, 300, integer=True) == (3, 0)  # one entry passes: first_last[1] stays 0
    assert O.first_last(v, 600, integer=True) == (-1, -1)
    assert O.first_last(v, 0, integer=True) == (0, 5)
    # as executed: the int32 sums are read as float bit patterns (denormals)
    assert O.first_last(v, 1, integer=False) == (-1, -1)
    assert O.first_last(v, 0, integer=False) == (0, 5)
    big = np.array([0, 0x3F800000, 5], dtype=np.int32)  # bit pattern of 1.0f
    assert O.first_last(big, 1, integer=False) == (1, 0)


def test_moving_average_restatement():
    rng = np.random.default_rng(3)
    for n, w in [(1, 5), (5, 5), (6, 5), (20, 5), (20, 1), (9, 3), (30, 7)]:
        v = rng.integers(-3, 900, size=n).astype(np.float64)
        ref = np.zeros(n, dtype=np.uint32)
        if w >= n:
            ref[:] = [np.uint32(np.int64(x) & 0xFFFFFFFF) for x in v]
        else:
            h = w // 2
            for i in range(n):
                if i < h or i >= n - h - 1:
                    ref[i] = np.uint32(np.int64(v[i]) & 0xFFFFFFFF)
                else:
                    ref[i] = np.uint32(np.int64(np.floor(v[i - h:i + h + 1].sum() / w)) & 0xFFFFFFFF)
        assert np.array_equal(O.moving_average(v, w), ref), (n, w)


def corrected_indicator(cfg, frame):
    """[readFrame(I) >= 3] for the identity calibration, no flip (:1302-1327)."""
    d = np.maximum(frame.astype(np.int32) - cfg.background.astype(np.int32), 0)
    mn, mx = d.min(), d.max()
    scale = 255.0 / (mx - mn) if mx - mn > np.finfo(np.float64).eps else 0.0
    shift = -mn * scale
    lut = np.rint(np.arange(256, dtype=np.float32) * np.float32(scale) + np.float32(shift))
    lut = np.clip(lut, 0, 255).astype(np.uint8)
    if abs(scale - 1) < np.finfo(np.float64).eps and abs(shift) < np.finfo(np.float64).eps:
        lut = np.arange(256, dtype=np.uint8)
    return lut[d] >= 3


def box_count_model(cfg, frames, k):
    """lm_bbox.hip's formulation: k x k window counts of 0/1 indicators, the
    border ring of I_median carried as 0/1 between frames."""
    p, thr = k // 2, (k * k + 1) // 2
    rows, cols = cfg.rows, cfg.cols
    state = np.zeros((rows + 2 * p, cols + 2 * p), dtype=np.int32)
    outs = []
    for fr in frames:
        M = state.copy()
        M[p:p + rows, p:p + cols] = corrected_indicator(cfg, fr)
        P = np.pad(M, p, mode="edge")
        S = np.zeros((P.shape[0] + 1, P.shape[1] + 1), dtype=np.int64)
        S[1:, 1:] = P.cumsum(0).cumsum(1)
        cnt = S[k:, k:] - S[:-k, k:] - S[k:, :-k] + S[:-k, :-k]
        F = (cnt >= thr).astype(np.int32)
        outs.append(F[p:p + rows, p:p + cols].astype(np.uint8))
        state = F
    return np.stack(outs)


@pytest.mark.parametrize("k,border,noise", [(11, True, 1), (11, False, 3), (3, True, 2), (1, False, 2), (21, True, 1)])
def test_box_count_formulation_matches_literal_median(k, border, noise):
    cfg = SyntheticConfig(rows=160, cols=256)
    cfg.setup.view_box_side = abi.lm_rect(0, 0, 256, 64)
    cfg.setup.view_box_bottom = abi.lm_rect(0, 64, 256, 96)
    frames = bb_frames(cfg, 6, noise=noise, seed=k, border=border)
    r = O.bb_run(cfg.setup, abi.bb_params(median_filter_size=k, semantics=abi.LM_BB_FIRSTLAST_INTEGER), frames,
                 binary=True)
    assert np.array_equal(box_count_model(cfg, frames, k), r["binary"])


def test_as_executed_pass_is_image_independent():
    cfg = SyntheticConfig()
    frames = bb_frames(cfg, 4, seed=1)
    r = O.bb_run(cfg.setup, abi.bb_params(), frames)
    per = r["frames"]
    assert np.all(per["x"] == -1) and np.all(per["y_side"] == -1)
    assert np.all(per["y_bottom"] == -1 + cfg.setup.view_box_bottom.y)
    assert np.all(per["width"] == 0)
    assert r["bb_side_mouse"] == (0, 0, 0, 0)
    assert np.all(r["x_pos"] == 0xFFFFFFFF)
    r0 = O.bb_run(cfg.setup, abi.bb_params(min_pixel_visible=0), frames)
    assert np.all(r0["frames"]["x"] == cfg.cols - 1)
    assert r0["bb_bottom_mouse"] == (0, 0, cfg.cols - 1, cfg.rows - cfg.setup.view_box_bottom.y - 1)


def test_integer_semantics_tracks_the_mouse():
    cfg = SyntheticConfig()
    frames = bb_frames(cfg, 8, seed=2)
    r = O.bb_run(cfg.setup, abi.bb_params(semantics=abi.LM_BB_FIRSTLAST_INTEGER), frames)
    per = r["frames"]
    assert np.all(per["width"] > 100) and np.all(per["width"] < cfg.cols // 2)
    assert np.all(per["height_side"] > 10)
    w, hs, hb = r["bb_side_mouse"][2], r["bb_side_mouse"][3], r["bb_bottom_mouse"][3]
    assert 100 < w <= per["width"].max() and 10 < hs <= per["height_side"].max() and 10 < hb


def np_imadjust_default_lut(hist):
    """numpy float32 model of imadjust_default (LocoMouse_class.cpp:3244-3311)."""
    f32 = np.float32
    total = f32(float(np.sum(hist.astype(np.float64))))
    cum, idx0, idx1, imin, imax, cmin, cmax = f32(0), 0, 0, 0, 0, True, True
    for i in range(256):
        cum = f32(cum + f32(hist[i]))
        cn = f32(cum / total)
        if cn > f32(0.01) and cmin:
            idx0 = imin = i
            cmin = False
        if cn >= f32(0.99) and cmax:
            idx1 = imax = i
            cmax = False
        if not (cmin or cmax):
            break
    if imin == imax:
        idx1 = 256
    r0, r1 = f32(f32(idx0) / f32(255)), f32(f32(idx1) / f32(255))
    d = float(f32(r1 - r0))
    alpha, beta = 1.0 * (1.0 / d), -float(r0) * (1.0 / d)
    if abs(alpha - 1) < np.finfo(np.float64).eps and abs(beta) < np.finfo(np.float64).eps:
        return np.arange(256, dtype=np.uint8)
    v = np.arange(256, dtype=np.float32) * f32(alpha) + f32(beta)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def test_imadjust_default_lut_restatement():
    rng = np.random.default_rng(21)
    for t in range(40):
        h = np.zeros(256, dtype=np.uint32)
        if t % 4 == 0:
            h[rng.integers(0, 256)] = 5000  # single value: imin == imax
        else:
            lo, hi = sorted(rng.integers(0, 256, size=2))
            h[lo:hi + 1] = rng.integers(0, 300, size=hi - lo + 1)
            h[rng.integers(0, 256, size=5)] += rng.integers(0, 50, size=5).astype(np.uint32)
        if h.sum() == 0:
            h[0] = 1
        assert np.array_equal(O.imadjust_default_lut(h), np_imadjust_default_lut(h)), t


def test_tm_as_executed_sums_never_reach_float_threshold():
    """Premise of the method-1 restatement: CV_32S sums in [0, 255*rows] read as
    floats pass firstLastOverT iff min_pixel_visible <= 0."""
    rng = np.random.default_rng(4)
    for rows in (96, 512, 4096):
        v = rng.integers(0, 255 * rows + 1, size=1024).astype(np.int32)
        v[rng.random(1024) < 0.3] = 0
        for th in (0, 1, 7, 255):
            assert O.first_last(v, th) == O.first_last(np.zeros(1024, np.int32), th)


def de_config():
    """1024 x 320 frames with a 160-row side view: computeMouseBox_DE's
    hard-coded rows [100, 149) lie inside it."""
    cfg = SyntheticConfig(rows=320, cols=1024, method=2)
    cfg.setup.view_box_side = abi.lm_rect(0, 0, 1024, 160)
    cfg.setup.view_box_bottom = abi.lm_rect(0, 160, 1024, 160)
    return cfg


def test_tm_de_pass_tracks_the_side_view_body():
    cfg = de_config()
    frames = bb_frames(cfg, 6, seed=3, side_h=250)
    r = O.bb_run(cfg.setup, abi.bb_params(), frames)
    x = r["frames"]["x"]
    assert np.all(x > 400) and np.all(x <= 1023)
    assert np.all(r["y_bottom_pos"] == 319) and np.all(r["y_side_pos"] == 159)
    assert r["bb_side_mouse"] == (0, 0, 400, 160) and r["bb_bottom_mouse"] == (0, 0, 400, 160)


def test_tm_pass_as_executed_is_constant():
    cfg = de_config()
    cfg.setup.method = 1
    frames = bb_frames(cfg, 4, seed=3, side_h=250)
    r = O.bb_run(cfg.setup, abi.bb_params(), frames)
    assert np.all(r["frames"]["x"] == -1) and np.all(r["x_pos"] == 0xFFFFFFFF)
    assert np.all(r["y_side_pos"] == 164) and r["bb_side_mouse"] == (0, 0, 400, 150)
    r0 = O.bb_run(cfg.setup, abi.bb_params(min_pixel_visible=0), frames)
    assert np.all(r0["frames"]["x"] == 1023)
    with pytest.raises(O.OracleError):
        O.bb_run(cfg.setup, abi.bb_params(semantics=abi.LM_BB_FIRSTLAST_INTEGER), frames)
