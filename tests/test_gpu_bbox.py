"""GPU parity of the whole-video bounding-box pass (lm_bb_*, SURVEY.md §8(f)
row 1) against the CPU restatement (oracle.bb_run) on the same frames.

Everything here is integer work, so the bar is bit-exact: the thresholded
median image of every frame, the six per-frame values of computeMouseBox,
the box sizes of computeMouseBoxSize and the moving-average corner tracks.
Parity against the reference itself is unpinned (OpenCV is absent; see
tests/test_bbox_oracle.py for how the oracle's pieces are pinned)."""
import numpy as np
import pytest

from locomouse_cpp_amd import abi
from locomouse_cpp_amd.synthetic import SyntheticConfig
from tests.bb_scenes import bb_frames

pytestmark = pytest.mark.gpu

AS_EXEC, INTEGER = abi.LM_BB_FIRSTLAST_AS_EXECUTED, abi.LM_BB_FIRSTLAST_INTEGER


def run_gpu(cfg, params, frames, batch, check_binary=None):
    from locomouse_cpp_amd.runtime import BBContext
    ctx = BBContext(cfg.setup, params, max_batch=batch)
    per, binary = [], []
    try:
        for s in range(0, len(frames), batch):
            chunk = frames[s:s + batch]
            per.append(ctx.push(chunk))
            if check_binary is not None:
                binary.extend(ctx.debug_binary(i) for i in range(len(chunk)))
        out = ctx.finish()
    finally:
        ctx.close()
    assert np.array_equal(np.concatenate(per), out["frames"])
    if check_binary is not None:
        out["binary"] = np.stack(binary)
    return out


def assert_bb_equal(got, ref):
    if "binary" in got:
        for f in range(len(ref["binary"])):
            if not np.array_equal(got["binary"][f], ref["binary"][f]):
                d = np.argwhere(got["binary"][f] != ref["binary"][f])
                raise AssertionError(f"binary image of frame {f} differs at {len(d)} pixels, first {d[:5].tolist()}")
    for name in ("x", "y_bottom", "y_side", "width", "height_bottom", "height_side"):
        a, b = got["frames"][name], ref["frames"][name]
        assert np.array_equal(a, b), f"{name}: first diff at frame {np.argmax(a != b)}: {a[np.argmax(a != b)]} vs {b[np.argmax(a != b)]}"
    for k in ("x_pos", "y_bottom_pos", "y_side_pos"):
        assert np.array_equal(got[k], ref[k]), k
    assert got["bb_side_mouse"] == ref["bb_side_mouse"]
    assert got["bb_bottom_mouse"] == ref["bb_bottom_mouse"]


def check(cfg, params, frames, batch=8):
    from oracle import oracle as O
    ref = O.bb_run(cfg.setup, params, frames, binary=True)
    got = run_gpu(cfg, params, frames, batch, check_binary=True)
    assert_bb_equal(got, ref)
    return got, ref


@pytest.mark.parametrize("semantics", [AS_EXEC, INTEGER])
@pytest.mark.parametrize("conn", [8, 4])
def test_bb_scene_bit_exact(semantics, conn):
    cfg = SyntheticConfig()
    frames = bb_frames(cfg, 20, seed=conn, border=True, noise=1)
    got, _ = check(cfg, abi.bb_params(connectivity=conn, semantics=semantics), frames, batch=8)
    if semantics == INTEGER:
        assert got["frames"]["width"].max() > 100


@pytest.mark.parametrize("k", [1, 3, 5, 15, 17, 21])
def test_bb_median_sizes(k):
    cfg = SyntheticConfig()
    frames = bb_frames(cfg, 9, seed=k, border=True, noise=2)
    check(cfg, abi.bb_params(median_filter_size=k, semantics=INTEGER), frames, batch=4)


def test_bb_default_synthetic_video_and_flip():
    cfg = SyntheticConfig(flip=True)
    frames = cfg.frames(0, 10)
    check(cfg, abi.bb_params(semantics=INTEGER), frames, batch=10)
    check(cfg, abi.bb_params(min_pixel_visible=0), frames, batch=3)


def test_bb_empty_frames_and_equal_area_ties():
    cfg = SyntheticConfig()
    frames = bb_frames(cfg, 12, seed=5, empty_every=4, ties=True, noise=0)
    for conn in (8, 4):
        check(cfg, abi.bb_params(connectivity=conn, semantics=INTEGER, min_pixel_visible=255 * 3), frames, batch=5)


def test_bb_window_and_single_frame_edge_cases():
    cfg = SyntheticConfig()
    frames = bb_frames(cfg, 7, seed=9)
    for w in (1, 3, 7, 9):
        check(cfg, abi.bb_params(moving_average_window=w, semantics=INTEGER), frames, batch=7)
    check(cfg, abi.bb_params(semantics=INTEGER), frames[:1], batch=1)


def test_bb_highres_geometry():
    cfg = SyntheticConfig(rows=512, cols=1920)
    frames = bb_frames(cfg, 4, seed=11, border=True)
    check(cfg, abi.bb_params(semantics=INTEGER), frames, batch=2)


def test_bb_long_video_device_frames():
    """256 frames pushed from device memory in batches of 64 (ring carried
    across pushes), checked against the oracle on the per-frame values."""
    import torch
    from locomouse_cpp_amd.runtime import BBContext
    from oracle import oracle as O
    cfg = SyntheticConfig()
    frames = bb_frames(cfg, 256, seed=13, border=True)
    params = abi.bb_params(semantics=INTEGER)
    ref = O.bb_run(cfg.setup, params, frames)
    d = torch.from_numpy(frames).to("cuda:0")
    ctx = BBContext(cfg.setup, params, max_batch=64)
    try:
        pitch = frames.shape[1] * frames.shape[2]
        for s in range(0, 256, 64):
            ctx.push_device(d.data_ptr() + s * pitch, pitch, 64, values=False)
        got = ctx.finish()
    finally:
        ctx.close()
    assert_bb_equal(got, ref)


def test_bb_argument_errors():
    from locomouse_cpp_amd.runtime import BBContext, LMError
    cfg = SyntheticConfig()
    for bad in (abi.bb_params(median_filter_size=4), abi.bb_params(min_pixel_visible=-1),
                abi.bb_params(moving_average_window=2), abi.bb_params(connectivity=6),
                abi.bb_params(semantics=7)):
        with pytest.raises(LMError) as e:
            BBContext(cfg.setup, bad)
        assert e.value.code == abi.LM_ERR_INVALID_ARGUMENT
    cfg.setup.method = 1
    with pytest.raises(LMError):
        BBContext(cfg.setup, abi.bb_params())
    cfg.setup.method = 0
    ctx = BBContext(cfg.setup, abi.bb_params(), max_batch=2)
    with pytest.raises(LMError):
        ctx.finish()  # no frame pushed
    with pytest.raises(LMError):
        ctx.push(cfg.frames(0, 3))  # n > max_batch
    ctx.close()


@pytest.mark.parametrize("k,conn,density", [(1, 8, 0.5), (1, 4, 0.3), (3, 4, 0.5)])
def test_bb_many_runs_global_fallback(k, conn, density):
    """Salt-and-pepper masks: with k = 1 a view holds tens of thousands of
    row runs, more than the LDS run table (LM_BB_RUN_CAP), so its run table
    lives in global memory; k = 3 smooths them back under the cap."""
    cfg = SyntheticConfig()
    rng = np.random.default_rng(int(density * 100) + k)
    frames = np.clip(cfg.background.astype(np.int32)[None] +
                     (rng.random((3, cfg.rows, cfg.cols)) < density) * 100, 0, 255).astype(np.uint8)
    check(cfg, abi.bb_params(median_filter_size=k, connectivity=conn, semantics=INTEGER), frames, batch=3)


@pytest.mark.parametrize("flip", [False, True])
def test_bb_tm_de_bit_exact(flip):
    """LocoMouse_TM_DE's pass (method 2): imadjust_default + fixed bands per frame."""
    from tests.test_bbox_oracle import de_config
    cfg = de_config()
    cfg.setup.flip = 1 if flip else 0
    frames = bb_frames(cfg, 24, seed=31, side_h=250, empty_every=7)
    for w in (5, 1):
        from oracle import oracle as O
        params = abi.bb_params(moving_average_window=w)
        ref = O.bb_run(cfg.setup, params, frames)
        assert_bb_equal(run_gpu(cfg, params, frames, batch=10), ref)


def test_bb_tm_as_executed():
    from oracle import oracle as O
    from locomouse_cpp_amd.runtime import BBContext, LMError
    from tests.test_bbox_oracle import de_config
    cfg = de_config()
    cfg.setup.method = 1
    frames = bb_frames(cfg, 9, seed=5, side_h=250)
    for mpv in (1, 0):
        params = abi.bb_params(min_pixel_visible=mpv, bb_width=380, bb_height_side=140)
        assert_bb_equal(run_gpu(cfg, params, frames, batch=4), O.bb_run(cfg.setup, params, frames))
    with pytest.raises(LMError):
        BBContext(cfg.setup, abi.bb_params(semantics=INTEGER))


def test_bb_unaligned_device_frames():
    """Device frames at an odd address / pitch are staged before the kernels."""
    import torch
    from locomouse_cpp_amd.runtime import BBContext
    from oracle import oracle as O
    cfg = SyntheticConfig()
    frames = bb_frames(cfg, 6, seed=23)
    npix = frames.shape[1] * frames.shape[2]
    pitch = npix + 7
    buf = torch.zeros(5 + pitch * 6, dtype=torch.uint8, device="cuda:0")
    for i in range(6):
        buf[5 + i * pitch: 5 + i * pitch + npix] = torch.from_numpy(frames[i].reshape(-1)).cuda()
    torch.cuda.synchronize()
    params = abi.bb_params(semantics=INTEGER)
    ctx = BBContext(cfg.setup, params, max_batch=6)
    try:
        ctx.push_device(buf.data_ptr() + 5, pitch, 6, values=False)
        got = ctx.finish()
    finally:
        ctx.close()
    assert_bb_equal(got, O.bb_run(cfg.setup, params, frames))
