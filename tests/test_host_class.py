"""The host C++ LocoMouse mirror (locomouse_cpp_amd/host) driven in
main.cpp's call order (tests/cpp/host_harness.cpp): its result containers
must equal the oracle's on the same frames, and it must raise the reference's
exception types."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import host_harness as H  # noqa: E402
from locomouse_cpp_amd import synthetic as S  # noqa: E402


def test_container_semantics():
    """P22D slot-0 rule and CV_Assert(S >= 0), MATSPARSE CSC layout and its
    always-zero get() (MyMat.cpp:371-374), compareCandidate."""
    H.selftest()


def test_whole_video_bb_pass_needs_a_rewindable_reader_and_method_0():
    cfg = S.SyntheticConfig()
    cfg.params.use_provided_bounding_box = 0
    with pytest.raises(H.HostError, match="rewind") as e:
        H.run_video(cfg, cfg.frames(0, 2))  # no bb_params -> no rewind callback
    assert e.value.code == 1
    cfg = S.SyntheticConfig(method=2)
    cfg.params.use_provided_bounding_box = 0
    with pytest.raises(H.HostError, match="rewind") as e:
        H.run_video(cfg, cfg.frames(0, 2))
    assert e.value.code == 1


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [5, 16])
def test_computed_bounding_box_then_main_loop_matches_oracle(batch):
    """use_provided_bounding_box = 0: getBoundingBox -> computeBoundingBox
    (lm_bb_*), rewind, then the per-frame loop on the computed boxes; against
    oracle.bb_run followed by the oracle loop on the same boxes."""
    import numpy as np
    from locomouse_cpp_amd import abi
    from oracle import oracle as O
    from test_gpu_parity import assert_same
    from bb_scenes import bb_frames
    cfg = S.SyntheticConfig()
    cfg.params.use_provided_bounding_box = 0
    frames = bb_frames(cfg, 12, seed=4)
    bbp = abi.bb_params(semantics=abi.LM_BB_FIRSTLAST_INTEGER)
    got, corners, sizes = H.run_video(cfg, frames, batch=batch, bb_params=bbp, with_bb=True)
    r = O.bb_run(cfg.setup, bbp, frames)
    ref_corners = np.stack([r["x_pos"], r["y_bottom_pos"], r["y_side_pos"]], 1)
    assert np.array_equal(corners, ref_corners)
    assert sizes == (r["bb_side_mouse"], r["bb_bottom_mouse"])
    cfg2 = S.SyntheticConfig(bounding_boxes={"side": r["bb_side_mouse"], "bottom": r["bb_bottom_mouse"]})
    assert_same(got, O.OracleRun(cfg2, frames, bb=ref_corners.astype(np.int32)).result, f"host bb b{batch}: ")


@pytest.mark.gpu
@pytest.mark.parametrize("batch,order", [(8, 0), (5, 1), (64, 0), (8, 8), (5, 1 | 8), (7, 1 | 8)])
def test_main_loop_matches_oracle(batch, order):
    """order bit 0: a result accessor called mid-batch (the batch is handed
    over early); bit 3: frames come from the batch reader read_frames, which
    reads a whole batch ahead — the read-ahead frames must survive an early
    hand-over."""
    from oracle import oracle as O
    from test_gpu_parity import assert_same
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, 20)
    got = H.run_video(cfg, frames, batch=batch, call_order=order)
    assert_same(got, O.OracleRun(cfg, frames).result, f"host b{batch}: ")


@pytest.mark.gpu
@pytest.mark.parametrize("method", [1, 2])
def test_factory_tm_methods(method):
    from oracle import oracle as O
    from test_gpu_parity import assert_same
    cfg = S.SyntheticConfig(method=method)
    frames = cfg.frames(10, 9)
    assert_same(H.run_video(cfg, frames, batch=4), O.OracleRun(cfg, frames).result, f"host TM{method}: ")


@pytest.mark.gpu
def test_read_past_end_of_video_raises_runtime_error():
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, 3)
    with pytest.raises(H.HostError, match="Failed to read image") as e:
        H.run_video(cfg, frames, n_frames=5)
    assert e.value.code == 2


@pytest.mark.gpu
def test_tm_de_computed_bounding_box_then_main_loop_matches_oracle():
    """LocoMouse_TM_DE with use_provided_bounding_box = 0 (method 2 pass)."""
    import numpy as np
    from locomouse_cpp_amd import abi
    from oracle import oracle as O
    from test_gpu_parity import assert_same
    from bb_scenes import bb_frames
    from test_bbox_oracle import de_config
    cfg = de_config()
    cfg.params.use_provided_bounding_box = 0
    frames = bb_frames(cfg, 10, seed=8, side_h=250)
    bbp = abi.bb_params()
    got, corners, sizes = H.run_video(cfg, frames, batch=4, bb_params=bbp, with_bb=True)
    r = O.bb_run(cfg.setup, bbp, frames)
    ref_corners = np.stack([r["x_pos"], r["y_bottom_pos"], r["y_side_pos"]], 1)
    assert np.array_equal(corners, ref_corners)
    assert sizes == (r["bb_side_mouse"], r["bb_bottom_mouse"])
    cfg2 = de_config()
    cfg2.params.bounding_box_side = abi.lm_rect(*r["bb_side_mouse"])
    cfg2.params.bounding_box_bottom = abi.lm_rect(*r["bb_bottom_mouse"])
    assert_same(got, O.OracleRun(cfg2, frames, bb=ref_corners.astype(np.int32)).result, "host TM_DE bb: ")
