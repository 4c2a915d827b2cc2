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


# ---------------------------------------------------- multi-GPU shards (§8(e))

def test_device_list_refusals():
    """LocoMouse_Inputs::devices: a device listed twice is refused unless
    oversubscribe is set, and a negative index is refused -- both by the
    constructor, before any device is touched (runs without a GPU)."""
    cfg = S.SyntheticConfig()
    with pytest.raises(H.HostError, match="listed twice") as e:
        H.run_video(cfg, cfg.frames(0, 2), devices=[0, 1, 0])
    assert e.value.code == 1
    with pytest.raises(H.HostError, match="invalid device index") as e:
        H.run_video(cfg, cfg.frames(0, 2), devices=[0, -1])
    assert e.value.code == 1


@pytest.mark.parametrize("n,batch,ndev", [(3, 8, 4), (23, 5, 4), (20, 5, 4), (9, 1, 3)])
def test_shard_plan_equals_unsharded_oracle(n, batch, ndev):
    """The multi-device plan of the host mirror -- batch k of `batch` frames
    on device k mod ndev, every batch but the first run with its predecessor
    frame as a 1-frame halo -- gives the unsharded results, on the oracle
    (CPU): fewer batches than devices, a ragged last batch, one-frame shards."""
    import numpy as np
    from locomouse_cpp_amd.results import concat_results, slice_results
    from oracle import oracle as O
    from test_gpu_parity import assert_same
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, n)
    ref = O.OracleRun(cfg, frames).result
    per_dev = {}
    parts = []
    for k, a in enumerate(range(0, n, batch)):
        b = min(n, a + batch)
        per_dev.setdefault(k % ndev, []).append(a)
        if a == 0:
            parts.append(O.OracleRun(cfg, frames[a:b]).result)
        else:
            parts.append(slice_results(O.OracleRun(cfg, frames[a - 1:b]).result, 1))
    assert sum(len(v) for v in per_dev.values()) == (n + batch - 1) // batch
    assert_same(concat_results(parts), ref, f"plan n{n} b{batch} d{ndev}: ")
    assert np.array_equal(concat_results(parts)["tail"], ref["tail"])


@pytest.mark.gpu
@pytest.mark.parametrize("n,batch,order", [(23, 5, 0), (23, 5, 1 | 8), (3, 8, 0), (40, 7, 8)])
def test_main_loop_on_four_devices_matches_oracle(n, batch, order):
    """LocoMouse_Inputs::devices = four entries of the one GPU (oversubscribe):
    shards of `batch` frames dealt to four device threads, each shard with its
    halo frame, results appended in frame order -- every container equals the
    oracle's (incl. mid-batch reads, the read-ahead reader, and fewer shards
    than devices)."""
    from oracle import oracle as O
    from test_gpu_parity import assert_same
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, n)
    got = H.run_video(cfg, frames, batch=batch, call_order=order, devices=[0, 0, 0, 0], oversubscribe=True)
    assert_same(got, O.OracleRun(cfg, frames).result, f"host 4 devices n{n} b{batch} o{order}: ")


@pytest.mark.gpu
def test_tracks_on_four_devices_match_single_device():
    """main.cpp's post-loop stage on the four-device containers: the tracks
    equal those of the one-device run."""
    import numpy as np
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, 30)
    r1, t1, _ = H.run_video_tracks(cfg, frames, batch=8)
    r4, t4, _ = H.run_video_tracks(cfg, frames, batch=4, devices=[0, 0, 0, 0], oversubscribe=True)
    for k in t1:
        assert np.array_equal(t1[k], t4[k]), k
