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


def test_whole_video_bb_pass_is_reported_not_on_path():
    cfg = S.SyntheticConfig()
    cfg.params.use_provided_bounding_box = 0
    with pytest.raises(H.HostError, match="computeBoundingBox") as e:
        H.run_video(cfg, cfg.frames(0, 2))
    assert e.value.code == 2  # std::runtime_error, caught by main.cpp:98-101


@pytest.mark.gpu
@pytest.mark.parametrize("batch,order", [(8, 0), (5, 1), (64, 0)])
def test_main_loop_matches_oracle(batch, order):
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
