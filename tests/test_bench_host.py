"""Host logic of bench.py without a GPU: the launcher's rank checks, the
video-shard split of the strong-scaling mode, its gather check, and the
oracle checker the bench runs on the timed batches (fed here with oracle
results, so a correct result passes and a perturbed one fails)."""
import os
import subprocess
import sys

import numpy as np
import pytest

import bench
from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.results import concat_results, head_results, same_results, slice_results

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env.update(env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env, capture_output=True,
                          text=True, timeout=timeout)


def test_world_size_must_match_gpus():
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "3", "RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=3 but --gpus 2" in p.stderr
    assert '"metric"' not in p.stdout


def test_spawned_ranks_fail_loudly_without_enough_gpus():
    # no GPU in this container: every spawned rank refuses, the launcher
    # returns non-zero and no JSON line is printed
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"], {})
    assert p.returncode != 0
    assert '"metric"' not in p.stdout
    assert "bench.py" in p.stderr


def test_video_shards_cover_the_video():
    for n, world, streams in ((10000, 8, 4), (10000, 1, 4), (11, 3, 2), (5, 4, 4)):
        pieces = [s for r in range(world) for s in bench.video_shards(n, world, r, streams)]
        pos = 0
        for lo, hi in pieces:
            assert lo == pos and hi > lo
            pos = hi
        assert pos == n
    # C4: 8 ranks x 1,250 frames
    assert bench.video_shards(10000, 8, 3, 1) == [(3750, 5000)]


def _oracle_video(cfg, n):
    from oracle import oracle as O
    return O.OracleRun(cfg, bench._scene_frames(cfg, range(n))).result


def test_head_and_slice_results_partition():
    cfg = S.SyntheticConfig()
    ref = _oracle_video(cfg, 7)
    for m in range(8):
        back = concat_results([head_results(ref, m), slice_results(ref, m)]) if 0 < m < 7 else ref
        assert same_results(back, ref)


def test_check_video_and_oracle_check():
    cfg = S.SyntheticConfig()
    n = 9
    ref = _oracle_video(cfg, n)
    pieces = [(0, head_results(ref, 4)), (4, slice_results(ref, 4))]
    parts = bench.check_video(list(reversed(pieces)), n)
    assert [p[0] for p in parts] == [0, 4]
    items = [(f, r, None if f == 0 else f - 1, list(range(f, f + r["n_frames"]))) for f, r in parts]
    chk = bench.oracle_check(cfg, items, threads=2, chunk=3)
    assert chk["bit_exact"] and chk["frames"] == n
    bad = dict(parts[1][1])
    bad["cand"] = bad["cand"].copy()
    bad["cand"]["score"][0] += 1e-9
    chk = bench.oracle_check(cfg, [items[0], (4, bad, 3, items[1][3])], threads=2, chunk=3)
    assert not chk["bit_exact"] and chk["mismatching"] == [4]
    with pytest.raises(RuntimeError):
        bench.check_video([pieces[0]], n)
    with pytest.raises(RuntimeError):
        bench.check_video([pieces[0], (3, pieces[1][1])], n)


def test_oracle_check_wrapped_stream_sample():
    # a bench stream wraps around its resident frames: the batch's halo is a
    # scene frame that does not precede its first frame
    cfg = S.SyntheticConfig()
    from oracle import oracle as O
    fr = bench._scene_frames(cfg, [40, 3, 4, 5])
    ref = slice_results(O.OracleRun(cfg, fr).result, 1)
    chk = bench.oracle_check(cfg, [("w", ref, 40, [3, 4, 5])], threads=1, chunk=2)
    assert chk["bit_exact"]


def test_executed_flops_counts_halo_slots():
    class G:
        class R:
            def __init__(self, w, h):
                self.width, self.height = w, h
        bb_bottom_mouse, bb_side_mouse, tail_box_width = R(400, 140), R(400, 90), 240

    class Ctx:
        cfg = S.SyntheticConfig()

        def geometry(self):
            return G

    w = Ctx.cfg.weights
    work = {"outputs": (0, 0)}
    tail = 2 * (140 * 240 * w["tail_bottom"].size + 90 * 240 * w["tail_side"].size)
    assert bench.executed_flops(Ctx(), work, 5) == 5 * tail
    assert bench.executed_flops(Ctx(), work, None) is None
    assert np.isclose(bench.executed_flops(Ctx(), {"outputs": (1, 0)}, 0),
                      2 * (w["paw_bottom"].size + w["snout_bottom"].size))


def test_default_shape_by_mode():
    """Unset --streams / --lanes / --batch: 8 contexts x 448 frames for the C3
    resident stream (profiles/r05/sweep/), by the rank's share for one C3
    video (profiles/r06/c4/), 4 x 1 x 256 for every other config and mode;
    explicit values are kept."""
    from types import SimpleNamespace

    def shape(**kw):
        a = dict(config="c3", video_frames=0, host_frames=False, lanes=None, precision="fp32", workload="detect",
                 streams=None, batch=None, gpus=1)
        a.update(kw)
        r = bench.resolve_shape(SimpleNamespace(**a))
        return r.streams, r.lanes, r.batch

    assert shape() == (8, 1, 448)
    assert shape(config="c5") == (4, 1, 256)
    assert shape(video_frames=10000) == (4, 2, 313)
    assert shape(video_frames=10000, gpus=8) == (1, 4, 209)  # a 1,250-frame shard: 6 batches
    assert shape(video_frames=1250) == (1, 4, 209)
    assert shape(video_frames=10000, config="c5") == (4, 1, 256)
    assert shape(host_frames=True) == (4, 1, 256)
    assert shape(lanes=4) == (4, 4, 256)
    assert shape(lanes=1) == (8, 1, 448)
    assert shape(precision="f16") == (4, 1, 256)
    assert shape(workload="bb") == (4, 1, 256)
    assert shape(streams=2, batch=100) == (2, 1, 100)
    assert shape(streams=2) == (2, 1, 448)
    assert shape(video_frames=10000, streams=8, batch=448) == (8, 2, 448)
