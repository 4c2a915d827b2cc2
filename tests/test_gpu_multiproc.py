"""The frame-sharded multi-GPU path (locomouse_cpp_amd/shard.py) with REAL HIP
contexts: two processes over gloo (world size 2), both ranks on GPU 0 here
(the driver's 8-GPU run gives each rank its own GPU), each running its shard
through lm_detect_batch with a one-frame halo; rank 0 gathers the compact
results in frame order.  Must equal the oracle's unsharded run bit for bit."""
import os
import socket

import numpy as np
import pytest

from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.results import KEYS

pytestmark = pytest.mark.gpu

N_FRAMES = 21


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path, batch):
    import torch.distributed as dist

    from locomouse_cpp_amd.runtime import Context
    from locomouse_cpp_amd.shard import run_sharded

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, N_FRAMES)
    ctx = Context(cfg, max_batch=batch, device=0)
    res = run_sharded(lambda fr, first, prev: ctx.detect(fr, first, prev_frame=prev), frames, N_FRAMES, batch=batch)
    ctx.close()
    if rank == 0:
        np.savez(out_path, **{k: res[k] for k in KEYS}, n_frames=res["n_frames"])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("batch", [4, 16])
def test_world2_hip_shards_match_oracle(tmp_path, batch):
    import torch.multiprocessing as mp

    from oracle import oracle as O
    from test_gpu_parity import assert_same
    out = str(tmp_path / "r0.npz")
    mp.spawn(_worker, args=(2, _free_port(), out, batch), nprocs=2, join=True)
    cfg = S.SyntheticConfig()
    ref = O.OracleRun(cfg, cfg.frames(0, N_FRAMES)).result
    z = np.load(out)
    assert int(z["n_frames"]) == N_FRAMES
    got = {k: z[k] for k in KEYS}
    got["n_frames"] = N_FRAMES
    assert_same(got, ref, f"world2 b{batch}: ")


@pytest.mark.parametrize("ranks,lanes", [(2, 1), (3, 4)])
def test_bench_video_mode_shards_whole_video(ranks, lanes):
    """BASELINE config 4's shape through bench.py itself: one video split into
    contiguous shards over `ranks` processes (spawned by bench.py --gpus,
    oversubscribed on this box's one GPU), several contexts per rank, batches
    with a 1-frame halo at every shard start; rank 0 gathers every frame and
    checks all of them against the oracle (video_check)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(ranks), "--oversubscribe",
                        "--video-frames", "700", "--batch", "64", "--streams", "2", "--lanes", str(lanes),
                        "--steps", "1", "--warmup", "1", "--no-cpu"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == ranks and line["scaling"] == "strong"
    assert line["gathered"]["frames"] == 700 and line["gathered"]["whole_and_disjoint"]
    assert line["video_check"]["frames"] == 700 and line["video_check"]["bit_exact"], line["video_check"]


@pytest.mark.timeout(600)
def test_bench_c4_eight_ranks_full_shape():
    """BASELINE config 4 at its own shape and bench.py's default shape for it:
    a 10,000-frame video as 8 contiguous 1,250-frame shards, one bench.py rank
    each (spawned by bench.py --gpus 8, oversubscribed on this box's one GPU; the driver's
    node gives each rank its own GPU), every shard but the first with its
    predecessor frame as the halo.  Rank 0 gathers all 10,000 frames, checks
    them whole and disjoint, and compares every one with the oracle."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "8", "--oversubscribe",
                        "--video-frames", "10000", "--steps", "1", "--warmup", "2", "--no-cpu"], env=env,
                       capture_output=True, text=True,
                       timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 8 and line["scaling"] == "strong"
    assert line["config"]["shards"] == "8 x ceil(10000/8) frames"
    # the default shape for a 1,250-frame share (bench.resolve_shape): one
    # context x 4 lanes, 6 batches of <= 209 frames
    assert (line["config"]["contexts_per_gpu"], line["config"]["lanes_per_context"]) == (1, 4)
    assert line["config"]["batch_frames"] == 209 and line["config"]["batches"] == [6]
    assert line["gathered"]["frames"] == 10000 and line["gathered"]["whole_and_disjoint"]
    assert line["video_check"]["frames"] == 10000 and line["video_check"]["bit_exact"], line["video_check"]
