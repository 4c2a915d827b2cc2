"""Frame-sharded path (locomouse_cpp_amd/shard.py) with world size 2 over
gloo on CPU: shards + one-frame halo must reproduce the unsharded run
exactly.  The per-shard detector is the oracle (the GPU variant of the same
logic is bench.py --gpus N and tests/test_gpu_parity.py::test_shard_with_halo_frame)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.results import KEYS, concat_results, slice_results
from locomouse_cpp_amd.shard import detect_range, shard_range

N_FRAMES = 11


def _same(a, b):
    for k in KEYS:
        x, y = a[k], b[k]
        if x.dtype.names:
            assert x.shape == y.shape and all(np.array_equal(x[n], y[n]) for n in x.dtype.names), k
        else:
            assert np.array_equal(x, y), k


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    import torch.distributed as dist
    from locomouse_cpp_amd.shard import run_sharded
    from oracle_detect import OracleDetector

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, N_FRAMES)
    res = run_sharded(OracleDetector(cfg), frames, N_FRAMES, batch=4)
    if rank == 0:
        np.savez(out_path, **{k: res[k] for k in KEYS}, n_frames=res["n_frames"])
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers():
    for n in (0, 1, 7, 10, 10000):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_halo_and_batches_match_unsharded():
    from oracle import oracle as O
    from oracle_detect import OracleDetector
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, 9)
    ref = O.OracleRun(cfg, frames).result
    det = OracleDetector(cfg)
    got = concat_results([detect_range(det, frames, 0, 5, 2), detect_range(OracleDetector(cfg), frames, 5, 9, 3)])
    _same(got, ref)
    _same(slice_results(ref, 4), slice_results(got, 4))


def test_gloo_world2(tmp_path):
    from oracle import oracle as O
    out = str(tmp_path / "r0.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    cfg = S.SyntheticConfig()
    ref = O.OracleRun(cfg, cfg.frames(0, N_FRAMES)).result
    z = np.load(out)
    got = {k: z[k] for k in KEYS}
    assert int(z["n_frames"]) == N_FRAMES
    _same(got, ref)
