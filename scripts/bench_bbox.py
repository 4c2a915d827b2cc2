"""Throughput of the whole-video bounding-box pass (lm_bb_push_device) on one
MI355X, plus the oracle's CPU rate on a bounded sample.

Frames are synthetic (include/lm_synth.h) and resident in HBM before timing;
one push = one batch of B frames through k_minmax_lut, k_bb_ingest,
k_bb_ring, k_bb_center, k_bb_cc plus the host's per-frame values."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=["c3", "c5"], default="c3")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--semantics", type=int, default=0)
    ap.add_argument("--cpu-frames", type=int, default=40)
    args = ap.parse_args()
    import torch
    from locomouse_cpp_amd import abi
    from locomouse_cpp_amd.runtime import BBContext, synth_frames_device
    from locomouse_cpp_amd.synthetic import SyntheticConfig
    rows, cols = (256, 1024) if args.config == "c3" else (512, 1920)
    cfg = SyntheticConfig(rows=rows, cols=cols)
    params = abi.bb_params(semantics=args.semantics)
    B = args.batch
    pitch = rows * cols
    nbuf = 4
    d = torch.empty(nbuf * B * pitch, dtype=torch.uint8, device="cuda:0")
    synth_frames_device(d.data_ptr(), rows, cols, 0, nbuf * B, pitch)
    ctx = BBContext(cfg.setup, params, max_batch=B)
    for i in range(args.warmup):
        ctx.push_device(d.data_ptr() + (i % nbuf) * B * pitch, pitch, B, values=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ctx.push_device(d.data_ptr() + (i % nbuf) * B * pitch, pitch, B, values=False)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    fps = args.steps * B / dt
    # CPU baseline: the oracle restatement, single thread, on a bounded sample
    from oracle import oracle as O
    fr = cfg.frames(0, args.cpu_frames)
    t1 = time.perf_counter()
    O.bb_run(cfg.setup, params, fr)
    cpu = args.cpu_frames / (time.perf_counter() - t1)
    print(json.dumps({"metric": "bb_pass_frames_per_s", "value": fps, "unit": "frames/s", "config": args.config,
                      "batch": B, "steps": args.steps, "ms_per_batch": 1e3 * dt / args.steps,
                      "cpu_baseline": {"value": cpu, "unit": "frames/s", "cores": 1, "kind": "port",
                                       "sample": f"{args.cpu_frames} frames"}}))
    ctx.close()


if __name__ == "__main__":
    main()
