"""Benchmark of the MI355X LocoMouse per-frame detection path.

`python bench.py --gpus N --steps K --warmup W` — one process per GPU (the
driver launches N>1 with torch.distributed.run).  A "step" is one batch of B
consecutive synthetic 1024x256 frames (already resident in HBM) through the
whole per-frame path — ingest, the six detectors, tail, NMS, unary/pairwise
costs, side<->bottom matching — up to and including the copy of the results
into host memory in the reference's container layout.  Frames are sharded
across ranks as independent streams (no collective on the data path):
scaling "weak".  Rank 0 prints one JSON line.
"""
import argparse
import json
import math
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "frames/sec whole-node + achieved HBM GB/s; 1024×256 gray, 6 templates"
CONFIGS = {  # BASELINE.json configs with a GPU bench line: (rows, cols, description)
    "c3": (256, 1024, "C3: 1024x256 u8 synthetic stream, 6 detectors (paw/snout/tail x bottom/side), "
                      "full per-frame path incl. D2H of results"),
    "c5": (512, 1920, "C5: 1920x512 u8 synthetic stream, geometry and detectors x2 (fp32, bit-exact mode), "
                      "full per-frame path incl. D2H of results"),
}
FP32_PEAK_TFLOPS = 157.3   # MI355X FP32 vector (= f32 MFMA) peak, MI355X_MICROARCH.md
F16_PEAK_TFLOPS = 2500.0   # MI355X dense f16 MFMA peak (MI355X_MICROARCH.md: ~2.5 PF dense)
HBM_PEAK_GBS = 8000.0
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r03", "pmc_k_corr.json")  # this tree's PMC passes (scripts/gpu_final.sh)


def algorithmic_flops_per_frame(ctx):
    """2 * sum over the six detectors of consumed outputs x taps (SURVEY.md
    §8(d)): 294,758,400 FLOP per frame at the 1024x256 config."""
    g = ctx.geometry()
    w = ctx.cfg.weights
    hb, wb, hs, ws, tw = (g.bb_bottom_mouse.height, g.bb_bottom_mouse.width, g.bb_side_mouse.height,
                          g.bb_side_mouse.width, g.tail_box_width)
    outs = {"paw_bottom": hb * wb, "snout_bottom": hb * wb, "tail_bottom": hb * tw,
            "paw_side": hs * ws, "snout_side": hs * ws, "tail_side": hs * tw}
    return 2 * sum(outs[k] * w[k].size for k in outs)


def executed_flops(ctx, work, n):
    """FLOP the correlation executed for a batch of n frames: the tail
    detectors over every output, the point detectors over the outputs of their
    bright tiles only (`work` = Context.corr_work(): dark tiles -- no mouse
    pixel > 25, all scores zeroed by the reference's mask -- are skipped).
    None when the batch's work was not recorded."""
    if work is None:
        return None
    g = ctx.geometry()
    w = ctx.cfg.weights
    tw = g.tail_box_width
    hb, hs = g.bb_bottom_mouse.height, g.bb_side_mouse.height
    ob, os_ = work["outputs"]
    return 2 * (ob * (w["paw_bottom"].size + w["snout_bottom"].size) + os_ * (w["paw_side"].size + w["snout_side"].size)
                + n * (hb * tw * w["tail_bottom"].size + hs * tw * w["tail_side"].size))


def union_ms(iv):
    """Length of the union of [t0, t1] intervals (ms)."""
    tot, end = 0.0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            tot += b - a
            end = b
        elif b > end:
            tot += b - end
            end = b
    return tot


def cpu_baseline(cfg, seconds=10.0, max_frames=2000, samples=()):
    """The oracle (CPU restatement, 1 thread, AVX2+FMA) on a bounded sample of
    the same workload.  It first runs the frames of the GPU result samples
    (`samples`: (first frame, GPU result dict, scene indices of its previous
    and first frame) per stream; the previous frame is the oracle's frame 0) and compares its outputs with the
    GPU's bit for bit -- the oracle as the checker of the benchmarked run --
    then chunks of 50 consecutive synthetic frames until `seconds` of CPU
    work.  Returns (baseline line, parity-sample line)."""
    from oracle import oracle as O
    from locomouse_cpp_amd.results import same_results, slice_results
    chunk = 50
    done, t = 0, 0.0
    checked, exact, mism = 0, True, []
    import numpy as np
    for first, got, prev_scene, first_scene in samples:
        fr = np.concatenate([cfg.frames(prev_scene, 1), cfg.frames(first_scene, got["n_frames"])])
        t0 = time.perf_counter()
        ref = O.OracleRun(cfg, fr).result
        t += time.perf_counter() - t0
        done += got["n_frames"] + 1
        ok = same_results(got, slice_results(ref, 1))
        exact &= ok
        checked += got["n_frames"]
        if not ok:
            mism.append(int(first))
    frames = cfg.frames(0, chunk)
    while t < seconds and done < max_frames:
        t0 = time.perf_counter()
        O.OracleRun(cfg, frames)
        t += time.perf_counter() - t0
        done += chunk
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    line = {"value": done / t, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{done} frames (the GPU parity samples, then chunks of {chunk} from frame 0), "
                      f"oracle/lm_oracle.cpp single thread, {t:.1f} s", "cpu": cpu}
    parity = None
    if samples:
        parity = {"frames": checked, "streams": len(samples), "bit_exact": bool(exact),
                  "first_frames": [int(smp[0]) for smp in samples][:16], "mismatching_batches": mism,
                  "compared": "every lm_batch_result array (candidates, P22D, unary, pairwise CSC, tail) against "
                              "oracle/lm_oracle.cpp on the same synthetic frames"}
    return line, parity


def host_cpu_share():
    """Host threads this GPU's share of the node may use: the CPUs this
    process may run on, capped by the box's per-GPU share (OMP_NUM_THREADS,
    16 per MI355X on the pool: a 128-core node split over 8 GPUs)."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(share))) if share and share.isdigit() else n


def cpu_baseline_threads(cfg, seconds=8.0, threads=None, chunk=50):
    """The fair CPU baseline of SURVEY.md §8(d)(ii): the oracle on `threads`
    host threads (default: this GPU's CPU share), each on its own contiguous
    chunk of frames (frame-sharded like the multi-GPU path; ctypes releases
    the GIL inside the oracle call)."""
    import threading
    from oracle import oracle as O
    if threads is None:
        threads = host_cpu_share()
    samples = [cfg.frames(chunk * t, chunk) for t in range(threads)]
    counts = [0] * threads
    stop = time.perf_counter() + seconds

    def work(t):
        while time.perf_counter() < stop:
            O.OracleRun(cfg, samples[t])
            counts[t] += chunk

    t0 = time.perf_counter()
    pool = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for th in pool:
        th.start()
    for th in pool:
        th.join()
    el = time.perf_counter() - t0
    return {"value": sum(counts) / el, "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"{sum(counts)} frames, {threads} threads x chunks of {chunk} frames, {el:.1f} s wall"}


def cpu_baseline_node(cfg, seconds=8.0):
    """BASELINE.md §2's `nproc`-thread line: one oracle thread per CPU this
    process may run on (the whole node where nothing restricts it), each on
    its own contiguous shard.  On a shared GPU box the per-GPU share
    (cpu_baseline_threads) is the fair per-GPU comparison; this line is the
    whole-node CPU figure to set beside an 8-GPU frames/s."""
    n = len(os.sched_getaffinity(0))
    line = cpu_baseline_threads(cfg, seconds, threads=n, chunk=8)
    line["nproc"] = os.cpu_count()
    return line


def gather_results(ctxs, frames, state, vbase, R, B, frame_bytes, world, rank):
    """The host gather of north_star's multi-GPU design, after the timed
    region: every stream of every rank runs its next batch, its compact
    results (the lm_batch_result arrays) go to rank 0 over the host process
    group, and rank 0 checks that the gathered frame ranges are whole and
    disjoint.  Returns (summary on rank 0 or None, this rank's
    (first frame, result dict, scene index of the previous frame, scene index
    of the first frame) per stream)."""
    import torch.distributed as dist

    from locomouse_cpp_amd.abi import result_to_numpy
    mine, local = [], []
    for k, c in enumerate(ctxs):
        f = state[k]["frame"]
        i = (f - vbase[k]) % R + 1
        n = min(B, R + 1 - i)
        # the context processed frame f - 1 last: it continues from that frame
        res = result_to_numpy(c.detect_device(frames[k].data_ptr() + i * frame_bytes, frame_bytes, n, f))
        # synthetic-scene indices of the pixels this batch saw: resident frame
        # i holds scene frame vbase - 1 + i, and the frame before it (the one
        # the context processed last) is resident frame i - 1, or frame R
        # when the stream wrapped around
        local.append((f, res, vbase[k] - 1 + (i - 1 if i > 1 else R), vbase[k] - 1 + i))
        mine.append({"first": f, "n": res["n_frames"], "want": n, "cand": res["cand"],
                     "cand_offset": res["cand_offset"], "tail": res["tail"]})
    allr = [None] * world if rank == 0 else None
    if world > 1:
        dist.gather_object(mine, allr, dst=0)
    else:
        allr = [mine]
    if rank != 0:
        return None, local
    parts = sorted((p for r in allr for p in r), key=lambda p: p["first"])
    for p in parts:
        if p["n"] != p["want"] or len(p["cand_offset"]) != 4 * p["n"] + 1 or p["tail"].shape[0] != p["n"]:
            raise RuntimeError(f"gathered batch at frame {p['first']} is not whole")
    for a, b in zip(parts, parts[1:]):
        if a["first"] + a["n"] > b["first"]:
            raise RuntimeError("gathered frame ranges overlap")
    return {"ranks": world, "streams": len(parts), "frames": int(sum(p["n"] for p in parts)),
            "candidates": int(sum(len(p["cand"]) for p in parts)),
            "first_frames": [int(p["first"]) for p in parts][:16], "whole_and_disjoint": True,
            "transport": "gloo gather_object (host)" if world > 1 else "local"}, local


def run_bb(args):
    """The whole-video bounding-box pass (lm_bb_push_device, method 0) on one
    GPU: frames resident in HBM, `--steps` pushes of `--batch` frames after
    `--warmup`; the CPU baseline is the oracle restatement on a bounded
    sample.  Prints one JSON line (not the headline metric)."""
    import time

    import torch

    from locomouse_cpp_amd import abi
    from locomouse_cpp_amd.runtime import BBContext, synth_frames_device
    from locomouse_cpp_amd.synthetic import SyntheticConfig
    rows, cols, workload = CONFIGS[args.config]
    cfg = SyntheticConfig(rows=rows, cols=cols)
    params = abi.bb_params(semantics=args.bb_semantics)
    B, pitch, nbuf = args.batch, rows * cols, 4
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
    ctx.close()
    line = {"metric": "whole-video bounding-box pass frames/s (method 0)", "value": args.steps * B / dt,
            "unit": "frames/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True, "scaling": "replicas",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (lm_synth.h scene, resident in HBM)",
            "config": {"workload": workload + "; LocoMouse::computeBoundingBox over the stream", "batch_frames": B,
                       "firstlast_semantics": "integer" if args.bb_semantics else "as executed"}}
    if not args.no_cpu:
        from oracle import oracle as O  # CPU baseline only
        nf = 40 if rows <= 256 else 10
        fr = cfg.frames(0, nf)
        t1 = time.perf_counter()
        O.bb_run(cfg.setup, params, fr)
        line["cpu_baseline"] = {"value": nf / (time.perf_counter() - t1), "unit": "frames/s", "cores": 1,
                                "kind": "port", "sample": f"{nf} frames, oracle/lm_oracle.cpp BBOracle, one thread"}
    print(json.dumps(line))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--precision", choices=["fp32", "f16"], default="fp32",
                    help="f16: the non-parity LM_CORR_F16 correlation (BASELINE config 5)")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--resident", type=int, default=6400, help="frames resident in HBM per stream (cycled)")
    ap.add_argument("--streams", type=int, default=4,
                    help="contexts per GPU (each with its own host thread)")
    ap.add_argument("--lanes", type=int, default=1,
                    help="pipeline lanes per context (lm_setup.pipeline_lanes: batches in flight on their own HIP "
                         "streams, driven with lm_detect_submit / lm_detect_collect)")
    ap.add_argument("--check-all-ranks", action="store_true",
                    help="every rank compares its gathered batches with the oracle (multi-rank rehearsals)")
    ap.add_argument("--round-robin", action="store_true", help="one host thread drives all streams in turn")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--workload", choices=["detect", "bb"], default="detect",
                    help="bb: the whole-video bounding-box pass (SURVEY.md §8(f) row 1) instead of the headline path")
    ap.add_argument("--bb-semantics", type=int, default=0, help="firstLastOverT: 0 as executed, 1 integer sums")
    args = ap.parse_args()
    if args.workload == "bb":
        return run_bb(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # One process per GPU.  The data path has no collective (frame shards are
    # independent), so the only inter-rank traffic -- the start/stop barrier
    # and the max-over-ranks of the elapsed time -- goes over gloo on the host.
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a GPU (no HIP device visible)")
    local = local % ndev  # ranks > devices only when rehearsing N>1 on a smaller box
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("gloo")

    from locomouse_cpp_amd import synthetic as S
    from locomouse_cpp_amd.runtime import Context, synth_frames_device

    B = args.batch
    NS = max(1, args.streams)
    # Frames resident per stream, cycled: a multiple of the batch and of the
    # scene's motion period (100 frames), so the wrap-around is a continuous
    # step of the video, not a jump.
    unit = B * 100 // math.gcd(B, 100)
    R = max(unit, args.resident // unit * unit)
    rows, cols, workload = CONFIGS[args.config]
    FRAME_BYTES = rows * cols
    cfg = S.SyntheticConfig(rows=rows, cols=cols)
    f16 = args.precision == "f16"
    if f16:  # non-parity mode (LM_CORR_F16): f16 weights, fp32 accumulation on the matrix cores
        cfg.setup.corr_precision = 1
        workload = workload.replace("(fp32, bit-exact mode)", "(LM_CORR_F16: f16 weights, fp32 accumulation, non-parity)")
        workload += "" if "LM_CORR_F16" in workload else " [LM_CORR_F16 non-parity correlation]"
    # NS contexts per GPU, each with its own HIP stream and host thread, each
    # on its own contiguous range of the video (rank-major): like a shard, its
    # first batch gets the previous frame as a 1-frame halo.
    NL = max(1, args.lanes)
    ctxs = [Context(cfg, max_batch=B, device=local, lanes=NL) for _ in range(NS)]
    frames = torch.empty((NS, R + 1, rows, cols), dtype=torch.uint8, device=f"cuda:{local}")
    vbase = [(rank * NS + k) * R for k in range(NS)]
    for k in range(NS):
        # index 0 holds frame vbase-1 (the halo), index i frame vbase+i-1
        synth_frames_device(frames[k].data_ptr(), rows, cols, vbase[k] - 1, R + 1, FRAME_BYTES, device=local)
    torch.cuda.synchronize()

    state = [{"frame": vbase[k]} for k in range(NS)]

    def record(k, timing):
        if timing:
            for name, t0, t1 in ctxs[k].kernel_spans():
                kernel_ms.setdefault(name, []).append(t1 - t0)
                spans.setdefault(name, []).append((t0, t1))
            executed.append(executed_flops(ctxs[k], ctxs[k].corr_work(), B))

    def step(k, timing):
        st = state[k]
        f = st["frame"]
        i = (f - vbase[k]) % R + 1
        halo = None
        if i == 1 and f > 0:
            # stream start (vbase > 0) or wrap-around: pass the previous frame
            halo = frames[k].data_ptr() + (0 if f == vbase[k] else R * FRAME_BYTES)
        c = ctxs[k]
        if NL == 1:
            c.detect_device(frames[k].data_ptr() + i * FRAME_BYTES, FRAME_BYTES, B, f, d_prev_ptr=halo)
            record(k, timing)
        else:  # pipelined: keep every lane busy (finished lanes are reused), collect in submission order
            if c.pending() == 2 * NL:
                c.collect(raw=True)
                record(k, timing)
            c.submit_device(frames[k].data_ptr() + i * FRAME_BYTES, FRAME_BYTES, B, f, d_prev_ptr=halo)
        st["frame"] = f + B

    def drain(k, timing):
        while ctxs[k].pending():
            ctxs[k].collect(raw=True)
            record(k, timing)

    def run(k, n, timing):
        for _ in range(n):
            step(k, timing)
        drain(k, timing)

    def run_all(n, timing):
        if NS == 1 or args.round_robin:
            for _ in range(n):
                for k in range(NS):
                    step(k, timing)
            for k in range(NS):
                drain(k, timing)
            return
        import threading
        errors = []

        def guarded(k):
            try:
                run(k, n, timing)
            except BaseException as e:  # re-raised below: a failed stream must fail the bench
                errors.append(e)

        th = [threading.Thread(target=guarded, args=(k,)) for k in range(NS)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errors:
            raise errors[0]

    kernel_ms, spans, executed = {}, {}, []
    run_all(args.warmup, False)
    for c in ctxs:
        c.set_debug(2)  # HIP events around every kernel on the ctx stream
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run_all(args.steps, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for c in ctxs:
        c.set_debug(0)
    ctx = ctxs[0]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    gathered, local_samples = gather_results(ctxs, frames, state, vbase, R, B, FRAME_BYTES, world, rank)
    total_frames = args.steps * B * NS * world
    fps = total_frames / elapsed

    flops = algorithmic_flops_per_frame(ctx)
    # One k_corr "launch" = the width-group dispatches of one batch.  With
    # several streams per GPU the launches of different streams overlap, so
    # the duration per launch is the union of all k_corr spans (HIP events
    # against one device epoch) divided by the number of launches; with one
    # stream this is the plain mean.
    corr_spans = spans.get("k_corr", [])
    corr_avg_ms = union_ms(corr_spans) / max(1, len(corr_spans))
    algorithmic_tf = flops * B / (corr_avg_ms * 1e-3) / 1e12
    # the kernel's own rate: the FLOP it executed (dark tiles skipped) per launch
    exec_per_launch = (sum(executed) / len(executed)) if executed and None not in executed else flops * B
    achieved_tf = exec_per_launch / (corr_avg_ms * 1e-3) / 1e12
    peak_tf = F16_PEAK_TFLOPS if f16 else FP32_PEAK_TFLOPS
    traffic = None  # HBM bytes per launch from this tree's PMC passes (scripts/pmc_traffic.py)
    if os.path.exists(PMC_TRAFFIC):
        with open(PMC_TRAFFIC) as fh:
            traffic = json.load(fh).get("hbm_bytes_per_launch")
    out = {
        "metric": METRIC,
        "value": round(fps, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16xf16->f32 (non-parity LM_CORR_F16)" if f16 else "f32",
        "data": "synthetic (lm_synth.h scene, resident in HBM)",
        "config": {"workload": workload,
                   "batch_frames": B, "streams_per_gpu": NS, "frames_per_rank": args.steps * B * NS,
                   "lanes_per_context": NL, "resident_frames_per_stream": R,
                   "stream_priorities": "alternating high/low" if os.environ.get("LM_STREAM_PRIO", "1") != "0" else "equal",
                   "corr_launches": ("one merged launch" if NS * NL == 1 else "one per detector width")
                   if os.environ.get("LM_CORR_PLAN") not in ("0", "1") else f"LM_CORR_PLAN={os.environ['LM_CORR_PLAN']}",
                   "dark_tiles": "skipped" if os.environ.get("LM_CORR_DARK", "1") != "0" else "computed",
                   "parallelism": f"frame shards x{world} (no collective)"},
        "hbm_gbs": round(fps * FRAME_BYTES / 1e9, 3),
        "roofline": {"bound": "mfma" if f16 else "valu",
                     "compute_roof": "dense f16 MFMA (v_mfma_f32_32x32x16_f16)" if f16 else
                     "fp32 VALU (v_pk_fma_f32; equals the f32 MFMA peak)",
                     "kernel": "k_corr", "achieved": round(achieved_tf, 3), "peak": peak_tf,
                     "unit": "TFLOP/s", "frac": round(achieved_tf / peak_tf, 4),
                     "traffic": traffic if not f16 and args.config == "c3" else None,
                     "executed_flop_per_launch": int(exec_per_launch),
                     "algorithmic_flop_per_launch": flops * B,
                     "executed_fraction": round(exec_per_launch / (flops * B), 4),
                     "algorithmic_tflops": round(algorithmic_tf, 3),
                     "algorithmic_frac": round(algorithmic_tf / peak_tf, 4),
                     "flop_note": "achieved/frac: FLOP executed per launch (point detectors' dark tiles, whose scores "
                                  "the reference zeroes with its brightness mask, are not computed); "
                                  "algorithmic_*: SURVEY.md 8(d)'s count over every consumed output",
                     "avg_launch_ms": round(corr_avg_ms, 5),
                     "launches": len(corr_spans),
                     "duration": "union of k_corr HIP-event spans over all streams / launches"},
        "kernel_avg_ms": {k: round(sum(v) / len(v), 5) for k, v in kernel_ms.items()},
        "kernel_busy_ms_per_batch": {k: round(union_ms(v) / len(v), 5) for k, v in spans.items()},
    }
    out["gathered"] = gathered
    if (rank == 0 and world == 1 and not args.no_cpu) or args.check_all_ranks:
        # the CPU baseline leg: the oracle timed on the same workload, and as
        # the checker of the GPU batches gathered above
        base, parity = cpu_baseline(cfg, args.cpu_seconds if world == 1 else 0.0, samples=local_samples)
        if world > 1:
            allp = [None] * world if rank == 0 else None
            dist.gather_object(parity, allp, dst=0)
            if rank == 0:
                parity = {"frames": sum(p["frames"] for p in allp), "streams": sum(p["streams"] for p in allp),
                          "bit_exact": all(p["bit_exact"] for p in allp), "ranks": world,
                          "first_frames": [f for p in allp for f in p["first_frames"]][:32],
                          "mismatching_batches": [m for p in allp for m in p["mismatching_batches"]],
                          "compared": allp[0]["compared"]}
        out["parity_sample"] = parity
        if parity is not None and not parity["bit_exact"]:
            print(f"bench: GPU results differ from the oracle at batches {parity['mismatching_batches']}",
                  file=sys.stderr, flush=True)
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = base
            out["cpu_baseline_threads"] = cpu_baseline_threads(cfg, min(8.0, args.cpu_seconds))
            out["cpu_baseline_node"] = cpu_baseline_node(cfg, min(8.0, args.cpu_seconds))
    if rank == 0:
        print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
