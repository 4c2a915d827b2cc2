"""Benchmark of the MI355X LocoMouse per-frame detection path.

`python bench.py --gpus N --steps K --warmup W` — one process per GPU.  The
driver launches N>1 with torch.distributed.run (RANK / WORLD_SIZE in the
environment); run without it, `--gpus N` spawns the N rank processes itself
before anything touches a GPU.  A WORLD_SIZE that differs from --gpus, or more
ranks on a node than it has GPUs (unless --oversubscribe), is an error.

Default mode ("weak"): a step is one batch of B consecutive synthetic
1024x256 frames (already resident in HBM) per context through the whole
per-frame path — ingest, the six detectors, tail, NMS, unary/pairwise costs,
side<->bottom matching — up to and including the copy of the results into
host memory in the reference's container layout.  Every rank runs its own
frames (no collective on the data path).  Rank 0 prints one JSON line.  The
last batch each context collected inside the timed loop is checked against
the CPU oracle (`parity_sample`).

`--video-frames N` ("strong", BASELINE config 4): ONE video of N frames split
into contiguous shards, one per rank (main.cpp:54-82's loop over a shard; a
shard > 0 starts with its predecessor frame as a 1-frame halo).  The timed
region covers the whole shard, pipeline fill included, with every batch's
results copied out of the context; rank 0 gathers all N frames' results and
checks every frame against the oracle on the host's threads.
"""
import argparse
import json
import math
import os
import platform
import socket
import subprocess
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
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r06", "pmc_k_corr.json")  # this tree's PMC passes at the default shape (scripts/gpu_r6.sh step traffic)


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


def executed_flops(ctx, work, slots):
    """FLOP the correlation executed for a batch that processed `slots` frame
    slots (n, or n + 1 when its halo frame was recomputed: the same slots
    the point-detector counts cover): the tail detectors over every output,
    the point detectors over the outputs of their bright tiles only (`work` =
    Context.corr_work(): dark tiles -- no mouse pixel > 25, all scores zeroed
    by the reference's mask -- are skipped).  None when not recorded."""
    if work is None or slots is None:
        return None
    g = ctx.geometry()
    w = ctx.cfg.weights
    tw = g.tail_box_width
    hb, hs = g.bb_bottom_mouse.height, g.bb_side_mouse.height
    ob, os_ = work["outputs"]
    return 2 * (ob * (w["paw_bottom"].size + w["snout_bottom"].size) + os_ * (w["paw_side"].size + w["snout_side"].size)
                + slots * (hb * tw * w["tail_bottom"].size + hs * tw * w["tail_side"].size))


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


def host_cpu_share():
    """Host threads this GPU's share of the node may use: the CPUs this
    process may run on, capped by the box's per-GPU share (OMP_NUM_THREADS,
    16 per MI355X on the pool: a 128-core node split over 8 GPUs)."""
    n = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(share))) if share and share.isdigit() else n


def cpu_model():
    cpu = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return cpu


def _scene_frames(cfg, idx):
    """Synthetic frames of the given scene indices (the oracle's C twin of
    lm_synth.h; test infrastructure, used by the checker only)."""
    import numpy as np

    from oracle import oracle as O
    idx = list(idx)
    out = np.empty((len(idx), cfg.rows, cfg.cols), dtype=np.uint8)
    i = 0
    while i < len(idx):  # runs of consecutive indices in one call
        j = i + 1
        while j < len(idx) and idx[j] == idx[j - 1] + 1:
            j += 1
        out[i:j] = O.synth_frames_c(cfg.rows, cfg.cols, idx[i], j - i)
        i = j
    return out


def oracle_check(cfg, items, threads=None, chunk=64):
    """The oracle as the checker of GPU results.  `items`: (label, GPU result
    dict, scene index of the frame before the first -- None when the result
    starts at frame 0 of the video --, scene indices of its frames).  Each
    result is cut into chunks of at most `chunk` frames; a chunk runs through
    oracle/lm_oracle.cpp with its predecessor frame as a 1-frame halo (the
    sharded path's semantics, tests/test_multiproc.py), in `threads` host
    threads, and every lm_batch_result array is compared bit for bit.
    Returns {"frames", "bit_exact", "mismatching", "seconds"}."""
    from concurrent.futures import ThreadPoolExecutor

    from locomouse_cpp_amd.results import head_results, same_results, slice_results
    from oracle import oracle as O
    jobs = []
    for label, got, prev_scene, scenes in items:
        n = got["n_frames"]
        for a in range(0, n, chunk):
            b = min(n, a + chunk)
            halo = (prev_scene if a == 0 else scenes[a - 1])
            jobs.append((label, got, a, b, halo, scenes[a:b]))

    def run(job):
        label, got, a, b, halo, sc = job
        fr = _scene_frames(cfg, ([] if halo is None else [halo]) + list(sc))
        ref = O.OracleRun(cfg, fr).result
        if halo is not None:
            ref = slice_results(ref, 1)
        mine = head_results(slice_results(got, a), b - a)
        return label, a, same_results(mine, ref)

    t0 = time.perf_counter()
    with ThreadPoolExecutor(max_workers=threads or host_cpu_share()) as ex:
        out = list(ex.map(run, jobs))
    bad = sorted({lab for lab, _, ok in out if not ok}, key=str)
    return {"frames": int(sum(it[1]["n_frames"] for it in items)), "bit_exact": not bad, "mismatching": bad[:32],
            "seconds": round(time.perf_counter() - t0, 2)}


def cpu_baseline(cfg, seconds=10.0, max_frames=2000, chunk=50):
    """The oracle (CPU restatement, 1 thread, AVX2+FMA) timed on a bounded
    sample of the same workload: chunks of `chunk` consecutive synthetic
    frames until `seconds` of CPU work."""
    from oracle import oracle as O
    frames = _scene_frames(cfg, range(chunk))
    done, t = 0, 0.0
    while (t < seconds and done < max_frames) or done == 0:
        t0 = time.perf_counter()
        O.OracleRun(cfg, frames)
        t += time.perf_counter() - t0
        done += chunk
    return {"value": done / t, "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{done} frames (chunks of {chunk} from frame 0), oracle/lm_oracle.cpp single thread, "
                      f"{t:.1f} s", "cpu": cpu_model()}


def cpu_baseline_threads(cfg, seconds=8.0, threads=None, chunk=50, pin=False):
    """The fair CPU baseline of SURVEY.md §8(d)(ii): the oracle on `threads`
    host threads (default: this GPU's CPU share), each on its own contiguous
    chunk of frames (frame-sharded like the multi-GPU path; ctypes releases
    the GIL inside the oracle call).  pin: each thread is bound to one CPU of
    the affinity mask (Linux sched_setaffinity on the calling thread)."""
    import threading

    from oracle import oracle as O
    if threads is None:
        threads = host_cpu_share()
    cpus = sorted(os.sched_getaffinity(0))
    samples = [_scene_frames(cfg, range(chunk * t, chunk * (t + 1))) for t in range(threads)]
    counts = [0] * threads
    stop = time.perf_counter() + seconds

    def work(t):
        if pin:
            os.sched_setaffinity(0, {cpus[t % len(cpus)]})
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
            "sample": f"{sum(counts)} frames, {threads} threads{' (pinned)' if pin else ''} x chunks of {chunk} "
                      f"frames, {el:.1f} s wall"}


def cgroup_cpus():
    """CPUs' worth of time the process's cgroup may use (cpu.max /
    cpu.cfs_quota_us), or None when unlimited or unreadable."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            return None if q == "max" else max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as fh:
            q = int(fh.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
            per = int(fh.read())
        return None if q <= 0 else max(1, math.ceil(q / per))
    except (OSError, ValueError):
        return None


def cpu_baseline_node(cfg, seconds=8.0):
    """BASELINE.md §2's `nproc`-thread line: one oracle thread per CPU this
    process may run on (capped by the cgroup's CPU quota: threads beyond it
    only time-slice), each pinned to its CPU, on its own contiguous chunks of
    50 frames.  On a shared GPU box the other GPUs' jobs use the same CPUs,
    so this is the whole-node figure as measured there; the per-GPU share
    (cpu_baseline_threads) is the fair per-GPU comparison."""
    n = len(os.sched_getaffinity(0))
    quota = cgroup_cpus()
    line = cpu_baseline_threads(cfg, seconds, threads=min(n, quota or n), chunk=50, pin=True)
    line["nproc"] = os.cpu_count()
    line["affinity_cpus"] = n
    line["cgroup_cpu_quota"] = quota
    return line


def run_bb(args):
    """The whole-video bounding-box pass (lm_bb_push_device, method 0) on one
    GPU: frames resident in HBM, `--steps` pushes of `--batch` frames after
    `--warmup`; the CPU baseline is the oracle restatement on a bounded
    sample.  Prints one JSON line (not the headline metric)."""
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


# ----------------------------------------------------------------- launcher

def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv):
    """`--gpus N` without torchrun: start N rank processes (RANK, LOCAL_RANK,
    WORLD_SIZE, LOCAL_WORLD_SIZE, MASTER_* set as torchrun sets them) before
    this process touches a GPU, forward their output, and return the first
    non-zero exit status (the other ranks are then stopped: a rank that
    failed would leave them waiting at the barrier)."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def rank_env(args):
    """(world, rank, local rank, ranks on this node) from the launcher's
    environment; None when this process must spawn the ranks itself."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus > 1:
            return None
        return 1, 0, 0, 1
    world = int(ws)
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
                         f"(torchrun --nproc-per-node {args.gpus}, or bench.py --gpus N alone)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    return world, rank, local, local_world


# ------------------------------------------------------------ one rank

def resolve_shape(args):
    """Contexts per GPU, pipeline lanes per context and frames per batch left
    unset on the command line.  C3 fp32 detection: 8 contexts x 448 frames for
    the resident stream (the headline line); for one video (--video-frames,
    BASELINE config 4) by the rank's share of it -- up to 2,500 frames (the
    8-GPU shard of the 10,000-frame video is 1,250): one context x 4 lanes in
    6 equal batches, else 4 contexts x 2 lanes x 313 frames.  4 x 1 x 256 for
    every other config and mode."""
    c3 = args.config == "c3" and args.precision == "fp32" and args.workload == "detect" and not args.host_frames
    shape = (4, 1, 256)
    if c3 and args.video_frames == 0 and args.lanes in (None, 1):
        shape = (8, 1, 448)
    elif c3 and args.video_frames > 0:
        share = -(-args.video_frames // max(1, args.gpus))
        shape = (1, 4, max(1, -(-share // 6))) if share <= 2500 else (4, 2, 313)
    if args.streams is None:
        args.streams = shape[0]
    if args.lanes is None:
        args.lanes = shape[1]
    if args.batch is None:
        args.batch = shape[2]
    return args


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--precision", choices=["fp32", "f16"], default="fp32",
                    help="f16: the non-parity LM_CORR_F16 correlation (BASELINE config 5)")
    ap.add_argument("--batch", type=int, default=None,
                    help="frames per batch (default: 448 for the C3 resident stream, else 256)")
    ap.add_argument("--resident", type=int, default=6400, help="frames resident in HBM per stream (cycled)")
    ap.add_argument("--streams", type=int, default=None,
                    help="contexts per GPU, each with its own host thread (default: 8 for the C3 resident stream, "
                         "else 4)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="pipeline lanes per context (lm_setup.pipeline_lanes: batches in flight on their own HIP "
                         "streams, driven with lm_detect_submit / lm_detect_collect; default: 1, or for one C3 "
                         "video 4 / 2 by the rank's share, see resolve_shape)")
    ap.add_argument("--video-frames", type=int, default=0,
                    help="strong scaling (BASELINE config 4): one video of this many frames sharded over the ranks; "
                         "steps = timed passes over the shard")
    ap.add_argument("--host-frames", action="store_true",
                    help="frames in pinned host memory, submitted with the host API (lm_detect_batch / "
                         "lm_detect_submit): the H2D copy is inside the timed loop (BASELINE.md §2's end-to-end figure)")
    ap.add_argument("--oversubscribe", action="store_true",
                    help="allow more ranks on a node than it has GPUs (rehearsals only: ranks share devices)")
    ap.add_argument("--check-all-ranks", action="store_true",
                    help="every rank compares its sampled batches with the oracle (multi-rank rehearsals)")
    ap.add_argument("--round-robin", action="store_true", help="one host thread drives all streams in turn")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip the oracle check of the timed batches")
    ap.add_argument("--workload", choices=["detect", "bb"], default="detect",
                    help="bb: the whole-video bounding-box pass (SURVEY.md §8(f) row 1) instead of the headline path")
    ap.add_argument("--bb-semantics", type=int, default=0, help="firstLastOverT: 0 as executed, 1 integer sums")
    args = ap.parse_args()
    # The C3 resident stream (the headline line) runs 8 contexts x 448-frame
    # batches: 4 x 256 478.4k, 8 x 320 491.0k frames/s over three same-box
    # repetitions (profiles/r05/sweep/shape_b.txt; 5, 6, 10 contexts
    # slower), then 8 x 448 493.9k vs 8 x 320 486.6k over six
    # (shape_c.txt, shape_d.txt; 512 and 640 no better; 12 or 16 contexts,
    # or 2 lanes each, no better either: shape_e.txt; re-checked on round 6's
    # final kernels, 8 x 512 and 10 x 448 within noise:
    # profiles/r06/corr_ab/r6s_c3_shape.txt).  One C3 video
    # (profiles/r06/c4/): the whole 10,000 frames on one GPU 410k at
    # 4 x 1 x 256, 440-447k at 4 x 2 x 256 / 313; the 1,250-frame shard
    # 3.32 ms at 1 x 4 x 250, 3.08 ms at 1 x 4 x 209.  The other configs and
    # modes keep the shapes they were measured with.
    resolve_shape(args)
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.workload == "bb":
        return run_bb(args)
    env = rank_env(args)
    if env is None:  # --gpus N without a launcher: one child process per rank, spawned before any GPU call
        return spawn_ranks(args.gpus, sys.argv[1:])
    world, rank, local, local_world = env

    import torch
    import torch.distributed as dist

    # One process per GPU.  The data path has no collective (frame shards are
    # independent), so the only inter-rank traffic -- the start/stop barrier,
    # the max-over-ranks of the elapsed time and the result gather -- goes
    # over gloo on the host.
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py needs a GPU (no HIP device visible)")
    if local_world > ndev and not args.oversubscribe:
        raise SystemExit(f"bench.py: {local_world} ranks on this node but {ndev} visible GPU(s); one rank per GPU "
                         f"(--oversubscribe only for rehearsals that share devices)")
    device = local % ndev
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("gloo")
    try:
        if args.video_frames > 0:
            out = run_video(args, world, rank, device)
        else:
            out = run_stream(args, world, rank, device)
        if rank == 0:
            print(json.dumps(out), flush=True)
        bad = out is not None and (out.get("parity_sample") or out.get("video_check") or {}).get("bit_exact") is False
    finally:
        if world > 1:
            dist.destroy_process_group()
    return 3 if bad else 0


def _setup(args, device):
    from locomouse_cpp_amd import synthetic as S
    rows, cols, workload = CONFIGS[args.config]
    cfg = S.SyntheticConfig(rows=rows, cols=cols)
    f16 = args.precision == "f16"
    if f16:  # non-parity mode (LM_CORR_F16): f16 weights, fp32 accumulation on the matrix cores
        cfg.setup.corr_precision = 1
        workload = workload.replace("(fp32, bit-exact mode)", "(LM_CORR_F16: f16 weights, fp32 accumulation, non-parity)")
        workload += "" if "LM_CORR_F16" in workload else " [LM_CORR_F16 non-parity correlation]"
    return cfg, rows, cols, workload, f16


def _roofline(ctx, f16, config, spans, executed, B):
    flops = algorithmic_flops_per_frame(ctx)
    # One k_corr "launch" = the width-group dispatches of one batch.  With
    # several streams per GPU the launches of different streams overlap, so
    # the duration per launch is the union of all k_corr spans (HIP events
    # against one device epoch) divided by the number of launches; with one
    # stream this is the plain mean.
    corr_spans = spans.get("k_corr", [])
    corr_avg_ms = union_ms(corr_spans) / max(1, len(corr_spans))
    algorithmic_tf = flops * B / (corr_avg_ms * 1e-3) / 1e12 if corr_avg_ms > 0 else 0.0
    # the kernel's own rate: the FLOP it executed (dark tiles skipped) per launch
    exec_per_launch = (sum(executed) / len(executed)) if executed and None not in executed else flops * B
    achieved_tf = exec_per_launch / (corr_avg_ms * 1e-3) / 1e12 if corr_avg_ms > 0 else 0.0
    peak_tf = F16_PEAK_TFLOPS if f16 else FP32_PEAK_TFLOPS
    traffic, measured, pmc = None, False, {}  # HBM bytes per launch from this tree's PMC passes (scripts/pmc_traffic.py)
    if os.path.exists(PMC_TRAFFIC) and not f16 and config == "c3":
        with open(PMC_TRAFFIC) as fh:
            pmc = json.load(fh)
        # measured at the default shape; per frame x this launch's frames
        # otherwise -- an estimate (per-launch weight and L2 traffic does not
        # scale with the frame count), labelled as such in traffic_source
        measured = pmc.get("batch_frames") == B
        traffic = pmc.get("hbm_bytes_per_launch") if measured else int(pmc["hbm_bytes_per_frame"] * B)
    return {"bound": "mfma" if f16 else "valu",
            "compute_roof": "dense f16 MFMA (v_mfma_f32_32x32x16_f16)" if f16 else
            "fp32 VALU (v_pk_fma_f32; equals the f32 MFMA peak)",
            "kernel": "k_corr", "achieved": round(achieved_tf, 3), "peak": peak_tf,
            "unit": "TFLOP/s", "frac": round(achieved_tf / peak_tf, 4),
            "traffic": traffic,
            "traffic_source": (os.path.relpath(PMC_TRAFFIC, ROOT) + ("" if measured else
                               f" (scaled from its {pmc.get('batch_frames')}-frame PMC launch to {B} frames: an estimate)"))
            if traffic else None,
            "executed_flop_per_launch": int(exec_per_launch),
            "algorithmic_flop_per_launch": flops * B,
            "executed_fraction": round(exec_per_launch / (flops * B), 4),
            "algorithmic_tflops": round(algorithmic_tf, 3),
            "algorithmic_frac": round(algorithmic_tf / peak_tf, 4),
            "flop_note": "achieved/frac: FLOP executed per launch (point detectors' dark tiles, whose scores "
                         "the reference zeroes with its brightness mask, are not computed; halo slots counted); "
                         "algorithmic_*: SURVEY.md 8(d)'s count over every consumed output of the batch's frames",
            "avg_launch_ms": round(corr_avg_ms, 5),
            "launches": len(corr_spans),
            "duration": "union of k_corr HIP-event spans over all streams / launches"}


def _threads_run(n, fn, serial=False):
    """fn(k) for k in range(n), one host thread each (serial: in this
    thread); the first exception is re-raised."""
    if n == 1 or serial:
        for k in range(n):
            fn(k)
        return
    import threading
    errors = []

    def guarded(k):
        try:
            fn(k)
        except BaseException as e:  # re-raised below: a failed stream must fail the bench
            errors.append(e)

    th = [threading.Thread(target=guarded, args=(k,)) for k in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise errors[0]


def run_stream(args, world, rank, device):
    """Weak scaling: NS contexts per GPU, each cycling its own resident
    stream of frames; --steps batches per context are timed."""
    import torch
    import torch.distributed as dist

    from locomouse_cpp_amd.abi import result_to_numpy
    from locomouse_cpp_amd.runtime import Context, synth_frames_device

    cfg, rows, cols, workload, f16 = _setup(args, device)
    B = args.batch
    NS = max(1, args.streams)
    NL = max(1, args.lanes)
    # Frames resident per stream, cycled: a multiple of the batch and of the
    # scene's motion period (100 frames), so the wrap-around is a continuous
    # step of the video, not a jump.
    unit = B * 100 // math.gcd(B, 100)
    R = max(unit, args.resident // unit * unit)
    FRAME_BYTES = rows * cols
    # NS contexts per GPU, each with its own HIP stream(s) and host thread, each
    # on its own contiguous range of the video (rank-major): like a shard, its
    # first batch gets the previous frame as a 1-frame halo.
    ctxs = [Context(cfg, max_batch=B, device=device, lanes=NL) for _ in range(NS)]
    frames = torch.empty((NS, R + 1, rows, cols), dtype=torch.uint8, device=f"cuda:{device}")
    vbase = [(rank * NS + k) * R for k in range(NS)]
    for k in range(NS):
        # index 0 holds frame vbase-1 (the halo), index i frame vbase+i-1
        synth_frames_device(frames[k].data_ptr(), rows, cols, vbase[k] - 1, R + 1, FRAME_BYTES, device=device)
    torch.cuda.synchronize()
    if args.host_frames:  # the same frames in page-locked host memory; the device copy is freed
        hframes = torch.empty(frames.shape, dtype=torch.uint8, pin_memory=True)
        hframes.copy_(frames)
        del frames
        torch.cuda.empty_cache()
        frames = hframes

    state = [{"frame": vbase[k]} for k in range(NS)]
    kernel_ms, spans, executed = {}, {}, []
    # the batches each context collected last inside the timed loop (the
    # parity sample): the very last one stays an lm_batch_result (valid until
    # the context's next call), the NL - 1 before it are copied out during
    # the drain while the later batches still run
    keep = [[] for _ in range(NS)]

    def record(k, timing, res, tail):
        c = ctxs[k]
        if timing:
            for name, t0, t1 in c.kernel_spans():
                kernel_ms.setdefault(name, []).append(t1 - t0)
                spans.setdefault(name, []).append((t0, t1))
            executed.append(executed_flops(c, c.corr_work(), c.batch_slots()))
            if tail is not None and tail < NL:
                keep[k].append(res if tail == 0 else result_to_numpy(res))

    def step(k, timing):
        st = state[k]
        f = st["frame"]
        i = (f - vbase[k]) % R + 1
        halo = None
        if i == 1 and f > 0:
            # stream start (vbase > 0) or wrap-around: pass the previous frame
            halo = frames[k].data_ptr() + (0 if f == vbase[k] else R * FRAME_BYTES)
        c = ctxs[k]
        ptr = frames[k].data_ptr() + i * FRAME_BYTES
        if NL == 1:
            if args.host_frames:
                res = c.detect_host_ptr(ptr, FRAME_BYTES, B, f, h_prev_ptr=halo)
            else:
                res = c.detect_device(ptr, FRAME_BYTES, B, f, d_prev_ptr=halo)
            st["last"] = res
            record(k, timing, res, None)
        else:  # pipelined: keep every lane busy (finished lanes are reused), collect in submission order
            if c.pending() == 2 * NL:
                record(k, timing, c.collect(raw=True), None)
            if args.host_frames:
                c.submit_host_ptr(ptr, FRAME_BYTES, B, f, h_prev_ptr=halo)
            else:
                c.submit_device(ptr, FRAME_BYTES, B, f, d_prev_ptr=halo)
        st["frame"] = f + B

    def drain(k, timing):
        c = ctxs[k]
        while c.pending():
            res = c.collect(raw=True)
            record(k, timing, res, c.pending())

    def run_all(n, timing):
        def one(k):
            for _ in range(n):
                step(k, timing)
            drain(k, timing)
        if NS > 1 and args.round_robin:
            for _ in range(n):
                for k in range(NS):
                    step(k, timing)
            for k in range(NS):
                drain(k, timing)
        else:
            _threads_run(NS, one)

    run_all(args.warmup, False)
    for c in ctxs:
        c.set_debug(2)  # HIP events around k_corr on the lane streams
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    run_all(args.steps, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if NL == 1:
        for k in range(NS):
            keep[k] = [state[k]["last"]]
    # the sample of timed batches, as plain arrays, with the scene indices of
    # the pixels they saw: resident frame i holds scene frame vbase - 1 + i;
    # the frame before a batch is resident frame i - 1, or the halo (frame 0
    # at the stream's start, frame R after a wrap-around)
    samples = []
    for k in range(NS):
        for r in keep[k]:
            res = r if isinstance(r, dict) else result_to_numpy(r)
            f = res["first_frame"]
            i = (f - vbase[k]) % R + 1
            prev = None if f == 0 else vbase[k] - 1 + (i - 1 if i > 1 else (0 if f == vbase[k] else R))
            samples.append((f, res, prev, [vbase[k] - 1 + i + j for j in range(res["n_frames"])]))
    for c in ctxs:
        c.set_debug(0)
    ctx = ctxs[0]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    gathered = gather_summary(samples, world, rank)
    total_frames = args.steps * B * NS * world
    fps = total_frames / elapsed
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
        "data": ("synthetic (lm_synth.h scene, in pinned host memory: H2D inside the timed loop)" if args.host_frames
                 else "synthetic (lm_synth.h scene, resident in HBM)"),
        "config": {"workload": workload + ("; frames from pinned host memory through the host API "
                                           "(lm_detect_batch / lm_detect_submit, H2D included)" if args.host_frames else ""),
                   "batch_frames": B, "streams_per_gpu": NS, "frames_per_rank": args.steps * B * NS,
                   "lanes_per_context": NL, "resident_frames_per_stream": R,
                   "stream_priorities": "alternating high/low" if os.environ.get("LM_STREAM_PRIO", "1") != "0" else "equal",
                   "corr_launches": ("one merged launch" if NS * NL == 1 else "one per detector width")
                   if os.environ.get("LM_CORR_PLAN") not in ("0", "1") else f"LM_CORR_PLAN={os.environ['LM_CORR_PLAN']}",
                   "dark_tiles": "skipped" if os.environ.get("LM_CORR_DARK", "1") != "0" else "computed",
                   "parallelism": f"frame shards x{world} (no collective)"},
        "hbm_gbs": round(fps * FRAME_BYTES / 1e9, 3),
        **({"h2d_gbs": round(fps * FRAME_BYTES / 1e9, 3)} if args.host_frames else {}),
        "roofline": _roofline(ctx, f16, args.config, spans, executed, B),
        "kernel_avg_ms": {k: round(sum(v) / len(v), 5) for k, v in kernel_ms.items()},
        "kernel_busy_ms_per_batch": {k: round(union_ms(v) / len(v), 5) for k, v in spans.items()},
        "gathered": gathered,
    }
    check = not args.no_check and (rank == 0 or args.check_all_ranks)
    if check and f16:
        out["parity_sample"] = {"skipped": "LM_CORR_F16 is the non-parity mode (candidate agreement: "
                                           "tests/test_gpu_f16.py)"}
    elif check:
        # the oracle as the checker of the batches timed above
        par = oracle_check(cfg, samples)
        par.update({"streams": NS, "lanes": NL, "batches": len(samples),
                    "first_frames": [int(s[0]) for s in samples][:16],
                    "source": "the last batches each context collected inside the timed loop",
                    "compared": "every lm_batch_result array (candidates, P22D, unary, pairwise CSC, tail) against "
                                "oracle/lm_oracle.cpp on the same synthetic frames"})
        if world > 1 and args.check_all_ranks:
            allp = [None] * world if rank == 0 else None
            dist.gather_object(par, allp, dst=0)
            if rank == 0:
                par = {"frames": sum(p["frames"] for p in allp), "batches": sum(p["batches"] for p in allp),
                       "bit_exact": all(p["bit_exact"] for p in allp), "ranks": world,
                       "mismatching": [m for p in allp for m in p["mismatching"]],
                       "source": allp[0]["source"], "compared": allp[0]["compared"]}
        out["parity_sample"] = par
        if not par["bit_exact"]:
            print(f"bench: GPU results differ from the oracle at batches {par['mismatching']}", file=sys.stderr,
                  flush=True)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
        out["cpu_baseline_threads"] = cpu_baseline_threads(cfg, min(8.0, args.cpu_seconds))
        out["cpu_baseline_node"] = cpu_baseline_node(cfg, min(8.0, args.cpu_seconds))
    for c in ctxs:
        c.close()
    return out if rank == 0 else None


def gather_summary(samples, world, rank):
    """The host gather of north_star's multi-GPU design: every rank's sampled
    batches (their compact candidate arrays) go to rank 0 over the host
    process group, and rank 0 checks that the frame ranges are whole and
    disjoint."""
    import torch.distributed as dist
    mine = [{"first": s[0], "n": s[1]["n_frames"], "cand": s[1]["cand"], "cand_offset": s[1]["cand_offset"],
             "tail": s[1]["tail"]} for s in samples]
    allr = [None] * world if rank == 0 else None
    if world > 1:
        dist.gather_object(mine, allr, dst=0)
    else:
        allr = [mine]
    if rank != 0:
        return None
    parts = sorted((p for r in allr for p in r), key=lambda p: p["first"])
    for p in parts:
        if len(p["cand_offset"]) != 4 * p["n"] + 1 or p["tail"].shape[0] != p["n"]:
            raise RuntimeError(f"gathered batch at frame {p['first']} is not whole")
    for a, b in zip(parts, parts[1:]):
        if a["first"] + a["n"] > b["first"]:
            raise RuntimeError("gathered frame ranges overlap")
    return {"ranks": world, "batches": len(parts), "frames": int(sum(p["n"] for p in parts)),
            "candidates": int(sum(len(p["cand"]) for p in parts)),
            "first_frames": [int(p["first"]) for p in parts][:16], "whole_and_disjoint": True,
            "transport": "gloo gather_object (host)" if world > 1 else "local"}


def video_shards(n_frames, world, rank, streams):
    """[(lo, hi)] of this rank's contexts: the rank's contiguous shard of the
    video (shard.shard_range) split again contiguously over its contexts."""
    from locomouse_cpp_amd.shard import shard_range
    lo, hi = shard_range(n_frames, rank, world)
    subs = []
    for k in range(streams):
        a, b = shard_range(hi - lo, k, streams)
        if b > a:
            subs.append((lo + a, lo + b))
    return subs


def piece_batches(n, max_batch):
    """Batch sizes for a piece of n frames: the fewest batches of at most
    max_batch frames, as equal as possible (larger ones first)."""
    if n <= 0:
        return []
    nb = -(-n // max_batch)
    q, r = divmod(n, nb)
    return [q + 1] * r + [q] * (nb - r)


def check_video(parts, n_frames):
    """Rank 0: the gathered (first frame, result dict) pieces of the whole
    video, sorted; raises unless they cover frames [0, n_frames) exactly
    once.  Returns the pieces in frame order."""
    parts = sorted(parts, key=lambda p: p[0])
    pos = 0
    for first, res in parts:
        if first != pos:
            raise RuntimeError(f"gathered video: frames {pos}..{first - 1} missing or overlapping (piece at {first})")
        if len(res["cand_offset"]) != 4 * res["n_frames"] + 1 or res["tail"].shape[0] != res["n_frames"]:
            raise RuntimeError(f"gathered piece at frame {first} is not whole")
        pos += res["n_frames"]
    if pos != n_frames:
        raise RuntimeError(f"gathered video has {pos} frames, expected {n_frames}")
    return parts


def run_video(args, world, rank, device):
    """Strong scaling over one video of --video-frames frames (BASELINE
    config 4): rank r's shard [r * ceil(N/W), ...) split over its contexts;
    each context runs its piece in batches of <= --batch (its first batch
    with the predecessor frame as halo).  --warmup untimed passes over the
    same pieces (graph capture for every batch shape and arena parity), then
    --steps timed passes; every batch's results are copied out of the context
    inside the timed region.  Rank 0 gathers the last pass and checks all N
    frames against the oracle."""
    import torch
    import torch.distributed as dist

    from locomouse_cpp_amd.results import concat_results
    from locomouse_cpp_amd.runtime import Context, synth_frames_device

    cfg, rows, cols, workload, f16 = _setup(args, device)
    N = args.video_frames
    NL = max(1, args.lanes)
    subs = video_shards(N, world, rank, max(1, args.streams))
    # each context's piece in equal batches of at most --batch frames (a
    # 313-frame piece is 2 x 157, not 256 + a ragged 57 whose kernels run
    # at a fraction of the device), one context per piece
    cuts = [piece_batches(hi - lo, args.batch) for lo, hi in subs]
    B = max(max(c) for c in cuts)
    FRAME_BYTES = rows * cols
    ctxs = [Context(cfg, max_batch=B, device=device, lanes=NL) for _ in subs]
    # piece k: device frames [lo - 1, hi) (index 0 = the halo frame lo - 1; unused when lo = 0)
    bufs = []
    for lo, hi in subs:
        t = torch.empty((hi - lo + 1, rows, cols), dtype=torch.uint8, device=f"cuda:{device}")
        if lo > 0:
            synth_frames_device(t.data_ptr(), rows, cols, lo - 1, hi - lo + 1, FRAME_BYTES, device=device)
        else:
            synth_frames_device(t[1:].data_ptr(), rows, cols, 0, hi - lo, FRAME_BYTES, device=device)
        bufs.append(t)
    torch.cuda.synchronize()
    results = [None] * len(subs)
    kernel_ms, spans, executed = {}, {}, []
    from locomouse_cpp_amd.abi import result_to_numpy

    def piece(k, timing):
        lo, hi = subs[k]
        c, buf = ctxs[k], bufs[k]
        base = buf.data_ptr()
        got = []

        def take(res):
            if timing:
                for name, t0, t1 in c.kernel_spans():
                    kernel_ms.setdefault(name, []).append(t1 - t0)
                    spans.setdefault(name, []).append((t0, t1))
                executed.append(executed_flops(c, c.corr_work(), c.batch_slots()))
            got.append(result_to_numpy(res))

        b0 = lo
        for n in cuts[k]:
            ptr = base + (b0 - lo + 1) * FRAME_BYTES
            halo = base if (b0 == lo and lo > 0) else None
            if NL == 1:
                take(c.detect_device(ptr, FRAME_BYTES, n, b0, d_prev_ptr=halo))
            else:
                if c.pending() == 2 * NL:
                    take(c.collect(raw=True))
                c.submit_device(ptr, FRAME_BYTES, n, b0, d_prev_ptr=halo)
            b0 += n
        while c.pending():
            take(c.collect(raw=True))
        results[k] = got

    def run_pass(timing):
        _threads_run(len(subs), lambda k: piece(k, timing))

    for _ in range(max(2, args.warmup)):  # both arena parities of every batch shape captured
        run_pass(False)
    for c in ctxs:
        c.set_debug(2)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_pass(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    for c in ctxs:
        c.set_debug(0)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    mine = [(subs[k][0], concat_results(results[k])) for k in range(len(subs))]
    allp = [None] * world if rank == 0 else None
    if world > 1:
        dist.gather_object(mine, allp, dst=0)
    else:
        allp = [mine]
    roof = _roofline(ctxs[0], f16, args.config, spans, executed, B)
    for c in ctxs:
        c.close()
    if rank != 0:
        return None
    parts = check_video([p for r in allp for p in r], N)
    fps = N * args.steps / elapsed
    out = {
        "metric": METRIC,
        "value": round(fps, 1),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f16xf16->f32 (non-parity LM_CORR_F16)" if f16 else "f32",
        "data": "synthetic (lm_synth.h scene, resident in HBM)",
        "config": {"workload": f"C4: one {N}-frame video sharded over {world} GPU(s) as contiguous frame ranges "
                               f"with a 1-frame halo (no collective); " + workload,
                   "video_frames": N, "batch_frames": B, "batches": [len(c) for c in cuts],
                   "contexts_per_gpu": len(subs), "lanes_per_context": NL,
                   "step": "one pass over the whole video (every rank's shard, pipeline fill included, results "
                           "copied to host arrays)",
                   "shards": [list(s) for s in subs] if world == 1 else f"{world} x ceil({N}/{world}) frames",
                   "parallelism": f"frame shards x{world} (no collective)"},
        "hbm_gbs": round(fps * FRAME_BYTES / 1e9, 3),
        "roofline": roof,
        "gathered": {"ranks": world, "pieces": len(parts), "frames": N, "whole_and_disjoint": True,
                     "transport": "gloo gather_object (host)" if world > 1 else "local"},
    }
    if not args.no_check and not f16:
        items = [(first, res, None if first == 0 else first - 1, list(range(first, first + res["n_frames"])))
                 for first, res in parts]
        chk = oracle_check(cfg, items, chunk=50)
        chk["compared"] = ("every frame of the video: every lm_batch_result array against oracle/lm_oracle.cpp "
                           "(chunks of 50 frames with a 1-frame halo, host threads)")
        out["video_check"] = chk
        if not chk["bit_exact"]:
            print(f"bench: GPU results differ from the oracle in pieces {chk['mismatching']}", file=sys.stderr,
                  flush=True)
    return out


if __name__ == "__main__":
    sys.exit(main())
