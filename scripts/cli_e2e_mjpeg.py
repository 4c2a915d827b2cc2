"""The drop-in program end to end on an MJPEG video.

Writes a synthetic C3 video of N frames (default 10,000; 1024 x 256, the
C3 scene of lm_synth.h) as an MJPEG AVI -- 4:2:0 colour JPEG frames encoded by
Pillow (libjpeg-turbo), the blue plane carrying the frame -- with its
config / model / calibration / background files, then runs
`locomouse_cpp_amd/bin/LocoMouse` (the reference's main.cpp sequence) on it
with LM_TIMING=1:

  * one device (LM_DEVICES unset), and
  * four "devices" on the one GPU (LM_DEVICES=0,0,0,0 LM_OVERSUBSCRIBE=1),

each REPS times, and reports frames/s of the whole program and the split of
its wall time: context setup, the per-frame loop (file reads + MJPEG decode
on `decode_threads` host threads; the hand-over of each batch, i.e. the
pinned copy and the H2D issue; waiting for the GPU's results), the tracker
and the YAML export.  After the runs the output YAML's tracks are checked
against the oracle: oracle detection (oracle/lm_oracle.cpp) on Pillow's
decoding of the same JPEG frames -- which the program's decoder reproduces
byte for byte (tests/test_mjpeg.py) -- in 64-frame chunks with their halo
frames on the host's threads, then the restated tracker
(oracle/track_oracle.py).  The oracle is the checker here, never the thing
timed.  Prints one JSON line (and writes it to --out).

  python scripts/cli_e2e_mjpeg.py [--frames 10000] [--reps 2] [--out FILE]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import media_writers as MW  # noqa: E402
from locomouse_cpp_amd import runtime  # noqa: E402
from locomouse_cpp_amd import synthetic as S  # noqa: E402


def host_threads():
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(n, int(omp))) if omp and omp.isdigit() else n


def encode(frames, threads, **jpeg):
    """JPEG frames (Pillow) and Pillow's channel-0 decoding of each."""
    chunks = [frames[i:i + 256] for i in range(0, len(frames), 256)]
    with ThreadPoolExecutor(threads) as ex:
        js = [j for part in ex.map(lambda c: MW.jpeg_frames(c, **jpeg), chunks) for j in part]
        dec = np.stack(list(ex.map(MW.decode_jpeg_channel0, js)))
    return js, dec


def parse_timing(stdout):
    for line in stdout.splitlines():
        if line.startswith("LM_TIMING"):
            f = line.split()[1:]
            return {k: float(v) for k, v in zip(f[::2], f[1::2])}
    return {}


def oracle_tracks(cfg, frames, threads, chunk=64):
    """Oracle detection over the whole video (chunks with their halo frame,
    as the sharded path runs) and the restated tracker."""
    from locomouse_cpp_amd.results import concat_results, slice_results
    from oracle import oracle as O
    from oracle import track_oracle as TO
    n = len(frames)

    def run(a):
        b = min(n, a + chunk)
        if a == 0:
            return O.OracleRun(cfg, frames[a:b]).result
        return slice_results(O.OracleRun(cfg, frames[a - 1:b]).result, 1)

    with ThreadPoolExecutor(threads) as ex:
        res = concat_results(list(ex.map(run, range(0, n, chunk))))
    p = cfg.params
    corner = [p.bounding_box_bottom.x + p.bounding_box_bottom.width,
              p.bounding_box_bottom.y + p.bounding_box_bottom.height,
              p.bounding_box_side.y + p.bounding_box_side.height]
    return TO.run_tracks(res, O.geometry(cfg), p, [corner] * n, n)


def check_tracks(yml, ref):
    from test_cli import fs_node
    ok = True
    for i in range(4):
        _, _, m = fs_node(yml, f"paw_tracks{i}", cap=1 << 22)
        ok &= np.array_equal(m.astype(np.int32), np.array(ref["paw_tracks"][i], np.int32))
    _, _, m = fs_node(yml, "snout_tracks0", cap=1 << 22)
    ok &= np.array_equal(m.astype(np.int32), np.array(ref["snout_tracks"][0], np.int32))
    _, _, m = fs_node(yml, "tracks_tail", cap=1 << 22)
    ok &= np.array_equal(m.astype(np.int32), np.array(ref["tracks_tail"], np.int32))
    return bool(ok)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--quality", type=int, default=92)
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-check", action="store_true")
    a = ap.parse_args()
    from oracle import oracle as O
    cfg = S.SyntheticConfig()
    n = a.frames
    threads = host_threads()
    out = {"what": "LocoMouse program end to end: MJPEG AVI -> output_<stem>.yml", "frames": n,
           "video": f"{cfg.cols}x{cfg.rows} 4:2:0 colour MJPEG (Pillow/libjpeg-turbo, quality {a.quality})",
           "host_threads": threads}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
        t0 = time.perf_counter()
        frames = O.synth_frames_c(cfg.rows, cfg.cols, 0, n)
        js, dec = encode(frames, threads, mode="RGB", quality=a.quality, subsampling=2)
        del frames
        paths = {k: os.path.join(d, v) for k, v in (("config", "config.yml"), ("video", "mouse_R.avi"),
                                                     ("background", "mouse_R.png"), ("model", "model.yml"),
                                                     ("calibration", "calibration.yml"))}
        MW.write_config(paths["config"], cfg)
        MW.write_model(paths["model"], cfg)
        MW.write_calibration(paths["calibration"], cfg)
        MW.write_png(paths["background"], cfg.background)
        MW.write_mjpeg_avi(paths["video"], js, cfg.cols, cfg.rows)
        out["video_bytes"] = os.path.getsize(paths["video"])
        out["mean_jpeg_bytes"] = round(out["video_bytes"] / n)
        del js
        out["input_write_s"] = round(time.perf_counter() - t0, 1)
        args = [runtime.CLI_PATH, "0", paths["config"], paths["video"], paths["background"], paths["model"],
                paths["calibration"], "R", d]
        yml = os.path.join(d, "output_mouse_R.yml")
        modes = {"1 device": {}, "4 devices on one GPU": {"LM_DEVICES": "0,0,0,0", "LM_OVERSUBSCRIBE": "1"}}
        runs = {}
        for name, env in modes.items():
            best = None
            for _ in range(a.reps):
                t0 = time.perf_counter()
                p = subprocess.run(args, capture_output=True, text=True, timeout=900,
                                   env=dict(os.environ, LM_TIMING="1", **env))
                wall = time.perf_counter() - t0
                if p.returncode:
                    print(p.stdout[-2000:], p.stderr[-2000:], file=sys.stderr)
                    sys.exit(p.returncode)
                st = parse_timing(p.stdout)
                r = {"wall_s": round(wall, 3), "frames_per_s": round(n / wall, 1), "stages_ms": st,
                     "loop_frames_per_s": round(n / (st.get("loop_ms", 0) / 1e3), 1) if st.get("loop_ms") else None}
                if st.get("decode_ms"):
                    r["decode_frames_per_s"] = round(n / (st["decode_ms"] / 1e3), 1)
                if best is None or r["wall_s"] < best["wall_s"]:
                    best = r
            best["env"] = env
            runs[name] = best
            os.rename(yml, yml + "." + ("1dev" if not env else "4dev"))
        out["runs"] = runs
        if not a.no_check:
            t0 = time.perf_counter()
            ref = oracle_tracks(cfg, dec, threads)
            out["tracks_check"] = {m: check_tracks(yml + "." + ("1dev" if not e else "4dev"), ref)
                                   for m, e in modes.items()}
            out["tracks_check"]["seconds"] = round(time.perf_counter() - t0, 1)
    line = json.dumps(out)
    print(line)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as fh:
            fh.write(line + "\n")
    if not a.no_check and not all(v for k, v in out["tracks_check"].items() if k != "seconds"):
        sys.exit(1)


if __name__ == "__main__":
    main()
