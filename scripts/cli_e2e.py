"""End-to-end rate of the LocoMouse program (file decode, host->device copies,
GPU detection, host tracker, YAML output) on a synthetic uncompressed AVI.
Inputs go to a scratch directory (not gpurun_out/).  Prints one JSON line.

Usage: python scripts/cli_e2e.py [n_frames] [bits]"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import media_writers as MW  # noqa: E402
from locomouse_cpp_amd import runtime  # noqa: E402
from locomouse_cpp_amd import synthetic as S  # noqa: E402


def main(n=2000, bits=8):
    cfg = S.SyntheticConfig()
    with tempfile.TemporaryDirectory() as d:
        t0 = time.perf_counter()
        paths = MW.write_inputs(d, cfg, n, stem="e2e_R", bits=bits)
        t_write = time.perf_counter() - t0
        args = [runtime.CLI_PATH, "0", paths["config"], paths["video"], paths["background"], paths["model"],
                paths["calibration"], "R", d]
        runs = []
        for _ in range(2):
            t0 = time.perf_counter()
            p = subprocess.run(args, capture_output=True, text=True, timeout=600, env=dict(os.environ, LM_TIMING="1"))
            runs.append(time.perf_counter() - t0)
            if p.returncode:
                print(p.stdout, p.stderr)
                sys.exit(p.returncode)
        size = os.path.getsize(paths["video"])
        stages = [line.split()[1:] for line in p.stdout.splitlines() if line.startswith("LM_TIMING")]
        stages = {k: float(v) for k, v in zip(stages[0][::2], stages[0][1::2])} if stages else {}
    best = min(runs)
    print(json.dumps({"what": "LocoMouse CLI end to end (uncompressed AVI -> output yml)", "frames": n, "bits": bits,
                      "video_bytes": size, "seconds": [round(r, 3) for r in runs],
                      "frames_per_s": round(n / best, 1), "last_run_stages_ms": stages, "input_write_s": round(t_write, 1),
                      "note": "includes process start, HIP init, file reads, H2D, detection, tracker, YAML"}))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
