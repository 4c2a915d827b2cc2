"""Single-context run over a video range (device frames, halo start) to
localise a failing batch; with --check every batch is compared with the
oracle run on (halo frame + batch) on the host."""
import argparse
import os
import sys
import time
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from locomouse_cpp_amd import synthetic as S  # noqa: E402
from locomouse_cpp_amd.results import KEYS, slice_results  # noqa: E402
from locomouse_cpp_amd.runtime import Context, synth_frames_device, LMError  # noqa: E402
from oracle import oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("start", type=int)
ap.add_argument("nb", type=int)
ap.add_argument("B", type=int, nargs="?", default=256)
ap.add_argument("--check", action="store_true")
a = ap.parse_args()
start, nb, B = a.start, a.nb, a.B
cfg = S.SyntheticConfig()
n = nb * B
fr = torch.empty((n + 1, 256, 1024), dtype=torch.uint8, device="cuda")
synth_frames_device(fr.data_ptr(), 256, 1024, start - 1, n + 1, 262144)
torch.cuda.synchronize()
ctx = Context(cfg, max_batch=B)
bad = 0
t0 = time.time()
for b in range(nb):
    f = start + b * B
    try:
        got = ctx.detect_device(fr.data_ptr() + (1 + b * B) * 262144, 262144, B, f,
                                d_prev_ptr=fr.data_ptr() if (b == 0 and start > 0) else None, raw=False)
    except LMError as e:
        print("batch", b, "frames", f, f + B - 1, "error:", e, flush=True)
        host = fr[b * B: b * B + B + 1].cpu().numpy()
        try:
            O.OracleRun(cfg, host)
            print("oracle: no error on the same frames (halo + batch)")
        except Exception as e2:
            print("oracle error too:", e2)
        for k in range(1, B + 1):
            c2 = Context(cfg, max_batch=2)
            try:
                c2.detect(host[k:k + 1], f + k - 1, prev_frame=host[k - 1])
            except LMError as e3:
                print("  frame", f + k - 1, "fails alone:", e3)
                break
        sys.exit(1)
    if a.check:
        host = fr[b * B: b * B + B + 1].cpu().numpy()
        ref = slice_results(O.OracleRun(cfg, host).result, 1) if f > 0 else O.OracleRun(cfg, host[1:]).result
        diff = []
        for k in KEYS:
            x, y = got[k], ref[k]
            same = x.shape == y.shape and (all(np.array_equal(x[m], y[m]) for m in x.dtype.names) if x.dtype.names
                                           else np.array_equal(x, y))
            if not same:
                diff.append(k)
        if diff:
            bad += 1
            print("batch", b, "frames", f, f + B - 1, "differs from the oracle in", diff, flush=True)
    if b % 8 == 7:
        print(f"  {b + 1}/{nb} batches, {time.time() - t0:.0f} s", flush=True)
print("done", start, start + n, "mismatching batches:", bad)
sys.exit(1 if bad else 0)
