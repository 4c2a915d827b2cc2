"""Multi-context / multi-thread consistency check: NS contexts on one GPU,
each in its own thread over its own contiguous frame range; every batch's
result is compared with a single-context reference run of the same range."""
import os
import sys
import threading
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
from locomouse_cpp_amd import synthetic as S  # noqa: E402
from locomouse_cpp_amd.runtime import Context, synth_frames_device  # noqa: E402
from locomouse_cpp_amd.results import KEYS  # noqa: E402

NS, NB, B = int(sys.argv[1]), int(sys.argv[2]), 256
debug = int(sys.argv[3]) if len(sys.argv) > 3 else 2
R = NB * B
cfg = S.SyntheticConfig()
fr = torch.empty((NS, R + 1, 256, 1024), dtype=torch.uint8, device="cuda")
for k in range(NS):
    synth_frames_device(fr[k].data_ptr(), 256, 1024, k * R - 1, R + 1, 262144)
torch.cuda.synchronize()


def run(k, ctx, out):
    base = fr[k].data_ptr()
    for b in range(NB):
        f = k * R + b * B
        try:
            r = ctx.detect_device(base + (1 + b * B) * 262144, 262144, B, f,
                                  d_prev_ptr=base if (b == 0 and f > 0) else None, raw=False)
            out.append(r)
        except Exception as e:
            out.append(e)


# reference: each range alone, one thread
ref = []
for k in range(NS):
    c = Context(cfg, max_batch=B)
    o = []
    run(k, c, o)
    ref.append(o)
    c.close()
ctxs = [Context(cfg, max_batch=B) for _ in range(NS)]
for c in ctxs:
    c.set_debug(debug)
outs = [[] for _ in range(NS)]
th = [threading.Thread(target=run, args=(k, ctxs[k], outs[k])) for k in range(NS)]
for t in th:
    t.start()
for t in th:
    t.join()
bad = 0
for k in range(NS):
    for b in range(NB):
        a, r = outs[k][b], ref[k][b]
        if isinstance(a, Exception) or isinstance(r, Exception):
            print("stream", k, "batch", b, "mt:", repr(a)[:400] if isinstance(a, Exception) else "ok",
                  "ref:", repr(r)[:120] if isinstance(r, Exception) else "ok")
            bad += 1
            continue
        for key in KEYS:
            x, y = a[key], r[key]
            same = x.shape == y.shape and (all(np.array_equal(x[n], y[n]) for n in x.dtype.names) if x.dtype.names
                                           else np.array_equal(x, y))
            if not same:
                print("stream", k, "batch", b, "differs in", key)
                bad += 1
                break
print("NS", NS, "NB", NB, "debug", debug, "bad batches:", bad)
if bad and debug & 4:
    # print the differing candidate lists of the first mismatching batch
    for k in range(NS):
        for b in range(NB):
            a, r = outs[k][b], ref[k][b]
            if isinstance(a, Exception):
                continue
            if not np.array_equal(a["cand"]["y"], r["cand"]["y"]) or a["cand"].shape != r["cand"].shape:
                co_a, co_r = a["cand_offset"], r["cand_offset"]
                for fl in range(len(co_a) - 1):
                    xa = a["cand"][co_a[fl]:co_a[fl + 1]]
                    xr = r["cand"][co_r[fl]:co_r[fl + 1]]
                    if xa.shape != xr.shape or not all(np.array_equal(xa[m], xr[m]) for m in xa.dtype.names):
                        print("stream", k, "batch", b, "frame", k * R + b * B + fl // 4, "list", fl % 4,
                              "n", len(xa), len(xr))
                        idx = [i for i in range(min(len(xa), len(xr))) if tuple(xa[i]) != tuple(xr[i])]
                        print("   first diffs:", [(i, tuple(xa[i]), tuple(xr[i])) for i in idx[:5]])
