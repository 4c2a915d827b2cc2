"""Debug aid (not a test): one 256-frame batch from frame 5000 on the GPU vs
the oracle; prints the first mismatching frames with the GPU and oracle
candidate counts per list and the oracle's positive-score counts."""
import sys

import numpy as np

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import torch  # noqa: E402

from locomouse_cpp_amd import synthetic as S  # noqa: E402
from locomouse_cpp_amd.abi import frame_views, result_to_numpy  # noqa: E402
from locomouse_cpp_amd.results import slice_results  # noqa: E402
from locomouse_cpp_amd.runtime import Context, synth_frames_device  # noqa: E402
from oracle import oracle as O  # noqa: E402

cfg = S.SyntheticConfig()
n, B, f0 = 256, 256, 5000
d = torch.empty((n + 1, 256, 1024), dtype=torch.uint8, device="cuda")
synth_frames_device(d.data_ptr(), 256, 1024, f0 - 1, n + 1, 262144)
torch.cuda.synchronize()
host = d.cpu().numpy()
ctx = Context(cfg, max_batch=B)
got = result_to_numpy(ctx.detect_device(d.data_ptr() + 262144, 262144, B, f0, d_prev_ptr=d.data_ptr()))
ref_run = O.OracleRun(cfg, host, flags=O.KEEP_DEBUG)
ref = slice_results(ref_run.result, 1)
bad = 0
for f in range(n):
    vg, vr = frame_views(got, f), frame_views(ref, f)
    cg = [len(x) for x in vg["cand"]]
    cr = [len(x) for x in vr["cand"]]
    same = cg == cr and all(np.array_equal(vg["cand"][k], vr["cand"][k]) for k in range(4))
    if not same:
        pos = [int((ref_run.scores(f + 1, det) > 0).sum()) for det in (0, 1, 3, 4)]
        print(f"frame {f}: gpu counts {cg} oracle {cr} oracle positives(raw) {pos}")
        bad += 1
        if bad > 12:
            break
print("mismatching frames:", bad)
