"""Single-context run over a video range (device frames, halo start) to
localise a failing batch; compares the failing batch with the oracle."""
import sys
import os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from locomouse_cpp_amd import synthetic as S  # noqa: E402
from locomouse_cpp_amd.runtime import Context, synth_frames_device, LMError  # noqa: E402

start, nb, B = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 256
cfg = S.SyntheticConfig()
n = nb * B
fr = torch.empty((n + 1, 256, 1024), dtype=torch.uint8, device="cuda")
synth_frames_device(fr.data_ptr(), 256, 1024, start - 1, n + 1, 262144)
torch.cuda.synchronize()
ctx = Context(cfg, max_batch=B)
for b in range(nb):
    f = start + b * B
    try:
        ctx.detect_device(fr.data_ptr() + (1 + b * B) * 262144, 262144, B, f,
                          d_prev_ptr=fr.data_ptr() if (b == 0 and start > 0) else None)
    except LMError as e:
        print("batch", b, "frames", f, f + B - 1, "error:", e)
        host = fr[b * B: b * B + B + 1].cpu().numpy()
        from oracle import oracle as O
        try:
            O.OracleRun(cfg, host)
            print("oracle: no error on the same frames (halo + batch)")
        except Exception as e2:
            print("oracle error too:", e2)
        # which frame? rerun smaller pieces on GPU
        for k in range(1, B + 1):
            c2 = Context(cfg, max_batch=2)
            try:
                c2.detect(host[k - 1:k + 1][1:], f + k - 1, prev_frame=host[k - 1])
            except LMError as e3:
                print("  frame", f + k - 1, "fails alone:", e3)
                break
        break
else:
    print("no error in", start, start + n)
