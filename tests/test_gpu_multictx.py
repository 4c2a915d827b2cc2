"""Several contexts on one GPU driven from several host threads (one HIP
stream each, bench.py --streams): every batch must equal the same range run
alone.  The contexts share no state: each has its own non-blocking stream,
device buffers and result arenas, and nothing on a context's path uses the
legacy stream (create/debug copies are stream-ordered), so graph capture on
one stream never meets another context's work."""
import threading

import numpy as np
import pytest

from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.results import KEYS

pytestmark = pytest.mark.gpu


def _run(ctx, frames_dev, k, R, NB, B, out):
    base = frames_dev[k].data_ptr()
    for b in range(NB):
        f = k * R + b * B
        try:
            out.append(ctx.detect_device(base + (1 + b * B) * 262144, 262144, B, f,
                                         d_prev_ptr=base if (b == 0 and f > 0) else None, raw=False))
        except Exception as e:  # compared below
            out.append(e)


def test_threads_and_contexts_are_independent():
    torch = pytest.importorskip("torch")
    from locomouse_cpp_amd.runtime import Context, synth_frames_device
    NS, NB, B = 3, 12, 128
    R = NB * B
    cfg = S.SyntheticConfig()
    fr = torch.empty((NS, R + 1, 256, 1024), dtype=torch.uint8, device="cuda")
    for k in range(NS):
        synth_frames_device(fr[k].data_ptr(), 256, 1024, k * R - 1, R + 1, 262144)
    torch.cuda.synchronize()
    ref = []
    for k in range(NS):
        o = []
        c = Context(cfg, max_batch=B)
        _run(c, fr, k, R, NB, B, o)
        c.close()
        ref.append(o)
    ctxs = [Context(cfg, max_batch=B) for _ in range(NS)]
    outs = [[] for _ in range(NS)]
    th = [threading.Thread(target=_run, args=(ctxs[k], fr, k, R, NB, B, outs[k])) for k in range(NS)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k in range(NS):
        for b in range(NB):
            a, r = outs[k][b], ref[k][b]
            assert not isinstance(r, Exception), r
            assert not isinstance(a, Exception), a
            for key in KEYS:
                x, y = a[key], r[key]
                if x.dtype.names:
                    assert x.shape == y.shape and all(np.array_equal(x[n], y[n]) for n in x.dtype.names), (k, b, key)
                else:
                    assert np.array_equal(x, y), (k, b, key)
    for c in ctxs:
        c.close()

