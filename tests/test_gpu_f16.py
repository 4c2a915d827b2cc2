"""LM_CORR_F16, the NON-PARITY half-precision correlation mode of BASELINE
config 5 ("fp16 correlation accumulators"): f16 weights
(per-detector power-of-two scaled), exact u8 pixels, fp32 accumulation on
v_mfma_f32_32x32x16_f16 (lm_corr.hip k_corr_f16).

Pinned exactly where f16 cannot differ: detectors on a 2^-12 grid with 3-bit
numerators are exact in f16 and every partial sum is exact in fp32, so the
f16 mode must reproduce the oracle bit for bit — which pins the banded
(Toeplitz) formulation, the MFMA lane maps, tiling and epilogue.  On the
real-valued synthetic detectors the mode is compared with the fp32 path:
candidate (x, y) agreement is measured and printed (a non-parity mode has
no bit-exact claim), with a floor on it."""
import numpy as np
import pytest

from locomouse_cpp_amd import abi
from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.runtime import Context, LMError

pytestmark = pytest.mark.gpu


def _quantized_config(rows, cols, rank=400):
    """Every detector on a 2^-12 grid (numerators -4..4: exact in f16 after any
    power-of-two scaling); point-detector biases at the rank-th oracle score
    so a few hundred pixels per list score > 0 (tails: a few thousand)."""
    from oracle import oracle as O
    base = S.SyntheticConfig(rows=rows, cols=cols)
    W = {name: np.round(w * w.size * 4) / 4 / 1024 for name, w in base.weights.items()}
    c0 = S.SyntheticConfig(rows=rows, cols=cols, weights=W, biases={n: 0.0 for n in W})
    r0 = O.OracleRun(c0, c0.frames(0, 1), flags=O.KEEP_DEBUG)
    biases = {}
    for det, name in ((0, "paw_bottom"), (1, "snout_bottom"), (3, "paw_side"), (4, "snout_side")):
        v = np.sort(r0.scores(0, det).ravel())[::-1]
        biases[name] = float(v[rank])
    for det, name in ((2, "tail_bottom"), (5, "tail_side")):
        v = np.sort(r0.scores(0, det).ravel())[::-1]
        biases[name] = float(v[8 * rank])
    return S.SyntheticConfig(rows=rows, cols=cols, weights=W, biases=biases)


def _f16(cfg):
    cfg.setup.corr_precision = abi.LM_CORR_F16
    return cfg


@pytest.mark.parametrize("shape", [(256, 1024), (512, 1920)])
def test_f16_exact_on_f16_representable_detectors(shape):
    from oracle import oracle as O
    from test_gpu_parity import assert_same
    cfg = _quantized_config(*shape)
    frames = cfg.frames(0, 6)
    ref = O.OracleRun(cfg, frames).result
    assert int(ref["cand_offset"][-1]) > 0
    got = Context(_f16(cfg), max_batch=8).detect(frames, 0)
    assert_same(got, ref, f"f16 exact {shape}: ")


def _cands(res, f, k):
    lo, hi = int(res["cand_offset"][4 * f + k]), int(res["cand_offset"][4 * f + k + 1])
    return [(int(c["x"]), int(c["y"])) for c in res["cand"][lo:hi]]


@pytest.mark.parametrize("shape,n", [((256, 1024), 32), ((512, 1920), 16)])
def test_f16_candidate_agreement_with_fp32(shape, n):
    cfg = S.SyntheticConfig(rows=shape[0], cols=shape[1])
    frames = cfg.frames(0, n)
    ref = Context(cfg, max_batch=n).detect(frames, 0)
    cfg16 = _f16(S.SyntheticConfig(rows=shape[0], cols=shape[1]))
    got = Context(cfg16, max_batch=n).detect(frames, 0)
    same = total = 0
    for f in range(n):
        for k in range(4):
            a, b = _cands(ref, f, k), _cands(got, f, k)
            total += max(len(a), len(b))
            same += len(set(a) & set(b))
    tail_same = float(np.mean(ref["tail"][:n] == got["tail"][:n]))
    print(f"\nf16 vs fp32 {shape}: candidate (x,y) agreement {same}/{total} = {same / max(total, 1):.4f}, "
          f"tail points equal {tail_same:.4f}")
    assert total > 0 and same / total >= 0.97
    assert tail_same >= 0.97


def test_f16_rejects_oversized_detectors():
    big = np.zeros((40, 200))
    big[20, 100] = 1e-3
    cfg = _f16(S.SyntheticConfig(weights={"paw_bottom": big}))
    with pytest.raises(LMError, match="too large for the f16"):
        Context(cfg, max_batch=4)
