"""Golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py):
the CPU restatement must keep reproducing them (CPU), and the HIP path must
match them bit for bit (GPU) without running the oracle."""
import os
import zlib

import numpy as np
import pytest

from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.results import KEYS

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = {
    "default_f0_6": (dict(), 0, 6),
    "tm_method1_f40_4": (dict(method=1), 40, 4),
    "flip_conn4_f7_4": (dict(flip=True, connectivity=4), 7, 4),
}


def _load(name):
    with np.load(os.path.join(HERE, name + ".npz")) as z:  # allow_pickle=False (default)
        return {k: z[k] for k in z.files}


def _assert_results(got, gold):
    for k in KEYS:
        a, b = got[k], gold[k]
        if a.dtype.names:
            assert a.shape == b.shape and all(np.array_equal(a[n], b[n]) for n in a.dtype.names), k
        else:
            assert a.shape == b.shape and np.array_equal(a, b), k


@pytest.mark.parametrize("name", sorted(CASES))
def test_generator_pinned(name):
    kw, first, n = CASES[name]
    frames = S.SyntheticConfig(**kw).frames(first, n)
    assert zlib.crc32(frames.tobytes()) == int(_load(name)["frames_crc"][0])


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_reproduces_golden(name):
    from oracle import oracle as O
    kw, first, n = CASES[name]
    gold = _load(name)
    cfg = S.SyntheticConfig(**kw)
    run = O.OracleRun(cfg, cfg.frames(first, n), flags=O.KEEP_DEBUG)
    _assert_results(run.result, gold)
    for f in range(n):
        for d in range(6):
            s = run.scores(f, d)
            if s is None:
                assert gold["score_crc"][f, d] == 0
                continue
            assert zlib.crc32(np.ascontiguousarray(s).tobytes()) == gold["score_crc"][f, d]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_hip_matches_golden(name):
    from locomouse_cpp_amd.runtime import Context
    kw, first, n = CASES[name]
    gold = _load(name)
    cfg = S.SyntheticConfig(**kw)
    frames = cfg.frames(first, n)
    ctx = Context(cfg, max_batch=8)
    ctx.set_debug(1)
    # the fixture's frame `first` is its run's frame 0 (no previous frame)
    got = ctx.detect(frames, 0)
    _assert_results(got, gold)
    for f in range(n):
        for d in range(6):
            if gold["score_crc"][f, d] == 0:
                continue
            s = ctx.debug_scores(f, d)
            assert zlib.crc32(np.ascontiguousarray(s).tobytes()) == gold["score_crc"][f, d], (f, d)
            assert np.array_equal(s.ravel()[gold["sample_idx"][f, d] % s.size], gold["score_samples"][f, d])
