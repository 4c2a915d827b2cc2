"""Generates the golden vectors in this directory from the CPU restatement
(oracle/lm_oracle.cpp) — run from the repo root:

    python tests/golden/make_golden.py

Each case stores the synthetic frames' CRC (pins the generator), per-detector
CRC32 of the fp32 score maps plus 64 sampled scores, and the full result
arrays of lm_batch_result.  The reference has no fixtures of its own
(SURVEY.md §4), so these pin the restatement against regressions; they are
not reference outputs ("parity unpinned")."""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from locomouse_cpp_amd import synthetic as S  # noqa: E402
from locomouse_cpp_amd.results import KEYS  # noqa: E402

CASES = {
    "default_f0_6": (dict(), 0, 6),
    "tm_method1_f40_4": (dict(method=1), 40, 4),
    "flip_conn4_f7_4": (dict(flip=True, connectivity=4), 7, 4),
}


def case_data(kw, first, n):
    from oracle import oracle as O
    cfg = S.SyntheticConfig(**kw)
    frames = cfg.frames(first, n)
    run = O.OracleRun(cfg, frames, flags=O.KEEP_DEBUG)
    out = {k: run.result[k] for k in KEYS}
    out["frames_crc"] = np.array([zlib.crc32(frames.tobytes())], np.uint32)
    crc = np.zeros((n, 6), np.uint32)
    samp = np.zeros((n, 6, 64), np.float32)
    out["sample_idx"] = np.random.default_rng(1234).integers(0, 2**31, (n, 6, 64))  # taken modulo the map size
    for f in range(n):
        for d in range(6):
            s = run.scores(f, d)
            if s is None:
                continue
            crc[f, d] = zlib.crc32(np.ascontiguousarray(s).tobytes())
            samp[f, d] = s.ravel()[out["sample_idx"][f, d] % s.size]
    out["score_crc"] = crc
    out["score_samples"] = samp
    return out


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    for name, (kw, first, n) in CASES.items():
        np.savez_compressed(os.path.join(here, name + ".npz"), **case_data(kw, first, n))
        print("wrote", name)


if __name__ == "__main__":
    main()
