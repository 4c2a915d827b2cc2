"""BASELINE config 1: a 100-frame synthetic 1024x256 grey AVI with the paw
template only — the plumbing case.  "Paw only" is a model whose snout and
tail detectors never fire (bias out of reach), so the reference's loop runs
all six filter2D calls but only the paw lists hold candidates.

CPU (the reference's own, GPU-less configuration): the video goes through the
native AVI reader and the oracle's per-frame path.  GPU: the same frames
through the HIP path must equal the oracle bit for bit, and the whole
`LocoMouse` program on the files must write the oracle's tracks."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import media_writers as MW  # noqa: E402
from locomouse_cpp_amd import synthetic as S  # noqa: E402

N = 100
SILENT = {"snout_bottom": 1e6, "snout_side": 1e6, "tail_bottom": 1e6, "tail_side": 1e6}


def c1_config():
    return S.SyntheticConfig(biases=SILENT)


def _check_paw_only(res, n):
    co = res["cand_offset"]
    paws = [int(co[4 * f + 1] - co[4 * f]) for f in range(n)]
    snouts = [int(co[4 * f + 2] - co[4 * f + 1]) + int(co[4 * f + 4] - co[4 * f + 3]) for f in range(n)]
    assert sum(paws) > 0 and max(snouts) == 0
    assert (res["tail"][:n] == -1).all()


def test_c1_cpu_path_on_the_avi(tmp_path):
    from oracle import oracle as O
    from test_cli import read_avi
    cfg = c1_config()
    frames = cfg.frames(0, N)
    p = tmp_path / "c1.avi"
    MW.write_avi(p, frames, bits=8)
    n, got = read_avi(p, max_frames=N)
    assert n == N and np.array_equal(got, frames)
    res = O.OracleRun(cfg, got).result
    _check_paw_only(res, N)


@pytest.mark.gpu
def test_c1_gpu_matches_oracle():
    from oracle import oracle as O
    from test_gpu_parity import _ctx, assert_same
    cfg = c1_config()
    frames = cfg.frames(0, N)
    ref = O.OracleRun(cfg, frames).result
    _check_paw_only(ref, N)
    from locomouse_cpp_amd.results import concat_results
    ctx = _ctx(cfg, max_batch=32)
    got = concat_results([ctx.detect(frames[i:i + 32], i) for i in range(0, N, 32)])
    ctx.close()
    assert_same(got, ref, "C1: ")


@pytest.mark.gpu
def test_c1_program_end_to_end(tmp_path):
    from oracle import oracle as O
    from oracle import track_oracle as TO
    from test_cli import cli_args, fs_node, run_cli
    cfg = c1_config()
    paths = MW.write_inputs(str(tmp_path), cfg, N, stem="c1_R", bits=8)
    rc, out = run_cli(cli_args(paths, outdir=str(tmp_path)), env={"LM_BATCH": "32"})
    assert rc == 0, out
    res = O.OracleRun(cfg, cfg.frames(0, N)).result
    p = cfg.params
    corner = [p.bounding_box_bottom.x + p.bounding_box_bottom.width,
              p.bounding_box_bottom.y + p.bounding_box_bottom.height,
              p.bounding_box_side.y + p.bounding_box_side.height]
    ref = TO.run_tracks(res, O.geometry(cfg), p, [corner] * N, N)
    yml = str(tmp_path / "output_c1_R.yml")
    for i in range(4):
        k, dt, m = fs_node(yml, f"paw_tracks{i}")
        assert np.array_equal(m.astype(np.int32), np.array(ref["paw_tracks"][i], np.int32))
    k, dt, m = fs_node(yml, "tracks_tail")
    assert (m == -1).all()
