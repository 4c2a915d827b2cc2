"""GPU parity: the HIP path (through the C-ABI) against the CPU restatement
oracle on the same synthetic frames.  Integer/index outputs must be
bit-identical; scores are compared bit-exactly too (the HIP correlation uses
the same fmaf chain as the oracle) and, separately, within 1e-5 relative of
the float64 cross-check in test_oracle.py.
"""
import numpy as np
import pytest

from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.abi import frame_views
from locomouse_cpp_amd.results import KEYS, concat_results

pytestmark = pytest.mark.gpu


def _ctx(cfg, max_batch=16):
    from locomouse_cpp_amd.runtime import Context
    return Context(cfg, max_batch=max_batch)


def _oracle(cfg, frames, flags=0, bb=None):
    from oracle import oracle as O
    return O.OracleRun(cfg, frames, bb=bb, flags=flags)


def assert_same(got, ref, label=""):
    for k in KEYS:
        a, b = got[k], ref[k]
        if a.dtype.names:
            ok = a.shape == b.shape and all(np.array_equal(a[n], b[n]) for n in a.dtype.names)
        else:
            ok = a.shape == b.shape and np.array_equal(a, b)
        if not ok:
            # locate the first differing frame for a readable message
            n = ref["n_frames"]
            for f in range(n):
                vg, vr = frame_views(got, f), frame_views(ref, f)
                for lk in range(4):
                    if not (len(vg["cand"][lk]) == len(vr["cand"][lk]) and
                            all(np.array_equal(vg["cand"][lk][x], vr["cand"][lk][x]) for x in ("x", "y", "score"))):
                        raise AssertionError(f"{label}{k}: frame {f} list {lk}\n gpu {vg['cand'][lk]}\n ref {vr['cand'][lk]}")
                if not np.array_equal(vg["tail"], vr["tail"]):
                    raise AssertionError(f"{label}{k}: frame {f} tail\n gpu {vg['tail']}\n ref {vr['tail']}")
                for fk in range(2):
                    if vg["p22d"][fk] != vr["p22d"][fk]:
                        raise AssertionError(f"{label}{k}: frame {f} p22d {fk}\n gpu {vg['p22d'][fk]}\n ref {vr['p22d'][fk]}")
                    if not np.array_equal(vg["unary"][fk], vr["unary"][fk]):
                        raise AssertionError(f"{label}{k}: frame {f} unary {fk}\n gpu {vg['unary'][fk]}\n ref {vr['unary'][fk]}")
                    pg, pr = vg["pairwise"][fk], vr["pairwise"][fk]
                    if (pg is None) != (pr is None) or (pg is not None and not all(
                            np.array_equal(pg[x], pr[x]) for x in ("jc", "ir", "pr")) or (pg and pg["n_rows"] != pr["n_rows"])):
                        raise AssertionError(f"{label}{k}: frame {f} pairwise {fk}\n gpu {pg}\n ref {pr}")
            raise AssertionError(f"{label}{k} differs: {a[:8]} vs {b[:8]}")


@pytest.fixture(scope="module")
def cfg():
    return S.SyntheticConfig()


def test_raw_scores_bit_exact(cfg):
    frames = cfg.frames(0, 3)
    ctx = _ctx(cfg)
    ctx.set_debug(1)
    ctx.detect(frames, 0)
    from oracle import oracle as O
    ref = _oracle(cfg, frames, flags=O.KEEP_DEBUG)
    g = ctx.geometry()
    for f in range(3):
        for det in range(6):
            got = ctx.debug_scores(f, det)
            exp = ref.scores(f, det, got.shape)
            assert exp is not None
            assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), (f, det, np.abs(got - exp).max())
        assert np.array_equal(ctx.debug_tail_mask(f), ref.tail_mask(f, (g.bb_bottom_mouse.height, g.tail_box_width)))


def test_geometry_matches_oracle(cfg):
    from oracle import oracle as O
    assert _ctx(cfg).geometry().as_dict() == O.geometry(cfg).as_dict()


def test_full_path_one_batch(cfg):
    frames = cfg.frames(0, 12)
    got = _ctx(cfg).detect(frames, 0)
    ref = _oracle(cfg, frames).result
    assert_same(got, ref)


def test_batches_carry_state(cfg):
    frames = cfg.frames(0, 12)
    ctx = _ctx(cfg, max_batch=5)
    parts = [ctx.detect(frames[i:i + 5], i) for i in range(0, 12, 5)]
    assert_same(concat_results(parts), _oracle(cfg, frames).result, "carry: ")


def test_shard_with_halo_frame(cfg):
    frames = cfg.frames(0, 12)
    ref = _oracle(cfg, frames).result
    ctx = _ctx(cfg, max_batch=8)
    a = _ctx(cfg, max_batch=8).detect(frames[:6], 0)
    b = ctx.detect(frames[6:], 6, prev_frame=frames[5])
    assert_same(concat_results([a, b]), ref, "halo: ")


@pytest.mark.parametrize("kw", [{"method": 1}, {"method": 2}, {"flip": True}, {"connectivity": 4}])
def test_variants(kw):
    c = S.SyntheticConfig(**kw)
    frames = c.frames(20, 6)
    assert_same(_ctx(c).detect(frames, 0), _oracle(c, frames).result, f"{kw}: ")


def test_device_frames_api(cfg):
    torch = pytest.importorskip("torch")
    frames = cfg.frames(30, 6)
    d = torch.from_numpy(frames).cuda()
    torch.cuda.synchronize()
    from locomouse_cpp_amd.abi import result_to_numpy
    ctx = _ctx(cfg)
    got = result_to_numpy(ctx.detect_device(d.data_ptr(), frames.shape[1] * frames.shape[2], 6, 0))
    assert_same(got, _oracle(cfg, frames).result, "device: ")


def test_device_frames_unaligned(cfg):
    """Device frames at an odd address and pitch (staged by a D2D copy), plus
    an unaligned halo frame."""
    torch = pytest.importorskip("torch")
    frames = cfg.frames(40, 7)
    npix = frames.shape[1] * frames.shape[2]
    pitch = npix + 5
    buf = torch.zeros(3 + pitch * 7, dtype=torch.uint8, device="cuda:0")
    for i in range(7):
        buf[3 + i * pitch: 3 + i * pitch + npix] = torch.from_numpy(frames[i].reshape(-1)).cuda()
    torch.cuda.synchronize()
    from locomouse_cpp_amd.abi import result_to_numpy
    ctx = _ctx(cfg)
    base = buf.data_ptr() + 3
    got = result_to_numpy(ctx.detect_device(base + pitch, pitch, 6, 41, d_prev_ptr=base))  # frame 40 as halo
    from locomouse_cpp_amd.results import slice_results
    assert_same(got, slice_results(_oracle(cfg, frames).result, 1), "unaligned device: ")


def test_error_mapping(cfg):
    from locomouse_cpp_amd.runtime import LMError
    with pytest.raises(LMError) as e:
        _ctx(S.SyntheticConfig(connectivity=5))
    assert e.value.code == 1
    ctx = _ctx(cfg)
    with pytest.raises(LMError) as e:
        ctx.detect(cfg.frames(3, 2), 3)  # frame 2 never seen and no halo
    assert e.value.code == 1
    for option in ("use_reference_image_brightness", "transform_gray_values"):  # §8(f) row 4, as executed
        bad = S.SyntheticConfig()
        setattr(bad.params, option, 1)
        bad.params.gray_value_transformation_depth = 5  # a CV_32F table (the CV_8U one works: test_gpu_edges.py)
        with pytest.raises(LMError) as e:
            _ctx(bad)
        assert e.value.code == 2


def _quantized_config(rank, side_rank=None):
    """Detector weights on a 2^-12 grid, so the fp32 correlation is exact and
    equal-sum windows tie exactly; biases put ~`rank` pixels above zero
    (`side_rank` for the side detectors when given)."""
    from oracle import oracle as O
    base = S.SyntheticConfig()
    W = {}
    for name in ("paw_bottom", "snout_bottom", "paw_side", "snout_side"):
        w = base.weights[name]
        W[name] = np.round(w * w.size * 4) / 4 / 1024
    c0 = S.SyntheticConfig(weights=W, biases={n: 0.0 for n in W})
    r0 = O.OracleRun(c0, c0.frames(0, 1), flags=O.KEEP_DEBUG)
    biases, dups = {}, 0
    for det, name in ((0, "paw_bottom"), (1, "snout_bottom"), (3, "paw_side"), (4, "snout_side")):
        rk = side_rank if (side_rank is not None and det >= 3) else rank
        v = np.sort(r0.scores(0, det).ravel())[::-1]
        biases[name] = float(v[rk])
        pos = v[v > v[rk]]
        dups += len(pos) - len(np.unique(pos))
    return S.SyntheticConfig(weights=W, biases=biases), dups


@pytest.mark.parametrize("rank", [400, 1500])
def test_nms_exact_score_ties(rank):
    """Exact ties take the std::sort replica path (lm_introsort.h); 1500
    positives also exercise the bitonic (> LM_NMS_RANKSORT) branch."""
    c, dups = _quantized_config(rank)
    assert dups > 20  # the case really has ties
    frames = c.frames(0, 6)
    assert_same(_ctx(c).detect(frames, 0), _oracle(c, frames).result, "ties: ")


def test_nms_large_lists_global_path():
    """> LM_NMS_CAP positives per list: NMS runs from global scratch."""
    c, dups = _quantized_config(5000)
    assert dups > 1000
    frames = c.frames(0, 4)
    assert_same(_ctx(c).detect(frames, 0), _oracle(c, frames).result, "large: ")


def test_c5_highres_geometry_bit_exact():
    """Config C5: 1920x512 frames, geometry and detectors x2 (widths 44-60:
    the wide width-specialised correlation kernels)."""
    c5 = S.SyntheticConfig(rows=512, cols=1920)
    frames = c5.frames(0, 4)
    ctx = _ctx(c5, max_batch=4)
    ctx.set_debug(1)
    got = ctx.detect(frames, 0)
    from oracle import oracle as O
    ref = _oracle(c5, frames, flags=O.KEEP_DEBUG)
    assert_same(got, ref.result, "C5: ")
    for det in range(6):
        s = ctx.debug_scores(3, det)
        assert np.array_equal(s.view(np.uint32), ref.scores(3, det, s.shape).view(np.uint32)), det
    ctx.close()


def test_c5_carry_and_halo():
    c5 = S.SyntheticConfig(rows=512, cols=1920)
    frames = c5.frames(37, 7)
    ref = _oracle(c5, frames).result
    ctx = _ctx(c5, max_batch=4)
    a = ctx.detect(frames[:3], 0)
    b = ctx.detect(frames[3:], 3)
    assert_same(concat_results([a, b]), ref, "C5 carry: ")
    ctx.close()


def test_long_stream_device_frames():
    """1024 consecutive frames (a shard start at frame 5000, halo frame 4999)
    in batches of 256 from device memory, against the oracle run on the same
    frames: the C3 path at bench batch size."""
    torch = pytest.importorskip("torch")
    from locomouse_cpp_amd.abi import result_to_numpy
    from locomouse_cpp_amd.results import slice_results
    from locomouse_cpp_amd.runtime import synth_frames_device
    from oracle import oracle as O
    cfg = S.SyntheticConfig()
    n, B, f0 = 1024, 256, 5000
    d = torch.empty((n + 1, 256, 1024), dtype=torch.uint8, device="cuda")
    synth_frames_device(d.data_ptr(), 256, 1024, f0 - 1, n + 1, 262144)
    torch.cuda.synchronize()
    host = d.cpu().numpy()
    ctx = _ctx(cfg, max_batch=B)
    parts = []
    for b in range(0, n, B):
        r = ctx.detect_device(d.data_ptr() + (1 + b) * 262144, 262144, B, f0 + b,
                              d_prev_ptr=d.data_ptr() if b == 0 else None)
        parts.append(result_to_numpy(r))
    ctx.close()
    ref = slice_results(O.OracleRun(cfg, host).result, 1)
    assert_same(concat_results(parts), ref, "long: ")


@pytest.mark.parametrize("rank", [900, 1500])
def test_nms_long_lists_across_batches(rank):
    """Lists of 900 / 1,500 positives (k_nms's rank sort / bitonic sort in
    LDS, ties through the std::sort replica) over three batches of one
    context, bit-exact against the oracle over the seams."""
    c, dups = _quantized_config(rank)
    assert dups > 20
    frames = c.frames(0, 9)
    ctx = _ctx(c, max_batch=3)
    parts = [ctx.detect(frames[i:i + 3], i) for i in range(0, 9, 3)]
    ctx.close()
    assert_same(concat_results(parts), _oracle(c, frames).result, f"nms cap rank {rank}: ")


def test_global_tier_few_overflowing_pairs():
    """A few (frame, feature) pairs of a batch with lists beyond the LDS
    capacity, the rest short (blank frames): every block of the global-scratch
    tier must walk the same pair list in the same order (an atomics-built list
    differed between blocks, so some pairs were never processed)."""
    c, dups = _quantized_config(2500)  # lists beyond k_nms's LDS capacity (LM_NMS_CAP)
    frames = c.frames(0, 12)
    frames[[1, 2, 4, 5, 7, 9, 10]] = 0
    ref = _oracle(c, frames).result
    for _ in range(3):
        ctx = _ctx(c, max_batch=12)
        got = ctx.detect(frames, 0)
        ctx.close()
        assert_same(got, ref, "few overflowing pairs: ")


def test_side_global_tier_bottom_lds_tier():
    """Side lists beyond LM_NMS_CAP (global-scratch k_nms) with short bottom
    lists (LDS k_nms): the side skip (detectSideCandidates runs only for a
    non-empty bottom list, :820-833) must not read bottom keys the bottom
    block has already overwritten with its staged candidates -- k_tail
    records the decision before k_nms runs.  Blank frames make some bottom
    lists empty, so both outcomes of the skip occur."""
    c, dups = _quantized_config(300, side_rank=2500)
    frames = c.frames(0, 10)
    frames[[2, 6]] = 0
    ref = _oracle(c, frames).result
    ctx = _ctx(c, max_batch=10)
    got = ctx.detect(frames, 0)
    ctx.close()
    assert_same(got, ref, "mixed tiers: ")
