"""GPU parity of the pipelined context (lm_setup.pipeline_lanes > 1,
lm_detect_submit / lm_detect_collect): several batches of one video in flight
on their own HIP streams, each continuing the previous one through the
device-side halo hand-off, must give exactly the oracle's per-frame loop
(main.cpp:54-82) on the whole video -- the same bar as one lane."""
import pytest

import edge_scenes as E
from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.results import concat_results, slice_results
from test_gpu_parity import _oracle, _quantized_config, assert_same

pytestmark = pytest.mark.gpu


def _pctx(cfg, lanes, max_batch):
    from locomouse_cpp_amd.runtime import Context
    return Context(cfg, max_batch=max_batch, lanes=lanes)


def _pipelined(ctx, frames, B, first=0):
    """Submit every batch of `frames` (keeping all lanes busy), collect in order."""
    parts, firsts = [], []
    lanes = ctx.lanes()
    for i in range(0, len(frames), B):
        if ctx.pending() == 2 * lanes:
            r = ctx.collect()
            firsts.append(r["first_frame"])
            parts.append(r)
        ctx.submit(frames[i:i + B], first + i)
    while ctx.pending():
        r = ctx.collect()
        firsts.append(r["first_frame"])
        parts.append(r)
    assert firsts == list(range(first, first + len(frames), B)), firsts
    return concat_results(parts)


@pytest.mark.parametrize("lanes,B", [(2, 5), (3, 4), (4, 6)])
def test_pipelined_video_matches_oracle(lanes, B):
    """23 frames (a ragged last batch) from frame 0 through 2-4 lanes."""
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, 23)
    ctx = _pctx(cfg, lanes, B)
    assert ctx.lanes() == lanes
    got = _pipelined(ctx, frames, B)
    assert_same(got, _oracle(cfg, frames).result, f"pipelined L{lanes} B{B}: ")


def test_pipelined_shard_start_and_moving_crops():
    """A shard starting at frame 40 with its previous frame as halo, per-frame
    crop corners, device frames read in place."""
    import torch
    cfg = S.SyntheticConfig()
    video = cfg.frames(39, 17)
    bb = E.moving_corners(cfg, 17, first=39)
    ref = slice_results(_oracle(cfg, video, bb=bb).result, 1)
    d = torch.from_numpy(video).to("cuda:0")
    fb = video.shape[1] * video.shape[2]
    ctx = _pctx(cfg, 3, 4)
    parts = []
    for j, i in enumerate(range(1, 17, 4)):
        if ctx.pending() == 3:
            parts.append(ctx.collect())
        n = min(4, 17 - i)
        ctx.submit_device(d.data_ptr() + i * fb, fb, n, 39 + i, d_prev_ptr=d.data_ptr() if j == 0 else None,
                          bb=bb[0:n + 1] if j == 0 else bb[i:i + n])
    while ctx.pending():
        parts.append(ctx.collect())
    torch.cuda.synchronize()
    assert_same(concat_results(parts), ref, "pipelined shard: ")


def test_pipelined_tie_heavy_and_blank_frames():
    """The exact-tie configuration (k_nms's std::sort replica) and the edge
    video's blank / half-blank frames across the lanes' seams."""
    c, dups = _quantized_config(1500)
    assert dups > 20
    frames = c.frames(200, 12)
    ref = _oracle(c, frames).result
    assert_same(_pipelined(_pctx(c, 4, 3), frames, 3), ref, "pipelined ties: ")
    cfg = S.SyntheticConfig()
    ev = E.edge_video(cfg)
    assert_same(_pipelined(_pctx(cfg, 2, 5), ev, 5), _oracle(cfg, ev).result, "pipelined edges: ")


def test_pipelined_errors_and_synchronous_mix():
    """At most 2 x lanes batches wait for collection (the lanes of finished
    batches are reused while their results wait); lm_detect_batch needs an
    empty pipeline; frame gaps are refused; a synchronous batch continues the
    pipelined ones."""
    from locomouse_cpp_amd.runtime import LMError
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, 24)
    ctx = _pctx(cfg, 2, 4)
    ctx.submit(frames[0:4], 0)
    with pytest.raises(LMError) as e:  # lm_detect_batch while a batch is in flight
        ctx.detect(frames[4:8], 4)
    assert e.value.code == 1
    for i in (4, 8, 12):  # four batches in flight on two lanes
        ctx.submit(frames[i:i + 4], i)
    assert ctx.pending() == 4
    with pytest.raises(LMError) as e:  # 2 x lanes waiting
        ctx.submit(frames[16:20], 16)
    assert e.value.code == 1
    parts = [ctx.collect()]
    with pytest.raises(LMError) as e:  # a gap in the frame sequence
        ctx.submit(frames[17:20], 17)
    assert e.value.code == 1
    ctx.submit(frames[16:20], 16)
    while ctx.pending():
        parts.append(ctx.collect())
    assert [p["first_frame"] for p in parts] == [0, 4, 8, 12, 16]
    # a synchronous batch continuing the pipelined ones (hand-off halo)
    parts.append(ctx.detect(frames[20:24], 20))
    assert_same(concat_results(parts), _oracle(cfg, frames).result, "mixed: ")
    with pytest.raises(LMError):
        ctx.collect()  # nothing in flight


def test_dropin_config_bench_scale():
    """The drop-in configuration the host mirror and INTEGRATION.md ship: one
    context x 4 pipeline lanes x B = 256, over 1,024 device frames (a shard
    start at frame 7000 with its halo), driven like bench.py --lanes 4
    --streams 1 (submit while lanes are busy, collect in order), against the
    oracle on the same frames (LocoMouse_class.cpp:771-1267)."""
    import torch
    from locomouse_cpp_amd.runtime import synth_frames_device
    cfg = S.SyntheticConfig()
    n, B, f0 = 1024, 256, 7000
    fb = 256 * 1024
    d = torch.empty((n + 1, 256, 1024), dtype=torch.uint8, device="cuda")
    synth_frames_device(d.data_ptr(), 256, 1024, f0 - 1, n + 1, fb)
    torch.cuda.synchronize()
    host = d.cpu().numpy()
    ctx = _pctx(cfg, 4, B)
    parts = []
    for j, i in enumerate(range(0, n, B)):
        if ctx.pending() == 8:
            parts.append(ctx.collect())
        ctx.submit_device(d.data_ptr() + (1 + i) * fb, fb, B, f0 + i, d_prev_ptr=d.data_ptr() if j == 0 else None)
    while ctx.pending():
        parts.append(ctx.collect())
    ctx.close()
    assert [p["first_frame"] for p in parts] == [f0 + i for i in range(0, n, B)]
    ref = slice_results(_oracle(cfg, host).result, 1)
    assert_same(concat_results(parts), ref, "1 ctx x 4 lanes x 256: ")


def test_debug_data_refused_after_lane_reuse():
    """Debug score maps / TAIL_MASK live on the lane that ran the batch: with
    2 x lanes batches submitted, the oldest batches were retired and their
    lanes reused, so asking for their maps must fail (not return another
    batch's data); the last batch's maps are still there and exact."""
    import numpy as np
    from locomouse_cpp_amd.runtime import LMError
    from oracle import oracle as O
    cfg = S.SyntheticConfig()
    frames = cfg.frames(0, 16)
    ctx = _pctx(cfg, 2, 4)
    ctx.set_debug(1)
    for i in range(0, 16, 4):
        ctx.submit(frames[i:i + 4], i)
    first = ctx.collect()
    assert first["first_frame"] == 0
    with pytest.raises(LMError) as e:
        ctx.debug_scores(0, 0)
    assert e.value.code == 1 and "newer batch" in str(e.value)
    with pytest.raises(LMError):
        ctx.debug_tail_mask(0)
    while ctx.pending():
        last = ctx.collect()
    assert last["first_frame"] == 12
    ref = O.OracleRun(cfg, frames, flags=O.KEEP_DEBUG)
    for det in range(6):
        got = ctx.debug_scores(2, det)
        exp = ref.scores(14, det, got.shape)
        assert np.array_equal(got.view(np.uint32), exp.view(np.uint32)), det
    g = ctx.geometry()
    assert np.array_equal(ctx.debug_tail_mask(2), ref.tail_mask(14, (g.bb_bottom_mouse.height, g.tail_box_width)))
    assert ctx.batch_slots() == 5  # handed-off halo frame recomputed in slot 0
    ctx.close()
