"""GPU parity on the reference's edge paths (tests/edge_scenes.py): the HIP
path through the C-ABI against the oracle, bit for bit, on blank and
half-blank frames across batch seams, zero-positive lists, dense and
checkerboard tail maps (k_tail's global run tables), detectors of sizes the
width-specialised kernels do not cover, the unfused filter2D arithmetic, the
CV_8U grey-level LUT, and three contexts on a tie-heavy configuration."""
import threading

import numpy as np
import pytest

import edge_scenes as E
from locomouse_cpp_amd import abi
from locomouse_cpp_amd import runtime as rt
from locomouse_cpp_amd import synthetic as S
from locomouse_cpp_amd.results import concat_results
from test_gpu_parity import _ctx, _oracle, _quantized_config, assert_same

pytestmark = pytest.mark.gpu


def _batched(cfg, frames, B, bb=None):
    ctx = _ctx(cfg, max_batch=B)
    parts = []
    for i in range(0, len(frames), B):
        parts.append(ctx.detect(frames[i:i + B], i, bb=None if bb is None else bb[i:i + B]))
    ctx.close()
    return concat_results(parts)


@pytest.mark.parametrize("B", [5, 14])
def test_blank_and_half_blank_frames(B):
    """Blank frames mid-batch and on both sides of a batch seam (B = 5),
    bottom-blank frames (side lists skipped, :820-833) and a side-blank frame
    (zero side positives, P22D without side candidates)."""
    cfg = S.SyntheticConfig()
    frames = E.edge_video(cfg)
    assert_same(_batched(cfg, frames, B), _oracle(cfg, frames).result, f"edges B{B}: ")


def test_half_blank_shard_start():
    """A shard that starts right after a blank frame (halo = the blank frame)
    and one whose halo frame has an empty bottom list."""
    cfg = S.SyntheticConfig()
    frames = E.edge_video(cfg)
    ref = _oracle(cfg, frames).result
    from locomouse_cpp_amd.results import slice_results
    for start in (6, 8):
        got = _ctx(cfg, max_batch=8).detect(frames[start:], start, prev_frame=frames[start - 1])
        assert_same(got, slice_results(ref, start), f"halo {start}: ")


@pytest.mark.parametrize("names", [("snout_bottom",), ("paw_side", "snout_side"), ("paw_bottom", "snout_bottom"),
                                   ("paw_bottom", "snout_bottom", "paw_side", "snout_side", "tail_bottom",
                                    "tail_side")])
def test_detectors_without_positives(names):
    cfg = E.silent_config(names)
    frames = cfg.frames(3, 9)
    assert_same(_batched(cfg, frames, 4), _oracle(cfg, frames).result, f"silent {names}: ")


def test_dense_tail_map():
    """Every tail score positive: one component filling the tail box (far
    beyond round 1's 6,144-pixel LDS limit), TAIL_MASK over the whole box."""
    cfg = E.dense_tail_config()
    frames = cfg.frames(0, 6)
    ctx = _ctx(cfg, max_batch=6)
    ctx.set_debug(1)
    got = ctx.detect(frames, 0)
    from oracle import oracle as O
    ref = _oracle(cfg, frames, flags=O.KEEP_DEBUG)
    assert_same(got, ref.result, "dense tail: ")
    g = ctx.geometry()
    for f in range(6):
        m = ctx.debug_tail_mask(f)
        assert np.array_equal(m, ref.tail_mask(f, (g.bb_bottom_mouse.height, g.tail_box_width)))
        assert m.all()


@pytest.mark.parametrize("conn", [8, 4])
def test_checkerboard_tail_maps(conn):
    """1x1 tail detectors over checkerboard frames: ~120 runs per tail row
    (more than k_tail keeps in LDS, so the run tables go to global memory);
    8-connectivity joins the diagonal cells into one component, with
    4-connectivity every cell is its own component and the first OpenCV label
    wins the area tie."""
    cfg = E.pixel_tail_config(conn)
    frames = E.checker_frames(cfg, 4)
    assert_same(_batched(cfg, frames, 4), _oracle(cfg, frames).result, f"checker c{conn}: ")


def test_detector_sizes_beyond_specialised_kernels():
    """70x70, 13x13 and 9x33 detectors (generic correlation kernel, row
    chunks); raw score maps bit-exact too."""
    cfg = E.odd_size_config()
    frames = cfg.frames(0, 4)
    ctx = _ctx(cfg, max_batch=4)
    ctx.set_debug(1)
    got = ctx.detect(frames, 0)
    from oracle import oracle as O
    ref = _oracle(cfg, frames, flags=O.KEEP_DEBUG)
    assert_same(got, ref.result, "odd sizes: ")
    for f in range(4):
        for det in range(6):
            s = ctx.debug_scores(f, det)
            assert np.array_equal(s.view(np.uint32), ref.scores(f, det, s.shape).view(np.uint32)), (f, det)


@pytest.mark.parametrize("plan", [0, 1])
@pytest.mark.parametrize("unfused", [False, True])
def test_wide_ring_widths(plan, unfused):
    """Ring widths 36-64 (40x40, 20x64, 16x36, 16x48 detectors) through the
    per-width launches (plan 0) and the single merged launch (plan 1), fused
    and unfused arithmetic: candidates and raw score maps bit-exact."""
    cfg = E.wide_ring_config()
    if unfused:
        cfg.setup.filter_arith = abi.LM_FILTER_UNFUSED
    frames = cfg.frames(10, 5)
    ctx = _ctx(cfg, max_batch=5)
    ctx.set_debug(1 | (abi.LM_DEBUG_PLAN_MERGED if plan else abi.LM_DEBUG_PLAN_PER_WIDTH))
    got = ctx.detect(frames, 10, prev_frame=cfg.frames(9, 1)[0])
    from oracle import oracle as O
    ref = _oracle(cfg, cfg.frames(9, 6), flags=O.KEEP_DEBUG)
    from locomouse_cpp_amd.results import slice_results
    assert_same(got, slice_results(ref.result, 1), f"wide ring plan {plan} unfused {unfused}: ")
    assert int(got["cand_offset"][-1]) > 0
    for f in range(5):
        for det in range(6):
            s = ctx.debug_scores(f, det)
            assert np.array_equal(s.view(np.uint32), ref.scores(f + 1, det, s.shape).view(np.uint32)), (f, det)


def _bright_tiles(cfg, frames):
    """Bright output tiles of the library's dark-tile grid (40 x 4) of the
    point detectors (some I_*_MOUSE
    pixel > 25 after readFrame's subtract + NORM_MINMAX, :1304-1310) and the
    outputs they hold, per view, summed over frames (identity calibration,
    provided boxes, no flip: the mouse crop ends at the box's bottom-right
    corner x + width, y + height (getBoundingBox :547-557, cropBoundingBox
    :1422-1423), one pixel right of and below the box rectangle)."""
    tw, th = rt.Context.dark_tile_shape()
    bk = cfg.background.astype(np.int32)
    p = cfg.params
    tiles, outs = [0, 0], [0, 0]
    for fr in frames:
        d = np.clip(fr.astype(np.int32) - bk, 0, 255)
        mn, mx = int(d.min()), int(d.max())
        scale = 255.0 / (mx - mn) if mx - mn > 2.220446049250313e-16 else 0.0
        shift = -mn * scale
        t = d.astype(np.float32) * np.float32(scale) + np.float32(shift)
        n = np.clip(np.rint(t), 0, 255)
        for v, r in enumerate((p.bounding_box_bottom, p.bounding_box_side)):
            crop = n[r.y + 1:r.y + 1 + r.height, r.x + 1:r.x + 1 + r.width] > 25
            for ty in range(0, r.height, th):
                for tx in range(0, r.width, tw):
                    blk = crop[ty:ty + th, tx:tx + tw]
                    if blk.any():
                        tiles[v] += 1
                        outs[v] += blk.size
    return tiles, outs


@pytest.mark.parametrize("plan", [0, 1])
def test_dark_tiles(plan, monkeypatch):
    """The point detectors' dark output tiles (no mouse pixel > 25: the
    reference zeroes all their scores, setTo(0, mask) :849, :864) are not
    computed: results identical to the oracle with the skip on and off, on
    the default scene and with blank frames (every tile dark), per-width and
    merged launches; the bright-tile counts equal a numpy count."""
    cfg = S.SyntheticConfig()
    frames = np.concatenate([cfg.frames(30, 3), np.zeros_like(cfg.frames(0, 1)), cfg.frames(34, 3)])
    ref = _oracle(cfg, frames).result
    for dark in ("1", "0"):
        monkeypatch.setenv("LM_CORR_DARK", dark)
        ctx = _ctx(cfg, max_batch=len(frames))
        ctx.set_debug(2 | (abi.LM_DEBUG_PLAN_MERGED if plan else abi.LM_DEBUG_PLAN_PER_WIDTH))
        got = ctx.detect(frames, 0)
        work = ctx.corr_work()
        ctx.close()
        assert_same(got, ref, f"dark={dark} plan {plan}: ")
        if dark == "1":
            tiles, outs = _bright_tiles(cfg, frames)
            assert work == {"tiles": tuple(tiles), "outputs": tuple(outs)}, (work, tiles, outs)
            assert tiles[0] < 360 * len(frames) and tiles[1] < 240 * len(frames)
        else:
            assert work is None


def test_dark_tiles_c5():
    """C5 (1920x512, detectors x2, bench batch shape per frame): dark-tile
    skipping against the oracle, and the executed-work counts the bench's
    roofline uses (lm_debug_corr_work) equal the numpy count of bright 40 x 4
    tiles and their outputs."""
    c5 = S.SyntheticConfig(rows=512, cols=1920)
    frames = np.concatenate([c5.frames(10, 2), np.zeros_like(c5.frames(0, 1)), c5.frames(13, 2)])
    ref = _oracle(c5, frames).result
    ctx = _ctx(c5, max_batch=len(frames))
    ctx.set_debug(2)
    got = ctx.detect(frames, 0)
    work = ctx.corr_work()
    slots = ctx.batch_slots()
    ctx.close()
    assert_same(got, ref, "C5 dark tiles: ")
    tiles, outs = _bright_tiles(c5, frames)
    assert work == {"tiles": tuple(tiles), "outputs": tuple(outs)}, (work, tiles, outs)
    assert slots == len(frames)  # a batch from frame 0 has no halo slot
    assert 0 < tiles[0] < 1400 * len(frames)


def test_dark_tiles_batch_over_512():
    """A batch of more than 512 frames: k_ingest's 65 slot groups share the 64
    list-segment counters of a view (segment c holds groups y0(c) .. y0(c+1)-1,
    lm_tl_y0), so some segments gather two groups' bright tiles; the
    correlation's segment lookup must find every one.  Against the oracle,
    with the work counts equal to the numpy count."""
    cfg = S.SyntheticConfig()
    frames = np.concatenate([cfg.frames(200, 260), np.zeros_like(cfg.frames(0, 1)), cfg.frames(461, 259)])
    ref = _oracle(cfg, frames).result
    ctx = _ctx(cfg, max_batch=len(frames))
    ctx.set_debug(2)
    got = ctx.detect(frames, 0)
    work = ctx.corr_work()
    ctx.close()
    assert_same(got, ref, "520-frame batch: ")
    tiles, outs = _bright_tiles(cfg, frames)
    assert work == {"tiles": tuple(tiles), "outputs": tuple(outs)}, (work, tiles, outs)


@pytest.mark.parametrize("c5", [False, True])
def test_dense_occlusion_grid(c5):
    """occlusion_grid_spacing_pixels_bottom = 5: 60 x 28 = 1,680 ONG nodes on
    the C3 box (k_post's LDS columns while the previous frame has few
    candidates), 120 x 56 = 6,720 on the C5 box (global-scratch k_post for
    every block); pairwise CSC bit-exact (pairwisePotential :1954-2070, grid
    :726-749)."""
    cfg = S.SyntheticConfig(rows=512, cols=1920) if c5 else S.SyntheticConfig()
    cfg.params.occlusion_grid_spacing_pixels_bottom = 5
    frames = cfg.frames(20, 4 if c5 else 7)
    ctx = _ctx(cfg, max_batch=3)
    g = ctx.geometry()
    assert g.ong_nx * g.ong_ny == (6720 if c5 else 1680)
    ctx.close()
    ref = _oracle(cfg, frames).result
    assert int(ref["pw_jc_offset"][-1]) > 1680 * 2
    assert_same(_batched(cfg, frames, 3), ref, f"ONG spacing 5 c5={c5}: ")


def test_tail_box_beyond_lds():
    """A 2000 x 700 tail box (k_tail on its global workspace) with a
    2,625-node occlusion grid, against the oracle."""
    cfg = E.big_tail_config()
    frames = cfg.frames(0, 4)
    ref = _oracle(cfg, frames).result
    assert (ref["tail"][:, 0] >= 0).any()
    assert_same(_batched(cfg, frames, 2), ref, "big tail box: ")


def test_unfused_filter_arithmetic():
    """LM_FILTER_UNFUSED (OpenCV's SSE2/scalar filter2D: rounded product,
    rounded sum) against the oracle's unfused restatement, bit for bit; its
    raw scores differ from the fused ones somewhere."""
    cfg = S.SyntheticConfig()
    cfg.setup.filter_arith = abi.LM_FILTER_UNFUSED
    frames = cfg.frames(0, 6)
    ctx = _ctx(cfg, max_batch=3)
    ctx.set_debug(1)
    parts = [ctx.detect(frames[:3], 0)]
    s_unf = ctx.debug_scores(1, 1).copy()
    parts.append(ctx.detect(frames[3:], 3))
    from oracle import oracle as O
    ref = _oracle(cfg, frames, flags=O.KEEP_DEBUG)
    assert_same(concat_results(parts), ref.result, "unfused: ")
    assert np.array_equal(s_unf.view(np.uint32), ref.scores(1, 1, s_unf.shape).view(np.uint32))
    fused = _oracle(S.SyntheticConfig(), frames[:2], flags=O.KEEP_DEBUG)
    assert not np.array_equal(s_unf.view(np.uint32), fused.scores(1, 1, s_unf.shape).view(np.uint32))


@pytest.mark.parametrize("moving", [False, True])
def test_gray_value_transformation_u8(moving):
    """transform_gray_values with a CV_8U table: LUT applied in place to the
    bottom crop (:1445-1448); later masks, the tail, and the next frame's
    motion test see the transformed pixels.  With moving crops the previous
    frame's transformed rectangle differs from the current one."""
    cfg = E.gray_lut_config()
    frames = cfg.frames(30, 10)
    bb = E.moving_corners(cfg, 10) if moving else None
    ref = _oracle(cfg, frames, bb=bb).result
    assert_same(_batched(cfg, frames, 4, bb=bb), ref, f"gray u8 moving={moving}: ")
    plain = _oracle(S.SyntheticConfig(), frames, bb=bb).result
    assert not np.array_equal(ref["cand"]["score"], plain["cand"]["score"]) if len(ref["cand"]) == len(plain["cand"]) \
        else True


def test_gray_value_transformation_side_overlap():
    """A side box low enough that its padded crop covers rows of the bottom
    crop: the side detectors read transformed pixels there."""
    cfg = E.gray_lut_config(bounding_boxes={"side": (300, 20, 400, 90), "bottom": (300, 106, 400, 140)})
    frames = cfg.frames(50, 6)
    assert_same(_batched(cfg, frames, 3), _oracle(cfg, frames).result, "gray overlap: ")


def test_gray_value_transformation_errors():
    from locomouse_cpp_amd.runtime import LMError
    cfg = E.gray_lut_config(depth=abi.LM_DEPTH_32F)
    with pytest.raises(LMError) as e:
        _ctx(cfg)
    assert e.value.code == 2  # the reference stops (cv::Exception / runtime_error)
    cfg = E.gray_lut_config()
    ctx = _ctx(cfg, max_batch=2)
    bb = E.moving_corners(cfg, 2)
    bb[:, 0] = 200  # bottom crop x in [-199, 200]: leaves the corrected image
    with pytest.raises(LMError) as e:
        ctx.detect(cfg.frames(0, 2), 0, bb=bb)
    assert e.value.code == 1


def test_three_contexts_tie_heavy_against_oracle():
    """Three contexts in three host threads on the exact-tie configuration
    (k_nms's std::sort replica path, whose missing barrier caused round 1's
    intermittent garbage candidates), each compared with the oracle."""
    c, dups = _quantized_config(1500)
    assert dups > 20
    frames = [c.frames(100 * k, 8) for k in range(3)]
    refs = [_oracle(c, fr).result for fr in frames]
    outs = [None] * 3

    def run(k):
        ctx = _ctx(c, max_batch=4)
        try:
            outs[k] = concat_results([ctx.detect(frames[k][i:i + 4], i) for i in (0, 4)])
        except Exception as e:  # reported below
            outs[k] = e
        ctx.close()
    th = [threading.Thread(target=run, args=(k,)) for k in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for k in range(3):
        assert not isinstance(outs[k], Exception), outs[k]
        assert_same(outs[k], refs[k], f"ctx {k}: ")


def test_long_candidate_lists_take_the_global_paths():
    """4x4 mean-filter paw detectors with a low threshold: ~2,000 bottom and
    ~5,800 side paw candidates per frame after clustering.  k_nms sorts and
    clusters from global scratch (> LM_NMS_CAP positives), and k_post builds
    the pairwise costs (~4M transitions) and the side matching from global
    scratch (> LM_POST_MAXC candidates; the reference has no limit)."""
    w = np.ones((4, 4)) / 16
    cfg = S.SyntheticConfig(weights={"paw_bottom": w, "paw_side": w}, biases={"paw_bottom": 60.5, "paw_side": 60.5})
    frames = cfg.frames(0, 4)
    ref = _oracle(cfg, frames).result
    co = ref["cand_offset"]
    assert min(int(co[4 * f + 1] - co[4 * f]) for f in range(4)) > 1500
    assert_same(_batched(cfg, frames, 3), ref, "long lists: ")


@pytest.mark.parametrize("plan", [0, 1])
def test_one_row_detectors_at_ring_widths(plan):
    """1 x 24 and 1 x 30 detectors: ring-kernel widths, but one row, so they
    must run k_corr_gen (the ring's two-step-ahead loop needs kh >= 2) in the
    per-width and the merged plans alike, beside ring detectors of the same
    widths (the ring kernel was picked by width alone)."""
    w = {"paw_side": S.dog_detector(1, 24, 4.0, 61), "tail_side": S.line_detector(1, 30, 0.5, 62),
         "snout_bottom": S.dog_detector(30, 30, 5.0, 12)}
    base = S.SyntheticConfig(weights=w)
    cfg = S.SyntheticConfig(weights=w, biases=E._bias_for_rate(base, ["paw_side", "snout_bottom"]))
    frames = cfg.frames(0, 4)
    ctx = _ctx(cfg, max_batch=4)
    ctx.set_debug(1 | (abi.LM_DEBUG_PLAN_MERGED if plan else abi.LM_DEBUG_PLAN_PER_WIDTH))
    got = ctx.detect(frames, 0)
    from oracle import oracle as O
    ref = _oracle(cfg, frames, flags=O.KEEP_DEBUG)
    assert_same(got, ref.result, f"one-row plan {plan}: ")
    for f in range(4):
        for det in range(6):
            s = ctx.debug_scores(f, det)
            assert np.array_equal(s.view(np.uint32), ref.scores(f, det, s.shape).view(np.uint32)), (f, det)
    ctx.close()


@pytest.mark.parametrize("quantized", [True, False])
@pytest.mark.parametrize("rank", [600, 750, 900])
def test_nms_lists_of_513_to_768_keys(quantized, rank):
    """Bottom and side lists of 513..768 kept keys: k_nms's tie pre-hash
    table (next power of two >= 2n) would be 2,048 entries, past its
    1,536-int LDS array, so such lists must skip the pre-hash;
    with and without exact score ties.  `rank`: positive scores of frame 0
    before the brightness and tail masks, so the kept lists land in or just
    below the range."""
    if quantized:
        c, _ = _quantized_config(rank)
    else:
        from oracle import oracle as O
        base = S.SyntheticConfig()
        c0 = S.SyntheticConfig(biases={n: 0.0 for n in S.DETECTOR_SPECS})
        r0 = O.OracleRun(c0, c0.frames(0, 1), flags=O.KEEP_DEBUG)
        b = dict(base.biases)
        for det, name in ((0, "paw_bottom"), (1, "snout_bottom"), (3, "paw_side"), (4, "snout_side")):
            b[name] = float(np.sort(r0.scores(0, det).ravel())[::-1][rank])
        c = S.SyntheticConfig(biases=b)
    frames = c.frames(0, 6)
    got = _ctx(c, max_batch=6).detect(frames, 0)
    assert_same(got, _oracle(c, frames).result, f"nms 513..768 rank {rank} q {quantized}: ")
