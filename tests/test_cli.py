"""The `LocoMouse` command-line program and its file readers (SURVEY.md §8(f)
row 2): OpenCV FileStorage YAML (config, model, calibration, output), 8-bit
PNG background, uncompressed and MJPEG AVI video (tests/test_mjpeg.py); the reference's arguments, messages
and exit codes (main.cpp:38-105, LocoMouse_ParseInputs.cpp, LocoMouse_class.cpp:
12-540, :3095-3162).  The GPU test runs the whole program on synthetic files
and compares its output YAML with the oracle's detection + restated tracker.

Parity unpinned against OpenCV (absent here): files are produced by the
writers in tests/media_writers.py; byte-level parity of colour-PNG grey
conversion and of FileStorage's own output formatting is not verified."""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import host_harness as H  # noqa: E402
import media_writers as MW  # noqa: E402
from locomouse_cpp_amd import runtime  # noqa: E402
from locomouse_cpp_amd import synthetic as S  # noqa: E402

CLI = runtime.CLI_PATH


def read_png(path, cap=1 << 22):
    r, c = C.c_int(), C.c_int()
    out = np.zeros(cap, np.uint8)
    rc = H.lib().lmh_read_png(os.fsencode(path), C.byref(r), C.byref(c), out.ctypes.data, cap)
    if rc:
        return None
    return out[:r.value * c.value].reshape(r.value, c.value)


def read_avi(path, max_frames=16, rewind_at=-1):
    r, c, n = C.c_int(), C.c_int(), C.c_int()
    cap = max_frames * 1024 * 512
    out = np.zeros(cap, np.uint8)
    k = H.lib().lmh_read_avi(os.fsencode(path), C.byref(r), C.byref(c), C.byref(n), out.ctypes.data, cap, rewind_at)
    if k > 0:
        return None
    fb = r.value * c.value
    return n.value, out[:(-k) * fb].reshape(-k, r.value, c.value)


def fs_node(path, key, cap=1 << 20):
    kind, rows, cols = C.c_int(), C.c_int(), C.c_int()
    dt = C.c_char()
    out = np.zeros(cap)
    text = C.create_string_buffer(256)
    rc = H.lib().lmh_fs_node(os.fsencode(path), key.encode(), C.byref(kind), C.byref(rows), C.byref(cols),
                             C.byref(dt), out.ctypes.data, cap, text, 256)
    if rc:
        raise RuntimeError(f"fs_node rc={rc}: {text.value.decode()}")
    k = ["none", "int", "real", "str", "seq", "map", "mat"][kind.value]
    if k == "mat":
        return k, dt.value.decode(), out[:rows.value * cols.value].reshape(rows.value, cols.value)
    if k in ("int", "real"):
        return k, out[0], int(out[1])
    if k == "str":
        return k, text.value.decode()
    if k == "seq":
        return k, out[:rows.value].copy()
    return (k,)


def run_cli(args, env=None, timeout=300):
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run([CLI, *args], capture_output=True, text=True, env=e, timeout=timeout)
    return p.returncode, p.stdout


def cli_args(paths, method="0", side="R", outdir="."):
    return [method, paths["config"], paths["video"], paths["background"], paths["model"], paths["calibration"], side,
            outdir]


# ------------------------------------------------------------ readers (CPU)

def test_png_grey_all_filters(tmp_path):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(37, 53), dtype=np.uint8)
    p = tmp_path / "g.png"
    MW.write_png(p, img)
    assert np.array_equal(read_png(p), img)


def test_png_rgb_uses_libpng_rgb_to_gray_weights(tmp_path):
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, size=(20, 31, 3), dtype=np.uint8)
    img[0, :5] = 77  # grey pixels pass through unchanged
    p = tmp_path / "c.png"
    MW.write_png(p, img)
    r, g, b = (img[..., k].astype(np.uint32) for k in range(3))
    want = ((9797 * r + 19234 * g + 3737 * b) >> 15).astype(np.uint8)
    same = (r == g) & (r == b)
    want[same] = r[same]
    assert np.array_equal(read_png(p), want)


def test_png_rejects_non_png(tmp_path):
    p = tmp_path / "x.png"
    p.write_bytes(b"not a png")
    assert read_png(p) is None
    assert read_png(tmp_path / "missing.png") is None


@pytest.mark.parametrize("bits", [24, 8])
def test_avi_channel0_and_rewind(tmp_path, bits):
    rng = np.random.default_rng(bits)
    frames = rng.integers(0, 256, size=(5, 23, 37), dtype=np.uint8)  # odd width: padded rows
    p = tmp_path / "v.avi"
    MW.write_avi(p, frames, bits=bits)
    n, got = read_avi(p)
    assert n == 5 and np.array_equal(got, frames)
    n, got = read_avi(p, rewind_at=3)  # V.set(CV_CAP_PROP_POS_FRAMES, 0) after 3 frames
    assert np.array_equal(got, np.concatenate([frames[:3], frames]))


def test_avi_rejects_non_avi(tmp_path):
    p = tmp_path / "v.avi"
    p.write_bytes(b"RIFF\0\0\0\0WAVEfmt ")
    assert read_avi(p) is None


def test_file_storage_config_model_calibration(tmp_path):
    cfg = S.SyntheticConfig()
    paths = MW.write_inputs(str(tmp_path), cfg, 2)
    assert fs_node(paths["config"], "conn_comp_connectivity")[2] == 8
    k, v, _ = fs_node(paths["config"], "alpha_vel_bottom")
    assert k == "real" and v == cfg.params.alpha_vel_bottom
    k, dt, m = fs_node(paths["config"], "location_prior")
    assert k == "mat" and dt == "d" and m.shape == (5, 7) and m[1, 1] == cfg.params.location_prior[1].y
    k, dt, m = fs_node(paths["model"], "modelSnout_bottom")
    assert dt == "d" and np.array_equal(m, cfg.weights["snout_bottom"])  # repr() round trip is exact
    assert fs_node(paths["model"], "biasTail_side")[1] == cfg.biases["tail_side"]
    k, dt, m = fs_node(paths["calibration"], "ind_warp_mapping")
    assert dt == "i" and np.array_equal(m, cfg.calib)
    assert fs_node(paths["config"], "no_such_key") == ("none",)


def test_file_storage_yaml_forms(tmp_path):
    p = tmp_path / "f.yml"
    p.write_text("%YAML:1.0\n---\n# comment\nname: \"a # b\"\nplain: hello world\nhexv: 0x1F\nneg: -3.5e-2\n"
                 "inf: .Inf\nflow: [1, 2.5,\n   3]\nnested:\n   a: 1\n   b: [4, 5]\nblock:\n   - 7\n   - 8\n"
                 "m: !!opencv-matrix\n   rows: 2\n   cols: 2\n   dt: f\n   data: [ 1.5, -2., 3e1, 4 ]\n")
    assert fs_node(p, "name") == ("str", "a # b")
    assert fs_node(p, "plain") == ("str", "hello world")
    assert fs_node(p, "hexv")[2] == 31
    assert fs_node(p, "neg")[1] == -3.5e-2
    assert fs_node(p, "inf")[1] == np.inf
    k, seq = fs_node(p, "flow")
    assert k == "seq" and seq.tolist() == [1, 2.5, 3]
    assert fs_node(p, "nested") == ("map",)
    assert fs_node(p, "block")[1].tolist() == [7, 8]
    k, dt, m = fs_node(p, "m")
    assert dt == "f" and m.tolist() == [[1.5, -2.0], [30.0, 4.0]]
    bad = tmp_path / "bad.yml"
    bad.write_text("%YAML:1.0\nm: !!opencv-matrix\n   rows: 2\n   cols: 2\n   dt: i\n   data: [ 1, 2, 3 ]\n")
    with pytest.raises(RuntimeError, match="rows x cols"):
        fs_node(bad, "m")


def test_file_storage_writer_layout(tmp_path):
    """FsWriter follows OpenCV's YAML emitter (persistence_yml.cpp): header,
    3-space block indent, flow sequences wrapped past column 71 with the
    struct's indent, "%d." / "%.16e" reals, "-" lines for nested block
    entries, "[]" for empty collections; and our reader reads it back."""
    p = tmp_path / "w.yml"
    assert H.lib().lmh_fs_write_demo(os.fsencode(p)) == 0
    text = p.read_text()
    head = ("%YAML:1.0\n---\nN_opencv_matrices: 7\nM: !!opencv-matrix\n   rows: 2\n   cols: 3\n   dt: i\n"
            "   data: [ 1, -2, 3, 4, 5, 6 ]\nreal: 5.0000000000000000e-01\nwhole: 15.\n"
            "neg: -3.7500000000000000e-01\nBB:\n   x: 1\n   y: 2\nseq: [ 0, 1000,")
    assert text.startswith(head), text[:400]
    tail = ("nested:\n   -\n      -\n         Candidate_bottom:\n            Point_x: 3\n"
            "            Score: 2.5000000000000000e-01\n         side: [ 4 ]\n   -\n      []\n"
            "empty_flow: []\nlast: text\n")
    assert text.endswith(tail), text[-300:]
    seq = text[text.index("seq: ["):text.index("nested:")].splitlines()
    assert len(seq) > 2 and all(len(line) <= 73 for line in seq)  # margin 71, plus " " and ","
    assert all(line.startswith("    ") and line[4] != " " for line in seq[1:])
    assert all(line.endswith(",") for line in seq[:-1]) and seq[-1].endswith(" ]")
    k, vals = fs_node(p, "seq")
    assert k == "seq" and vals.tolist() == [1000 * k for k in range(40)]
    k, dt, m = fs_node(p, "M")
    assert dt == "i" and m.tolist() == [[1, -2, 3], [4, 5, 6]]
    assert fs_node(p, "neg")[1] == -0.375 and fs_node(p, "whole")[1] == 15.0
    assert fs_node(p, "last") == ("str", "text")
    assert fs_node(p, "nested")[0] == "seq"


# ------------------------------------------------------- CLI, no GPU needed

def test_cli_reads_every_input(tmp_path):
    cfg = S.SyntheticConfig()
    paths = MW.write_inputs(str(tmp_path), cfg, 3, stem="clip_L")
    rc, out = run_cli(cli_args(paths, method="1", side="L", outdir=str(tmp_path)), env={"LM_PRINT_INPUTS": "1"})
    assert rc == 0, out
    d = dict(line.split(" ", 1) for line in out.splitlines() if " " in line)
    assert d["method"] == "1" and d["flip"] == "1"
    assert d["video"] == f"{cfg.rows} {cfg.cols} 3" and d["calib"] == f"{cfg.rows} {cfg.cols}"
    assert d["output"] == str(tmp_path) + "/output_clip_L.yml"
    p = cfg.params
    assert d["bb_bottom"] == " ".join(str(v) for v in (p.bounding_box_bottom.x, p.bounding_box_bottom.y,
                                                      p.bounding_box_bottom.width, p.bounding_box_bottom.height))
    doubles = [float(v) for v in d["doubles"].split()]
    assert doubles == [p.side_bottom_min_overlap, p.occlusion_grid_max_width, p.tail_sub_bounding_box,
                       p.alpha_vel_bottom, p.alpha_vel_side, p.pairwise_occluded_cost]
    prior = [float(v) for v in d["prior"].split()]
    assert prior[7:14] == [p.location_prior[1].x, p.location_prior[1].y, p.location_prior[1].max_distance,
                           p.location_prior[1].min_x, p.location_prior[1].max_x, p.location_prior[1].min_y,
                           p.location_prior[1].max_y]
    dets = [line.split()[1:] for line in out.splitlines() if line.startswith("detector")]
    order = ["paw_bottom", "paw_side", "snout_bottom", "snout_side", "tail_bottom", "tail_side"]
    for name, (r, c, b, s) in zip(order, dets):
        w = cfg.weights[name]
        assert (int(r), int(c)) == w.shape and float(b) == cfg.biases[name]
    assert int(d["background_sum"]) == int(cfg.background.astype(np.int64).sum())


@pytest.mark.parametrize("case", ["calibration", "connectivity", "median", "prior", "flip", "method", "video",
                                  "background", "size", "args", "devices_twice", "devices_text"])
def test_cli_errors_match_the_reference(tmp_path, case):
    cfg = S.SyntheticConfig()
    paths = MW.write_inputs(str(tmp_path), cfg, 2)
    args = cli_args(paths, outdir=str(tmp_path))
    want = None
    if case == "calibration":
        args[5] = str(tmp_path / "none.yml")
        want = "Invalid inputs: Error: Could not open the calibration file: " + args[5] + "."
    elif case == "connectivity":
        MW.write_config(paths["config"], cfg, overrides={"conn_comp_connectivity": 6})
        want = "Invalid inputs: Invalid configuration parameter: conn_comp_connectivity must be either 4 or 8. Was 6."
    elif case == "median":
        MW.write_config(paths["config"], cfg, overrides={"median_filter_size": 10})
        want = "Invalid inputs: Invalid configuration parameter: median_filter_size must be odd. Was 10."
    elif case == "prior":
        text = open(paths["config"]).read().replace("rows: 5", "rows: 4").replace("cols: 7", "cols: 7")
        text = text.replace("data: [ 0.25", "data: [ 0.25", 1)
        lines = text.split("location_prior")[0]
        open(paths["config"], "w").write(lines)  # no location_prior at all -> empty 0x0 matrix
        want = "Invalid inputs: Invalid configuration parameter: location_prior must be a 5x7 matrix. Was 0."
    elif case == "flip":
        args[6] = "X"
        want = 'Invalid inputs: Mouse side option must be either "L" or "R".'
    elif case == "method":
        args[0] = "zero"
        want = "Invalid inputs: stoi"
    elif case == "video":
        args[2] = str(tmp_path / "none.avi")
        want = "Invalid inputs: Could not open the video file: " + args[2] + "."
    elif case == "background":
        args[3] = str(tmp_path / "none.png")
        want = "Invalid inputs: Could not open the background image: " + args[3] + "."
    elif case == "size":
        MW.write_png(paths["background"], cfg.background[:, :-1])
        want = "Runtime Error: Error: Background image does not match video size."
    elif case == "args":
        args = args[:3]
        want = "Invalid inputs: Error: Could not open the calibration file: "
    env = None
    if case == "devices_twice":  # LocoMouse_Inputs::devices: refused before any device is touched
        env = {"LM_DEVICES": "0,1,0"}
        want = "Invalid inputs: LocoMouse: a device is listed twice"
    elif case == "devices_text":
        env = {"LM_DEVICES": "0,gpu1"}
        want = "Invalid inputs: LM_DEVICES: not a device index: gpu1"
    rc, out = run_cli(args, env=env)
    assert rc == 1, out
    assert want in out, out
    assert "Total Elapsed time:" in out
    if case == "args":
        assert out.startswith("Warning: Invalid input list.")


# ------------------------------------------------------------- GPU: full run

MULTI_DEVICE_ENV = {"LM_DEVICES": "0,0,0,0", "LM_OVERSUBSCRIBE": "1"}  # 4 "devices" on the one GPU


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["R24", "L8", "RJ", "R24-4dev"])
def test_cli_end_to_end_matches_oracle(tmp_path, variant):
    """The whole program on synthetic files: its output YAML holds the
    oracle's tracks (oracle detection on the same frames + the restated
    tracker).  "RJ": an MJPEG video (4:2:0 colour JPEG frames), the oracle
    fed Pillow's decoding of the same frames.  "-4dev": LM_DEVICES with four
    entries (one GPU, oversubscribed): shards of 7 frames dealt to four
    device threads, each with its halo frame."""
    from oracle import oracle as O
    from oracle import track_oracle as TO
    flip = variant.startswith("L")
    n = 40
    cfg = S.SyntheticConfig(flip=flip)
    stem = "mouse_" + variant[0]
    jpeg = dict(mode="RGB", quality=92, subsampling=2) if variant.endswith("J") else None
    multi = variant.endswith("-4dev")
    bits = 24 if jpeg else int(variant[1:].split("-")[0])
    paths = MW.write_inputs(str(tmp_path), cfg, n, stem=stem, bits=bits, jpeg=jpeg)
    env = dict(MULTI_DEVICE_ENV, LM_BATCH="7") if multi else {"LM_BATCH": "16"}
    rc, out = run_cli(cli_args(paths, side=variant[0], outdir=str(tmp_path)), env=env)
    assert rc == 0, out
    res = O.OracleRun(cfg, paths["decoded"] if jpeg else cfg.frames(0, n)).result
    p = cfg.params
    corner = [p.bounding_box_bottom.x + p.bounding_box_bottom.width,
              p.bounding_box_bottom.y + p.bounding_box_bottom.height,
              p.bounding_box_side.y + p.bounding_box_side.height]
    bb = [corner] * n
    ref = TO.run_tracks(res, O.geometry(cfg), p, bb, n)
    yml = str(tmp_path / f"output_{stem}.yml")
    for i in range(4):
        k, dt, m = fs_node(yml, f"paw_tracks{i}")
        assert dt == "i" and np.array_equal(m.astype(np.int32), np.array(ref["paw_tracks"][i], np.int32))
    k, dt, m = fs_node(yml, "snout_tracks0")
    assert np.array_equal(m.astype(np.int32), np.array(ref["snout_tracks"][0], np.int32))
    k, dt, m = fs_node(yml, "tracks_tail")
    assert np.array_equal(m.astype(np.int32), np.array(ref["tracks_tail"], np.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("multi", [False, True])
def test_cli_timing_split(tmp_path, multi):
    """LM_TIMING=1 (not in the reference): the program prints one LM_TIMING
    line with its wall split (scripts/cli_e2e_mjpeg.py reads it for the
    10,000-frame MJPEG run).  On a 40-frame MJPEG video in 16-frame batches
    (or 7-frame shards over four "devices"): every field present and >= 0,
    the decode inside the frame loop, every frame counted, the batches
    handed over, and the output YAML written as without the variable."""
    n = 40
    cfg = S.SyntheticConfig()
    paths = MW.write_inputs(str(tmp_path), cfg, n, stem="mouse_R", bits=24,
                            jpeg=dict(mode="RGB", quality=92, subsampling=2))
    env = dict(MULTI_DEVICE_ENV, LM_BATCH="7", LM_TIMING="1") if multi else {"LM_BATCH": "16", "LM_TIMING": "1"}
    rc, out = run_cli(cli_args(paths, side="R", outdir=str(tmp_path)), env=env)
    assert rc == 0, out
    lines = [ln for ln in out.splitlines() if ln.startswith("LM_TIMING ")]
    assert len(lines) == 1, out
    f = lines[0].split()[1:]
    t = {k: float(v) for k, v in zip(f[::2], f[1::2])}
    keys = ("init_ms", "loop_ms", "tracks_ms", "export_ms", "decode_ms", "decode_threads", "submit_ms", "wait_ms",
            "batches", "frames")
    assert set(keys) <= set(t), t
    assert all(t[k] >= 0 for k in keys), t
    assert t["frames"] == n and t["decode_threads"] >= 1
    assert t["batches"] == (6 if multi else 3), t  # ceil(40 / 7) shards, ceil(40 / 16) batches
    assert t["decode_ms"] <= t["loop_ms"] + 1e-6, t
    assert os.path.exists(tmp_path / "output_mouse_R.yml")


def _load_cv_yaml(path):
    """An independent reader for the FileStorage YAML (PyYAML, safe loader with
    a constructor for !!opencv-matrix)."""
    import yaml

    class Loader(yaml.SafeLoader):
        pass

    def mat(loader, node):
        m = loader.construct_mapping(node, deep=True)
        return np.array(m["data"]).reshape(m["rows"], m["cols"])

    Loader.add_constructor("tag:yaml.org,2002:opencv-matrix", mat)
    text = open(path).read().replace("%YAML:1.0", "", 1)
    return yaml.load(text, Loader=Loader)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [1, 4])
def test_cli_verbose_debug_outputs(tmp_path, devices):
    """verbose_debug: 1 with N_debug_frames: 30 of a 40-frame video — the run
    stops after 30 frames (loadVideo :380-389), and debug_<stem>.yml holds
    exportDebugVariables' content (:2769-2920) equal to the oracle's
    containers and tracks; debug_<stem>.txt logs each frame's stages.
    devices=4: the same through LM_DEVICES (four device threads on the one
    GPU, 6-frame shards): every container of the debug YAML still equals the
    oracle's."""
    import re

    from oracle import oracle as O
    from oracle import track_oracle as TO
    n, nd = 40, 30
    cfg = S.SyntheticConfig()
    stem = "dbg_R"
    paths = MW.write_inputs(str(tmp_path), cfg, n, stem=stem,
                            config_overrides={"verbose_debug": 1, "N_debug_frames": nd})
    env = dict(MULTI_DEVICE_ENV, LM_BATCH="6") if devices > 1 else {"LM_BATCH": "16"}
    rc, out = run_cli(cli_args(paths, outdir=str(tmp_path)), env=env)
    assert rc == 0, out
    res = O.OracleRun(cfg, cfg.frames(0, nd)).result
    p = cfg.params
    corner = [p.bounding_box_bottom.x + p.bounding_box_bottom.width,
              p.bounding_box_bottom.y + p.bounding_box_bottom.height,
              p.bounding_box_side.y + p.bounding_box_side.height]
    geom = O.geometry(cfg)
    ref = TO.run_tracks(res, geom, p, [corner] * nd, nd)
    k, dt, m = fs_node(str(tmp_path / f"output_{stem}.yml"), "paw_tracks0")
    assert np.array_equal(m.astype(np.int32), np.array(ref["paw_tracks"][0], np.int32))

    d = _load_cv_yaml(tmp_path / f"debug_{stem}.yml")
    assert d["N_opencv_matrices"] == 7 and d["N_frames"] == nd
    assert np.array_equal(d["M_paw_bottom"], np.array(ref["track_index_paw_bottom"]))
    assert np.array_equal(d["M_snout_bottom"], np.array(ref["track_index_snout_bottom"]))
    for i in range(4):
        assert d[f"M_paw_side_{i}"].ravel().tolist() == list(ref["track_index_paw_side"][i])
    assert d["M_snout_side_0"].ravel().tolist() == list(ref["track_index_snout_side"][0])
    assert d["occluded_distance"] == p.max_displacement_bottom
    assert d["BB_bottom"] == {"x": 0, "y": 0, "width": p.bounding_box_bottom.width,
                              "height": p.bounding_box_bottom.height}
    assert d["bb_x_avg"] == [corner[0]] * nd and d["bb_yb_avg"] == [corner[1]] * nd
    assert d["bb_yt_avg"] == [corner[2]] * nd
    ong = d["ONG"]
    assert ong["points"] == geom.ong_nx * geom.ong_ny == len(ong["x_y_coordinates"]) // 2
    assert ong["x_y_coordinates"][:2] == [geom.ong_br_x, geom.ong_br_y]
    assert d["ONG_side"]["z_coordinates"][0] == geom.ong_side_lowest
    for feat, key in ((0, "candidates_paw_bottom_side_matched"), (1, "candidates_snout_bottom_side_matched")):
        ml = TO.matched_list(res, feat)
        assert len(d[key]) == nd
        for f in range(nd):
            got = d[key][f] or []
            assert len(got) == len(ml[f])
            for e, (x, y, ys, ss) in zip(got, ml[f]):
                assert (e["Candidate_bottom"]["Point_x"], e["Candidate_bottom"]["Point_y"]) == (x, y)
                assert e["n_candidates_side"] == len(e["Candidates_side"])
                if e["Scores_side"][0] >= 0:
                    assert e["Candidates_side"] == ys and e["Scores_side"] == ss
                else:
                    assert ys == []
    for feat, key in ((0, "Unary_paws"), (1, "Unary_snout")):
        assert len(d[key]) == nd
        for f in range(nd):
            lo, hi = int(res["unary_offset"][2 * f + feat]), int(res["unary_offset"][2 * f + feat + 1])
            u = d[key][f]
            assert u["n_rows"] * u["n_cols"] == hi - lo and u["n_cols"] == (4 if feat == 0 else 1)
            assert (u["data"] or []) == [float(v) for v in res["unary"][lo:hi]]  # %.16e round-trips
    for feat, key in ((0, "Pairwise_paws"), (1, "Pairwise_snout")):
        assert len(d[key]) == nd - 1
        for f in range(1, nd):
            q = 2 * f + feat
            lo, hi = int(res["pw_nz_offset"][q]), int(res["pw_nz_offset"][q + 1])
            e = d[key][f - 1]
            assert (e["data"] or []) == [float(v) for v in res["pw_pr"][lo:hi]]
            assert (e["row_index"] or []) == [int(v) for v in res["pw_ir"][lo:hi]]

    txt = (tmp_path / f"debug_{stem}.txt").read_text()
    counts = [int(c) for c in re.findall(r"Detected (\d+) paw candidates\.", txt)]
    want = [int(res["cand_offset"][4 * f + 1] - res["cand_offset"][4 * f]) for f in range(nd)]
    assert counts == want
    assert txt.count("=== readFrame: ") == nd and "=== exportResults: " in txt
    assert "--- exportDebugVariables() " in txt and txt.rstrip().endswith("=== Done")
