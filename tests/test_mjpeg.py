"""MJPEG AVI input: the native
sequential-JPEG decoder behind AviReader (locomouse_cpp_amd/host/Jpeg.cpp)
against libjpeg-turbo as Pillow links it, frame for frame and byte for byte.

The reference reads its video with cv::VideoCapture and keeps channel 0 of
each BGR frame (LocoMouse_class.cpp:367-403, :1273-1293).  Pinned here: the
libjpeg decoding defaults (ISLOW IDCT, fancy upsampling, jdcolor.c tables).
Unpinned: OpenCV's FFmpeg MJPEG path (FFmpeg IDCT + swscale), absent here."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import media_writers as MW  # noqa: E402
from test_cli import read_avi  # noqa: E402


def _frames(n, h, w, seed):
    """Smooth structure + noise + hard edges: every coefficient range occurs."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    out = []
    for k in range(n):
        base = 128 + 90 * np.sin(x / (3.0 + k) + y / 7.0) * np.cos(y / (5.0 + k))
        base += rng.normal(0, 25, size=(h, w))
        base[(x // 9 + y // 5 + k) % 4 == 0] = 255 if k % 2 else 0
        out.append(np.clip(base, 0, 255).astype(np.uint8))
    return np.stack(out)


def _check(tmp_path, frames, name="v", **kw):
    js = MW.jpeg_frames(frames, **kw)
    p = tmp_path / f"{name}.avi"
    h, w = frames.shape[1:]
    MW.write_mjpeg_avi(p, js, w, h)
    r = read_avi(p, max_frames=len(js))
    assert r is not None, "MJPEG AVI did not open"
    n, got = r
    want = np.stack([MW.decode_jpeg_channel0(MW._strip_segments(j, 0xFFFF)) for j in js])
    assert n == len(js) and got.shape == want.shape
    diff = np.argwhere(got != want)
    assert diff.size == 0, f"{len(diff)} samples differ, first {diff[:5].tolist()}"
    return got


@pytest.mark.parametrize("q", [5, 50, 75, 95, 100])
def test_grey(tmp_path, q):
    _check(tmp_path, _frames(3, 37, 53, q), mode="L", quality=q)


@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("shape", [(37, 53), (48, 64), (17, 9), (1, 1), (8, 200)])
def test_colour_subsampling(tmp_path, sub, shape):
    _check(tmp_path, _frames(2, *shape, sub), mode="RGB", quality=85, subsampling=sub)


def test_colour_q100_range_limit(tmp_path):
    f = _frames(2, 40, 40, 3)
    f[:, ::2, ::2] = 255
    f[:, 1::2, 1::2] = 0
    _check(tmp_path, f, mode="RGB", quality=100, subsampling=2)


@pytest.mark.parametrize("mode", ["L", "RGB"])
@pytest.mark.parametrize("kw", [dict(restart_marker_blocks=3), dict(restart_marker_rows=1),
                                dict(restart_marker_blocks=1)])
def test_restart_markers(tmp_path, mode, kw):
    _check(tmp_path, _frames(2, 45, 70, 7), mode=mode, quality=80, subsampling=2, **kw)


@pytest.mark.parametrize("mode", ["L", "RGB"])
def test_avi1_frames_without_huffman_tables(tmp_path, mode):
    """MJPEG cameras leave DHT out and rely on the standard tables (T.81 K.3)."""
    f = _frames(3, 32, 48, 11)
    js = MW.jpeg_frames(f, mode=mode, quality=70, subsampling=1)
    stripped = [MW._strip_segments(j, 0xC4) for j in js]
    assert all(b"\xff\xc4" not in s.split(b"\xff\xda")[0] for s in stripped)
    p = tmp_path / "avi1.avi"
    MW.write_mjpeg_avi(p, stripped, 48, 32)
    n, got = read_avi(p)
    want = np.stack([MW.decode_jpeg_channel0(j) for j in js])
    assert np.array_equal(got, want)


@pytest.mark.parametrize("mode", ["L", "RGB"])
def test_sixteen_bit_quantisation_tables(tmp_path, mode):
    """SOF1 with 16-bit (Pq = 1) quantisation tables (entries up to 1,900):
    parsed and decoded byte-identical to libjpeg-turbo.  The IDCT computes in
    JLONG as jidctint.c does (no 32-bit overflow for any table); for
    dequantised products beyond 16 bits libjpeg-turbo's SIMD IDCT wraps its
    16-bit lanes instead, which is not restated (unpinned: such streams do
    not come out of an encoder)."""
    qt = [[257 + 27 * i for i in range(64)], [300 + 25 * i for i in range(64)]]
    kw = {"qtables": qt[:1]} if mode == "L" else {"qtables": qt, "subsampling": 0}
    f = _frames(2, 40, 48, 11)
    js = MW.jpeg_frames(f, mode=mode, **kw)
    assert all(j.find(b"\xff\xc1") >= 0 for j in js)  # extended sequential (16-bit tables)
    _check(tmp_path, f, name="q16" + mode, mode=mode, **kw)


def test_optimized_huffman_tables(tmp_path):
    _check(tmp_path, _frames(2, 33, 65, 4), mode="RGB", quality=90, optimize=True)
    _check(tmp_path, _frames(2, 33, 65, 5), name="g", mode="L", quality=90, optimize=True)


def test_camera_sized_frames(tmp_path):
    """A LocoMouse-sized grey recording (synthetic scene, 1024 x 256)."""
    from locomouse_cpp_amd import synthetic as S
    cfg = S.SyntheticConfig()
    _check(tmp_path, cfg.frames(0, 4), mode="L", quality=90)
    _check(tmp_path, cfg.frames(0, 2), name="c", mode="RGB", quality=90, subsampling=2)


@pytest.mark.parametrize("fourcc", [b"MJPG", b"mjpg", b"JPEG", b"AVI1"])
def test_fourccs(tmp_path, fourcc):
    f = _frames(1, 16, 16, 1)
    js = MW.jpeg_frames(f, mode="L")
    p = tmp_path / "f.avi"
    MW.write_mjpeg_avi(p, js, 16, 16, fourcc=fourcc)
    assert np.array_equal(read_avi(p)[1], np.stack([MW.decode_jpeg_channel0(j) for j in js]))


def test_undecodable_frames_fail(tmp_path):
    f = _frames(2, 24, 24, 2)
    prog = MW.jpeg_frames(f, mode="L", progressive=True)
    p = tmp_path / "p.avi"
    MW.write_mjpeg_avi(p, prog, 24, 24)
    assert read_avi(p) is None or read_avi(p)[1].shape[0] == 0
    good = MW.jpeg_frames(f, mode="L")
    MW.write_mjpeg_avi(p, good, 24, 25)  # header size disagrees with the JPEG
    assert read_avi(p) is None or read_avi(p)[1].shape[0] == 0
    MW.write_mjpeg_avi(p, [good[0], b"\xff\xd8\xff\xd9"], 24, 24)  # no frame header
    r = read_avi(p)
    assert r is not None and r[1].shape[0] == 1
