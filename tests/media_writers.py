"""Writers of the reference CLI's input files, for tests: OpenCV FileStorage
YAML (config.yml, the model and calibration files), 8-bit PNG,
uncompressed AVI and MJPEG AVI (frames encoded by Pillow).  Test infrastructure: these produce the files the
reference's users hand to `LocoMouse`."""
import struct
import zlib

import numpy as np


def _fmt(v):
    if isinstance(v, (int, np.integer)):
        return str(int(v))
    return repr(float(v))


def yaml_matrix(name, a, dt, per_line=8):
    a = np.asarray(a)
    vals = [_fmt(v) for v in a.reshape(-1)]
    lines = [", ".join(vals[i:i + per_line]) for i in range(0, len(vals), per_line)]
    body = (",\n       ").join(lines)
    return f"{name}: !!opencv-matrix\n   rows: {a.shape[0]}\n   cols: {a.shape[1]}\n   dt: {dt}\n   data: [ {body} ]\n"


def write_config(path, cfg, bb_params=None, overrides=None):
    p = cfg.params
    keys = {
        "verbose_debug": 0, "N_debug_frames": 0, "parameters_for_visual_debug": 0,
        "conn_comp_connectivity": p.conn_comp_connectivity,
        "median_filter_size": bb_params.median_filter_size if bb_params else 11,
        "min_pixel_visible": bb_params.min_pixel_visible if bb_params else 1,
        "side_bottom_min_overlap": p.side_bottom_min_overlap,
        "max_displacement_bottom": p.max_displacement_bottom, "max_displacement_side": p.max_displacement_side,
        "occlusion_grid_spacing_pixels_side": p.occlusion_grid_spacing_pixels_side,
        "occlusion_grid_spacing_pixels_bottom": p.occlusion_grid_spacing_pixels_bottom,
        "occlusion_grid_max_width": p.occlusion_grid_max_width, "tail_sub_bounding_box": p.tail_sub_bounding_box,
        "alpha_vel_bottom": p.alpha_vel_bottom, "alpha_vel_side": p.alpha_vel_side,
        "pairwise_occluded_cost": p.pairwise_occluded_cost,
        "moving_average_window": bb_params.moving_average_window if bb_params else 5,
        "transform_gray_values": 0, "use_reference_image_brightness": 0,
        "use_provided_bounding_box": p.use_provided_bounding_box,
    }
    keys.update(overrides or {})
    out = ["%YAML:1.0", "---"]
    for k, v in keys.items():
        if v is None:
            continue
        out.append(f"{k}: {v if isinstance(v, str) else _fmt(v)}")
    text = "\n".join(out) + "\n"
    prior = np.array([[lp.x, lp.y, lp.max_distance, lp.min_x, lp.max_x, lp.min_y, lp.max_y] for lp in p.location_prior])
    text += "# location prior: x y max_distance min_x max_x min_y max_y\n"
    text += yaml_matrix("location_prior", prior, "d")
    for name, r in (("bounding_box_side", p.bounding_box_side), ("bounding_box_bottom", p.bounding_box_bottom)):
        text += yaml_matrix(name, np.array([[r.x, r.y, r.width, r.height]]), "i")
    with open(path, "w") as fh:
        fh.write(text)


MODEL_KEYS = {"paw_side": "Paw_side", "paw_bottom": "Paw_bottom", "tail_side": "Tail_side",
              "tail_bottom": "Tail_bottom", "snout_side": "Snout_side", "snout_bottom": "Snout_bottom"}


def write_model(path, cfg):
    text = "%YAML:1.0\n---\n"
    for name, suffix in MODEL_KEYS.items():
        text += yaml_matrix("model" + suffix, cfg.weights[name], "d", per_line=4)
    for name, suffix in MODEL_KEYS.items():
        text += f"bias{suffix}: {_fmt(cfg.biases[name])}\n"
    with open(path, "w") as fh:
        fh.write(text)


def write_calibration(path, cfg):
    su = cfg.setup
    boxes = np.array([[su.view_box_side.x, su.view_box_side.y, su.view_box_side.width, su.view_box_side.height],
                      [su.view_box_bottom.x, su.view_box_bottom.y, su.view_box_bottom.width,
                       su.view_box_bottom.height]])
    text = "%YAML:1.0\n---\n" + yaml_matrix("ind_warp_mapping", cfg.calib, "i", per_line=32)
    text += yaml_matrix("view_boxes", boxes, "i")
    with open(path, "w") as fh:
        fh.write(text)


def _chunk(tag, data):
    c = struct.pack(">I", len(data)) + tag + data
    return c + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)


def write_png(path, img, filters=(0, 1, 2, 3, 4)):
    """8-bit grey (H x W) or RGB (H x W x 3); rows use the given filter types
    in turn, so the reader's unfiltering is exercised."""
    img = np.asarray(img, np.uint8)
    ch = 1 if img.ndim == 2 else img.shape[2]
    h, w = img.shape[:2]
    flat = img.reshape(h, w * ch).astype(np.int32)
    raw = bytearray()
    prev = np.zeros(w * ch, np.int32)
    for y in range(h):
        ft = filters[y % len(filters)]
        cur = flat[y]
        left = np.concatenate([np.zeros(ch, np.int32), cur[:-ch]])
        upleft = np.concatenate([np.zeros(ch, np.int32), prev[:-ch]])
        if ft == 0:
            out = cur
        elif ft == 1:
            out = cur - left
        elif ft == 2:
            out = cur - prev
        elif ft == 3:
            out = cur - (left + prev) // 2
        else:
            p = left + prev - upleft
            pa, pb, pc = np.abs(p - left), np.abs(p - prev), np.abs(p - upleft)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, upleft))
            out = cur - pred
        raw.append(ft)
        raw += (out & 0xFF).astype(np.uint8).tobytes()
        prev = cur
    ctype = {1: 0, 3: 2, 4: 6}[ch]
    data = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0))
    data += _chunk(b"IDAT", zlib.compress(bytes(raw), 6)) + _chunk(b"IEND", b"")
    with open(path, "wb") as fh:
        fh.write(data)


def write_avi(path, frames, bits=24, other=None, fps=30):
    """Uncompressed AVI: `frames` (n x H x W u8) become channel 0 (blue) of
    24-bit BGR frames (green/red from `other`, default a pattern) stored
    bottom-up with 4-byte row padding, or 8-bit palettised frames whose
    palette maps index i to blue = frames value (identity here: blue = i)."""
    frames = np.asarray(frames, np.uint8)
    n, h, w = frames.shape
    if bits == 24:
        stride = (w * 3 + 3) & ~3
    else:
        stride = (w + 3) & ~3
    size = stride * h
    strh = b"vids" + b"DIB " + struct.pack("<IHHIIIIIIIIhhhh", 0, 0, 0, 0, 1, fps, 0, n, size, 0xFFFFFFFF, 0, 0, 0, w, h)
    bih = struct.pack("<IiiHHIIiiII", 40, w, h, 1, bits, 0, size, 0, 0, 256 if bits == 8 else 0, 0)
    if bits == 8:
        bih += b"".join(struct.pack("<BBBB", i, (i * 7) & 0xFF, (i * 13) & 0xFF, 0) for i in range(256))

    def ck(tag, data):
        return tag + struct.pack("<I", len(data)) + data + (b"\0" if len(data) & 1 else b"")

    def lst(tag, data):
        return b"LIST" + struct.pack("<I", len(data) + 4) + tag + data

    avih = struct.pack("<IIIIIIIIIIIIII", 1000000 // fps, 0, 0, 0x10, n, 0, 1, size, w, h, 0, 0, 0, 0)
    hdrl = lst(b"hdrl", ck(b"avih", avih) + lst(b"strl", ck(b"strh", strh) + ck(b"strf", bih)))
    movi = bytearray()
    for f in range(n):
        img = frames[f][::-1]  # bottom-up
        if bits == 24:
            g = other[f] if other is not None else (img.astype(np.int32) * 3 + 17) & 0xFF
            bgr = np.stack([img, g.astype(np.uint8), (255 - img)], axis=2).reshape(h, w * 3)
        else:
            bgr = img
        rows = np.zeros((h, stride), np.uint8)
        rows[:, :bgr.shape[1]] = bgr
        movi += ck(b"00db", rows.tobytes())
    body = b"AVI " + hdrl + ck(b"JUNK", b"\0" * 12) + lst(b"movi", bytes(movi))
    with open(path, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def jpeg_frames(frames, mode="L", other=None, strip_dht=False, **save_kw):
    """Each frame (H x W u8) as a JPEG encoded by Pillow (libjpeg-turbo): grey
    ('L'), or colour ('RGB') whose blue channel is the frame (red / green from
    `other` or a pattern) — channel 0 of the BGR rendering is then the frame
    up to the codec's loss.  save_kw go to Image.save (quality, subsampling,
    optimize, restart_marker_blocks, progressive ...).  strip_dht drops the
    Huffman table segments, as MJPEG "AVI1" frames do (valid only with the
    standard tables, i.e. without optimize)."""
    import io

    from PIL import Image
    out = []
    for f, img in enumerate(np.asarray(frames, np.uint8)):
        if mode == "L":
            im = Image.fromarray(img, "L")
        else:
            g = other[f] if other is not None else (img.astype(np.int32) * 3 + 17) & 0xFF
            rgb = np.stack([(255 - img), g.astype(np.uint8), img], axis=2)
            im = Image.fromarray(rgb, "RGB")
        b = io.BytesIO()
        im.save(b, "JPEG", **save_kw)
        d = b.getvalue()
        if strip_dht:
            d = _strip_segments(d, 0xC4)
        out.append(d)
    return out


def _strip_segments(d, marker):
    out, i = bytearray(d[:2]), 2
    while i < len(d):
        m = d[i + 1]
        if m == 0xDA:
            out += d[i:]
            break
        n = 2 + (d[i + 2] << 8 | d[i + 3])
        if m != marker:
            out += d[i:i + n]
        i += n
    return bytes(out)


def decode_jpeg_channel0(data):
    """Pillow's (libjpeg-turbo's) decoding of one JPEG, as channel 0 of BGR:
    the blue plane of its RGB rendering, or the grey plane itself."""
    import io

    from PIL import Image
    im = Image.open(io.BytesIO(data))
    im.load()
    a = np.asarray(im)
    return a if a.ndim == 2 else a[:, :, 2]


def write_mjpeg_avi(path, jpegs, w, h, fps=30, fourcc=b"MJPG"):
    """MJPEG AVI: one JPEG per '00dc' chunk, BITMAPINFOHEADER compression
    `fourcc` (24 bits), frame size w x h."""
    n = len(jpegs)
    size = max(len(j) for j in jpegs)
    strh = b"vids" + fourcc + struct.pack("<IHHIIIIIIIIhhhh", 0, 0, 0, 0, 1, fps, 0, n, size, 0xFFFFFFFF, 0, 0, 0, w, h)
    bih = struct.pack("<IiiHH", 40, w, h, 1, 24) + fourcc + struct.pack("<IiiII", w * h * 3, 0, 0, 0, 0)

    def ck(tag, data):
        return tag + struct.pack("<I", len(data)) + data + (b"\0" if len(data) & 1 else b"")

    def lst(tag, data):
        return b"LIST" + struct.pack("<I", len(data) + 4) + tag + data

    avih = struct.pack("<IIIIIIIIIIIIII", 1000000 // fps, 0, 0, 0x10, n, 0, 1, size, w, h, 0, 0, 0, 0)
    hdrl = lst(b"hdrl", ck(b"avih", avih) + lst(b"strl", ck(b"strh", strh) + ck(b"strf", bih)))
    movi = b"".join(ck(b"00dc", j) for j in jpegs)
    body = b"AVI " + hdrl + lst(b"movi", movi)
    with open(path, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def write_inputs(dirpath, cfg, n_frames, stem="synth_R", bits=24, config_overrides=None, bb_params=None,
                 jpeg=None):
    """The five input files of one CLI run; returns their paths."""
    import os
    paths = {k: os.path.join(dirpath, v) for k, v in (
        ("config", "config.yml"), ("video", stem + ".avi"), ("background", stem + ".png"),
        ("model", "model.yml"), ("calibration", "calibration.yml"))}
    write_config(paths["config"], cfg, bb_params=bb_params, overrides=config_overrides)
    write_model(paths["model"], cfg)
    write_calibration(paths["calibration"], cfg)
    write_png(paths["background"], cfg.background)
    if jpeg is None:
        write_avi(paths["video"], cfg.frames(0, n_frames), bits=bits)
    else:  # MJPEG: jpeg = jpeg_frames keyword arguments; the decoded frames are returned too
        js = jpeg_frames(cfg.frames(0, n_frames), **jpeg)
        write_mjpeg_avi(paths["video"], js, cfg.cols, cfg.rows)
        paths["decoded"] = np.stack([decode_jpeg_channel0(j) for j in js])
    return paths
