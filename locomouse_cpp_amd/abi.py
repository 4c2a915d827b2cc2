"""ctypes mirror of include/locomouse_hip.h (the C-ABI drop-in boundary).

Struct layouts here must match the header field for field; tests/test_abi.py
checks sizes and offsets against a compiled probe.
"""
import ctypes as C

import numpy as np

LM_OK, LM_ERR_INVALID_ARGUMENT, LM_ERR_RUNTIME, LM_ERR_HIP = 0, 1, 2, 3
LM_N_TAIL_POINTS = 15
LM_FILTER_FUSED, LM_FILTER_UNFUSED = 0, 1
# lm_ctx_set_debug flags
LM_DEBUG_SCORES, LM_DEBUG_TIMING = 1, 2
LM_DEBUG_PLAN_PER_WIDTH, LM_DEBUG_PLAN_MERGED = 16, 32
LM_CORR_FP32, LM_CORR_F16 = 0, 1
LM_DEPTH_8U, LM_DEPTH_32F, LM_DEPTH_64F = 0, 5, 6
DETECTORS = ("paw_bottom", "snout_bottom", "tail_bottom", "paw_side", "snout_side", "tail_side")


class lm_rect(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("width", C.c_int32), ("height", C.c_int32)]

    def tuple(self):
        return (self.x, self.y, self.width, self.height)


class lm_location_prior(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("x", "y", "max_distance", "min_x", "max_x", "min_y", "max_y")]


class lm_params(C.Structure):
    _fields_ = [
        ("conn_comp_connectivity", C.c_int32),
        ("max_displacement_bottom", C.c_int32),
        ("max_displacement_side", C.c_int32),
        ("occlusion_grid_spacing_pixels_side", C.c_int32),
        ("occlusion_grid_spacing_pixels_bottom", C.c_int32),
        ("use_provided_bounding_box", C.c_int32),
        ("transform_gray_values", C.c_int32),
        ("use_reference_image_brightness", C.c_int32),
        ("side_bottom_min_overlap", C.c_double),
        ("occlusion_grid_max_width", C.c_double),
        ("tail_sub_bounding_box", C.c_double),
        ("alpha_vel_bottom", C.c_double),
        ("alpha_vel_side", C.c_double),
        ("pairwise_occluded_cost", C.c_double),
        ("location_prior", lm_location_prior * 5),
        ("bounding_box_side", lm_rect),
        ("bounding_box_bottom", lm_rect),
        ("gray_value_transformation", C.c_float * 256),
        ("gray_value_transformation_depth", C.c_int32),
    ]


class lm_detector(C.Structure):
    _fields_ = [("weights", C.POINTER(C.c_double)), ("rows", C.c_int32), ("cols", C.c_int32), ("bias", C.c_double)]


class lm_model(C.Structure):
    _fields_ = [(n, lm_detector) for n in ("paw_bottom", "paw_side", "snout_bottom", "snout_side", "tail_bottom", "tail_side")]


class lm_setup(C.Structure):
    _fields_ = [
        ("method", C.c_int32),
        ("flip", C.c_int32),
        ("video_rows", C.c_int32),
        ("video_cols", C.c_int32),
        ("background", C.POINTER(C.c_uint8)),
        ("calib_rows", C.c_int32),
        ("calib_cols", C.c_int32),
        ("ind_warp_mapping", C.POINTER(C.c_int32)),
        ("view_box_side", lm_rect),
        ("view_box_bottom", lm_rect),
        ("filter_arith", C.c_int32),
        ("corr_precision", C.c_int32),
        ("pipeline_lanes", C.c_int32),
    ]


class lm_geometry(C.Structure):
    _fields_ = (
        [(n, C.c_int32) for n in ("n_rows", "n_cols", "pad_pre_rows", "pad_pre_cols", "pad_post_rows", "pad_post_cols",
                                  "ipad_rows", "ipad_cols", "spre_b_w", "spre_b_h", "spost_b_w", "spost_b_h",
                                  "spre_t_w", "spre_t_h", "spost_t_w", "spost_t_h")]
        + [(n, lm_rect) for n in ("bb_bottom_mouse", "bb_side_mouse", "bb_bottom_mouse_pad", "bb_side_mouse_pad",
                                  "bb_unpad_mouse_bottom", "bb_unpad_mouse_side", "bb_bottom_tail_pad",
                                  "bb_unpad_tail_bottom", "bb_bottom_tail", "bb_side_tail_pad", "bb_unpad_tail_side")]
        + [("tail_box_width", C.c_int32), ("ong_nx", C.c_int32), ("ong_ny", C.c_int32),
           ("ong_br_x", C.c_double), ("ong_br_y", C.c_double), ("n_ong_side", C.c_int32), ("ong_side_lowest", C.c_int32)]
        + [(n, lm_rect) for n in ("match_box_paw_bottom", "match_box_paw_side", "match_box_snout_bottom",
                                  "match_box_snout_side")]
    )

    def as_dict(self):
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = v.tuple() if isinstance(v, lm_rect) else v
        return out


class lm_candidate(C.Structure):
    _fields_ = [("x", C.c_int32), ("y", C.c_int32), ("score", C.c_double)]


class lm_p22d(C.Structure):
    _fields_ = [("bottom", lm_candidate), ("side_offset", C.c_int32), ("side_count", C.c_int32)]


class lm_batch_result(C.Structure):
    _fields_ = [
        ("n_frames", C.c_int32),
        ("first_frame", C.c_int32),
        ("cand_offset", C.POINTER(C.c_int64)),
        ("cand", C.POINTER(lm_candidate)),
        ("p22d_offset", C.POINTER(C.c_int64)),
        ("p22d", C.POINTER(lm_p22d)),
        ("side_y", C.POINTER(C.c_int32)),
        ("side_s", C.POINTER(C.c_double)),
        ("unary_offset", C.POINTER(C.c_int64)),
        ("unary", C.POINTER(C.c_double)),
        ("pw_dims", C.POINTER(C.c_int32)),
        ("pw_jc_offset", C.POINTER(C.c_int64)),
        ("pw_jc", C.POINTER(C.c_int32)),
        ("pw_nz_offset", C.POINTER(C.c_int64)),
        ("pw_ir", C.POINTER(C.c_int32)),
        ("pw_pr", C.POINTER(C.c_double)),
        ("tail", C.POINTER(C.c_int32)),
    ]


LM_BB_FIRSTLAST_AS_EXECUTED, LM_BB_FIRSTLAST_INTEGER = 0, 1


class lm_bb_params(C.Structure):
    _fields_ = [
        ("median_filter_size", C.c_int32),
        ("min_pixel_visible", C.c_int32),
        ("moving_average_window", C.c_int32),
        ("conn_comp_connectivity", C.c_int32),
        ("firstlast_semantics", C.c_int32),
        ("zero_col_pre", C.c_int32),
        ("zero_col_post", C.c_int32),
        ("zero_row_pre", C.c_int32),
        ("zero_row_post", C.c_int32),
        ("bb_width", C.c_int32),
        ("bb_height_side", C.c_int32),
        ("reserved0", C.c_int32),
    ]


class lm_bb_frame(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("x", "y_bottom", "y_side", "width", "height_bottom", "height_side")]


class lm_bb_result(C.Structure):
    _fields_ = [
        ("n_frames", C.c_int32),
        ("reserved0", C.c_int32),
        ("bb_side_mouse", lm_rect),
        ("bb_bottom_mouse", lm_rect),
        ("x_pos", C.POINTER(C.c_uint32)),
        ("y_bottom_pos", C.POINTER(C.c_uint32)),
        ("y_side_pos", C.POINTER(C.c_uint32)),
        ("frames", C.POINTER(lm_bb_frame)),
    ]


BB_FRAME_DTYPE = np.dtype([(n, "<f8") for n in ("x", "y_bottom", "y_side", "width", "height_bottom", "height_side")])


def bb_params(median_filter_size=11, min_pixel_visible=1, moving_average_window=5, connectivity=8,
              semantics=LM_BB_FIRSTLAST_AS_EXECUTED, zero_cols=(46, 760), zero_rows=(100, 149), bb_width=400,
              bb_height_side=150):
    """lm_bb_params with the reference defaults (LocoMouse_class.hpp:53-69,
    LocoMouse_TM.hpp:19-31)."""
    return lm_bb_params(median_filter_size, min_pixel_visible, moving_average_window, connectivity, semantics,
                        zero_cols[0], zero_cols[1], zero_rows[0], zero_rows[1], bb_width, bb_height_side, 0)


CAND_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("score", "<f8")])
P22D_DTYPE = np.dtype([("x", "<i4"), ("y", "<i4"), ("score", "<f8"), ("side_offset", "<i4"), ("side_count", "<i4")])


def _arr(ptr, n, dtype):
    if n <= 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    buf = C.cast(ptr, C.POINTER(C.c_uint8 * (n * np.dtype(dtype).itemsize))).contents
    return np.frombuffer(buf, dtype=dtype, count=n).copy()


def result_to_numpy(r: lm_batch_result):
    """Copy an lm_batch_result into plain numpy arrays (same layout)."""
    n = r.n_frames
    cand_off = _arr(r.cand_offset, 4 * n + 1, np.int64)
    p_off = _arr(r.p22d_offset, 2 * n + 1, np.int64)
    u_off = _arr(r.unary_offset, 2 * n + 1, np.int64)
    jc_off = _arr(r.pw_jc_offset, 2 * n + 1, np.int64)
    nz_off = _arr(r.pw_nz_offset, 2 * n + 1, np.int64)
    p22d = _arr(r.p22d, int(p_off[-1]), P22D_DTYPE)
    n_side = int((p22d["side_offset"] + p22d["side_count"]).max()) if len(p22d) else 0
    return {
        "n_frames": n,
        "first_frame": r.first_frame,
        "cand_offset": cand_off,
        "cand": _arr(r.cand, int(cand_off[-1]), CAND_DTYPE),
        "p22d_offset": p_off,
        "p22d": p22d,
        "side_y": _arr(r.side_y, n_side, np.int32),
        "side_s": _arr(r.side_s, n_side, np.float64),
        "unary_offset": u_off,
        "unary": _arr(r.unary, int(u_off[-1]), np.float64),
        "pw_dims": _arr(r.pw_dims, 6 * n, np.int32).reshape(n, 2, 3),
        "pw_jc_offset": jc_off,
        "pw_jc": _arr(r.pw_jc, int(jc_off[-1]), np.int32),
        "pw_nz_offset": nz_off,
        "pw_ir": _arr(r.pw_ir, int(nz_off[-1]), np.int32),
        "pw_pr": _arr(r.pw_pr, int(nz_off[-1]), np.float64),
        "tail": _arr(r.tail, 45 * n, np.int32).reshape(n, 3, 15),
    }


def frame_views(res, f):
    """Per-frame, reference-shaped view of a result dict: the four candidate
    lists, the two P22D lists (as (bottom, yt, st) tuples), the two unary
    MyMats (N x k, column-major restored), the two MATSPARSE (or None) and the
    3x15 tail track."""
    out = {}
    co = res["cand_offset"]
    out["cand"] = [res["cand"][co[4 * f + k]:co[4 * f + k + 1]] for k in range(4)]
    po = res["p22d_offset"]
    p22 = []
    for k in range(2):
        lst = []
        for p in res["p22d"][po[2 * f + k]:po[2 * f + k + 1]]:
            o, c = int(p["side_offset"]), int(p["side_count"])
            lst.append(((int(p["x"]), int(p["y"]), float(p["score"])),
                        res["side_y"][o:o + c].tolist(), res["side_s"][o:o + c].tolist()))
        p22.append(lst)
    out["p22d"] = p22
    uo = res["unary_offset"]
    out["unary"] = [res["unary"][uo[2 * f + k]:uo[2 * f + k + 1]] for k in range(2)]
    pw = []
    for k in range(2):
        nr, nc, nnz = res["pw_dims"][f, k]
        if nr < 0:
            pw.append(None)
            continue
        jo, no = res["pw_jc_offset"], res["pw_nz_offset"]
        pw.append({"n_rows": int(nr), "n_cols": int(nc), "jc": res["pw_jc"][jo[2 * f + k]:jo[2 * f + k + 1]],
                   "ir": res["pw_ir"][no[2 * f + k]:no[2 * f + k + 1]], "pr": res["pw_pr"][no[2 * f + k]:no[2 * f + k + 1]]})
    out["pairwise"] = pw
    out["tail"] = res["tail"][f]
    return out


class lm_tracks(C.Structure):  # include/locomouse_track.h
    _fields_ = [
        ("n_frames", C.c_int32),
        ("paw_tracks", C.POINTER(C.c_int32)),
        ("snout_tracks", C.POINTER(C.c_int32)),
        ("tracks_tail", C.POINTER(C.c_int32)),
        ("track_index_bottom", C.POINTER(C.c_int32)),
        ("track_index_side", C.POINTER(C.c_int32)),
    ]


def numpy_to_result(res):
    """An lm_batch_result pointing into a result dict's arrays (the dict must
    outlive it; arrays are made contiguous in place)."""
    r = lm_batch_result()
    keep = {}
    for k in ("cand_offset", "cand", "p22d_offset", "p22d", "side_y", "side_s", "unary_offset", "unary", "pw_dims",
              "pw_jc_offset", "pw_jc", "pw_nz_offset", "pw_ir", "pw_pr", "tail"):
        a = np.ascontiguousarray(res[k])
        keep[k] = a
        setattr(r, k, C.cast(a.ctypes.data, dict(lm_batch_result._fields_)[k]))
    r.n_frames = int(res["n_frames"])
    r.first_frame = int(res.get("first_frame", 0))
    r._keep = keep
    return r
