"""ctypes binding of the CPU restatement oracle (oracle/liblm_oracle.so).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  PARITY UNPINNED (see lm_oracle.cpp header).
"""
import ctypes as C
import os
import subprocess

import numpy as np

from locomouse_cpp_amd.abi import BB_FRAME_DTYPE, lm_batch_result, lm_geometry, lm_rect, result_to_numpy

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblm_oracle.so")

KEEP_DEBUG = 1
UNFUSED_FILTER = 2

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.lmo_last_error.restype = C.c_char_p
        L.lmo_run.restype = C.c_int
        L.lmo_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p,
                              C.c_int32, C.POINTER(C.c_void_p), C.POINTER(lm_batch_result)]
        L.lmo_free.argtypes = [C.c_void_p]
        L.lmo_geometry.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(lm_geometry)]
        L.lmo_debug_scores.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32]
        L.lmo_debug_scores_dims.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.lmo_debug_tail_mask.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32]
        L.lmo_debug_ipad.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32]
        L.lmo_std_sort_perm.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
        L.lmo_synth_frames.argtypes = [C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_void_p]
        L.lmo_synth_background.argtypes = [C.c_int32, C.c_int32, C.c_void_p]
        L.lmo_median_blur.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_void_p]
        L.lmo_first_last.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_int32, C.c_void_p]
        L.lmo_imadjust_default_lut.argtypes = [C.c_void_p, C.c_void_p]
        L.lmo_movavg.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
        L.lmo_bb_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p,
                                 C.POINTER(lm_rect), C.POINTER(lm_rect), C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p]
        _lib = L
    return _lib


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"oracle status {code}: {msg}")
        self.code = code


def geometry(cfg):
    g = lm_geometry()
    rc = lib().lmo_geometry(C.byref(cfg.setup), C.byref(cfg.params), C.byref(cfg.model), C.byref(g))
    if rc:
        raise OracleError(rc, lib().lmo_last_error().decode())
    return g


class OracleRun:
    """Frames 0..n-1 through the restated per-frame loop (main.cpp:54-82)."""

    def __init__(self, cfg, frames, bb=None, flags=0):
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        self.n = frames.shape[0]
        self.cfg = cfg
        self._h = C.c_void_p()
        view = lm_batch_result()
        bbp = None
        if bb is not None:
            self._bb = np.ascontiguousarray(bb, dtype=np.int32)
            bbp = self._bb.ctypes.data
        rc = lib().lmo_run(C.byref(cfg.setup), C.byref(cfg.params), C.byref(cfg.model), frames.ctypes.data,
                           frames.shape[1] * frames.shape[2], self.n, bbp, flags, C.byref(self._h), C.byref(view))
        if rc:
            raise OracleError(rc, lib().lmo_last_error().decode())
        self.result = result_to_numpy(view)

    def scores(self, f, det, shape=None):
        if shape is None:
            r, c = C.c_int32(), C.c_int32()
            if lib().lmo_debug_scores_dims(self._h, f, det, C.byref(r), C.byref(c)) or r.value == 0:
                return None
            shape = (r.value, c.value)
        out = np.zeros(shape, dtype=np.float32)
        rc = lib().lmo_debug_scores(self._h, f, det, out.ctypes.data, shape[0], shape[1])
        if rc:
            return None
        return out

    def tail_mask(self, f, shape):
        out = np.zeros(shape, dtype=np.uint8)
        rc = lib().lmo_debug_tail_mask(self._h, f, out.ctypes.data, shape[0], shape[1])
        if rc:
            raise OracleError(rc, "tail mask")
        return out

    def ipad(self, f, shape):
        out = np.zeros(shape, dtype=np.uint8)
        rc = lib().lmo_debug_ipad(self._h, f, out.ctypes.data, shape[0], shape[1])
        if rc:
            raise OracleError(rc, "ipad")
        return out

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().lmo_free(self._h)
            self._h = C.c_void_p()


def std_sort_perm(scores):
    s = np.ascontiguousarray(scores, dtype=np.float64)
    perm = np.zeros(len(s), dtype=np.int32)
    lib().lmo_std_sort_perm(s.ctypes.data, len(s), perm.ctypes.data)
    return perm


def synth_frames_c(rows, cols, first, n):
    out = np.zeros((n, rows, cols), dtype=np.uint8)
    lib().lmo_synth_frames(rows, cols, first, n, out.ctypes.data)
    return out


def synth_background_c(rows, cols):
    out = np.zeros((rows, cols), dtype=np.uint8)
    lib().lmo_synth_background(rows, cols, out.ctypes.data)
    return out


def bb_run(setup, bb_params, frames, binary=False):
    """Whole-video BB pass, method 0 (LocoMouse::computeBoundingBox,
    LocoMouse_class.cpp:579-653) over frames [n, rows, cols] u8."""
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    n = frames.shape[0]
    per = np.zeros(n, dtype=BB_FRAME_DTYPE)
    xs, yb, ys = (np.zeros(n, dtype=np.uint32) for _ in range(3))
    side, bottom = lm_rect(), lm_rect()
    binimg = np.zeros((n, setup.calib_rows, setup.calib_cols), dtype=np.uint8) if binary else None
    rc = lib().lmo_bb_run(C.byref(setup), C.byref(bb_params), frames.ctypes.data, frames.shape[1] * frames.shape[2], n,
                          per.ctypes.data, C.byref(side), C.byref(bottom), xs.ctypes.data, yb.ctypes.data,
                          ys.ctypes.data, binimg.ctypes.data if binary else None)
    if rc:
        raise OracleError(rc, lib().lmo_last_error().decode())
    out = {"frames": per, "x_pos": xs, "y_bottom_pos": yb, "y_side_pos": ys, "bb_side_mouse": side.tuple(),
           "bb_bottom_mouse": bottom.tuple()}
    if binary:
        out["binary"] = binimg
    return out


def median_blur(img, ksize):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.zeros_like(img)
    lib().lmo_median_blur(img.ctypes.data, img.shape[0], img.shape[1], ksize, out.ctypes.data)
    return out


def first_last(values, th, integer=False, length=None):
    v = np.ascontiguousarray(values, dtype=np.int32)
    out = np.zeros(2, dtype=np.int32)
    lib().lmo_first_last(v.ctypes.data, len(v) if length is None else length, th, 1 if integer else 0, out.ctypes.data)
    return tuple(int(x) for x in out)


def moving_average(values, window):
    v = np.ascontiguousarray(values, dtype=np.float64)
    out = np.zeros(len(v), dtype=np.uint32)
    lib().lmo_movavg(v.ctypes.data, len(v), window, out.ctypes.data)
    return out


def imadjust_default_lut(hist):
    h = np.ascontiguousarray(hist, dtype=np.uint32)
    out = np.zeros(256, dtype=np.uint8)
    lib().lmo_imadjust_default_lut(h.ctypes.data, out.ctypes.data)
    return out
