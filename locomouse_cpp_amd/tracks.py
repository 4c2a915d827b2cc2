"""ctypes binding of the tracking stage's C-ABI (include/locomouse_track.h,
exported by liblocomouse_host.so): match2nd, the bottom/side tracks and the
track export that follow the per-frame detection path.
Host code; no GPU is needed to call it."""
import ctypes as C
import os

import numpy as np

from . import runtime
from .abi import lm_geometry, lm_params, lm_tracks, numpy_to_result

EXPORTED = ("lm_track_last_error", "lm_match2nd", "lm_compute_tracks", "lm_write_tracks_yaml")

_lib = None


class TrackError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{'invalid_argument' if code == 1 else 'runtime_error'}: {msg}")
        self.code = code


def lib():
    global _lib
    if _lib is None:
        runtime.lib()  # the C-ABI library the host library links against
        if not os.path.exists(runtime.HOST_LIB_PATH):
            raise RuntimeError(f"{runtime.HOST_LIB_PATH} is missing: run locomouse_cpp_amd.runtime.build()")
        L = C.CDLL(runtime.HOST_LIB_PATH)
        L.lm_track_last_error.restype = C.c_char_p
        L.lm_match2nd.argtypes = [C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_double, C.c_double] + [C.c_void_p] * 12
        L.lm_compute_tracks.argtypes = [C.c_void_p, C.POINTER(lm_geometry), C.POINTER(lm_params), C.c_void_p,
                                        C.POINTER(lm_tracks)]
        L.lm_write_tracks_yaml.argtypes = [C.c_char_p, C.POINTER(lm_tracks)]
        _lib = L
    return _lib


def _check(rc):
    if rc:
        raise TrackError(rc, lib().lm_track_last_error().decode())


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def match2nd(unary, pairwise, nong, points, perm, occ_cost=0.0, bam=0.0, with_cost=False):
    """unary: list of (n_loc x n_cols) float64 arrays; pairwise: list of
    (rows, cols, jc, ir, pr) for f -> f+1.  Returns the points x frames labels
    (and computeCostTrack when with_cost)."""
    n = len(unary)
    n_cols = unary[0].shape[1] if n else points
    n_loc = np.array([u.shape[0] for u in unary], np.int32)
    u_off = np.zeros(n + 1, np.int64)
    u_off[1:] = np.cumsum([u.size for u in unary])
    u = np.concatenate([np.asarray(x, np.float64).reshape(-1, order="F") for x in unary]) if n else np.zeros(0)
    dims = np.array([[p[0], p[1], len(p[3])] for p in pairwise], np.int32).reshape(-1)
    jc_off = np.zeros(len(pairwise) + 1, np.int64)
    jc_off[1:] = np.cumsum([len(p[2]) for p in pairwise])
    nz_off = np.zeros(len(pairwise) + 1, np.int64)
    nz_off[1:] = np.cumsum([len(p[3]) for p in pairwise])
    cat = lambda i, dt: (np.concatenate([np.asarray(p[i], dt) for p in pairwise]) if pairwise else np.zeros(0, dt))
    jc, ir, pr = cat(2, np.int32), cat(3, np.int32), cat(4, np.float64)
    perm = np.asarray(perm, np.int32)
    labels = np.zeros((points, n), np.int32)
    cost = C.c_double(0)
    # keep empty arrays addressable
    u = u if u.size else np.zeros(1)
    ir = ir if ir.size else np.zeros(1, np.int32)
    pr = pr if pr.size else np.zeros(1)
    jc = jc if jc.size else np.zeros(1, np.int32)
    dims = dims if dims.size else np.zeros(3, np.int32)
    _check(lib().lm_match2nd(n, points, n_cols, nong, occ_cost, bam, n_loc.ctypes.data, u_off.ctypes.data,
                             u.ctypes.data, dims.ctypes.data, jc_off.ctypes.data, jc.ctypes.data, nz_off.ctypes.data,
                             ir.ctypes.data, pr.ctypes.data, perm.ctypes.data, labels.ctypes.data,
                             C.byref(cost) if with_cost else None))
    return (labels, cost.value) if with_cost else labels


def _arr(ptr, n):
    return np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n else np.zeros(0, np.int32)


def compute_tracks(res, geometry, params, bb):
    """computeBottomTracks + computeSideTracks + exportResults over a whole
    video's result dict.  bb: [n][3] uint32 BR corners (x, y_bottom, y_side)."""
    r = numpy_to_result(res)
    bb = np.ascontiguousarray(bb, np.uint32)
    out = lm_tracks()
    _check(lib().lm_compute_tracks(C.byref(r), C.byref(geometry), C.byref(params), bb.ctypes.data, C.byref(out)))
    n = out.n_frames
    d = {
        "paw_tracks": _arr(out.paw_tracks, 12 * n).reshape(4, n, 3),
        "snout_tracks": _arr(out.snout_tracks, 3 * n).reshape(1, n, 3),
        "tracks_tail": _arr(out.tracks_tail, 45 * n).reshape(3, 15 * n),
        "track_index_bottom": _arr(out.track_index_bottom, 5 * n).reshape(5, n),
        "track_index_side": _arr(out.track_index_side, 5 * n).reshape(5, n),
    }
    return d


def write_yaml(path, tracks):
    n = tracks["paw_tracks"].shape[1]
    keep = {k: np.ascontiguousarray(tracks[k], np.int32) for k in ("paw_tracks", "snout_tracks", "tracks_tail")}
    t = lm_tracks()
    t.n_frames = n
    for k, a in keep.items():
        setattr(t, k, a.ctypes.data_as(C.POINTER(C.c_int32)))
    _check(lib().lm_write_tracks_yaml(os.fsencode(path), C.byref(t)))
