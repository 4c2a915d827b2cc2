"""ctypes binding of liblocomouse_hip.so (the C-ABI in include/locomouse_hip.h).

This is how tests and bench.py drive the HIP path.  There is no CPU fallback:
if the shared library is missing or no HIP device is present, Context()
raises.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from .abi import BB_FRAME_DTYPE, LM_OK, lm_batch_result, lm_bb_result, lm_geometry, result_to_numpy

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB_PATH = os.path.join(PKG, "liblocomouse_hip.so")
CSRC = os.path.join(PKG, "csrc")

EXPORTED = (
    "lm_abi_version", "lm_last_error", "lm_ctx_create", "lm_ctx_destroy", "lm_get_geometry", "lm_ctx_stream",
    "lm_detect_batch", "lm_detect_batch_device", "lm_ctx_set_debug", "lm_debug_scores", "lm_debug_tail_mask",
    "lm_debug_kernel_times", "lm_debug_kernel_spans", "lm_synth_frames_device",
    "lm_bb_create", "lm_bb_destroy", "lm_bb_push", "lm_bb_push_device", "lm_bb_finish", "lm_bb_debug_binary",
    "lm_bb_stream", "lm_host_alloc", "lm_host_free",
    "lm_detect_submit", "lm_detect_submit_device", "lm_detect_collect", "lm_ctx_lanes", "lm_ctx_pending",
    "lm_debug_corr_work", "lm_debug_batch_slots", "lm_debug_dark_tile_width",
    "lm_debug_dark_tile_height",
)

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-slp-vectorize",
               "-fvisibility=hidden", "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


HOST_DIR = os.path.join(PKG, "host")
HOST_LIB_PATH = os.path.join(PKG, "liblocomouse_host.so")
CLI_PATH = os.path.join(PKG, "bin", "LocoMouse")


HIP_UNITS = ("lm_runtime.hip", "lm_corr.hip", "lm_bbox.hip")  # translation units of liblocomouse_hip.so


def _up_to_date(obj, cmd):
    """True when obj was built by the same command and is newer than every
    file its dependency list (hipcc -MMD) names."""
    try:
        with open(obj + ".cmd") as fh:
            if fh.read() != " ".join(cmd):
                return False
        with open(obj + ".d") as fh:
            deps = fh.read().replace("\\\n", " ").split(":", 1)[1].split()
        t = os.path.getmtime(obj)
        return all(os.path.getmtime(d) <= t for d in deps)
    except (OSError, IndexError):
        return False


def build(verbose=False, defines=(), out=None):
    """Compile liblocomouse_hip.so for gfx950 in-tree (hipcc cross-compiles
    without a GPU), then the host C++ LocoMouse mirror above it.  The
    translation units compile in parallel, then link into one library.
    `defines` / `out`: experiment builds (-D flags, another output path; the
    host mirror is then not rebuilt)."""
    objdir = os.path.join(ROOT, "build", "hip" if out is None else "hip_" + os.path.basename(out))
    os.makedirs(objdir, exist_ok=True)
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC, *["-D" + d for d in defines]]
    flags = [f for f in HIPCC_FLAGS if f != "-shared"]
    procs, objs = [], []
    for u in HIP_UNITS:
        o = os.path.join(objdir, u.replace(".hip", ".o"))
        cmd = ["hipcc", *flags, *inc, "-c", "-MMD", "-MF", o + ".d", "-o", o, os.path.join(CSRC, u)]
        objs.append(o)
        if _up_to_date(o, cmd):
            continue
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), cmd, o))
    for p, cmd, o in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
        with open(o + ".cmd", "w") as fh:
            fh.write(" ".join(cmd))
    target = out or LIB_PATH
    cmd = ["hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", target, *objs]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    if out is None:
        build_host(verbose)
    return target


def build_host(verbose=False):
    """liblocomouse_host.so: the LocoMouse / Candidate / P22D / MyMat C++
    surface (locomouse_cpp_amd/host) linked against the C-ABI library."""
    srcs = [os.path.join(HOST_DIR, f)
            for f in ("LocoMouse.cpp", "Tracks.cpp", "match2nd.cpp", "FileStorage.cpp", "Media.cpp", "Jpeg.cpp", "Debug.cpp")]
    flags = ["g++", "-O3", "-std=c++17", "-ffp-contract=off", "-pthread", "-Wall", "-Wextra", "-I" + os.path.join(ROOT, "include"),
             "-I" + HOST_DIR]
    cmd = [*flags, "-fPIC", "-shared", "-o", HOST_LIB_PATH, *srcs, "-L" + PKG, "-llocomouse_hip", "-lz",
           "-Wl,-rpath,$ORIGIN"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    # the reference's command-line program (main.cpp), SURVEY.md §8(f) row 2
    os.makedirs(os.path.dirname(CLI_PATH), exist_ok=True)
    cmd = [*flags, "-o", CLI_PATH, os.path.join(HOST_DIR, "Cli.cpp"), "-L" + PKG, "-llocomouse_host",
           "-llocomouse_hip", "-Wl,-rpath,$ORIGIN/.."]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return HOST_LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's):
        # load it first so this library and torch share one HIP runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run locomouse_cpp_amd.runtime.build() (no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        L.lm_abi_version.restype = C.c_int32
        L.lm_last_error.restype = C.c_char_p
        L.lm_ctx_create.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]
        L.lm_ctx_destroy.argtypes = [C.c_void_p]
        L.lm_get_geometry.argtypes = [C.c_void_p, C.POINTER(lm_geometry)]
        L.lm_ctx_stream.argtypes = [C.c_void_p]
        L.lm_ctx_stream.restype = C.c_void_p
        for fn in (L.lm_detect_batch, L.lm_detect_batch_device):
            fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p,
                           C.POINTER(lm_batch_result)]
        for fn in (L.lm_detect_submit, L.lm_detect_submit_device):
            fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.lm_detect_collect.argtypes = [C.c_void_p, C.POINTER(lm_batch_result)]
        for fn in (L.lm_ctx_lanes, L.lm_ctx_pending):
            fn.argtypes = [C.c_void_p]
            fn.restype = C.c_int32
        L.lm_ctx_set_debug.argtypes = [C.c_void_p, C.c_int32]
        L.lm_debug_scores.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.c_int32]
        L.lm_debug_tail_mask.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32]
        L.lm_debug_kernel_times.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_double), C.c_int32]
        L.lm_debug_kernel_times.restype = C.c_int32
        L.lm_debug_kernel_spans.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_double),
                                            C.POINTER(C.c_double), C.c_int32]
        L.lm_debug_kernel_spans.restype = C.c_int32
        L.lm_debug_corr_work.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        L.lm_debug_batch_slots.argtypes = [C.c_void_p]
        L.lm_debug_batch_slots.restype = C.c_int32
        L.lm_synth_frames_device.argtypes = [C.c_int32, C.c_void_p, C.c_int32, C.c_int32, C.c_int64, C.c_int32,
                                             C.c_int64]
        L.lm_bb_create.argtypes = [C.c_int32, C.c_void_p, C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]
        L.lm_bb_destroy.argtypes = [C.c_void_p]
        for fn in (L.lm_bb_push, L.lm_bb_push_device):
            fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int32, C.c_void_p]
        L.lm_bb_finish.argtypes = [C.c_void_p, C.POINTER(lm_bb_result)]
        L.lm_bb_debug_binary.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32, C.c_int32]
        L.lm_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p)]
        L.lm_host_free.argtypes = [C.c_void_p]
        L.lm_bb_stream.argtypes = [C.c_void_p]
        L.lm_bb_stream.restype = C.c_void_p
        _lib = L
    return _lib


class LMError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"lm status {code}: {msg}")
        self.code = code


def _check(rc):
    if rc != LM_OK:
        raise LMError(rc, lib().lm_last_error().decode())


def synth_frames_device(d_ptr, rows, cols, first, n, pitch, device=0):
    """Fill device memory with synthetic frames (bench/test input utility)."""
    _check(lib().lm_synth_frames_device(device, C.c_void_p(d_ptr), rows, cols, first, n, pitch))


class Context:
    """One lm_ctx on one HIP device (the per-frame loop's state)."""

    def __init__(self, cfg, max_batch=64, device=0, lanes=None):
        """lanes: pipeline lanes (lm_setup.pipeline_lanes; None keeps cfg.setup's)."""
        self.cfg = cfg  # keeps the arrays behind the structs alive
        self._h = C.c_void_p()
        setup = cfg.setup
        if lanes is not None:
            setup = type(cfg.setup).from_buffer_copy(cfg.setup)
            setup.pipeline_lanes = lanes
        self._setup = setup
        _check(lib().lm_ctx_create(device, C.byref(setup), C.byref(cfg.params), C.byref(cfg.model), max_batch,
                                   C.byref(self._h)))
        self.max_batch = max_batch

    def lanes(self):
        return lib().lm_ctx_lanes(self._h)

    def pending(self):
        return lib().lm_ctx_pending(self._h)

    def submit(self, frames, first_frame, prev_frame=None, bb=None):
        """Pipelined lm_detect_submit of host frames [n, rows, cols] u8."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        pp = None if prev_frame is None else np.ascontiguousarray(prev_frame, dtype=np.uint8)
        bbp = None if bb is None else np.ascontiguousarray(bb, dtype=np.int32)
        _check(lib().lm_detect_submit(self._h, frames.ctypes.data, frames.shape[1] * frames.shape[2], frames.shape[0],
                                      first_frame, None if pp is None else pp.ctypes.data,
                                      None if bbp is None else bbp.ctypes.data))

    def submit_device(self, d_frames_ptr, pitch, n, first_frame, d_prev_ptr=None, bb=None):
        """Pipelined lm_detect_submit_device (frames stay in device memory until collected)."""
        bbp = None if bb is None else np.ascontiguousarray(bb, dtype=np.int32)
        _check(lib().lm_detect_submit_device(self._h, C.c_void_p(d_frames_ptr), pitch, n, first_frame,
                                             C.c_void_p(d_prev_ptr) if d_prev_ptr else None,
                                             None if bbp is None else bbp.ctypes.data))

    def collect(self, raw=False):
        """Results of the oldest submitted batch (lm_detect_collect)."""
        res = lm_batch_result()
        _check(lib().lm_detect_collect(self._h, C.byref(res)))
        return res if raw else result_to_numpy(res)

    def geometry(self):
        g = lm_geometry()
        _check(lib().lm_get_geometry(self._h, C.byref(g)))
        return g

    def stream(self):
        return lib().lm_ctx_stream(self._h)

    def set_debug(self, flags):
        _check(lib().lm_ctx_set_debug(self._h, flags))

    def detect(self, frames, first_frame, prev_frame=None, bb=None, raw=False):
        """Host frames [n, rows, cols] u8 -> result dict (abi.result_to_numpy)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        n = frames.shape[0]
        res = lm_batch_result()
        pp = None
        if prev_frame is not None:
            self._prev = np.ascontiguousarray(prev_frame, dtype=np.uint8)
            pp = self._prev.ctypes.data
        bbp = None
        if bb is not None:
            self._bb = np.ascontiguousarray(bb, dtype=np.int32)
            bbp = self._bb.ctypes.data
        _check(lib().lm_detect_batch(self._h, frames.ctypes.data, frames.shape[1] * frames.shape[2], n, first_frame,
                                     pp, bbp, C.byref(res)))
        return res if raw else result_to_numpy(res)

    def detect_host_ptr(self, h_frames_ptr, pitch, n, first_frame, h_prev_ptr=None, raw=True):
        """lm_detect_batch on frames at a host address (e.g. a pinned torch
        tensor's data_ptr()): the H2D copy is part of the call."""
        res = lm_batch_result()
        _check(lib().lm_detect_batch(self._h, C.c_void_p(h_frames_ptr), pitch, n, first_frame,
                                     C.c_void_p(h_prev_ptr) if h_prev_ptr else None, None, C.byref(res)))
        return res if raw else result_to_numpy(res)

    def submit_host_ptr(self, h_frames_ptr, pitch, n, first_frame, h_prev_ptr=None):
        """Pipelined lm_detect_submit of frames at a host address (copied to
        the device before it returns)."""
        _check(lib().lm_detect_submit(self._h, C.c_void_p(h_frames_ptr), pitch, n, first_frame,
                                      C.c_void_p(h_prev_ptr) if h_prev_ptr else None, None))

    def detect_device(self, d_frames_ptr, pitch, n, first_frame, d_prev_ptr=None, bb=None, raw=True):
        """Frames already in device memory (e.g. a torch.cuda uint8 tensor's data_ptr())."""
        res = lm_batch_result()
        bbp = None
        if bb is not None:
            self._bb = np.ascontiguousarray(bb, dtype=np.int32)
            bbp = self._bb.ctypes.data
        _check(lib().lm_detect_batch_device(self._h, C.c_void_p(d_frames_ptr), pitch, n, first_frame,
                                            C.c_void_p(d_prev_ptr) if d_prev_ptr else None, bbp, C.byref(res)))
        return res if raw else result_to_numpy(res)

    def debug_scores(self, f, det):
        g = self.geometry()
        shapes = {0: (g.bb_bottom_mouse.height, g.bb_bottom_mouse.width), 1: (g.bb_bottom_mouse.height, g.bb_bottom_mouse.width),
                  2: (g.bb_bottom_mouse.height, g.tail_box_width), 3: (g.bb_side_mouse.height, g.bb_side_mouse.width),
                  4: (g.bb_side_mouse.height, g.bb_side_mouse.width), 5: (g.bb_side_mouse.height, g.tail_box_width)}
        out = np.zeros(shapes[det], dtype=np.float32)
        _check(lib().lm_debug_scores(self._h, f, det, out.ctypes.data, out.shape[0], out.shape[1]))
        return out

    def debug_tail_mask(self, f):
        g = self.geometry()
        out = np.zeros((g.bb_bottom_mouse.height, g.tail_box_width), dtype=np.uint8)
        _check(lib().lm_debug_tail_mask(self._h, f, out.ctypes.data, out.shape[0], out.shape[1]))
        return out

    def kernel_times(self):
        names = (C.c_char_p * 64)()
        ms = (C.c_double * 64)()
        n = lib().lm_debug_kernel_times(self._h, names, ms, 64)
        return [(names[i].decode(), ms[i]) for i in range(min(n, 64))]

    def kernel_spans(self):
        """[(name, t0_ms, t1_ms)] of the last batch against the device epoch."""
        names = (C.c_char_p * 64)()
        t0 = (C.c_double * 64)()
        t1 = (C.c_double * 64)()
        n = lib().lm_debug_kernel_spans(self._h, names, t0, t1, 64)
        return [(names[i].decode(), t0[i], t1[i]) for i in range(min(n, 64))]

    def corr_work(self):
        """Bright (computed) output tiles and their consumed outputs of the last
        batch, bottom and side point detectors (lm_debug_corr_work), or None."""
        out = (C.c_int32 * 4)()
        _check(lib().lm_debug_corr_work(self._h, out))
        return None if out[0] < 0 else {"tiles": (out[0], out[1]), "outputs": (out[2], out[3])}

    def batch_slots(self):
        """Frame slots the last collected batch processed (n, or n + 1 with
        its halo frame recomputed; lm_debug_batch_slots)."""
        return lib().lm_debug_batch_slots(self._h)

    @staticmethod
    def dark_tile_shape():
        """(columns, rows) of the dark-tile grid's tiles
        (lm_debug_dark_tile_width / _height)."""
        L = lib()  # (bound here, not at load: A/B runs load older libraries)
        return int(L.lm_debug_dark_tile_width()), int(L.lm_debug_dark_tile_height())

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().lm_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BBContext:
    """One lm_bb_ctx: the whole-video bounding-box pass (method 0,
    LocoMouse::computeBoundingBox, LocoMouse_class.cpp:579-653) on one HIP
    device.  Frames are pushed in video order; finish() post-processes."""

    def __init__(self, setup, bb_params, max_batch=64, device=0):
        self._setup, self._params = setup, bb_params  # keep the structs alive
        self._h = C.c_void_p()
        _check(lib().lm_bb_create(device, C.byref(setup), C.byref(bb_params), max_batch, C.byref(self._h)))
        self.max_batch = max_batch
        self.rows, self.cols = setup.calib_rows, setup.calib_cols

    def push(self, frames):
        """Host frames [n, rows, cols] u8 -> per-frame values (BB_FRAME_DTYPE)."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        out = np.zeros(frames.shape[0], dtype=BB_FRAME_DTYPE)
        _check(lib().lm_bb_push(self._h, frames.ctypes.data, frames.shape[1] * frames.shape[2], frames.shape[0],
                                out.ctypes.data))
        return out

    def push_device(self, d_frames_ptr, pitch, n, values=True):
        out = np.zeros(n, dtype=BB_FRAME_DTYPE) if values else None
        _check(lib().lm_bb_push_device(self._h, C.c_void_p(d_frames_ptr), pitch, n,
                                       out.ctypes.data if values else None))
        return out

    def finish(self):
        r = lm_bb_result()
        _check(lib().lm_bb_finish(self._h, C.byref(r)))
        n = r.n_frames

        def arr(ptr, dtype):
            return np.ctypeslib.as_array(ptr, shape=(n,)).astype(dtype).copy()
        per = np.frombuffer(C.cast(r.frames, C.POINTER(C.c_uint8 * (n * BB_FRAME_DTYPE.itemsize))).contents,
                            dtype=BB_FRAME_DTYPE, count=n).copy()
        return {"frames": per, "x_pos": arr(r.x_pos, np.uint32), "y_bottom_pos": arr(r.y_bottom_pos, np.uint32),
                "y_side_pos": arr(r.y_side_pos, np.uint32), "bb_side_mouse": r.bb_side_mouse.tuple(),
                "bb_bottom_mouse": r.bb_bottom_mouse.tuple()}

    def debug_binary(self, f):
        out = np.zeros((self.rows, self.cols), dtype=np.uint8)
        _check(lib().lm_bb_debug_binary(self._h, f, out.ctypes.data, self.rows, self.cols))
        return out

    def stream(self):
        return lib().lm_bb_stream(self._h)

    @staticmethod
    def dark_tile_shape():
        """(columns, rows) of the dark-tile grid's tiles
        (lm_debug_dark_tile_width / _height)."""
        L = lib()  # (bound here, not at load: A/B runs load older libraries)
        return int(L.lm_debug_dark_tile_width()), int(L.lm_debug_dark_tile_height())

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().lm_bb_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
