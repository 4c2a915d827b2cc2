"""ctypes access to tests/cpp/host_harness.cpp, which drives the host C++
LocoMouse mirror (locomouse_cpp_amd/host) in main.cpp's call order."""
import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "locomouse_cpp_amd")
SO = os.path.join(HERE, "cpp", "_build", "libhost_harness.so")


def build(verbose=False):
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(PKG, "host"), "-o", SO, os.path.join(HERE, "cpp", "host_harness.cpp"), "-L" + PKG,
           "-llocomouse_host", "-llocomouse_hip", "-Wl,-rpath,$ORIGIN/../../../locomouse_cpp_amd"]
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    return SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        from locomouse_cpp_amd import runtime
        runtime.lib()  # torch's HIP runtime first, then the C-ABI library
        if not os.path.exists(SO):
            raise RuntimeError(f"{SO} is missing: run tests/host_harness.build()")
        L = C.CDLL(SO)
        L.lmh_run.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int,
                              C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p, C.c_int]
        L.lmh_run.restype = C.c_int
        L.lmh_set_output.argtypes = [C.c_char_p]
        L.lmh_set_devices.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.lmh_read_png.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]
        L.lmh_read_avi.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int]
        L.lmh_fs_node.argtypes = [C.c_char_p, C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_int64, C.c_char_p, C.c_int]
        L.lmh_get_tracks.argtypes = [C.c_int] + [C.c_void_p] * 5
        L.lmh_fs_write_demo.argtypes = [C.c_char_p]
        L.lmh_selftest.argtypes = [C.c_char_p, C.c_int]
        L.lmh_selftest.restype = C.c_int
        _lib = L
    return _lib


class HostError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{'invalid_argument' if code == 1 else 'runtime_error'}: {msg}")
        self.code = code


def run_video(cfg, frames, batch=8, device=0, n_frames=None, call_order=0, bb_params=None, with_bb=False,
              devices=None, oversubscribe=False):
    """LocoMouse_Initialize + main.cpp's loop over `frames`; returns the
    result containers as a result dict (abi.result_to_numpy layout).
    bb_params: lm_bb_params for the whole-video BB pass (used when
    cfg.params.use_provided_bounding_box == 0); with_bb also returns the
    corners [n][3] (x, y_bottom, y_side) and the (side, bottom) box sizes.
    devices / oversubscribe: LocoMouse_Inputs::devices (multi-GPU shards)."""
    import numpy as np
    from locomouse_cpp_amd.abi import lm_batch_result, lm_rect, result_to_numpy
    frames = np.ascontiguousarray(frames, dtype=np.uint8)
    out = lm_batch_result()
    err = C.create_string_buffer(512)
    n = frames.shape[0] if n_frames is None else n_frames
    corners = np.zeros((n, 3), dtype=np.uint32)
    sizes = (lm_rect * 2)()
    devs = np.ascontiguousarray(devices or [], dtype=np.int32)
    lib().lmh_set_devices(devs.ctypes.data, len(devs), int(oversubscribe))
    try:
        rc = lib().lmh_run(C.byref(cfg.setup), C.byref(cfg.params), C.byref(cfg.model),
                           C.byref(bb_params) if bb_params is not None else None, frames.ctypes.data, n,
                           frames.shape[0], batch, device, call_order, C.byref(out), corners.ctypes.data, sizes, err,
                           512)
    finally:
        lib().lmh_set_devices(None, 0, 0)
    if rc:
        raise HostError(rc, err.value.decode())
    res = result_to_numpy(out)
    if with_bb:
        return res, corners, (sizes[0].tuple(), sizes[1].tuple())
    return res


def run_video_tracks(cfg, frames, batch=8, device=0, output_file=None, devices=None, oversubscribe=False):
    """run_video with main.cpp's post-loop calls (computeBottomTracks,
    computeSideTracks, exportResults): returns (result dict, tracks dict,
    corners)."""
    import numpy as np
    lib().lmh_set_output(os.fsencode(output_file) if output_file else None)
    try:
        res, corners, _ = run_video(cfg, frames, batch=batch, device=device, call_order=4, with_bb=True,
                                    devices=devices, oversubscribe=oversubscribe)
    finally:
        lib().lmh_set_output(None)
    n = res["n_frames"]
    t = {"paw_tracks": np.zeros((4, n, 3), np.int32), "snout_tracks": np.zeros((1, n, 3), np.int32),
         "tracks_tail": np.zeros((3, 15 * n), np.int32), "track_index_bottom": np.zeros((5, n), np.int32),
         "track_index_side": np.zeros((5, n), np.int32)}
    rc = lib().lmh_get_tracks(n, *(t[k].ctypes.data for k in ("paw_tracks", "snout_tracks", "tracks_tail",
                                                               "track_index_bottom", "track_index_side")))
    if rc:
        raise HostError(2, "no tracks recorded")
    return res, t, corners


def selftest():
    err = C.create_string_buffer(512)
    rc = lib().lmh_selftest(err, 512)
    if rc:
        raise HostError(rc, err.value.decode())
