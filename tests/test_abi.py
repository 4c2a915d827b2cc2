"""The C-ABI library loads and exports every function include/locomouse_hip.h
declares (no compute calls: runs without a GPU), and the ctypes mirror of
its structs has the header's layout."""
import ctypes as C
import os
import re
import subprocess

import pytest

from locomouse_cpp_amd import abi, runtime

HDR = os.path.join(runtime.ROOT, "include", "locomouse_hip.h")


def declared_functions():
    text = open(HDR).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(lm_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_entry_points():
    names = declared_functions()
    for must in ("lm_ctx_create", "lm_detect_batch", "lm_detect_batch_device", "lm_ctx_destroy", "lm_last_error"):
        assert must in names
    assert set(names) == set(runtime.EXPORTED)


def test_library_exports_every_declared_symbol():
    L = runtime.lib()
    for name in declared_functions():
        assert getattr(L, name) is not None
    assert L.lm_abi_version() == 6
    assert L.lm_debug_dark_tile_width() in (40, 80) and L.lm_debug_dark_tile_height() in (4, 8)


def test_last_error_and_null_arguments_without_gpu():
    L = runtime.lib()
    assert L.lm_ctx_create(0, None, None, None, 4, None) == abi.LM_ERR_INVALID_ARGUMENT
    assert b"out is NULL" in L.lm_last_error()
    out = C.c_void_p()
    assert L.lm_ctx_create(0, None, None, None, 0, C.byref(out)) == abi.LM_ERR_INVALID_ARGUMENT


@pytest.mark.parametrize("name", ["lm_rect", "lm_location_prior", "lm_params", "lm_detector", "lm_model", "lm_setup",
                                  "lm_geometry", "lm_candidate", "lm_p22d", "lm_batch_result",
                                  "lm_bb_params", "lm_bb_frame", "lm_bb_result"])
def test_struct_layout_matches_header(tmp_path, name):
    src = tmp_path / "sz.c"
    src.write_text(f'#include <stdio.h>\n#include "locomouse_hip.h"\nint main(void){{printf("%zu", sizeof({name}));}}\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I" + os.path.dirname(HDR), str(src), "-o", str(exe)])
    assert int(subprocess.check_output([str(exe)])) == C.sizeof(getattr(abi, name))
