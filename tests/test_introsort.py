"""The GPU's std::sort replica (locomouse_cpp_amd/csrc/lm_introsort.h) against
libstdc++ std::sort on tie-heavy inputs, including the depth-limit heap path.
Compiled for the host with g++ (the same header is used in device code)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_introsort_replica_matches_libstdcxx(tmp_path):
    exe = str(tmp_path / "isc")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I" + os.path.join(ROOT, "locomouse_cpp_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "introsort_check.cpp"), "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "fails=0" in out.stdout
