"""scripts/trace_passes.py on a synthetic kernel trace: two passes of two
batches each, correlation in the middle of each pass, an idle gap between
the passes."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_trace_passes_split(tmp_path):
    hdr = '"Kind","Kernel_Name","Start_Timestamp","End_Timestamp"\n'
    rows = []
    for p0 in (0, 2_000_000):  # ns; pass length 1 ms, then 1 ms idle
        for b in (0, 400_000):
            rows.append(("k_minmax", p0 + b, p0 + b + 100_000))
            rows.append(("void k_corr_rw<24, false>(x)", p0 + b + 100_000, p0 + b + 500_000))
        rows.append(("k_out", p0 + 900_000, p0 + 1_000_000))
    path = tmp_path / "t.csv"
    path.write_text(hdr + "".join(f'"KERNEL_DISPATCH","{n}",{a},{b}\n' for n, a, b in rows))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "trace_passes.py"), str(path), "2"],
                         capture_output=True, text=True, check=True).stdout.splitlines()
    assert len(out) == 2, out
    assert out[0].startswith("pass 0: span 1.000 ms, any kernel 1.000, correlation 0.800")
    assert "idle before the next pass 1.000 ms" in out[0]
    assert out[1].startswith("pass 1: span 1.000 ms") and "idle before" not in out[1]
