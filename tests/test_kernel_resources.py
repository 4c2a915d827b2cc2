"""Register / scratch budget of every gfx950 kernel in liblocomouse_hip.so,
read from the code objects' metadata (no GPU needed).

The ring correlation (k_corr_rw) loads its pixel pairs with inline-asm
ds_read2_b32 and waits for them with an explicit s_waitcnt at each chunk
start; a spill or register copy of those pairs between issue and wait would
read stale LDS data unnoticed by the compiler.  So no kernel may spill VGPRs
or use scratch, and the width-specialised ring kernels must hold 5 waves per
SIMD (<= 96 VGPRs) with no SGPR spills either."""
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
LIB = os.path.join(ROOT, "locomouse_cpp_amd", "liblocomouse_hip.so")


@pytest.fixture(scope="module")
def kernels():
    if not os.path.exists(LIB):
        pytest.skip("liblocomouse_hip.so not built")
    import kernel_resources
    ks = kernel_resources.kernels(LIB)
    assert ks, "no kernel metadata found in the library"
    return ks


def test_no_vgpr_spills_or_scratch(kernels):
    bad = {k: r for k, r in kernels.items()
           if r.get("vgpr_spill_count", 0) or r.get("private_segment_fixed_size", 0)}
    assert not bad, f"kernels spilling VGPRs / using scratch: {bad}"


def test_ring_correlation_budget(kernels):
    ring = {k: r for k, r in kernels.items() if re.match(r"_Z9k_corr_rwILi\d+ELb[01]EE", k)}
    assert len(ring) >= 2 * 25, "expected the 25 ring widths x 2 arithmetic modes"
    for k, r in ring.items():
        kw = int(re.match(r"_Z9k_corr_rwILi(\d+)E", k).group(1))
        assert r["sgpr_spill_count"] == 0, (k, r)
        # 5 waves per SIMD up to kw 32; wider rings (>= 8.5 KB of LDS per
        # wave) run at most 4 waves per SIMD, which 128 VGPRs allow
        assert r["vgpr_count"] <= (96 if kw <= 32 else 128), (k, r)
