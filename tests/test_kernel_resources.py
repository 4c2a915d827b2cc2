"""Register / scratch budget of every gfx950 kernel in liblocomouse_hip.so,
read from the code objects' metadata, and the ring correlation's LDS-wait
discipline, read from their disassembly (llvm-objdump; no GPU needed).

The ring correlation (k_corr_rw) loads its pixel pairs with inline-asm
ds_read2_b32 and waits for them with an explicit s_waitcnt at each chunk
start; a spill or register copy of those pairs between issue and wait would
read stale LDS data unnoticed by the compiler.  So no kernel may spill VGPRs
or use scratch, the width-specialised ring kernels must hold the 4 waves per
SIMD their LDS rings allow (<= 128 VGPRs) with no SGPR spill
(to VGPR lanes) inside a loop of v_pk_fma_f32, and in every ring kernel no
instruction may read a VGPR a ds_read2_b32 wrote before the next
s_waitcnt lgkmcnt(0), nor write it (a dead read's registers reused by the
compiler are overwritten when the read returns; test_ring_reads_wait_for_lds)."""
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
    hot = _lane_spills_in_fma_loops()
    for k, r in ring.items():
        kw = int(re.match(r"_Z9k_corr_rwILi(\d+)E", k).group(1))
        # SGPRs spilled to VGPR lanes (v_writelane / v_readlane, no memory)
        # are allowed around the step loop, never inside it
        assert not hot.get(k), (k, r, hot.get(k))
        # eight 40 x 4 sub-tiles per wave: the rings (~9.5 KB of LDS per wave
        # at kw 30) allow at most 4 waves per SIMD, which 128 VGPRs allow;
        # the wider kernels' rings allow fewer (lm_corr.h rw_ring_floats)
        assert r["vgpr_count"] <= _ring_vgpr_budget(kw), (k, r, _ring_vgpr_budget(kw))


def _lane_spills_in_fma_loops():
    """{ring kernel: [SGPR spill code (v_writelane, or v_readlane of a VGPR
    some v_writelane fills) inside an innermost loop holding v_pk_fma_f32]}.
    A loop is a backward branch's address range; the innermost ones hold no
    other such range (the step loops; the CFG's outer ranges span the whole
    kernel)."""
    import kernel_resources
    out = {}
    for name, ins in kernel_resources.disassemble_cfg(LIB, "k_corr_rw").items():
        addr = [a for a, _, _ in ins]
        spill_v = {t.split()[1].rstrip(",") for _, t, _ in ins if t.startswith("v_writelane")}
        loops = []
        for i, (a, t, b) in enumerate(ins):
            if b is not None and b <= a and b in addr:
                j = addr.index(b)
                if any(x.startswith("v_pk_fma_f32") for _, x, _ in ins[j:i + 1]):
                    loops.append((j, i))
        inner = [(j, i) for j, i in loops if not any(j <= j2 and i2 <= i and (j2, i2) != (j, i) for j2, i2 in loops)]
        bad = []
        for j, i in inner:
            for _, t, _ in ins[j:i + 1]:
                if t.startswith("v_writelane") or (t.startswith("v_readlane") and t.split()[2].rstrip(",") in spill_v):
                    bad.append(t)
        if bad:
            out[name] = bad[:4]
    return out


def _ring_vgpr_budget(kw, fw=40, hs=3, nq=8, waves_per_wg=4):
    """VGPRs a k_corr_rw<kw> wave may use without lowering the occupancy its
    LDS rings allow (a 4-wave workgroup puts one wave on each SIMD)."""
    stride = (fw + kw - 1 + 6) // 4 * 4
    qpitch = (hs + 1) * stride + ((fw // 5 - ((hs + 1) * stride) % 32) + 32) % 32
    wg_bytes = waves_per_wg * nq * qpitch * 4
    waves = min(4, (160 * 1024) // wg_bytes)  # per SIMD (the kernels ask for at most 4)
    return 512 // waves // 8 * 8


def test_ring_reads_wait_for_lds():
    import kernel_resources
    if not os.path.exists(LIB):
        pytest.skip("liblocomouse_hip.so not built")
    funcs = kernel_resources.disassemble_cfg(LIB, "k_corr_rw")
    assert len(funcs) >= 2 * 25 + 2, sorted(funcs)[:4]
    for name, ins in funcs.items():
        assert sum(1 for _, i, _ in ins if i.startswith("ds_read2_b32")) > 0, name
        assert any(t is not None for _, _, t in ins), name  # branch targets parsed
        bad = kernel_resources.early_reads_of_lds_pairs(ins)
        assert not bad, (name, bad[:4])


def test_lds_wait_checker_flags_an_early_read():
    import kernel_resources
    ok = ["ds_read2_b32 v[2:3], v9 offset0:1 offset1:117", "s_waitcnt lgkmcnt(0)",
          "v_pk_fma_f32 v[4:5], s[8:9], v[2:3], v[4:5] op_sel_hi:[0,1,1]"]
    early = ["ds_read2_b32 v[2:3], v9 offset0:1 offset1:117", "v_mov_b32_e32 v10, v3", "s_waitcnt lgkmcnt(0)"]
    overwritten = ["ds_read2_b32 v[2:3], v9 offset0:1 offset1:117", "s_waitcnt lgkmcnt(0)", "v_mov_b32_e32 v2, v7",
                   "v_add_u32_e32 v11, v2, v1"]
    assert kernel_resources.early_reads_of_lds_pairs(ok) == []
    assert kernel_resources.early_reads_of_lds_pairs(early) == ["v_mov_b32_e32 v10, v3"]
    assert kernel_resources.early_reads_of_lds_pairs(overwritten) == []


def test_lds_wait_checker_follows_branches():
    import kernel_resources
    # a use reached by a branch around the ds_read2 is fine; a path through it
    # without a wait is not, wherever the blocks are laid out
    ok = [(0, "s_cbranch_scc1 2", 12), (4, "ds_read2_b32 v[2:3], v9 offset0:1 offset1:117", None),
          (8, "s_waitcnt lgkmcnt(0)", None), (12, "v_mov_b32_e32 v10, v3", None), (16, "s_endpgm", None)]
    bad = [(0, "s_cbranch_scc1 2", 12), (4, "ds_read2_b32 v[2:3], v9 offset0:1 offset1:117", None),
           (8, "s_nop 0", None), (12, "v_mov_b32_e32 v10, v3", None), (16, "s_endpgm", None)]
    laid_out = [(0, "s_branch 3", 16), (4, "ds_read2_b32 v[2:3], v9 offset0:1 offset1:117", None),
                (8, "s_nop 0", None), (12, "s_endpgm", None), (16, "v_mov_b32_e32 v10, v3", None),
                (20, "s_endpgm", None)]
    assert kernel_resources.early_reads_of_lds_pairs(ok) == []
    assert kernel_resources.early_reads_of_lds_pairs(bad) == ["v_mov_b32_e32 v10, v3"]
    assert kernel_resources.early_reads_of_lds_pairs(laid_out) == []  # program order alone would flag it


def test_lds_wait_checker_flag_branches():
    """The compiler merges paths through a flag SGPR pair (s_mov_b64 s[6:7],
    0 / -1; s_andn2_b64 vcc, exec, s[6:7]; s_cbranch_vccnz): a path whose
    flag sends the branch the other way is not followed, one whose flag is
    unknown is."""
    import kernel_resources
    rd = "ds_read2_b32 v[24:25], v9 offset0:1 offset1:117"

    def prog(flag_init):
        # 0: ds_read2 in flight; 1: flag; 2: branch to 4 (the merge) ...
        return [(0, rd, None), (4, flag_init, None), (8, "s_branch 1", 16),
                (12, "s_waitcnt lgkmcnt(0)", None),
                (16, "s_andn2_b64 vcc, exec, s[6:7]", None), (20, "s_cbranch_vccnz 2", 32),
                (24, "s_waitcnt lgkmcnt(0)", None), (28, "s_endpgm", None),
                (32, "v_mov_b32_e32 v24, 0", None), (36, "s_endpgm", None)]
    # flag -1: vcc = exec & ~(-1) = 0, the branch to the write is not taken
    assert kernel_resources.early_reads_of_lds_pairs(prog("s_mov_b64 s[6:7], -1")) == []
    # flag 0: vcc = exec, the write follows the pending read
    assert kernel_resources.early_reads_of_lds_pairs(prog("s_mov_b64 s[6:7], 0")) == ["WAW v_mov_b32_e32 v24, 0"]
    # flag unknown (a compare result): both ways
    assert kernel_resources.early_reads_of_lds_pairs(prog("v_cmp_ne_u32_e64 s[6:7], v1, v2")) == \
        ["WAW v_mov_b32_e32 v24, 0"]
