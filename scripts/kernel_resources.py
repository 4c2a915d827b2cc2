"""Per-kernel resource usage of the gfx950 code objects inside a HIP shared
library: VGPR / SGPR counts, spills and scratch (private segment) bytes, read
from the code objects' AMDGPU metadata notes.

    python scripts/kernel_resources.py [lib.so] [--filter SUBSTR]

Used by tests/test_kernel_resources.py (no GPU needed)."""
import os
import re
import struct
import subprocess
import sys
import tempfile

READELF = "/opt/rocm/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(path, name):
    """Bytes of ELF section `name` (64-bit little-endian ELF)."""
    with open(path, "rb") as fh:
        data = fh.read()
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    stro = sh(shstrndx)[4]
    for i in range(shnum):
        s = sh(i)
        nm = data[stro + s[0]:data.index(b"\0", stro + s[0])].decode()
        if nm == name:
            return data[s[4]:s[4] + s[5]]
    raise KeyError(name)


def code_objects(lib):
    """The amdgcn code objects of every offload bundle in lib's .hip_fatbin."""
    fb = _section(lib, ".hip_fatbin")
    out = []
    pos = fb.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fb, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fb, p)
            triple = fb[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "amdgcn" in triple and size:
                out.append(fb[pos + off:pos + off + size])
        pos = fb.find(MAGIC, pos + 32)
    return out


def kernels(lib):
    """{kernel symbol: {field: value}} for every kernel of lib."""
    res = {}
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as fh:
            fh.write(co)
            name = fh.name
        try:
            txt = subprocess.run([READELF, "--notes", name], capture_output=True, text=True, check=True).stdout
        finally:
            os.unlink(name)
        cur = None
        for line in txt.splitlines():
            m = re.match(r"\s*-?\s*\.(\w+):\s+(.*)$", line)
            if not m:
                continue
            key, val = m.group(1), m.group(2).strip()
            if key == "name" and not val.endswith(".kd"):
                cur = {}
                res[val] = cur
                continue
            if cur is not None and key in ("vgpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                                           "private_segment_fixed_size", "group_segment_fixed_size", "agpr_count"):
                cur[key] = int(val)
    return res


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "locomouse_cpp_amd", "liblocomouse_hip.so")
    flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
    ks = kernels(lib)
    print(f"{'kernel':70s} {'vgpr':>5s} {'sgpr':>5s} {'vspill':>6s} {'sspill':>6s} {'scratch':>7s}")
    for k in sorted(ks):
        if flt not in k:
            continue
        r = ks[k]
        print(f"{k[:70]:70s} {r.get('vgpr_count', -1):5d} {r.get('sgpr_count', -1):5d} {r.get('vgpr_spill_count', -1):6d} "
              f"{r.get('sgpr_spill_count', -1):6d} {r.get('private_segment_fixed_size', -1):7d}")


if __name__ == "__main__":
    main()


OBJDUMP = "/opt/rocm/llvm/bin/llvm-objdump"


def disassemble(lib, symbol_filter):
    """{function symbol: [instruction text]} of the code objects' functions
    whose names contain symbol_filter (llvm-objdump, no GPU needed)."""
    return {k: [t for _, t, _ in v] for k, v in disassemble_cfg(lib, symbol_filter).items()}


def disassemble_cfg(lib, symbol_filter):
    """{function symbol: [(address, instruction text, branch target address
    or None)]}, for control-flow aware checks."""
    out = {}
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as fh:
            fh.write(co)
            name = fh.name
        try:
            txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", name], capture_output=True, text=True,
                                 check=True).stdout
        finally:
            os.unlink(name)
        cur = None
        for line in txt.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                cur = m.group(1) if symbol_filter in m.group(1) else None
                if cur is not None:
                    out[cur] = []
                continue
            if cur is not None:
                ins, _, comment = line.partition("//")
                ins = ins.strip()
                if ins:
                    ma = re.match(r"\s*([0-9A-Fa-f]+):", comment)
                    mt = re.search(r"<[^>+]+\+0x([0-9a-f]+)>", comment)
                    addr = int(ma.group(1), 16) if ma else None
                    out[cur].append((addr, ins, mt and int(mt.group(1), 16)))
    # branch targets are function-relative: make them absolute
    for k, items in out.items():
        base = items[0][0] if items and items[0][0] is not None else 0
        out[k] = [(a, t, None if b is None or not t.startswith("s_") or "branch" not in t else base + b)
                  for a, t, b in items]
    return out


def _vregs(operand):
    """VGPR numbers an operand names (v7, v[4:5])."""
    m = re.fullmatch(r"v(\d+)", operand)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", operand)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def _lds_pair_step(ins, pending, bad):
    """One instruction of early_reads_of_lds_pairs' scan: returns the pending
    set after it (appending ins to bad when it reads a pending register)."""
    op, _, rest = ins.partition(" ")
    ops = [o.strip() for o in rest.split(",")] if rest else []
    if op.startswith("s_waitcnt") and ("lgkmcnt(0)" in rest or "lgkmcnt" not in rest and "vmcnt" not in rest
                                       and "expcnt" not in rest):
        return frozenset()
    srcs = set()
    for o in ops[1:] if ops else []:
        srcs |= _vregs(o.split()[0]) if o else set()
    if op.startswith("ds_write") or op.startswith("ds_read") or op.startswith("global_store"):
        # stores read their data/address operands; a ds_read2 reads its address (operand 1)
        srcs = set().union(*[_vregs(o.split()[0]) for o in ops[1:] if o]) if op.startswith(("ds_write", "global_store")) \
            else (_vregs(ops[1].split()[0]) if len(ops) > 1 else set())
    if srcs & pending and bad is not None:
        bad.append(ins)
    # a write to a pending destination (WAW): the late LDS return would
    # overwrite the new value (a dead read's registers reused by the
    # compiler).  Another LDS read into them is fine: a wave's LDS reads
    # return in order.
    if ops and bad is not None and (op.startswith("v_") or
                                    op.startswith(("global_load", "buffer_load", "flat_load"))):
        if _vregs(ops[0].split()[0]) & pending:
            bad.append("WAW " + ins)
    if op == "ds_read2_b32" and ops:
        return pending | _vregs(ops[0])
    if ops and op.startswith("v_"):
        return pending - _vregs(ops[0])  # overwritten: no longer the load's destination
    return pending


def _sregs(operand):
    """SGPR numbers an operand names (s7, s[4:5])."""
    m = re.fullmatch(r"s(\d+)", operand)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", operand)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def _flag_step(ins, consts, vcc):
    """Constant tracking for the compiler's boolean-flag branches: an SGPR
    pair set to 0 / -1 (s_mov_b64), VCC computed from it with EXEC
    (s_and_b64 / s_andn2_b64 vcc, exec, s[a:b]).  Returns (consts, vcc): vcc
    is "zero", "nonzero" or None (unknown).  Conservative: any other
    instruction naming VCC makes it unknown, and any instruction naming an
    SGPR of a tracked pair (as its first operand, or any operand of a vector
    instruction) forgets that pair."""
    op, _, rest = ins.partition(" ")
    ops = [o.strip().split(" ")[0] for o in rest.split(",")] if rest else []
    if not ops:
        return consts, vcc
    if op == "s_mov_b64" and len(ops) == 2 and ops[1] in ("0", "-1") and ops[0].startswith("s["):
        d = _sregs(ops[0])
        keep = frozenset(kv for kv in consts if not (_sregs(kv[0]) & d))
        return keep | {(ops[0], int(ops[1]))}, vcc
    if op in ("s_and_b64", "s_andn2_b64") and len(ops) == 3 and ops[0] == "vcc" and ops[1] == "exec":
        c = dict(consts).get(ops[2])
        if c is None:
            return consts, None
        on = (c == -1) if op == "s_and_b64" else (c == 0)  # EXEC is never zero where the branch executes
        return consts, "nonzero" if on else "zero"
    if any(o.startswith("vcc") for o in ops):
        vcc = None
    touched = set()
    for o in (ops if op.startswith("v_") else ops[:1]):
        touched |= _sregs(o)
    if touched:
        consts = frozenset(kv for kv in consts if not (_sregs(kv[0]) & touched))
    return consts, vcc


def early_reads_of_lds_pairs(instrs):
    """Instructions that read -- or write ("WAW ...", except another LDS read) --
    a VGPR written by a ds_read2_b32 before an s_waitcnt that drains the LDS
    counter (lgkmcnt(0)) has executed, on some control-flow path.  The ring correlation issues those reads as inline asm
    the compiler's wait insertion does not see, so a register copy or use
    before the explicit wait would read stale data.  instrs: disassemble_cfg
    items (address, text, branch target) -- a forward may-analysis over the
    branches -- or plain instruction texts (scanned in program order).  The
    CFG analysis is path-sensitive for one pattern the compiler uses to merge
    control flow: a flag SGPR pair set to 0 or -1 on each incoming path and a
    VCC branch on it (s_mov_b64 s[a:b], -1 / s_andn2_b64 vcc, exec, s[a:b] /
    s_cbranch_vccnz); a path whose flag decides the branch the other way is
    not followed."""
    if not instrs or isinstance(instrs[0], str):
        pending, bad = frozenset(), []
        for ins in instrs:
            pending = _lds_pair_step(ins, pending, bad)
        return bad
    idx = {a: i for i, (a, _, _) in enumerate(instrs)}
    n = len(instrs)

    def succs(i, vcc):
        _, t, tgt = instrs[i]
        op = t.split(" ")[0]
        if op in ("s_endpgm", "s_setpc_b64", "s_trap"):
            return []
        nxt = [i + 1] if i + 1 < n else []
        if tgt is not None and tgt in idx:
            if op == "s_branch":
                return [idx[tgt]]
            if op == "s_cbranch_vccnz" and vcc is not None:
                return [idx[tgt]] if vcc == "nonzero" else nxt
            if op == "s_cbranch_vccz" and vcc is not None:
                return [idx[tgt]] if vcc == "zero" else nxt
            return [idx[tgt]] + nxt
        return nxt

    CAP = 64  # states kept per instruction before they are merged (the analysis stays sound)
    states = [set() for _ in range(n)]
    states[0].add((frozenset(), frozenset(), None))
    work = [(0, (frozenset(), frozenset(), None))]
    while work:
        i, (pend, consts, vcc) = work.pop()
        out = _lds_pair_step(instrs[i][1], pend, None)
        c2, v2 = _flag_step(instrs[i][1], consts, vcc)
        for j in succs(i, v2):
            st = (out, c2, v2)
            if st in states[j]:
                continue
            if len(states[j]) >= CAP:  # collapse: one state with every pending register, no flags
                allp = frozenset().union(out, *[s_[0] for s_ in states[j]])
                st = (allp, frozenset(), None)
                if st in states[j]:
                    continue
                states[j] = {st}
            else:
                states[j].add(st)
            work.append((j, st))
    bad = []
    for i in range(n):
        pend = frozenset().union(*[s_[0] for s_ in states[i]]) if states[i] else None
        if pend is not None:
            _lds_pair_step(instrs[i][1], pend, bad)
    return bad
