"""Instruction census of the loops of one kernel of a HIP shared library
(no GPU needed): for every backward branch (a loop), the count of each
instruction class between its target and the branch.

    python scripts/isa_census.py [lib.so] SYMBOL_SUBSTR

Classes: v_pk_fma (the correlation's FMAs), other VALU, ds_read / ds_write,
global / buffer loads and stores, s_load (scalar memory), other SALU,
s_waitcnt, branches."""
import os
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kernel_resources as KR  # noqa: E402


def klass(t):
    op = t.split()[0]
    if op.startswith("v_pk_fma") or op.startswith("v_pk_mul") or op.startswith("v_pk_add"):
        return "v_pk_fma/mul/add"
    if op.startswith("v_"):
        return "valu_other"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_"):
        return "ds_write/other"
    if op.startswith("global_load") or op.startswith("buffer_load") or op.startswith("flat_load"):
        return "vmem_load"
    if op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
        return "vmem_store/atomic"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "s_load"
    if op.startswith("s_waitcnt"):
        return "s_waitcnt"
    if "branch" in op:
        return "branch"
    if op.startswith("s_"):
        return "salu_other"
    return "other"


def census(lib, sym):
    out = []
    for name, items in KR.disassemble_cfg(lib, sym).items():
        addr = [a for a, _, _ in items]
        for i, (a, t, b) in enumerate(items):
            if b is not None and b <= a:  # backward branch: a loop [b, a]
                j = addr.index(b) if b in addr else None
                if j is None:
                    continue
                body = [items[k][1] for k in range(j, i + 1)]
                out.append((name, b, a, len(body), Counter(klass(x) for x in body)))
    return out


def main():
    args = sys.argv[1:]
    lib = args.pop(0) if args and args[0].endswith(".so") else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "locomouse_cpp_amd", "liblocomouse_hip.so")
    sym = args[0]
    for name, b, a, n, c in census(lib, sym):
        if n < 40:
            continue
        print(f"{name[:60]} loop {b:#x}..{a:#x}: {n} instructions")
        for k, v in sorted(c.items(), key=lambda kv: -kv[1]):
            print(f"    {k:18s} {v}")


if __name__ == "__main__":
    main()
