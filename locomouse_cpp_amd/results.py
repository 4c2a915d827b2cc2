"""Host-side handling of per-batch results (the dicts of abi.result_to_numpy).

A result dict holds the flat arrays of lm_batch_result for consecutive frames
(include/locomouse_hip.h).  The reference appends every frame's containers to
its vectors in frame order (LocoMouse_class.hpp:219-236); `concat_results`
does the same for batches and shards, `slice_results` drops leading frames
(a shard's halo frame).
"""
import numpy as np

KEYS = ("cand_offset", "cand", "p22d_offset", "p22d", "side_y", "side_s", "unary_offset", "unary", "pw_dims",
        "pw_jc_offset", "pw_jc", "pw_nz_offset", "pw_ir", "pw_pr", "tail")

# offset array -> (entries per frame, data arrays it indexes)
_OFFSETS = {
    "cand_offset": (4, ("cand",)),
    "p22d_offset": (2, ("p22d",)),
    "unary_offset": (2, ("unary",)),
    "pw_jc_offset": (2, ("pw_jc",)),
    "pw_nz_offset": (2, ("pw_ir", "pw_pr")),
}


def concat_results(parts):
    """Concatenate per-batch result dicts in order (offsets rebased)."""
    parts = list(parts)
    out = {}
    for k in KEYS:
        if k.endswith("offset"):
            acc, base = [np.zeros(1, np.int64)], 0
            for p in parts:
                acc.append(p[k][1:] + base)
                base += int(p[k][-1])
            out[k] = np.concatenate(acc)
        elif k == "p22d":
            arrs, base = [], 0
            for p in parts:
                a = p[k].copy()
                a["side_offset"] += base
                base += len(p["side_y"])
                arrs.append(a)
            out[k] = np.concatenate(arrs) if arrs else np.zeros(0, parts[0][k].dtype)
        else:
            out[k] = np.concatenate([p[k] for p in parts])
    out["n_frames"] = sum(p["n_frames"] for p in parts)
    out["first_frame"] = parts[0].get("first_frame", 0) if parts else 0
    return out


def slice_results(res, start):
    """The frames [start, n) of a result dict, rebased to start at 0."""
    n = res["n_frames"]
    assert 0 <= start <= n
    out = {"n_frames": n - start, "first_frame": res.get("first_frame", 0) + start}
    for k, (per, data) in _OFFSETS.items():
        off = res[k]
        lo, hi = int(off[per * start]), int(off[-1])
        out[k] = off[per * start:] - lo
        for d in data:
            out[d] = res[d][lo:hi]
    plo, phi = int(res["p22d_offset"][2 * start]), int(res["p22d_offset"][-1])
    p22d = res["p22d"][plo:phi].copy()
    side_lo = int(p22d["side_offset"].min()) if len(p22d) else len(res["side_y"])
    # side arrays of the dropped frames come first; P22D side offsets are
    # increasing in frame order, so the first kept entry marks the cut
    if len(p22d):
        p22d["side_offset"] -= side_lo
    out["p22d"] = p22d
    out["side_y"] = res["side_y"][side_lo:]
    out["side_s"] = res["side_s"][side_lo:]
    out["pw_dims"] = res["pw_dims"][start:]
    out["tail"] = res["tail"][start:]
    return out


def head_results(res, m):
    """The frames [0, m) of a result dict."""
    n = res["n_frames"]
    assert 0 <= m <= n
    if m == n:
        return res
    out = {"n_frames": m, "first_frame": res.get("first_frame", 0)}
    for k, (per, data) in _OFFSETS.items():
        off = res[k][:per * m + 1]
        out[k] = off
        for d in data:
            out[d] = res[d][:int(off[-1])]
    p22d = out["p22d"]
    # side arrays are laid out in frame order, so the kept frames' entries come first
    n_side = int((p22d["side_offset"] + p22d["side_count"]).max()) if len(p22d) else 0
    out["side_y"] = res["side_y"][:n_side]
    out["side_s"] = res["side_s"][:n_side]
    out["pw_dims"] = res["pw_dims"][:m]
    out["tail"] = res["tail"][:m]
    return out


def same_results(a, b):
    """True when two result dicts hold bit-identical arrays (every KEYS entry;
    structured arrays field by field, floats compared as stored)."""
    for k in KEYS:
        x, y = a[k], b[k]
        if x.shape != y.shape:
            return False
        if x.dtype.names:
            if not all(np.array_equal(x[n], y[n]) for n in x.dtype.names):
                return False
        elif not np.array_equal(x, y):
            return False
    return True
