import sys, numpy as np
sys.path.insert(0, '/root/repo')
from locomouse_cpp_amd import synthetic as S
from oracle import oracle as O
cfg = S.SyntheticConfig()
for fn in sys.argv[1:]:
    raw = open(fn, 'rb').read()
    hd = np.frombuffer(raw[:68], np.int32); np_ = np.frombuffer(raw[68:84], np.int32)
    frame, slot, feat = (int(x) for x in hd[:3])
    print(fn, "frame", frame, "slot", slot, "feat", feat, "npos(k_corr)", np_, "hdr.n_pos", hd[5:9], "cand_cnt", hd[9:13], "ties", hd[13:17])
    g = O.geometry(cfg)
    caps = [g.bb_bottom_mouse.height*g.bb_bottom_mouse.width]*2 + [g.bb_side_mouse.height*g.bb_side_mouse.width]*2
    off = 84
    keys = []
    for l in range(4):
        k = np.frombuffer(raw[off:off+8*caps[l]], np.uint64); off += 8*caps[l]; keys.append(k)
    fr = cfg.frames(frame - 1, 2)
    ref = O.OracleRun(cfg, fr, flags=O.KEEP_DEBUG)
    res = ref.result
    for l in (0, 1):
        det = [0, 1][l]  # paw_b, snout_b
        sc = ref.scores(1, det, (g.bb_bottom_mouse.height, g.bb_bottom_mouse.width))
        ip = ref.ipad(1, None) if False else None
        pos = np.flatnonzero(sc.ravel() > 0)
        co = res["cand_offset"]; cands = res["cand"][co[4+l]:co[5+l]]
        nc = int(hd[9+l]); n = int(np_[l])
        k = keys[l][2*nc:n]  # raw keys past the staged candidates
        idx = (k & np.uint64(0xFFFFFFFF)).astype(np.int64)
        sbits = (~(k >> np.uint64(32))).astype(np.uint32)
        s = sbits.view(np.float32)
        bad = (idx >= caps[l]) | ~(s > 0)
        ok_scores = np.zeros(len(k), bool)
        good = ~bad
        ok_scores[good] = sc.ravel()[idx[good]] == s[good]
        print(f"  list {l}: oracle positives(score>0) {len(pos)} gpu npos {n}; oracle cands {len(cands)} gpu cand_cnt {nc}; raw keys checked {len(k)}: invalid {bad.sum()}, score mismatch {(good & ~ok_scores).sum()}")
        if bad.sum():
            w = np.flatnonzero(bad)[:5]
            print("    first invalid at", w + 2*nc, [hex(int(x)) for x in k[w]])
