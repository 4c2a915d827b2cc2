import sys, numpy as np
sys.path.insert(0, '/root/repo')
from locomouse_cpp_amd import synthetic as S
from oracle import oracle as O
cfg = S.SyntheticConfig()
g = O.geometry(cfg)
for frame in [int(x) for x in sys.argv[1:]]:
    ref = O.OracleRun(cfg, cfg.frames(frame - 1, 2), flags=O.KEEP_DEBUG)
    for det in (0, 1):
        sc = ref.scores(1, det, (g.bb_bottom_mouse.height, g.bb_bottom_mouse.width)).ravel()
        pos = sc[sc > 0]
        u, c = np.unique(pos, return_counts=True)
        print(frame, "det", det, "positives", len(pos), "duplicate score values", int((c > 1).sum()), u[c > 1][:5])
