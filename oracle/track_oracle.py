"""CPU restatement of the tracking stage — TEST
INFRASTRUCTURE ONLY.

Only tests/ import this module; the product path is the host C++ in
locomouse_cpp_amd/host/match2nd.cpp and LocoMouse.cpp.  Pure-Python loops,
meant for videos of tens to a few hundred frames.

What it restates, function by function (reference file:line):

* match2nd                 match2nd/match2nd.cpp:11-166 with the `point` /
                           `bundle` classes of match2nd/match2nd.h:29-563
* compute_cost_track       match2nd.cpp:168-190 (MATSPARSE::get returns 0
                           before its lookup, MyMat/MyMat.cpp:371-374, so only
                           the unary terms add up)
* pairwise_side            LocoMouse_class.cpp:2073-2150 (pairwisePotential_SideView)
* compute_bottom_tracks    LocoMouse_class.cpp:2153-2200 (4 of the 24 rows of
                           PAW_PERMUTATIONS, LocoMouse_class.hpp:91-92, are tried)
* best_side_view_match     LocoMouse_class.cpp:2216-2346 (+ computeSideTracks :2202-2214)
* export_results           LocoMouse_class.cpp:2348-2482 (exportPointTracks,
                           exportLineTracks)

Parity unpinned: the reference ships no tests or fixtures for the tracker and
cannot be compiled here (needs OpenCV).  The restatement is checked against
hand-built cases whose optimum is known (tests/test_tracks.py).
"""
import math

NEG_INF = -math.inf

# First four entries of rows 0-3 of PAW_PERMUTATIONS (a 4x24 CV_32S matrix read
# with ptr<int>(i_perm) for i_perm < N_paws, LocoMouse_class.cpp:2170-2171).
PAW_ORDERS = ((3, 2, 1, 0), (2, 3, 1, 0), (1, 2, 3, 0), (0, 2, 1, 3))


class TrackError(RuntimeError):
    pass


def _max(a, b):  # std::max(a, b): b only if a < b
    return b if a < b else a


def match2nd(unary, pairwise, nong, occ_cost, bam, frames, points, perm):
    """unary[f] = (nrows, ncols, column-major values); pairwise[f] = (nrows,
    ncols, jc, ir, pr) for the transition f -> f+1.  Returns points x frames
    labels (lists)."""
    T = [[0] * frames for _ in range(points)]
    if frames < 2 or points < 1:  # match2nd.cpp:24-27
        return T
    loc = []
    for f in range(frames):  # :40-60
        nr, nc, _ = unary[f]
        if nc != points:
            return T
        loc.append(nr)
    for f in range(frames - 1):  # :83-100 (size checks, silent zero result)
        nr, nc = pairwise[f][0], pairwise[f][1]
        if nr != loc[f + 1] + nong or nc != loc[f] + nong:
            return T
    L = frames
    jc = [pairwise[f][2] for f in range(L - 1)]
    ir = [pairwise[f][3] for f in range(L - 1)]
    pr = [pairwise[f][4] for f in range(L - 1)]
    nt = [int(pairwise[f][2][-1]) if len(pairwise[f][2]) else 0 for f in range(L - 1)]
    msg = [[0.0] * (loc[f] + nong) for f in range(L)]  # bundle: one message array shared by all points

    class Pt:
        pass

    pts = []
    for p in range(points):
        s = Pt()
        s.col = perm[p]
        s.fwd = [[NEG_INF] * nt[f] for f in range(L - 1)]
        s.bwd = [[NEG_INF] * nt[f] for f in range(L - 1)]
        s.lab = [0] * L
        s.best = [0.0] * L
        s.second = [0.0] * L
        s.bestloc = [0] * L
        pts.append(s)

    def un(s, a, b):  # point::un, match2nd.h:33-44
        if b < loc[a]:
            return unary[a][2][s.col * loc[a] + b] + msg[a][b]
        return occ_cost + msg[a][b]

    def clear(s):  # clearmargin
        s.lab = [-2] * L
        for f in range(L - 1):
            s.fwd[f] = [NEG_INF] * nt[f]
            s.bwd[f] = [NEG_INF] * nt[f]

    def forward_point(s, f):
        fw = s.fwd
        if f:
            for jj in range(nt[f - 1]):
                j = ir[f - 1][jj]
                for kk in range(jc[f][j], jc[f][j + 1]):
                    fw[f][kk] = _max(fw[f][kk], fw[f - 1][jj])
        else:
            for i in range(loc[0] + nong):
                for jj in range(jc[0][i], jc[0][i + 1]):
                    fw[0][jj] = un(s, 0, i)
        for i in range(nt[f]):
            fw[f][i] += un(s, f + 1, ir[f][i]) + pr[f][i]

    def backward_point(s, f):
        bw = s.bwd
        if f < L - 2:
            for jj in range(nt[f]):
                j = ir[f][jj]
                for kk in range(jc[f + 1][j], jc[f + 1][j + 1]):
                    bw[f][jj] = _max(bw[f][jj], bw[f + 1][kk])
        else:
            for jj in range(nt[f]):
                bw[f][jj] = un(s, f + 1, ir[f][jj])
        for i in range(loc[f] + nong):
            for jj in range(jc[f][i], jc[f][i + 1]):
                bw[f][jj] += pr[f][jj] + un(s, f, i)

    def findbest(s, f):
        s.best[f] = s.best[f + 1] = NEG_INF
        s.second[f] = s.second[f + 1] = NEG_INF
        lo = 0
        for i in range(nt[f]):
            while jc[f][lo + 1] <= i:
                lo += 1
            e = ir[f][i]
            temp = s.bwd[f][i] + s.fwd[f][i] - un(s, f, lo) - un(s, f + 1, e) - pr[f][i]
            if s.best[f] < temp:
                if s.bestloc[f] == lo:
                    s.best[f] = temp
                else:
                    s.second[f] = s.best[f]
                    s.best[f] = temp
                    s.bestloc[f] = lo
                if s.bestloc[f + 1] == e:
                    s.best[f + 1] = temp
                else:
                    s.second[f + 1] = s.best[f + 1]
                    s.best[f + 1] = temp
                    s.bestloc[f + 1] = e
            else:
                if s.second[f] < temp and s.bestloc[f] != lo:
                    s.second[f] = temp
                if s.second[f + 1] < temp and s.bestloc[f + 1] != e:
                    s.second[f + 1] = temp

    def forward_set(s, f):
        best = NEG_INF
        if f == 1:
            return
        if f == 0:
            for lo in range(loc[0] + nong):
                for i in range(jc[0][lo], jc[0][lo + 1]):
                    cost = s.bwd[0][i]
                    if best <= cost:
                        best = cost
                        s.lab[0] = lo
                        s.lab[1] = ir[0][i]
            if best == NEG_INF:
                s.lab[0] = s.lab[1] = -1
            return
        lo = 0
        for i in range(nt[f - 2]):
            while jc[f - 2][lo + 1] <= i:
                lo += 1
            j = ir[f - 2][i]
            if lo == s.lab[f - 2] and j == s.lab[f - 1]:
                for k in range(jc[f - 1][j], jc[f - 1][j + 1]):
                    cost = pr[f - 1][k] + s.bwd[f - 1][k]
                    if best < cost:
                        best = cost
                        s.lab[f] = ir[f - 1][k]
        if best == NEG_INF:
            s.lab[f] = -1

    def margin(s):
        clear(s)
        for f in range(L - 1):
            forward_point(s, f)
        for f in range(L - 2, -1, -1):
            backward_point(s, f)
        for f in range(L - 1):
            findbest(s, f)
        for f in range(L):  # update_unary_first
            if s.bestloc[f] < loc[f]:
                msg[f][s.bestloc[f]] += s.second[f] - s.best[f] - bam

    def assign(s):
        clear(s)
        for f in range(L):  # update_unary_second_pre
            if bam == math.inf:
                msg[f][s.bestloc[f]] = 0.0
            elif s.bestloc[f] < loc[f]:
                msg[f][s.bestloc[f]] += -s.second[f] + s.best[f] + bam
        for f in range(L - 2, -1, -1):
            backward_point(s, f)
        for f in range(L):
            forward_set(s, f)
        for f in range(L):  # update_unary_second
            if 0 <= s.lab[f] < loc[f]:
                msg[f][s.lab[f]] += NEG_INF

    for s in pts:  # bundle::run
        margin(s)
    for s in reversed(pts):
        assign(s)
    return [list(s.lab) for s in pts]


def compute_cost_track(M, unary, perm):
    """computeCostTrack (match2nd.cpp:168-190): tracks 0..3, unary terms only."""
    c = 0.0
    n_frames = len(M[0])
    for t in range(4):
        for f in range(n_frames):
            lab = M[t][f]
            nr, _, vals = unary[f]
            if lab < nr:
                idx = (perm[t] * nr + lab) & 0xFFFFFFFF  # MyMat::get(unsigned i, unsigned j)
                if idx >= len(vals):
                    raise TrackError("computeCostTrack reads outside the unary matrix (label -1 in column 0)")
                c += vals[idx]
            else:
                c += 0.0
    return c


def _csc(dense_cols, nrows):
    """MATSPARSE(&D): column by column, non-zero entries (MyMat.cpp:141-178)."""
    jc, ir, pr = [0], [], []
    for col in dense_cols:
        for r in range(nrows):
            v = col[r]
            if v != 0:
                ir.append(r)
                pr.append(v)
        jc.append(len(ir))
    return jc, ir, pr


def _round_half_away(x):  # C round(): x - trunc(x) is exact, so no x + 0.5 double rounding
    r = math.trunc(x)
    if abs(x - r) >= 0.5:
        r += 1 if x > 0 else -1
    return r


def pairwise_side(Zi, Zip1, grid_mapping, grid_spacing, nong, max_disp, alpha, poc):
    Ni, Nip1 = len(Zi), len(Zip1)
    occ = poc * alpha
    nrows, ncols = Nip1 + nong, Ni + nong
    D = [[0.0] * nrows for _ in range(ncols)]  # D[col][row]
    aux = nong - 1
    for i in range(Ni):
        z = int(_round_half_away((grid_mapping - float(Zi[i])) / grid_spacing))
        D[i][Nip1 + min(max(z, 0), aux)] = occ
        for j in range(Nip1):
            dist = abs(float(Zip1[j]) - float(Zi[i]))
            if dist < max_disp:
                D[i][j] = (1 - dist / max_disp) * alpha
    for j in range(Nip1):
        z = int(_round_half_away((grid_mapping - float(Zip1[j])) / grid_spacing))
        D[Ni + min(max(z, 0), aux)][j] = occ
    for i in range(nong):
        D[Ni + i][Nip1 + i] = occ
    jc, ir, pr = _csc(D, nrows)
    return (nrows, ncols, jc, ir, pr)


# ---- views of a result dict (locomouse_cpp_amd/results.py layout) ----

def unary_list(res, feature):
    ncols = 4 if feature == 0 else 1
    out = []
    for f in range(res["n_frames"]):
        lo, hi = int(res["unary_offset"][2 * f + feature]), int(res["unary_offset"][2 * f + feature + 1])
        vals = [float(v) for v in res["unary"][lo:hi]]
        out.append((len(vals) // ncols, ncols, vals))
    return out


def pairwise_list(res, feature):
    out = []
    for f in range(1, res["n_frames"]):
        k = 2 * f + feature
        nr, nc, nz = (int(v) for v in res["pw_dims"].reshape(-1)[3 * k:3 * k + 3])
        jlo = int(res["pw_jc_offset"][k])
        zlo = int(res["pw_nz_offset"][k])
        jc = [int(v) for v in res["pw_jc"][jlo:jlo + nc + 1]]
        ir = [int(v) for v in res["pw_ir"][zlo:zlo + nz]]
        pr = [float(v) for v in res["pw_pr"][zlo:zlo + nz]]
        out.append((nr, nc, jc, ir, pr))
    return out


def matched_list(res, feature):
    """Per frame, per bottom candidate: (x, y_bottom, side y list, side score
    list) of the P22D, with number_of_candidates() applied (st[0] < 0 -> none)."""
    out = []
    for f in range(res["n_frames"]):
        lo, hi = int(res["p22d_offset"][2 * f + feature]), int(res["p22d_offset"][2 * f + feature + 1])
        fr = []
        for p in res["p22d"][lo:hi]:
            so, sc = int(p["side_offset"]), int(p["side_count"])
            ys = [int(v) for v in res["side_y"][so:so + sc]]
            ss = [float(v) for v in res["side_s"][so:so + sc]]
            if ss and ss[0] < 0:
                ys, ss = [], []
            fr.append((int(p["x"]), int(p["y"]), ys, ss))
        out.append(fr)
    return out


def compute_bottom_tracks(res, nong, n_frames):
    up, pp = unary_list(res, 0), pairwise_list(res, 0)
    cur_cost, cur_perm, Mperm = -1.0, 0, None
    for ip, order in enumerate(PAW_ORDERS):
        M = match2nd(up, pp, nong, 0.0, 0.0, n_frames, 4, order)
        c = compute_cost_track(M, up, order)
        if c > cur_cost:
            cur_perm, cur_cost, Mperm = ip, c, M
    if Mperm is None:
        raise TrackError("no paw permutation scored above -1 (the reference asserts in Mat::row)")
    paw = [None] * 4
    for r in range(4):
        paw[PAW_ORDERS[cur_perm][r]] = list(Mperm[r])
    snout = match2nd(unary_list(res, 1), pairwise_list(res, 1), nong, 0.0, 0.0, n_frames, 1, (0,))
    return paw, snout


def best_side_view_match(T, matched, nong_side, lowest, spacing, max_disp, alpha, poc, n_frames):
    out = []
    for row in T:
        unary, pw, zprev = [], [], []
        for f in range(n_frames):
            lab = row[f]
            if 0 <= lab < len(matched[f]):
                _, _, ys, ss = matched[f][lab]
                Z = [y & 0xFFFFFFFF for y in ys]
                unary.append((len(ss), 1, list(ss)))
            else:
                Z = []
                unary.append((0, 1, []))
            if f > 0:
                pw.append(pairwise_side(zprev, Z, float(lowest), float(spacing), nong_side, float(max_disp), alpha, poc))
            zprev = Z
        out.append(match2nd(unary, pw, nong_side, 0.0, 0.0, n_frames, 1, (0,))[0])
    return out


def _i32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= (1 << 31) else v


def export_point_tracks(Tb, Ts, matched, bb, sizes, n_frames):
    """bb[f] = (BB_X_POS, BB_Y_BOTTOM_POS, BB_Y_SIDE_POS) (uint32); sizes =
    (W_bottom, H_bottom, H_side).  One N x 3 list per feature."""
    Wb, Hb, Hs = sizes
    out = []
    for i in range(len(Tb)):
        M = [[-1, -1, -1] for _ in range(n_frames)]
        for f in range(n_frames):
            lab = Tb[i][f]
            if 0 <= lab < len(matched[f]):
                x, yb, ys, _ = matched[f][lab]
                M[f][0] = _i32(bb[f][0] - Wb + 1 + x)
                M[f][1] = _i32(bb[f][1] - Hb + 1 + yb)
                ls = Ts[i][f]
                if ls < len(ys):
                    if ls < 0:
                        raise TrackError("side label -1 with side candidates (the reference reads yt[-1])")
                    M[f][2] = _i32(bb[f][2] - Hs + 1 + ys[ls])
        out.append(M)
    return out


def export_line_tracks(tail, bb, sizes, n_frames, n_points=15):
    """tail[f] = 3 x 15 ints; returns 3 x (15 N)."""
    Wb, Hb, Hs = sizes
    out = [[-1] * (n_points * n_frames) for _ in range(3)]
    for f in range(n_frames):
        for t in range(n_points):
            c = f * n_points + t
            if tail[f][0][t] >= 0:
                out[0][c] = _i32(bb[f][0] - Wb + 1 + tail[f][0][t])
            if tail[f][1][t] >= 0:
                out[1][c] = _i32(bb[f][1] - Hb + 1 + tail[f][1][t])
            if tail[f][2][t] >= 0:
                out[2][c] = _i32(bb[f][2] - Hs + 1 + tail[f][2][t])
    return out


def run_tracks(res, geom, params, bb, n_frames):
    """computeBottomTracks -> computeSideTracks -> exportResults over one
    video's result dict.  bb: per-frame BR corners (x, y_bottom, y_side)."""
    nong = geom.ong_nx * geom.ong_ny
    paw_b, snout_b = compute_bottom_tracks(res, nong, n_frames)
    side_args = (geom.n_ong_side, geom.ong_side_lowest, params.occlusion_grid_spacing_pixels_side,
                 params.max_displacement_side, params.alpha_vel_side, params.pairwise_occluded_cost, n_frames)
    mp, ms = matched_list(res, 0), matched_list(res, 1)
    paw_s = best_side_view_match(paw_b, mp, *side_args)
    snout_s = best_side_view_match(snout_b, ms, *side_args)
    sizes = (geom.bb_bottom_mouse.width, geom.bb_bottom_mouse.height, geom.bb_side_mouse.height)
    tail = [res["tail"][f].reshape(3, 15).tolist() for f in range(n_frames)]
    return {
        "track_index_paw_bottom": paw_b, "track_index_snout_bottom": snout_b,
        "track_index_paw_side": paw_s, "track_index_snout_side": snout_s,
        "paw_tracks": export_point_tracks(paw_b, paw_s, mp, bb, sizes, n_frames),
        "snout_tracks": export_point_tracks(snout_b, snout_s, ms, bb, sizes, n_frames),
        "tracks_tail": export_line_tracks(tail, bb, sizes, n_frames),
    }
