// Tracks.cpp — see Tracks.hpp.  Every function cites the reference code whose
// results it reproduces.
#include "Tracks.hpp"

#include "FileStorage.hpp"

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <fstream>
#include <future>
#include <stdexcept>

namespace locomouse {

const int PAW_ORDERS[4][4] = {{3, 2, 1, 0}, {2, 3, 1, 0}, {1, 2, 3, 0}, {0, 2, 1, 3}};

void FrameResults::append(const lm_batch_result& r) {
  auto list = [&](int f, int k) {
    const lm_candidate* b = r.cand + r.cand_offset[4 * f + k];
    const lm_candidate* e = r.cand + r.cand_offset[4 * f + k + 1];
    return std::vector<Candidate>(reinterpret_cast<const Candidate*>(b), reinterpret_cast<const Candidate*>(e));
  };
  for (int f = 0; f < r.n_frames; ++f) {
    CANDIDATES_BOTTOM_PAW.push_back(list(f, 0));
    CANDIDATES_BOTTOM_SNOUT.push_back(list(f, 1));
    CANDIDATES_SIDE_PAW.push_back(list(f, 2));
    CANDIDATES_SIDE_SNOUT.push_back(list(f, 3));
    for (int k = 0; k < LM_N_FEATURES; ++k) {
      const int q = 2 * f + k;
      std::vector<P22D> pv;
      for (int64_t i = r.p22d_offset[q]; i < r.p22d_offset[q + 1]; ++i) {
        const lm_p22d& p = r.p22d[i];
        P22D v(Candidate(p.bottom.x, p.bottom.y, p.bottom.score), Candidate());
        v.set_side_raw(r.side_y + p.side_offset, r.side_s + p.side_offset, p.side_count);
        pv.push_back(std::move(v));
      }
      (k ? CANDIDATES_MATCHED_VIEWS_SNOUT : CANDIDATES_MATCHED_VIEWS_PAW).push_back(std::move(pv));
      const int ncol = k ? 1 : LM_N_PAWS;  // N_cand x 4 (paw) / x 1 (snout), column-major
      const int64_t u0 = r.unary_offset[q], nu = r.unary_offset[q + 1] - u0;
      MyMat U((unsigned)(nu / ncol), (unsigned)ncol);
      std::copy(r.unary + u0, r.unary + u0 + nu, U.getValues());
      (k ? UNARY_BOTTOM_SNOUT : UNARY_BOTTOM_PAW).push_back(std::move(U));
      const int32_t* d = r.pw_dims + 3 * q;
      if (d[0] >= 0)  // frames > 0 only (:896-919)
        (k ? PAIRWISE_BOTTOM_SNOUT : PAIRWISE_BOTTOM_PAW)
            .emplace_back(d[0], d[1], r.pw_jc + r.pw_jc_offset[q], r.pw_ir + r.pw_nz_offset[q],
                          r.pw_pr + r.pw_nz_offset[q]);
    }
    TailTrack t;
    std::copy(r.tail + 45 * f, r.tail + 45 * (f + 1), t.begin());
    TRACKS_TAIL.push_back(t);
  }
}

TrackSetup make_track_setup(const lm_geometry& g, const lm_params& p, unsigned n_frames) {
  TrackSetup S;
  S.n_frames = n_frames;
  S.nong_bottom = g.ong_nx * g.ong_ny;
  S.nong_side = g.n_ong_side;
  S.ong_side_lowest = (unsigned)g.ong_side_lowest;
  S.occlusion_grid_spacing_pixels_side = p.occlusion_grid_spacing_pixels_side;
  S.max_displacement_side = p.max_displacement_side;
  S.alpha_vel_side = p.alpha_vel_side;
  S.pairwise_occluded_cost = p.pairwise_occluded_cost;
  S.bb_bottom_mouse = g.bb_bottom_mouse;
  S.bb_side_mouse = g.bb_side_mouse;
  return S;
}

static void check_frames(const FrameResults& R, const TrackSetup& S) {
  if (R.UNARY_BOTTOM_PAW.size() != S.n_frames || R.CANDIDATES_MATCHED_VIEWS_PAW.size() != S.n_frames ||
      R.TRACKS_TAIL.size() != S.n_frames)
    throw std::runtime_error("tracks: the per-frame loop has not processed N_FRAMES frames.");
}

// :2153-2200.  Four orders of the paws are tracked; the one whose unary cost
// (computeCostTrack) is largest — strictly above the previous best, starting
// from -1 — wins, and its rows are put back in paw order.
void computeBottomTracks(const FrameResults& R, const TrackSetup& S, TrackResults& out) {
  check_frames(R, S);
  // The four orders and the snout are independent match2nd problems: solved
  // concurrently, then compared in the reference's order (strict >).
  // Inputs match2nd would reject print a message per call: run those calls
  // one after another so the messages come out in the reference's order.
  bool quiet = S.n_frames >= 2;
  for (unsigned f = 0; quiet && f < S.n_frames && f < R.UNARY_BOTTOM_PAW.size(); ++f)
    quiet = R.UNARY_BOTTOM_PAW[f].Ncols() == LM_N_PAWS;
  const auto policy = quiet ? std::launch::async : std::launch::deferred;
  std::future<IntMat> runs[LM_N_PAWS];
  for (int ip = 0; ip < LM_N_PAWS; ++ip)
    runs[ip] = std::async(policy, [&R, &S, ip] {
      return match2nd(R.UNARY_BOTTOM_PAW, R.PAIRWISE_BOTTOM_PAW, S.nong_bottom, 0, 0, S.n_frames, LM_N_PAWS,
                      PAW_ORDERS[ip]);
    });
  if (!quiet)
    for (auto& r : runs) r.wait();  // deferred: runs now, in order, before the snout call below
  const int zero = 0;
  IntMat snout = match2nd(R.UNARY_BOTTOM_SNOUT, R.PAIRWISE_BOTTOM_SNOUT, S.nong_bottom, 0, 0, S.n_frames, 1, &zero);
  double current_cost = -1;
  int current_perm = 0;
  IntMat best;
  for (int ip = 0; ip < LM_N_PAWS; ++ip) {
    IntMat M = runs[ip].get();
    const double c = computeCostTrack(M, R.UNARY_BOTTOM_PAW, R.PAIRWISE_BOTTOM_PAW, PAW_ORDERS[ip]);
    if (c > current_cost) {
      current_perm = ip;
      current_cost = c;
      best = std::move(M);
    }
  }
  // The reference then copies rows of an empty cv::Mat and CV_Assert fails.
  if (best.empty()) throw std::runtime_error("computeBottomTracks: no paw order scored above -1.");
  IntMat T(best.rows, best.cols, 0);
  for (int r = 0; r < LM_N_PAWS; ++r)
    std::copy(best.row(r), best.row(r) + best.cols, T.row(PAW_ORDERS[current_perm][r]));
  out.TRACK_INDEX_PAW_BOTTOM = std::move(T);
  out.TRACK_INDEX_SNOUT_BOTTOM = std::move(snout);
}

// :2073-2150.  D is (|Zip1| + Nong) x (|Zi| + Nong): candidate -> nearest side
// occlusion point, candidate -> candidate within max_displacement, occlusion
// point -> candidate, occlusion point -> itself; stored as CSC without zeros.
MATSPARSE pairwisePotential_SideView(const std::vector<uint32_t>& Zi, const std::vector<uint32_t>& Zip1,
                                     double grid_mapping, double grid_spacing, unsigned Nong,
                                     double max_displacement, double alpha_vel, double pairwise_occluded_cost) {
  const int Ni = (int)Zi.size(), Nip1 = (int)Zip1.size();
  const double occ = pairwise_occluded_cost * alpha_vel;
  const int last = (int)Nong - 1;
  auto grid_index = [&](uint32_t z) {  // matchToRange(round((mapping - z) / spacing), 0, Nong-1)
    const int32_t k = (int32_t)std::round((grid_mapping - (double)z) / grid_spacing);
    return k < 0 ? 0 : (k > last ? last : k);
  };
  MyMat D((unsigned)(Nip1 + (int)Nong), (unsigned)(Ni + (int)Nong));
  for (int i = 0; i < Ni; ++i) {
    D.put((unsigned)(Nip1 + grid_index(Zi[i])), (unsigned)i, occ);
    for (int j = 0; j < Nip1; ++j) {
      const double dist = std::fabs((double)Zip1[j] - (double)Zi[i]);
      if (dist < max_displacement) D.put((unsigned)j, (unsigned)i, (1 - dist / max_displacement) * alpha_vel);
    }
  }
  for (int j = 0; j < Nip1; ++j) D.put((unsigned)j, (unsigned)(Ni + grid_index(Zip1[j])), occ);
  for (int i = 0; i < (int)Nong; ++i) D.put((unsigned)(Nip1 + i), (unsigned)(Ni + i), occ);
  return MATSPARSE(&D);
}

// :2216-2346.  For each feature, the side-view problem over the frames: the
// side candidates matched to the bottom track's candidate (scores as unary
// costs; none when the bottom track is occluded), then match2nd with one track.
IntMat bestSideViewMatch(const IntMat& T, const std::vector<std::vector<P22D>>& matched, const TrackSetup& S,
                         unsigned N_features) {
  const unsigned N = S.n_frames;
  IntMat T_side((int)N_features, (int)N, 0);
  for (unsigned feat = 0; feat < N_features; ++feat) {
    const int32_t* pT = T.row((int)feat);
    std::vector<MyMat> unary;
    std::vector<MATSPARSE> pairwise;
    unary.reserve(N);
    pairwise.reserve(N ? N - 1 : 0);
    std::vector<uint32_t> Z_prev;
    for (unsigned f = 0; f < N; ++f) {
      std::vector<uint32_t> Z;
      if ((size_t)(uint32_t)pT[f] < matched[f].size() && pT[f] >= 0) {
        const P22D& p = matched[f][pT[f]];
        const int n = p.number_of_candidates();
        MyMat U((unsigned)n, 1);
        for (int i = 0; i < n; ++i) {
          U.put((unsigned)i, 0, p.score_side((unsigned)i));
          Z.push_back((uint32_t)p.y_side_coord((unsigned)i));
        }
        unary.push_back(std::move(U));
      } else {
        unary.emplace_back(0u, 1u);
      }
      if (f > 0)
        pairwise.push_back(pairwisePotential_SideView(
            Z_prev, Z, (double)S.ong_side_lowest, (double)S.occlusion_grid_spacing_pixels_side, (unsigned)S.nong_side,
            (double)S.max_displacement_side, S.alpha_vel_side, S.pairwise_occluded_cost));
      Z_prev = std::move(Z);
    }
    const int zero = 0;
    IntMat t = match2nd(unary, pairwise, S.nong_side, 0, 0, N, 1, &zero);
    std::copy(t.row(0), t.row(0) + N, T_side.row((int)feat));
  }
  return T_side;
}

void computeSideTracks(const FrameResults& R, const TrackSetup& S, TrackResults& out) {  // :2202-2214
  check_frames(R, S);
  out.TRACK_INDEX_PAW_SIDE = bestSideViewMatch(out.TRACK_INDEX_PAW_BOTTOM, R.CANDIDATES_MATCHED_VIEWS_PAW, S, LM_N_PAWS);
  out.TRACK_INDEX_SNOUT_SIDE = bestSideViewMatch(out.TRACK_INDEX_SNOUT_BOTTOM, R.CANDIDATES_MATCHED_VIEWS_SNOUT, S, 1);
}

// :2385-2444.  Crop coordinates back to image coordinates through the
// per-frame bottom-right corners (unsigned arithmetic, stored as int32).
IntMat exportPointTracks(const IntMat& T_bottom, const IntMat& T_side, const std::vector<std::vector<P22D>>& matched,
                         const TrackSetup& S, unsigned i_feature) {
  const unsigned N = S.n_frames;
  IntMat M((int)N, 3, -1);
  const int32_t* pT = T_bottom.row((int)i_feature);
  const int32_t* pS = T_side.row((int)i_feature);
  const uint32_t Wb = (uint32_t)S.bb_bottom_mouse.width, Hb = (uint32_t)S.bb_bottom_mouse.height;
  const uint32_t Hs = (uint32_t)S.bb_side_mouse.height;
  for (unsigned f = 0; f < N; ++f) {
    if (pT[f] < 0 || (size_t)pT[f] >= matched[f].size()) continue;
    const P22D& p = matched[f][pT[f]];
    int32_t* m = M.row((int)f);
    m[0] = (int32_t)((*S.bb_x_pos)[f] - Wb + 1u + (uint32_t)p.x_coord());
    m[1] = (int32_t)((*S.bb_y_bottom_pos)[f] - Hb + 1u + (uint32_t)p.y_bottom_coord());
    if (pS[f] < p.number_of_candidates()) {
      // the reference indexes yt with (uint)-1 here
      if (pS[f] < 0) throw std::runtime_error("exportPointTracks: side label -1 with side candidates present.");
      m[2] = (int32_t)((*S.bb_y_side_pos)[f] - Hs + 1u + (uint32_t)p.y_side_coord((unsigned)pS[f]));
    }
  }
  return M;
}

IntMat exportLineTracks(const std::vector<TailTrack>& tracks, const TrackSetup& S, int n_line_points) {  // :2446-2482
  const unsigned N = S.n_frames;
  IntMat out(3, n_line_points * (int)N, -1);
  const uint32_t Wb = (uint32_t)S.bb_bottom_mouse.width, Hb = (uint32_t)S.bb_bottom_mouse.height;
  const uint32_t Hs = (uint32_t)S.bb_side_mouse.height;
  for (unsigned f = 0; f < N; ++f)
    for (int t = 0; t < n_line_points; ++t) {
      const int c = (int)f * n_line_points + t;
      const int32_t x = tracks[f][t], y = tracks[f][LM_N_TAIL_POINTS + t], z = tracks[f][2 * LM_N_TAIL_POINTS + t];
      if (x >= 0) out.at(0, c) = (int32_t)((*S.bb_x_pos)[f] - Wb + 1u + (uint32_t)x);
      if (y >= 0) out.at(1, c) = (int32_t)((*S.bb_y_bottom_pos)[f] - Hb + 1u + (uint32_t)y);
      if (z >= 0) out.at(2, c) = (int32_t)((*S.bb_y_side_pos)[f] - Hs + 1u + (uint32_t)z);
    }
  return out;
}

void exportTracks(const FrameResults& R, const TrackSetup& S, TrackResults& out) {  // :2348-2383
  check_frames(R, S);
  if (!S.bb_x_pos || S.bb_x_pos->size() < S.n_frames || !S.bb_y_bottom_pos || !S.bb_y_side_pos)
    throw std::runtime_error("exportResults: no bounding-box corners for every frame.");
  out.paw_tracks.clear();
  out.snout_tracks.clear();
  for (unsigned i = 0; i < LM_N_PAWS; ++i)
    out.paw_tracks.push_back(
        exportPointTracks(out.TRACK_INDEX_PAW_BOTTOM, out.TRACK_INDEX_PAW_SIDE, R.CANDIDATES_MATCHED_VIEWS_PAW, S, i));
  out.snout_tracks.push_back(exportPointTracks(out.TRACK_INDEX_SNOUT_BOTTOM, out.TRACK_INDEX_SNOUT_SIDE,
                                               R.CANDIDATES_MATCHED_VIEWS_SNOUT, S, 0));
  out.tracks_tail = exportLineTracks(R.TRACKS_TAIL, S, LM_N_TAIL_POINTS);
}

void writeOutputYaml(const std::string& path, const TrackResults& T) {  // OUTPUT << name << M (:2384-2482)
  FsWriter fs(path);
  if (!fs.isOpened()) throw std::runtime_error("exportResults: cannot open " + path + " for writing.");
  auto put = [&](const std::string& name, const IntMat& M) {
    fs << name;
    fs.write_mat_i(M.data.data(), M.rows, M.cols);
  };
  for (size_t i = 0; i < T.paw_tracks.size(); ++i) put("paw_tracks" + std::to_string(i), T.paw_tracks[i]);
  for (size_t i = 0; i < T.snout_tracks.size(); ++i) put("snout_tracks" + std::to_string(i), T.snout_tracks[i]);
  put("tracks_tail", T.tracks_tail);
  fs.release();
}

}  // namespace locomouse

// ------------------------------------------------------------------ C-ABI
// include/locomouse_track.h

#include "locomouse_track.h"

namespace {

thread_local std::string t_error;
thread_local locomouse::TrackResults t_tracks;
thread_local std::vector<int32_t> t_paw, t_snout, t_index_bottom, t_index_side;

template <class Fn>
lm_status guarded(Fn&& fn) {
  try {
    fn();
    t_error.clear();
    return LM_OK;
  } catch (const std::invalid_argument& e) {
    t_error = e.what();
    return LM_ERR_INVALID_ARGUMENT;
  } catch (const std::exception& e) {
    t_error = e.what();
    return LM_ERR_RUNTIME;
  }
}

}  // namespace

extern "C" {

const char* lm_track_last_error(void) { return t_error.c_str(); }

lm_status lm_match2nd(int32_t n_frames, int32_t n_points, int32_t n_cols, int32_t nong, double occlusion_point_cost,
                      double bam_tie, const int32_t* n_loc, const int64_t* unary_offset, const double* unary,
                      const int32_t* pw_dims, const int64_t* pw_jc_offset, const int32_t* pw_jc,
                      const int64_t* pw_nz_offset, const int32_t* pw_ir, const double* pw_pr,
                      const int32_t* permutation, int32_t* labels, double* cost) {
  return guarded([&] {
    using namespace locomouse;
    if (n_frames < 0 || n_points < 0 || n_cols < 0 || nong < 0 || !labels || (n_points > 0 && !permutation))
      throw std::invalid_argument("lm_match2nd: invalid sizes or NULL output.");
    for (int32_t p = 0; p < n_points; ++p)
      if (permutation[p] < 0 || permutation[p] >= n_cols)
        throw std::invalid_argument("lm_match2nd: permutation entry outside the unary columns.");
    std::vector<MyMat> U;
    std::vector<MATSPARSE> P;
    for (int32_t f = 0; f < n_frames; ++f) {
      if (n_loc[f] < 0 || unary_offset[f + 1] - unary_offset[f] != (int64_t)n_loc[f] * n_cols)
        throw std::invalid_argument("lm_match2nd: unary sizes do not match n_loc x n_cols.");
      MyMat M((unsigned)n_loc[f], (unsigned)n_cols);
      std::copy(unary + unary_offset[f], unary + unary_offset[f + 1], M.getValues());
      U.push_back(std::move(M));
    }
    for (int32_t f = 0; f + 1 < n_frames; ++f) {
      const int32_t* d = pw_dims + 3 * f;
      if (d[0] < 0 || d[1] < 0 || d[2] < 0 || pw_nz_offset[f + 1] - pw_nz_offset[f] != d[2] ||
          pw_jc_offset[f + 1] - pw_jc_offset[f] != (int64_t)d[1] + 1)
        throw std::invalid_argument("lm_match2nd: pairwise CSC sizes are inconsistent.");
      const int32_t* jc = pw_jc + pw_jc_offset[f];
      if (jc[0] != 0 || jc[d[1]] != d[2]) throw std::invalid_argument("lm_match2nd: pairwise Jc must run 0..nnz.");
      for (int32_t c = 0; c < d[1]; ++c)
        if (jc[c + 1] < jc[c]) throw std::invalid_argument("lm_match2nd: pairwise Jc must be non-decreasing.");
      for (int32_t k = 0; k < d[2]; ++k)
        if (pw_ir[pw_nz_offset[f] + k] < 0 || pw_ir[pw_nz_offset[f] + k] >= d[0])
          throw std::invalid_argument("lm_match2nd: pairwise row index out of range.");
      P.emplace_back(d[0], d[1], jc, pw_ir + pw_nz_offset[f], pw_pr + pw_nz_offset[f]);
    }
    const IntMat T = match2nd(U, P, nong, occlusion_point_cost, bam_tie, (unsigned)n_frames, (unsigned)n_points,
                              permutation);
    std::copy(T.data.begin(), T.data.end(), labels);
    if (cost) *cost = computeCostTrack(T, U, P, permutation);
  });
}

lm_status lm_compute_tracks(const lm_batch_result* video, const lm_geometry* geometry, const lm_params* params,
                            const uint32_t* bb, lm_tracks* out) {
  return guarded([&] {
    using namespace locomouse;
    if (!video || !geometry || !params || !bb || !out) throw std::invalid_argument("lm_compute_tracks: NULL argument.");
    if (video->first_frame != 0) throw std::invalid_argument("lm_compute_tracks: results must start at frame 0.");
    const bool timing = std::getenv("LM_TRACK_TIMING") != nullptr;
    auto t0 = std::chrono::steady_clock::now();
    auto lap = [&](const char* what) {
      if (!timing) return;
      const auto t1 = std::chrono::steady_clock::now();
      std::fprintf(stderr, "lm_compute_tracks %s: %.3f ms\n", what, std::chrono::duration<double, std::milli>(t1 - t0).count());
      t0 = t1;
    };
    FrameResults R;
    R.append(*video);
    lap("containers");
    const unsigned N = (unsigned)video->n_frames;
    std::vector<uint32_t> bx(N), byb(N), bys(N);
    for (unsigned f = 0; f < N; ++f) {
      bx[f] = bb[3 * f];
      byb[f] = bb[3 * f + 1];
      bys[f] = bb[3 * f + 2];
    }
    TrackSetup S = make_track_setup(*geometry, *params, N);
    S.bb_x_pos = &bx;
    S.bb_y_bottom_pos = &byb;
    S.bb_y_side_pos = &bys;
    TrackResults T;
    computeBottomTracks(R, S, T);
    lap("bottom tracks");
    computeSideTracks(R, S, T);
    lap("side tracks");
    exportTracks(R, S, T);
    lap("export");
    t_tracks = std::move(T);
    t_paw.clear();
    for (const auto& m : t_tracks.paw_tracks) t_paw.insert(t_paw.end(), m.data.begin(), m.data.end());
    t_snout = t_tracks.snout_tracks[0].data;
    t_index_bottom = t_tracks.TRACK_INDEX_PAW_BOTTOM.data;
    t_index_bottom.insert(t_index_bottom.end(), t_tracks.TRACK_INDEX_SNOUT_BOTTOM.data.begin(),
                          t_tracks.TRACK_INDEX_SNOUT_BOTTOM.data.end());
    t_index_side = t_tracks.TRACK_INDEX_PAW_SIDE.data;
    t_index_side.insert(t_index_side.end(), t_tracks.TRACK_INDEX_SNOUT_SIDE.data.begin(),
                        t_tracks.TRACK_INDEX_SNOUT_SIDE.data.end());
    out->n_frames = (int32_t)N;
    out->paw_tracks = t_paw.data();
    out->snout_tracks = t_snout.data();
    out->tracks_tail = t_tracks.tracks_tail.data.data();
    out->track_index_bottom = t_index_bottom.data();
    out->track_index_side = t_index_side.data();
  });
}

lm_status lm_write_tracks_yaml(const char* path, const lm_tracks* tracks) {
  return guarded([&] {
    using namespace locomouse;
    if (!path || !tracks) throw std::invalid_argument("lm_write_tracks_yaml: NULL argument.");
    const int N = tracks->n_frames;
    TrackResults T;
    for (int i = 0; i < LM_N_PAWS; ++i) {
      IntMat M(N, 3);
      std::copy(tracks->paw_tracks + (size_t)i * N * 3, tracks->paw_tracks + (size_t)(i + 1) * N * 3, M.data.begin());
      T.paw_tracks.push_back(std::move(M));
    }
    IntMat S(N, 3);
    std::copy(tracks->snout_tracks, tracks->snout_tracks + (size_t)N * 3, S.data.begin());
    T.snout_tracks.push_back(std::move(S));
    T.tracks_tail = IntMat(3, LM_N_TAIL_POINTS * N);
    std::copy(tracks->tracks_tail, tracks->tracks_tail + (size_t)3 * LM_N_TAIL_POINTS * N, T.tracks_tail.data.begin());
    writeOutputYaml(path, T);
  });
}

}  // extern "C"
