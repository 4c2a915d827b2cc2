// host_harness.cpp — test harness for the host C++ LocoMouse mirror
// (locomouse_cpp_amd/host).  lmh_run() drives a LocoMouse exactly as the
// reference's main.cpp:45-82 does (factory, getBoundingBox,
// initializeFeatureLoop, the nine per-frame calls per frame) over frames held
// in memory, then flattens the result containers into an lm_batch_result so
// the Python tests compare them with the oracle field by field.
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "FileStorage.hpp"
#include "LocoMouse.hpp"
#include "Media.hpp"

namespace {

struct Flat {
  std::vector<int64_t> cand_off, p22d_off, unary_off, jc_off, nz_off;
  std::vector<lm_candidate> cand;
  std::vector<lm_p22d> p22d;
  std::vector<int32_t> side_y, pw_dims, pw_jc, pw_ir, tail;
  std::vector<double> side_s, unary, pw_pr;
} g_flat;

locomouse::TrackResults g_tracks;
std::string g_output_file;
std::vector<int> g_devices;  // LocoMouse_Inputs::devices of the next lmh_run (empty: the device argument)
bool g_oversubscribe = false;

int fail(const std::exception& e, int code, char* err, int errlen) {
  if (err && errlen > 0) {
    std::strncpy(err, e.what(), (size_t)errlen - 1);
    err[errlen - 1] = 0;
  }
  return code;
}

}  // namespace

extern "C" void lmh_set_devices(const int* devices, int n, int oversubscribe) {
  g_devices.assign(devices, devices + (n > 0 ? n : 0));
  g_oversubscribe = oversubscribe != 0;
}

extern "C" int lmh_run(const lm_setup* setup, const lm_params* params, const lm_model* model,
                       const lm_bb_params* bb_params, const uint8_t* frames, int n_frames, int n_read, int batch,
                       int device, int call_order, lm_batch_result* out, uint32_t* bb_corners, lm_rect* bb_sizes,
                       char* err, int errlen) {
  try {
    locomouse::LocoMouse_Inputs in;
    in.setup = *setup;
    in.params = *params;
    in.model = *model;
    in.n_frames = (uint32_t)n_frames;
    in.device = device;
    in.devices = g_devices;
    in.oversubscribe = g_oversubscribe;
    in.batch = batch;
    in.output_file = g_output_file;
    const size_t fb = (size_t)setup->video_rows * setup->video_cols;
    int next = 0;
    in.read_frame = [&](uint8_t* dst) {  // V >> F over the frames given
      if (next >= n_read) return false;
      std::memcpy(dst, frames + (size_t)next++ * fb, fb);
      return true;
    };
    if (call_order & 8) {  // the batch reader (read_frames), as the CLI uses it
      in.read_frames = [&](uint8_t* dst, int n) {
        int k = 0;
        for (; k < n && next < n_read; ++k, ++next) std::memcpy(dst + (size_t)k * fb, frames + (size_t)next * fb, fb);
        return k;
      };
    }
    if (bb_params) {
      in.bb_params = *bb_params;
      in.rewind = [&] { next = 0; };  // V.set(CV_CAP_PROP_POS_FRAMES, 0)
    }
    std::unique_ptr<LocoMouse> L = LocoMouse_Initialize(in);
    L->getBoundingBox();
    L->initializeFeatureLoop();
    if (bb_corners)
      for (unsigned i = 0; i < L->N_frames(); ++i) {
        bb_corners[3 * i] = L->bb_x_pos()[i];
        bb_corners[3 * i + 1] = L->bb_y_bottom_pos()[i];
        bb_corners[3 * i + 2] = L->bb_y_side_pos()[i];
      }
    if (bb_sizes) {
      bb_sizes[0] = L->bb_side_mouse();
      bb_sizes[1] = L->bb_bottom_mouse();
    }
    for (unsigned i = 0; i < L->N_frames(); ++i) {  // main.cpp:54-82
      L->readFrame();
      L->cropBoundingBox();
      L->detectTail();
      L->detectBottomCandidates();
      L->computeUnaryCostsBottom();
      L->computePairwiseCostsBottom();
      L->detectSideCandidates();
      L->matchBottomSideCandidates();
      if ((call_order & 1) && i % 3 == 1) (void)L->candidates_bottom_paw();  // mid-batch reads flush early
      L->storePreviousImage();
    }
    if (call_order & 4) {  // main.cpp:86-91
      L->computeBottomTracks();
      L->computeSideTracks();
      L->exportResults();
      g_tracks = L->tracks();
    }
    Flat& F = g_flat;
    F = Flat();
    const auto& cbp = L->candidates_bottom_paw();
    const auto& cbs = L->candidates_bottom_snout();
    const auto& csp = L->candidates_side_paw();
    const auto& css = L->candidates_side_snout();
    const auto& mp = L->candidates_matched_views_paw();
    const auto& ms = L->candidates_matched_views_snout();
    const auto& up = L->unary_bottom_paw();
    const auto& us = L->unary_bottom_snout();
    const auto& pp = L->pairwise_bottom_paw();
    const auto& ps = L->pairwise_bottom_snout();
    const auto& tt = L->tracks_tail();
    const int n = (int)cbp.size();
    F.cand_off.push_back(0);
    F.p22d_off.push_back(0);
    F.unary_off.push_back(0);
    F.jc_off.push_back(0);
    F.nz_off.push_back(0);
    for (int f = 0; f < n; ++f) {
      for (const auto* lst : {&cbp[f], &cbs[f], &csp[f], &css[f]}) {
        for (const Candidate& c : *lst) F.cand.push_back(lm_candidate{c.p.x, c.p.y, c.s});
        F.cand_off.push_back((int64_t)F.cand.size());
      }
      for (int k = 0; k < 2; ++k) {
        for (const P22D& p : (k ? ms : mp)[f]) {
          lm_p22d q;
          q.bottom = lm_candidate{p.x_coord(), p.y_bottom_coord(), p.score_bottom()};
          q.side_offset = (int32_t)F.side_y.size();
          q.side_count = (int32_t)p.raw_side_y().size();
          F.side_y.insert(F.side_y.end(), p.raw_side_y().begin(), p.raw_side_y().end());
          F.side_s.insert(F.side_s.end(), p.raw_side_s().begin(), p.raw_side_s().end());
          F.p22d.push_back(q);
        }
        F.p22d_off.push_back((int64_t)F.p22d.size());
        const MyMat& U = (k ? us : up)[f];
        F.unary.insert(F.unary.end(), U.getValues(), U.getValues() + U.Numel());
        F.unary_off.push_back((int64_t)F.unary.size());
        // pairwise entries exist for frames >= 1 only
        if (f >= 1) {
          const MATSPARSE& P = (k ? ps : pp)[f - 1];
          F.pw_dims.insert(F.pw_dims.end(), {P.Nrows(), P.Ncols(), P.nz()});
          F.pw_jc.insert(F.pw_jc.end(), P.getJc(), P.getJc() + P.Ncols() + 1);
          F.pw_ir.insert(F.pw_ir.end(), P.getIr(), P.getIr() + P.nz());
          F.pw_pr.insert(F.pw_pr.end(), P.getPr(), P.getPr() + P.nz());
        } else {
          F.pw_dims.insert(F.pw_dims.end(), {-1, -1, 0});
        }
        F.jc_off.push_back((int64_t)F.pw_jc.size());
        F.nz_off.push_back((int64_t)F.pw_ir.size());
      }
      F.tail.insert(F.tail.end(), tt[f].begin(), tt[f].end());
    }
    out->n_frames = n;
    out->first_frame = 0;
    out->cand_offset = F.cand_off.data();
    out->cand = F.cand.data();
    out->p22d_offset = F.p22d_off.data();
    out->p22d = F.p22d.data();
    out->side_y = F.side_y.data();
    out->side_s = F.side_s.data();
    out->unary_offset = F.unary_off.data();
    out->unary = F.unary.data();
    out->pw_dims = F.pw_dims.data();
    out->pw_jc_offset = F.jc_off.data();
    out->pw_jc = F.pw_jc.data();
    out->pw_nz_offset = F.nz_off.data();
    out->pw_ir = F.pw_ir.data();
    out->pw_pr = F.pw_pr.data();
    out->tail = F.tail.data();
    return 0;
  } catch (const std::invalid_argument& e) {
    return fail(e, 1, err, errlen);
  } catch (const std::runtime_error& e) {
    return fail(e, 2, err, errlen);
  } catch (const std::exception& e) {
    return fail(e, 3, err, errlen);
  }
}

// Output file for exportResults (empty: none).
extern "C" void lmh_set_output(const char* path) { g_output_file = path ? path : ""; }

// The tracks of the last lmh_run with call_order & 4: paw [4][n][3], snout
// [n][3], tail [3][15n], index_bottom / index_side [5][n].
extern "C" int lmh_get_tracks(int n, int32_t* paw, int32_t* snout, int32_t* tail, int32_t* idx_b, int32_t* idx_s) {
  const auto& T = g_tracks;
  if (T.paw_tracks.size() != 4 || T.tracks_tail.cols != 15 * n) return 1;
  for (int i = 0; i < 4; ++i) std::copy(T.paw_tracks[i].data.begin(), T.paw_tracks[i].data.end(), paw + (size_t)i * n * 3);
  std::copy(T.snout_tracks[0].data.begin(), T.snout_tracks[0].data.end(), snout);
  std::copy(T.tracks_tail.data.begin(), T.tracks_tail.data.end(), tail);
  std::copy(T.TRACK_INDEX_PAW_BOTTOM.data.begin(), T.TRACK_INDEX_PAW_BOTTOM.data.end(), idx_b);
  std::copy(T.TRACK_INDEX_SNOUT_BOTTOM.data.begin(), T.TRACK_INDEX_SNOUT_BOTTOM.data.end(), idx_b + 4 * n);
  std::copy(T.TRACK_INDEX_PAW_SIDE.data.begin(), T.TRACK_INDEX_PAW_SIDE.data.end(), idx_s);
  std::copy(T.TRACK_INDEX_SNOUT_SIDE.data.begin(), T.TRACK_INDEX_SNOUT_SIDE.data.end(), idx_s + 4 * n);
  return 0;
}

// Container semantics that need no GPU (P22D slot-0 rule, MATSPARSE CSC).
extern "C" int lmh_selftest(char* err, int errlen) {
  try {
    P22D p(Candidate(5, 7, 2.0), Candidate());
    if (p.number_of_candidates() != 0) throw std::runtime_error("empty P22D must have 0 side candidates");
    p.add_side_candidate(11, 0.5);  // fills slot 0
    p.add_side_candidate(12, 0.25);
    if (p.number_of_candidates() != 2 || p.y_side_coord(0) != 11 || p.score_side(1) != 0.25)
      throw std::runtime_error("add_side_candidate order");
    bool threw = false;
    try {
      p.add_side_candidate(13, -1.0);
    } catch (const std::runtime_error&) {
      threw = true;
    }
    if (!threw) throw std::runtime_error("CV_Assert(S >= 0) not enforced");
    MyMat M(3, 2);
    M.put(0, 0, 1.5);
    M.put(2, 0, -2);
    M.put(1, 1, 4);
    MATSPARSE S(&M);
    const int jc[] = {0, 2, 3}, ir[] = {0, 2, 1};
    const double pr[] = {1.5, -2, 4};
    if (!(S == MATSPARSE(3, 2, jc, ir, pr))) throw std::runtime_error("MATSPARSE CSC layout");
    if (S.at(2, 0) != -2 || S.get(2, 0) != 0) throw std::runtime_error("MATSPARSE get/at");
    if (!compareCandidate(Candidate(0, 0, 2), Candidate(0, 0, 1))) throw std::runtime_error("compareCandidate");
    return 0;
  } catch (const std::exception& e) {
    return fail(e, 2, err, errlen);
  }
}

// Readers behind the CLI (Media.hpp, FileStorage.hpp), CPU only.
extern "C" int lmh_read_png(const char* path, int* rows, int* cols, uint8_t* out, int64_t cap) {
  std::vector<uint8_t> px;
  if (!locomouse::read_png_gray(path, *rows, *cols, px)) return 1;
  if ((int64_t)px.size() > cap) return 2;
  std::memcpy(out, px.data(), px.size());
  return 0;
}

extern "C" int lmh_read_avi(const char* path, int* rows, int* cols, int* n, uint8_t* out, int64_t cap, int rewind_at) {
  locomouse::AviReader r;
  if (!r.open(path)) return 1;
  *rows = r.rows();
  *cols = r.cols();
  *n = (int)r.frame_count();
  const int64_t fb = (int64_t)r.rows() * r.cols();
  int64_t k = 0;
  for (int i = 0;; ++i) {
    if (i == rewind_at) r.rewind();
    if ((k + 1) * fb > cap) break;
    if (!r.read(out + k * fb)) break;
    ++k;
  }
  return -(int)k;  // frames read, as a non-positive number
}

// A matrix or scalar of a FileStorage file: kind, dims and values (doubles).
extern "C" int lmh_fs_node(const char* path, const char* key, int* kind, int* rows, int* cols, char* dt, double* out,
                           int64_t cap, char* text, int textlen) {
  try {
    locomouse::FsNode root;
    if (!locomouse::read_file_storage(path, root)) return 1;
    const locomouse::FsNode& n = root[key];
    *kind = (int)n.kind;
    *rows = *cols = 0;
    if (n.kind == locomouse::FsNode::MAT) {
      *rows = n.mat.rows;
      *cols = n.mat.cols;
      *dt = n.mat.dt;
      if ((int64_t)n.mat.v.size() > cap) return 2;
      std::copy(n.mat.v.begin(), n.mat.v.end(), out);
    } else if (n.kind == locomouse::FsNode::INT || n.kind == locomouse::FsNode::REAL) {
      out[0] = n.to_double();
      out[1] = n.to_int();
    } else if (n.kind == locomouse::FsNode::STR) {
      std::strncpy(text, n.s.c_str(), (size_t)textlen - 1);
      text[textlen - 1] = 0;
    } else if (n.kind == locomouse::FsNode::SEQ) {
      *rows = (int)n.seq.size();
      for (size_t i = 0; i < n.seq.size() && (int64_t)i < cap; ++i) out[i] = n.seq[i].to_double();
    }
    return 0;
  } catch (const std::exception& e) {
    std::strncpy(text, e.what(), (size_t)textlen - 1);
    text[textlen - 1] = 0;
    return 3;
  }
}

// FsWriter (cv::FileStorage WRITE, YAML) on a document with every construct
// exportResults / exportDebugVariables use.
extern "C" int lmh_fs_write_demo(const char* path) {
  locomouse::FsWriter fs(path);
  if (!fs.isOpened()) return 1;
  fs << "N_opencv_matrices" << 7;
  const int m[6] = {1, -2, 3, 4, 5, 6};
  fs << "M";
  fs.write_mat_i(m, 2, 3);
  fs << "real" << 0.5 << "whole" << 15.0 << "neg" << -0.375;
  fs << "BB" << "{" << "x" << 1 << "y" << 2 << "}";
  fs << "seq" << "[:";
  for (int k = 0; k < 40; ++k) fs << 1000 * k;
  fs << "]";
  fs << "nested" << "[";
  fs << "[";
  fs << "{" << "Candidate_bottom" << "{" << "Point_x" << 3 << "Score" << 0.25 << "}";
  fs << "side" << "[:" << 4 << "]" << "}";
  fs << "]";
  fs << "[" << "]";
  fs << "]";
  fs << "empty_flow" << "[:" << "]";
  fs << "last" << "text";
  fs.release();
  return 0;
}
