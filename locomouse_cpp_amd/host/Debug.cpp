// Debug.cpp — the reference's verbose_debug outputs:
// the DEBUG_TEXT stage log and exportDebugVariables' debug_<stem>.yml
// (LocoMouse_class.cpp:2769-2920), written from the containers the device
// path fills.
//
// The log keeps the reference's stage lines (readFrame :1279-1330,
// cropBoundingBox :1418-1474, detectTail :2544-2550, detectBottomCandidates
// :775-802, computeUnaryCostsBottom :876-890, computePairwiseCostsBottom
// :899-914, detectSideCandidates :812-836, matchBottomSideCandidates
// :1002-1016).  The stages run fused on the GPU, a batch at a time, so each
// frame's lines are written when its batch's results arrive, in frame order;
// lines that print OpenCV-internal state (Mat continuity, per-candidate
// matching traces) have no counterpart and are left out.
#include <sstream>
#include <stdexcept>

#include "FileStorage.hpp"
#include "LocoMouse.hpp"

namespace locomouse {

std::string debug_rect(const lm_rect& r) {
  std::ostringstream o;
  o << "[" << r.width << " x " << r.height << " from (" << r.x << ", " << r.y << ")]";
  return o.str();
}

void LocoMouse::debug_frames(int first, int n) {
  const lm_geometry g = geometry();
  std::ostream& T = DEBUG_TEXT;
  for (int f = first; f < first + n; ++f) {
    T << "=== readFrame: " << std::endl << "Read frame from image. Current frame is: " << f << std::endl;
    if (METHOD != 0) T << "convertColorOK" << std::endl;
    T << "Removed background." << std::endl << "Normalized input image range." << std::endl
      << "Applied calibration matrix." << std::endl;
    if (IN.setup.flip) T << "Flipped image" << std::endl;
    T << "=== Done" << std::endl;

    const lm_rect bp = g.bb_bottom_mouse_pad, sp = g.bb_side_mouse_pad;
    const int bx = ((int)BB_X_POS[f] + g.pad_pre_cols) - (bp.width - g.spost_b_w) + 1;
    const int by = ((int)BB_Y_BOTTOM_POS[f] + g.pad_pre_rows) - (bp.height - g.spost_b_h) + 1;
    const int sy = ((int)BB_Y_SIDE_POS[f] + g.pad_pre_rows) - (sp.height - g.spost_t_h) + 1;
    T << "=== cropBoundingBox:" << std::endl
      << "BB_BOTTOM_MOUSE_PAD.x = (" << BB_X_POS[f] << "+" << g.pad_pre_cols << ") - (" << bp.width << "-"
      << g.spost_b_w << ") + 1" << std::endl
      << "BB_BOTTOM_MOUSE_PAD.y = (" << BB_Y_BOTTOM_POS[f] << "+" << g.pad_pre_rows << ") - (" << bp.height << "-"
      << g.spost_b_h << ") + 1" << std::endl
      << "I_PAD.size(): [" << g.ipad_cols << " x " << g.ipad_rows << "]" << std::endl
      << "BB_BOTTOM_MOUSE_PAD: " << debug_rect(lm_rect{bx, by, bp.width, bp.height}) << std::endl
      << "BB_UNPAD_MOUSE_BOTTOM: " << debug_rect(g.bb_unpad_mouse_bottom) << std::endl;
    if (IN.params.transform_gray_values) T << "Gray Level Transformation Done" << std::endl;
    T << "BB_SIDE_MOUSE_PAD: " << debug_rect(lm_rect{bx, sy, sp.width, sp.height}) << std::endl
      << "BB_UNPAD_MOUSE_SIDE: " << debug_rect(g.bb_unpad_mouse_side) << std::endl;
    if (f > 0) T << "Cropped previous frame. " << std::endl;
    T << "=== Done." << std::endl;

    T << "=== Detect Tail: " << std::endl;
    int tail_points = 0;
    for (int k = 0; k < LM_N_TAIL_POINTS; ++k) tail_points += TRACKS_TAIL[f][k] >= 0;
    if (tail_points == 0) T << "No tail region found. Returning -1." << std::endl;
    T << "=== Done" << std::endl;

    T << "=== detectBottomCandidateS(): " << std::endl
      << "BB_BOTTOM_TAIL: [" << g.bb_bottom_tail.width << " x " << g.bb_bottom_tail.height << "]" << std::endl
      << "I_BOTTOM_MOUSE: [" << g.bb_bottom_mouse.width << " x " << g.bb_bottom_mouse.height << "]" << std::endl
      << "Masked the tail." << std::endl
      << "Detected " << CANDIDATES_BOTTOM_PAW[f].size() << " paw candidates." << std::endl
      << "Detected " << CANDIDATES_BOTTOM_SNOUT[f].size() << " snout candidates." << std::endl
      << "=== Done " << std::endl;

    T << "=== computeUnaryCostsBottom() " << std::endl
      << "Bottom Paw done. " << std::endl
      << "Bottom Snout done. " << std::endl
      << "=== Done " << std::endl;
    T << "=== computePairwiseCostsBottom() " << std::endl << "=== Done " << std::endl;
    T << "=== detectSideCandidates(): " << std::endl << "=== Done " << std::endl;
    T << "=== matchBottomSideCandidates: " << std::endl << "=== Done " << std::endl;
  }
  T.flush();
}

namespace {

void write_candidate(FsWriter& fs, const Candidate& c) {  // Candidates.cpp:19-21
  fs << "{" << "Point_x" << c.point().x << "Point_y" << c.point().y << "Score" << c.score() << "}";
}

void write_p22d(FsWriter& fs, const P22D& p) {  // Candidates.cpp:158-174 (n_candidates_side = yt.size())
  fs << "{" << "Candidate_bottom";
  write_candidate(fs, p.get_candidate_bottom());
  fs << "n_candidates_side" << (int)p.raw_side_y().size();
  fs << "Candidates_side" << "[:";
  for (int y : p.raw_side_y()) fs << y;
  fs << "]";
  fs << "Scores_side" << "[:";
  for (double s : p.raw_side_s()) fs << s;
  fs << "]";
  fs << "}";
}

void write_mymat(FsWriter& fs, const MyMat& M) {  // MyMat.cpp:84-96 (values in storage order)
  fs << "{" << "n_rows" << M.Nrows() << "n_cols" << M.Ncols() << "data" << "[:";
  for (int i = 0; i < M.Numel(); ++i) fs << M.getValues()[i];
  fs << "]" << "}";
}

void write_matsparse(FsWriter& fs, const MATSPARSE& M) {  // MyMat.cpp:310-349
  const int* Jc = M.getJc();
  const int* Ir = M.getIr();
  const double* Pr = M.getPr();
  fs << "{" << "data" << "[:";
  for (int k = 0; k < M.nz(); ++k) fs << Pr[k];
  fs << "]" << "row_index" << "[:";
  for (int k = 0; k < M.nz(); ++k) fs << Ir[k];
  fs << "]" << "col_index" << "[:";
  for (int c = 0; c < M.Ncols(); ++c)
    for (int k = Jc[c]; k < Jc[c + 1]; ++k) fs << c;
  fs << "]" << "}";
}

void write_row(FsWriter& fs, const std::string& name, const IntMat& M, int r) {  // M.row(r)
  if (r >= M.rows) throw std::runtime_error("exportDebugVariables: computeSideTracks() has not been called.");
  fs << name;
  fs.write_mat_i(M.row(r), 1, M.cols);
}

}  // namespace

void LocoMouse::exportDebugVariables() {
  if (DEBUG_TEXT.is_open()) DEBUG_TEXT << "--- exportDebugVariables() " << std::endl;
  if (IN.debug_file.empty()) return;
  sync();
  FsWriter fs(IN.debug_file);
  if (!fs.isOpened()) throw std::runtime_error("Could not create debug file: " + IN.debug_file + "\n");
  const TrackResults& T = TRACKS;
  fs << "N_opencv_matrices" << 7;
  fs << "M_paw_bottom";
  fs.write_mat_i(T.TRACK_INDEX_PAW_BOTTOM.data.data(), T.TRACK_INDEX_PAW_BOTTOM.rows, T.TRACK_INDEX_PAW_BOTTOM.cols);
  fs << "M_snout_bottom";
  fs.write_mat_i(T.TRACK_INDEX_SNOUT_BOTTOM.data.data(), T.TRACK_INDEX_SNOUT_BOTTOM.rows,
                 T.TRACK_INDEX_SNOUT_BOTTOM.cols);
  for (int i = 0; i < LM_N_PAWS; ++i) write_row(fs, "M_paw_side_" + std::to_string(i), T.TRACK_INDEX_PAW_SIDE, i);
  for (int i = 0; i < 1; ++i) write_row(fs, "M_snout_side_" + std::to_string(i), T.TRACK_INDEX_SNOUT_SIDE, i);
  fs << "N_frames" << (int)N_FRAMES;
  fs << "occluded_distance" << IN.params.max_displacement_bottom;
  fs << "BB_side" << "{" << "x" << BB_SIDE_MOUSE.x << "y" << BB_SIDE_MOUSE.y << "width" << BB_SIDE_MOUSE.width
     << "height" << BB_SIDE_MOUSE.height << "}";
  fs << "BB_bottom" << "{" << "x" << BB_BOTTOM_MOUSE.x << "y" << BB_BOTTOM_MOUSE.y << "width"
     << BB_BOTTOM_MOUSE.width << "height" << BB_BOTTOM_MOUSE.height << "}";
  auto uint_seq = [&](const char* name, const std::vector<uint32_t>& v) {
    fs << name << "[:";
    for (unsigned i = 0; i < N_FRAMES; ++i) fs << (int)v[i];
    fs << "]";
  };
  uint_seq("bb_x_avg", BB_X_POS);
  uint_seq("bb_yt_avg", BB_Y_SIDE_POS);
  uint_seq("bb_yb_avg", BB_Y_BOTTOM_POS);

  // ONG / ONG_SIDE as initializeFeatureLoop builds them (:726-759).
  const lm_geometry g = geometry();
  const int sp_b = IN.params.occlusion_grid_spacing_pixels_bottom, sp_s = IN.params.occlusion_grid_spacing_pixels_side;
  fs << "ONG" << "{" << "points" << g.ong_nx * g.ong_ny << "x_y_coordinates" << "[:";
  for (int j = 0; j < g.ong_ny; ++j)
    for (int i = 0; i < g.ong_nx; ++i)
      fs << g.ong_br_x - (double)((unsigned)i * (unsigned)sp_b) << g.ong_br_y - (double)((unsigned)j * (unsigned)sp_b);
  fs << "]" << "}";
  fs << "ONG_side" << "{" << "points" << g.n_ong_side << "z_coordinates" << "[:";
  for (int i = 0; i < g.n_ong_side; ++i) fs << (int)((unsigned)g.ong_side_lowest - (unsigned)(i * sp_s));
  fs << "]" << "}";

  auto matched = [&](const char* name, const std::vector<std::vector<P22D>>& C) {
    fs << name << "[";
    for (unsigned i = 0; i < N_FRAMES; ++i) {
      fs << "[";
      for (const P22D& p : C[i]) write_p22d(fs, p);
      fs << "]";
    }
    fs << "]";
  };
  matched("candidates_paw_bottom_side_matched", CANDIDATES_MATCHED_VIEWS_PAW);
  matched("candidates_snout_bottom_side_matched", CANDIDATES_MATCHED_VIEWS_SNOUT);
  fs << "Pairwise_paws" << "[";
  for (unsigned i = 0; i + 1 < N_FRAMES; ++i) write_matsparse(fs, PAIRWISE_BOTTOM_PAW[i]);
  fs << "]";
  fs << "Pairwise_snout" << "[";
  for (unsigned i = 0; i + 1 < N_FRAMES; ++i) write_matsparse(fs, PAIRWISE_BOTTOM_SNOUT[i]);
  fs << "]";
  fs << "Unary_paws" << "[";
  for (unsigned i = 0; i < N_FRAMES; ++i) write_mymat(fs, UNARY_BOTTOM_PAW[i]);
  fs << "]";
  fs << "Unary_snout" << "[";
  for (unsigned i = 0; i < N_FRAMES; ++i) write_mymat(fs, UNARY_BOTTOM_SNOUT[i]);
  fs << "]";
  fs.release();
}

}  // namespace locomouse
