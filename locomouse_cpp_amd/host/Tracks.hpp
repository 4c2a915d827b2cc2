// Tracks.hpp — the stage after the per-frame loop:
// computeBottomTracks, computeSideTracks and the track export of
// exportResults, over the containers the detection path fills.
//
// Reference: LocoMouse_class.cpp:2073-2150 (pairwisePotential_SideView),
// :2153-2200 (computeBottomTracks), :2202-2214 (computeSideTracks),
// :2216-2346 (bestSideViewMatch), :2348-2482 (exportResults,
// exportPointTracks, exportLineTracks).  The tracker is sequential in frames
// and tiny next to detection, so it runs on the host (match2nd.hpp).
#ifndef LOCOMOUSE_HOST_TRACKS_HPP
#define LOCOMOUSE_HOST_TRACKS_HPP

#include <array>
#include <string>
#include <vector>

#include "Candidates.hpp"
#include "MyMat.hpp"
#include "locomouse_hip.h"
#include "match2nd.hpp"

namespace locomouse {

using TailTrack = std::array<int32_t, 3 * LM_N_TAIL_POINTS>;  // TRACKS_TAIL entry: 3x15, row-major, -1 = missing

// The per-frame result vectors of LocoMouse_class.hpp:219-236, in frame order.
struct FrameResults {
  std::vector<std::vector<Candidate>> CANDIDATES_BOTTOM_PAW, CANDIDATES_BOTTOM_SNOUT;
  std::vector<std::vector<Candidate>> CANDIDATES_SIDE_PAW, CANDIDATES_SIDE_SNOUT;
  std::vector<std::vector<P22D>> CANDIDATES_MATCHED_VIEWS_PAW, CANDIDATES_MATCHED_VIEWS_SNOUT;
  std::vector<MyMat> UNARY_BOTTOM_PAW, UNARY_BOTTOM_SNOUT;
  std::vector<MATSPARSE> PAIRWISE_BOTTOM_PAW, PAIRWISE_BOTTOM_SNOUT;
  std::vector<TailTrack> TRACKS_TAIL;

  // Appends the frames of one lm_batch_result (include/locomouse_hip.h).
  void append(const lm_batch_result& r);
};

// What the track stage reads besides the containers.
struct TrackSetup {
  unsigned n_frames = 0;                    // N_FRAMES
  int nong_bottom = 0;                      // ONG.size() (:726-749)
  int nong_side = 0;                        // ONG_SIDE.size() (:752-759)
  unsigned ong_side_lowest = 0;             // ONG_SIDE_LOWEST_POINT
  int occlusion_grid_spacing_pixels_side = 20;
  int max_displacement_side = 15;
  double alpha_vel_side = 100;
  double pairwise_occluded_cost = 0.01;
  // bottom-right corners per frame and the box sizes (getBoundingBox)
  const std::vector<uint32_t>* bb_x_pos = nullptr;
  const std::vector<uint32_t>* bb_y_bottom_pos = nullptr;
  const std::vector<uint32_t>* bb_y_side_pos = nullptr;
  lm_rect bb_bottom_mouse{}, bb_side_mouse{};
};

TrackSetup make_track_setup(const lm_geometry& g, const lm_params& p, unsigned n_frames);

// The tracks and their export (OUTPUT << "paw_tracks0" << M ...).
struct TrackResults {
  IntMat TRACK_INDEX_PAW_BOTTOM, TRACK_INDEX_SNOUT_BOTTOM;  // 4 x N, 1 x N
  IntMat TRACK_INDEX_PAW_SIDE, TRACK_INDEX_SNOUT_SIDE;
  std::vector<IntMat> paw_tracks;    // 4 of N x 3 (x, y_bottom, z), -1 = missing
  std::vector<IntMat> snout_tracks;  // 1 of N x 3
  IntMat tracks_tail;                // 3 x (15 N)
};

// First four entries of PAW_PERMUTATIONS rows 0..3 (LocoMouse_class.hpp:91-92):
// the reference's loop runs i_perm < N_paws over a 4 x 24 matrix read by row.
extern const int PAW_ORDERS[4][4];

void computeBottomTracks(const FrameResults& R, const TrackSetup& S, TrackResults& out);
void computeSideTracks(const FrameResults& R, const TrackSetup& S, TrackResults& out);
void exportTracks(const FrameResults& R, const TrackSetup& S, TrackResults& out);

MATSPARSE pairwisePotential_SideView(const std::vector<uint32_t>& Zi, const std::vector<uint32_t>& Zip1,
                                     double grid_mapping, double grid_spacing, unsigned Nong,
                                     double max_displacement, double alpha_vel, double pairwise_occluded_cost);
IntMat bestSideViewMatch(const IntMat& T, const std::vector<std::vector<P22D>>& matched, const TrackSetup& S,
                         unsigned N_features);
IntMat exportPointTracks(const IntMat& T_bottom, const IntMat& T_side, const std::vector<std::vector<P22D>>& matched,
                         const TrackSetup& S, unsigned i_feature);
IntMat exportLineTracks(const std::vector<TailTrack>& tracks, const TrackSetup& S, int n_line_points);

// OpenCV FileStorage YAML of exportResults (LocoMouse_class.cpp:360, :2348-2482):
// paw_tracks0..3, snout_tracks0, tracks_tail as !!opencv-matrix, dt: i.
void writeOutputYaml(const std::string& path, const TrackResults& T);

}  // namespace locomouse

#endif
