// match2nd.hpp — the tracker that turns the per-frame cost containers of the
// detection path into tracks.
//
// Same entry points and results as the reference's match2nd/match2nd.cpp:
//   match2nd(unary, pairwise, Nong, occlusion_point_cost, bam_tie, frames,
//            points, permutation)                       (match2nd.cpp:11-166)
//   computeCostTrack(M, unary, pairwise, permutation)   (match2nd.cpp:168-190)
// The reference keeps its problem in file-scope globals (locations, occ,
// occ_score, BAM) and per-frame malloc'd margin arrays; here one call owns a
// Lattice (frame sizes, the CSC transition views, the message array every
// track shares) and each track keeps its forward/backward margins in one
// flat buffer indexed by transition.  The arithmetic — order of the
// max-plus sweeps, the best/second-best bookkeeping, the message updates
// between tracks — is the reference's, so labels are bit-identical
// (tests/test_tracks.py against oracle/track_oracle.py).
#ifndef LOCOMOUSE_HOST_MATCH2ND_HPP
#define LOCOMOUSE_HOST_MATCH2ND_HPP

#include <cstdint>
#include <vector>

#include "MyMat.hpp"

namespace locomouse {

// cv::Mat of CV_32SC1 as the tracker returns it: rows x cols, row-major.
struct IntMat {
  int rows = 0, cols = 0;
  std::vector<int32_t> data;
  IntMat() = default;
  IntMat(int r, int c, int32_t fill = 0) : rows(r), cols(c), data((size_t)r * c, fill) {}
  int32_t* row(int r) { return data.data() + (size_t)r * cols; }
  const int32_t* row(int r) const { return data.data() + (size_t)r * cols; }
  int32_t& at(int r, int c) { return data[(size_t)r * cols + c]; }
  int32_t at(int r, int c) const { return data[(size_t)r * cols + c]; }
  bool empty() const { return data.empty(); }
};

// points x frames labels: for track i (unary column permutation[i]) and frame
// f, the index of the chosen location — a row of unary_costs[f] (a candidate)
// or locations[f] + k for occlusion point k; -1 when no labelling exists.
// On malformed input (frames < 2, points < 1, a unary matrix without `points`
// columns, a pairwise matrix of the wrong size) the reference returns zeros
// (match2nd.cpp:24-27, :46-49, :83-100); so does this.
IntMat match2nd(const std::vector<MyMat>& unary_costs, const std::vector<MATSPARSE>& pairwise_costs, int Nong,
                double occlusion_point_cost, double bam_tie, unsigned frames, unsigned points, const int* permutation);

// Sum over tracks 0..3 and frames of the unary cost of the chosen label
// (0 for occlusion points).  The pairwise term goes through MATSPARSE::get,
// which returns 0 (MyMat.cpp:371-374), so it adds nothing — kept.
// A label of -1 makes the reference read unary[(perm*rows - 1) mod 2^32];
// that element is returned when it lies inside the matrix, otherwise
// std::runtime_error is thrown (the reference reads unmapped memory).
double computeCostTrack(const IntMat& M, const std::vector<MyMat>& unary_costs,
                        const std::vector<MATSPARSE>& pairwise_costs, const int* permutation);

}  // namespace locomouse

#ifndef LOCOMOUSE_NO_GLOBAL_NAMES
using locomouse::IntMat;
#endif

#endif
