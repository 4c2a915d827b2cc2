// Candidates.hpp — host-side value types of the per-frame detection results.
//
// Same names, members and method semantics as the reference's Candidate /
// P22D (Candidates/Candidates.hpp:16-105, Candidates.cpp:1-156), without the
// OpenCV dependency: Point_<int> is a two-int struct and the FileStorage
// read/write methods belong to the YAML formats, not
// to this path.  Candidate is layout-identical to lm_candidate of the C-ABI
// (include/locomouse_hip.h), so batch results are appended without conversion.
#ifndef LOCOMOUSE_HOST_CANDIDATES_HPP
#define LOCOMOUSE_HOST_CANDIDATES_HPP

#include <cstddef>
#include <ostream>
#include <vector>

#include "locomouse_hip.h"

namespace locomouse {

template <class T>
struct Point_ {
  T x, y;
  Point_() : x(0), y(0) {}
  Point_(T X, T Y) : x(X), y(Y) {}
  bool operator==(const Point_& o) const { return x == o.x && y == o.y; }
  bool operator!=(const Point_& o) const { return !(*this == o); }
};

// Candidate (Candidates.hpp:16-34): default (-1,-1) with score -1 (Candidates.cpp:4-7).
class Candidate {
 public:
  Point_<int> p;
  double s;

  Candidate() : p(-1, -1), s(-1) {}
  Candidate(int x, int y, double scr) : p(x, y), s(scr) {}
  Candidate(Point_<int> P, double scr) : p(P), s(scr) {}

  inline Point_<int> point() const { return p; }
  inline double score() const { return s; }
  inline void set_score(double new_s) { s = new_s; }
};

// std::sort comparator of nmsMax / peakClustering (Candidates.cpp:33-36).
bool compareCandidate(Candidate a, Candidate b);

// P22D (Candidates.hpp:63-105): a bottom-view candidate plus the side-view
// y positions / scores matched to it.  yt/st always hold >= 1 entry; the
// "no side candidate" state is st[0] < 0 (Candidates.cpp:148-156).
class P22D {
  Candidate CB;
  std::vector<int> yt;
  std::vector<double> st;

 public:
  P22D();                                          // CB = Candidate(), yt = {-1}, st = {-1}
  P22D(int xc, int ybc, int ytc, double scr_b, double scr_t);
  P22D(Point_<int> Pb, Point_<int> Pt, double scr_b, double scr_t);
  P22D(Candidate Cb, Candidate Ct);

  Point_<int> point_bottom() const;
  Point_<int> point_side(unsigned index) const;
  double score_bottom() const;
  double score_side(unsigned index) const;
  int x_coord() const;
  int y_bottom_coord() const;
  int y_side_coord(unsigned index) const;

  void add_side_candidate(Candidate C);
  void add_side_candidate(Point_<int> P, double s);
  void add_side_candidate(int y, double s);

  int number_of_candidates() const;
  Candidate get_candidate_side(unsigned index) const;
  Candidate get_candidate_bottom() const;

  // Restores the raw yt/st vectors recorded by the device path (entry j of
  // the side arrays), including the st[0] < 0 "no match" state.
  void set_side_raw(const int* y, const double* s, int count);
  const std::vector<int>& raw_side_y() const { return yt; }
  const std::vector<double>& raw_side_s() const { return st; }

  bool operator==(const P22D& o) const;

 private:
  void add_side_candidate_safe(int X, int Y, double S);
};

std::ostream& operator<<(std::ostream& out, const Candidate& c);
std::ostream& operator<<(std::ostream& out, const P22D& c);

static_assert(sizeof(Candidate) == sizeof(lm_candidate), "Candidate must match lm_candidate");
static_assert(offsetof(Candidate, s) == offsetof(lm_candidate, score), "Candidate must match lm_candidate");

}  // namespace locomouse

#ifndef LOCOMOUSE_NO_GLOBAL_NAMES
using locomouse::Candidate;
using locomouse::compareCandidate;
using locomouse::P22D;
#endif

#endif
