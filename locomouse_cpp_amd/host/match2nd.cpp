// match2nd.cpp — see match2nd.hpp.  Reference: match2nd/match2nd.cpp:11-190
// and the point/bundle classes of match2nd/match2nd.h:29-563.
#include "match2nd.hpp"

#include <cmath>
#include <iostream>
#include <stdexcept>

namespace locomouse {

namespace {

constexpr double NEG_INF = -INFINITY;

inline double max_of(double a, double b) { return a < b ? b : a; }  // std::max(a, b)

// One match2nd problem.  Frame f has nloc[f] candidate locations followed by
// nong occlusion points; the transitions f -> f+1 are the non-zeros of
// pairwise_costs[f] (CSC: column = location at f, jc[f][c] .. jc[f][c+1];
// ir = location at f+1; pr = cost).
struct Lattice {
  int L = 0, nong = 0;
  double occ_cost = 0, bam = 0;
  std::vector<int> nloc;
  std::vector<const int*> jc, ir;
  std::vector<const double*> pr;
  std::vector<int> nt;        // transitions of pair f
  std::vector<size_t> toff;   // first transition of pair f in a track's margin buffers
  std::vector<size_t> moff;   // first message of frame f
  std::vector<double> msg;    // bundle::message, shared by every track
  double& message(int f, int b) { return msg[moff[f] + (size_t)b]; }
};

// One track (a `point` of the reference) and the sweeps over it.
class TrackSolver {
 public:
  TrackSolver(Lattice& g, std::vector<const double*> unary_cols)
      : G(g), U(std::move(unary_cols)), fwd(g.toff.back()), bwd(g.toff.back()), label(g.L, 0), bestloc(g.L, 0),
        best(g.L, 0.0), second(g.L, 0.0) {}

  // point::margin (match2nd.h:398-418)
  void margin() {
    clear();
    refresh_un();
    for (int f = 0; f < G.L - 1; ++f) forward(f);
    for (int f = G.L - 2; f >= 0; --f) backward(f);
    for (int f = 0; f < G.L - 1; ++f) find_best(f);
    for (int f = 0; f < G.L; ++f)  // update_unary_first
      if (bestloc[f] < G.nloc[f]) G.message(f, bestloc[f]) += second[f] - best[f] - G.bam;
  }

  // point::assign (match2nd.h:445-472)
  void assign() {
    clear();
    for (int f = 0; f < G.L; ++f) {  // update_unary_second_pre
      if (G.bam == INFINITY)
        G.message(f, bestloc[f]) = 0;
      else if (bestloc[f] < G.nloc[f])
        G.message(f, bestloc[f]) += -second[f] + best[f] + G.bam;
    }
    refresh_un();
    for (int f = G.L - 2; f >= 0; --f) backward(f);
    for (int f = 0; f < G.L; ++f) set_label(f);
    for (int f = 0; f < G.L; ++f)  // update_unary_second: a taken candidate is barred for later tracks
      if (label[f] < G.nloc[f] && label[f] >= 0) G.message(f, label[f]) += NEG_INF;
  }

  int label_at(int f) const { return label[f]; }

 private:
  Lattice& G;
  std::vector<const double*> U;  // unary column of this track, per frame
  std::vector<double> fwd, bwd;  // marginforward / marginbackward, by transition
  std::vector<double> unv;       // point::un of every location, valid for one sweep phase
  std::vector<int> label, bestloc;
  std::vector<double> best, second;

  double& F(int f, int k) { return fwd[G.toff[f] + (size_t)k]; }
  double& B(int f, int k) { return bwd[G.toff[f] + (size_t)k]; }

  // point::un: unary (or the occlusion cost) plus the shared message.  The
  // messages change only between sweep phases, so each phase evaluates it
  // once per location (same operands, same value) instead of per transition.
  void refresh_un() {
    unv.resize(G.moff.back());
    for (int f = 0; f < G.L; ++f) {
      double* u = unv.data() + G.moff[f];
      const double* m = G.msg.data() + G.moff[f];
      for (int b = 0; b < G.nloc[f] + G.nong; ++b) u[b] = b < G.nloc[f] ? U[f][b] + m[b] : G.occ_cost + m[b];
    }
  }
  double un(int f, int b) const { return unv[G.moff[f] + (size_t)b]; }

  void clear() {  // clearmargin
    std::fill(label.begin(), label.end(), -2);
    std::fill(fwd.begin(), fwd.end(), NEG_INF);
    std::fill(bwd.begin(), bwd.end(), NEG_INF);
  }

  // forward_point (match2nd.h:200-239): max-plus forward sweep, then the
  // arrival cost of each transition of pair f.
  void forward(int f) {
    if (f) {
      const int* jc = G.jc[f];
      for (int a = 0; a < G.nt[f - 1]; ++a) {
        const int j = G.ir[f - 1][a];
        const double v = F(f - 1, a);
        for (int k = jc[j]; k != jc[j + 1]; ++k) F(f, k) = max_of(F(f, k), v);
      }
    } else {
      for (int i = 0; i < G.nloc[0] + G.nong; ++i)
        for (int k = G.jc[0][i]; k != G.jc[0][i + 1]; ++k) F(0, k) = un(0, i);
    }
    for (int k = 0; k < G.nt[f]; ++k) F(f, k) += un(f + 1, G.ir[f][k]) + G.pr[f][k];
  }

  // backward_point (match2nd.h:241-279)
  void backward(int f) {
    if (f < G.L - 2) {
      const int* jc = G.jc[f + 1];
      for (int a = 0; a < G.nt[f]; ++a) {
        const int j = G.ir[f][a];
        double& b = B(f, a);
        for (int k = jc[j]; k != jc[j + 1]; ++k) b = max_of(b, B(f + 1, k));
      }
    } else {
      for (int a = 0; a < G.nt[f]; ++a) B(f, a) = un(f + 1, G.ir[f][a]);
    }
    for (int i = 0; i < G.nloc[f] + G.nong; ++i)
      for (int k = G.jc[f][i]; k != G.jc[f][i + 1]; ++k) B(f, k) += G.pr[f][k] + un(f, i);
  }

  // findbest (match2nd.h:282-333): best and second-best min-marginal per
  // frame, where only a change of location demotes the best to second.
  void find_best(int f) {
    best[f] = best[f + 1] = NEG_INF;
    second[f] = second[f + 1] = NEG_INF;
    const int* jc = G.jc[f];
    int loc = 0;
    for (int k = 0; k < G.nt[f]; ++k) {
      while (jc[loc + 1] <= k) ++loc;
      const int e = G.ir[f][k];
      const double t = B(f, k) + F(f, k) - un(f, loc) - un(f + 1, e) - G.pr[f][k];
      if (best[f] < t) {
        if (bestloc[f] == loc) {
          best[f] = t;
        } else {
          second[f] = best[f];
          best[f] = t;
          bestloc[f] = loc;
        }
        if (bestloc[f + 1] == e) {
          best[f + 1] = t;
        } else {
          second[f + 1] = best[f + 1];
          best[f + 1] = t;
          bestloc[f + 1] = e;
        }
      } else {
        if (second[f] < t && bestloc[f] != loc) second[f] = t;
        if (second[f + 1] < t && bestloc[f + 1] != e) second[f + 1] = t;
      }
    }
  }

  // forward_set (match2nd.h:335-384): decode the labelling front to back.
  void set_label(int f) {
    double bst = NEG_INF;
    if (f == 1) return;  // set together with frame 0
    if (f == 0) {
      for (int loc = 0; loc < G.nloc[0] + G.nong; ++loc)
        for (int k = G.jc[0][loc]; k != G.jc[0][loc + 1]; ++k) {
          const double c = B(0, k);
          if (bst <= c) {
            bst = c;
            label[0] = loc;
            label[1] = G.ir[0][k];
          }
        }
      if (bst == NEG_INF) label[0] = label[1] = -1;
      return;
    }
    // Only the transition (label[f-2] -> label[f-1]) of pair f-2 qualifies;
    // then the best continuation out of label[f-1].
    const int* jc2 = G.jc[f - 2];
    int loc = 0;
    for (int k = 0; k < G.nt[f - 2]; ++k) {
      while (jc2[loc + 1] <= k) ++loc;
      const int j = G.ir[f - 2][k];
      if (loc != label[f - 2] || j != label[f - 1]) continue;
      for (int q = G.jc[f - 1][j]; q != G.jc[f - 1][j + 1]; ++q) {
        const double c = G.pr[f - 1][q] + B(f - 1, q);
        if (bst < c) {
          bst = c;
          label[f] = G.ir[f - 1][q];
        }
      }
    }
    if (bst == NEG_INF) label[f] = -1;
  }
};

}  // namespace

IntMat match2nd(const std::vector<MyMat>& unary_costs, const std::vector<MATSPARSE>& pairwise_costs, int Nong,
                double occlusion_point_cost, double bam_tie, unsigned frames, unsigned points, const int* permutation) {
  IntMat T((int)points, (int)frames, 0);
  if (frames < 2 || points < 1) {
    std::cout << "There must be at least one point and 2 frames." << std::endl;  // match2nd.cpp:24-27
    return T;
  }
  if (unary_costs.size() < frames || pairwise_costs.size() < frames - 1)
    throw std::runtime_error("match2nd: fewer cost matrices than frames.");
  Lattice G;
  G.L = (int)frames;
  G.nong = Nong;
  G.occ_cost = occlusion_point_cost;
  G.bam = bam_tie;
  G.nloc.resize(frames);
  for (unsigned f = 0; f < frames; ++f) {
    if (unary_costs[f].Ncols() != (int)points) {
      std::cout << "Wrong form of unary potentials." << unary_costs[f].Ncols() << "!=" << points << std::endl;
      return T;
    }
    G.nloc[f] = unary_costs[f].Nrows();
  }
  G.toff.assign(1, 0);
  for (unsigned f = 0; f + 1 < frames; ++f) {
    const MATSPARSE& P = pairwise_costs[f];
    if (P.Nrows() != G.nloc[f + 1] + Nong || P.Ncols() != G.nloc[f] + Nong) return T;  // :83-100
    G.jc.push_back(P.getJc());
    G.ir.push_back(P.getIr());
    G.pr.push_back(P.getPr());
    G.nt.push_back(P.nz());
    G.toff.push_back(G.toff.back() + (size_t)P.nz());
  }
  G.moff.assign(1, 0);
  for (unsigned f = 0; f < frames; ++f) G.moff.push_back(G.moff.back() + (size_t)(G.nloc[f] + Nong));
  G.msg.assign(G.moff.back(), 0.0);

  std::vector<TrackSolver> tracks;
  tracks.reserve(points);
  for (unsigned p = 0; p < points; ++p) {
    std::vector<const double*> cols(frames);
    for (unsigned f = 0; f < frames; ++f)
      cols[f] = unary_costs[f].getValues() + (size_t)permutation[p] * (size_t)G.nloc[f];
    tracks.emplace_back(G, std::move(cols));
  }
  for (auto& t : tracks) t.margin();  // bundle::run (match2nd.h:521-548)
  for (int p = (int)points - 1; p >= 0; --p) tracks[p].assign();
  for (unsigned p = 0; p < points; ++p)
    for (unsigned f = 0; f < frames; ++f) T.at((int)p, (int)f) = tracks[p].label_at((int)f);
  return T;
}

double computeCostTrack(const IntMat& M, const std::vector<MyMat>& unary_costs, const std::vector<MATSPARSE>&,
                        const int* permutation) {
  double c = 0;
  const int n_frames = M.cols;
  if (M.rows < 4) throw std::runtime_error("computeCostTrack: fewer than 4 tracks.");
  if ((int)unary_costs.size() < n_frames) throw std::runtime_error("computeCostTrack: fewer unary matrices than frames.");
  for (int t = 0; t < 4; ++t) {
    const int32_t* m = M.row(t);
    for (int f = 0; f < n_frames; ++f) {
      const MyMat& U = unary_costs[f];
      double un = 0;  // occlusion point
      if (m[f] < U.Nrows()) {
        const uint32_t idx = (uint32_t)permutation[t] * (uint32_t)U.Nrows() + (uint32_t)m[f];
        if (idx >= (uint32_t)U.Numel())
          throw std::runtime_error("computeCostTrack: label -1 reads outside the unary matrix.");
        un = U.getValues()[idx];
      }
      c += un;
      if (f < n_frames - 1) c += 0.0;  // MATSPARSE::get(...) == 0
    }
  }
  return c;
}

}  // namespace locomouse
