/*
 * lm_oracle.cpp — CPU restatement of LocoMouse_cpp's per-frame detection path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * product (locomouse_cpp_amd/csrc) and the timed CPU baseline of bench.py
 * ("kind": "port").  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it; the product never links or calls it.
 *
 * PARITY UNPINNED.  The reference (/root/reference, C++11 + OpenCV 3.x) cannot
 * be built here: OpenCV is absent from this image and from the GPU box, and
 * the reference ships no tests, fixtures or golden data.
 * This restatement therefore follows the reference source line by line (each
 * function cites reference file:line) and spells out the OpenCV 3.x primitive
 * semantics the reference relies on (filter2D, normalize/convertTo, threshold,
 * connectedComponentsWithStats, moments, Rect/Point arithmetic, cvRound).
 * libstdc++'s std::sort (the reference's only other dependency on the path)
 * is called directly, so candidate tie order is the real libstdc++ order.
 *
 * Documented choices where OpenCV's behaviour is build dependent:
 *  - filter2D 8U->32F accumulates from (float)delta over the non-zero taps in
 *    row-major order.  OpenCV >= 3.4.9 / 4.x dispatched to AVX2 fuses each tap
 *    (v_muladd -> vfmadd); 3.x SSE2 builds do mul then add.  Default here:
 *    fused (flag LMO_UNFUSED_FILTER selects mul+add for comparison).
 *  - normalize(NORM_MINMAX) -> convertTo(CV_8U, scale, shift) evaluates
 *    sat_u8(cvRound((float)p * (float)scale + (float)shift)) unfused (3.x).
 *  - connectedComponentsWithStats label order (only visible through the
 *    strict '>' largest-area tie-break, LocoMouse_class.cpp:2752-2756):
 *    8-connectivity = Grana BBDT 2x2-block raster order of a component's first
 *    block; 4-connectivity = Wu/SAUF pixel raster order.
 *
 * Build: oracle/Makefile (g++ -O3 -march=x86-64-v3 -ffp-contract=off).
 */
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "locomouse_hip.h"
#include "lm_synth.h"

#define LMO_API extern "C" __attribute__((visibility("default")))

enum { LMO_KEEP_DEBUG = 1, LMO_UNFUSED_FILTER = 2 };

namespace lmo {

// ---------------------------------------------------------------- cv-lite
struct Point {
  int x = 0, y = 0;
};
struct Rect {  // cv::Rect
  int x = 0, y = 0, width = 0, height = 0;
  Rect() = default;
  Rect(int x_, int y_, int w_, int h_) : x(x_), y(y_), width(w_), height(h_) {}
  int area() const { return width * height; }
};
static Rect operator&(const Rect& a, const Rect& b) {  // cv::Rect operator&= (types.hpp)
  int x1 = std::max(a.x, b.x), y1 = std::max(a.y, b.y);
  int w = std::min(a.x + a.width, b.x + b.width) - x1;
  int h = std::min(a.y + a.height, b.y + b.height) - y1;
  if (w <= 0 || h <= 0) return Rect();
  return Rect(x1, y1, w, h);
}
static Rect shift(const Rect& r, int dx, int dy) { return Rect(r.x + dx, r.y + dy, r.width, r.height); }

template <class T>
struct Mat {
  int rows = 0, cols = 0;
  std::vector<T> d;
  Mat() = default;
  Mat(int r, int c, T v = T()) : rows(r), cols(c), d((size_t)r * c, v) {}
  T& at(int r, int c) { return d[(size_t)r * cols + c]; }
  const T& at(int r, int c) const { return d[(size_t)r * cols + c]; }
  T* row(int r) { return d.data() + (size_t)r * cols; }
  const T* row(int r) const { return d.data() + (size_t)r * cols; }
};
using Mat8 = Mat<uint8_t>;
using Matf = Mat<float>;

static void check_roi(const Rect& roi, int rows, int cols, const char* what) {
  // cv::Mat(const Mat&, const Rect&) asserts (matrix.cpp)
  if (roi.x < 0 || roi.y < 0 || roi.width < 0 || roi.height < 0 || roi.x + roi.width > cols ||
      roi.y + roi.height > rows)
    throw std::runtime_error(std::string("ROI out of image bounds: ") + what);
}

struct Candidate {  // Candidates.hpp:16-34
  int x = -1, y = -1;
  double s = -1;
  Candidate() = default;
  Candidate(int x_, int y_, double s_) : x(x_), y(y_), s(s_) {}
};
static bool compareCandidate(Candidate a, Candidate b) { return a.s > b.s; }  // Candidates.cpp:33-36

struct P22D {  // Candidates.hpp:63-105
  Candidate CB;
  std::vector<int> yt;
  std::vector<double> st;
  P22D(const Candidate& cb, const Candidate& ct) {  // Candidates.cpp:72-80
    CB = Candidate(cb.x, cb.y, cb.s);
    yt.push_back(ct.y);
    st.push_back(ct.s);
  }
  int number_of_candidates() const { return st[0] < 0 ? 0 : (int)st.size(); }  // :148-156
  void add_side_candidate(const Candidate& c) {                            // :106-115
    if (number_of_candidates() == 0) {
      yt[0] = c.y;
      st[0] = c.s;
      return;
    }
    if (!(c.s >= 0)) throw std::runtime_error("P22D::add_side_candidate_safe: CV_Assert(S >= 0)");
    yt.push_back(c.y);
    st.push_back(c.s);
  }
};

struct MyMat {  // MyMat.cpp:55-70 — column-major doubles
  int nrows = 0, ncols = 0;
  std::vector<double> v;
  MyMat(int n, int m) : nrows(n), ncols(m), v((size_t)n * m, 0.0) {}
  void put(int i, int j, double val) { v[(size_t)j * nrows + i] = val; }
  double get(int i, int j) const { return v[(size_t)j * nrows + i]; }
};

struct MatSparse {  // MyMat.cpp:141-178
  int n_rows = 0, n_cols = 0;
  std::vector<int> jc, ir;
  std::vector<double> pr;
  explicit MatSparse(const MyMat& M) {
    n_rows = M.nrows;
    n_cols = M.ncols;
    jc.push_back(0);
    int nz = 0;
    for (int j = 0; j < M.ncols; ++j) {
      for (int i = 0; i < M.nrows; ++i) {
        double g = M.get(i, j);
        if (g != 0) {
          ir.push_back(i);
          pr.push_back(g);
          ++nz;
        }
      }
      jc.push_back(nz);
    }
  }
};

struct LocationPrior {  // LocoMouse_class.cpp:3196-3202
  double px, py, max_distance;
  double ax, ay, aw, ah;  // Rect_<double>(minx, miny, maxx - minx, maxy - miny)
  explicit LocationPrior(const lm_location_prior& p) {
    if (!(p.min_x < p.max_x) || !(p.min_y < p.max_y))
      throw std::invalid_argument("location_prior: CV_Assert(minx < maxx && miny < maxy)");
    px = p.x;
    py = p.y;
    max_distance = p.max_distance;
    ax = p.min_x;
    ay = p.min_y;
    aw = p.max_x - p.min_x;
    ah = p.max_y - p.min_y;
  }
  bool contains(double x, double y) const {  // Point_::inside -> Rect_::contains
    return ax <= x && x < ax + aw && ay <= y && y < ay + ah;
  }
};

struct Feature {  // LocoMouse_Feature, LocoMouse_class.cpp:2941-2990
  std::vector<float> wb, ws;  // kernels converted to float (filter2D kdepth = CV_32F)
  int rows_b = 0, cols_b = 0, rows_s = 0, cols_s = 0;
  double rho_b = 0, rho_s = 0;
  Rect match_b, match_s;
  Feature() = default;
  Feature(const lm_detector& b, const lm_detector& s) {
    rows_b = b.rows;
    cols_b = b.cols;
    rows_s = s.rows;
    cols_s = s.cols;
    rho_b = b.bias;
    rho_s = s.bias;
    wb.resize((size_t)rows_b * cols_b);
    ws.resize((size_t)rows_s * cols_s);
    for (size_t i = 0; i < wb.size(); ++i) wb[i] = (float)b.weights[i];
    for (size_t i = 0; i < ws.size(); ++i) ws[i] = (float)s.weights[i];
    int new_b_w = (int)std::round((double)cols_b / 2), new_b_h = (int)std::round((double)rows_b / 2);
    int new_t_w = (int)std::round((double)cols_s / 2), new_t_h = (int)std::round((double)rows_s / 2);
    match_b = Rect(-(new_b_w / 2), -(new_b_h / 2), new_b_w, new_b_h);
    match_s = Rect(-(new_t_w / 2), -(new_t_h / 2), new_t_w, new_t_h);
  }
};

// ------------------------------------------------------------- primitives

// cv::filter2D(src_roi, dst, CV_32F, K, Point(-1,-1), delta, BORDER_CONSTANT) on a
// ROI of `parent` WITHOUT BORDER_ISOLATED: taps outside the ROI read the parent,
// taps outside the parent read 0.  Only the sub-rectangle `sub` (relative to the
// ROI) of the output is produced — the only part the reference consumes.
static void filter2D_roi(const Mat8& parent, const Rect& roi, const std::vector<float>& k, int kh, int kw,
                         double delta_d, const Rect& sub, Matf& out, bool fused) {
  const int ay = kh / 2, ax = kw / 2;  // anchor (-1,-1) -> ksize/2
  const float delta = (float)delta_d;   // saturate_cast<float>(delta)
  const int r0 = roi.y + sub.y - ay, c0 = roi.x + sub.x - ax;
  const int pr = sub.height + kh - 1, pc = sub.width + kw - 1;
  Mat8 pad(pr, pc, 0);
  for (int r = 0; r < pr; ++r) {
    int sr = r0 + r;
    if (sr < 0 || sr >= parent.rows) continue;
    for (int c = 0; c < pc; ++c) {
      int sc = c0 + c;
      if (sc >= 0 && sc < parent.cols) pad.at(r, c) = parent.at(sr, sc);
    }
  }
  out = Matf(sub.height, sub.width, delta);
  for (int y = 0; y < sub.height; ++y) {
    float* acc = out.row(y);
    for (int i = 0; i < kh; ++i) {
      const uint8_t* srow = pad.row(y + i);
      for (int j = 0; j < kw; ++j) {
        const float w = k[(size_t)i * kw + j];
        if (w == 0.0f) continue;  // preprocess2DKernel keeps non-zero taps only
        const uint8_t* s = srow + j;
        if (fused) {
          for (int x = 0; x < sub.width; ++x) acc[x] = std::fmaf(w, (float)s[x], acc[x]);
        } else {
          for (int x = 0; x < sub.width; ++x) acc[x] = acc[x] + w * (float)s[x];
        }
      }
    }
  }
}

// Label image of the largest connected component (selectLargestRegion,
// LocoMouse_class.cpp:2744-2767): 255 on the chosen component, else 0.
static Mat8 selectLargestRegion(const Mat8& bin, int connectivity) {
  const int R = bin.rows, C = bin.cols;
  std::vector<int> parent((size_t)R * C, -1);
  auto find = [&](int a) {
    while (parent[a] != a) {
      parent[a] = parent[parent[a]];
      a = parent[a];
    }
    return a;
  };
  auto unite = [&](int a, int b) {
    a = find(a);
    b = find(b);
    if (a == b) return;
    if (a < b) parent[b] = a; else parent[a] = b;
  };
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c) {
      if (!bin.at(r, c)) continue;
      int id = r * C + c;
      parent[id] = id;
      auto link = [&](int rr, int cc) {
        if (rr < 0 || cc < 0 || cc >= C) return;
        if (bin.at(rr, cc)) unite(id, rr * C + cc);
      };
      link(r, c - 1);
      link(r - 1, c);
      if (connectivity == 8) {
        link(r - 1, c - 1);
        link(r - 1, c + 1);
      }
    }
  std::map<int, std::pair<long, long>> comp;  // root -> (area, first key)
  const int nbx = (C + 1) / 2;
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c) {
      if (!bin.at(r, c)) continue;
      int root = find(r * C + c);
      long key = connectivity == 8 ? (long)(r / 2) * nbx + c / 2 : (long)r * C + c;
      auto it = comp.find(root);
      if (it == comp.end()) comp[root] = {1, key};
      else {
        it->second.first += 1;
        it->second.second = std::min(it->second.second, key);
      }
    }
  Mat8 out(R, C, 0);
  if (comp.empty()) return out;  // N_labels == 1 -> zeros (:2762-2764)
  // OpenCV numbers labels by first (block) occurrence; strict '>' keeps the first.
  std::vector<std::pair<long, std::pair<long, int>>> order;  // (key, (area, root))
  for (auto& kv : comp) order.push_back({kv.second.second, {kv.second.first, kv.first}});
  std::sort(order.begin(), order.end());
  long best_area = order[0].second.first;
  int best_root = order[0].second.second;
  for (size_t i = 1; i < order.size(); ++i)
    if (order[i].second.first > best_area) {
      best_area = order[i].second.first;
      best_root = order[i].second.second;
    }
  for (int r = 0; r < R; ++r)
    for (int c = 0; c < C; ++c)
      if (bin.at(r, c) && find(r * C + c) == best_root) out.at(r, c) = 255;
  return out;
}

// cv::moments(roi, binaryImage = true) — m00, m10, m01 only.  OpenCV (moments.cpp)
// walks 32x32 tiles in raster order, binarises each tile to 0/255 (compare NE 0),
// accumulates integer tile moments, scales them by 1./255 and adds
// m00 += t00; m10 += t10 + x*t00; m01 += t01 + y*t00 (x, y = tile origin).
struct Moments3 {
  double m00 = 0, m10 = 0, m01 = 0;
};
static Moments3 moments_binary(const Mat8& img, const Rect& roi) {
  const int TILE = 32;
  Moments3 m;
  if (roi.width <= 0 || roi.height <= 0) return m;
  for (int y = 0; y < roi.height; y += TILE) {
    const int th = std::min(TILE, roi.height - y);
    for (int x = 0; x < roi.width; x += TILE) {
      const int tw = std::min(TILE, roi.width - x);
      long t00 = 0, t10 = 0, t01 = 0;
      for (int yy = 0; yy < th; ++yy) {
        long x0 = 0, x1 = 0;
        for (int xx = 0; xx < tw; ++xx) {
          long p = img.at(roi.y + y + yy, roi.x + x + xx) ? 255 : 0;
          x0 += p;
          x1 += xx * p;
        }
        t01 += yy * x0;
        t10 += x1;
        t00 += x0;
      }
      const double s = 1. / 255;
      double mom0 = (double)t00 * s, mom1 = (double)t10 * s, mom2 = (double)t01 * s;
      double xm = x * mom0, ym = y * mom0;
      m.m00 += mom0;
      m.m10 += mom1 + xm;
      m.m01 += mom2 + ym;
    }
  }
  return m;
}

// cvRound(double): round half to even (lrint under the default rounding mode)
static int cvRound(double v) { return (int)std::nearbyint(v); }

// nmsMax, LocoMouse_class.cpp:1610-1747
static std::vector<Candidate> nmsMax(const Matf& box, int bw, int bh, double overlap) {
  std::vector<Candidate> detections;
  for (int r = 0; r < box.rows; ++r) {
    const float* p = box.row(r);
    for (int c = 0; c < box.cols; ++c)
      if (p[c] > 0) detections.push_back(Candidate(c, r, p[c]));
  }
  const unsigned N = (unsigned)detections.size();
  if (N == 0) return {};
  std::sort(detections.begin(), detections.end(), compareCandidate);
  std::vector<unsigned> maxima_index(N), candidate_index;
  std::map<unsigned, unsigned> maxima_index_mapping;
  unsigned candidate_counter = 0;
  const double area2 = 2.0 * (bw * bh);
  std::vector<bool> discard(N, false);
  for (unsigned i = 0; i < N; ++i) {
    Rect r1(detections[i].x, detections[i].y, bw, bh);
    if (!discard[i]) {
      candidate_index.push_back(i);
      maxima_index[i] = i;
      maxima_index_mapping[i] = candidate_counter++;
    }
    for (unsigned j = i + 1; j < N; ++j) {
      if (discard[j]) continue;
      Rect R = r1 & Rect(detections[j].x, detections[j].y, bw, bh);
      if (R.area() == 0) continue;
      double criterion = R.area() / (area2 - R.area());
      if (criterion > overlap) {
        discard[j] = true;
        maxima_index[j] = maxima_index[i];
      }
    }
  }
  const unsigned NC = (unsigned)candidate_index.size();
  std::vector<double> wx(NC, 0.0), wy(NC, 0.0), ss(NC, 0.0);
  for (unsigned k = 0; k < N; ++k) {
    unsigned m = maxima_index_mapping[maxima_index[k]];
    const double s = detections[k].s;
    wx[m] += (double)detections[k].x * s;  // Point_<double> * double, then +=
    wy[m] += (double)detections[k].y * s;
    ss[m] += s;
  }
  std::vector<Candidate> out(NC);
  for (unsigned m = 0; m < NC; ++m)  // Point_<double> / double -> Point_<int> via cvRound
    out[m] = Candidate(cvRound(wx[m] / ss[m]), cvRound(wy[m] / ss[m]), detections[candidate_index[m]].s);
  return out;
}

// peakClustering, LocoMouse_class.cpp:1749-1905 (cluster_method ignored)
static std::vector<Candidate> peakClustering(const Matf& box, int bw, int bh, double overlap) {
  std::vector<Candidate> candidates, detections;
  for (int r = 0; r < box.rows; ++r) {
    const float* p = box.row(r);
    for (int c = 0; c < box.cols; ++c)
      if (p[c] > 0) detections.push_back(Candidate(c, r, p[c]));
  }
  const int N = (int)detections.size();
  if (N == 0) return candidates;
  std::sort(detections.begin(), detections.end(), compareCandidate);
  const double area2 = 2.0 * bh * bw;
  std::vector<bool> kp(N, false);
  for (int i = 0; i < N; ++i) {
    if (kp[i]) continue;
    std::vector<Candidate> cluster{detections[i]};
    Rect r1(detections[i].x, detections[i].y, bw, bh);
    for (int j = i + 1; j < N; ++j) {
      if (kp[j]) continue;
      Rect R = r1 & Rect(detections[j].x, detections[j].y, bw, bh);
      if (R.area() == 0) continue;
      double criterion = R.area() / (area2 - R.area());
      if (criterion > overlap) {
        kp[j] = true;
        cluster.push_back(detections[j]);
      }
    }
    if (cluster.size() > 1) {
      double px = 0, py = 0, sum = 0;
      for (const Candidate& c : cluster) {
        px += (double)c.x * c.s;
        py += (double)c.y * c.s;
        sum += c.s;
      }
      px = px / sum;
      py = py / sum;
      candidates.push_back(Candidate((int)std::round(px), (int)std::round(py), detections[i].s));
    } else {
      candidates.push_back(cluster[0]);
    }
  }
  return candidates;
}

// ------------------------------------------------------------ the pipeline

struct Result {
  std::vector<int64_t> cand_offset{0};
  std::vector<lm_candidate> cand;
  std::vector<int64_t> p22d_offset{0};
  std::vector<lm_p22d> p22d;
  std::vector<int32_t> side_y;
  std::vector<double> side_s;
  std::vector<int64_t> unary_offset{0};
  std::vector<double> unary;
  std::vector<int32_t> pw_dims;
  std::vector<int64_t> pw_jc_offset{0}, pw_nz_offset{0};
  std::vector<int32_t> pw_jc, pw_ir;
  std::vector<double> pw_pr;
  std::vector<int32_t> tail;
  // debug
  std::vector<std::vector<Matf>> scores;  // [frame][6]
  std::vector<Mat8> tail_mask;
  std::vector<Mat8> ipad;
};

class LocoMouseOracle {
 public:
  LocoMouseOracle(const lm_setup& su, const lm_params& pa, const lm_model& mo, int flags) : flags_(flags), P(pa) {
    // --- LocoMouse_Parameters validation (LocoMouse_class.cpp:33-249)
    if (P.conn_comp_connectivity != 4 && P.conn_comp_connectivity != 8)
      throw std::invalid_argument("Invalid configuration parameter: conn_comp_connectivity must be either 4 or 8.");
    if (P.side_bottom_min_overlap < 0 || P.side_bottom_min_overlap > 1)
      throw std::invalid_argument("Invalid configuration parameter: side_bottom_min_overlap must belong to [0,1].");
    if (P.max_displacement_bottom < 0 || P.max_displacement_side < 0 || P.occlusion_grid_spacing_pixels_side < 0 ||
        P.occlusion_grid_spacing_pixels_bottom < 0 || P.alpha_vel_bottom < 0 || P.alpha_vel_side < 0 ||
        P.pairwise_occluded_cost < 0)
      throw std::invalid_argument("Invalid configuration parameter: must be non-negative.");
    if (P.occlusion_grid_max_width < 0 || P.occlusion_grid_max_width > 1 || P.tail_sub_bounding_box < 0 ||
        P.tail_sub_bounding_box > 1)
      throw std::invalid_argument("Invalid configuration parameter: must belong to [0,1].");
    if (!P.use_provided_bounding_box)
      throw std::invalid_argument("use_provided_bounding_box = 0 needs the whole-video BB pass (not on this path).");
    if (P.use_reference_image_brightness)
      throw std::runtime_error("use_reference_image_brightness: computeNormalizedCDF into an unallocated cv::Mat (LocoMouse_class.cpp:189, :3392-3405).");
    if (P.transform_gray_values && !P.use_reference_image_brightness) {
      // LUT(I_BOTTOM_MOUSE, REF_CDF_GLT, I_BOTTOM_MOUSE) (:1445-1448): cv::LUT creates dst with the
      // table's depth; only a CV_8U table leaves the ROI of I_PAD in place, any other depth makes
      // I_BOTTOM_MOUSE a new Mat whose threshold / setTo(0, mask) asserts (:782, :849).
      if (P.gray_value_transformation_depth != LM_DEPTH_8U)
        throw std::runtime_error("transform_gray_values: LUT with a non-8U table re-creates the bottom crop with the table's type (LocoMouse_class.cpp:1448, :782, :849).");
      for (int i = 0; i < 256; ++i) {
        const float v = P.gray_value_transformation[i];
        if (!(v >= 0.f && v <= 255.f && v == std::floor(v)))
          throw std::invalid_argument("gray_value_transformation: a CV_8U table holds integers 0..255.");
        GLT[i] = (uint8_t)v;
      }
      use_glt = true;
    }
    for (int k = 0; k < 4; ++k) prior_paw.emplace_back(P.location_prior[k]);
    prior_snout.emplace_back(P.location_prior[4]);
    // --- loaders / validateImageVideoSize (:402-540)
    if (!su.background || !su.ind_warp_mapping) throw std::invalid_argument("background / calibration missing.");
    VR = su.video_rows;
    VC = su.video_cols;
    N_ROWS = su.calib_rows;
    N_COLS = su.calib_cols;
    if (VR <= 0 || VC <= 0 || N_ROWS <= 0 || N_COLS <= 0) throw std::invalid_argument("empty video or calibration.");
    BKG.assign(su.background, su.background + (size_t)VR * VC);
    CAL.assign(su.ind_warp_mapping, su.ind_warp_mapping + (size_t)N_ROWS * N_COLS);
    int32_t mn = *std::min_element(CAL.begin(), CAL.end()), mx = *std::max_element(CAL.begin(), CAL.end());
    if (mn < 0 || mx >= VR * VC) throw std::runtime_error("Calibration mapping indices out of range.");
    const lm_rect& ub = P.bounding_box_bottom;
    const lm_rect& us = P.bounding_box_side;
    if (ub.x < 0 || ub.y < 0 || ub.x + ub.width >= N_COLS || ub.y + ub.height >= N_ROWS)
      throw std::runtime_error("Provided bounding box for the bottom view exceeds the image dimensions.");
    if (us.x < 0 || us.y < 0 || us.x + us.width >= N_COLS || us.y + us.height >= N_ROWS)
      throw std::runtime_error("Provided bounding box for the side view exceeds the image dimensions.");
    METHOD = su.method;
    IMAGE_FLIP = su.flip != 0;
    FILTER_ARITH = su.filter_arith;
    // --- LocoMouse_Model (:3095-3179)
    auto chk = [](const lm_detector& d, const char* n) {
      if (!d.weights || d.rows <= 0 || d.cols <= 0)
        throw std::invalid_argument(std::string("Error: ") + n + " cannot be empty.");
    };
    chk(mo.paw_side, "modelPaw_side");
    chk(mo.paw_bottom, "modelPaw_bottom");
    chk(mo.tail_side, "modelTail_side");
    chk(mo.tail_bottom, "modelTail_bottom");
    chk(mo.snout_side, "modelSnout_side");
    chk(mo.snout_bottom, "modelSnout_bottom");
    paw = Feature(mo.paw_bottom, mo.paw_side);
    snout = Feature(mo.snout_bottom, mo.snout_side);
    tail = Feature(mo.tail_bottom, mo.tail_side);
    int mts_c = std::max(mo.paw_side.cols, mo.snout_side.cols), mts_r = std::max(mo.paw_side.rows, mo.snout_side.rows);
    int mtb_c = std::max(mo.paw_bottom.cols, mo.snout_bottom.cols),
        mtb_r = std::max(mo.paw_bottom.rows, mo.snout_bottom.rows);
    spre_t = Point{(int)std::ceil((double)(mts_c - 1) / 2), (int)std::ceil((double)(mts_r - 1) / 2)};
    spre_b = Point{(int)std::ceil((double)(mtb_c - 1) / 2), (int)std::ceil((double)(mtb_r - 1) / 2)};
    spost_t = Point{(mts_c - 1) / 2, (mts_r - 1) / 2};
    spost_b = spre_b;  // move-assign bug: spost_b = other.size_pre_bottom() (:3173)
    // --- getBoundingBox, provided-box branch (:545-568)
    BB_X = (unsigned)(ub.x + ub.width);
    BB_YS = (unsigned)(us.y + us.height);
    BB_YB = (unsigned)(ub.y + ub.height);
    BB_BOTTOM_MOUSE = Rect(0, 0, ub.width, ub.height);
    BB_SIDE_MOUSE = Rect(0, 0, us.width, us.height);
    initializeFeatureLoop();
  }

  // LocoMouse::initializeFeatureLoop, :655-769
  void initializeFeatureLoop() {
    PAD_PRE_ROWS = std::max({BB_SIDE_MOUSE.height, spre_t.y, spre_b.y});
    PAD_POST_ROWS = spost_b.y > spost_t.y ? spost_b.y : spost_t.y;
    PAD_PRE_COLS = std::max({BB_BOTTOM_MOUSE.width, spre_t.x, spre_b.x});
    PAD_POST_COLS = spost_b.x > spost_t.x ? spost_b.x : spost_t.x;
    I_PAD = Mat8(PAD_PRE_ROWS + N_ROWS + PAD_POST_ROWS, PAD_PRE_COLS + N_COLS + PAD_POST_COLS, 0);
    I_PREV_PAD = Mat8(I_PAD.rows, I_PAD.cols, 0);
    I_UNPAD = Rect(PAD_PRE_COLS, PAD_PRE_ROWS, N_COLS, N_ROWS);
    BB_BOTTOM_MOUSE_PAD = Rect(0, 0, spre_b.x + BB_BOTTOM_MOUSE.width + spost_b.x, spre_b.y + BB_BOTTOM_MOUSE.height + spost_b.y);
    BB_SIDE_MOUSE_PAD = Rect(0, 0, spre_t.x + BB_SIDE_MOUSE.width + spost_t.x, spre_t.y + BB_SIDE_MOUSE.height + spost_t.y);
    BB_UNPAD_MOUSE_BOTTOM = Rect(spre_b.x, spre_b.y, BB_BOTTOM_MOUSE.width, BB_BOTTOM_MOUSE.height);
    BB_UNPAD_MOUSE_SIDE = Rect(spre_t.x, spre_t.y, BB_SIDE_MOUSE.width, BB_SIDE_MOUSE.height);
    tail_box_width = (unsigned)((int)(double)(BB_BOTTOM_MOUSE.width) * P.tail_sub_bounding_box);
    BB_BOTTOM_TAIL_PAD = Rect(0, 0, tail_box_width + spre_b.x + spost_b.x, BB_BOTTOM_MOUSE.height + spre_b.y + spost_b.y);
    BB_UNPAD_TAIL_BOTTOM = Rect(spre_b.x, spre_b.y, tail_box_width, BB_BOTTOM_MOUSE.height);
    BB_BOTTOM_TAIL = Rect(0, 0, tail_box_width, BB_BOTTOM_MOUSE.height);
    BB_SIDE_TAIL_PAD = Rect(0, 0, tail_box_width + spre_t.x + spost_t.x, BB_SIDE_MOUSE.height + spre_t.y + spost_t.y);
    BB_UNPAD_TAIL_SIDE = Rect(spre_t.x, spre_t.y, tail_box_width, BB_SIDE_MOUSE.height);
    const int sp = P.occlusion_grid_spacing_pixels_bottom;
    unsigned ngrid_y = ((BB_BOTTOM_MOUSE.height - sp) / sp) + 1;
    unsigned ngrid_x = (unsigned)(((P.occlusion_grid_max_width * BB_BOTTOM_MOUSE.width) - sp) / sp + 1);
    ONG_nx = (int)ngrid_x;
    ONG_ny = (int)ngrid_y;
    ONG_BR_x = (double)(BB_BOTTOM_MOUSE.width - 1 - sp / 2);
    ONG_BR_y = (double)(BB_BOTTOM_MOUSE.height - 1 - sp / 2);
    Nong = ngrid_x * ngrid_y;
    const int sps = P.occlusion_grid_spacing_pixels_side;
    Nong_side = (unsigned)(((BB_SIDE_MOUSE.height - sps) / sps) + 1);
    ONG_SIDE_LOWEST = (unsigned)(BB_SIDE_MOUSE.height - 1 - sps / 2);
    CURRENT_FRAME = -1;
  }

  void fill_geometry(lm_geometry& g) const {
    auto R = [](const Rect& r) { return lm_rect{r.x, r.y, r.width, r.height}; };
    std::memset(&g, 0, sizeof(g));
    g.n_rows = N_ROWS;
    g.n_cols = N_COLS;
    g.pad_pre_rows = PAD_PRE_ROWS;
    g.pad_pre_cols = PAD_PRE_COLS;
    g.pad_post_rows = PAD_POST_ROWS;
    g.pad_post_cols = PAD_POST_COLS;
    g.ipad_rows = I_PAD.rows;
    g.ipad_cols = I_PAD.cols;
    g.spre_b_w = spre_b.x;
    g.spre_b_h = spre_b.y;
    g.spost_b_w = spost_b.x;
    g.spost_b_h = spost_b.y;
    g.spre_t_w = spre_t.x;
    g.spre_t_h = spre_t.y;
    g.spost_t_w = spost_t.x;
    g.spost_t_h = spost_t.y;
    g.bb_bottom_mouse = R(BB_BOTTOM_MOUSE);
    g.bb_side_mouse = R(BB_SIDE_MOUSE);
    g.bb_bottom_mouse_pad = R(Rect(0, 0, BB_BOTTOM_MOUSE_PAD.width, BB_BOTTOM_MOUSE_PAD.height));
    g.bb_side_mouse_pad = R(Rect(0, 0, BB_SIDE_MOUSE_PAD.width, BB_SIDE_MOUSE_PAD.height));
    g.bb_unpad_mouse_bottom = R(BB_UNPAD_MOUSE_BOTTOM);
    g.bb_unpad_mouse_side = R(BB_UNPAD_MOUSE_SIDE);
    g.bb_bottom_tail_pad = R(BB_BOTTOM_TAIL_PAD);
    g.bb_unpad_tail_bottom = R(BB_UNPAD_TAIL_BOTTOM);
    g.bb_bottom_tail = R(BB_BOTTOM_TAIL);
    g.bb_side_tail_pad = R(BB_SIDE_TAIL_PAD);
    g.bb_unpad_tail_side = R(BB_UNPAD_TAIL_SIDE);
    g.tail_box_width = (int32_t)tail_box_width;
    g.ong_nx = ONG_nx;
    g.ong_ny = ONG_ny;
    g.ong_br_x = ONG_BR_x;
    g.ong_br_y = ONG_BR_y;
    g.n_ong_side = (int32_t)Nong_side;
    g.ong_side_lowest = (int32_t)ONG_SIDE_LOWEST;
    g.match_box_paw_bottom = R(paw.match_b);
    g.match_box_paw_side = R(paw.match_s);
    g.match_box_snout_bottom = R(snout.match_b);
    g.match_box_snout_side = R(snout.match_s);
  }

  // ---- per-frame methods, main.cpp:57-80

  // LocoMouse::readFrame(Mat&), :1273-1333 (+ LocoMouse_TM::readFrame, TM.cpp:243-249)
  void readFrame(const uint8_t* F_raw) {
    CURRENT_FRAME += 1;
    correct_frame(F_raw, BKG.data(), CAL.data(), VR, VC, N_ROWS, N_COLS, IMAGE_FLIP, METHOD == 1 || METHOD == 2,
                  I_PAD.row(I_UNPAD.y) + I_UNPAD.x, I_PAD.cols);
  }

  // The image work of readFrame(Mat& I) (:1302-1327): subtract, normalize,
  // correctImage, flip, written into rows of I at dst (row stride dst_stride).
  static void correct_frame(const uint8_t* F_raw, const uint8_t* BKG, const int32_t* CAL, int VR, int VC, int N_ROWS,
                            int N_COLS, bool flip, bool tm_adjust, uint8_t* dst0, int dst_stride) {
    const size_t NP = (size_t)VR * VC;
    std::vector<uint8_t> F(NP);
    for (size_t i = 0; i < NP; ++i) F[i] = F_raw[i] > BKG[i] ? (uint8_t)(F_raw[i] - BKG[i]) : 0;  // subtract (:1304)
    // normalize(F, F, 0, 255, NORM_MINMAX, CV_8UC1) (:1310)
    uint8_t mn = 255, mx = 0;
    for (size_t i = 0; i < NP; ++i) {
      mn = std::min(mn, F[i]);
      mx = std::max(mx, F[i]);
    }
    const double smin = mn, smax = mx, dmin = 0, dmax = 255;
    const double scale = (dmax - dmin) * (smax - smin > DBL_EPSILON ? 1. / (smax - smin) : 0);
    const double shift = dmin - smin * scale;
    uint8_t lut[256];
    const float sf = (float)scale, hf = (float)shift;
    for (int p = 0; p < 256; ++p) {
      float v = (float)p * sf;
      v = v + hf;
      long iv = std::lrint(v);  // cvRound
      lut[p] = (uint8_t)(iv < 0 ? 0 : iv > 255 ? 255 : iv);
    }
    if (std::fabs(scale - 1) < DBL_EPSILON && std::fabs(shift) < DBL_EPSILON)
      for (int p = 0; p < 256; ++p) lut[p] = (uint8_t)p;  // convertTo noScale copy
    // TM imadjust(I, I, 0, 0.6, 0, 1) (LocoMouse_class.cpp:3204-3242)
    uint8_t adj[256];
    for (int p = 0; p < 256; ++p) adj[p] = (uint8_t)p;
    if (tm_adjust) imadjust_lut(0, 0.6, 0, 1, adj);
    // correctImage (:1337-1406) + flip(I, I, 1) (:1323-1327)
    for (int r = 0; r < N_ROWS; ++r) {
      uint8_t* dst = dst0 + (size_t)r * dst_stride;
      for (int c = 0; c < N_COLS; ++c) {
        int cs = flip ? (N_COLS - 1 - c) : c;
        dst[c] = adj[lut[F[CAL[(size_t)r * N_COLS + cs]]]];
      }
    }
  }

  static void imadjust_lut(double low_in, double high_in, double low_out, double high_out, uint8_t* pL) {
    low_in = low_in * 255;
    high_in = high_in * 255;
    low_out = low_out * 255;
    high_out = high_out * 255;
    double range_in = high_in - low_in, range_out = high_out - low_out, range_div = range_out / range_in;
    for (int i = 0; i < 256; ++i) {
      double temp;
      if (i <= low_in) temp = 0;
      else if (i >= high_in) temp = range_out;
      else temp = (i - low_in) * (range_div);
      pL[i] = (uint8_t)std::round((temp + low_out));
    }
  }

  // LocoMouse::cropBoundingBox, :1408-1478
  void cropBoundingBox(unsigned bx, unsigned byb, unsigned bys) {
    BB_BOTTOM_MOUSE_PAD.x = (int)((bx + PAD_PRE_COLS) - (BB_BOTTOM_MOUSE_PAD.width - spost_b.x) + 1);
    BB_BOTTOM_MOUSE_PAD.y = (int)((byb + PAD_PRE_ROWS) - (BB_BOTTOM_MOUSE_PAD.height - spost_b.y) + 1);
    check_roi(BB_BOTTOM_MOUSE_PAD, I_PAD.rows, I_PAD.cols, "BB_BOTTOM_MOUSE_PAD");
    if (use_glt)  // LUT(I_BOTTOM_MOUSE, REF_CDF_GLT, I_BOTTOM_MOUSE), in place on I_PAD (:1445-1448)
      for (int r = 0; r < BB_BOTTOM_MOUSE.height; ++r) {
        uint8_t* row = I_PAD.row(BB_BOTTOM_MOUSE_PAD.y + BB_UNPAD_MOUSE_BOTTOM.y + r) + BB_BOTTOM_MOUSE_PAD.x + BB_UNPAD_MOUSE_BOTTOM.x;
        for (int c = 0; c < BB_BOTTOM_MOUSE.width; ++c) row[c] = GLT[row[c]];
      }
    BB_SIDE_MOUSE_PAD.x = (int)((PAD_PRE_COLS + bx) - (BB_SIDE_MOUSE_PAD.width - spost_t.x) + 1);
    BB_SIDE_MOUSE_PAD.y = (int)((PAD_PRE_ROWS + bys) - (BB_SIDE_MOUSE_PAD.height - spost_t.y) + 1);
    check_roi(BB_SIDE_MOUSE_PAD, I_PAD.rows, I_PAD.cols, "BB_SIDE_MOUSE_PAD");
  }

  uint8_t bottom_px(int r, int c) const {  // I_BOTTOM_MOUSE(r, c)
    return I_PAD.at(BB_BOTTOM_MOUSE_PAD.y + BB_UNPAD_MOUSE_BOTTOM.y + r, BB_BOTTOM_MOUSE_PAD.x + BB_UNPAD_MOUSE_BOTTOM.x + c);
  }
  uint8_t side_px(int r, int c) const {
    return I_PAD.at(BB_SIDE_MOUSE_PAD.y + BB_UNPAD_MOUSE_SIDE.y + r, BB_SIDE_MOUSE_PAD.x + BB_UNPAD_MOUSE_SIDE.x + c);
  }

  bool fused() const { return !(flags_ & LMO_UNFUSED_FILTER) && FILTER_ARITH != LM_FILTER_UNFUSED; }

  // detectTail :2541-2555 -> detectLineCandidates :2558-2742
  void detectTail() {
    Rect tail_b_roi = shift(BB_BOTTOM_TAIL_PAD, BB_BOTTOM_MOUSE_PAD.x, BB_BOTTOM_MOUSE_PAD.y);
    Rect tail_s_roi = shift(BB_SIDE_TAIL_PAD, BB_SIDE_MOUSE_PAD.x, BB_SIDE_MOUSE_PAD.y);
    Matf ftb, fts;
    filter2D_roi(I_PAD, tail_b_roi, tail.wb, tail.rows_b, tail.cols_b, -tail.rho_b, BB_UNPAD_TAIL_BOTTOM, ftb, fused());
    filter2D_roi(I_PAD, tail_s_roi, tail.ws, tail.rows_s, tail.cols_s, -tail.rho_s, BB_UNPAD_TAIL_SIDE, fts, fused());
    if (flags_ & LMO_KEEP_DEBUG) {
      dbg_scores[2] = ftb;
      dbg_scores[5] = fts;
    }
    // threshold(>0 -> 1) + convertTo(CV_8UC1) (:2593-2598)
    Mat8 bin_b(ftb.rows, ftb.cols, 0);
    for (size_t i = 0; i < ftb.d.size(); ++i) bin_b.d[i] = ftb.d[i] > 0 ? 1 : 0;
    std::vector<int32_t> tracks(3 * 15, -1);  // -Mat::ones(3, N_line_points) (:2601)
    Mat8 sel_b = selectLargestRegion(bin_b, P.conn_comp_connectivity);
    TAIL_MASK = sel_b;  // (:2611)
    // reduce(MAX, dim 0) (:2615)
    std::vector<uint8_t> colmax(sel_b.cols, 0);
    for (int r = 0; r < sel_b.rows; ++r)
      for (int c = 0; c < sel_b.cols; ++c) colmax[c] = std::max(colmax[c], sel_b.at(r, c));
    // (Filtered_tail_side > 0) & repeat(colmax) (:2623-2624)
    Mat8 bin_s(fts.rows, fts.cols, 0);
    for (int r = 0; r < fts.rows; ++r)
      for (int c = 0; c < fts.cols; ++c) bin_s.at(r, c) = (fts.at(r, c) > 0 ? 255 : 0) & colmax[c];
    Mat8 sel_s = selectLargestRegion(bin_s, P.conn_comp_connectivity);
    int first = -1, last = -1;
    for (int i = 0; i < (int)colmax.size(); ++i)
      if (colmax[i] > 0) {
        first = i;
        break;
      }
    if (first >= 0) {
      last = first;
      for (int i = (int)colmax.size() - 1; i > first; i--)
        if (colmax[i] > 0) {
          last = i;
          break;
        }
      const int N_line_points = 15;
      int tail_width = last - first;
      int remainder = tail_width % N_line_points;
      int regular_length = (tail_width - remainder) / N_line_points;
      std::vector<int> segw(N_line_points, regular_length);
      for (int i = 0; i < remainder; i++) segw[i] = regular_length + 1;
      int sx = first;
      for (int i = 0; i < N_line_points; i++) {  // moments(segment, true) (:2702-2725)
        Moments3 M = moments_binary(sel_b, Rect(sx, 0, segw[i], sel_b.rows));
        if (M.m00 > 0) {
          tracks[i] = (int)(M.m10 / M.m00) + sx;
          tracks[15 + i] = (int)(M.m01 / M.m00) + 0;
        }
        sx += segw[i];
      }
      for (int i = 0; i < N_line_points; i++) {  // :2728-2737
        if (tracks[i] > 0) {
          Moments3 M = moments_binary(sel_s, Rect(tracks[i], 0, 1, sel_s.rows));
          if (M.m00 > 0) tracks[30 + i] = (int)(M.m01 / M.m00) + 0;
        }
      }
    }
    res.tail.insert(res.tail.end(), tracks.begin(), tracks.end());
  }

  // detectBottomCandidates :771-807 with detectPointCandidatesBottom :841-854
  void detectBottomCandidates() {
    const int H = BB_BOTTOM_MOUSE.height, W = BB_BOTTOM_MOUSE.width;
    Mat8 mask(H, W, 0);
    for (int r = 0; r < H; ++r)
      for (int c = 0; c < W; ++c) mask.at(r, c) = bottom_px(r, c) > 25 ? 0 : 255;  // threshold(25.5 -> 25, BINARY_INV)
    for (int r = 0; r < BB_BOTTOM_TAIL.height; ++r)
      for (int c = 0; c < BB_BOTTOM_TAIL.width; ++c)
        if (TAIL_MASK.at(r, c)) mask.at(r, c) = 255;
    cand_bottom_paw.push_back(detectPointBottom(paw, mask, 0));
    cand_bottom_snout.push_back(detectPointBottom(snout, mask, 1));
  }

  std::vector<Candidate> detectPointBottom(const Feature& F, const Mat8& mask, int det) {
    Matf s;
    filter2D_roi(I_PAD, BB_BOTTOM_MOUSE_PAD, F.wb, F.rows_b, F.cols_b, -F.rho_b, BB_UNPAD_MOUSE_BOTTOM, s, fused());
    if (flags_ & LMO_KEEP_DEBUG) dbg_scores[det] = s;
    for (size_t i = 0; i < s.d.size(); ++i)
      if (mask.d[i]) s.d[i] = 0;
    return nmsMax(s, F.cols_b, F.rows_b, 0.5);
  }

  // detectSideCandidates :809-838 with detectPointCandidatesSide :856-870
  void detectSideCandidates() {
    const int H = BB_SIDE_MOUSE.height, W = BB_SIDE_MOUSE.width;
    Mat8 mask(H, W, 0);
    for (int r = 0; r < H; ++r)
      for (int c = 0; c < W; ++c) mask.at(r, c) = side_px(r, c) > 25 ? 0 : 255;
    cand_side_paw.push_back(cand_bottom_paw.back().size() > 0 ? detectPointSide(paw, mask, 3) : std::vector<Candidate>());
    cand_side_snout.push_back(cand_bottom_snout.back().size() > 0 ? detectPointSide(snout, mask, 4) : std::vector<Candidate>());
  }

  std::vector<Candidate> detectPointSide(const Feature& F, const Mat8& mask, int det) {
    Matf s;
    filter2D_roi(I_PAD, BB_SIDE_MOUSE_PAD, F.ws, F.rows_s, F.cols_s, -F.rho_s, BB_UNPAD_MOUSE_SIDE, s, fused());
    if (flags_ & LMO_KEEP_DEBUG) dbg_scores[det] = s;
    for (size_t i = 0; i < s.d.size(); ++i)
      if (mask.d[i]) s.d[i] = 0;
    return peakClustering(s, F.cols_s, F.rows_s, 0.5);
  }

  // unaryCostBox :1909-1952 via computeUnaryCostsBottom :873-894
  MyMat unaryCostBox(const std::vector<Candidate>& pc, const std::vector<LocationPrior>& lp) const {
    const int N = (int)pc.size(), NF = (int)lp.size();
    MyMat M(N, NF);
    const double norm_fact = 1 / std::sqrt(2);
    for (int i = 0; i < N; ++i) {
      const double cx = (double)pc[i].x / (double)BB_BOTTOM_MOUSE.width;
      const double cy = (double)pc[i].y / (double)BB_BOTTOM_MOUSE.height;
      for (int j = 0; j < NF; ++j) {
        if (lp[j].contains(cx, cy)) {
          const double dx = cx - lp[j].px, dy = cy - lp[j].py;
          const double val = std::sqrt(dx * dx + dy * dy) * norm_fact;
          if (val <= lp[j].max_distance) M.put(i, j, (1 - val) * pc[i].s);
        }
      }
    }
    return M;
  }

  void computeUnaryCostsBottom() {
    MyMat a = unaryCostBox(cand_bottom_paw.back(), prior_paw);
    MyMat b = unaryCostBox(cand_bottom_snout.back(), prior_snout);
    res.unary.insert(res.unary.end(), a.v.begin(), a.v.end());
    res.unary_offset.push_back((int64_t)res.unary.size());
    res.unary.insert(res.unary.end(), b.v.begin(), b.v.end());
    res.unary_offset.push_back((int64_t)res.unary.size());
  }

  // pairwisePotential :1954-2070
  MatSparse pairwisePotential(const std::vector<Candidate>& Ci, const std::vector<Candidate>& Cip1) const {
    const int Ni = (int)Ci.size(), Nip1 = (int)Cip1.size();
    const double grid_spacing = (double)P.occlusion_grid_spacing_pixels_bottom;
    const double max_disp = (double)P.max_displacement_bottom, alpha = P.alpha_vel_bottom;
    const double occ = P.pairwise_occluded_cost * alpha;
    const int nxa = ONG_nx - 1, nya = ONG_ny - 1;
    auto clampi = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };  // matchToRange
    MyMat D(Nip1 + (int)Nong, Ni + (int)Nong);
    for (int i = 0; i < Ni; ++i) {
      int32_t xc = (int32_t)std::round((ONG_BR_x - (double)Ci[i].x) / grid_spacing);
      int32_t yc = (int32_t)std::round((ONG_BR_y - (double)Ci[i].y) / grid_spacing);
      int ox = clampi(xc, 0, nxa), oy = clampi(yc, 0, nya);
      D.put(Nip1 + (oy * ONG_nx + ox), i, occ);
      for (int j = 0; j < Nip1; ++j) {
        if (i == 0) {
          int32_t x2 = (int32_t)std::round((ONG_BR_x - (double)Cip1[j].x) / grid_spacing);
          int32_t y2 = (int32_t)std::round((ONG_BR_y - (double)Cip1[j].y) / grid_spacing);
          int ox2 = clampi(x2, 0, nxa), oy2 = clampi(y2, 0, nya);
          D.put(j, Ni + (oy2 * ONG_nx + ox2), occ);
        }
        const double dx = ((double)Cip1[j].x - (double)Ci[i].x);
        const double dy = ((double)Cip1[j].y - (double)Ci[i].y);
        const double dist = std::sqrt(dx * dx + dy * dy);
        if (dist < max_disp) {
          double inv_dist = 1 - (dist / max_disp);
          inv_dist = inv_dist * alpha;
          D.put(j, i, inv_dist);
        }
      }
    }
    for (int i = 0; i < (int)Nong; ++i) D.put(Nip1 + i, Ni + i, occ);
    return MatSparse(D);
  }

  void push_sparse(const MatSparse* S) {
    if (!S) {
      res.pw_dims.insert(res.pw_dims.end(), {-1, -1, 0});
    } else {
      res.pw_dims.insert(res.pw_dims.end(), {S->n_rows, S->n_cols, (int32_t)S->ir.size()});
      res.pw_jc.insert(res.pw_jc.end(), S->jc.begin(), S->jc.end());
      res.pw_ir.insert(res.pw_ir.end(), S->ir.begin(), S->ir.end());
      res.pw_pr.insert(res.pw_pr.end(), S->pr.begin(), S->pr.end());
    }
    res.pw_jc_offset.push_back((int64_t)res.pw_jc.size());
    res.pw_nz_offset.push_back((int64_t)res.pw_ir.size());
  }

  // computePairwiseCostsBottom :896-919
  void computePairwiseCostsBottom() {
    if (CURRENT_FRAME > 0) {
      MatSparse a = pairwisePotential(cand_bottom_paw.end()[-2], cand_bottom_paw.end()[-1]);
      MatSparse b = pairwisePotential(cand_bottom_snout.end()[-2], cand_bottom_snout.end()[-1]);
      push_sparse(&a);
      push_sparse(&b);
    } else {
      push_sparse(nullptr);
      push_sparse(nullptr);
    }
  }

  // checkVelCriterion :1256-1267 (box in padded-crop coordinates)
  bool checkVelCriterion(const Rect& crop, const Rect& im_box, int box_area, double alpha, double T) const {
    Rect abs = shift(im_box, crop.x, crop.y);
    check_roi(im_box, crop.height, crop.width, "checkVelCriterion box");
    long sum = 0;
    const int t = (int)std::floor(T);  // threshold on 8U floors the threshold
    for (int r = 0; r < abs.height; ++r)
      for (int c = 0; c < abs.width; ++c) {
        int a = I_PAD.at(abs.y + r, abs.x + c), b = I_PREV_PAD.at(abs.y + r, abs.x + c);
        int s = a > b ? a - b : 0;
        if (s > t) sum += 1;
      }
    return (double)sum >= ((double)box_area) * alpha;
  }

  // matchingWithVelocityConstraint :1023-1073 + xDist :1075-1107 + matchViews :1109-1254
  std::vector<P22D> matching(const std::vector<Candidate>& Cb, const std::vector<Candidate>& Ct, bool vel_check,
                             const Feature& F, double T) const {
    const int ovlp = (int)(F.cols_b * (1 - T));
    const int Nb = (int)Cb.size(), Ns = (int)Ct.size();
    std::vector<P22D> C;
    if (Nb == 0) return C;
    std::vector<uint8_t> boolD;
    std::vector<double> W;
    std::vector<float> bottom_per_side(Ns, 0.f), top_per_bottom(Nb, 0.f);
    if (Ns > 0) {
      std::vector<int> D((size_t)Nb * Ns);
      for (int i = 0; i < Nb; ++i)
        for (int j = 0; j < Ns; ++j) D[(size_t)i * Ns + j] = std::abs(Cb[i].x - Ct[j].x);
      boolD.resize(D.size());
      for (size_t k = 0; k < D.size(); ++k) boolD[k] = D[k] <= ovlp ? 255 : 0;
      // normalize(boolD, boolD, 0, 1, NORM_MINMAX): 255 -> 1; all-equal -> all 0
      uint8_t mn = *std::min_element(boolD.begin(), boolD.end()), mx = *std::max_element(boolD.begin(), boolD.end());
      for (auto& b : boolD) b = (mx - mn > 0 && b == 255) ? 1 : 0;
      // 1 - D / ovlp  ==  convertTo(alpha = -(1./ovlp), beta = 1)
      const double alpha = -(1. / (double)ovlp);
      W.resize(D.size());
      for (size_t k = 0; k < D.size(); ++k) {
        double v = (double)D[k] * alpha;
        W[k] = v + 1.0;
      }
      for (int i = 0; i < Nb; ++i)
        for (int j = 0; j < Ns; ++j) {
          bottom_per_side[j] += (float)boolD[(size_t)i * Ns + j];
          top_per_bottom[i] += (float)boolD[(size_t)i * Ns + j];
        }
    }
    const double moving_alpha_bottom = 0.02, moving_alpha_side = 0.05, moving_threshold = 25;
    std::vector<bool> need_to_check(Ns, true), moving_t(Ns, false);
    const Candidate none(-1, -1, -1);
    for (int ib = 0; ib < Nb; ib++) {
      if (Ns == 0 || top_per_bottom[ib] == 0) {
        C.push_back(P22D(Cb[ib], none));
        continue;
      }
      bool is_first = true, moving_b = false, need_b = true, match = true;
      for (int is = 0; is < Ns; is++) {
        if (boolD[(size_t)ib * Ns + is] < 1) continue;
        if ((bottom_per_side[is] > 1) & vel_check) {
          if (need_b) {
            Rect box(F.match_b.x + Cb[ib].x + spre_b.x, F.match_b.y + Cb[ib].y + spre_b.y, F.match_b.width, F.match_b.height);
            moving_b = checkVelCriterion(BB_BOTTOM_MOUSE_PAD, box, F.cols_b * F.rows_b, moving_alpha_bottom, moving_threshold);
            need_b = false;
          }
          if (need_to_check[is]) {
            Rect box(F.match_s.x + Ct[is].x + spre_t.x, F.match_s.y + Ct[is].y + spre_t.y, F.match_s.width, F.match_s.height);
            moving_t[is] = checkVelCriterion(BB_SIDE_MOUSE_PAD, box, F.cols_s * F.rows_s, moving_alpha_side, moving_threshold);
            need_to_check[is] = false;
          }
          match = moving_b == moving_t[is];
        } else {
          match = true;
        }
        if (match) {
          Candidate ct(Ct[is].x, Ct[is].y, Ct[is].s * W[(size_t)ib * Ns + is]);
          if (is_first) {
            C.push_back(P22D(Cb[ib], ct));
            is_first = false;
          } else {
            C.back().add_side_candidate(ct);
          }
        }
      }
      if (is_first) C.push_back(P22D(Cb[ib], none));
    }
    return C;
  }

  // matchBottomSideCandidates :999-1021
  void matchBottomSideCandidates() {
    for (int k = 0; k < 2; ++k) {
      const std::vector<Candidate>& b = k == 0 ? cand_bottom_paw.back() : cand_bottom_snout.back();
      const std::vector<Candidate>& s = k == 0 ? cand_side_paw.back() : cand_side_snout.back();
      std::vector<P22D> Pm = matching(b, s, CURRENT_FRAME > 0, k == 0 ? paw : snout, P.side_bottom_min_overlap);
      for (const P22D& p : Pm) {
        lm_p22d o;
        o.bottom = lm_candidate{p.CB.x, p.CB.y, p.CB.s};
        o.side_offset = (int32_t)res.side_y.size();
        o.side_count = (int32_t)p.yt.size();
        res.side_y.insert(res.side_y.end(), p.yt.begin(), p.yt.end());
        res.side_s.insert(res.side_s.end(), p.st.begin(), p.st.end());
        res.p22d.push_back(o);
      }
      res.p22d_offset.push_back((int64_t)res.p22d.size());
    }
  }

  void storePreviousImage() { I_PREV_PAD = I_PAD; }  // :1508-1513

  void run_frame(const uint8_t* F, unsigned bx, unsigned byb, unsigned bys) {
    readFrame(F);
    cropBoundingBox(bx, byb, bys);
    if (flags_ & LMO_KEEP_DEBUG) dbg_scores.assign(6, Matf());
    detectTail();
    detectBottomCandidates();
    computeUnaryCostsBottom();
    computePairwiseCostsBottom();
    detectSideCandidates();
    matchBottomSideCandidates();
    storePreviousImage();
    for (auto* L : {&cand_bottom_paw, &cand_bottom_snout, &cand_side_paw, &cand_side_snout}) {
      for (const Candidate& c : L->back()) res.cand.push_back(lm_candidate{c.x, c.y, c.s});
      res.cand_offset.push_back((int64_t)res.cand.size());
    }
    if (flags_ & LMO_KEEP_DEBUG) {
      res.scores.push_back(dbg_scores);
      res.tail_mask.push_back(TAIL_MASK);
      res.ipad.push_back(I_PAD);
    }
  }

  unsigned bb_x() const { return BB_X; }
  unsigned bb_yb() const { return BB_YB; }
  unsigned bb_ys() const { return BB_YS; }

  Result res;

 private:
  int flags_;
  lm_params P;
  std::vector<LocationPrior> prior_paw, prior_snout;
  int VR = 0, VC = 0, N_ROWS = 0, N_COLS = 0, METHOD = 0, FILTER_ARITH = 0;
  bool IMAGE_FLIP = false;
  bool use_glt = false;  // transform_gray_values with a CV_8U table
  uint8_t GLT[256] = {0};
  std::vector<uint8_t> BKG;
  std::vector<int32_t> CAL;
  Feature paw, snout, tail;
  Point spre_b, spre_t, spost_b, spost_t;  // (width, height)
  unsigned BB_X = 0, BB_YS = 0, BB_YB = 0;
  Rect BB_BOTTOM_MOUSE, BB_SIDE_MOUSE, BB_BOTTOM_MOUSE_PAD, BB_SIDE_MOUSE_PAD, BB_UNPAD_MOUSE_BOTTOM, BB_UNPAD_MOUSE_SIDE;
  Rect BB_BOTTOM_TAIL_PAD, BB_UNPAD_TAIL_BOTTOM, BB_BOTTOM_TAIL, BB_SIDE_TAIL_PAD, BB_UNPAD_TAIL_SIDE, I_UNPAD;
  int PAD_PRE_ROWS = 0, PAD_PRE_COLS = 0, PAD_POST_ROWS = 0, PAD_POST_COLS = 0;
  unsigned tail_box_width = 0, Nong = 0, Nong_side = 0, ONG_SIDE_LOWEST = 0;
  int ONG_nx = 0, ONG_ny = 0;
  double ONG_BR_x = 0, ONG_BR_y = 0;
  int CURRENT_FRAME = -1;
  Mat8 I_PAD, I_PREV_PAD, TAIL_MASK;
  std::vector<std::vector<Candidate>> cand_bottom_paw, cand_bottom_snout, cand_side_paw, cand_side_snout;
  std::vector<Matf> dbg_scores;
};

// ------------------------------------------------ whole-video BB pass (method 0)
// LocoMouse::computeBoundingBox (LocoMouse_class.cpp:579-653).

// medianBlur(src, dst, ksize), CV_8UC1 (imgproc median_blur.cpp): the exact
// median (rank n/2 of the n = ksize^2 window values) with BORDER_REPLICATE;
// src is the whole matrix (no ROI parent).  Huang's running histogram per row.
static Mat8 medianBlur8u(const Mat8& src, int ksize) {
  if (ksize == 1) return src;
  const int p = ksize / 2, R = src.rows, C = src.cols, half = ksize * ksize / 2;
  auto cl = [](int v, int n) { return v < 0 ? 0 : (v >= n ? n - 1 : v); };
  Mat8 out(R, C, 0);
  for (int r = 0; r < R; ++r) {
    int hist[256] = {0};
    for (int dr = -p; dr <= p; ++dr)
      for (int dc = -p; dc <= p; ++dc) hist[src.at(cl(r + dr, R), cl(dc, C))]++;
    for (int c = 0; c < C; ++c) {
      if (c > 0)
        for (int dr = -p; dr <= p; ++dr) {
          hist[src.at(cl(r + dr, R), cl(c - 1 - p, C))]--;
          hist[src.at(cl(r + dr, R), cl(c + p, C))]++;
        }
      int s = 0, v = 0;
      while ((s += hist[v]) <= half) ++v;
      out.at(r, c) = (uint8_t)v;
    }
  }
  return out;
}

// firstLastOverT<int> (LocoMouse_class.hpp:411-440).  The sums are CV_32S but
// are read through values.ptr<float>(0) (:419): as executed, each int32 sum's
// bit pattern is compared as a float with (float)th.  integer = 1 compares the
// int32 values instead.  Note first_last[1] stays 0 when exactly one entry
// passes (the index bookkeeping of :424-433).
static void firstLastOverT(const int32_t* v, unsigned L, int first_last[2], int th, bool integer) {
  bool has_first = false;
  first_last[0] = 0;
  first_last[1] = 0;
  int index = 0;
  for (unsigned i = 0; i < L; ++i) {
    bool pass;
    if (integer) {
      pass = v[i] >= th;
    } else {
      float f;
      std::memcpy(&f, &v[i], 4);
      pass = f >= (float)th;
    }
    if (pass) {
      first_last[index] = (int)i;
      if (!has_first) {
        index = 1;
        has_first = true;
      }
    }
  }
  if (!has_first) {
    first_last[0] = -1;
    first_last[1] = -1;
  }
}

// (uint32_t)double as the reference's x86-64 build evaluates it (cvttsd2si to
// 64 bits, low 32 bits kept): negative values wrap (e.g. -1.0 -> 4294967295).
static uint32_t x86_u32(double d) {
  if (!(d > -9.2e18 && d < 9.2e18)) return 0;
  return (uint32_t)(uint64_t)(int64_t)d;
}

// medianvec (:1516-1533): sorts v in place; odd N returns v[N/2 - 1].
static double medianvec(std::vector<double>& v, int N) {
  if (N == 1) return v[0];
  std::sort(v.begin(), v.end());
  int half = N / 2;
  if (N % 2 == 0) return (v[half - 1] + v[half]) / 2;
  return v[half - 1];
}

// stdvec (:1535-1556): sample standard deviation, summed in vector order.
static double stdvec(const std::vector<double>& v, int N) {
  if (N == 1) return 0.0;
  double sum = 0.0;
  for (int i = 0; i < N; ++i) sum += v[i];
  double mean = sum / N;
  double sq = 0.0;
  for (int i = 0; i < N; ++i) {
    double d = v[i] - mean;
    sq = sq + d * d;
  }
  return std::sqrt(sq / (N - 1));
}

// vecmovingaverage (:1558-1608).
static void vecmovingaverage(const std::vector<double>& v, std::vector<uint32_t>& vout, int N_window) {
  const size_t n = v.size();
  vout.assign(n, 0);
  if ((size_t)N_window >= n) {
    for (size_t i = 0; i < n; ++i) vout[i] = x86_u32(v[i]);
    return;
  }
  double cur = 0;
  int h = N_window / 2;
  for (int i = 0; i < h; ++i) vout[i] = x86_u32(v[i]);
  for (int i = 0; i < N_window; ++i) cur += v[i];
  vout[h] = x86_u32(std::floor(cur / N_window));
  for (size_t i = 0; i < n - N_window; ++i) {
    cur = cur - v[i] + v[i + N_window];
    vout[h + 1 + i] = x86_u32(std::floor(cur / N_window));
  }
  for (size_t i = n - h - 1; i < n; ++i) vout[i] = x86_u32(v[i]);
}

class BBOracle {
 public:
  BBOracle(const lm_setup& su, const lm_bb_params& bp) : P(bp) {
    METHOD = su.method;
    if (METHOD < 0 || METHOD > 2) throw std::invalid_argument("BB pass: method must be 0, 1 or 2.");
    if (METHOD == 1 && P.firstlast_semantics != LM_BB_FIRSTLAST_AS_EXECUTED)
      throw std::invalid_argument("BB pass, method 1: only the as-executed firstLastOverT is restated.");
    if (P.median_filter_size % 2 == 0 || P.median_filter_size < 1 || P.median_filter_size > 63)
      throw std::invalid_argument("Invalid configuration parameter: median_filter_size must be odd.");
    if (P.min_pixel_visible < 0)
      throw std::invalid_argument("Invalid configuration parameter: min_pixel_visible must be non-negative.");
    if (P.moving_average_window % 2 == 0 || P.moving_average_window < 1)
      throw std::invalid_argument("Invalid configuration parameter: moving_average_window must be odd.");
    if (P.conn_comp_connectivity != 4 && P.conn_comp_connectivity != 8)
      throw std::invalid_argument("Invalid configuration parameter: conn_comp_connectivity must be either 4 or 8.");
    VR = su.video_rows;
    VC = su.video_cols;
    N_ROWS = su.calib_rows;
    N_COLS = su.calib_cols;
    BKG.assign(su.background, su.background + (size_t)VR * VC);
    CAL.assign(su.ind_warp_mapping, su.ind_warp_mapping + (size_t)N_ROWS * N_COLS);
    flip = su.flip != 0;
    side = Rect(su.view_box_side.x, su.view_box_side.y, su.view_box_side.width, su.view_box_side.height);
    bottom = Rect(su.view_box_bottom.x, su.view_box_bottom.y, su.view_box_bottom.width, su.view_box_bottom.height);
    // :585-591
    pad = P.median_filter_size / 2;
    I_median = Mat8(N_ROWS + 2 * pad, N_COLS + 2 * pad, 0);
    if (METHOD == 1) {  // computeMouseBox_DD's colRange / rowRange bounds (TM.cpp:205-208)
      if (P.zero_col_pre > side.width || P.zero_col_post > N_COLS || N_COLS > side.width ||
          P.zero_row_pre > side.height || P.zero_row_post > side.height)
        throw std::runtime_error("BB pass, method 1: zero_* ranges exceed the side view (cv::Mat::colRange/rowRange assert).");
    }
    if (METHOD == 2) {  // computeMouseBox_DE's hard-coded ranges (TM_DE.cpp:69-72)
      if (46 > side.width || 760 > N_COLS || N_COLS > side.width || 100 > side.height || 149 > side.height)
        throw std::runtime_error("BB pass, method 2: the hard-coded zero ranges exceed the side view (cv::Mat::colRange/rowRange assert).");
    }
  }

  // imadjust_default (LocoMouse_class.cpp:3244-3311) as a LUT over the image's
  // histogram: the 1% / 99% cumulative bins (float arithmetic), then the
  // MatExpr (I - r0) / (r1 - r0) that OpenCV evaluates as
  // convertTo(alpha = 1/(r1-r0), beta = -r0/(r1-r0)) with float scale/shift.
  static void imadjust_default_lut(const std::vector<uint32_t>& hist, uint8_t lut[256]) {
    float sum_histf = 0;
    {
      double s = 0;
      for (int i = 0; i < 256; ++i) s += (float)hist[i];
      sum_histf = (float)s;
    }
    const float min_tol = 0.01f, max_tol = 0.99f;
    float cumsum_step = 0;
    int idx0 = 0, idx1 = 0, imin = 0, imax = 0;
    bool check_min = true, check_max = true;
    for (int i = 0; i < 256; ++i) {
      cumsum_step += (float)hist[i];
      const float cn = cumsum_step / sum_histf;
      if ((cn > min_tol) & check_min) {
        idx0 = i;
        check_min = false;
        imin = i;
      }
      if ((cn >= max_tol) & check_max) {
        idx1 = i;
        check_max = false;
        imax = i;
      }
      if (!(check_min || check_max)) break;
    }
    if (imin == imax) idx1 = 256;
    const float r0 = (float)idx0 / (float)255, r1 = (float)idx1 / (float)255;
    const double d = (double)(r1 - r0);
    const double alpha = 1.0 * (1. / d), beta = -(double)r0 * (1. / d);
    const bool noscale = std::fabs(alpha - 1) < DBL_EPSILON && std::fabs(beta) < DBL_EPSILON;
    const float sf = (float)alpha, hf = (float)beta;
    for (int p = 0; p < 256; ++p) {
      if (noscale) {
        lut[p] = (uint8_t)p;
        continue;
      }
      float v = (float)p * sf;
      v = v + hf;
      long iv = std::lrint(v);
      lut[p] = (uint8_t)(iv < 0 ? 0 : iv > 255 ? 255 : iv);
    }
  }

  // LocoMouse_TM_DE::computeMouseBox_DE (TM_DE.cpp:56-113) on the frame's
  // corrected image (base readFrame, :31).
  double frame_de(const uint8_t* F) {
    Mat8 I(N_ROWS, N_COLS, 0);
    LocoMouseOracle::correct_frame(F, BKG.data(), CAL.data(), VR, VC, N_ROWS, N_COLS, flip, false, I.row(0), N_COLS);
    std::vector<uint32_t> hist(256, 0);  // calcHist over I_SIDE
    for (int r = 0; r < side.height; ++r)
      for (int c = 0; c < side.width; ++c) hist[I.at(side.y + r, side.x + c)]++;
    uint8_t lut[256];
    imadjust_default_lut(hist, lut);
    std::vector<float> colsum(side.width, 0.f);
    for (int r = 0; r < side.height; ++r)
      for (int c = 0; c < side.width; ++c) {
        uint8_t v = lut[I.at(side.y + r, side.x + c)];
        if (c < 46 || c >= 760 || r < 100 || r >= 149) v = 0;  // colRange/rowRange(...).setTo(0)
        colsum[c] += v > 12 ? 1.f : 0.f;  // threshold(12.75) -> 1; reduce CV_32FC1
      }
    int fl[2];
    bool has_first = false;  // firstLastOverT<int> on float sums, th = MIN_PIXEL_COUNT = 10
    fl[0] = fl[1] = 0;
    int index = 0;
    for (int i = 0; i < N_COLS; ++i)
      if (colsum[i] >= (float)10) {
        fl[index] = i;
        if (!has_first) {
          index = 1;
          has_first = true;
        }
      }
    if (!has_first) fl[0] = fl[1] = -1;
    return std::min((double)(side.width - 1), (double)fl[1] * 1.1);  // WIDTH_MARGIN (TM_DE.hpp:28)
  }

  // LocoMouse_TM::computeMouseBox_DD (TM.cpp:192-241): imadjust_default, zero
  // bands, threshold, bwAreaOpen, disk filter2D, imfill, then reduce to CV_32S
  // and firstLastOverT.  The CV_32S column sums are integers in
  // [0, 255 * rows] < 2^23, so read as floats (ptr<float>, :419) they are +0
  // or denormal: each passes (>= (float)min_pixel_visible) iff
  // min_pixel_visible <= 0, whatever the image.  The restatement therefore
  // evaluates firstLastOverT on an all-zero sum vector (tests/test_bbox_oracle.py
  // checks the premise on random sums).
  double frame_dd() {
    std::vector<int32_t> zero(N_COLS, 0);
    int fl[2];
    firstLastOverT(zero.data(), (unsigned)N_COLS, fl, P.min_pixel_visible, false);
    return (double)fl[1];
  }

  // One iteration of the frame loop :614-626 (method 0), TM.cpp:137-142
  // (method 1), TM_DE.cpp:33-38 (method 2).
  void frame(const uint8_t* F) {
    if (METHOD != 0) {
      lm_bb_frame o{};
      o.x = METHOD == 1 ? frame_dd() : frame_de(F);
      o.y_bottom = (double)(N_ROWS - 1);
      o.y_side = METHOD == 1 ? 164.0 : (double)(side.height - 1);  // 165 - 1 (TM.cpp:141)
      frames.push_back(o);
      return;
    }
    // readFrame(I_center): writes the central ROI of I_median only.
    LocoMouseOracle::correct_frame(F, BKG.data(), CAL.data(), VR, VC, N_ROWS, N_COLS, flip, false,
                                   I_median.row(pad) + pad, I_median.cols);
    // computeMouseBox :948-997
    I_median = medianBlur8u(I_median, P.median_filter_size);  // in place (:952), border ring kept
    Mat8 I(N_ROWS, N_COLS, 0);
    for (int r = 0; r < N_ROWS; ++r)
      for (int c = 0; c < N_COLS; ++c) {
        uint8_t& v = I_median.at(pad + r, pad + c);
        v = v > 2.55 ? 1 : 0;  // threshold(I, I, 2.55, 1, THRESH_BINARY) (:955)
        I.at(r, c) = v;
      }
    binary.push_back(I);
    int lrs[2], lcs[2], lrb[2], lcb[2];
    view_lims(I, side, lrs, lcs);
    view_lims(I, bottom, lrb, lcb);
    lm_bb_frame o;
    o.x = (lrb[1] > lrs[1]) ? (double)lrb[1] : (double)lrs[1];  // :983
    o.y_bottom = (double)lcb[1];
    o.y_side = (double)lcs[1];
    unsigned wt = (unsigned)(lrs[1] - lrs[0]), wb = (unsigned)(lrb[1] - lrb[0]);  // :988-991
    o.width = wt > wb ? (double)wt : (double)wb;
    o.height_bottom = (double)(lcb[1] - lcb[0]);
    o.height_side = (double)(lcs[1] - lcs[0]);
    o.y_bottom += bottom.y;  // :636
    frames.push_back(o);
  }

  // largestBWAreaObject (:921-946) on the view, then reduce + firstLastOverT
  // (:961-978).  The view's pixels of I_median become the 0/255 mask.
  void view_lims(const Mat8& I, const Rect& v, int lr[2], int lc[2]) {
    Mat8 bin(v.height, v.width, 0);
    for (int r = 0; r < v.height; ++r)
      for (int c = 0; c < v.width; ++c) bin.at(r, c) = I.at(v.y + r, v.x + c);
    Mat8 m = selectLargestRegion(bin, P.conn_comp_connectivity);
    std::vector<int32_t> rowsum(v.width, 0), colsum(v.height, 0);
    for (int r = 0; r < v.height; ++r)
      for (int c = 0; c < v.width; ++c) {
        rowsum[c] += m.at(r, c);
        colsum[r] += m.at(r, c);
        I_median.at(pad + v.y + r, pad + v.x + c) = m.at(r, c);
      }
    const bool integer = P.firstlast_semantics == LM_BB_FIRSTLAST_INTEGER;
    firstLastOverT(rowsum.data(), (unsigned)N_COLS, lr, P.min_pixel_visible, integer);  // L = I.cols (:975)
    firstLastOverT(colsum.data(), (unsigned)v.height, lc, P.min_pixel_visible, integer);
  }

  // :628-646 (method 0); TM.cpp:145-155; TM_DE.cpp:41-52
  void finish() {
    const int N = (int)frames.size();
    if (METHOD != 0) {
      std::vector<double> bb_x(N);
      for (int i = 0; i < N; ++i) bb_x[i] = frames[i].x;
      vecmovingaverage(bb_x, x_pos, P.moving_average_window);
      yb_pos.assign(N, (uint32_t)(N_ROWS - 1));
      ys_pos.assign(N, METHOD == 1 ? 164u : (uint32_t)(side.height - 1));
      const int w = METHOD == 1 ? P.bb_width : 400;
      bb_side = lm_rect{0, 0, w, METHOD == 1 ? P.bb_height_side : side.height};
      bb_bottom = lm_rect{0, 0, w, bottom.height};
      return;
    }
    std::vector<double> bb_x(N), bb_yb(N), bb_ys(N), bw(N), bhb(N), bht(N);
    for (int i = 0; i < N; ++i) {
      bb_x[i] = frames[i].x;
      bb_yb[i] = frames[i].y_bottom;
      bb_ys[i] = frames[i].y_side;
      bw[i] = frames[i].width;
      bhb[i] = frames[i].height_bottom;
      bht[i] = frames[i].height_side;
    }
    // computeMouseBoxSize (:1481-1506): the medians sort the vectors first.
    double mw = medianvec(bw, N), mhb = medianvec(bhb, N), mht = medianvec(bht, N);
    double sw = stdvec(bw, N), shb = stdvec(bhb, N), sht = stdvec(bht, N);
    uint32_t w3 = x86_u32(mw + 3 * sw), hb3 = x86_u32(mhb + 3 * shb), ht3 = x86_u32(mht + 3 * sht);
    uint32_t fw = ((double)w3 < bw[N - 1]) ? w3 : x86_u32(bw[N - 1]);
    uint32_t fhb = ((double)hb3 < bhb[N - 1]) ? hb3 : x86_u32(bhb[N - 1]);
    uint32_t fht = ((double)ht3 < bht[N - 1]) ? ht3 : x86_u32(bht[N - 1]);
    bb_side = lm_rect{0, 0, (int32_t)fw, (int32_t)fht};
    bb_bottom = lm_rect{0, 0, (int32_t)fw, (int32_t)fhb};
    vecmovingaverage(bb_x, x_pos, P.moving_average_window);
    vecmovingaverage(bb_yb, yb_pos, P.moving_average_window);
    vecmovingaverage(bb_ys, ys_pos, P.moving_average_window);
  }

  lm_bb_params P;
  int METHOD = 0;
  int VR = 0, VC = 0, N_ROWS = 0, N_COLS = 0, pad = 0;
  bool flip = false;
  std::vector<uint8_t> BKG;
  std::vector<int32_t> CAL;
  Rect side, bottom;
  Mat8 I_median;
  std::vector<lm_bb_frame> frames;
  std::vector<Mat8> binary;
  lm_rect bb_side{}, bb_bottom{};
  std::vector<uint32_t> x_pos, yb_pos, ys_pos;
};

}  // namespace lmo

// ------------------------------------------------------------------ C API
static thread_local std::string g_err;

struct lmo_result {
  lmo::Result r;
  int32_t n_frames = 0;
};

LMO_API const char* lmo_last_error(void) { return g_err.c_str(); }

static int map_exc(const std::exception& e, int code) {
  g_err = e.what();
  return code;
}

LMO_API int lmo_geometry(const lm_setup* su, const lm_params* pa, const lm_model* mo, lm_geometry* out) {
  try {
    lmo::LocoMouseOracle L(*su, *pa, *mo, 0);
    L.fill_geometry(*out);
    return LM_OK;
  } catch (const std::invalid_argument& e) {
    return map_exc(e, LM_ERR_INVALID_ARGUMENT);
  } catch (const std::exception& e) {
    return map_exc(e, LM_ERR_RUNTIME);
  }
}

/* Run frames 0..n-1 of a video through the restated per-frame loop
 * (main.cpp:54-82).  bb: NULL (provided box) or [n][3] BR corners. */
LMO_API int lmo_run(const lm_setup* su, const lm_params* pa, const lm_model* mo, const uint8_t* frames, int64_t pitch,
                    int32_t n, const int32_t* bb, int32_t flags, lmo_result** out, lm_batch_result* view) {
  try {
    auto R = std::make_unique<lmo_result>();
    lmo::LocoMouseOracle L(*su, *pa, *mo, flags);
    for (int32_t f = 0; f < n; ++f) {
      unsigned bx = bb ? (unsigned)bb[3 * f] : L.bb_x();
      unsigned byb = bb ? (unsigned)bb[3 * f + 1] : L.bb_yb();
      unsigned bys = bb ? (unsigned)bb[3 * f + 2] : L.bb_ys();
      L.run_frame(frames + (size_t)f * pitch, bx, byb, bys);
    }
    R->r = std::move(L.res);
    R->n_frames = n;
    lmo::Result& r = R->r;
    view->n_frames = n;
    view->first_frame = 0;
    view->cand_offset = r.cand_offset.data();
    view->cand = r.cand.data();
    view->p22d_offset = r.p22d_offset.data();
    view->p22d = r.p22d.data();
    view->side_y = r.side_y.data();
    view->side_s = r.side_s.data();
    view->unary_offset = r.unary_offset.data();
    view->unary = r.unary.data();
    view->pw_dims = r.pw_dims.data();
    view->pw_jc_offset = r.pw_jc_offset.data();
    view->pw_jc = r.pw_jc.data();
    view->pw_nz_offset = r.pw_nz_offset.data();
    view->pw_ir = r.pw_ir.data();
    view->pw_pr = r.pw_pr.data();
    view->tail = r.tail.data();
    *out = R.release();
    return LM_OK;
  } catch (const std::invalid_argument& e) {
    return map_exc(e, LM_ERR_INVALID_ARGUMENT);
  } catch (const std::exception& e) {
    return map_exc(e, LM_ERR_RUNTIME);
  }
}

LMO_API void lmo_free(lmo_result* r) { delete r; }

LMO_API int lmo_debug_scores(const lmo_result* r, int32_t f, int32_t det, float* out, int32_t rows, int32_t cols) {
  if (!r || f < 0 || f >= (int)r->r.scores.size() || det < 0 || det >= 6) return LM_ERR_INVALID_ARGUMENT;
  const lmo::Matf& m = r->r.scores[f][det];
  if (m.rows == 0) return LM_ERR_RUNTIME;  // detector not run (side skipped)
  if (m.rows != rows || m.cols != cols) return LM_ERR_INVALID_ARGUMENT;
  std::memcpy(out, m.d.data(), m.d.size() * sizeof(float));
  return LM_OK;
}

LMO_API int lmo_debug_scores_dims(const lmo_result* r, int32_t f, int32_t det, int32_t* rows, int32_t* cols) {
  if (!r || !rows || !cols || f < 0 || f >= (int)r->r.scores.size() || det < 0 || det >= 6) return LM_ERR_INVALID_ARGUMENT;
  *rows = r->r.scores[f][det].rows;
  *cols = r->r.scores[f][det].cols;
  return LM_OK;
}

LMO_API int lmo_debug_tail_mask(const lmo_result* r, int32_t f, uint8_t* out, int32_t rows, int32_t cols) {
  if (!r || f < 0 || f >= (int)r->r.tail_mask.size()) return LM_ERR_INVALID_ARGUMENT;
  const lmo::Mat8& m = r->r.tail_mask[f];
  if (m.rows != rows || m.cols != cols) return LM_ERR_INVALID_ARGUMENT;
  std::memcpy(out, m.d.data(), m.d.size());
  return LM_OK;
}

LMO_API int lmo_debug_ipad(const lmo_result* r, int32_t f, uint8_t* out, int32_t rows, int32_t cols) {
  if (!r || f < 0 || f >= (int)r->r.ipad.size()) return LM_ERR_INVALID_ARGUMENT;
  const lmo::Mat8& m = r->r.ipad[f];
  if (m.rows != rows || m.cols != cols) return LM_ERR_INVALID_ARGUMENT;
  std::memcpy(out, m.d.data(), m.d.size());
  return LM_OK;
}

/* std::sort(compareCandidate) of candidates (x = i, y = 0, s = scores[i]);
 * writes the resulting permutation (libstdc++ tie order). */
LMO_API void lmo_std_sort_perm(const double* scores, int32_t n, int32_t* perm) {
  std::vector<lmo::Candidate> v((size_t)n);
  for (int32_t i = 0; i < n; ++i) v[i] = lmo::Candidate(i, 0, scores[i]);
  std::sort(v.begin(), v.end(), lmo::compareCandidate);
  for (int32_t i = 0; i < n; ++i) perm[i] = v[i].x;
}

/* Synthetic frames/background (lm_synth.h) on the CPU. */
LMO_API void lmo_synth_frames(int32_t rows, int32_t cols, int64_t first, int32_t n, uint8_t* out) {
  lm_synth_scene sc = lm_synth_default_scene(rows, cols);
  for (int32_t f = 0; f < n; ++f)
    for (int32_t r = 0; r < rows; ++r)
      for (int32_t c = 0; c < cols; ++c)
        out[((size_t)f * rows + r) * cols + c] = lm_synth_pixel(&sc, first + f, r, c);
}

LMO_API void lmo_synth_background(int32_t rows, int32_t cols, uint8_t* out) {
  for (int64_t i = 0; i < (int64_t)rows * cols; ++i) out[i] = lm_synth_background(i);
}

/* Whole-video BB pass (method 0) over frames 0..n-1: per-frame values, the
 * final box sizes and BR corner tracks; binary (optional) receives the
 * thresholded median images [n][N_ROWS][N_COLS]. */
LMO_API int lmo_bb_run(const lm_setup* su, const lm_bb_params* bp, const uint8_t* frames, int64_t pitch, int32_t n,
                       lm_bb_frame* per_frame, lm_rect* bb_side, lm_rect* bb_bottom, uint32_t* x_pos,
                       uint32_t* yb_pos, uint32_t* ys_pos, uint8_t* binary) {
  try {
    if (n < 1) throw std::invalid_argument("BB pass needs at least one frame.");
    lmo::BBOracle B(*su, *bp);
    for (int32_t f = 0; f < n; ++f) B.frame(frames + (size_t)f * pitch);
    B.finish();
    for (int32_t f = 0; f < n; ++f) {
      per_frame[f] = B.frames[f];
      x_pos[f] = B.x_pos[f];
      yb_pos[f] = B.yb_pos[f];
      ys_pos[f] = B.ys_pos[f];
      if (binary && B.METHOD == 0)
        std::memcpy(binary + (size_t)f * B.N_ROWS * B.N_COLS, B.binary[f].d.data(), B.binary[f].d.size());
    }
    *bb_side = B.bb_side;
    *bb_bottom = B.bb_bottom;
    return LM_OK;
  } catch (const std::invalid_argument& e) {
    return map_exc(e, LM_ERR_INVALID_ARGUMENT);
  } catch (const std::exception& e) {
    return map_exc(e, LM_ERR_RUNTIME);
  }
}

/* Pieces of the BB pass, for the oracle's own unit tests. */
LMO_API void lmo_median_blur(const uint8_t* src, int32_t rows, int32_t cols, int32_t ksize, uint8_t* dst) {
  lmo::Mat8 m(rows, cols, 0);
  std::memcpy(m.d.data(), src, (size_t)rows * cols);
  lmo::Mat8 o = lmo::medianBlur8u(m, ksize);
  std::memcpy(dst, o.d.data(), (size_t)rows * cols);
}

LMO_API void lmo_first_last(const int32_t* v, uint32_t L, int32_t th, int32_t integer, int32_t* out2) {
  int fl[2];
  lmo::firstLastOverT(v, L, fl, th, integer != 0);
  out2[0] = fl[0];
  out2[1] = fl[1];
}

LMO_API void lmo_movavg(const double* v, int32_t n, int32_t window, uint32_t* out) {
  std::vector<double> in(v, v + n);
  std::vector<uint32_t> o;
  lmo::vecmovingaverage(in, o, window);
  std::memcpy(out, o.data(), sizeof(uint32_t) * n);
}

LMO_API void lmo_imadjust_default_lut(const uint32_t* hist, uint8_t* lut) {
  std::vector<uint32_t> h(hist, hist + 256);
  lmo::BBOracle::imadjust_default_lut(h, lut);
}
