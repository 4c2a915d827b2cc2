// LocoMouse.cpp — host C++ mirror of the reference's per-frame LocoMouse
// surface over the MI355X C-ABI.  See LocoMouse.hpp for the contract; every
// method cites the reference code whose observable behaviour it keeps.
#include "LocoMouse.hpp"

#include <algorithm>
#include <condition_variable>
#include <cstring>
#include <iostream>
#include <mutex>
#include <set>
#include <stdexcept>
#include <chrono>
#include <thread>

namespace locomouse {

// ------------------------------------------------------------- Candidates

bool compareCandidate(Candidate a, Candidate b) { return a.score() > b.score(); }  // Candidates.cpp:33-36

P22D::P22D() : CB(), yt{-1}, st{-1} {}
P22D::P22D(int xc, int ybc, int ytc, double scr_b, double scr_t) : CB(xc, ybc, scr_b), yt{ytc}, st{scr_t} {}
P22D::P22D(Point_<int> Pb, Point_<int> Pt, double scr_b, double scr_t) : CB(Pb, scr_b), yt{Pt.y}, st{scr_t} {}
P22D::P22D(Candidate Cb, Candidate Ct) : CB(Cb.point(), Cb.score()), yt{Ct.point().y}, st{Ct.score()} {}

Point_<int> P22D::point_bottom() const { return CB.point(); }
Point_<int> P22D::point_side(unsigned index) const { return Point_<int>(CB.point().x, yt.at(index)); }
double P22D::score_bottom() const { return CB.score(); }
double P22D::score_side(unsigned index) const { return st.at(index); }
int P22D::x_coord() const { return CB.point().x; }
int P22D::y_bottom_coord() const { return CB.point().y; }
int P22D::y_side_coord(unsigned index) const { return yt.at(index); }

void P22D::add_side_candidate(Candidate C) { add_side_candidate_safe(C.point().x, C.point().y, C.score()); }
void P22D::add_side_candidate(Point_<int> P, double s) { add_side_candidate_safe(P.x, P.y, s); }
void P22D::add_side_candidate(int y, double s) { add_side_candidate_safe(CB.point().x, y, s); }

// Candidates.cpp:106-115: an empty P22D takes the first side candidate in
// slot 0; later ones are appended and must have S >= 0 (CV_Assert).
void P22D::add_side_candidate_safe(int, int Y, double S) {
  if (number_of_candidates() == 0) {
    yt[0] = Y;
    st[0] = S;
    return;
  }
  if (!(S >= 0)) throw std::runtime_error("P22D::add_side_candidate_safe: CV_Assert(S >= 0) failed.");
  yt.push_back(Y);
  st.push_back(S);
}

int P22D::number_of_candidates() const { return st[0] < 0 ? 0 : (int)st.size(); }  // Candidates.cpp:148-156
Candidate P22D::get_candidate_side(unsigned index) const { return Candidate(CB.point().x, yt.at(index), st.at(index)); }
Candidate P22D::get_candidate_bottom() const { return CB; }

void P22D::set_side_raw(const int* y, const double* s, int count) {
  if (count < 1) throw std::invalid_argument("P22D::set_side_raw: a P22D holds at least one side entry.");
  yt.assign(y, y + count);
  st.assign(s, s + count);
}

bool P22D::operator==(const P22D& o) const {
  return CB.p == o.CB.p && CB.s == o.CB.s && yt == o.yt && st == o.st;
}

std::ostream& operator<<(std::ostream& out, const Candidate& c) {
  return out << "[(" << c.point().x << ", " << c.point().y << ") with score = " << c.s << "]";
}

std::ostream& operator<<(std::ostream& out, const P22D& c) {
  out << "Bottom candidate: " << c.get_candidate_bottom() << "\n" << c.number_of_candidates() << " top candidate(s):\n";
  for (int i = 0; i < c.number_of_candidates(); ++i)
    out << "[" << c.y_side_coord(i) << " with score = " << c.score_side(i) << "]\n";
  return out;
}

// ------------------------------------------------------------------ MyMat

void MyMat::put(unsigned i, unsigned j, double val) {
  if ((int)i >= nrows || (int)j >= ncols) throw std::out_of_range("MyMat::put index out of range");
  values[(size_t)j * nrows + i] = val;  // column-major (MyMat.cpp:64-70)
}

double MyMat::get(unsigned i, unsigned j) const {
  if ((int)i >= nrows || (int)j >= ncols) throw std::out_of_range("MyMat::get index out of range");
  return values[(size_t)j * nrows + i];
}

MATSPARSE::MATSPARSE(const MyMat* M) : n_rows(M->Nrows()), n_cols(M->Ncols()) {
  Jc.reserve((size_t)n_cols + 1);
  Jc.push_back(0);
  for (int j = 0; j < n_cols; ++j) {  // MyMat.cpp:141-178
    for (int i = 0; i < n_rows; ++i) {
      const double v = M->get(i, j);
      if (v != 0) {
        Ir.push_back(i);
        Pr.push_back(v);
      }
    }
    Jc.push_back((int)Ir.size());
  }
  nzel = (int)Ir.size();
}

MATSPARSE::MATSPARSE(int rows, int cols, const int* jc, const int* ir, const double* pr)
    : Jc(jc, jc + cols + 1), nzel(jc[cols]), n_rows(rows), n_cols(cols) {
  Ir.assign(ir, ir + nzel);
  Pr.assign(pr, pr + nzel);
}

double MATSPARSE::get(int, int) const { return 0; }  // MyMat.cpp:371-374 returns before its lookup

double MATSPARSE::at(int irow, int icol) const {
  if (icol < 0 || icol >= n_cols || irow < 0 || irow >= n_rows) throw std::out_of_range("MATSPARSE::at");
  double val = 0;
  for (int k = Jc[icol]; k < Jc[icol + 1]; ++k)
    if (Ir[k] == irow) val = Pr[k];
  return val;
}

bool MATSPARSE::operator==(const MATSPARSE& o) const {
  return n_rows == o.n_rows && n_cols == o.n_cols && Jc == o.Jc && Ir == o.Ir && Pr == o.Pr;
}

std::ostream& operator<<(std::ostream& out, const MyMat& M) {
  if (M.Nrows() == 0 || M.Ncols() == 0) return out << "Matrix is empty!\n";
  out << "[";
  for (int i = 0; i < M.Nrows(); ++i) {
    for (int j = 0; j < M.Ncols(); ++j) out << M.get(i, j) << (j + 1 < M.Ncols() ? ", " : "");
    out << (i + 1 < M.Nrows() ? ";\n" : "]\n");
  }
  return out;
}

// -------------------------------------------------------------- LocoMouse

void throw_on_error(lm_status s) {
  if (s == LM_OK) return;
  if (s == LM_ERR_INVALID_ARGUMENT) throw std::invalid_argument(lm_last_error());
  throw std::runtime_error(lm_last_error());
}

// ------------------------------------------------------- multi-GPU shards
//
// main.cpp:54-82 is a loop over frames whose only cross-frame state is the
// previous frame (pairwise costs read frame f-1's candidates, the motion
// check its pixels), so contiguous frame ranges run independently given
// their predecessor frame as a 1-frame halo.  The reader
// delivers frames in order, so the shards are the batches themselves: batch
// k goes to device k mod D with the last frame of batch k-1 as its halo.
// One host thread per device owns that device's context; it submits its
// batches (lm_detect_submit copies host frames before returning, so the
// pinned buffer goes straight back to the pool) and collects them into a
// FrameResults chunk, which the caller's thread appends in frame order.
struct LocoMouse::DevicePool {
  struct Job {
    int first = 0, n = 0;
    uint8_t* frames = nullptr;     // pinned batch buffer (returned to the pool once submitted)
    std::vector<uint8_t> halo;     // frame first-1 (empty for the video's first batch)
    std::vector<int32_t> bb;       // per-frame corners, halo frame first when present
    std::promise<std::unique_ptr<FrameResults>> done;
  };
  struct Worker {
    int device = 0;
    lm_ctx* ctx = nullptr;
    std::thread th;
    std::mutex m;
    std::condition_variable cv;
    std::deque<std::shared_ptr<Job>> queue;
    bool stop = false;
  };

  size_t frame_bytes = 0;
  int batch = 0, lanes = 1;
  std::vector<std::unique_ptr<Worker>> workers;
  std::mutex free_m;
  std::condition_variable free_cv;
  std::vector<uint8_t*> free_bufs;
  std::vector<uint8_t*> all_bufs;
  std::deque<std::future<std::unique_ptr<FrameResults>>> results;  // oldest batch first
  size_t next = 0;                                                  // the next batch's worker

  DevicePool(const std::vector<int>& devices, const lm_setup& setup, const lm_params& params, const lm_model& model,
             int batch_, size_t frame_bytes_)
      : frame_bytes(frame_bytes_), batch(batch_), lanes(std::max(1, setup.pipeline_lanes)) {
    try {
      for (int d : devices) {
        auto w = std::make_unique<Worker>();
        w->device = d;
        throw_on_error(lm_ctx_create(d, &setup, &params, &model, batch, &w->ctx));
        workers.push_back(std::move(w));
      }
      // two buffers per device: one being filled by the reader while another waits for its worker
      for (size_t i = 0; i < 2 * workers.size(); ++i) {
        void* q = nullptr;
        throw_on_error(lm_host_alloc(frame_bytes * (size_t)batch, &q));
        all_bufs.push_back(static_cast<uint8_t*>(q));
      }
    } catch (...) {
      release();
      throw;
    }
    free_bufs = all_bufs;
    for (auto& w : workers) w->th = std::thread([this, p = w.get()] { run(*p); });
  }
  ~DevicePool() {
    for (auto& w : workers) {
      {
        std::lock_guard<std::mutex> g(w->m);
        w->stop = true;
      }
      w->cv.notify_all();
    }
    for (auto& w : workers)
      if (w->th.joinable()) w->th.join();
    release();
  }
  void release() {
    for (auto& w : workers)
      if (w->ctx) {
        lm_ctx_destroy(w->ctx);
        w->ctx = nullptr;
      }
    for (uint8_t* p : all_bufs) lm_host_free(p);
    all_bufs.clear();
  }
  lm_ctx* first_ctx() const { return workers.front()->ctx; }
  size_t capacity() const { return workers.size() * 2 * (size_t)lanes; }

  uint8_t* take_buffer() {
    std::unique_lock<std::mutex> g(free_m);
    free_cv.wait(g, [this] { return !free_bufs.empty(); });
    uint8_t* p = free_bufs.back();
    free_bufs.pop_back();
    return p;
  }
  void give_buffer(uint8_t* p) {
    {
      std::lock_guard<std::mutex> g(free_m);
      free_bufs.push_back(p);
    }
    free_cv.notify_one();
  }

  void submit(std::shared_ptr<Job> j) {
    results.push_back(j->done.get_future());
    Worker& w = *workers[next];
    next = (next + 1) % workers.size();
    {
      std::lock_guard<std::mutex> g(w.m);
      w.queue.push_back(std::move(j));
    }
    w.cv.notify_one();
  }

  // A device's thread: submit queued batches while fewer than 2 x lanes are
  // waiting for collection, otherwise collect the oldest.
  void run(Worker& w) {
    std::deque<std::shared_ptr<Job>> inflight;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> g(w.m);
        w.cv.wait(g, [&] { return w.stop || !w.queue.empty() || !inflight.empty(); });
        if (w.stop) {  // the object is going away: batches not yet submitted are dropped
          for (auto& q : w.queue) give_buffer(q->frames);
          w.queue.clear();
        }
        if (!w.queue.empty() && (int)inflight.size() < 2 * lanes) {
          j = std::move(w.queue.front());
          w.queue.pop_front();
        } else if (inflight.empty()) {
          return;  // stopped, nothing queued or in flight
        }
      }
      if (j) {
        try {
          throw_on_error(lm_detect_submit(w.ctx, j->frames, (int64_t)frame_bytes, j->n, j->first,
                                          j->halo.empty() ? nullptr : j->halo.data(), j->bb.data()));
          give_buffer(j->frames);
          inflight.push_back(std::move(j));
        } catch (...) {
          give_buffer(j->frames);
          j->done.set_exception(std::current_exception());
        }
        continue;
      }
      std::shared_ptr<Job> o = std::move(inflight.front());
      inflight.pop_front();
      try {
        lm_batch_result r{};
        throw_on_error(lm_detect_collect(w.ctx, &r));
        auto fr = std::make_unique<FrameResults>();
        fr->append(r);
        o->done.set_value(std::move(fr));
      } catch (...) {
        o->done.set_exception(std::current_exception());
      }
    }
  }
};

namespace {
template <class T>
void move_append(std::vector<T>& dst, std::vector<T>& src) {
  dst.insert(dst.end(), std::make_move_iterator(src.begin()), std::make_move_iterator(src.end()));
}
}  // namespace

LocoMouse::LocoMouse(const LocoMouse_Inputs& inputs) : IN(inputs), METHOD(0), N_FRAMES(inputs.n_frames) {
  if (!IN.read_frame && !IN.read_frames) throw std::invalid_argument("LocoMouse: no frame reader (V) given.");
  if (IN.batch < 1) throw std::invalid_argument("LocoMouse: batch must be >= 1.");
  if (IN.setup.video_rows <= 0 || IN.setup.video_cols <= 0)
    throw std::invalid_argument("LocoMouse: video size must be positive.");
  FRAME_BYTES = (size_t)IN.setup.video_rows * IN.setup.video_cols;
  IN.setup.method = 0;
  if (IN.devices.empty()) IN.devices.push_back(IN.device);
  if (!IN.oversubscribe && std::set<int>(IN.devices.begin(), IN.devices.end()).size() != IN.devices.size())
    throw std::invalid_argument("LocoMouse: a device is listed twice (set oversubscribe to share devices).");
  for (int d : IN.devices)
    if (d < 0) throw std::invalid_argument("LocoMouse: invalid device index " + std::to_string(d) + ".");
  IN.device = IN.devices.front();  // the BB pass and the geometry queries
  if (IN.verbose_debug && !IN.debug_text.empty()) DEBUG_TEXT.open(IN.debug_text);  // :341-343
}

LocoMouse::~LocoMouse() {
  // both wait for the batches in flight; their errors die with the object
  if (POOL) {
    PENDING.p = nullptr;  // a pool buffer: the pool frees it
    POOL.reset();
  } else if (CTX) {
    lm_ctx_destroy(CTX);
  }
}

// :543-569: with use_provided_bounding_box the bottom-right corners are the
// provided boxes' for every frame; otherwise the whole-video pass runs.
void LocoMouse::getBoundingBox() {
  if (IN.params.use_provided_bounding_box) {
    const lm_rect& b = IN.params.bounding_box_bottom;
    const lm_rect& s = IN.params.bounding_box_side;
    BB_X_POS.assign(N_FRAMES, (uint32_t)(b.x + b.width));
    BB_Y_SIDE_POS.assign(N_FRAMES, (uint32_t)(s.y + s.height));
    BB_Y_BOTTOM_POS.assign(N_FRAMES, (uint32_t)(b.y + b.height));
    BB_BOTTOM_MOUSE = lm_rect{0, 0, b.width, b.height};
    BB_SIDE_MOUSE = lm_rect{0, 0, s.width, s.height};
    HAVE_BB = true;
  } else {
    if (DEBUG_TEXT.is_open()) DEBUG_TEXT << "===== Computing the bounding box coordinates: " << std::endl;  // :582
    computeBoundingBox();
    if (DEBUG_TEXT.is_open())  // :638-650
      DEBUG_TEXT << "----- Final BB sizes: " << std::endl
                 << "BB_SIDE_MOUSE: " << debug_rect(BB_SIDE_MOUSE) << std::endl
                 << "BB_BOTTOM_MOUSE: " << debug_rect(BB_BOTTOM_MOUSE) << std::endl
                 << "===== END " << std::endl
                 << std::endl;
  }
}

// :579-653: every frame of the video through computeMouseBox (readFrame into
// the padded median image, :615), then computeMouseBoxSize and the moving
// averages — all in lm_bb_push / lm_bb_finish.  The video is re-read from
// frame 0 afterwards, as initializeFeatureLoop's V.set(POS_FRAMES, 0)
// (:761-762) does in the reference.
void LocoMouse::computeBoundingBox() { runBoundingBoxPass(0); }

// The pass of LocoMouse (method 0), LocoMouse_TM (1) or LocoMouse_TM_DE (2).
void LocoMouse::runBoundingBoxPass(int method) {
  if (!IN.rewind)
    throw std::invalid_argument("computeBoundingBox: the frame reader cannot rewind (V.set(CV_CAP_PROP_POS_FRAMES, 0)).");
  if (N_FRAMES == 0) throw std::runtime_error("computeBoundingBox: the video has no frames.");
  lm_setup su = IN.setup;
  su.method = method;
  lm_bb_ctx* raw = nullptr;
  throw_on_error(lm_bb_create(IN.device, &su, &IN.bb_params, IN.batch, &raw));
  std::unique_ptr<lm_bb_ctx, void (*)(lm_bb_ctx*)> bb(raw, lm_bb_destroy);
  std::vector<uint8_t> buf(FRAME_BYTES * (size_t)IN.batch);
  for (unsigned done = 0; done < N_FRAMES;) {
    const int n = (int)std::min<unsigned>((unsigned)IN.batch, N_FRAMES - done);
    if (IN.read_frames) {
      if (IN.read_frames(buf.data(), n) != n) throw std::runtime_error("Error: Failed to read image from video file.\n");
    } else {
      for (int i = 0; i < n; ++i)
        if (!IN.read_frame(buf.data() + (size_t)i * FRAME_BYTES))
          throw std::runtime_error("Error: Failed to read image from video file.\n");  // :1284-1286
    }
    throw_on_error(lm_bb_push(bb.get(), buf.data(), (int64_t)FRAME_BYTES, n, nullptr));
    done += (unsigned)n;
  }
  lm_bb_result r{};
  throw_on_error(lm_bb_finish(bb.get(), &r));
  BB_X_POS.assign(r.x_pos, r.x_pos + r.n_frames);
  BB_Y_BOTTOM_POS.assign(r.y_bottom_pos, r.y_bottom_pos + r.n_frames);
  BB_Y_SIDE_POS.assign(r.y_side_pos, r.y_side_pos + r.n_frames);
  BB_SIDE_MOUSE = r.bb_side_mouse;
  BB_BOTTOM_MOUSE = r.bb_bottom_mouse;
  // The detection context derives its geometry from these sizes (:655-700);
  // the per-frame corners go to lm_detect_batch.
  IN.params.bounding_box_side = BB_SIDE_MOUSE;
  IN.params.bounding_box_bottom = BB_BOTTOM_MOUSE;
  IN.params.use_provided_bounding_box = 1;
  HAVE_BB = true;
  IN.rewind();
}

// :655-769 derives the geometry; here the device context does (lm_ctx_create
// validates the same inputs and raises the reference's errors).
void LocoMouse::initializeFeatureLoop() {
  if (!HAVE_BB) throw std::runtime_error("initializeFeatureLoop: getBoundingBox() has not been called.");
  if (CTX) return;
  IN.setup.method = METHOD;
  if (DEBUG_TEXT.is_open())  // :662-667
    DEBUG_TEXT << "===== Preparing Feature Tracking Loop: " << std::endl
               << "BB_SIDE_MOUSE: " << debug_rect(BB_SIDE_MOUSE) << std::endl
               << "BB_BOTTOM_MOUSE: " << debug_rect(BB_BOTTOM_MOUSE) << std::endl;
  IN.setup.pipeline_lanes = std::max(1, std::min(IN.lanes, LM_MAX_LANES));
  if (IN.devices.size() > 1) {
    POOL = std::make_unique<DevicePool>(IN.devices, IN.setup, IN.params, IN.model, IN.batch, FRAME_BYTES);
    CTX = POOL->first_ctx();
    PENDING.p = POOL->take_buffer();  // pool-owned: handed to the workers and swapped at every flush
  } else {
    throw_on_error(lm_ctx_create(IN.device, &IN.setup, &IN.params, &IN.model, IN.batch, &CTX));
    PENDING.allocate(FRAME_BYTES * (size_t)IN.batch);
  }
  N_PENDING = 0;
  if (DEBUG_TEXT.is_open()) {  // :700-704, :766
    const lm_geometry g = geometry();
    DEBUG_TEXT << "M_size_pre_side().height, M_size_pre_bottom().height: " << g.spre_t_h << " " << g.spre_b_h
               << std::endl
               << "M_size_pre_side().width, M_size_pre_bottom().width: " << g.spre_t_w << " " << g.spre_b_w
               << std::endl
               << "I_PAD: [" << g.ipad_cols << " x " << g.ipad_rows << "]" << std::endl
               << "I_UNPAD: " << debug_rect(lm_rect{g.pad_pre_cols, g.pad_pre_rows, g.n_cols, g.n_rows}) << std::endl
               << "BB_BOTTOM_MOUSE_PAD, UNPAD: " << debug_rect(g.bb_bottom_mouse_pad) << " "
               << debug_rect(g.bb_unpad_mouse_bottom) << std::endl
               << "BB_SIDE_MOUSE_PAD, UNPAD: " << debug_rect(g.bb_side_mouse_pad) << " "
               << debug_rect(g.bb_unpad_mouse_side) << std::endl
               << "===== Done " << std::endl;
  }
}

// :1273-1333 reads the next frame (V >> F, channel 0).  The frame is queued;
// background subtraction, normalisation, calibration and (TM) imadjust run on
// the device when its batch is processed.
void LocoMouse::readFrame() {
  if (!CTX) throw std::runtime_error("readFrame: initializeFeatureLoop() has not been called.");
  if (N_PENDING == IN.batch) flush();  // a caller that skips storePreviousImage
  const unsigned left = N_FRAMES - (unsigned)(CURRENT_FRAME + 1);
  if (IN.read_frames && N_PENDING == N_READ_AHEAD && left > 0) {
    const int want = (int)std::min<unsigned>((unsigned)(IN.batch - N_PENDING), left);
    N_READ_AHEAD += std::max(0, IN.read_frames(PENDING.data() + (size_t)N_PENDING * FRAME_BYTES, want));
  }
  const bool ok = left > 0 && (IN.read_frames ? N_PENDING < N_READ_AHEAD
                                              : IN.read_frame(PENDING.data() + (size_t)N_PENDING * FRAME_BYTES));
  if (!ok) throw std::runtime_error("Error: Failed to read image from video file.\n");  // :1284-1286
  ++N_PENDING;
  ++CURRENT_FRAME;
}

// The eight per-frame stages of main.cpp:60-80 run inside lm_detect_batch.
void LocoMouse::cropBoundingBox() {}
void LocoMouse::detectTail() {}
void LocoMouse::detectBottomCandidates() {}
void LocoMouse::computeUnaryCostsBottom() {}
void LocoMouse::computePairwiseCostsBottom() {}
void LocoMouse::detectSideCandidates() {}
void LocoMouse::matchBottomSideCandidates() {}

// :1508-1513 keeps I_PAD for the next frame; the device keeps the previous
// frame across batches, so this is where a full batch (or the video's last
// frame) is handed over.
void LocoMouse::storePreviousImage() {
  if (N_PENDING && (N_PENDING == IN.batch || (unsigned)(CURRENT_FRAME + 1) == N_FRAMES)) flush();
}

void LocoMouse::HostBuffer::allocate(size_t bytes) {
  lm_host_free(p);
  p = nullptr;
  void* q = nullptr;
  throw_on_error(lm_host_alloc(bytes, &q));
  p = static_cast<uint8_t*>(q);
}

void LocoMouse::sync() {
  if (N_PENDING) flush();
  while (!INFLIGHT.empty()) collect_oldest();
}

// The oldest batch in flight: its results are appended in frame order.  Its
// errors (the reference's exceptions) surface here: at the per-frame call
// that hands over a batch while every lane is busy, or at sync().
void LocoMouse::collect_oldest() {
  const auto t0 = std::chrono::steady_clock::now();
  struct Tally {  // wall time of this call, also when it throws
    std::chrono::steady_clock::time_point t0;
    double& acc;
    ~Tally() { acc += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
  } tally{t0, TIMES.wait_s};
  const std::pair<int, int> b = INFLIGHT.front();
  INFLIGHT.pop_front();
  if (POOL) {  // the batch's device thread collected it into a chunk of containers
    auto fut = std::move(POOL->results.front());
    POOL->results.pop_front();
    std::unique_ptr<FrameResults> R = fut.get();
    move_append(CANDIDATES_BOTTOM_PAW, R->CANDIDATES_BOTTOM_PAW);
    move_append(CANDIDATES_BOTTOM_SNOUT, R->CANDIDATES_BOTTOM_SNOUT);
    move_append(CANDIDATES_SIDE_PAW, R->CANDIDATES_SIDE_PAW);
    move_append(CANDIDATES_SIDE_SNOUT, R->CANDIDATES_SIDE_SNOUT);
    move_append(CANDIDATES_MATCHED_VIEWS_PAW, R->CANDIDATES_MATCHED_VIEWS_PAW);
    move_append(CANDIDATES_MATCHED_VIEWS_SNOUT, R->CANDIDATES_MATCHED_VIEWS_SNOUT);
    move_append(UNARY_BOTTOM_PAW, R->UNARY_BOTTOM_PAW);
    move_append(UNARY_BOTTOM_SNOUT, R->UNARY_BOTTOM_SNOUT);
    move_append(PAIRWISE_BOTTOM_PAW, R->PAIRWISE_BOTTOM_PAW);
    move_append(PAIRWISE_BOTTOM_SNOUT, R->PAIRWISE_BOTTOM_SNOUT);
    move_append(TRACKS_TAIL, R->TRACKS_TAIL);
  } else {
    lm_batch_result r{};
    throw_on_error(lm_detect_collect(CTX, &r));
    append(r);
  }
  if (DEBUG_TEXT.is_open()) debug_frames(b.first, b.second);
}

lm_geometry LocoMouse::geometry() const {
  lm_geometry g{};
  if (!CTX) throw std::runtime_error("geometry: initializeFeatureLoop() has not been called.");
  throw_on_error(lm_get_geometry(CTX, &g));
  return g;
}

// A full batch goes to the device (lm_detect_submit copies the frames and
// returns); up to IN.lanes batches run on the device at once while the
// caller reads the next frames, and up to 2 x IN.lanes wait for their results
// to be appended (oldest first, so results are appended in frame order).
void LocoMouse::flush() {
  const int n = N_PENDING, first = CURRENT_FRAME + 1 - n;
  // multi-GPU: every batch but the video's first carries its predecessor frame (and its corners) as a halo
  const int h = (POOL && first > 0) ? 1 : 0;
  std::vector<int32_t> bb((size_t)3 * (n + h));
  for (int i = -h; i < n; ++i) {
    bb[3 * (i + h)] = (int32_t)BB_X_POS[first + i];
    bb[3 * (i + h) + 1] = (int32_t)BB_Y_BOTTOM_POS[first + i];
    bb[3 * (i + h) + 2] = (int32_t)BB_Y_SIDE_POS[first + i];
  }
  // Frames already read ahead past this batch (read_frames fills up to a whole
  // batch; a caller that reads results mid-batch flushes early) move to the
  // front of the pending buffer, so the reader's position and the frame
  // numbering stay in step.
  const int ahead = std::max(0, N_READ_AHEAD - n);
  ++TIMES.batches;
  if (POOL) {
    while (INFLIGHT.size() >= POOL->capacity()) collect_oldest();
    auto j = std::make_shared<DevicePool::Job>();
    j->first = first;
    j->n = n;
    j->frames = PENDING.p;
    j->bb = std::move(bb);
    if (h) j->halo = LAST_FRAME;
    LAST_FRAME.assign(PENDING.p + (size_t)(n - 1) * FRAME_BYTES, PENDING.p + (size_t)n * FRAME_BYTES);
    const auto t0 = std::chrono::steady_clock::now();
    uint8_t* fresh = POOL->take_buffer();  // waits while every buffer is queued or being submitted
    if (ahead) std::memcpy(fresh, PENDING.p + (size_t)n * FRAME_BYTES, (size_t)ahead * FRAME_BYTES);
    PENDING.p = fresh;
    POOL->submit(std::move(j));
    TIMES.submit_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    INFLIGHT.push_back({first, n});
  } else {
    while ((int)INFLIGHT.size() >= 2 * lm_ctx_lanes(CTX)) collect_oldest();
    const auto t0 = std::chrono::steady_clock::now();
    throw_on_error(lm_detect_submit(CTX, PENDING.data(), (int64_t)FRAME_BYTES, n, first, nullptr, bb.data()));
    TIMES.submit_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    INFLIGHT.push_back({first, n});
    if (ahead)
      std::memmove(PENDING.data(), PENDING.data() + (size_t)n * FRAME_BYTES, (size_t)ahead * FRAME_BYTES);
  }
  N_PENDING = 0;
  N_READ_AHEAD = ahead;
}

// After the loop (main.cpp:86-91): the tracker over the containers above.
TrackSetup LocoMouse::track_setup() {
  sync();
  if (CURRENT_FRAME + 1 != (int)N_FRAMES)
    throw std::runtime_error("computeBottomTracks: the per-frame loop has not read every frame.");
  TrackSetup S = make_track_setup(geometry(), IN.params, N_FRAMES);
  S.bb_x_pos = &BB_X_POS;
  S.bb_y_bottom_pos = &BB_Y_BOTTOM_POS;
  S.bb_y_side_pos = &BB_Y_SIDE_POS;
  return S;
}

void LocoMouse::computeBottomTracks() {
  const TrackSetup S = track_setup();
  if (DEBUG_TEXT.is_open()) DEBUG_TEXT << "=== Compute Bottom Tracks: " << std::endl;  // :2161-2197
  locomouse::computeBottomTracks(*this, S, TRACKS);
  if (DEBUG_TEXT.is_open()) DEBUG_TEXT << "=== Done " << std::endl;
}

void LocoMouse::computeSideTracks() {
  const TrackSetup S = track_setup();
  if (DEBUG_TEXT.is_open()) DEBUG_TEXT << "=== computeSideTracks(): " << std::endl;  // :2205-2214
  locomouse::computeSideTracks(*this, S, TRACKS);
  if (DEBUG_TEXT.is_open()) DEBUG_TEXT << "=== Done " << std::endl;
}

void LocoMouse::exportResults() {  // :2348-2383
  const TrackSetup S = track_setup();
  if (DEBUG_TEXT.is_open()) DEBUG_TEXT << "=== exportResults: " << std::endl;
  exportTracks(*this, S, TRACKS);
  if (!IN.output_file.empty()) writeOutputYaml(IN.output_file, TRACKS);
  if (DEBUG_TEXT.is_open())
    DEBUG_TEXT << "Paw tracks exported" << std::endl
               << "Snout tracks exported" << std::endl
               << "Tail Tracks exported" << std::endl;
  if (IN.verbose_debug) {
    exportDebugVariables();
    if (DEBUG_TEXT.is_open()) DEBUG_TEXT << "=== Done " << std::endl;
  }
}

#define LM_ACCESSOR(fn, member) \
  const decltype(LocoMouse::member)& LocoMouse::fn() { \
    sync();                                       \
    return member;                                \
  }
LM_ACCESSOR(candidates_bottom_paw, CANDIDATES_BOTTOM_PAW)
LM_ACCESSOR(candidates_bottom_snout, CANDIDATES_BOTTOM_SNOUT)
LM_ACCESSOR(candidates_side_paw, CANDIDATES_SIDE_PAW)
LM_ACCESSOR(candidates_side_snout, CANDIDATES_SIDE_SNOUT)
LM_ACCESSOR(candidates_matched_views_paw, CANDIDATES_MATCHED_VIEWS_PAW)
LM_ACCESSOR(candidates_matched_views_snout, CANDIDATES_MATCHED_VIEWS_SNOUT)
LM_ACCESSOR(unary_bottom_paw, UNARY_BOTTOM_PAW)
LM_ACCESSOR(unary_bottom_snout, UNARY_BOTTOM_SNOUT)
LM_ACCESSOR(pairwise_bottom_paw, PAIRWISE_BOTTOM_PAW)
LM_ACCESSOR(pairwise_bottom_snout, PAIRWISE_BOTTOM_SNOUT)
LM_ACCESSOR(tracks_tail, TRACKS_TAIL)
#undef LM_ACCESSOR

// ------------------------------------------------------------ TM, TM_DE

LocoMouse_TM::LocoMouse_TM(const LocoMouse_Inputs& inputs) : LocoMouse(inputs) { METHOD = 1; }
void LocoMouse_TM::readFrame() { LocoMouse::readFrame(); }  // + imadjust (TM.cpp:243-249), on the device
void LocoMouse_TM::computeBoundingBox() { runBoundingBoxPass(1); }  // TM.cpp:115-157

LocoMouse_TM_DE::LocoMouse_TM_DE(const LocoMouse_Inputs& inputs) : LocoMouse(inputs) { METHOD = 2; }
void LocoMouse_TM_DE::readFrame() { LocoMouse::readFrame(); }
void LocoMouse_TM_DE::computeBoundingBox() { runBoundingBoxPass(2); }  // TM_DE.cpp:8-54

std::unique_ptr<LocoMouse> LocoMouse_Initialize(const LocoMouse_Inputs& inputs) {
  switch (inputs.setup.method) {
    case 0:
      return std::unique_ptr<LocoMouse>(new LocoMouse(inputs));
    case 1:
      return std::unique_ptr<LocoMouse>(new LocoMouse_TM(inputs));
    case 2:
      return std::unique_ptr<LocoMouse>(new LocoMouse_TM_DE(inputs));
    default:
      std::cout << "Unknown method option. Attempting to track with the default method." << std::endl;
      return std::unique_ptr<LocoMouse>(new LocoMouse(inputs));
  }
}

}  // namespace locomouse
