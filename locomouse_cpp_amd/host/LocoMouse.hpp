// LocoMouse.hpp — host C++ mirror of the reference's LocoMouse class surface
// for the per-frame detection path, running on the MI355X C-ABI
// (include/locomouse_hip.h).
//
// Reference surface kept (LocoMouse_Core/LocoMouse_class.hpp:169-350,
// main.cpp:45-82): the factory LocoMouse_Initialize (LocoMouse_Methods.cpp:3-26)
// choosing LocoMouse / LocoMouse_TM / LocoMouse_TM_DE by method, the virtual
// readFrame / getBoundingBox / computeBoundingBox, and the per-frame methods
// called in main.cpp's order:
//
//   L->getBoundingBox(); L->initializeFeatureLoop();
//   for (i < L->N_frames()) { readFrame; cropBoundingBox; detectTail;
//     detectBottomCandidates; computeUnaryCostsBottom; computePairwiseCostsBottom;
//     detectSideCandidates; matchBottomSideCandidates; storePreviousImage; }
//
// The per-frame methods are thin shims: readFrame copies the raw frame into a
// batch buffer and storePreviousImage hands full batches (or the video's last
// frames) to lm_detect_batch; the results are appended in frame order to the
// same containers the reference fills (LocoMouse_class.hpp:219-236), exposed
// here through accessors that first flush any pending frames.  Errors are the
// reference's: std::invalid_argument / std::runtime_error (main.cpp:94-101).
//
// Inputs are already-decoded data (lm_setup / lm_params / lm_model plus a
// frame reader): the YAML/AVI/PNG readers behind LocoMouse_ParseInputs are the
// on-disk formats of SURVEY.md §8(f) row 2, outside this path.
#ifndef LOCOMOUSE_HOST_LOCOMOUSE_HPP
#define LOCOMOUSE_HOST_LOCOMOUSE_HPP

#include <array>
#include <cstdint>
#include <fstream>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "Candidates.hpp"
#include "MyMat.hpp"
#include "Tracks.hpp"
#include "locomouse_hip.h"

namespace locomouse {

// What LocoMouse_ParseInputs + the file loaders provide (ParseInputs.cpp:62-99,
// LocoMouse_class.cpp:307-540, :3095-3162), already in memory.  The pointers
// inside setup/params/model must stay valid until initializeFeatureLoop().
struct LocoMouse_Inputs {
  lm_setup setup{};    // setup.method: 0 LocoMouse, 1 LocoMouse_TM, 2 LocoMouse_TM_DE
  lm_params params{};
  lm_model model{};
  uint32_t n_frames = 0;  // N_FRAMES (CV_CAP_PROP_FRAME_COUNT)
  // V >> F; extractChannel(F, F, 0): writes the next frame (video_rows x
  // video_cols u8, row-major) and returns false at the end of the video.
  std::function<bool(uint8_t* dst)> read_frame;
  // Optional: the next (up to) n frames into dst (n x video_rows x video_cols,
  // contiguous), returning how many were read.  When given, readFrame reads a
  // whole batch ahead at its first frame (so a decoder can fill it in
  // parallel, without a per-frame copy); frames are still consumed in order.
  // It may return fewer than n frames only at the end of the video or on a
  // read error: the shortfall is reported ("Failed to read image") when the
  // missing frame is consumed.  Frames read ahead survive a batch handed over
  // early (a result accessor called mid-batch).
  std::function<int(uint8_t* dst, int n)> read_frames;
  int device = 0;      // HIP device of this instance (one per GPU / host thread)
  int batch = 256;     // frames per lm_detect_submit / lm_bb_push call
  int lanes = 4;       // batches in flight on the device (lm_setup.pipeline_lanes)
  // Multi-GPU detection: with more than one
  // entry, the video is cut into contiguous shards of `batch` frames dealt to
  // the devices in turn, each shard run with its predecessor frame as a
  // 1-frame halo (the per-frame path has no other cross-frame state); one
  // host thread per device submits and collects, and the results are
  // appended in frame order into the same containers.  Empty: {device}.
  // The whole-video BB pass runs on the first device.  A device listed twice
  // is refused unless `oversubscribe` (rehearsals on fewer GPUs).
  std::vector<int> devices;
  bool oversubscribe = false;
  // Whole-video BB pass (use_provided_bounding_box = 0): config.yml's
  // median_filter_size / min_pixel_visible / moving_average_window /
  // conn_comp_connectivity, and V.set(CV_CAP_PROP_POS_FRAMES, 0) (:761-762)
  // to re-read the video from frame 0 after the pass.
  lm_bb_params bb_params{11, 1, 5, 8, LM_BB_FIRSTLAST_AS_EXECUTED, 46, 760, 100, 149, 400, 150, 0};
  std::function<void()> rewind;
  // exportResults writes <output_file> (the reference's
  // <outdir>/output_<stem>.yml, :360) when non-empty.
  std::string output_file;
  // config.yml's verbose_debug (LM_DEBUG, :17-19): a text log of the stages
  // (DEBUG_TEXT, opened at :341-343) into debug_text, and exportResults'
  // exportDebugVariables (:2769-2920) into debug_file — the reference's
  // <outdir>/debug_<stem>.txt / .yml (:361-362).  Empty paths: not written.
  bool verbose_debug = false;
  std::string debug_file, debug_text;
};

class LocoMouse : protected FrameResults {
 public:
  explicit LocoMouse(const LocoMouse_Inputs& inputs);
  virtual ~LocoMouse();
  LocoMouse(const LocoMouse&) = delete;
  LocoMouse& operator=(const LocoMouse&) = delete;

  virtual void readFrame();           // LocoMouse_class.cpp:1273-1333
  virtual void getBoundingBox();      // :543-653 (provided box: constant BR corners)
  virtual void computeBoundingBox();  // :575-653 — whole-video pass (lm_bb_*), §8(f) row 1
  void initializeFeatureLoop();       // :655-769 (creates the device context)
  void cropBoundingBox();             // :1408-1478
  void detectTail();                  // :2541-2555
  void detectBottomCandidates();      // :771-807
  void computeUnaryCostsBottom();     // :873-894
  void computePairwiseCostsBottom();  // :896-919
  void detectSideCandidates();        // :809-838
  void matchBottomSideCandidates();   // :999-1021
  void storePreviousImage();          // :1508-1513
  // After the per-frame loop (main.cpp:86-91; SURVEY.md §8(f) row 3, host C++):
  void computeBottomTracks();         // :2153-2200 (match2nd, 4 paw orders + snout)
  void computeSideTracks();           // :2202-2214 (bestSideViewMatch)
  void exportResults();               // :2348-2482 (track export; YAML when output_file is set)
  void exportDebugVariables();        // :2769-2920 (debug_<stem>.yml; called by exportResults when verbose_debug)
  unsigned int N_frames() const { return N_FRAMES; }

  // The reference's protected result vectors (LocoMouse_class.hpp:219-236),
  // one entry per processed frame, in frame order.
  const std::vector<std::vector<Candidate>>& candidates_bottom_paw();
  const std::vector<std::vector<Candidate>>& candidates_bottom_snout();
  const std::vector<std::vector<Candidate>>& candidates_side_paw();
  const std::vector<std::vector<Candidate>>& candidates_side_snout();
  const std::vector<std::vector<P22D>>& candidates_matched_views_paw();
  const std::vector<std::vector<P22D>>& candidates_matched_views_snout();
  const std::vector<MyMat>& unary_bottom_paw();
  const std::vector<MyMat>& unary_bottom_snout();
  const std::vector<MATSPARSE>& pairwise_bottom_paw();  // frames >= 1 only (:896-919)
  const std::vector<MATSPARSE>& pairwise_bottom_snout();
  const std::vector<TailTrack>& tracks_tail();
  const TrackResults& tracks() const { return TRACKS; }  // TRACK_INDEX_* and the exported matrices
  int current_frame() const { return CURRENT_FRAME; }
  lm_geometry geometry() const;

  // Processes the frames read so far (called by every accessor above).
  void sync();

  // Wall seconds the caller's thread spent handing batches to the device
  // (lm_detect_submit: the pinned staging copy and the H2D issue, or the
  // queue to a device thread) and waiting for results (lm_detect_collect, or
  // a device thread's chunk), and the batches handed over.  Not in the
  // reference: the LocoMouse program prints them under LM_TIMING.
  struct StageTimes {
    double submit_s = 0, wait_s = 0;
    int batches = 0;
  };
  StageTimes stage_times() const { return TIMES; }

 protected:
  LocoMouse_Inputs IN;
  int METHOD = 0;
  unsigned int N_FRAMES = 0;
  int CURRENT_FRAME = -1;
  std::vector<uint32_t> BB_X_POS, BB_Y_SIDE_POS, BB_Y_BOTTOM_POS;  // per-frame BR corners (:547-557)
  lm_rect BB_SIDE_MOUSE{}, BB_BOTTOM_MOUSE{};                       // box sizes (x = y = 0)
  bool HAVE_BB = false;

 public:
  const std::vector<uint32_t>& bb_x_pos() const { return BB_X_POS; }
  const std::vector<uint32_t>& bb_y_side_pos() const { return BB_Y_SIDE_POS; }
  const std::vector<uint32_t>& bb_y_bottom_pos() const { return BB_Y_BOTTOM_POS; }
  lm_rect bb_side_mouse() const { return BB_SIDE_MOUSE; }
  lm_rect bb_bottom_mouse() const { return BB_BOTTOM_MOUSE; }

 protected:
  // The result vectors (CANDIDATES_*, UNARY_*, PAIRWISE_*, TRACKS_TAIL) are
  // the FrameResults members; the tracks below are computed from them.
  TrackResults TRACKS;
  TrackSetup track_setup();

 private:
  lm_ctx* CTX = nullptr;  // the (first) device's context
  struct DevicePool;      // per-device contexts and host threads of a multi-GPU run
  std::unique_ptr<DevicePool> POOL;
  std::vector<uint8_t> LAST_FRAME;  // multi-GPU: the last raw frame handed over, the next shard's halo
 protected:
  void runBoundingBoxPass(int method);  // lm_bb_* over the whole video, then rewind
 private:
  // Page-locked (lm_host_alloc) batch buffers: DMA host->device copies.
  struct HostBuffer {
    uint8_t* p = nullptr;
    HostBuffer() = default;
    HostBuffer(const HostBuffer&) = delete;
    HostBuffer& operator=(const HostBuffer&) = delete;
    ~HostBuffer() { lm_host_free(p); }
    void allocate(size_t bytes);
    uint8_t* data() { return p; }
    void swap(HostBuffer& o) { std::swap(p, o.p); }
  };
  std::ofstream DEBUG_TEXT;  // verbose_debug log (LocoMouse_class.hpp:180)
  void debug_frames(int first, int n);  // the per-frame stage lines of frames [first, first + n)
  HostBuffer PENDING;    // raw frames read but not yet submitted
  std::deque<std::pair<int, int>> INFLIGHT;  // (first frame, n) of the submitted batches, oldest first
  int N_PENDING = 0;
  int N_READ_AHEAD = 0;  // frames of PENDING already filled by read_frames
  size_t FRAME_BYTES = 0;
  void flush();
  void collect_oldest();
  StageTimes TIMES;
};

// LocoMouse_TM (LocoMouse_TM.hpp:30-55): readFrame adds imadjust
// (TM.cpp:243-249), applied on the device for method 1.
class LocoMouse_TM : public LocoMouse {
 public:
  explicit LocoMouse_TM(const LocoMouse_Inputs& inputs);
  void readFrame() override;
  void computeBoundingBox() override;  // TM.cpp:115-241 — §8(f) row 1 (lm_bb_*, method 1)
};

// LocoMouse_TM_DE (LocoMouse_TM_DE.hpp:30-45): the same readFrame as TM.
class LocoMouse_TM_DE : public LocoMouse {
 public:
  explicit LocoMouse_TM_DE(const LocoMouse_Inputs& inputs);
  void readFrame() override;
  void computeBoundingBox() override;  // TM_DE.cpp:8-113 — §8(f) row 1 (lm_bb_*, method 2)
};

// LocoMouse_Methods.cpp:3-26: 0 LocoMouse, 1 LocoMouse_TM, 2 LocoMouse_TM_DE,
// anything else prints a notice and uses LocoMouse.
std::unique_ptr<LocoMouse> LocoMouse_Initialize(const LocoMouse_Inputs& inputs);

// lm_status -> the reference's exception types (main.cpp:94-101).
void throw_on_error(lm_status s);

// cv::Rect's operator<<: "[w x h from (x, y)]" (debug log lines).
std::string debug_rect(const lm_rect& r);

}  // namespace locomouse

#ifndef LOCOMOUSE_NO_GLOBAL_NAMES
using locomouse::LocoMouse;
using locomouse::LocoMouse_Initialize;
using locomouse::LocoMouse_Inputs;
using locomouse::LocoMouse_TM;
using locomouse::LocoMouse_TM_DE;
#endif

#endif
