// lm_runtime.hip — host runtime behind include/locomouse_hip.h.
//
// Owns the device state of one LocoMouse context: setup validation and
// geometry (LocoMouse::LocoMouse :307-345, validateImageVideoSize :486-540,
// initializeFeatureLoop :655-769, LocoMouse_Model :3095-3179), the per-batch
// buffers, the kernel chain of lm_kernels.hip and the assembly of results
// into the reference's container layout (Candidate / P22D / MyMat /
// MATSPARSE, in frame order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <numeric>
#include <atomic>
#include <deque>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "locomouse_hip.h"
#include "lm_host.h"
#include "lm_kernels.hip"

namespace {

// LDS window of one k_corr_gen workgroup (row chunks are sized to fit it)
constexpr size_t kCorrLdsBudget = 64 * 1024;
constexpr size_t kF16LdsMax = 160 * 1024;  // one k_corr_f16 workgroup per CU at most

struct Rect {
  int x = 0, y = 0, w = 0, h = 0;
};

int ceil_half(int v) { return (int)std::ceil((double)v / 2); }

struct Arena {
  // k_post's per-(frame, feature) outputs, bump-allocated (unordered)
  DevBuf<LmP22D> p22d;
  DevBuf<int32_t> side_y;
  DevBuf<double> side_s;
  DevBuf<double> unary;
  DevBuf<int32_t> jc, ir;
  DevBuf<double> pr;
  DevBuf<LmSlotOut> hdr;
  DevBuf<LmArenaCtl> ctl;
  // packed results (lm_batch_result layout), its header and side-array bases
  DevBuf<uint8_t> pack;
  DevBuf<LmPackHdr> ph;
  DevBuf<int64_t> side_base;
  int64_t pack_cap = 0;
  int cap[AR_COUNT] = {0};
  void alloc(const int* c, int nslots) {
    for (int k = 0; k < AR_COUNT; ++k) cap[k] = c[k];
    p22d.alloc(cap[AR_P22D]);
    side_y.alloc(cap[AR_SIDE]);
    side_s.alloc(cap[AR_SIDE]);
    unary.alloc(cap[AR_UNARY]);
    jc.alloc(cap[AR_PWJC]);
    ir.alloc(cap[AR_PWNZ]);
    pr.alloc(cap[AR_PWNZ]);
    if (!hdr.p) hdr.alloc(nslots);
    if (!ctl.p) ctl.alloc(1);
    if (!ph.p) ph.alloc(1);
    if (!side_base.p) side_base.alloc(2 * (size_t)nslots + 1);
    const int64_t tot[PK_COUNT] = {cap[AR_CAND], cap[AR_P22D], cap[AR_SIDE], cap[AR_UNARY], cap[AR_PWJC], cap[AR_PWNZ]};
    alloc_pack(lm_pack_layout(nslots, tot).bytes);
  }
  void alloc_pack(int64_t bytes) {
    if (bytes <= pack_cap) return;
    pack.alloc((size_t)bytes);
    pack_cap = bytes;
  }
};

// One batch in flight: its HIP stream, the per-batch device buffers and the
// packed results of its last batch.  A context owns `lanes` of them and
// submits consecutive batches round-robin, so several batches of one video
// run concurrently (batch k + 1's correlation overlaps batch k's post-
// correlation kernels); see submit_batch.
struct Lane {
  int index = 0;
  int device = 0;
  hipStream_t stream = nullptr;
  DevBuf<uint8_t> frames, halo, luts, ext, tailbin;
  DevBuf<unsigned long long> tailmask;  // TAIL_MASK bitmaps, 64 columns per word
  DevBuf<int32_t> npos, err;
  DevBuf<unsigned> mm;        // k_minmax partial (min, max) pairs per slot
  DevBuf<unsigned> tscratch;  // k_tail run tables beyond its LDS
  DevBuf<uint8_t> tail_ws;    // k_tail<true>: per-slot workspace (tail boxes beyond the LDS)
  DevBuf<float> dbg;
  DevBuf<int64_t> dbg_offd;
  DevBuf<const uint8_t*> frame_ptr;
  DevBuf<LmSlot> slots;
  DevBuf<unsigned long long> keys, gscratch;
  // k_ingest's source map (k_srcmap) for the crop position skey_h (per view)
  DevBuf<int2> smap;
  DevBuf<uint4> sbkg;
  DevBuf<int32_t> skey;
  int skey_h[4] = {-1, -1, -1, -1};
  DevBuf<uint8_t> dark_flags;  // dark tiles (CorrDark): flag bytes, bright-tile lists and counts
  DevBuf<uint32_t> dark_list;
  DevBuf<int32_t> dark_cnt;
  HostBuf<int32_t> h_cnt;   // debug bit 1: dark_cnt of the submitted batch, copied on its stream
  bool h_cnt_valid = false;
  DevBuf<long long> kprof;  // LM_KPROF=1: kernel phase timestamps
  DevBuf<long long> kprof_ing;  // LM_KPROF=1: k_ingest's, 16 per workgroup
  Arena arena[2];
  int parity = 0;
  // host
  HostBuf<LmSlot> h_slots;
  HostBuf<const uint8_t*> h_frame_ptr;
  HostBuf<LmArenaCtl> h_ctl;
  HostBuf<int32_t> h_err;
  HostBuf<LmPackHdr> h_ph;
  DevBuf<LmPackHdr> zero_ph;
  // this lane's last batch: the state a batch continuing it on this lane carries over
  bool have_state = false;
  int last_frame = -1, last_n = 0, last_parity = 0;
  // the submitted batch (collected by finish_batch)
  struct Pending {
    bool on = false;
    int n = 0, first = 0, s_lut0 = 1, s_proc0 = 1, plan = 0, cur = 0, prv = 0, last_n = 0;
    int pack = -1;  // the context's result buffer the batch's k_out writes
    bool carry = false;
  } pend;
  int64_t seq = -1;               // submission number of the batch running on this lane (-1: idle)
  int64_t done_seq = -1;          // submission number of the last batch finished here (its debug data)
  int batch_n = 0, batch_s0 = 1;  // last finished batch
  // pipelined halos: the batch's last frame copied to the context's handoff
  // buffer / the predecessor's handoff frame copied into this lane's halo
  hipEvent_t ev_snap = nullptr, ev_consumed = nullptr;
  // recorded after the batch's kernels (blocking sync): acquire_lane waits on
  // it without burning a host core
  hipEvent_t ev_done = nullptr;
  // timing (debug bit 1): events around k_corr on this lane's stream
  std::vector<std::pair<const char*, int>> t_ev;  // (kernel, index of its begin event in ev_pool)
  std::vector<const char*> t_names;               // static kernel names
  std::vector<double> t_ms, t_t0, t_t1;
  int32_t t_work[4] = {-1, -1, -1, -1};  // debug bit 1: dark-tile counts of the batch (lm_debug_corr_work)
  std::vector<hipEvent_t> ev_pool;
  // captured per-batch kernel chains, keyed by (n, parity, carry, last n, s_lut0, s_proc0, plan)
  struct GraphEntry {
    hipGraphExec_t exec[3];  // kernels before k_corr, k_corr, after
  };
  std::map<std::array<int, 7>, GraphEntry> graphs;
  bool use_graphs = true;
  void drop_graphs() {
    for (auto& g : graphs)
      for (hipGraphExec_t x : g.second.exec)
        if (x) (void)hipGraphExecDestroy(x);
    graphs.clear();
  }
  ~Lane() {
    drop_graphs();
    if (stream) {
      (void)hipSetDevice(device);
      (void)hipStreamSynchronize(stream);
      for (hipEvent_t e : ev_pool) (void)hipEventDestroy(e);
      if (ev_snap) (void)hipEventDestroy(ev_snap);
      if (ev_consumed) (void)hipEventDestroy(ev_consumed);
      if (ev_done) (void)hipEventDestroy(ev_done);
      (void)hipStreamDestroy(stream);
    }
  }
};

}  // namespace

struct lm_ctx {
  int device = 0;
  int max_batch = 0, nslots = 0;
  int debug = 0;
  lm_setup setup{};
  lm_params params{};
  lm_geometry geo{};
  LmConst K{};
  int npix = 0;
  int64_t fstride = 0;                 // device frame pitch of the staging slots
  int bb_x = 0, bb_yb = 0, bb_ys = 0;  // provided-box bottom-right corners
  int spost_b_w = 0, spost_b_h = 0, spost_t_w = 0, spost_t_h = 0;
  int64_t ext_slot_bytes = 0, tailbin_slot_bytes = 0, dbg_slot_floats = 0;
  int64_t dbg_off[LM_NDET] = {0};
  int64_t gscratch_slot = 0;
  bool unfused = false;                                         // LM_FILTER_UNFUSED
  // The correlation launches of a batch, two plans: [0] one k_corr_rw launch
  // per detector width, [1] every ring detector in one k_corr_rw_all launch
  // (see corr_plan_for)
  struct CorrPlan {
    std::vector<std::pair<const void*, LmDetGroup>> groups;  // (correlation kernel, its detectors)
    std::vector<size_t> lds;                                 // dynamic LDS bytes per group launch
    std::vector<int> threads;                                // block size per group launch
    std::vector<char> ring;                                  // group runs k_corr_rw* (one wave per tile)
  } corr_plan[2];
  // frame-invariant device data
  DevBuf<uint8_t> bkg, adj;
  DevBuf<int32_t> cal;
  DevBuf<float> weights;
  DevBuf<_Float16> weights16;  // LM_CORR_F16 rows (LmDet::w16_off)
  DevBuf<LmConst> dK;  // the per-context constants, passed to every kernel by pointer
  size_t tail_lds = 0;
  bool tail_big = false;        // k_tail<true>: tail tables in global memory
  int64_t tail_ws_slot = 0;     // its workspace bytes per slot
  bool kprof_on = false;
  bool dark_on = true;  // skip the point detectors' dark tiles (LM_CORR_DARK=0: compute every tile)
  // pipeline
  std::vector<std::unique_ptr<Lane>> lanes;
  DevBuf<uint8_t> handoff;     // two frames: the last frame of submitted batch k in slot k & 1
  // Pinned result buffers.  Each submitted batch takes a free one (k_out
  // writes its packed results there; the address reaches the captured graph
  // through the lane's control block), which then backs its lm_batch_result
  // until the next lm_detect_* call after its collection -- no copy when a
  // batch is retired from its lane early (a 1.2 MB copy per C3 batch made the
  // single host thread of a pipelined context the bottleneck).
  std::vector<std::unique_ptr<HostBuf<uint8_t>>> packs;
  std::vector<char> pack_busy;
  int take_pack(size_t cap) {
    size_t i = 0;
    while (i < packs.size() && pack_busy[i]) ++i;
    if (i == packs.size()) {
      packs.emplace_back(new HostBuf<uint8_t>());
      pack_busy.push_back(0);
    }
    if (packs[i]->n < cap) packs[i]->alloc(cap);
    pack_busy[i] = 1;
    return (int)i;
  }
  void drop_pack(int i) {
    if (i >= 0 && i < (int)pack_busy.size()) pack_busy[i] = 0;
  }
  // Submitted batches not yet returned by lm_detect_collect, in submission
  // order.  A batch runs on a lane until it is finished: when it is
  // collected, or earlier when a submission needs its lane ("retired": its
  // results stay in its buffer), so a lane that finishes early is fed again
  // at once while results still come back in frame order.
  struct BatchRec {
    int64_t seq = 0;
    int lane = -1;      // running there; -1 once retired
    int ran_lane = -1;  // the lane it ran on (its debug score maps / tail mask stay there until reused)
    int first = 0, n = 0;
    int slots = 0;      // frame slots processed: n, or n + 1 when the halo frame was recomputed
    lm_status status = LM_OK;  // a failure found while retiring, reported when collected
    std::string err;
    int pack = -1;  // its pinned result buffer (lm_batch_result layout), lm_ctx::packs
    LmPackHdr ph{};
    std::vector<const char*> t_names;  // kernel timings (debug bit 1)
    std::vector<double> t_ms, t_t0, t_t1;
    int32_t work[4] = {-1, -1, -1, -1};
  };
  std::deque<BatchRec> queue;
  BatchRec delivered;          // the last collected batch (its arrays back the returned pointers)
  int last_lane = -1;
  int64_t nsub = 0;            // batches submitted
  // the video position after the last submitted batch
  bool have_state = false;
  int last_frame = -1;
  int last_bb[3] = {0, 0, 0};  // bottom-right corners of frame last_frame
};

namespace {

void validate_and_build(lm_ctx* c, const lm_setup* su, const lm_params* P, const lm_model* M) {
  if (!su || !P || !M) throw std::invalid_argument("null setup/params/model");
  // LocoMouse_Parameters (:33-249)
  if (P->conn_comp_connectivity != 4 && P->conn_comp_connectivity != 8)
    throw std::invalid_argument("Invalid configuration parameter: conn_comp_connectivity must be either 4 or 8.");
  if (P->side_bottom_min_overlap < 0 || P->side_bottom_min_overlap > 1)
    throw std::invalid_argument("Invalid configuration parameter: side_bottom_min_overlap must belong to [0,1].");
  if (P->max_displacement_bottom < 0 || P->max_displacement_side < 0 || P->occlusion_grid_spacing_pixels_side < 0 ||
      P->occlusion_grid_spacing_pixels_bottom < 0 || P->alpha_vel_bottom < 0 || P->alpha_vel_side < 0 ||
      P->pairwise_occluded_cost < 0)
    throw std::invalid_argument("Invalid configuration parameter: must be non-negative.");
  if (P->occlusion_grid_max_width < 0 || P->occlusion_grid_max_width > 1 || P->tail_sub_bounding_box < 0 ||
      P->tail_sub_bounding_box > 1)
    throw std::invalid_argument("Invalid configuration parameter: must belong to [0,1].");
  for (int k = 0; k < 5; ++k) {
    const lm_location_prior& q = P->location_prior[k];
    if (!(q.min_x < q.max_x) || !(q.min_y < q.max_y))
      throw std::invalid_argument("location_prior: CV_Assert(minx < maxx && miny < maxy)");
  }
  if (!P->use_provided_bounding_box)
    throw std::invalid_argument("use_provided_bounding_box = 0: run the whole-video BB pass (lm_bb_*) first and pass its boxes and corners.");
  if (P->use_reference_image_brightness)
    throw std::runtime_error(
        "use_reference_image_brightness: computeNormalizedCDF writes the reference CDF through an unallocated cv::Mat "
        "(LocoMouse_class.cpp:189, :3392-3405); the reference cannot start with this option.");
  if (P->transform_gray_values && !P->use_reference_image_brightness) {
    // LUT(I_BOTTOM_MOUSE, REF_CDF_GLT, I_BOTTOM_MOUSE) (:1445-1448): dst takes the table's depth
    if (P->gray_value_transformation_depth != LM_DEPTH_8U)
      throw std::runtime_error(
          "transform_gray_values: LUT with a non-8U table re-creates the bottom crop with the table's type; the mask "
          "threshold / Mat::setTo(0, mask) then asserts (LocoMouse_class.cpp:1448, :782, :849).");
    for (int i = 0; i < 256; ++i) {
      const float v = P->gray_value_transformation[i];
      if (!(v >= 0.f && v <= 255.f && v == std::floor(v)))
        throw std::invalid_argument("gray_value_transformation: a CV_8U table holds integers 0..255.");
    }
  }
  if (P->occlusion_grid_spacing_pixels_bottom <= 0) throw std::invalid_argument("occlusion_grid_spacing_pixels_bottom must be > 0.");
  // loaders / validateImageVideoSize
  if (!su->background || !su->ind_warp_mapping) throw std::invalid_argument("background / calibration missing.");
  if (su->video_rows <= 0 || su->video_cols <= 0 || su->calib_rows <= 0 || su->calib_cols <= 0)
    throw std::invalid_argument("empty video or calibration.");
  if (su->method < 0 || su->method > 2) throw std::invalid_argument("method must be 0, 1 or 2.");
  const int64_t nv = (int64_t)su->video_rows * su->video_cols;
  const int64_t nc = (int64_t)su->calib_rows * su->calib_cols;
  int32_t mn = INT32_MAX, mx = INT32_MIN;
  for (int64_t i = 0; i < nc; ++i) {
    mn = std::min(mn, su->ind_warp_mapping[i]);
    mx = std::max(mx, su->ind_warp_mapping[i]);
  }
  if (mn < 0 || mx >= nv) throw std::runtime_error("Calibration mapping indices out of range.");
  const int NR = su->calib_rows, NC = su->calib_cols;
  const lm_rect ub = P->bounding_box_bottom, us = P->bounding_box_side;
  if (ub.x < 0 || ub.y < 0 || ub.x + ub.width >= NC || ub.y + ub.height >= NR)
    throw std::runtime_error("Provided bounding box for the bottom view exceeds the image dimensions.");
  if (us.x < 0 || us.y < 0 || us.x + us.width >= NC || us.y + us.height >= NR)
    throw std::runtime_error("Provided bounding box for the side view exceeds the image dimensions.");
  if (ub.width <= 0 || ub.height <= 0 || us.width <= 0 || us.height <= 0)
    throw std::runtime_error("Empty mouse bounding box: cropBoundingBox / filter2D would work on an empty image.");
  // model (:3095-3162)
  const lm_detector* dets[6] = {&M->paw_bottom, &M->snout_bottom, &M->tail_bottom, &M->paw_side, &M->snout_side, &M->tail_side};
  const char* names[6] = {"modelPaw_bottom", "modelSnout_bottom", "modelTail_bottom", "modelPaw_side", "modelSnout_side", "modelTail_side"};
  for (int d = 0; d < 6; ++d) {
    if (!dets[d]->weights || dets[d]->rows <= 0 || dets[d]->cols <= 0)
      throw std::invalid_argument(std::string("Error: ") + names[d] + " cannot be empty.");
    // any size: k_corr_gen walks the taps in LDS-sized row chunks; one LDS row
    // of the 80-column tile window must still fit (a detector wider than ~40k)
    if ((size_t)(LM_TH + 1) * pk_stride(LM_TW + dets[d]->cols + LM_JC) * sizeof(float) > kCorrLdsBudget)
      throw std::invalid_argument(std::string(names[d]) + ": detector too wide for the correlation window.");
    if (su->corr_precision == LM_CORR_F16 &&
        (f16_nch(dets[d]->cols) > LM_F16_MAX_NCH || f16_lds_bytes(f16_nch(dets[d]->cols), dets[d]->rows) > kF16LdsMax))
      throw std::invalid_argument(std::string(names[d]) + ": detector too large for the f16 correlation (LM_CORR_F16).");
  }
  if (su->corr_precision != LM_CORR_FP32 && su->corr_precision != LM_CORR_F16)
    throw std::invalid_argument("corr_precision must be LM_CORR_FP32 or LM_CORR_F16.");

  c->setup = *su;
  c->params = *P;
  lm_geometry& g = c->geo;
  std::memset(&g, 0, sizeof(g));
  g.n_rows = NR;
  g.n_cols = NC;
  const int mts_c = std::max(M->paw_side.cols, M->snout_side.cols), mts_r = std::max(M->paw_side.rows, M->snout_side.rows);
  const int mtb_c = std::max(M->paw_bottom.cols, M->snout_bottom.cols), mtb_r = std::max(M->paw_bottom.rows, M->snout_bottom.rows);
  g.spre_t_w = ceil_half(mts_c - 1);
  g.spre_t_h = ceil_half(mts_r - 1);
  g.spre_b_w = ceil_half(mtb_c - 1);
  g.spre_b_h = ceil_half(mtb_r - 1);
  g.spost_t_w = (mts_c - 1) / 2;
  g.spost_t_h = (mts_r - 1) / 2;
  g.spost_b_w = g.spre_b_w;  // LocoMouse_Model move-assign: spost_b = other.size_pre_bottom() (:3173)
  g.spost_b_h = g.spre_b_h;
  g.bb_bottom_mouse = lm_rect{0, 0, ub.width, ub.height};
  g.bb_side_mouse = lm_rect{0, 0, us.width, us.height};
  g.pad_pre_rows = std::max({us.height, g.spre_t_h, g.spre_b_h});
  g.pad_post_rows = g.spost_b_h > g.spost_t_h ? g.spost_b_h : g.spost_t_h;
  g.pad_pre_cols = std::max({ub.width, g.spre_t_w, g.spre_b_w});
  g.pad_post_cols = g.spost_b_w > g.spost_t_w ? g.spost_b_w : g.spost_t_w;
  g.ipad_rows = g.pad_pre_rows + NR + g.pad_post_rows;
  g.ipad_cols = g.pad_pre_cols + NC + g.pad_post_cols;
  g.bb_bottom_mouse_pad = lm_rect{0, 0, g.spre_b_w + ub.width + g.spost_b_w, g.spre_b_h + ub.height + g.spost_b_h};
  g.bb_side_mouse_pad = lm_rect{0, 0, g.spre_t_w + us.width + g.spost_t_w, g.spre_t_h + us.height + g.spost_t_h};
  g.bb_unpad_mouse_bottom = lm_rect{g.spre_b_w, g.spre_b_h, ub.width, ub.height};
  g.bb_unpad_mouse_side = lm_rect{g.spre_t_w, g.spre_t_h, us.width, us.height};
  const int tw = (int)(unsigned)((int)(double)(ub.width) * P->tail_sub_bounding_box);
  g.tail_box_width = tw;
  g.bb_bottom_tail_pad = lm_rect{0, 0, tw + g.spre_b_w + g.spost_b_w, ub.height + g.spre_b_h + g.spost_b_h};
  g.bb_unpad_tail_bottom = lm_rect{g.spre_b_w, g.spre_b_h, tw, ub.height};
  g.bb_bottom_tail = lm_rect{0, 0, tw, ub.height};
  g.bb_side_tail_pad = lm_rect{0, 0, tw + g.spre_t_w + g.spost_t_w, us.height + g.spre_t_h + g.spost_t_h};
  g.bb_unpad_tail_side = lm_rect{g.spre_t_w, g.spre_t_h, tw, us.height};
  const int sp = P->occlusion_grid_spacing_pixels_bottom;
  g.ong_ny = (int)(unsigned)(((ub.height - sp) / sp) + 1);
  g.ong_nx = (int)(unsigned)(((P->occlusion_grid_max_width * ub.width) - sp) / sp + 1);
  g.ong_br_x = (double)(ub.width - 1 - sp / 2);
  g.ong_br_y = (double)(ub.height - 1 - sp / 2);
  const int sps = P->occlusion_grid_spacing_pixels_side;
  g.n_ong_side = sps > 0 ? (int)(unsigned)(((us.height - sps) / sps) + 1) : 0;
  g.ong_side_lowest = (int)(unsigned)(us.height - 1 - sps / 2);
  auto mrect = [](const lm_detector& d) {  // LocoMouse_Feature :2954-2969
    const int nw = (int)std::round((double)d.cols / 2), nh = (int)std::round((double)d.rows / 2);
    return lm_rect{-(nw / 2), -(nh / 2), nw, nh};
  };
  g.match_box_paw_bottom = mrect(M->paw_bottom);
  g.match_box_paw_side = mrect(M->paw_side);
  g.match_box_snout_bottom = mrect(M->snout_bottom);
  g.match_box_snout_side = mrect(M->snout_side);
  if (g.ong_nx <= 0 || g.ong_ny <= 0) throw std::invalid_argument("occlusion grid is empty for this bounding box.");
  if (tw <= 0) throw std::invalid_argument("tail box width is 0.");

  c->bb_x = ub.x + ub.width;  // getBoundingBox provided-box branch (:547-557)
  c->bb_ys = us.y + us.height;
  c->bb_yb = ub.y + ub.height;
  c->npix = (int)nv;

  // ---------------- kernel constants
  LmConst& K = c->K;
  std::memset(&K, 0, sizeof(K));
  const int view_of[6] = {0, 0, 0, 1, 1, 1};
  const int kind_of[6] = {0, 0, 1, 0, 0, 1};
  const int list_of[6] = {LIST_PAW_B, LIST_SNOUT_B, 0, LIST_PAW_S, LIST_SNOUT_S, 1};
  Rect out_rel[6];  // output region relative to the padded crop
  out_rel[DET_PAW_B] = out_rel[DET_SNOUT_B] = Rect{g.spre_b_w, g.spre_b_h, ub.width, ub.height};
  out_rel[DET_TAIL_B] = Rect{g.spre_b_w, g.spre_b_h, tw, ub.height};
  out_rel[DET_PAW_S] = out_rel[DET_SNOUT_S] = Rect{g.spre_t_w, g.spre_t_h, us.width, us.height};
  out_rel[DET_TAIL_S] = Rect{g.spre_t_w, g.spre_t_h, tw, us.height};
  int tile = 0, w_off = 0;
  int ey0[2] = {INT32_MAX, INT32_MAX}, ex0[2] = {INT32_MAX, INT32_MAX}, ey1[2] = {INT32_MIN, INT32_MIN},
      ex1[2] = {INT32_MIN, INT32_MIN};
  for (int d = 0; d < 6; ++d) {
    LmDet& D = K.det[d];
    const lm_detector& src = *dets[d];
    D.view = view_of[d];
    D.kind = kind_of[d];
    D.list = list_of[d];
    D.kh = src.rows;
    D.kw = src.cols;
    D.kwp = (src.cols + LM_JC - 1) / LM_JC * LM_JC;
    D.w_off = w_off;
    w_off += D.kh * D.kwp;
    D.delta = (float)(-src.bias);  // saturate_cast<float>(delta)
    D.oh = out_rel[d].h;
    D.ow = out_rel[d].w;
    const bool f16 = su->corr_precision == LM_CORR_F16;
    const bool ring = !f16 && corr_ring(D.kw) && D.kh >= 2;  // one-row detectors: k_corr_gen
    D.tile_w = f16 ? LM_F16_TW : LM_TW;
    D.tile_h = f16 ? LM_F16_TH : ring ? LM_RW_TH : LM_TH;
    D.tiles_x = (D.ow + D.tile_w - 1) / D.tile_w;
    D.tiles_y = (D.oh + D.tile_h - 1) / D.tile_h;
    D.tile_base = tile;
    tile += D.tiles_x * D.tiles_y;
    D.box_w = src.cols;
    D.box_h = src.rows;
    const int ay = src.rows / 2, ax = src.cols / 2;  // anchor Point(-1,-1)
    const int y0 = out_rel[d].y - ay, x0 = out_rel[d].x - ax;
    const int v = D.view;
    ey0[v] = std::min(ey0[v], y0);
    ex0[v] = std::min(ex0[v], x0);
    ey1[v] = std::max(ey1[v], y0 + D.tiles_y * D.tile_h + D.kh - 1);
    const int win_w = f16 ? f16_cols(f16_nch(D.kw)) : LM_TW + D.kwp - 1 + 4;  // columns a tile's window reads
    ex1[v] = std::max(ex1[v], x0 + (D.tiles_x - 1) * D.tile_w + win_w);
    D.in_y = y0;  // rebased below
    D.in_x = x0;
    D.m_y = out_rel[d].y;
    D.m_x = out_rel[d].x;
  }
  K.n_tiles = tile;
  // LM_RW_WIDEN=1: a ring detector whose zero-padded row (kwp) reaches the
  // width of another ring detector of the context runs on that width's
  // kernel: the extra taps have weight 0 and add +0 (bit-identical, the ext
  // crops already hold kwp columns), and one launch per batch fewer ends in
  // its own tail (C3: paw side 22 -> 24 with paw bottom).  Measured with four
  // contexts: 466.9k vs 470.0k frames/s without (profiles/r04/widen/) -- the
  // other contexts fill the tails anyway -- so off by default.
  {
    static const bool widen = [] {
      const char* v = getenv("LM_RW_WIDEN");
      return v && atoi(v) != 0;
    }();
    for (int d = 0; d < 6; ++d) {
      LmDet& D = K.det[d];
      D.kw_ring = D.kw;
      if (!widen || !corr_ring(D.kw) || D.kh < 2) continue;
      for (int e = 0; e < 6; ++e) {
        const int w = K.det[e].kw;
        if (e != d && corr_ring(w) && w > D.kw && w <= D.kwp && (D.kw_ring == D.kw || w < D.kw_ring)) D.kw_ring = w;
      }
    }
  }
  for (int v = 0; v < 2; ++v) {
    K.ext_oy[v] = ey0[v];
    K.ext_ox[v] = ex0[v];
    K.ext_h[v] = ey1[v] - ey0[v];
    K.ext_w[v] = ((ex1[v] - ex0[v]) + 15) / 16 * 16;
  }
  for (int d = 0; d < 6; ++d) {
    LmDet& D = K.det[d];
    D.in_y -= K.ext_oy[D.view];
    D.in_x -= K.ext_ox[D.view];
    D.m_y -= K.ext_oy[D.view];
    D.m_x -= K.ext_ox[D.view];
  }
  K.crop_h[0] = g.bb_bottom_mouse_pad.height;
  K.crop_w[0] = g.bb_bottom_mouse_pad.width;
  K.crop_h[1] = g.bb_side_mouse_pad.height;
  K.crop_w[1] = g.bb_side_mouse_pad.width;
  K.unpad_y[0] = g.spre_b_h;
  K.unpad_x[0] = g.spre_b_w;
  K.unpad_y[1] = g.spre_t_h;
  K.unpad_x[1] = g.spre_t_w;
  K.video_rows = su->video_rows;
  K.video_cols = su->video_cols;
  K.n_rows = NR;
  K.n_cols = NC;
  K.pad_pre_rows = g.pad_pre_rows;
  K.pad_pre_cols = g.pad_pre_cols;
  K.ipad_rows = g.ipad_rows;
  K.ipad_cols = g.ipad_cols;
  K.flip = su->flip ? 1 : 0;
  K.tail_w = tw;
  K.tail_hb = ub.height;
  K.tail_hs = us.height;
  K.connectivity = P->conn_comp_connectivity;
  // dark-tile flags of the point detectors' outputs (paw and snout of a view
  // share the output region, out_rel above)
  {
    int o = 0;
    for (int v = 0; v < 2; ++v) {
      const LmDet& D = K.det[v ? DET_PAW_S : DET_PAW_B];
      K.fl_tx[v] = (D.ow + LM_FW - 1) / LM_FW;
      K.fl_ty[v] = (D.oh + LM_FH - 1) / LM_FH;
      K.fl_off[v] = o;
      o += (K.fl_tx[v] * K.fl_ty[v] + 3) / 4 * 4;
    }
    K.fl_slot = o;
    K.tl_stride = c->nslots * std::max(K.fl_tx[0] * K.fl_ty[0], K.fl_tx[1] * K.fl_ty[1]);
    if (K.fl_tx[0] * K.fl_ty[0] > 65535 || K.fl_tx[1] * K.fl_ty[1] > 65535 || c->nslots > 65535 ||
        std::max(K.fl_tx[0], K.fl_tx[1]) > LM_INGEST_MAXTX)
      throw std::invalid_argument("bounding box or batch too large for the correlation tile lists.");
    // k_ingest's bands: 8 ext rows each, aligned with the flag grid's rows
    int maxcw = 0;
    for (int v = 0; v < 2; ++v) {
      const LmDet& D = K.det[v ? DET_PAW_S : DET_PAW_B];
      K.fl_my[v] = D.m_y;
      K.fl_mx[v] = D.m_x;
      K.fl_oh[v] = D.oh;
      K.fl_ow[v] = D.ow;
      const int above = (D.m_y + 7) / 8;  // bands above the output rows (m_y >= 0)
      K.ing_b0[v] = -above;
      K.ing_nb[v] = above + (K.ext_h[v] - D.m_y + 7) / 8;
      maxcw = std::max(maxcw, K.ext_w[v] / LM_INGEST_VEC);
    }
    K.ing_threads = std::min(1024, (8 * maxcw + 63) / 64 * 64);
  }
  // k_tail's LDS: bitmaps, column tables and moment tiles from the geometry,
  // plus as many runs as fit 64 KiB (more go to global scratch)
  K.tail_ntc = (((tw - 1) / 15 + 1) + 31) / 32;
  K.tail_cap = 4096;
  while (K.tail_cap > 64 && tail_layout(tw, ub.height, us.height, K.tail_cap, K.tail_ntc).bytes > 64 * 1024) K.tail_cap -= 64;
  c->tail_lds = (size_t)tail_layout(tw, ub.height, us.height, K.tail_cap, K.tail_ntc).bytes;
  // a tail box whose bitmaps do not fit the LDS runs k_tail<true> on a
  // global per-slot workspace instead
  c->tail_big = c->tail_lds > 160 * 1024;
  if (c->tail_big) {
    K.tail_cap = 0;
    c->tail_lds = 0;
    c->tail_ws_slot = ((int64_t)tail_layout(tw, ub.height, us.height, 0, K.tail_ntc).bytes + 255) / 256 * 256;
  }
  int64_t off = 0;
  for (int l = 0; l < LM_NLIST; ++l) {
    const int d = l == 0 ? DET_PAW_B : l == 1 ? DET_SNOUT_B : l == 2 ? DET_PAW_S : DET_SNOUT_S;
    K.list_cap[l] = K.det[d].oh * K.det[d].ow;
    K.list_off[l] = off;
    off += K.list_cap[l];
  }
  K.keys_per_slot = off;
  K.side_bottom_min_overlap = P->side_bottom_min_overlap;
  K.alpha_vel_bottom = P->alpha_vel_bottom;
  K.pairwise_occluded_cost = P->pairwise_occluded_cost;
  K.max_displacement_bottom = P->max_displacement_bottom;
  K.ong_spacing_bottom = sp;
  K.ong_nx = g.ong_nx;
  K.ong_ny = g.ong_ny;
  K.ong_br_x = g.ong_br_x;
  K.ong_br_y = g.ong_br_y;
  K.bb_bottom_w = ub.width;
  K.bb_bottom_h = ub.height;
  K.spre_b_w = g.spre_b_w;
  K.spre_b_h = g.spre_b_h;
  K.spre_t_w = g.spre_t_w;
  K.spre_t_h = g.spre_t_h;
  const lm_rect mb[2] = {g.match_box_paw_bottom, g.match_box_snout_bottom};
  const lm_rect ms[2] = {g.match_box_paw_side, g.match_box_snout_side};
  for (int f = 0; f < 2; ++f) {
    K.match_b[f][0] = mb[f].x;
    K.match_b[f][1] = mb[f].y;
    K.match_b[f][2] = mb[f].width;
    K.match_b[f][3] = mb[f].height;
    K.match_s[f][0] = ms[f].x;
    K.match_s[f][1] = ms[f].y;
    K.match_s[f][2] = ms[f].width;
    K.match_s[f][3] = ms[f].height;
    const lm_detector& db = f == 0 ? M->paw_bottom : M->snout_bottom;
    const lm_detector& ds = f == 0 ? M->paw_side : M->snout_side;
    K.size_b[f][0] = db.cols;
    K.size_b[f][1] = db.rows;
    K.size_s[f][0] = ds.cols;
    K.size_s[f][1] = ds.rows;
  }
  for (int k = 0; k < 5; ++k) {
    const lm_location_prior& q = P->location_prior[k];
    const double row[7] = {q.x, q.y, q.max_distance, q.min_x, q.max_x, q.min_y, q.max_y};
    for (int j = 0; j < 7; ++j) K.prior[k][j] = row[j];
  }
  K.gray_lut_on = P->transform_gray_values && !P->use_reference_image_brightness ? 1 : 0;
  for (int i = 0; i < 256; ++i) K.gray_lut[i] = K.gray_lut_on ? (uint8_t)P->gray_value_transformation[i] : (uint8_t)i;

  // per-slot sizes
  c->ext_slot_bytes = ((int64_t)K.ext_h[0] * K.ext_w[0] + (int64_t)K.ext_h[1] * K.ext_w[1] + 255) / 256 * 256;
  K.tail_nw = 2 * ((K.tail_w + 63) / 64);
  K.tail_bm_words = (K.tail_hb + K.tail_hs) * K.tail_nw;
  c->tailbin_slot_bytes = (int64_t)K.tail_bm_words * 4;
  int64_t doff = 0;
  for (int d = 0; d < 6; ++d) {
    c->dbg_off[d] = doff;
    doff += (int64_t)K.det[d].oh * K.det[d].ow;
  }
  c->dbg_slot_floats = doff;
  int np = 1;
  while (np < std::max(K.list_cap[0], K.list_cap[2])) np <<= 1;
  // one region per block of the global-scratch k_nms / k_post launches: k_nms's keys (u64) + assign, cluster list, xy (32-bit)
  // per entry; then reused by k_post for lists beyond its LDS capacity
  // (offsets np + Nong + 1, motion flags 2 np, counts 2 np: 32-bit each)
  c->gscratch_slot = std::max(3 * (int64_t)np, (5 * (int64_t)np + K.ong_nx * K.ong_ny + 2) / 2 + 1);
  c->unfused = su->filter_arith == LM_FILTER_UNFUSED;
  if (const char* v = getenv("LM_KPROF")) c->kprof_on = atoi(v) != 0;
  if (const char* v = getenv("LM_CORR_DARK")) c->dark_on = atoi(v) != 0;
  // Detectors grouped by correlation kernel: one width-specialised k_corr_rw
  // launch per width, every other detector in one k_corr_gen launch.  Each
  // launch gets exactly the LDS its detectors' rings / windows need, so narrow
  // groups keep more waves per CU.
  // ring detectors ordered longest waves ((kh + 2) x kw taps) first
  int order[6] = {0, 1, 2, 3, 4, 5};
  std::stable_sort(order, order + 6, [&](int x, int y) {
    return (int64_t)(K.det[x].kh + 2) * K.det[x].kw > (int64_t)(K.det[y].kh + 2) * K.det[y].kw;
  });
  for (int m = 0; m < 2; ++m) {
    lm_ctx::CorrPlan& P = c->corr_plan[m];
    P = lm_ctx::CorrPlan{};
    for (int oi = 0; oi < 6; ++oi) {
      const int d = order[oi];
      LmDet& D = K.det[d];
      const bool f16 = su->corr_precision == LM_CORR_F16;
      const bool ring = !f16 && corr_ring(D.kw_ring) && D.kh >= 2;
      // a detector that is not a ring detector (a width without an
      // instantiation, or one row at a ring width) runs k_corr_gen explicitly:
      // corr_kernel() picks by width alone
      const void* fn = f16     ? corr_kernel_f16(D.kw)
                       : !ring ? corr_kernel_gen(c->unfused)
                       : m == 1 && rw_all_width(D.kw_ring) ? corr_kernel_rw_all(c->unfused)
                                                           : corr_kernel(D.kw_ring, c->unfused);
      size_t need;
      if (f16) {
        D.chunk_rows = D.kh;
        need = f16_lds_bytes(f16_nch(D.kw), D.kh);
      } else if (ring) {
        D.chunk_rows = D.kh;
        need = corr_rw_lds(D.kw_ring);
      } else {
        const size_t row = (size_t)pk_stride(LM_TW + D.kwp - 1) * sizeof(float);
        D.chunk_rows = std::max(1, std::min(D.kh, (int)(kCorrLdsBudget / row) - (LM_TH - 1)));
        need = (size_t)(LM_TH + D.chunk_rows - 1) * row;
      }
      size_t gi = 0;
      while (gi < P.groups.size() && P.groups[gi].first != fn) ++gi;
      if (gi == P.groups.size()) {
        LmDetGroup G;
        std::memset(&G, 0, sizeof(G));
        P.groups.push_back({fn, G});
        P.lds.push_back(0);
        P.threads.push_back(f16 ? LM_F16_THREADS : ring ? LM_RW_THREADS : LM_CORR_THREADS);
        P.ring.push_back(ring);
      }
      LmDetGroup& G = P.groups[gi].second;
      const int prev = G.n ? G.tile_end[G.n - 1] : 0;
      G.ids[G.n] = d;
      G.tile_end[G.n] = prev + D.tiles_x * D.tiles_y;
      ++G.n;
      if (ring) G.ring_floats = std::max(G.ring_floats, rw_ring_floats(D.kw_ring));
      P.lds[gi] = std::max(P.lds[gi], need);
    }
  }

  // weights (float, rows zero-padded to kwp) and TM imadjust LUT
  std::vector<float> wts((size_t)w_off, 0.f);
  for (int d = 0; d < 6; ++d) {
    const LmDet& D = K.det[d];
    for (int i = 0; i < D.kh; ++i)
      for (int j = 0; j < D.kw; ++j) wts[(size_t)D.w_off + i * D.kwp + j] = (float)dets[d]->weights[(size_t)i * D.kw + j];
  }
  // LM_CORR_F16: each detector's B fragments (lm_corr.hip k_corr_f16) as f16,
  // scaled by 2^s so that the largest |w| lands in [2^14, 2^15) (the rounding
  // is then relative and no weight of interest is subnormal; 2^s and 2^-s
  // are exact in fp32)
  std::vector<_Float16> w16;
  if (su->corr_precision == LM_CORR_F16) {
    for (int d = 0; d < 6; ++d) {
      LmDet& D = K.det[d];
      const int nch = f16_nch(D.kw);
      double mx = 0;
      for (int k = 0; k < D.kh * D.kw; ++k) mx = std::max(mx, std::fabs(dets[d]->weights[k]));
      int e = 0;
      if (mx > 0) std::frexp(mx, &e);  // mx in [2^(e-1), 2^e)
      const int sc = mx > 0 ? 15 - e : 0;
      D.wscale = std::ldexp(1.0f, sc);
      D.inv_wscale = std::ldexp(1.0f, -sc);
      D.w16_off = (int32_t)(w16.size() / 8);  // in 16-byte fragments
      for (int i = 0; i < D.kh; ++i)
        for (int c = 0; c < nch; ++c)
          for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 8; ++j)
              w16.push_back((_Float16)std::ldexp(f16_bfrag_weight(dets[d]->weights, D.kw, i, c, l, j), sc));
    }
  }
  uint8_t adj[256];
  {
    // imadjust(I, I, 0, 0.6, 0, 1) (LocoMouse_class.cpp:3204-3242)
    double low_in = 0 * 255, high_in = 0.6 * 255, low_out = 0 * 255, high_out = 1 * 255.0;
    double range_in = high_in - low_in, range_out = high_out - low_out, range_div = range_out / range_in;
    for (int i = 0; i < 256; ++i) {
      double temp;
      if (i <= low_in) temp = 0;
      else if (i >= high_in) temp = range_out;
      else temp = (i - low_in) * (range_div);
      adj[i] = (uint8_t)std::round((temp + low_out));
    }
  }

  // ---------------- frame-invariant device data (create-time copies on a
  // temporary stream: see COPY_SYNC)
  hipStream_t cs = nullptr;
  HIPCHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamDestroy(s); }
  } cs_guard{cs};
  c->bkg.alloc(nv);
  COPY_SYNC(c->bkg.p, su->background, nv, hipMemcpyHostToDevice, cs);
  c->cal.alloc(nc);
  COPY_SYNC(c->cal.p, su->ind_warp_mapping, nc * sizeof(int32_t), hipMemcpyHostToDevice, cs);
  c->weights.alloc(wts.size());
  COPY_SYNC(c->weights.p, wts.data(), wts.size() * sizeof(float), hipMemcpyHostToDevice, cs);
  if (!w16.empty()) {
    c->weights16.alloc(w16.size());
    COPY_SYNC(c->weights16.p, w16.data(), w16.size() * sizeof(_Float16), hipMemcpyHostToDevice, cs);
  }
  c->adj.alloc(256);
  COPY_SYNC(c->adj.p, adj, 256, hipMemcpyHostToDevice, cs);
  c->dK.alloc(1);
  COPY_SYNC(c->dK.p, &c->K, sizeof(LmConst), hipMemcpyHostToDevice, cs);
  c->fstride = (nv + 255) / 256 * 256;
  HIPCHK(hipFuncSetAttribute((const void*)k_tail<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->tail_lds));
  for (const auto& P : c->corr_plan)
    for (size_t g = 0; g < P.groups.size(); ++g)
      HIPCHK(hipFuncSetAttribute(P.groups[g].first, hipFuncAttributeMaxDynamicSharedMemorySize, (int)P.lds[g]));
}


// The per-batch buffers of one lane (B = max_batch, slots 0..B).
void lane_alloc(lm_ctx* c, Lane& L) {
  const LmConst& K = c->K;
  const lm_geometry& g = c->geo;
  const int ns = c->nslots;
  const int64_t fstride = c->fstride;
  hipStream_t st = L.stream;
  L.frames.alloc((size_t)fstride * ns);
  L.halo.alloc(fstride);
  SET_SYNC(L.halo.p, 0, fstride, st);
  L.luts.alloc((size_t)256 * ns);
  L.mm.alloc((size_t)2 * LM_MM_SPLIT * ns);
  // slack: the last tiles' windows (and the fill's 16-byte rounding) read past
  // the last slot's side view; those pixels only feed outputs that are discarded
  L.ext.alloc((size_t)c->ext_slot_bytes * ns + (size_t)(LM_F16_TH + 16) * std::max(K.ext_w[0], K.ext_w[1]) + 64);
  L.tailbin.alloc((size_t)c->tailbin_slot_bytes * ns);
  SET_SYNC(L.tailbin.p, 0, (size_t)c->tailbin_slot_bytes * ns, st);
  L.tailmask.alloc((size_t)K.tail_hb * ((K.tail_w + 63) / 64) * ns);
  L.tscratch.alloc((size_t)5 * std::max(K.tail_hb, K.tail_hs) * ((K.tail_w + 1) / 2) * ns);
  if (c->tail_big) L.tail_ws.alloc((size_t)c->tail_ws_slot * ns);
  L.keys.alloc((size_t)K.keys_per_slot * ns);
  L.npos.alloc((size_t)LM_NLIST * ns);
  {
    const int64_t nchunks = ((int64_t)K.ext_h[0] * K.ext_w[0] + (int64_t)K.ext_h[1] * K.ext_w[1]) / LM_INGEST_VEC;
    L.smap.alloc((size_t)nchunks);
    L.sbkg.alloc((size_t)nchunks);
    L.skey.alloc(4);
    SET_SYNC(L.skey.p, 0x80, 4 * sizeof(int32_t), st);  // no position: every k_ingest locates until k_srcmap ran
  }
  if (c->dark_on) {
    L.dark_flags.alloc((size_t)K.fl_slot * ns);
    SET_SYNC(L.dark_flags.p, 0, (size_t)K.fl_slot * ns, st);
    L.dark_list.alloc((size_t)2 * K.tl_stride);
    L.dark_cnt.alloc(4 * LM_TL_NC);
    L.h_cnt.alloc(4 * LM_TL_NC);
  }
  L.err.alloc(16);
  L.frame_ptr.alloc(ns);
  L.slots.alloc(ns);
  L.h_slots.alloc(ns);
  L.h_frame_ptr.alloc(ns);
  L.h_ctl.alloc(1);
  L.h_ph.alloc(1);
  L.zero_ph.alloc(1);  // an all-zero pack header: k_out with it copies only the halo
  SET_SYNC(L.zero_ph.p, 0, sizeof(LmPackHdr), st);
  L.h_err.alloc(16);
  int cap[AR_COUNT];
  cap[AR_CAND] = ns * LM_NLIST * 64;
  cap[AR_P22D] = ns * LM_NFEAT * 64;
  cap[AR_SIDE] = ns * LM_NFEAT * 256;
  cap[AR_UNARY] = ns * LM_NFEAT * 64 * 4;
  cap[AR_PWJC] = ns * LM_NFEAT * (64 + g.ong_nx * g.ong_ny + 1);
  cap[AR_PWNZ] = ns * LM_NFEAT * (1024 + g.ong_nx * g.ong_ny);  // an ONG column holds at least its diagonal
  for (int a = 0; a < 2; ++a) L.arena[a].alloc(cap, ns);
  HIPCHK(hipEventCreateWithFlags(&L.ev_snap, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&L.ev_consumed, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&L.ev_done, hipEventDisableTiming | hipEventBlockingSync));
}

// One epoch event per device (recorded when timing is switched on) that every
// context's kernel spans are measured against.
std::mutex g_epoch_mu;
std::map<int, hipEvent_t> g_epoch;

hipEvent_t epoch_event(const lm_ctx* c) {
  std::lock_guard<std::mutex> lk(g_epoch_mu);
  auto it = g_epoch.find(c->device);
  return it == g_epoch.end() ? nullptr : it->second;
}


struct Timer {  // HIP events around the timed kernels of a lane's batch (debug bit 1)
  Lane& L;
  bool on;
  Timer(lm_ctx* c, Lane& l) : L(l), on(c->debug & 2) {}
  hipEvent_t pool(size_t i) {
    while (L.ev_pool.size() <= i) {
      hipEvent_t e;
      HIPCHK(hipEventCreate(&e));
      L.ev_pool.push_back(e);
    }
    return L.ev_pool[i];
  }
  bool capturing = false;  // inside a graph capture: a failed record aborts the capture, not the batch
  void record(hipEvent_t e) {
    const hipError_t r = hipEventRecord(e, L.stream);
    if (r != hipSuccess && !capturing) hip_check(r, "hipEventRecord");
  }
  void begin(const char* name) {
    if (!on) return;
    const int i = (int)L.t_ev.size() * 2;
    record(pool(i));
    L.t_ev.push_back({name, i});
  }
  void end() {
    if (!on) return;
    record(pool(L.t_ev.back().second + 1));
  }
  // Durations, plus start/end against the device's epoch event so callers can
  // take the union of one kernel's spans over several streams.
  static void collect(lm_ctx* c, Lane& L) {
    L.t_names.clear();
    L.t_ms.clear();
    L.t_t0.clear();
    L.t_t1.clear();
    const hipEvent_t ep = epoch_event(c);
    for (auto& e : L.t_ev) {
      float ms = 0, t0 = 0, t1 = 0;
      HIPCHK(hipEventElapsedTime(&ms, L.ev_pool[e.second], L.ev_pool[e.second + 1]));
      if (ep) {
        HIPCHK(hipEventElapsedTime(&t0, ep, L.ev_pool[e.second]));
        HIPCHK(hipEventElapsedTime(&t1, ep, L.ev_pool[e.second + 1]));
      }
      L.t_names.push_back(e.first);
      L.t_ms.push_back(ms);
      L.t_t0.push_back(t0);
      L.t_t1.push_back(t1);
    }
    L.t_ev.clear();
    for (int k = 0; k < 4; ++k) L.t_work[k] = -1;
    if (L.dark_cnt.p) {  // the segment counters summed per view
      // normally copied on the batch's stream when it was submitted (no
      // synchronous copy on the host's path); the timing was switched on
      // after that submit: copy now
      int32_t h[4 * LM_TL_NC];
      if (L.h_cnt_valid)
        std::copy(L.h_cnt.p, L.h_cnt.p + 4 * LM_TL_NC, h);
      else
        COPY_SYNC(h, L.dark_cnt.p, sizeof(h), hipMemcpyDeviceToHost, L.stream);
      for (int k = 0; k < 4; ++k) L.t_work[k] = std::accumulate(h + k * LM_TL_NC, h + (k + 1) * LM_TL_NC, 0);
    }
  }
};

// Batch streams per device (every lane of every live context).  With one
// stream on its device a batch runs the merged correlation plan (one
// k_corr_rw_all launch: the widths share one tail instead of ending four);
// with several, the per-width launches interleave better with the other
// streams' post-correlation kernels (4 streams: 340k vs 322k frames/s merged;
// profiles/r02/merged/).  LM_CORR_PLAN=0 / 1 or debug bits 4 / 5 force one.
std::atomic<int> g_live_streams[64];

int corr_plan_for(const lm_ctx* c) {
  static const int forced = [] {
    const char* v = getenv("LM_CORR_PLAN");
    return v ? atoi(v) : -1;
  }();
  if (forced == 0 || forced == 1) return forced;
  if (c->debug & 16) return 0;
  if (c->debug & 32) return 1;
  return g_live_streams[c->device & 63].load(std::memory_order_relaxed) <= 1 ? 1 : 0;
}

// LM_KPROF=1: mean cycles per k_nms / k_tail / k_post phase over the batch's blocks (stderr)
void kprof_report(lm_ctx* c, Lane& L, int n) {
  std::vector<long long> h((size_t)4 * 16 * 2 * c->nslots);
  COPY_SYNC(h.data(), L.kprof.p, h.size() * sizeof(long long), hipMemcpyDeviceToHost, L.stream);
  if (L.kprof_ing.p) {  // k_ingest: phases 1-4 per workgroup, start spread (launch rounds)
    const LmConst& K = c->K;
    const size_t nb = (size_t)(K.ing_nb[0] + K.ing_nb[1]) * ((c->nslots + LM_INGEST_FB - 1) / LM_INGEST_FB);
    std::vector<long long> g(16 * nb);
    COPY_SYNC(g.data(), L.kprof_ing.p, g.size() * sizeof(long long), hipMemcpyDeviceToHost, L.stream);
    double acc[8] = {0}, life = 0;
    int cntb = 0;
    long long t_min = 0, t_max = 0, s_max = 0;
    std::vector<long long> starts;
    for (size_t b = 0; b < nb; ++b) {
      const long long* t = g.data() + b * 16;
      if (!t[0] || !t[4]) continue;
      for (int k = 1; k <= 4; ++k) acc[k] += (double)(t[k] - t[k - 1]);
      life += (double)(t[4] - t[0]);
      t_min = t_min ? std::min(t_min, t[14]) : t[14];
      t_max = std::max(t_max, t[15]);
      starts.push_back(t[14]);
      ++cntb;
    }
    for (long long st0 : starts) s_max = std::max(s_max, st0 - t_min);
    std::sort(starts.begin(), starts.end());
    const double p50 = starts.empty() ? 0.0 : (starts[starts.size() / 2] - t_min) * 0.01;
    const double p90 = starts.empty() ? 0.0 : (starts[starts.size() * 9 / 10] - t_min) * 0.01;
    if (cntb) {
      fprintf(stderr, "kprof k_ingest: blocks=%d life=%.0f cyc, span=%.1f us, start p50 %.1f p90 %.1f last %.1f us:", cntb,
              life / cntb, (t_max - t_min) * 0.01, p50, p90, s_max * 0.01);
      for (int k = 1; k <= 4; ++k) fprintf(stderr, " p%d=%.0f", k, acc[k] / cntb);
      fprintf(stderr, "\n");
    }
  }
  {  // k_post (LDS instantiation): region 3, one block per (frame, feature)
    const long long* base = h.data() + (size_t)3 * 16 * 2 * c->nslots;
    double acc[8] = {0}, life = 0;
    int nb = 0;
    long long t_min = 0, t_max = 0, worst = 0;
    int wb = -1;
    for (int b = 0; b < 2 * n; ++b) {
      const long long* t0 = base + (size_t)b * 16;
      if (!t0[0] || !t0[6]) continue;
      // a phase a block skips (e.g. phase 2 of a feature without side
      // candidates) leaves its stamp at 0: it took no time (round 5 printed
      // p2 = 0 - t1 and p3 = t3 - 0 for such blocks)
      long long t[16];
      for (int k = 0; k < 16; ++k) t[k] = t0[k];
      for (int k = 1; k <= 6; ++k)
        if (!t[k]) t[k] = t[k - 1];
      for (int k = 1; k <= 6; ++k) acc[k] += (double)(t[k] - t[k - 1]);
      life += (double)(t[6] - t[0]);
      if (t[6] - t[0] > worst) {
        worst = t[6] - t[0];
        wb = b;
      }
      t_min = t_min ? std::min(t_min, t[14]) : t[14];
      t_max = std::max(t_max, t[15]);
      ++nb;
    }
    if (nb) {
      fprintf(stderr, "kprof k_post: blocks=%d life=%.0f cyc, span=%.1f us:", nb, life / nb, (t_max - t_min) * 0.01);
      for (int k = 1; k <= 6; ++k) fprintf(stderr, " p%d=%.0f", k, acc[k] / nb);
      long long t[16];
      for (int k = 0; k < 16; ++k) t[k] = base[(size_t)wb * 16 + k];
      for (int k = 1; k <= 6; ++k)
        if (!t[k]) t[k] = t[k - 1];
      fprintf(stderr, " | slowest blk %d cyc=%lld:", wb, worst);
      for (int k = 1; k <= 6; ++k) fprintf(stderr, " %lld", t[k] - t[k - 1]);
      fprintf(stderr, "\n");
    }
  }
  {  // k_tail: region 2, one block per processed slot
    const long long* base = h.data() + (size_t)2 * 16 * 2 * c->nslots;
    double acc[16] = {0}, life = 0, wlife = 0, runs = 0;
    int nb = 0;
    long long t_min = 0, t_max = 0;
    for (int b = 0; b < 2 * c->nslots; ++b) {
      const long long* t = base + (size_t)b * 16;
      if (!t[0] || !t[9]) continue;
      for (int k = 1; k <= 9; ++k) acc[k] += (double)(t[k] - t[k - 1]);
      life += (double)(t[9] - t[0]);
      wlife += (double)(t[15] - t[14]) * 0.01;
      runs += (double)t[13];
      t_min = t_min ? std::min(t_min, t[14]) : t[14];
      t_max = std::max(t_max, t[15]);
      ++nb;
    }
    if (nb) {
      fprintf(stderr, "kprof k_tail: blocks=%d life=%.0f cyc = %.1f us, span=%.1f us, side runs %.0f:", nb, life / nb,
              wlife / nb, (t_max - t_min) * 0.01, runs / nb);
      for (int k = 1; k <= 9; ++k) fprintf(stderr, " p%d=%.0f", k, acc[k] / nb);
      fprintf(stderr, "\n");
    }
  }
  for (int side = 0; side < 2; ++side) {
    double acc[16] = {0}, life = 0, wlife = 0;
    int cnt[16] = {0}, nb = 0;
    long long t_min = 0, t_max = 0;
    for (int b = 0; b < 2 * n; ++b) {
      const long long* t = h.data() + (size_t)side * 16 * 2 * c->nslots + (size_t)b * 16;
      long long last = t[0];
      if (!last) continue;
      for (int k = 1; k < 8; ++k)  // phases 1-7 (8-10: the tie re-sort inside phase 2, in the slowest-block lines)
        if (t[k]) {
          acc[k] += (double)(t[k] - last);
          ++cnt[k];
          last = t[k];
        }
      life += (double)(last - t[0]);
      wlife += t[15] ? (double)(t[15] - t[14]) * 0.01 : 0.0;
      ++nb;
      t_min = t_min ? std::min(t_min, t[14]) : t[14];
      t_max = std::max(t_max, t[15]);
    }
    long long s_max = 0;
    for (int b = 0; b < 2 * n; ++b) {
      const long long* t = h.data() + (size_t)side * 16 * 2 * c->nslots + (size_t)b * 16;
      if (t[14]) s_max = std::max(s_max, t[14] - t_min);
    }
    {
      std::vector<std::pair<long long, int>> lv;
      for (int b = 0; b < 2 * n; ++b) {
        const long long* t = h.data() + (size_t)side * 16 * 2 * c->nslots + (size_t)b * 16;
        if (t[15]) lv.push_back({t[15] - t[14], b});
      }
      std::sort(lv.rbegin(), lv.rend());
      fprintf(stderr, "kprof slowest:");
      for (size_t i = 0; i < lv.size() && i < 6; ++i) {
        const long long* t = h.data() + (size_t)side * 16 * 2 * c->nslots + (size_t)lv[i].second * 16;
        fprintf(stderr, " [blk %d n=%lld %.1fus cyc=%lld:", lv[i].second, t[13], lv[i].first * 0.01, t[7] - t[0]);
        for (int k = 1; k <= 11; ++k) fprintf(stderr, " %lld", t[k] ? t[k] - t[0] : -1);
        fprintf(stderr, " levels %lld", t[12]);
        fprintf(stderr, "]");
      }
      fprintf(stderr, "\n");
    }
    fprintf(stderr, "kprof k_nms %s: blocks=%d life=%.0f cyc = %.1f us, span=%.1f us, last start=%.1f us", side ? "side" : "bottom",
            nb, nb ? life / nb : 0.0, nb ? wlife / nb : 0.0, (t_max - t_min) * 0.01, s_max * 0.01);
    for (int k = 1; k < 13; ++k)
      if (cnt[k]) fprintf(stderr, " p%d=%.0f", k, acc[k] / cnt[k]);
    fprintf(stderr, "\n");
  }
}

// Diagnostics (LM_DUMP_DIR): one slot's candidate-path state after a failed
// batch -> <dir>/dump_<frame>.bin: int32 [frame, slot, feat, npos_b, npos_s,
// hdr.n_pos[4], hdr.cand_cnt[4], hdr.ties[4]] then, per list 0..3, the list's
// whole key area (u64 x list_cap).
void dump_slot(lm_ctx* c, Lane& L, const char* dir, int frame, int slot, int feat) {
  const LmConst& K = c->K;
  std::vector<int32_t> np(LM_NLIST);
  COPY_SYNC(np.data(), L.npos.p + (int64_t)slot * LM_NLIST, LM_NLIST * sizeof(int32_t), hipMemcpyDeviceToHost, L.stream);
  LmSlotOut h;
  COPY_SYNC(&h, L.arena[L.parity].hdr.p + slot, sizeof(h), hipMemcpyDeviceToHost, L.stream);
  std::string path = std::string(dir) + "/dump_" + std::to_string(frame) + ".bin";
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return;
  int32_t hd[5 + 12] = {frame, slot, feat, np[0], np[1]};
  for (int l = 0; l < 4; ++l) {
    hd[5 + l] = h.n_pos[l];
    hd[9 + l] = h.cand_cnt[l];
    hd[13 + l] = h.ties[l];
  }
  fwrite(hd, sizeof(hd), 1, f);
  fwrite(np.data(), sizeof(int32_t), LM_NLIST, f);
  for (int l = 0; l < LM_NLIST; ++l) {
    std::vector<unsigned long long> kv((size_t)K.list_cap[l]);
    HIPCHK(hipMemcpy(kv.data(), L.keys.p + (int64_t)slot * K.keys_per_slot + K.list_off[l],
                     kv.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    fwrite(kv.data(), sizeof(unsigned long long), kv.size(), f);
  }
  fclose(f);
}

CorrDark lane_dark(const lm_ctx* c, Lane& L) {
  CorrDark d;
  if (c->dark_on) {
    d.flags = L.dark_flags.p;
    d.cnt = L.dark_cnt.p;
    d.list = L.dark_list.p;
  }
  return d;
}

// The kernel chain of one batch attempt on lane L (part: 0 the kernels before
// k_corr, 1 k_corr, 2 the kernels after, -1 all).  Kernel arguments depend
// only on the key of L.graphs (frame pointers and slots reach the kernels
// through k_prep's copies of mapped host arrays), so the chain is captured
// once per key into hipGraphs and replayed.
void enqueue_chain(lm_ctx* c, Lane& L, Arena& A, const Lane::Pending& P, Timer& T, bool do_carry, int part) {
  const LmConst& K = c->K;
  const LmConst* dK = c->dK.p;
  hipStream_t st = L.stream;
  const int n = P.n, s_lut0 = P.s_lut0, s_proc0 = P.s_proc0;
  const int nproc = n + 1 - s_proc0;
  if (part <= 0) {
    // block 1: k_carry (a rerun keeps slot 0's staged candidates)
    k_prep<<<do_carry ? 2 : 1, 256, 0, st>>>(L.h_slots.d, L.h_frame_ptr.d, L.h_ctl.d, n + 1, L.slots.p, L.frame_ptr.p,
                                             A.ctl.p, L.npos.p, L.err.p, dK, L.keys.p, L.arena[P.prv].hdr.p, P.last_n,
                                             A.hdr.p, L.dark_cnt.p);
    T.begin("k_minmax");
    k_minmax<<<dim3(LM_MM_SPLIT, n + 1 - s_lut0), LM_MM_THREADS, 0, st>>>(L.frame_ptr.p, c->bkg.p, c->npix, s_lut0,
                                                                        L.mm.p);
    k_lut<<<(n + 1 - s_lut0 + 3) / 4, 256, 0, st>>>(L.mm.p, s_lut0, n + 1, c->adj.p, c->setup.method != 0, L.luts.p);
    T.end();
    // ext crops of both views, and (dark tiles) the bright-tile flags and lists
    T.begin("k_ingest");
    const CorrDark dk = lane_dark(c, L);
    long long* kpi = nullptr;
    const size_t ing_blocks = (size_t)(K.ing_nb[0] + K.ing_nb[1]) * ((c->nslots + LM_INGEST_FB - 1) / LM_INGEST_FB);
    if (c->kprof_on) {
      if (!L.kprof_ing.p) L.kprof_ing.alloc(16 * ing_blocks);
      HIPCHK(hipMemsetAsync(L.kprof_ing.p, 0, sizeof(long long) * 16 * ing_blocks, st));
      kpi = L.kprof_ing.p;
    }
    k_ingest<<<dim3((unsigned)(K.ing_nb[0] + K.ing_nb[1]), (unsigned)((nproc + LM_INGEST_FB - 1) / LM_INGEST_FB)),
               K.ing_threads, 0, st>>>(dK, L.frame_ptr.p, c->bkg.p, c->cal.p, L.luts.p, L.slots.p, s_proc0, n + 1, L.ext.p,
                                        c->ext_slot_bytes, reinterpret_cast<unsigned*>(L.tailbin.p), L.smap.p, L.sbkg.p,
                                        L.skey.p, dk.flags, dk.cnt, dk.list, kpi);
    T.end();
  }
  if (part == 1 || part < 0) {
    T.begin("k_corr");
    const lm_ctx::CorrPlan& CP = c->corr_plan[P.plan];
    for (size_t gi = 0; gi < CP.groups.size(); ++gi) {
      const auto& grp = CP.groups[gi];
      const LmDetGroup& G = grp.second;
      const void* w = c->setup.corr_precision == LM_CORR_F16 ? (const void*)c->weights16.p : (const void*)c->weights.p;
      HIPCHK(launch_corr(grp.first, CP.ring[gi], dim3(G.tile_end[G.n - 1], nproc), CP.threads[gi], CP.lds[gi], st, dK,
                         G, L.ext.p, c->ext_slot_bytes, w, s_proc0, L.keys.p, L.npos.p, L.tailbin.p,
                         c->tailbin_slot_bytes, lane_dark(c, L)));
    }
    T.end();
  }
  if (part == 2 || part < 0) {
    if (c->debug & 1) {
      if (!L.dbg.p) {
        L.dbg.alloc((size_t)c->dbg_slot_floats * c->nslots);
        L.dbg_offd.alloc(LM_NDET);
        COPY_SYNC(L.dbg_offd.p, c->dbg_off, sizeof(c->dbg_off), hipMemcpyHostToDevice, st);
      }
      HIPCHK(launch_corr_dbg(c->unfused, dim3(64, nproc, LM_NDET), st, dK, L.ext.p, c->ext_slot_bytes, c->weights.p,
                             s_proc0, L.dbg.p, L.dbg_offd.p, c->dbg_slot_floats));
    }
    long long *kp0 = nullptr, *kp1 = nullptr, *kp2 = nullptr, *kp3 = nullptr;
    if (c->kprof_on) {
      if (!L.kprof.p) L.kprof.alloc((size_t)4 * 16 * 2 * c->nslots);
      HIPCHK(hipMemsetAsync(L.kprof.p, 0, sizeof(long long) * 4 * 16 * 2 * c->nslots, st));
      kp0 = L.kprof.p;
      kp1 = L.kprof.p + 16 * 2 * c->nslots;
      kp2 = L.kprof.p + 2 * 16 * 2 * c->nslots;
      kp3 = L.kprof.p + 3 * 16 * 2 * c->nslots;
    }
    T.begin("k_tail");
    if (c->tail_big)
      k_tail<true><<<nproc, LM_TAIL_THREADS, 0, st>>>(dK, s_proc0, L.tailbin.p, c->tailbin_slot_bytes, L.tailmask.p,
                                                      L.tscratch.p, A.hdr.p, kp2, L.tail_ws.p, c->tail_ws_slot,
                                                      L.keys.p, L.npos.p);
    else
      k_tail<false><<<nproc, LM_TAIL_THREADS, c->tail_lds, st>>>(dK, s_proc0, L.tailbin.p, c->tailbin_slot_bytes,
                                                                 L.tailmask.p, L.tscratch.p, A.hdr.p, kp2, nullptr, 0,
                                                                 L.keys.p, L.npos.p);
    T.end();
    T.begin("k_nms");
    // one block per (slot, list); lists beyond the LDS capacity in global scratch
    k_nms<false><<<dim3(nproc, 4), LM_NMS_THREADS, 0, st>>>(dK, s_proc0, L.keys.p, L.npos.p, L.tailmask.p, L.gscratch.p,
                                                           c->gscratch_slot, A.hdr.p, L.err.p, kp0, kp1, 0);
    k_nms<true><<<LM_GLOB_BLOCKS, LM_NMS_THREADS, 0, st>>>(dK, s_proc0, L.keys.p, L.npos.p, L.tailmask.p, L.gscratch.p,
                                              c->gscratch_slot, A.hdr.p, L.err.p, nullptr, nullptr, 4 * nproc);
    T.end();
    T.begin("k_post");
    k_post<false><<<dim3(n, 2), LM_POST_THREADS, 0, st>>>(dK, L.slots.p, L.frame_ptr.p, c->bkg.p, c->cal.p, L.luts.p,
                                                         A.hdr.p, L.keys.p, A.p22d.p, A.side_y.p, A.side_s.p, A.unary.p,
                                                         A.jc.p, A.ir.p, A.pr.p, A.ctl.p, L.err.p, L.gscratch.p,
                                                         c->gscratch_slot, kp3, 0);
    k_post<true><<<LM_GLOB_BLOCKS, LM_POST_THREADS, 0, st>>>(dK, L.slots.p, L.frame_ptr.p, c->bkg.p, c->cal.p, L.luts.p, A.hdr.p,
                                                L.keys.p, A.p22d.p, A.side_y.p, A.side_s.p, A.unary.p, A.jc.p, A.ir.p,
                                                A.pr.p, A.ctl.p, L.err.p, L.gscratch.p, c->gscratch_slot, nullptr,
                                                2 * n);
    T.end();
    T.begin("k_pack");
    k_pack_scan<<<1, 1024, 0, st>>>(A.hdr.p, n, A.ctl.p, L.err.p, A.ph.p, A.pack.p, A.pack_cap, A.side_base.p);
    k_pack_copy<<<dim3(n, 2), 256, 0, st>>>(dK, A.hdr.p, n, L.keys.p, A.p22d.p, A.side_y.p, A.side_s.p, A.unary.p,
                                            A.jc.p, A.ir.p, A.pr.p, A.ph.p, A.pack.p, A.side_base.p);
    T.end();
    // header + results to host memory, then frame n as the next batch's halo
    k_out<<<128, 256, 0, st>>>(A.ph.p, L.h_ph.d, A.pack.p, nullptr, 0, A.ctl.p, nullptr, L.frame_ptr.p, n, L.halo.p,
                               c->npix);
  }
}

// Launch attempt `attempt` of the lane's pending batch (attempt 0 from the
// captured graphs; reruns after a result-arena overflow directly).
void launch_attempt(lm_ctx* c, Lane& L, int attempt) {
  static const bool graphs_env = [] {
    const char* v = getenv("LM_GRAPH");
    return !v || atoi(v) != 0;
  }();
  const Lane::Pending& P = L.pend;
  hipStream_t st = L.stream;
  Arena& A = L.arena[P.cur];
  LmArenaCtl& hc = *L.h_ctl.p;
  std::memset(&hc, 0, sizeof(hc));
  for (int k = 0; k < AR_COUNT; ++k) hc.cap[k] = A.cap[k];
  hc.pack_dst = c->packs[P.pack]->d;
  hc.pack_cap = (int64_t)c->packs[P.pack]->n;
  hc.nparts = std::min(LM_SUBARENA, 2 * P.n);  // k_post has 2n blocks: every part gets used
  Timer T(c, L);
  const bool graph = graphs_env && L.use_graphs && attempt == 0 && !(c->debug & 1) && !c->kprof_on;
  if (graph) {
    // Three graphs per key (before / k_corr / after), so the timing events
    // of k_corr (the roofline kernel) are recorded on the stream between
    // graph launches; the other kernels are not timed on this path.
    const std::array<int, 7> key{P.n, P.cur, P.carry ? 1 : 0, P.carry ? P.last_n : 0, P.s_lut0, P.s_proc0, P.plan};
    auto it = L.graphs.find(key);
    if (it == L.graphs.end()) {
      Lane::GraphEntry ent{};
      bool ok = true;
      const bool t_on = T.on;
      T.on = false;
      for (int part = 0; part < 3 && ok; ++part) {
        hipGraph_t g = nullptr;
        ok = hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) == hipSuccess;
        if (!ok) break;
        try {
          enqueue_chain(c, L, A, P, T, P.carry, part);
        } catch (const std::exception&) {
          ok = false;
        }
        const hipError_t e = hipStreamEndCapture(st, &g);
        ok = ok && e == hipSuccess && g;
        if (ok) ok = hipGraphInstantiate(&ent.exec[part], g, nullptr, nullptr, 0) == hipSuccess;
        if (g) (void)hipGraphDestroy(g);
      }
      T.on = t_on;
      (void)hipGetLastError();
      if (ok) {
        it = L.graphs.emplace(key, ent).first;
      } else {  // capture unsupported here: run the chain directly from now on
        for (hipGraphExec_t x : ent.exec)
          if (x) (void)hipGraphExecDestroy(x);
        L.use_graphs = false;
      }
    }
    if (it != L.graphs.end()) {
      HIPCHK(hipGraphLaunch(it->second.exec[0], st));
      T.begin("k_corr");
      HIPCHK(hipGraphLaunch(it->second.exec[1], st));
      T.end();
      HIPCHK(hipGraphLaunch(it->second.exec[2], st));
    } else {
      enqueue_chain(c, L, A, P, T, P.carry, -1);
    }
  } else {
    enqueue_chain(c, L, A, P, T, P.carry && attempt == 0, -1);
  }
  HIPCHK(hipGetLastError());
}

void finish_batch(lm_ctx* c, Lane& L);

// The batch running on lane L is complete (or failed): finish it now and
// keep its packed results (or its error) in its queue record, so the lane
// can take the next batch while the results wait to be collected in order.
void retire(lm_ctx* c, Lane& L) {
  lm_ctx::BatchRec* rec = nullptr;
  for (auto& r : c->queue)
    if (r.lane == L.index && r.seq == L.seq) rec = &r;
  if (!rec) throw std::runtime_error("pipeline: no record of the batch running on lane " + std::to_string(L.index));
  try {
    finish_batch(c, L);
    rec->ph = *L.h_ph.p;
  } catch (const std::invalid_argument& e) {
    rec->status = LM_ERR_INVALID_ARGUMENT;
    rec->err = e.what();
  } catch (const HipError& e) {
    rec->status = LM_ERR_HIP;
    rec->err = e.what();
  } catch (const std::exception& e) {
    rec->status = LM_ERR_RUNTIME;
    rec->err = e.what();
  }
  if (rec->status != LM_OK) L.have_state = false;
  rec->t_names = L.t_names;
  std::copy(L.t_work, L.t_work + 4, rec->work);
  rec->t_ms = L.t_ms;
  rec->t_t0 = L.t_t0;
  rec->t_t1 = L.t_t1;
  rec->ran_lane = L.index;
  rec->lane = -1;
  L.seq = -1;
}

// A free lane for the next batch: the lane that ran the previous batch when
// nothing ran there since (it carries that batch's state), else any idle
// lane; when every lane is busy, the first one whose batch has completed is
// retired and reused -- or, when none has, the host thread sleeps on the
// oldest batch's completion event (blocking sync, not a polling loop) and
// retires that one.
Lane& acquire_lane(lm_ctx* c, int prev_frame) {
  Lane* pick = nullptr;
  for (auto& l : c->lanes) {
    if (l->seq >= 0) continue;
    if (l->index == c->last_lane && l->have_state && l->last_frame == prev_frame) return *l;
    if (!pick) pick = l.get();
  }
  if (pick) return *pick;
  Lane* oldest = nullptr;
  for (auto& l : c->lanes) {
    const hipError_t q = hipStreamQuery(l->stream);
    if (q != hipErrorNotReady) {
      (void)hipGetLastError();
      retire(c, *l);
      return *l;
    }
    if (!oldest || l->seq < oldest->seq) oldest = l.get();
  }
  (void)hipGetLastError();
  HIPCHK(hipEventSynchronize(oldest->ev_done));
  retire(c, *oldest);
  return *oldest;
}

// Submit frames [first, first + n) to a free lane (acquire_lane).  Host
// frames are copied to the lane's staging slots before this returns; device
// frames are read in place while the batch runs.  At most 2 x lanes batches
// may wait for collection.  Batch k + 1 continues batch k:
//  - on the lane that ran batch k (nothing run there since): slot 0 carries
//    batch k's last frame and candidates (k_carry; k_out left the frame in
//    the lane's halo);
//  - on another lane: batch k copied its last frame to handoff[k & 1] at its
//    start (event ev_snap); batch k + 1 copies it into its own halo (event
//    ev_consumed) and runs it as a 1-frame halo (its candidates recomputed),
//    so the two batches' kernels never wait for each other.
void submit_batch(lm_ctx* c, const uint8_t* frames, int64_t pitch, int n, int first, const uint8_t* prev,
                  const int32_t* bb, bool device_frames) {
  if (n <= 0 || n > c->max_batch) throw std::invalid_argument("n must be in [1, max_batch].");
  if (first < 0) throw std::invalid_argument("first_frame must be >= 0.");
  if (!frames) throw std::invalid_argument("frames is NULL.");
  if (pitch < c->npix) throw std::invalid_argument("frame_pitch smaller than one frame.");
  if (c->queue.size() >= 2 * c->lanes.size())
    throw std::invalid_argument("2 x pipeline_lanes batches wait for collection: lm_detect_collect first.");
  HIPCHK(hipSetDevice(c->device));
  const bool pipelined = c->lanes.size() > 1;
  const bool given_halo = prev != nullptr && first > 0;
  const bool cont = !given_halo && first > 0;
  if (cont && !(c->have_state && c->last_frame == first - 1))
    throw std::invalid_argument("frame first_frame-1 was not processed by this context: pass prev_frame (shard start).");
  Lane& L = acquire_lane(c, cont ? first - 1 : -2);
  const bool carry = cont && c->last_lane == L.index && L.have_state && L.last_frame == first - 1;
  const bool handoff = cont && !carry;
  if (handoff && !pipelined)
    throw std::invalid_argument("the previous batch failed: pass prev_frame to continue from frame first_frame.");
  const bool halo = given_halo || handoff;
  const lm_geometry& g = c->geo;
  const LmConst& K = c->K;
  const int64_t fstride = c->fstride;
  hipStream_t st = L.stream;

  // Device frames are read in place when 16-byte aligned (the kernels load
  // 16 B per lane); otherwise they are first copied into the staging slots.
  const bool direct = device_frames && ((((uintptr_t)frames | (uintptr_t)pitch) & 15) == 0);
  // ---- slots: frame pointers and crop rectangles (cropBoundingBox :1420-1470)
  const int s_lut0 = first > 0 ? 0 : 1, s_proc0 = halo ? 0 : 1;
  int new_last_bb[3] = {c->bb_x, c->bb_yb, c->bb_ys};
  for (int s = 0; s <= n; ++s) {
    LmSlot& S = L.h_slots.p[s];
    std::memset(&S, 0, sizeof(S));
    const int gframe = first - 1 + s;
    S.frame = gframe;
    S.active = s >= s_lut0;
    if (s == 0) L.h_frame_ptr.p[0] = L.halo.p;
    else L.h_frame_ptr.p[s] = direct ? frames + (int64_t)(s - 1) * pitch : L.frames.p + (int64_t)s * fstride;
    if (s < s_lut0) continue;
    const int bi = given_halo ? s : s - 1;  // index into bb[]
    int bx = c->bb_x, byb = c->bb_yb, bys = c->bb_ys;
    if (bb && (s > 0 || given_halo)) {
      bx = bb[3 * bi];
      byb = bb[3 * bi + 1];
      bys = bb[3 * bi + 2];
    } else if (s == 0 && cont) {  // the previous batch's last frame
      bx = c->last_bb[0];
      byb = c->last_bb[1];
      bys = c->last_bb[2];
    }
    if (s == n) {
      new_last_bb[0] = bx;
      new_last_bb[1] = byb;
      new_last_bb[2] = bys;
    }
    S.crop_x[0] = (int)((unsigned)(bx + g.pad_pre_cols) - (unsigned)(g.bb_bottom_mouse_pad.width - g.spost_b_w) + 1u);
    S.crop_y[0] = (int)((unsigned)(byb + g.pad_pre_rows) - (unsigned)(g.bb_bottom_mouse_pad.height - g.spost_b_h) + 1u);
    S.crop_x[1] = (int)((unsigned)(g.pad_pre_cols + bx) - (unsigned)(g.bb_side_mouse_pad.width - g.spost_t_w) + 1u);
    S.crop_y[1] = (int)((unsigned)(g.pad_pre_rows + bys) - (unsigned)(g.bb_side_mouse_pad.height - g.spost_t_h) + 1u);
    const int w[2] = {g.bb_bottom_mouse_pad.width, g.bb_side_mouse_pad.width};
    const int h[2] = {g.bb_bottom_mouse_pad.height, g.bb_side_mouse_pad.height};
    if (s >= s_proc0)
      for (int v = 0; v < 2; ++v)
        if (S.crop_x[v] < 0 || S.crop_y[v] < 0 || S.crop_x[v] + w[v] > g.ipad_cols || S.crop_y[v] + h[v] > g.ipad_rows)
          throw std::runtime_error(std::string("ROI out of image bounds: ") + (v ? "BB_SIDE_MOUSE_PAD" : "BB_BOTTOM_MOUSE_PAD"));
    if (K.gray_lut_on) {  // the in-place LUT must stay inside I_UNPAD (see locomouse_hip.h)
      const int ux = S.crop_x[0] + g.spre_b_w, uy = S.crop_y[0] + g.spre_b_h;
      if (ux < g.pad_pre_cols || uy < g.pad_pre_rows || ux + g.bb_bottom_mouse.width > g.pad_pre_cols + g.n_cols ||
          uy + g.bb_bottom_mouse.height > g.pad_pre_rows + g.n_rows)
        throw std::invalid_argument("transform_gray_values: frame " + std::to_string(S.frame) +
                                    ": the bottom crop leaves the corrected image, so the in-place LUT would reach "
                                    "I_PAD's zero padding (not supported).");
    }
  }

  // ---- inputs.  Host frames (and a host halo frame) are the only runtime
  // copies from the caller's memory; the stream is drained after them, so
  // the caller may reuse its buffer once this returns (see k_prep / k_out for
  // why the stream otherwise holds only kernels).
  if (!device_frames) {
    // one 2-D transfer for the batch (DMA from page-locked buffers, e.g. lm_host_alloc)
    HIPCHK(hipMemcpy2DAsync(L.frames.p + fstride, (size_t)fstride, frames, (size_t)pitch, (size_t)c->npix, (size_t)n,
                            hipMemcpyHostToDevice, st));
    if (given_halo) HIPCHK(hipMemcpyAsync(L.halo.p, prev, c->npix, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
  } else {
    if (!direct)
      HIPCHK(hipMemcpy2DAsync(L.frames.p + fstride, (size_t)fstride, frames, (size_t)pitch, (size_t)c->npix, (size_t)n,
                              hipMemcpyDeviceToDevice, st));
    if (given_halo && ((uintptr_t)prev & 15) == 0)
      k_out<<<64, 256, 0, st>>>(L.zero_ph.p, L.h_ph.d, nullptr, nullptr, 0, nullptr, prev, nullptr, 0, L.halo.p,
                                c->npix);
    else if (given_halo)
      HIPCHK(hipMemcpyAsync(L.halo.p, prev, (size_t)c->npix, hipMemcpyDeviceToDevice, st));
  }
  // ---- pipelined halo hand-off (every batch of a multi-lane context)
  if (pipelined) {
    const uint8_t* last = direct ? frames + (int64_t)(n - 1) * pitch : L.frames.p + (int64_t)n * fstride;
    // handoff[k & 1] was last read by batch k - 1 (it took batch k - 2's frame from there)
    if (c->last_lane >= 0) HIPCHK(hipStreamWaitEvent(st, c->lanes[c->last_lane]->ev_consumed, 0));
    HIPCHK(hipMemcpyAsync(c->handoff.p + (c->nsub & 1) * fstride, last, (size_t)c->npix, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipEventRecord(L.ev_snap, st));
    if (handoff) {
      HIPCHK(hipStreamWaitEvent(st, c->lanes[c->last_lane]->ev_snap, 0));
      HIPCHK(hipMemcpyAsync(L.halo.p, c->handoff.p + ((c->nsub - 1) & 1) * fstride, (size_t)c->npix,
                            hipMemcpyDeviceToDevice, st));
    }
    HIPCHK(hipEventRecord(L.ev_consumed, st));
  }
  if (!L.gscratch.p) L.gscratch.alloc((size_t)c->gscratch_slot * LM_GLOB_BLOCKS);  // one region per block of the <true> launches
  // k_ingest's source map: rebuilt for a view when every processed slot has
  // its crop at one position that the lane's map does not hold
  for (int v = 0; v < 2; ++v) {
    const LmSlot& S0 = L.h_slots.p[s_proc0];
    bool uni = true;
    for (int s = s_proc0 + 1; s <= n && uni; ++s)
      uni = L.h_slots.p[s].crop_x[v] == S0.crop_x[v] && L.h_slots.p[s].crop_y[v] == S0.crop_y[v];
    if (uni && (L.skey_h[2 * v] != S0.crop_x[v] || L.skey_h[2 * v + 1] != S0.crop_y[v])) {
      const int64_t nv = (int64_t)K.ext_h[v] * K.ext_w[v] / LM_INGEST_VEC;
      k_srcmap<<<(unsigned)((nv + 255) / 256), 256, 0, st>>>(c->dK.p, c->cal.p, c->bkg.p, v, S0.crop_x[v], S0.crop_y[v],
                                                            L.smap.p, L.sbkg.p, L.skey.p);
      HIPCHK(hipGetLastError());
      L.skey_h[2 * v] = S0.crop_x[v];
      L.skey_h[2 * v + 1] = S0.crop_y[v];
    }
  }

  Lane::Pending& P = L.pend;
  P.on = true;
  P.n = n;
  P.first = first;
  P.s_lut0 = s_lut0;
  P.s_proc0 = s_proc0;
  P.plan = corr_plan_for(c);
  P.cur = L.parity;
  P.prv = L.last_parity;
  P.carry = carry;
  P.last_n = carry ? L.last_n : 0;
  P.pack = c->take_pack((size_t)L.arena[P.cur].pack_cap);
  try {
    launch_attempt(c, L, 0);
    L.h_cnt_valid = (c->debug & 2) && L.dark_cnt.p;
    if (L.h_cnt_valid)
      HIPCHK(hipMemcpyAsync(L.h_cnt.p, L.dark_cnt.p, 4 * LM_TL_NC * sizeof(int32_t), hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(L.ev_done, st));
  } catch (...) {
    // kernels of this batch may already be enqueued: the lane (and the pack
    // k_out writes into) is free only once its stream has drained
    (void)hipStreamSynchronize(st);
    (void)hipGetLastError();
    c->drop_pack(P.pack);
    P.on = false;
    throw;
  }

  // the video position and the lane's carry state advance now; a batch that
  // fails at collection clears the lane's state (a later batch on another
  // lane only needs this batch's pixels)
  c->have_state = true;
  c->last_frame = first + n - 1;
  for (int k = 0; k < 3; ++k) c->last_bb[k] = new_last_bb[k];
  c->last_lane = L.index;
  L.seq = c->nsub;
  lm_ctx::BatchRec rec;
  rec.seq = c->nsub;
  rec.lane = L.index;
  rec.pack = P.pack;
  rec.first = first;
  rec.n = n;
  rec.slots = n + 1 - s_proc0;
  c->queue.push_back(std::move(rec));
  ++c->nsub;
  L.have_state = true;
  L.last_frame = first + n - 1;
  L.last_n = n;
  L.last_parity = P.cur;
  L.parity = 1 - P.cur;
}

// Wait for the lane's batch and rerun it while its result arena overflows;
// its packed results are then in the batch's result buffer.
void finish_batch(lm_ctx* c, Lane& L) {
  Lane::Pending& P = L.pend;
  hipStream_t st = L.stream;
  const int n = P.n, first = P.first;
  HIPCHK(hipSetDevice(c->device));
  for (int attempt = 0;; ++attempt) {
    if (attempt > 0) {
      launch_attempt(c, L, attempt);
      L.h_cnt_valid = false;  // (the counters of the rerun: read synchronously)
    }
    HIPCHK(hipStreamSynchronize(st));
    Arena& A = L.arena[P.cur];
    const LmPackHdr& ph = *L.h_ph.p;
    const int e = (c->debug & 4) ? (ph.err & ~4) : ph.err;  // debug bit 2: report but keep going
    if ((c->debug & 4) && (ph.err & 4)) {
      COPY_SYNC(L.h_err.p, L.err.p, 16 * sizeof(int32_t), hipMemcpyDeviceToHost, st);
      const int32_t* d = L.h_err.p;
      fprintf(stderr, "[lm debug] vel box error frame %d tag %x box (%d,%d,%d,%d)\n", first - 1 + (d[2] >> 16), d[2],
              d[3], d[4], d[5], d[6]);
    }
    if (e & 4) {
      COPY_SYNC(L.h_err.p, L.err.p, 16 * sizeof(int32_t), hipMemcpyDeviceToHost, st);
      const int32_t* d = L.h_err.p;
      const int tag = d[2], slot = tag >> 16;
      if (const char* dir = getenv("LM_DUMP_DIR")) dump_slot(c, L, dir, first - 1 + slot, slot, (tag >> 12) & 1);
      char buf[256];
      snprintf(buf, sizeof buf, " [frame %d, %s %s candidate %d: box (%d,%d,%d,%d) in crop %dx%d]",
               first - 1 + slot, (tag >> 12 & 1) ? "snout" : "paw", (tag & 0x800) ? "side" : "bottom", tag & 0x7FF,
               d[3], d[4], d[5], d[6], d[7], d[8]);
      throw std::runtime_error(std::string("checkVelCriterion: match box outside the padded crop (cv::Mat ROI "
                                           "assertion).") + buf);
    }
    if (e & 16) throw std::runtime_error("P22D::add_side_candidate_safe: CV_Assert(S >= 0) failed.");
    if (e & 8) throw std::runtime_error("candidate list exceeds the k_post scratch capacity.");
    if (e & 32) throw std::runtime_error("candidate staging overflow.");
    if (e) throw std::runtime_error("device error flags " + std::to_string(e));
    if (!ph.overflow) break;
    if (attempt >= 3) throw std::runtime_error("result arena overflow persists.");
    L.drop_graphs();  // arena / pack buffers are reallocated below
    if (ph.overflow & 2) {
      int ncap[AR_COUNT];
      for (int k = 0; k < AR_COUNT; ++k) ncap[k] = std::max(A.cap[k], (int)(ph.used[k] * 1.25) + 1024);
      A.alloc(ncap, c->nslots);
    }
    A.alloc_pack(ph.bytes + ph.bytes / 4);
  }
  if (c->debug & 2) {
    Timer::collect(c, L);
  } else {
    L.t_ev.clear();
    for (int k = 0; k < 4; ++k) L.t_work[k] = -1;
  }
  if (c->kprof_on) kprof_report(c, L, n);

  // ---- the packed results (lm_batch_result layout) are in the batch's
  // buffer unless they outgrew it: then grow it and let k_out copy them (and
  // the halo) again
  Arena& A = L.arena[P.cur];
  const LmPackHdr ph = *L.h_ph.p;
  HostBuf<uint8_t>& HP = *c->packs[P.pack];
  if ((int64_t)HP.n < ph.bytes) {
    HP.alloc((size_t)(ph.bytes + ph.bytes / 4));
    k_out<<<128, 256, 0, st>>>(A.ph.p, L.h_ph.d, A.pack.p, HP.d, (int64_t)HP.n, nullptr, nullptr, L.frame_ptr.p, n,
                               L.halo.p, c->npix);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
  }
  if (guard_mode()) {
    HIPCHK(hipDeviceSynchronize());
    guard_check_all();
  }
  if (c->debug & 8) {  // diagnostics: a second, synchronous copy of the pack must equal the async one
    HIPCHK(hipDeviceSynchronize());
    std::vector<uint8_t> chk((size_t)ph.bytes);
    HIPCHK(hipMemcpy(chk.data(), A.pack.p, (size_t)ph.bytes, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < ph.bytes; ++i)
      if (chk[i] != HP.p[i]) {
        int64_t j = ph.bytes - 1;
        while (j > i && chk[j] == HP.p[j]) --j;
        fprintf(stderr, "[lm debug] D2H pack mismatch frames %d..%d: bytes [%ld, %ld] of %ld differ\n", first,
                first + n - 1, (long)i, (long)j, (long)ph.bytes);
        break;
      }
  }
  L.batch_n = n;
  L.batch_s0 = P.s_proc0;
  L.done_seq = L.seq;
  P.on = false;
}

// lm_batch_result pointers into packed results `hp` (lm_pack_layout).
void fill_result(lm_batch_result* out, const uint8_t* hp, int n, int first, const LmPackHdr& ph) {
  const LmPackLayout PL = lm_pack_layout(n, ph.tot);
  out->n_frames = n;
  out->first_frame = first;
  out->cand_offset = reinterpret_cast<const int64_t*>(hp + PL.cand_off);
  out->cand = reinterpret_cast<const lm_candidate*>(hp + PL.cand);
  out->p22d_offset = reinterpret_cast<const int64_t*>(hp + PL.p22d_off);
  out->p22d = reinterpret_cast<const lm_p22d*>(hp + PL.p22d);
  out->side_y = reinterpret_cast<const int32_t*>(hp + PL.side_y);
  out->side_s = reinterpret_cast<const double*>(hp + PL.side_s);
  out->unary_offset = reinterpret_cast<const int64_t*>(hp + PL.unary_off);
  out->unary = reinterpret_cast<const double*>(hp + PL.unary);
  out->pw_dims = reinterpret_cast<const int32_t*>(hp + PL.pw_dims);
  out->pw_jc_offset = reinterpret_cast<const int64_t*>(hp + PL.jc_off);
  out->pw_jc = reinterpret_cast<const int32_t*>(hp + PL.jc);
  out->pw_nz_offset = reinterpret_cast<const int64_t*>(hp + PL.nz_off);
  out->pw_ir = reinterpret_cast<const int32_t*>(hp + PL.ir);
  out->pw_pr = reinterpret_cast<const double*>(hp + PL.pr);
  out->tail = reinterpret_cast<const int32_t*>(hp + PL.tail);
}

// The oldest submitted batch's results (valid until the next lm_detect_*
// call on the context).
void collect_batch(lm_ctx* c, lm_batch_result* out) {
  if (c->queue.empty()) throw std::invalid_argument("no batch in flight: lm_detect_submit one first.");
  lm_ctx::BatchRec rec = std::move(c->queue.front());
  c->queue.pop_front();
  // the previously delivered batch's arrays are no longer valid (the caller
  // made another lm_detect_* call): its buffer is free again
  c->drop_pack(c->delivered.pack);
  c->delivered.pack = -1;
  if (rec.lane >= 0) {  // still on its lane: finish it there
    Lane& L = *c->lanes[rec.lane];
    rec.ran_lane = L.index;
    try {
      finish_batch(c, L);
    } catch (...) {
      L.pend.on = false;
      L.have_state = false;
      L.seq = -1;
      c->drop_pack(rec.pack);
      throw;
    }
    L.seq = -1;
    rec.t_names = L.t_names;
    std::copy(L.t_work, L.t_work + 4, rec.work);
    rec.t_ms = L.t_ms;
    rec.t_t0 = L.t_t0;
    rec.t_t1 = L.t_t1;
    rec.ph = *L.h_ph.p;
  }
  if (rec.status != LM_OK) {
    c->drop_pack(rec.pack);
    if (rec.status == LM_ERR_INVALID_ARGUMENT) throw std::invalid_argument(rec.err);
    if (rec.status == LM_ERR_HIP) throw HipError(rec.err);
    throw std::runtime_error(rec.err);
  }
  c->delivered = std::move(rec);
  fill_result(out, c->packs[c->delivered.pack]->p, c->delivered.n, c->delivered.first, c->delivered.ph);
}

// One synchronous batch (submit + collect); nothing may be in flight.
void run_batch(lm_ctx* c, const uint8_t* frames, int64_t pitch, int n, int first, const uint8_t* prev, const int32_t* bb,
               bool device_frames, lm_batch_result* out) {
  if (!c->queue.empty())
    throw std::invalid_argument("batches are in flight: lm_detect_collect them before lm_detect_batch.");
  submit_batch(c, frames, pitch, n, first, prev, bb, device_frames);
  collect_batch(c, out);
}

}  // namespace

// ------------------------------------------------------------------- C ABI

LM_API int32_t lm_abi_version(void) { return LM_ABI_VERSION; }

LM_API const char* lm_last_error(void) { return g_err.c_str(); }

LM_API lm_status lm_ctx_create(int32_t device, const lm_setup* setup, const lm_params* params, const lm_model* model,
                               int32_t max_batch, lm_ctx** out) {
  if (!out) return fail(LM_ERR_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  if (max_batch <= 0) return fail(LM_ERR_INVALID_ARGUMENT, "max_batch must be > 0");
  if (setup && (setup->pipeline_lanes < 0 || setup->pipeline_lanes > LM_MAX_LANES))
    return fail(LM_ERR_INVALID_ARGUMENT, "pipeline_lanes must be in [0, " + std::to_string(LM_MAX_LANES) + "].");
  lm_ctx* c = new lm_ctx();
  lm_status s = guarded([&] {
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) throw HipError("invalid HIP device index");
    c->device = device;
    HIPCHK(hipSetDevice(device));
    c->max_batch = max_batch;
    c->nslots = max_batch + 1;
    validate_and_build(c, setup, params, model);
    const int nl = setup->pipeline_lanes > 0 ? setup->pipeline_lanes : 1;
    // Lanes (of all contexts of the process) alternate between the highest
    // and the lowest stream priority.  With equal priorities, concurrent
    // streams share the CUs during their correlation launches, finish them
    // together and then all run their short post-correlation kernels at once
    // (a convoy: ~19 % of the time no correlation ran, profiles/r02/rw/).
    // Unequal priorities let one stream's correlation go first, which keeps
    // the streams out of phase: +4-5 % frames/s at 4 streams per GPU.
    // LM_STREAM_PRIO=0: one priority for all.
    const char* pv = getenv("LM_STREAM_PRIO");
    const bool prio = !pv || atoi(pv) != 0;
    static std::atomic<int> n_created{0};
    int lo = 0, hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (int i = 0; i < nl; ++i) {
      c->lanes.emplace_back(new Lane());
      Lane& L = *c->lanes.back();
      L.index = i;
      L.device = device;
      if (prio) HIPCHK(hipStreamCreateWithPriority(&L.stream, hipStreamNonBlocking, (n_created++ & 1) ? lo : hi));
      else HIPCHK(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
      lane_alloc(c, L);
    }
    if (nl > 1) c->handoff.alloc((size_t)2 * c->fstride);
    // result buffers for every batch that can be in flight or delivered at
    // once (2 x lanes queued + the delivered one), pinned now rather than on
    // a timed submission
    for (int i = 0; i < 2 * nl + 1; ++i) c->take_pack((size_t)c->lanes[0]->arena[0].pack_cap);
    for (int i = 0; i < 2 * nl + 1; ++i) c->drop_pack(i);
  });
  if (s != LM_OK) {
    delete c;
    return s;
  }
  g_live_streams[c->device & 63].fetch_add((int)c->lanes.size());
  *out = c;
  return LM_OK;
}

LM_API void lm_ctx_destroy(lm_ctx* ctx) {
  if (!ctx) return;
  g_live_streams[ctx->device & 63].fetch_sub((int)ctx->lanes.size());
  // batches still in flight may copy to or from the context's buffers (the
  // hand-off frames, the arenas): every lane stream drains on the context's
  // device before anything is freed
  if (hipSetDevice(ctx->device) == hipSuccess)
    for (auto& l : ctx->lanes)
      if (l->stream) (void)hipStreamSynchronize(l->stream);
  delete ctx;
}

LM_API lm_status lm_get_geometry(const lm_ctx* ctx, lm_geometry* out) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  *out = ctx->geo;
  return LM_OK;
}

LM_API void* lm_ctx_stream(lm_ctx* ctx) { return ctx && !ctx->lanes.empty() ? (void*)ctx->lanes[0]->stream : nullptr; }

LM_API int32_t lm_ctx_lanes(const lm_ctx* ctx) { return ctx ? (int32_t)ctx->lanes.size() : 0; }

LM_API int32_t lm_ctx_pending(const lm_ctx* ctx) { return ctx ? (int32_t)ctx->queue.size() : 0; }

LM_API lm_status lm_detect_batch(lm_ctx* ctx, const uint8_t* frames, int64_t frame_pitch, int32_t n, int32_t first_frame,
                                 const uint8_t* prev_frame, const int32_t* bb, lm_batch_result* out) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  return guarded([&] { run_batch(ctx, frames, frame_pitch, n, first_frame, prev_frame, bb, false, out); });
}

LM_API lm_status lm_detect_batch_device(lm_ctx* ctx, const uint8_t* d_frames, int64_t frame_pitch, int32_t n,
                                        int32_t first_frame, const uint8_t* d_prev_frame, const int32_t* bb,
                                        lm_batch_result* out) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  return guarded([&] { run_batch(ctx, d_frames, frame_pitch, n, first_frame, d_prev_frame, bb, true, out); });
}

LM_API lm_status lm_detect_submit(lm_ctx* ctx, const uint8_t* frames, int64_t frame_pitch, int32_t n, int32_t first_frame,
                                  const uint8_t* prev_frame, const int32_t* bb) {
  if (!ctx) return fail(LM_ERR_INVALID_ARGUMENT, "null ctx");
  return guarded([&] { submit_batch(ctx, frames, frame_pitch, n, first_frame, prev_frame, bb, false); });
}

LM_API lm_status lm_detect_submit_device(lm_ctx* ctx, const uint8_t* d_frames, int64_t frame_pitch, int32_t n,
                                         int32_t first_frame, const uint8_t* d_prev_frame, const int32_t* bb) {
  if (!ctx) return fail(LM_ERR_INVALID_ARGUMENT, "null ctx");
  return guarded([&] { submit_batch(ctx, d_frames, frame_pitch, n, first_frame, d_prev_frame, bb, true); });
}

LM_API lm_status lm_detect_collect(lm_ctx* ctx, lm_batch_result* out) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  return guarded([&] { collect_batch(ctx, out); });
}

LM_API lm_status lm_ctx_set_debug(lm_ctx* ctx, int32_t flags) {
  if (!ctx) return fail(LM_ERR_INVALID_ARGUMENT, "null ctx");
  return guarded([&] {
    if (flags & 2) {
      std::lock_guard<std::mutex> lk(g_epoch_mu);
      if (!g_epoch.count(ctx->device)) {
        HIPCHK(hipSetDevice(ctx->device));
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        HIPCHK(hipEventRecord(e, ctx->lanes[0]->stream));
        HIPCHK(hipEventSynchronize(e));
        g_epoch[ctx->device] = e;
      }
    }
    ctx->debug = flags;
  });
}

LM_API int32_t lm_debug_kernel_spans(lm_ctx* ctx, const char** names, double* t0, double* t1, int32_t cap) {
  if (!ctx) return 0;
  const lm_ctx::BatchRec& L = ctx->delivered;
  const int32_t n = (int32_t)L.t_names.size();
  for (int32_t i = 0; i < n && i < cap; ++i) {
    if (names) names[i] = L.t_names[i];
    if (t0) t0[i] = L.t_t0[i];
    if (t1) t1[i] = L.t_t1[i];
  }
  return n;
}

LM_API lm_status lm_debug_corr_work(const lm_ctx* ctx, int32_t* out) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  for (int k = 0; k < 4; ++k) out[k] = ctx->delivered.work[k];
  return LM_OK;
}

LM_API int32_t lm_debug_batch_slots(const lm_ctx* ctx) { return ctx ? ctx->delivered.slots : 0; }

LM_API int32_t lm_debug_dark_tile_width(void) { return LM_FW; }

LM_API int32_t lm_debug_dark_tile_height(void) { return LM_FH; }

namespace {
// The lane whose device buffers still hold the last collected batch's debug
// data (raw score maps, TAIL_MASK), or null: the data is gone once a newer
// batch was submitted to that lane (a retired batch's lane is reused at once).
const Lane* delivered_lane(const lm_ctx* ctx) {
  const lm_ctx::BatchRec& D = ctx->delivered;
  if (D.ran_lane < 0 || D.ran_lane >= (int)ctx->lanes.size()) return nullptr;
  const Lane& L = *ctx->lanes[D.ran_lane];
  return (L.done_seq == D.seq && L.seq < 0) ? &L : nullptr;
}
const char* kLaneReused =
    "the collected batch's lane already runs a newer batch, so its debug data is gone: collect it before submitting "
    "more batches (or use one pipeline lane)";
}  // namespace

LM_API lm_status lm_debug_scores(lm_ctx* ctx, int32_t f, int32_t det, float* out, int32_t rows, int32_t cols) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  const Lane* Lp = delivered_lane(ctx);
  if (!Lp) return fail(LM_ERR_INVALID_ARGUMENT, kLaneReused);
  const Lane& L = *Lp;
  if (!(ctx->debug & 1) || !L.dbg.p) return fail(LM_ERR_INVALID_ARGUMENT, "debug scores not enabled");
  if (f < 0 || f >= L.batch_n || det < 0 || det >= LM_NDET) return fail(LM_ERR_INVALID_ARGUMENT, "index out of range");
  const LmDet& D = ctx->K.det[det];
  if (rows != D.oh || cols != D.ow) return fail(LM_ERR_INVALID_ARGUMENT, "shape mismatch");
  return guarded([&] {
    HIPCHK(hipSetDevice(ctx->device));
    COPY_SYNC(out, L.dbg.p + (int64_t)(f + 1) * ctx->dbg_slot_floats + ctx->dbg_off[det], sizeof(float) * rows * cols,
              hipMemcpyDeviceToHost, L.stream);
  });
}

LM_API lm_status lm_debug_tail_mask(lm_ctx* ctx, int32_t f, uint8_t* out, int32_t rows, int32_t cols) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  const Lane* Lp = delivered_lane(ctx);
  if (!Lp) return fail(LM_ERR_INVALID_ARGUMENT, kLaneReused);
  const Lane& L = *Lp;
  if (f < 0 || f >= L.batch_n) return fail(LM_ERR_INVALID_ARGUMENT, "index out of range");
  if (rows != ctx->K.tail_hb || cols != ctx->K.tail_w) return fail(LM_ERR_INVALID_ARGUMENT, "shape mismatch");
  return guarded([&] {
    HIPCHK(hipSetDevice(ctx->device));
    const int nb = (cols + 63) / 64;
    std::vector<unsigned long long> bits((size_t)rows * nb);
    COPY_SYNC(bits.data(), L.tailmask.p + (int64_t)(f + 1) * rows * nb, bits.size() * 8, hipMemcpyDeviceToHost, L.stream);
    for (int r = 0; r < rows; ++r)
      for (int x = 0; x < cols; ++x) out[(size_t)r * cols + x] = ((bits[(size_t)r * nb + (x >> 6)] >> (x & 63)) & 1) ? 255 : 0;
  });
}

LM_API int32_t lm_debug_kernel_times(lm_ctx* ctx, const char** names, double* ms, int32_t cap) {
  if (!ctx) return 0;
  const lm_ctx::BatchRec& L = ctx->delivered;
  const int32_t n = (int32_t)L.t_names.size();
  for (int32_t i = 0; i < n && i < cap; ++i) {
    if (names) names[i] = L.t_names[i];
    if (ms) ms[i] = L.t_ms[i];
  }
  return n;
}

// ------------------------------------------------------- synthetic source
#include "lm_synth.h"

__global__ void k_synth(uint8_t* __restrict__ out, lm_synth_scene sc, int64_t first, int64_t pitch) {
  const int64_t f = blockIdx.y;
  const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int64_t np = (int64_t)sc.rows * sc.cols;
  if (q >= np) return;
  uint32_t w = 0;
  for (int k = 0; k < 4 && q + k < np; ++k) {
    const int64_t p = q + k;
    w |= (uint32_t)lm_synth_pixel(&sc, first + f, (int32_t)(p / sc.cols), (int32_t)(p % sc.cols)) << (8 * k);
  }
  uint8_t* o = out + f * pitch + q;
  if (q + 4 <= np && ((uintptr_t)o & 3) == 0) {
    *reinterpret_cast<uint32_t*>(o) = w;
  } else {
    for (int k = 0; k < 4 && q + k < np; ++k) o[k] = (uint8_t)(w >> (8 * k));
  }
}

LM_API lm_status lm_host_alloc(size_t bytes, void** out) {
  return guarded([&] {
    if (!out) throw std::invalid_argument("lm_host_alloc: out is NULL.");
    *out = nullptr;
    HIPCHK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
  });
}

LM_API void lm_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

LM_API lm_status lm_synth_frames_device(int32_t device, uint8_t* d_out, int32_t rows, int32_t cols, int64_t first_frame,
                                        int32_t n, int64_t frame_pitch) {
  if (!d_out || rows <= 0 || cols <= 0 || n <= 0 || frame_pitch < (int64_t)rows * cols)
    return fail(LM_ERR_INVALID_ARGUMENT, "bad synth arguments");
  return guarded([&] {
    HIPCHK(hipSetDevice(device));
    const lm_synth_scene sc = lm_synth_default_scene(rows, cols);
    const int64_t np = (int64_t)rows * cols;
    k_synth<<<dim3((unsigned)((np / 4 + 255) / 256 + 1), n), 256>>>(d_out, sc, first_frame, frame_pitch);
    HIPCHK(hipGetLastError());
    HIPCHK(hipDeviceSynchronize());
  });
}

// k_minmax + k_lut for the whole-video BB pass (lm_bbox.hip, its own translation unit)
hipError_t launch_minmax_lut(const uint8_t* const* frame_ptr, const uint8_t* bkg, int npix, int s0, int n,
                             unsigned* mm, const uint8_t* adj, int use_adj, uint8_t* luts, hipStream_t st) {
  k_minmax<<<dim3(LM_MM_SPLIT, n - s0), LM_MM_THREADS, 0, st>>>(frame_ptr, bkg, npix, s0, mm);
  k_lut<<<(n - s0 + 3) / 4, 256, 0, st>>>(mm, s0, n, adj, use_adj, luts);
  return hipGetLastError();
}
