/*
 * locomouse_hip.h — C-ABI of the MI355X-native LocoMouse per-frame detection path.
 *
 * This is the drop-in boundary between host code that keeps the reference's
 * `LocoMouse` call surface (LocoMouse_class.hpp:169-350, main.cpp:54-82) and the
 * hand-written gfx950 HIP kernels in liblocomouse_hip.so.  Plain C types only:
 * no OpenCV, no torch, no HIP types in any signature.
 *
 * What each entry point replaces in the reference (paths relative to the
 * reference root):
 *
 *   lm_ctx_create         LocoMouse::LocoMouse  LocoMouse_class.cpp:307-345 (parameters
 *                         already parsed), LocoMouse_Model ctor :3095-3162 and the
 *                         geometry of LocoMouse::initializeFeatureLoop :655-769.
 *   lm_detect_submit /    the same, pipelined: up to lm_setup.pipeline_lanes batches of
 *   lm_detect_collect     consecutive frames in flight on their own HIP streams
 *                         (main.cpp:54-82 runs the frames one after another; results
 *                         come back in the same order).
 *   lm_detect_batch       one iteration of the per-frame loop main.cpp:57-80, for n
 *                         consecutive frames:  readFrame :1273-1333 (+ LocoMouse_TM::
 *                         readFrame TM.cpp:243-249), cropBoundingBox :1408-1478,
 *                         detectTail :2541-2767, detectBottomCandidates :771-807 +
 *                         :841-854 + nmsMax :1610-1747, computeUnaryCostsBottom
 *                         :873-894 + :1909-1952, computePairwiseCostsBottom :896-919 +
 *                         :1954-2070, detectSideCandidates :809-838 + :856-870 +
 *                         peakClustering :1749-1905, matchBottomSideCandidates
 *                         :999-1267 and storePreviousImage :1508-1513.
 *   lm_candidate          Candidate (Candidates.hpp:16-34) — byte-identical layout.
 *   lm_p22d + side arrays P22D (Candidates.hpp:63-105).
 *   unary / pw_* arrays   MyMat (column-major doubles, MyMat.cpp:64-70) and
 *                         MATSPARSE (MATLAB CSC, MyMat.cpp:141-178).
 *   lm_status + lm_last_error   the std::invalid_argument / std::runtime_error
 *                         exceptions caught at main.cpp:94-101.
 *
 * Threading: one context per (device, host thread); a context is not re-entrant.
 * Results returned through lm_batch_result are owned by the context and stay
 * valid until the next lm_detect_* call on it or lm_ctx_destroy.
 */
#ifndef LOCOMOUSE_HIP_H
#define LOCOMOUSE_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LM_ABI_VERSION 6  /* 6: lm_debug_dark_tile_width / _height (40 x 4 dark tiles); 5: lm_debug_batch_slots */
#define LM_N_PAWS 4          /* LocoMouse_class.hpp:84 */
#define LM_N_TAIL_POINTS 15  /* LocoMouse_class.hpp:86 */
#define LM_N_LISTS 4         /* candidate lists per frame */
#define LM_N_FEATURES 2      /* paw, snout */

typedef enum {
  LM_OK = 0,
  LM_ERR_INVALID_ARGUMENT = 1, /* reference: std::invalid_argument            */
  LM_ERR_RUNTIME = 2,          /* reference: std::runtime_error / cv asserts  */
  LM_ERR_HIP = 3               /* HIP runtime failure (no reference analogue) */
} lm_status;

/* cv::Rect */
typedef struct {
  int32_t x, y, width, height;
} lm_rect;

/* One row of config.yml `location_prior` (LocoMouse_class.cpp:132-145):
 * [x y max_distance min_x max_x min_y max_y]. */
typedef struct {
  double x, y, max_distance, min_x, max_x, min_y, max_y;
} lm_location_prior;

/* config.yml keys the per-frame path reads (LocoMouse_class.cpp:18-249;
 * defaults LocoMouse_class.hpp:53-74).  Keys that only feed the whole-video
 * bounding-box pass (median_filter_size, min_pixel_visible,
 * moving_average_window, the TM zero_* / bb_* keys) are in lm_bb_params. */
typedef struct {
  int32_t conn_comp_connectivity;               /* 4 or 8 */
  int32_t max_displacement_bottom;
  int32_t max_displacement_side;
  int32_t occlusion_grid_spacing_pixels_side;
  int32_t occlusion_grid_spacing_pixels_bottom;
  int32_t use_provided_bounding_box;            /* must be 1: a computed box (lm_bb_*) is passed as
                                                   its sizes here + per-frame corners (bb) */
  int32_t transform_gray_values;                /* LUT on the bottom crop, :1445-1454 (see below) */
  int32_t use_reference_image_brightness;       /* histogram matching, :1437-1443 (see below) */
  double side_bottom_min_overlap;
  double occlusion_grid_max_width;
  double tail_sub_bounding_box;
  double alpha_vel_bottom;
  double alpha_vel_side;
  double pairwise_occluded_cost;
  lm_location_prior location_prior[5];          /* rows 0-3 paws, row 4 snout */
  lm_rect bounding_box_side;                    /* bounding_box_side  (x y w h) */
  lm_rect bounding_box_bottom;                  /* bounding_box_bottom (x y w h) */
  float gray_value_transformation[256];         /* used iff transform_gray_values */
  int32_t gray_value_transformation_depth;      /* OpenCV depth of that matrix as read from config.yml
                                                   (dt u -> LM_DEPTH_8U, f -> LM_DEPTH_32F, ...) */
} lm_params;
/* Grey-level options, as the reference executes them:
 *  - use_reference_image_brightness: LocoMouse_Parameters computes the
 *    reference CDF with computeNormalizedCDF into an unallocated cv::Mat
 *    (:189, :3392-3405: ptr<float>(0) of an empty Mat), so the reference
 *    cannot start with it set; lm_ctx_create fails with LM_ERR_RUNTIME.
 *  - transform_gray_values: LUT(I_BOTTOM_MOUSE, table, I_BOTTOM_MOUSE)
 *    (:1445-1448).  A CV_8U table (depth LM_DEPTH_8U, values 0..255) keeps
 *    the type, so the LUT is applied in place to the bottom crop of I_PAD:
 *    every later step of that frame (tail, masks, both views where they
 *    overlap the crop) and the next frame's motion test (I_PREV_PAD) see the
 *    transformed pixels — supported.  Any other table depth re-creates the
 *    crop with the table's type and a later threshold / Mat::setTo(0, mask)
 *    asserts (:782, :849): lm_ctx_create fails with LM_ERR_RUNTIME, as the
 *    reference would stop.  The in-place LUT also reaches the zero padding
 *    of I_PAD when a frame's bottom crop leaves the corrected image, and the
 *    reference keeps those transformed pad pixels across frames; batches
 *    with such a frame fail with LM_ERR_INVALID_ARGUMENT (never the case
 *    with a provided bounding box, which must lie inside the image). */
#define LM_DEPTH_8U 0
#define LM_DEPTH_8S 1
#define LM_DEPTH_16U 2
#define LM_DEPTH_16S 3
#define LM_DEPTH_32S 4
#define LM_DEPTH_32F 5
#define LM_DEPTH_64F 6

/* One linear detector (model.yml modelX_view / biasX_view, :3106-3148).
 * Weights are row-major doubles as read from the model file; they are rounded
 * to float exactly as cv::filter2D does with a CV_64F kernel on CV_8U input. */
typedef struct {
  const double* weights;
  int32_t rows, cols;
  double bias;
} lm_detector;

typedef struct {
  lm_detector paw_bottom, paw_side;
  lm_detector snout_bottom, snout_side;
  lm_detector tail_bottom, tail_side;
} lm_model;

/* Video/background/calibration description (loadVideo/loadBackground/
 * loadCalibration/loadFlip, :367-484). */
typedef struct {
  int32_t method;                 /* 0 LocoMouse, 1 LocoMouse_TM, 2 LocoMouse_TM_DE (Methods.cpp:3-26) */
  int32_t flip;                   /* 1 when the side character is 'L' (:471-473) */
  int32_t video_rows, video_cols; /* raw frame size (channel 0 of the decoded frame) */
  const uint8_t* background;      /* video_rows x video_cols, row-major, copied at create */
  int32_t calib_rows, calib_cols; /* N_ROWS x N_COLS of ind_warp_mapping */
  const int32_t* ind_warp_mapping;/* calib_rows x calib_cols, copied at create */
  lm_rect view_box_side, view_box_bottom;
  int32_t filter_arith;           /* LM_FILTER_FUSED (default) or LM_FILTER_UNFUSED, see below */
  int32_t corr_precision;         /* LM_CORR_FP32 (default, bit-exact) or LM_CORR_F16, see below */
  int32_t pipeline_lanes;         /* batches in flight at once (lm_detect_submit); 0 = 1, at most LM_MAX_LANES */
} lm_setup;
#define LM_MAX_LANES 16
/* filter2D's fp32 tap arithmetic depends on the OpenCV build the reference
 * links (no version is pinned, CMakeLists.txt:3): AVX2 builds of OpenCV
 * >= 3.4.9 fuse each tap (fma), SSE2/scalar builds round the product and then
 * the sum.  Pick the one matching the installation being replaced; both are
 * bit-exact against the restatement of that build (tests/test_gpu_parity.py). */
#define LM_FILTER_FUSED 0
#define LM_FILTER_UNFUSED 1
/* LM_CORR_F16 is a NON-PARITY mode (BASELINE config 5, "fp16 correlation
 * accumulators"): the six correlations run on f16 matrix cores with each
 * detector's weights rounded to f16 (after an exact power-of-two scaling) and
 * fp32 accumulation.  Pixels are exact; scores differ from the fp32 chain by
 * the weight rounding (about 2^-12 relative per tap) and the summation order,
 * so candidates near a threshold or a score tie can differ.  filter_arith is
 * ignored in this mode.  Detectors must fit the kernel's LDS window
 * (LM_ERR_INVALID_ARGUMENT otherwise); lm_debug_scores still returns the
 * fp32 chain. */
#define LM_CORR_FP32 0
#define LM_CORR_F16 1

/* Geometry derived at create time (initializeFeatureLoop :655-769 and the
 * LocoMouse_Model pads :3157-3161 incl. the spost_b = spre_b move-assign at :3173). */
typedef struct {
  int32_t n_rows, n_cols;
  int32_t pad_pre_rows, pad_pre_cols, pad_post_rows, pad_post_cols;
  int32_t ipad_rows, ipad_cols;
  int32_t spre_b_w, spre_b_h, spost_b_w, spost_b_h;
  int32_t spre_t_w, spre_t_h, spost_t_w, spost_t_h;
  lm_rect bb_bottom_mouse, bb_side_mouse;
  lm_rect bb_bottom_mouse_pad, bb_side_mouse_pad;     /* x,y = 0; placed per frame */
  lm_rect bb_unpad_mouse_bottom, bb_unpad_mouse_side;
  lm_rect bb_bottom_tail_pad, bb_unpad_tail_bottom, bb_bottom_tail;
  lm_rect bb_side_tail_pad, bb_unpad_tail_side;
  int32_t tail_box_width;
  int32_t ong_nx, ong_ny;                             /* ONG_size */
  double ong_br_x, ong_br_y;                          /* ONG_BR_corner */
  int32_t n_ong_side, ong_side_lowest;
  lm_rect match_box_paw_bottom, match_box_paw_side;   /* LocoMouse_Feature :2954-2969 */
  lm_rect match_box_snout_bottom, match_box_snout_side;
} lm_geometry;

/* Candidate: {Point_<int> p; double s;} — x@0, y@4, score@8 (16 bytes). */
typedef struct {
  int32_t x, y;
  double score;
} lm_candidate;

/* P22D: bottom candidate + the raw yt/st vectors (always >= 1 entry; the
 * "no side match" state is st[0] < 0, Candidates.cpp:148-156). */
typedef struct {
  lm_candidate bottom;
  int32_t side_offset;  /* into side_y / side_s */
  int32_t side_count;   /* yt.size() */
} lm_p22d;

/* Per-batch results, in frame order.  List k of frame f (k: 0 bottom paw,
 * 1 bottom snout, 2 side paw, 3 side snout) is cand[cand_offset[4f+k] ..
 * cand_offset[4f+k+1]).  Feature k (0 paw, 1 snout) of frame f owns
 * p22d[p22d_offset[2f+k] ..), unary[unary_offset[2f+k] ..) (column-major,
 * N_cand x 4 for paws, N_cand x 1 for the snout) and one MATSPARSE when its
 * global frame index is > 0 (pw_dims[3(2f+k)+0] = n_rows, +1 = n_cols,
 * +2 = nnz; n_rows = -1 when absent).  tail holds 3x15 int32 per frame
 * (rows x, y, z; -1 = missing). */
typedef struct {
  int32_t n_frames;
  int32_t first_frame;
  const int64_t* cand_offset;   /* [4n+1] */
  const lm_candidate* cand;
  const int64_t* p22d_offset;   /* [2n+1] */
  const lm_p22d* p22d;
  const int32_t* side_y;
  const double* side_s;
  const int64_t* unary_offset;  /* [2n+1] */
  const double* unary;
  const int32_t* pw_dims;       /* [2n][3] */
  const int64_t* pw_jc_offset;  /* [2n+1] */
  const int32_t* pw_jc;
  const int64_t* pw_nz_offset;  /* [2n+1] */
  const int32_t* pw_ir;
  const double* pw_pr;
  const int32_t* tail;          /* [n][3][15] */
} lm_batch_result;

typedef struct lm_ctx lm_ctx;

/* Library identity. */
int32_t lm_abi_version(void);

/* Error text of the last failing call on this thread (create errors
 * included).  Never NULL. */
const char* lm_last_error(void);

/* Create a context on HIP device `device`.  Copies background, calibration and
 * model weights to the device.  max_batch bounds n in lm_detect_batch*.
 * Fails with LM_ERR_INVALID_ARGUMENT on the reference's validation errors
 * (:35-249, :486-540, :3097-3140) and on use_provided_bounding_box == 0.
 * Contexts share no state; several may run concurrently from different host
 * threads.  setup->pipeline_lanes HIP streams are created (each with its own
 * per-batch buffers, about 0.5 GB at 1024x256 and max_batch 256).  Results
 * never depend on how many contexts or lanes exist, but two scheduling
 * choices do: lanes alternate between the highest and the lowest HIP stream
 * priority, and a lane alone on its device runs its correlation widths in
 * one launch (several lanes: one launch per width). */
lm_status lm_ctx_create(int32_t device, const lm_setup* setup, const lm_params* params,
                        const lm_model* model, int32_t max_batch, lm_ctx** out);
void lm_ctx_destroy(lm_ctx* ctx);

lm_status lm_get_geometry(const lm_ctx* ctx, lm_geometry* out);

/* The ctx's first lane's HIP stream (hipStream_t as void*), for event timing by callers. */
void* lm_ctx_stream(lm_ctx* ctx);

/* Run frames [first_frame, first_frame + n) through the per-frame path.
 * frames: host memory, n raw frames of video_rows x video_cols u8 at
 * frame_pitch bytes apart.  bb: NULL for the provided bounding box (the only
 * mode on this path), else per-frame bottom-right corners [n'][3] = {x,
 * y_bottom, y_side} (LocoMouse_class.cpp:547-557), n' = n (+1 if prev_frame).
 * prev_frame: the raw frame first_frame-1 when the context did not process it
 * in its previous call (shard start); it is run as a 1-frame halo and its own
 * results are not returned.  NULL continues from the context state (or starts
 * the video when first_frame == 0). */
lm_status lm_detect_batch(lm_ctx* ctx, const uint8_t* frames, int64_t frame_pitch,
                          int32_t n, int32_t first_frame, const uint8_t* prev_frame,
                          const int32_t* bb, lm_batch_result* out);

/* Same, with frames (and prev_frame) already resident in device memory of the
 * context's device.  Results are copied back to host memory owned by ctx. */
lm_status lm_detect_batch_device(lm_ctx* ctx, const uint8_t* d_frames, int64_t frame_pitch,
                                 int32_t n, int32_t first_frame, const uint8_t* d_prev_frame,
                                 const int32_t* bb, lm_batch_result* out);

/* Pipelined form of lm_detect_batch*: up to pipeline_lanes batches in flight.
 * Submit puts batch [first_frame, first_frame + n) on the next free lane and
 * returns once its inputs are staged (host frames are copied before it
 * returns, so the caller may reuse its buffer; device frames -- and a device
 * prev_frame -- must stay unchanged until the batch is collected).  Batches
 * follow each other as in lm_detect_batch (contiguous frames, or prev_frame at
 * a shard start).  A batch continuing another lane's batch takes that batch's
 * last frame as a 1-frame halo copied on the device, so consecutive batches
 * run concurrently; results are bit-identical to one lane.  When every lane
 * is busy, submit waits for the first lane whose batch completes and reuses
 * it (that batch's results are kept until collected); with 2 x
 * pipeline_lanes batches waiting for collection it fails
 * (LM_ERR_INVALID_ARGUMENT): collect first.  Collect returns the OLDEST
 * submitted batch's results (valid until the next lm_detect_* call on the
 * context), waiting for it if needed; its errors are the ones
 * lm_detect_batch would report.  lm_detect_batch* require that no batch is
 * waiting. */
lm_status lm_detect_submit(lm_ctx* ctx, const uint8_t* frames, int64_t frame_pitch, int32_t n, int32_t first_frame,
                           const uint8_t* prev_frame, const int32_t* bb);
lm_status lm_detect_submit_device(lm_ctx* ctx, const uint8_t* d_frames, int64_t frame_pitch, int32_t n,
                                  int32_t first_frame, const uint8_t* d_prev_frame, const int32_t* bb);
lm_status lm_detect_collect(lm_ctx* ctx, lm_batch_result* out);
/* Lanes of the context / batches submitted and not yet collected (<= 2 x lanes). */
int32_t lm_ctx_lanes(const lm_ctx* ctx);
int32_t lm_ctx_pending(const lm_ctx* ctx);

/* ---- diagnostics (parity tests and benchmarks; not part of the reference surface) ---- */

/* flags: bit 0 keep raw filter2D score maps of the last batch;
 *        bit 1 record per-kernel HIP event timings;
 *        bit 4 force one correlation launch per detector width, bit 5 force
 *        one merged launch (otherwise chosen per batch; results are identical). */
lm_status lm_ctx_set_debug(lm_ctx* ctx, int32_t flags);

/* Copy the raw correlation scores (before masking) of detector det
 * (0 paw_b, 1 snout_b, 2 tail_b, 3 paw_s, 4 snout_s, 5 tail_s) for frame
 * index f of the last collected batch: UNPAD region, row-major, rows x cols
 * floats.  The maps live on the lane that ran the batch: once a newer batch
 * was submitted to that lane (pipelined contexts reuse a finished lane at
 * once) they are gone and this fails with LM_ERR_INVALID_ARGUMENT, as does
 * lm_debug_tail_mask. */
lm_status lm_debug_scores(lm_ctx* ctx, int32_t f, int32_t det, float* out, int32_t rows, int32_t cols);

/* Copy the bottom TAIL_MASK (0/255, tail_box_width x bottom height) of frame f. */
lm_status lm_debug_tail_mask(lm_ctx* ctx, int32_t f, uint8_t* out, int32_t rows, int32_t cols);

/* Kernel timings of the last batch when debug bit 1 is set: fills up to cap
 * (name, milliseconds) pairs; returns the number of kernels. */
int32_t lm_debug_kernel_times(lm_ctx* ctx, const char** names, double* ms, int32_t cap);

/* Same kernels as lm_debug_kernel_times, as [t0, t1] milliseconds since the
 * device's epoch event (recorded by the first lm_ctx_set_debug with bit 1 on
 * that device), so the spans of several contexts' streams can be merged. */
int32_t lm_debug_kernel_spans(lm_ctx* ctx, const char** names, double* t0, double* t1, int32_t cap);

/* Correlation work of the last collected batch when debug bit 1 is set:
 * out[0], out[1] = bright output tiles (the dark-tile grid's) of the
 * bottom / side point detectors, out[2], out[3] = the consumed outputs those
 * tiles hold.  The point detectors' dark tiles (no I_*_MOUSE pixel > 25, so
 * every score is zeroed by setTo(0, mask), LocoMouse_class.cpp:849, :864)
 * are not computed.  -1 when not recorded (timing off, LM_CORR_DARK=0). */
lm_status lm_debug_corr_work(const lm_ctx* ctx, int32_t* out);

/* The dark-tile grid: tiles of lm_debug_dark_tile_width() x
 * lm_debug_dark_tile_height() outputs (40 x 4 in the default build; 40 x 8
 * and 80 x 8 as build options, -DLM_FH=8 / -DLM_FW=80). */
int32_t lm_debug_dark_tile_width(void);
int32_t lm_debug_dark_tile_height(void);

/* Frame slots the last collected batch processed: n, or n + 1 when its halo
 * frame (slot 0: prev_frame, or the pipelined hand-off) was recomputed --
 * the slots lm_debug_corr_work's counts and the tail detectors cover. */
int32_t lm_debug_batch_slots(const lm_ctx* ctx);

/* ---- whole-video bounding-box pass ----
 *
 * Replaces the virtual computeBoundingBox of the three methods:
 *   method 0  LocoMouse::computeBoundingBox (LocoMouse_class.cpp:579-653) with
 *             computeMouseBox (:948-997), largestBWAreaObject (:921-946),
 *             firstLastOverT (LocoMouse_class.hpp:411-440), computeMouseBoxSize
 *             (:1481-1506), medianvec / stdvec / vecmovingaverage (:1516-1608);
 *   method 1  LocoMouse_TM::computeBoundingBox (LocoMouse_TM.cpp:115-157,
 *             computeMouseBox_DD :192-241);
 *   method 2  LocoMouse_TM_DE::computeBoundingBox (LocoMouse_TM_DE.cpp:8-113)
 *             with imadjust_default (LocoMouse_class.cpp:3244-3311).
 * Frames are pushed in video order (method 0's median filter carries its
 * zero-padded border from frame to frame, :585-603 + :952); lm_bb_finish
 * runs the whole-video post-processing.  The results feed the detection path
 * as lm_params.bounding_box_* sizes plus the per-frame `bb` corners of
 * lm_detect_batch. */

/* firstLastOverT reads the CV_32S row/column sums of methods 0 and 1 through
 * ptr<float> (LocoMouse_class.hpp:419), i.e. it compares the sums' bit
 * patterns as floats against min_pixel_visible.  AS_EXECUTED reproduces that
 * (the drop-in default); INTEGER compares the integer sums, as the comment at
 * :967-970 intends (method 0 only).  Method 2 sums in CV_32F and is unaffected. */
#define LM_BB_FIRSTLAST_AS_EXECUTED 0
#define LM_BB_FIRSTLAST_INTEGER 1

typedef struct {
  int32_t median_filter_size;     /* odd, 1..63 (config.yml, :41-45) — method 0 */
  int32_t min_pixel_visible;      /* >= 0 (:47-50) — methods 0, 1 */
  int32_t moving_average_window;  /* odd, >= 1 (:120-123) */
  int32_t conn_comp_connectivity; /* 4 or 8 (:33-39) — method 0 */
  int32_t firstlast_semantics;    /* LM_BB_FIRSTLAST_* */
  /* LocoMouse_TM config keys (TM.cpp:44-113, defaults TM.hpp:19-31) — method 1 */
  int32_t zero_col_pre, zero_col_post, zero_row_pre, zero_row_post;
  int32_t bb_width, bb_height_side;
  int32_t reserved0;
} lm_bb_params;

/* The six per-frame values of computeMouseBox, after :636
 * (bb_y_bottom += BB_BOTTOM_VIEW.y).  Methods 1 and 2 compute x only; their
 * y values are the fixed corners they assign (TM.cpp:140-141,
 * TM_DE.cpp:36-37) and the sizes are 0. */
typedef struct {
  double x, y_bottom, y_side, width, height_bottom, height_side;
} lm_bb_frame;

typedef struct {
  int32_t n_frames;
  int32_t reserved0;
  lm_rect bb_side_mouse, bb_bottom_mouse; /* computeMouseBoxSize (x = y = 0) */
  const uint32_t* x_pos;                  /* BB_X_POS[n_frames] (vecmovingaverage) */
  const uint32_t* y_bottom_pos;           /* BB_Y_BOTTOM_POS */
  const uint32_t* y_side_pos;             /* BB_Y_SIDE_POS */
  const lm_bb_frame* frames;              /* per-frame values [n_frames] */
} lm_bb_result;

typedef struct lm_bb_ctx lm_bb_ctx;

/* setup: as for lm_ctx_create; setup->method selects the pass.  The view
 * boxes must span the full corrected width (firstLastOverT reads N_COLS
 * sums) and, for method 0, must not overlap.  max_batch bounds n of
 * lm_bb_push*.  Method 1 supports LM_BB_FIRSTLAST_AS_EXECUTED only: its
 * result then depends on min_pixel_visible alone. */
lm_status lm_bb_create(int32_t device, const lm_setup* setup, const lm_bb_params* params, int32_t max_batch,
                       lm_bb_ctx** out);
void lm_bb_destroy(lm_bb_ctx* ctx);

/* Push the next n frames of the video (host memory / device memory).  out
 * (may be NULL) receives their lm_bb_frame values. */
lm_status lm_bb_push(lm_bb_ctx* ctx, const uint8_t* frames, int64_t frame_pitch, int32_t n, lm_bb_frame* out);
lm_status lm_bb_push_device(lm_bb_ctx* ctx, const uint8_t* d_frames, int64_t frame_pitch, int32_t n,
                            lm_bb_frame* out);

/* Post-processing over every frame pushed so far; arrays are owned by ctx and
 * valid until the next call on it.  Fails when no frame was pushed. */
lm_status lm_bb_finish(lm_bb_ctx* ctx, lm_bb_result* out);

/* Diagnostics: the thresholded median image (0/1, N_ROWS x N_COLS, before the
 * connected-component step) of frame f of the last push. */
lm_status lm_bb_debug_binary(lm_bb_ctx* ctx, int32_t f, uint8_t* out, int32_t rows, int32_t cols);

/* The ctx's HIP stream (hipStream_t as void*). */
void* lm_bb_stream(lm_bb_ctx* ctx);

/* Benchmark/test input utility (not a reference interface): writes frames
 * [first_frame, first_frame + n) of the synthetic scene of include/lm_synth.h
 * (rows x cols u8, frame_pitch bytes apart) into device memory of `device`. */
/* Page-locked host memory (hipHostMalloc) for batches of host frames: frames
 * in such a buffer reach the device by DMA at full PCIe rate, and a batch of
 * frames at a common pitch is copied in one 2-D transfer.  No reference
 * counterpart (the reference reads frames into a cv::Mat). */
lm_status lm_host_alloc(size_t bytes, void** out);
void lm_host_free(void* p);

lm_status lm_synth_frames_device(int32_t device, uint8_t* d_out, int32_t rows, int32_t cols, int64_t first_frame,
                                 int32_t n, int64_t frame_pitch);

#ifdef __cplusplus
}
#endif

#endif /* LOCOMOUSE_HIP_H */
