/*
 * lm_device.h — layouts shared by the gfx950 kernels (lm_kernels.hip) and the
 * host runtime (lm_runtime.hip).
 *
 * Device-memory layout of one batch ("slots"): slot 0 is the previous frame
 * (carried from the last batch or run as a 1-frame halo), slots 1..B are the
 * frames of the batch.  Everything per slot is laid out slot-major so one
 * launch covers a whole batch.
 */
#ifndef LM_DEVICE_H
#define LM_DEVICE_H

#include <stdint.h>

// Correlation tile width (k_corr_rw: 80 x 16 per wave; k_corr_gen: 80 x 48
// per 192-thread workgroup, 16 x 12 threads of LM_C x 4 outputs).
#define LM_C 5
#define LM_R 3
#define LM_TW (16 * LM_C)  // 80
#define LM_TH (16 * LM_R)  // 48
#define LM_JC 4            // tap chunk along a detector row (kw padded to a multiple)
// The dark-tile grid: LM_FW x LM_FH output tiles (40 x 4; 40 x 8 and 80 x 8
// as build options).  k_corr_rw's wave computes LM_RW_NQ independent
// sub-tiles of that size (the LM_RW_NQX x LM_RW_NQY sub-tiles of an 80 x 16
// tile, or as many bright tiles from the lists), LM_FW / 5 x LM_FH / 4
// threads each.
#ifndef LM_FW
#define LM_FW 40
#endif
#ifndef LM_FH
#define LM_FH 4
#endif
static_assert((LM_FW == 40 || LM_FW == 80) && (LM_FH == 4 || LM_FH == 8), "dark-tile grid");
#define LM_RW_NQX (LM_TW / LM_FW)
#define LM_RW_NQY (16 / LM_FH)
#define LM_RW_NQ (LM_RW_NQX * LM_RW_NQY)
// k_ingest: frames per workgroup (the calibration / background loads are
// reused across them); its workgroups of slot group y append their bright
// tiles to list segment (y LM_TL_NC) / G of their view (G slot groups), one
// counter per segment: ~40 bands per counter instead of every workgroup of
// the batch on one address (same-address atomics serialise in L2: 52 -> 38 us
// per batch without them, profiles/r04/ingest/)
#ifndef LM_INGEST_FB
#define LM_INGEST_FB 8
#endif
#define LM_TL_NC 64
// first slot group of list segment c (G slot groups): the segment holds the
// tiles of slot groups y0(c) .. y0(c + 1) - 1
__host__ __device__ inline int lm_tl_y0(int c, int G) { return (c * G + LM_TL_NC - 1) / LM_TL_NC; }

// k_minmax: each frame split over LM_MM_SPLIT workgroups of LM_MM_THREADS
#define LM_MM_SPLIT 8
#define LM_MM_THREADS 256

#define LM_NDET 6
#define LM_NLIST 4
#define LM_NFEAT 2

// detector ids (also debug ids of lm_debug_scores)
enum { DET_PAW_B = 0, DET_SNOUT_B = 1, DET_TAIL_B = 2, DET_PAW_S = 3, DET_SNOUT_S = 4, DET_TAIL_S = 5 };
// list ids (lm_batch_result order)
enum { LIST_PAW_B = 0, LIST_SNOUT_B = 1, LIST_PAW_S = 2, LIST_SNOUT_S = 3 };

struct LmDet {
  int32_t view;      // 0 bottom, 1 side
  int32_t kind;      // 0 point detector (list), 1 tail detector (binary map)
  int32_t list;      // list id for kind 0, 0/1 (bottom/side) for kind 1
  int32_t kh, kw, kwp;
  int32_t kw_ring;  // k_corr_rw width that runs it: kw, or a wider one <= kwp that another detector uses
  int32_t w_off;     // float offset of the kh x kwp zero-padded weights
  float delta;       // (float)(-rho): filter2D delta (LocoMouse_class.cpp:845)
  int32_t oh, ow;    // consumed output region (UNPAD)
  int32_t in_y, in_x;  // ext-crop coords of tap (0,0) of output (0,0)
  int32_t m_y, m_x;    // ext-crop coords of the I_*_MOUSE pixel of output (0,0)
  int32_t tiles_x, tiles_y, tile_base;
  int32_t tile_w, tile_h;  // output columns / rows per correlation tile (LM_TW x LM_TH; f16 mode 128 x 64)
  int32_t box_w, box_h;  // NMS box (detector cols, rows)
  int32_t chunk_rows;    // k_corr_gen: detector rows per LDS window
  // LM_CORR_F16: f16 weight rows (kh x f16_wrow, zero-padded) at w16_off
  // halfs, scaled by wscale = 2^s (inv_wscale = 2^-s, both exact)
  int32_t w16_off;
  float wscale, inv_wscale;
};

struct LmConst {
  LmDet det[LM_NDET];
  int32_t n_tiles;
  // per view (0 bottom, 1 side): extended crop (all taps of all detectors)
  int32_t ext_h[2], ext_w[2];
  int32_t ext_oy[2], ext_ox[2];  // origin relative to the padded crop (BB_*_MOUSE_PAD)
  int32_t crop_h[2], crop_w[2];  // padded crop size
  int32_t unpad_y[2], unpad_x[2];  // BB_UNPAD_MOUSE_* offset inside the padded crop
  // images
  int32_t video_rows, video_cols;
  int32_t n_rows, n_cols;  // corrected image (calibration) size
  int32_t pad_pre_rows, pad_pre_cols, ipad_rows, ipad_cols;
  int32_t flip;
  // tail
  int32_t tail_w, tail_hb, tail_hs;  // tail box width, bottom/side heights
  int32_t tail_cap, tail_ntc;        // k_tail: runs held in LDS, 32-column tiles per segment
  // tail detector maps (filter2D > 0) as bitmaps, bottom then side per slot:
  // rows of tail_nw u32 words (tail_nw = 2 * ceil(tail_w / 64), so a row is
  // also ceil(tail_w / 64) u64 words); set by k_corr, zeroed by k_ingest
  int32_t tail_nw, tail_bm_words;
  int32_t connectivity;
  // dark tiles (flagged and listed by k_ingest): per view, the point
  // detectors' outputs in LM_FW x LM_FH tiles (fl_tx x fl_ty of them); one
  // flag byte per (slot, view, tile) at slot * fl_slot + fl_off[view] + tile;
  // the bright tiles of view v listed at v * tl_stride of the tile list, in
  // LM_TL_NC segments: segment c at lm_tl_y0(c, G) * LM_INGEST_FB * fl_tx * fl_ty
  int32_t fl_tx[2], fl_ty[2], fl_off[2], fl_slot;
  int32_t tl_stride;
  // the point detectors' output region per view: output (y, x) has its
  // I_*_MOUSE pixel at ext (fl_my + y, fl_mx + x); fl_oh x fl_ow outputs
  int32_t fl_my[2], fl_mx[2], fl_oh[2], fl_ow[2];
  // k_ingest: 8-row bands of each view's ext crop aligned with the flag grid
  // (band b = ext rows fl_my + 8b ..), bands ing_b0[v] .. ing_b0[v] +
  // ing_nb[v] - 1, one workgroup of ing_threads per (band, slot group)
  int32_t ing_b0[2], ing_nb[2], ing_threads;
  // per-list capacities (= output area) and list offsets inside a slot's key area
  int32_t list_cap[LM_NLIST];
  int64_t list_off[LM_NLIST];
  int64_t keys_per_slot;
  // matching / costs (config.yml)
  double side_bottom_min_overlap;
  double alpha_vel_bottom, pairwise_occluded_cost;
  int32_t max_displacement_bottom, ong_spacing_bottom;
  int32_t ong_nx, ong_ny;
  double ong_br_x, ong_br_y;
  int32_t bb_bottom_w, bb_bottom_h;
  int32_t spre_b_w, spre_b_h, spre_t_w, spre_t_h;
  int32_t match_b[LM_NFEAT][4];  // match_box_bottom x,y,w,h (paw, snout)
  int32_t match_s[LM_NFEAT][4];
  int32_t size_b[LM_NFEAT][2];   // detector (cols, rows) bottom
  int32_t size_s[LM_NFEAT][2];   // side
  double prior[5][7];            // location_prior rows
  // transform_gray_values with a CV_8U table: LUT applied in place to the
  // bottom crop (LocoMouse_class.cpp:1445-1448)
  int32_t gray_lut_on;
  uint8_t gray_lut[256];
};

// per-slot frame info (uploaded per batch)
struct LmSlot {
  int32_t crop_x[2], crop_y[2];  // padded crop top-left in I_PAD coords (bottom, side)
  int32_t frame;                 // global frame index (CURRENT_FRAME)
  int32_t active;                // 1 when the slot is processed in this batch
};

// per-slot output header (device -> host)
struct LmSlotOut {
  int32_t n_pos[LM_NLIST];       // positive detections (after masking)
  int32_t cand_off[LM_NLIST];    // into the candidate arena
  int32_t cand_cnt[LM_NLIST];
  int32_t p22d_off[LM_NFEAT], p22d_cnt[LM_NFEAT];
  int32_t side_off[LM_NFEAT], side_cnt[LM_NFEAT];
  int32_t unary_off[LM_NFEAT], unary_cnt[LM_NFEAT];
  int32_t pw_rows[LM_NFEAT], pw_cols[LM_NFEAT], pw_nnz[LM_NFEAT];
  int32_t pw_jc_off[LM_NFEAT], pw_nz_off[LM_NFEAT];
  int32_t tail[45];
  int32_t ties[LM_NLIST];        // 1 when the exact-tie std::sort replica ran
  int32_t bottom_kept[LM_NFEAT]; // k_tail: some bottom key of the feature survives TAIL_MASK (k_nms' side skip)
  int32_t pad_[1];
};

// arena counters (device -> host)
enum { AR_CAND = 0, AR_P22D, AR_SIDE, AR_UNARY, AR_PWJC, AR_PWNZ, AR_COUNT };
// Each arena is split into nparts = min(LM_SUBARENA, k_post blocks) equal
// parts with their own bump counters (one 128-byte line each), so the blocks
// of a batch do not all queue on one cache line of atomics; a (slot, feature)
// block allocates from part (block % nparts).  `used` is filled by
// k_pack_scan with what the fullest part implies for the whole arena
// (nparts x its count), which is what the host grows the capacity to after
// an overflow.
#define LM_SUBARENA 16
struct LmArenaCtl {
  int32_t used[AR_COUNT];
  int32_t cap[AR_COUNT];
  int32_t overflow;
  int32_t nparts;                  // parts in use this batch (set by the host)
  uint8_t* pack_dst;               // the batch's pinned result buffer (device view) and its size:
  int64_t pack_cap;                //   k_out reads them here, so a captured graph takes any buffer
  int32_t sub[LM_SUBARENA][32];  // sub[g][k]: part g's count of arena k (k < AR_COUNT)
};

struct LmCand {  // == lm_candidate / Candidate
  int32_t x, y;
  double s;
};

struct LmP22D {  // == lm_p22d
  LmCand bottom;
  int32_t side_off;
  int32_t side_cnt;
};

// Candidate staging: k_nms writes the candidates of (slot, list) over that
// list's key area (list_cap[l] u64 = room for list_cap[l]/2 candidates),
// after it has read the keys.  k_post reads them there; k_pack packs them.
#define LM_CAND_STAGE(K, keys, slot, list) \
  ((LmCand*)((keys) + (int64_t)(slot) * (K).keys_per_slot + (K).list_off[list]))

// Packed per-batch results, laid out exactly as lm_batch_result's arrays
// (frame order), so the host does one D2H and hands out pointers.
enum { PK_CAND = 0, PK_P22D, PK_SIDE, PK_UNARY, PK_JC, PK_NZ, PK_COUNT };
struct LmPackHdr {
  int64_t tot[PK_COUNT];
  int64_t bytes;        // packed size for this batch
  int32_t overflow;     // bit0: pack buffer too small, bit1: staging arena overflow
  int32_t err;          // copy of the kernels' error bits
  int32_t used[AR_COUNT];
  int32_t pad_[2];
};

struct LmPackLayout {  // byte offsets inside the packed buffer
  int64_t cand_off, p22d_off, unary_off, jc_off, nz_off, pw_dims, tail;
  int64_t cand, p22d, side_y, side_s, unary, jc, ir, pr, bytes;
};

#if defined(__HIPCC__)
__host__ __device__
#endif
inline LmPackLayout lm_pack_layout(int n, const int64_t* tot) {
  LmPackLayout L;
  int64_t o = 0;
  auto take = [&o](int64_t bytes) {
    const int64_t r = o;
    o += (bytes + 15) / 16 * 16;
    return r;
  };
  L.cand_off = take(8 * (4 * (int64_t)n + 1));
  L.p22d_off = take(8 * (2 * (int64_t)n + 1));
  L.unary_off = take(8 * (2 * (int64_t)n + 1));
  L.jc_off = take(8 * (2 * (int64_t)n + 1));
  L.nz_off = take(8 * (2 * (int64_t)n + 1));
  L.pw_dims = take(4 * 6 * (int64_t)n);
  L.tail = take(4 * 45 * (int64_t)n);
  L.cand = take(16 * tot[PK_CAND]);
  L.p22d = take(24 * tot[PK_P22D]);
  L.side_y = take(4 * tot[PK_SIDE]);
  L.side_s = take(8 * tot[PK_SIDE]);
  L.unary = take(8 * tot[PK_UNARY]);
  L.jc = take(4 * tot[PK_JC]);
  L.ir = take(4 * tot[PK_NZ]);
  L.pr = take(8 * tot[PK_NZ]);
  L.bytes = o;
  return L;
}

#endif  // LM_DEVICE_H
