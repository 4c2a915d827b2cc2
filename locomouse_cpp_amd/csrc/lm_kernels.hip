// lm_kernels.hip — gfx950 kernels of the LocoMouse per-frame detection path.
//
// Batch pipeline (one launch each, grid over frame slots; see lm_device.h):
//   k_minmax      per-frame min/max of sat(F - BKG), frames split over workgroups
//   k_lut         -> normalize LUT (+ TM imadjust)
//                 LocoMouse_class.cpp:1304-1310, TM.cpp:247, :3204-3242
//   k_ingest      calibration gather + flip + LUT (+ the in-place grey-level LUT of
//                 transform_gray_values) -> extended padded crops (u8)
//                 :1316-1327 (correctImage :1337-1406), cropBoundingBox :1408-1478
//   k_corr        all six filter2D detectors, fp32 row-major FMA chains, LDS-tiled;
//                 epilogue: brightness mask + score>0 compaction / tail binarisation
//                 :845, :860, :2575-2576, :782, :817, :849, :864, :2593-2598
//   k_tail        largest connected component (bottom, then side AND column mask),
//                 TAIL_MASK, 15-segment binary moments  :2558-2767
//   k_nms         tail-mask filter, sort (bitonic; libstdc++ introsort replica on
//                 exact ties), nmsMax (bottom) / peakClustering (side)  :1610-1905
//   k_post        unary costs, pairwise CSC, side<->bottom matching with the
//                 motion criterion  :873-919, :999-1267, :1909-2070
//   k_carry       previous frame's bottom candidates into slot 0 of the next batch
//
// All floating-point code is compiled with -ffp-contract=off; the correlation
// uses explicit fmaf in the reference's row-major tap order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "lm_device.h"
#include "lm_introsort.h"

#include "lm_dev_common.h"

// ------------------------------------------------------------------ helpers

template <class FP>
DEV uint8_t ipad_pixel(FP __restrict__ F, const uint8_t* __restrict__ bkg,
                       const int32_t* __restrict__ cal, const uint8_t* lut, const LmConst& K, int R, int C) {
  // I_PAD(R, C): zero outside I_UNPAD (:684-689); inside, the corrected,
  // normalised, optionally flipped frame.
  const int r = R - K.pad_pre_rows;
  int c = C - K.pad_pre_cols;
  if (r < 0 || r >= K.n_rows || c < 0 || c >= K.n_cols) return 0;
  if (K.flip) c = K.n_cols - 1 - c;
  const int idx = cal[r * K.n_cols + c];
  const int f = F[idx], b = bkg[idx];
  return lut[f > b ? f - b : 0];
}

// --------------------------------------------------------------- k_minmax
// normalize(F, F, 0, 255, NORM_MINMAX, CV_8UC1) after subtract(F, BKG, F)
// (LocoMouse_class.cpp:1304-1310) needs min and max of sat(F - BKG) per frame.
// Each frame is split over LM_MM_SPLIT workgroups (16-byte loads of frame and
// background, wave and block reductions); each workgroup writes its partial
// min/max pair, and k_lut folds the LM_MM_SPLIT pairs of a slot into its LUT.
__global__ __launch_bounds__(LM_MM_THREADS) void k_minmax(const uint8_t* const* __restrict__ frame_ptr,
                                                          const uint8_t* __restrict__ bkg, int npix, int s0,
                                                          unsigned* __restrict__ mm) {
  const int slot = s0 + blockIdx.y;
  const lm_gu8* __restrict__ F = as_global(frame_ptr[slot]);
  const int nvec = npix >> 4;
  const int per = (nvec + LM_MM_SPLIT - 1) / LM_MM_SPLIT;
  const int v0 = blockIdx.x * per, v1 = min(nvec, v0 + per);
  const lm_gu4* F4 = reinterpret_cast<const lm_gu4*>(F);
  const uint4* B4 = reinterpret_cast<const uint4*>(bkg);
  unsigned mn = 255, mx = 0;
  auto fold = [&](unsigned fw, unsigned bw) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned fv = (fw >> (8 * k)) & 255u, bv = (bw >> (8 * k)) & 255u;
      const unsigned d = fv > bv ? fv - bv : 0u;
      mn = min(mn, d);
      mx = max(mx, d);
    }
  };
  int i = v0 + threadIdx.x;
  for (; i + 3 * LM_MM_THREADS < v1; i += 4 * LM_MM_THREADS) {  // four 16-byte loads in flight per lane
    lm_u32x4 f[4];
    uint4 b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      f[u] = F4[i + u * LM_MM_THREADS];
      b[u] = B4[i + u * LM_MM_THREADS];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      fold(f[u].x, b[u].x);
      fold(f[u].y, b[u].y);
      fold(f[u].z, b[u].z);
      fold(f[u].w, b[u].w);
    }
  }
  for (; i < v1; i += LM_MM_THREADS) {
    const lm_u32x4 f = F4[i];
    const uint4 b = B4[i];
    fold(f.x, b.x);
    fold(f.y, b.y);
    fold(f.z, b.z);
    fold(f.w, b.w);
  }
  if (blockIdx.x == LM_MM_SPLIT - 1)  // the bytes past the last 16-byte word
    for (int q = (nvec << 4) + threadIdx.x; q < npix; q += LM_MM_THREADS) {
      const unsigned fv = F[q], bv = bkg[q];
      const unsigned d = fv > bv ? fv - bv : 0u;
      mn = min(mn, d);
      mx = max(mx, d);
    }
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (unsigned)__shfl_xor((int)mn, o));
    mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
  }
  __shared__ unsigned smn[LM_MM_THREADS / 64], smx[LM_MM_THREADS / 64];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    smn[wid] = mn;
    smx[wid] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < LM_MM_THREADS / 64; ++w) {
      mn = min(mn, smn[w]);
      mx = max(mx, smx[w]);
    }
    mm[2 * (slot * LM_MM_SPLIT + blockIdx.x)] = mn;
    mm[2 * (slot * LM_MM_SPLIT + blockIdx.x) + 1] = mx;
  }
}

// Entry p of a frame's LUT from its min/max: normalize(NORM_MINMAX) ->
// convertTo(CV_8U, scale, shift) = sat_u8(cvRound((float)p*(float)scale +
// (float)shift)) (OpenCV 3.x, unfused), the noScale copy when scale == 1 and
// shift == 0, then the LocoMouse_TM imadjust LUT (methods 1/2, TM.cpp:247).
DEV int norm_lut_entry(unsigned mnv, unsigned mxv, int p, const uint8_t* adj, int use_adj) {
  const double smin = (double)mnv, smax = (double)mxv, dmin = 0.0, dmax = 255.0;
  const double scale = (dmax - dmin) * (smax - smin > 2.220446049250313e-16 ? 1. / (smax - smin) : 0.0);
  const double shift = dmin - smin * scale;
  int v;
  if (fabs(scale - 1.0) < 2.220446049250313e-16 && fabs(shift) < 2.220446049250313e-16) {
    v = p;  // convertTo noScale -> copy
  } else {
    const float sf = (float)scale, hf = (float)shift;
    float t = __fmul_rn((float)p, sf);
    t = __fadd_rn(t, hf);
    const int iv = (int)rintf(t);
    v = iv < 0 ? 0 : (iv > 255 ? 255 : iv);
  }
  return use_adj ? adj[v] : v;
}

// k_lut: the 256-entry LUT of every slot from k_minmax's partial min/max
// pairs.  4 slots per block.
__global__ __launch_bounds__(256) void k_lut(const unsigned* __restrict__ mm, int s0, int s_end,
                                             const uint8_t* __restrict__ adj, int use_adj, uint8_t* __restrict__ luts) {
  for (int s = s0 + blockIdx.x * 4; s < min(s_end, s0 + (int)blockIdx.x * 4 + 4); ++s) {
    unsigned mn = 255, mx = 0;
#pragma unroll
    for (int b = 0; b < LM_MM_SPLIT; ++b) {
      mn = min(mn, mm[2 * (s * LM_MM_SPLIT + b)]);
      mx = max(mx, mm[2 * (s * LM_MM_SPLIT + b) + 1]);
    }
    luts[s * 256 + threadIdx.x] = (uint8_t)norm_lut_entry(mn, mx, threadIdx.x, adj, use_adj);
  }
}

// I_PAD(R, C) of frame slot `sl` as the per-frame steps after
// cropBoundingBox see it: transform_gray_values with a CV_8U table rewrites
// the frame's bottom crop I_BOTTOM_MOUSE in place (LUT(I_BOTTOM_MOUSE, table,
// I_BOTTOM_MOUSE), LocoMouse_class.cpp:1445-1448), so that rectangle of I_PAD
// holds table[v] for the rest of the frame and in I_PREV_PAD for the next.
struct GrayRect {  // the LmConst fields in_gray_rect reads
  int32_t unpad_y[1], unpad_x[1], bb_bottom_h, bb_bottom_w;
};
template <class KT>
DEV bool in_gray_rect(const KT& K, const LmSlot& sl, int R, int C) {
  const int y = R - sl.crop_y[0] - K.unpad_y[0], x = C - sl.crop_x[0] - K.unpad_x[0];
  return (unsigned)y < (unsigned)K.bb_bottom_h && (unsigned)x < (unsigned)K.bb_bottom_w;
}

template <class FP>
DEV uint8_t ipad_pixel_t(FP __restrict__ F, const uint8_t* __restrict__ bkg, const int32_t* __restrict__ cal,
                         const uint8_t* lut, const LmConst& K, const LmSlot& sl, int R, int C) {
  const uint8_t v = ipad_pixel(F, bkg, cal, lut, K, R, C);
  return K.gray_lut_on && in_gray_rect(K, sl, R, C) ? K.gray_lut[v] : v;
}

// ---------------------------------------------------------------- k_ingest
// Builds the extended padded crops of both views for LM_INGEST_FB consecutive
// slots: every I_PAD pixel any detector tap reads (readFrame's correctImage +
// flip, :1316-1327 / :1337-1406; cropBoundingBox, :1408-1478).  One workgroup
// per (view, 8-row band of the view's ext crop, slot group): the bands are
// aligned with the dark-tile flag grid (band b holds the point detectors'
// output rows 8b .. 8b + 7), so the workgroup that writes a tile row's pixels
// also decides which of its LM_FW x LM_FH output tiles are bright (some I_*_MOUSE
// pixel > 25, LocoMouse_class.cpp:782, :817), writes their flag bytes and
// appends the bright ones to the view's tile list -- no second pass over the
// crops.  Each thread owns 16 consecutive crop bytes of the band (one 16-byte
// store per frame).  The calibration index and background byte of each are
// loaded once and reused for every slot whose crop sits at the same place
// (always, with a provided bounding box); per frame only the frame gather, the
// LUTs and the store remain.  Where the 16 source pixels are consecutive in
// the frame (a calibration map that is locally a translation, flipped or not)
// the gather is five aligned dword loads instead of sixteen byte loads.
#define LM_INGEST_VEC 16
static_assert(LM_FW >= LM_INGEST_VEC, "a 16-byte chunk spans at most two flag tiles");
#define LM_INGEST_MAXTX 128  // flag-grid columns a band's workgroup can hold (ow <= 128 LM_FW)

// Gather index of crop pixel I_PAD (R, C) (-1 outside I_UNPAD).
DEV int ingest_index(const LmConst& K, const int32_t* __restrict__ cal, int R, int C) {
  const int r = R - K.pad_pre_rows;
  int c = C - K.pad_pre_cols;
  if (r < 0 || r >= K.n_rows || c < 0 || c >= K.n_cols) return -1;
  if (K.flip) c = K.n_cols - 1 - c;
  return cal[r * K.n_cols + c];
}

// Gather indices and background bytes of the 16 crop pixels that start at
// I_PAD (R, C0) (0 background outside I_UNPAD).  inside: bit k set when
// pixel k lies inside I_UNPAD.  Returns 1 when the inside pixels are a run
// idx[k] = lo + k, -1 when idx[k] = lo + 15 - k (a flipped translation) --
// a chunk at the pad's edge is a run too, its outside bytes masked to 0
// after the LUT (I_PAD is zero outside I_UNPAD), and a chunk with no inside
// pixel is an empty run -- else 0 (a gather).  lo is the first source byte
// of the 20 the run's five dwords cover; a run whose dwords would leave the
// frame is a gather.  (k_ingest keeps only run, lo, inside and the
// background bytes: a gather re-reads the indices per frame, ingest_index,
// so no 16-register index array stays live.)
DEV int ingest_locate(const LmConst& K, const int32_t* __restrict__ cal, const uint8_t* __restrict__ bkg, int R, int C0,
                      uint32_t (&bw)[4], int& lo, unsigned& inside) {
  const int r = R - K.pad_pre_rows;
  inside = 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) bw[j] = 0u;
  // one pass, no index array: the first inside pixel fixes the candidate
  // runs' virtual idx[0] (up0 for a run, dn0 for a flipped one), the later
  // ones are tested against them
  int up0 = 0, dn0 = 0;
  bool any = false, up = true, down = true;
#pragma unroll
  for (int k = 0; k < LM_INGEST_VEC; ++k) {
    int c = C0 + k - K.pad_pre_cols;
    if (r >= 0 && r < K.n_rows && c >= 0 && c < K.n_cols) {
      if (K.flip) c = K.n_cols - 1 - c;
      const int ix = cal[r * K.n_cols + c];
      bw[k >> 2] |= (uint32_t)bkg[ix] << (8 * (k & 3));
      inside |= 1u << k;
      if (!any) {
        up0 = ix - k;
        dn0 = ix + k;
        any = true;
      } else {
        up = up && ix == up0 + k;
        down = down && ix == dn0 - k;
      }
    }
  }
  if (!any) {  // no pixel inside I_UNPAD: all zeros
    lo = 0;
    return 1;
  }
  int run = up ? 1 : (down ? -1 : 0);
  lo = up ? up0 : dn0 - (LM_INGEST_VEC - 1);
  if (run != 0 && (lo < 0 || (lo & ~3) + 20 > K.video_rows * K.video_cols)) run = 0;  // the dwords would leave the frame
  return run;
}

// 0xFF in byte j of the result for bit j of the 4-bit n (masking a word's
// outside bytes)
DEV uint32_t byte_keep4(uint32_t n) { return ((n * 0x00204081u) & 0x01010101u) * 0xFFu; }

// Source map of one view's crop at a fixed position (cx, cy): per 16-byte
// ext-crop chunk, {first source byte, run code | inside mask} and the 16
// background bytes, so
// k_ingest's batches with their crop there (always, with a provided bounding
// box) skip the calibration and background gathers (frame-invariant data,
// LocoMouse_class.cpp:1337-1406).  key[2 v], key[2 v + 1] = the position.
__global__ __launch_bounds__(256) void k_srcmap(const LmConst* __restrict__ Kp, const int32_t* __restrict__ cal,
                                                const uint8_t* __restrict__ bkg, int v, int cx, int cy,
                                                int2* __restrict__ smap, uint4* __restrict__ sbkg,
                                                int32_t* __restrict__ key) {
  const LmConst& K = *Kp;
  const int64_t e0 = (int64_t)K.ext_h[0] * K.ext_w[0];
  const int64_t nv = (int64_t)K.ext_h[v] * K.ext_w[v];
  const int64_t qq = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * LM_INGEST_VEC;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    key[2 * v] = cx;
    key[2 * v + 1] = cy;
  }
  if (qq >= nv) return;
  const int er = (int)(qq / K.ext_w[v]), ec = (int)(qq % K.ext_w[v]);
  uint32_t w[4];
  int lo;
  unsigned inside;
  const int run = ingest_locate(K, cal, bkg, cy + K.ext_oy[v] + er, cx + K.ext_ox[v] + ec, w, lo, inside);
  const int64_t ci = ((v ? e0 : 0) + qq) / LM_INGEST_VEC;
  // y: run code (1 up, 2 down, 0 a gather) | inside mask << 16
  smap[ci] = make_int2(lo, (run > 0 ? 1 : run < 0 ? 2 : 0) | (int)(inside << 16));
  sbkg[ci] = make_uint4(w[0], w[1], w[2], w[3]);
}

// Bright bytes (> 25: threshold(25.5, BINARY_INV) leaves them unmasked) of a
// packed word, as 0x80 in each such byte.
DEV uint32_t bright_bytes(uint32_t w) {
  return (((w & 0x7F7F7F7Fu) + 0x66666666u) | w) & 0x80808080u;
}
// 0x80 in byte i of the result for bit i of the 4-bit n
DEV uint32_t byte_mask4(uint32_t n) { return ((n * 0x00204081u) & 0x01010101u) << 7; }

// The five aligned dwords that cover the 16 source bytes [lo, lo + 16) of a
// run: one dwordx4 (gfx950 global loads need only dword alignment) plus one
// dword -- two vector-memory instructions instead of five.
#ifndef LM_INGEST_X4
#define LM_INGEST_X4 1
#endif
typedef uint32_t lm_u4a4 __attribute__((ext_vector_type(4), aligned(4)));
DEV void ingest_run_load(const lm_gu8* F, int lo, uint32_t (&d)[5]) {
  const lm_gu32* w = reinterpret_cast<const lm_gu32*>(F + (lo & ~3));
#if LM_INGEST_X4
  const lm_u4a4 a = *reinterpret_cast<const __attribute__((address_space(1))) lm_u4a4*>(w);
  d[0] = a.x;
  d[1] = a.y;
  d[2] = a.z;
  d[3] = a.w;
  d[4] = w[4];
#else
#pragma unroll
  for (int u = 0; u < 5; ++u) d[u] = w[u];
#endif
}

#ifndef LM_INGEST_PIPE
#define LM_INGEST_PIPE 3  // frames whose run loads are in flight at once
#endif
#ifndef LM_INGEST_WPE
#define LM_INGEST_WPE 5  // amdgpu_waves_per_eu minimum: <= 96 VGPRs, so 5 four-wave groups per CU (one round at C3)
#endif
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(LM_INGEST_WPE, 8))) void k_ingest(const LmConst* __restrict__ Kp, const uint8_t* const* __restrict__ frame_ptr,
                                                 const uint8_t* __restrict__ bkg, const int32_t* __restrict__ cal,
                                                 const uint8_t* __restrict__ luts, const LmSlot* __restrict__ slots,
                                                 int s0, int s_end, uint8_t* __restrict__ ext, int64_t ext_slot_bytes,
                                                 unsigned* __restrict__ tailbm, const int2* __restrict__ smap,
                                                 const uint4* __restrict__ sbkg, const int32_t* __restrict__ skey,
                                                 uint8_t* __restrict__ flags, int32_t* __restrict__ tl_cnt,
                                                 uint32_t* __restrict__ tl_list, long long* __restrict__ prof) {
  const LmConst& K = *Kp;
  // LM_KPROF=1: clock64() of thread 0 at the phase ends, wall clock at start / end
  long long* pb = prof ? prof + (int64_t)(blockIdx.y * gridDim.x + blockIdx.x) * 16 : nullptr;
#define ING_PROF(k) \
  if (pb && threadIdx.x == 0) pb[k] = clock64();
  ING_PROF(0)
  if (pb && threadIdx.x == 0) pb[14] = wall_clock64();
  const int sb = s0 + blockIdx.y * LM_INGEST_FB;
  const int nf = min(LM_INGEST_FB, s_end - sb);
  const int T = (int)blockDim.x, tid = (int)threadIdx.x;
  {  // this block's share of the group's tail bitmaps is zeroed (k_corr ORs the tail detectors' bits in)
    const int per = (K.tail_bm_words + (int)gridDim.x - 1) / (int)gridDim.x;
    const int w0 = (int)blockIdx.x * per, w1 = min(K.tail_bm_words, w0 + per);
    for (int f = 0; f < nf; ++f) {
      unsigned* __restrict__ t = tailbm + (int64_t)(sb + f) * K.tail_bm_words;
      for (int w = w0 + tid; w < w1; w += T) t[w] = 0u;
    }
  }
  // this block's view and band
  const int v = (int)blockIdx.x < K.ing_nb[0] ? 0 : 1;
  const int band = K.ing_b0[v] + (int)blockIdx.x - (v ? K.ing_nb[0] : 0);
  const int ew = K.ext_w[v], cw = ew / LM_INGEST_VEC, nch = 8 * cw;
  const int64_t e0 = (int64_t)K.ext_h[0] * K.ext_w[0];
  constexpr int FPB = 8 / LM_FH;  // flag rows per band
  const bool fl_band = flags != nullptr && band >= 0 && band * FPB < K.fl_ty[v];
  const int ftx = K.fl_tx[v];
  // One round of independent loads (the group's LUTs into registers, the
  // slots, the first chunk's source map entry), then the frame loads the map
  // points at, and only then the LUTs into LDS and the barrier: the group
  // costs two load latencies, not four (LUT copy, slots, map, frames one
  // after another).
  __shared__ __attribute__((aligned(16))) uint8_t lut[LM_INGEST_FB][256];
  __shared__ uint8_t glut[256];
  __shared__ uint8_t s_fl[LM_INGEST_FB][8 / LM_FH][LM_INGEST_MAXTX];  // bright output tiles of the band, per slot
  __shared__ uint32_t s_ent[LM_INGEST_FB * (8 / LM_FH) * LM_INGEST_MAXTX];
  __shared__ int s_n, s_outs, s_base;
  for (int i = tid; i < LM_INGEST_FB * 256 / 8; i += T) {
    const int li = i * 8;
    if (li < nf * 256) *reinterpret_cast<uint2*>(&lut[0][0] + li) = *reinterpret_cast<const uint2*>(luts + (int64_t)sb * 256 + li);
  }
  for (int i = tid; i < 256; i += T) glut[i] = K.gray_lut[i];
  for (int i = tid; i < LM_INGEST_FB * FPB * LM_INGEST_MAXTX; i += T) (&s_fl[0][0][0])[i] = 0;
  if (tid == 0) {
    s_n = 0;
    s_outs = 0;
  }
  // the grey LUT's switch and rectangle, read once (in_gray_rect takes them from gk)
  const bool gray_on = K.gray_lut_on != 0;
  GrayRect gk;
  gk.unpad_y[0] = K.unpad_y[0];
  gk.unpad_x[0] = K.unpad_x[0];
  gk.bb_bottom_h = K.bb_bottom_h;
  gk.bb_bottom_w = K.bb_bottom_w;
  const LmSlot sl0 = slots[sb];
  bool same = true;
  for (int f = 1; f < nf; ++f)
    same = same && slots[sb + f].crop_x[v] == sl0.crop_x[v] && slots[sb + f].crop_y[v] == sl0.crop_y[v];
  const bool mapped = same && smap && skey[2 * v] == sl0.crop_x[v] && skey[2 * v + 1] == sl0.crop_y[v];
  // chunk i of the band: ext row er, byte column ec (a multiple of 16)
  auto chunk_pos = [&](int i, int& er, int& ec) {
    const int rr = i / cw;
    er = K.fl_my[v] + 8 * band + rr;
    ec = (i - rr * cw) * LM_INGEST_VEC;
    return i < nch && er >= 0 && er < K.ext_h[v];
  };
  // the run loads of frames f .. f + LM_INGEST_PIPE - 1 in flight at once:
  // frame f's registers take frame f + LM_INGEST_PIPE's loads as soon as they
  // are consumed, so the group needs LM_INGEST_PIPE x 5 registers for them,
  // not LM_INGEST_FB x 5 (five waves per SIMD: the grid is one round)
  constexpr int PIPE = LM_INGEST_PIPE;
  uint32_t d[PIPE][5];
  int2 m = make_int2(0, 0);
  uint4 b4 = make_uint4(0u, 0u, 0u, 0u);
  auto frame_load = [&](int f, int lo_, uint32_t (&dd)[5]) {
    ingest_run_load(as_global(frame_ptr[sb + f]), lo_, dd);
  };
  // the fast path's loads of chunk i (source map entry, then the first frames' run dwords)
  auto fast_loads = [&](int i) {
    int er, ec;
    const bool act = chunk_pos(i, er, ec);
    m = make_int2(0, 0);
    if (act && mapped) {
      const int64_t ci = ((v ? e0 : 0) + (int64_t)er * ew + ec) / LM_INGEST_VEC;
      m = smap[ci];
      b4 = sbkg[ci];
      if ((m.y & 3) != 0) {
#pragma unroll
        for (int f = 0; f < PIPE; ++f)
          if (f < nf) frame_load(f, m.x, d[f]);
      }
    }
  };
  ING_PROF(1)
  fast_loads(tid);
  __syncthreads();
  ING_PROF(2)

  for (int i = tid; i < nch; i += T) {
    if (i != tid) fast_loads(i);
    int er, ec;
    if (!chunk_pos(i, er, ec)) continue;
    const int64_t q = (v ? e0 : 0) + (int64_t)er * ew + ec;  // byte offset in the slot's ext crops
    // dark-tile flags: the bytes of this chunk that are point-detector
    // outputs' I_*_MOUSE pixels (output (y, x) = ext (fl_my + y, fl_mx + x)),
    // split at the LM_FW-column tile boundary: tile ta and ta + 1
    uint32_t ma[4] = {0u, 0u, 0u, 0u}, mb[4] = {0u, 0u, 0u, 0u};
    int ta = 0;
    const int y = er - K.fl_my[v];
    const int fr = (y - 8 * band) / LM_FH;  // the chunk's flag row in the band (when fl_band)
    if (fl_band && y < K.fl_oh[v]) {
      const int x0 = ec - K.fl_mx[v];
      ta = x0 >= 0 ? x0 / LM_FW : -((LM_FW - 1 - x0) / LM_FW);
      const int lo = max(0, -x0), hi = min(LM_INGEST_VEC, K.fl_ow[v] - x0), ks = (ta + 1) * LM_FW - x0;
      auto range = [](int a, int b) -> uint32_t {  // bits [a, b) of 16
        return a < b ? ((b >= 32 ? 0xFFFFFFFFu : (1u << b) - 1u) & ~((1u << a) - 1u)) & 0xFFFFu : 0u;
      };
      const uint32_t bits_a = range(lo, min(hi, ks)), bits_b = range(max(lo, ks), hi);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ma[j] = byte_mask4((bits_a >> (4 * j)) & 0xFu);
        mb[j] = byte_mask4((bits_b >> (4 * j)) & 0xFu);
      }
    }
    const bool flag_chunk = (ma[0] | ma[1] | ma[2] | ma[3] | mb[0] | mb[1] | mb[2] | mb[3]) != 0u;
    uint32_t bw[4];  // background bytes, packed
    int run = 0;  // 1: idx[k] = idx[0] + k, -1: idx[k] = idx[0] - k, 0: gather
    int lo = 0;   // a run's first source byte
    unsigned inside = 0xFFFFu;  // bit k: pixel k inside I_UNPAD (the others are masked to 0 after the LUT)
    // the 16 source bytes of a run span [lo, lo + 16): five aligned dwords cover them
    // (funnel shifts by the byte offset, then a byte reversal for a flipped run:
    // no register array is indexed with a run-time value, so nothing spills)
    auto run_bytes = [&](const uint32_t (&dd)[5], uint32_t (&w)[4]) {
      const unsigned sh = (unsigned)(lo & 3);
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = __builtin_amdgcn_alignbyte(dd[j + 1], dd[j], sh);
      if (run < 0) {
        const uint32_t r0 = __builtin_bswap32(w[3]), r1 = __builtin_bswap32(w[2]), r2 = __builtin_bswap32(w[1]),
                       r3 = __builtin_bswap32(w[0]);
        w[0] = r0;
        w[1] = r1;
        w[2] = r2;
        w[3] = r3;
      }
    };
    // background subtraction, the slot's LUT, the grey LUT, the 16-byte store
    // and the chunk's bright-tile bits (pixels and background bytes stay
    // packed four to a register)
    // Pixels outside I_UNPAD (inside bit clear: the pad, or the background-
    // and-LUT of a don't-care byte) are zeroed after the LUT, once per word.
    // The grey LUT is a separate instantiation (GRAY, chosen once per
    // kernel): a K field tested per byte made the compiler re-load it per
    // byte and wait for it -- with the LUT read just issued, whose wait
    // counter the scalar load shares -- so every byte's LDS read was waited
    // for on its own.
    auto emit = [&](int f, const uint32_t (&pw)[4], const LmSlot& sl, int R, int C0, unsigned in_mask, auto gray_c) {
      constexpr bool GRAY = decltype(gray_c)::value;
      uint32_t word[4] = {0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < LM_INGEST_VEC; ++k) {
        const uint32_t pk = (pw[k >> 2] >> (8 * (k & 3))) & 0xFFu, bk = (bw[k >> 2] >> (8 * (k & 3))) & 0xFFu;
        uint32_t o = lut[f][pk > bk ? pk - bk : 0];
        // (the grey LUT's rectangle never reaches the pad: the host rejects that)
        if (GRAY && in_gray_rect(gk, sl, R, C0 + k)) o = glut[o];
        word[k >> 2] |= o << (8 * (k & 3));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) word[j] &= byte_keep4((in_mask >> (4 * j)) & 0xFu);
      *reinterpret_cast<uint4*>(ext + (int64_t)(sb + f) * ext_slot_bytes + q) = make_uint4(word[0], word[1], word[2], word[3]);
      if (flag_chunk) {
        uint32_t ha = 0u, hb = 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t br = bright_bytes(word[j]);
          ha |= br & ma[j];
          hb |= br & mb[j];
        }
        if (ha) s_fl[f][fr][ta] = 1;
        if (hb) s_fl[f][fr][ta + 1] = 1;
      }
    };

    const int R = sl0.crop_y[v] + K.ext_oy[v] + er, C0 = sl0.crop_x[v] + K.ext_ox[v] + ec;
    if (mapped && (m.y & 3) != 0) {  // the source map holds this crop position: no calibration / background gathers
      run = (m.y & 3) == 1 ? 1 : -1;
      lo = m.x;
      inside = (unsigned)m.y >> 16;
      bw[0] = b4.x;
      bw[1] = b4.y;
      bw[2] = b4.z;
      bw[3] = b4.w;
#pragma unroll
      for (int f = 0; f < LM_INGEST_FB; ++f)
        if (f < nf) {
          uint32_t pw[4];
          run_bytes(d[f % PIPE], pw);
          if (f + PIPE < nf) frame_load(f + PIPE, lo, d[f % PIPE]);
          if (gray_on) emit(f, pw, slots[sb + f], R, C0, inside, std::true_type{});
          else emit(f, pw, sl0, R, C0, inside, std::false_type{});
        }
      continue;
    }
    run = ingest_locate(K, cal, bkg, R, C0, bw, lo, inside);
    if (same && run != 0) {
      // Every slot of the group has its crop at the same place and the pixels
      // are a run, but the source map does not hold it: the group's frame
      // loads are issued PIPE ahead of their use.
#pragma unroll
      for (int f = 0; f < PIPE; ++f)
        if (f < nf) frame_load(f, lo, d[f]);
#pragma unroll
      for (int f = 0; f < LM_INGEST_FB; ++f)
        if (f < nf) {
          uint32_t pw[4];
          run_bytes(d[f % PIPE], pw);
          if (f + PIPE < nf) frame_load(f + PIPE, lo, d[f % PIPE]);
          if (gray_on) emit(f, pw, slots[sb + f], R, C0, inside, std::true_type{});
          else emit(f, pw, sl0, R, C0, inside, std::false_type{});
        }
      continue;
    }
    // General case: frame by frame, the indices recomputed whenever the crop moves.
    int px = sl0.crop_x[v], py = sl0.crop_y[v];
    for (int f = 0; f < nf; ++f) {
      const int slot = sb + f;
      const LmSlot sl = slots[slot];
      const int Rf = sl.crop_y[v] + K.ext_oy[v] + er;
      const int Cf = sl.crop_x[v] + K.ext_ox[v] + ec;
      if (sl.crop_x[v] != px || sl.crop_y[v] != py) {  // crop moved: recompute the gather indices
        px = sl.crop_x[v];
        py = sl.crop_y[v];
        run = ingest_locate(K, cal, bkg, Rf, Cf, bw, lo, inside);
      }
      const lm_gu8* __restrict__ F = as_global(frame_ptr[slot]);
      uint32_t pw[4] = {0, 0, 0, 0};
      if (run != 0) {
        uint32_t d1[5];
        ingest_run_load(F, lo, d1);
        run_bytes(d1, pw);
      } else {
#pragma unroll
        for (int k = 0; k < LM_INGEST_VEC; ++k)
          if ((inside >> k) & 1u) pw[k >> 2] |= (uint32_t)F[ingest_index(K, cal, Rf, Cf + k)] << (8 * (k & 3));
      }
      if (gray_on) emit(f, pw, sl, Rf, Cf, inside, std::true_type{});
      else emit(f, pw, sl, Rf, Cf, inside, std::false_type{});
    }
  }
  ING_PROF(3)
  if (!fl_band || !tl_list) {
    if (pb && threadIdx.x == 0) {
      pb[4] = clock64();
      pb[15] = wall_clock64();
    }
  }
  if (!fl_band) return;
  // the band's flag bytes (each written by this block only: no zeroing pass)
  // and its bright tiles appended to the view's list (any order: the
  // correlation's waves take them LM_RW_NQ at a time, and the keys they
  // produce are sorted by k_nms)
  __syncthreads();
  for (int i = tid; i < nf * FPB * ftx; i += T) {
    const int f = i / (FPB * ftx), r = (i / ftx) % FPB, tx = i % ftx;
    const int ty = band * FPB + r;
    if (ty >= K.fl_ty[v]) continue;
    const int oh_t = min(LM_FH, K.fl_oh[v] - LM_FH * ty);
    const uint8_t b = s_fl[f][r][tx];
    flags[(int64_t)(sb + f) * K.fl_slot + K.fl_off[v] + ty * ftx + tx] = b;
    if (b && tl_list) {
      s_ent[atomicAdd(&s_n, 1)] = ((uint32_t)(sb + f) << 16) | (uint32_t)(ty * ftx + tx);
      atomicAdd(&s_outs, oh_t * min(LM_FW, K.fl_ow[v] - tx * LM_FW));
    }
  }
  if (!tl_list) return;
  __syncthreads();
  // this workgroup's list segment and its counter (tl_cnt: bright tiles of
  // view v at v LM_TL_NC + c, their outputs at (2 + v) LM_TL_NC + c)
  const int G = (int)gridDim.y, c = (int)blockIdx.y * LM_TL_NC / G;
  if (tid == 0) {
    s_base = s_n ? atomicAdd(&tl_cnt[v * LM_TL_NC + c], s_n) : 0;
    if (s_outs) atomicAdd(&tl_cnt[(2 + v) * LM_TL_NC + c], s_outs);
  }
  __syncthreads();
  uint32_t* __restrict__ out = tl_list + (int64_t)v * K.tl_stride +
                               (int64_t)lm_tl_y0(c, G) * LM_INGEST_FB * K.fl_tx[v] * K.fl_ty[v] + s_base;
  for (int p = tid; p < s_n; p += T) out[p] = s_ent[p];
  if (pb && threadIdx.x == 0) {
    pb[4] = clock64();
    pb[15] = wall_clock64();
  }
#undef ING_PROF
}

#include "lm_corr.h"  // the correlation kernels are their own translation unit (lm_corr.hip)

#include "lm_cc.h"

// ------------------------------------------------------------------ k_tail
// keys of positive scores: (~float_bits(score) << 32) | row-major output index
DEV float key_score(unsigned long long k) { return __uint_as_float(~(unsigned)(k >> 32)); }
DEV unsigned key_lo(unsigned long long k) { return (unsigned)(k & 0xFFFFFFFFu); }
// detectTail (:2541-2555) -> detectLineCandidates (:2558-2742), one
// workgroup per frame:
//   bottom: largest component of (tail_b > 0) (selectLargestRegion :2604,
//     lm_cc.h) -> TAIL_MASK (:2611, a bitmap here: 64 columns per word),
//     colmax = reduce(MAX) over rows (:2615), first / last occupied columns
//     (:2642-2670), tail_width = last - first (:2677), 15 segments, the first
//     tail_width % 15 one column wider (:2678-2685), per segment the binary
//     moments m00, m10, m01 (:2702-2725) -> track x, y;
//   side: largest component of (tail_s > 0) & repeat(colmax) (:2623-2626),
//     then at every track x > 0 the moments of that one column (:2728-2737)
//     -> track z.
// cv::moments(binary) walks 32x32 tiles in raster order, accumulates integer
// tile sums (count, sum of x and of y inside the tile), scales them by 1/255
// and adds x0*m00 / y0*m00 of the tile origin; the sums are built here from
// the component's runs (arithmetic series per run and tile) and turned into
// doubles in that same tile order, so the tracks are bit-identical.
// No size limit: run tables beyond the LDS capacity go to global scratch.
#ifndef LM_TAIL_THREADS
#define LM_TAIL_THREADS 256
#endif
#define LM_TAIL_SEGS 15

struct TailLayout {  // byte offsets into k_tail's dynamic LDS
  int rowoff, colc, colm, mask, bm, par, area, key, rs, re, mb, ms, bytes;
};
__host__ __device__ inline TailLayout tail_layout(int TW, int HB, int HS, int cap, int ntc) {
  const int Hm = HB > HS ? HB : HS, nb64 = (TW + 63) / 64;
  const int ntrb = (HB + 31) / 32, ntrs = (HS + 31) / 32;
  TailLayout L;
  int o = 0;
  L.rowoff = o;
  o += 4 * (Hm + 1);
  L.colc = o;
  o += 4 * (TW + 2);
  o = (o + 15) & ~15;
  L.colm = o;
  o += 8 * nb64;
  L.mask = o;
  o += 8 * HB * nb64;
  L.bm = o;
  L.par = o;
  L.area = o + 4 * cap;
  L.key = o + 8 * cap;
  const int bmb = 8 * Hm * (nb64 + 1), ufb = 12 * cap;
  o += bmb > ufb ? bmb : ufb;
  L.rs = o;
  o += 2 * cap;
  L.re = o;
  o += 2 * cap;
  o = (o + 15) & ~15;
  L.mb = o;
  o += 4 * LM_TAIL_SEGS * ntrb * ntc * 3;
  L.ms = o;
  o += 4 * LM_TAIL_SEGS * ntrs * 2;
  L.bytes = o;
  return L;
}

// Segment of column offset rx in [0, tail_width) and its start (:2678-2685).
DEV void tail_segment(int rx, int rem, int reg, int* seg, int* sx) {
  if (rx < rem * (reg + 1)) {
    *seg = rx / (reg + 1);
    *sx = *seg * (reg + 1);
  } else {
    *seg = rem + (rx - rem * (reg + 1)) / reg;
    *sx = rem * (reg + 1) + (*seg - rem) * reg;
  }
}

// Bottom pass 1 over the chosen component's runs: TAIL_MASK bits, the column
// counts (difference array) and the first / last occupied columns.
template <bool G, class IX>
DEV void tail_bottom_runs(const CCRuns<IX> S, int R, const int* rowoff, int H, unsigned broot, int nb64,
                          unsigned long long* mask, int* colc, int* s_first, int* s_last) {
  for (int i = threadIdx.x; i < R; i += blockDim.x) {
    if (rld<G>(&S.par[i]) != broot) continue;
    const int y = cc_row_of(rowoff, H, i);
    const int x0 = (int)rld<G>(&S.rs[i]), x1 = (int)rld<G>(&S.re[i]);
    for (int k = x0 >> 6; k <= (x1 >> 6); ++k) {
      const int a = max(x0, 64 * k) - 64 * k, b = min(x1, 64 * k + 63) - 64 * k;
      const unsigned long long bits = (b == 63 ? ~0ull : ((1ull << (b + 1)) - 1)) & ~((1ull << a) - 1);
      atomicOr(&mask[(int64_t)y * nb64 + k], bits);
    }
    atomicAdd(&colc[x0], 1);
    atomicSub(&colc[x1 + 1], 1);
    atomicMin(s_first, x0);
    atomicMax(s_last, x1);
  }
}

// Bottom pass 2: integer tile sums of every segment's moments from the runs
// inside [first, first + tail_width).
template <bool G, class IX>
DEV void tail_bottom_moments(const CCRuns<IX> S, int R, const int* rowoff, int H, unsigned broot, int first, int tw,
                             int rem, int reg, unsigned* mb, int ntrb, int ntc) {
  for (int i = threadIdx.x; i < R; i += blockDim.x) {
    if (rld<G>(&S.par[i]) != broot) continue;
    const int y = cc_row_of(rowoff, H, i);
    const int a = max((int)rld<G>(&S.rs[i]), first) - first, b = min((int)rld<G>(&S.re[i]), first + tw - 1) - first;
    int rx = a;
    while (rx <= b) {
      int seg, sx;
      tail_segment(rx, rem, reg, &seg, &sx);
      const int wseg = seg < rem ? reg + 1 : reg;
      const int end = min(b, sx + wseg - 1);  // this segment's part of the run
      for (int l0 = rx - sx; l0 <= end - sx;) {  // 32-column tiles inside the segment
        const int tx = l0 >> 5, l1 = min(end - sx, 32 * tx + 31);
        const unsigned cnt = (unsigned)(l1 - l0 + 1);
        const unsigned sumx = (unsigned)((l0 + l1 - 64 * tx) * (int)cnt / 2);  // sum of (l - 32 tx), l in [l0, l1]
        unsigned* t = mb + ((seg * ntrb + (y >> 5)) * ntc + tx) * 3;
        atomicAdd(&t[0], cnt);
        atomicAdd(&t[1], sumx);
        atomicAdd(&t[2], (unsigned)(y & 31) * cnt);
        l0 = l1 + 1;
      }
      rx = end + 1;
    }
  }
}

// Side: every track column x > 0 the chosen component covers in a row adds
// that row to the column's tile sums.
template <bool G, class IX>
DEV void tail_side_moments(const CCRuns<IX> S, int R, const int* rowoff, int H, unsigned broot, const int* s_tx,
                           unsigned* ms, int ntrs) {
  for (int i = threadIdx.x; i < R; i += blockDim.x) {
    if (rld<G>(&S.par[i]) != broot) continue;
    const int y = cc_row_of(rowoff, H, i);
    const int x0 = (int)rld<G>(&S.rs[i]), x1 = (int)rld<G>(&S.re[i]);
    for (int k = 0; k < LM_TAIL_SEGS; ++k)
      if (s_tx[k] > 0 && s_tx[k] >= x0 && s_tx[k] <= x1) {
        atomicAdd(&ms[(k * ntrs + (y >> 5)) * 2], 1u);
        atomicAdd(&ms[(k * ntrs + (y >> 5)) * 2 + 1], (unsigned)(y & 31));
      }
  }
}

// BIG: tail boxes whose bitmaps and tables do not fit the CU's LDS (the
// reference has no size limit, LocoMouse_class.cpp:2604-2626): the same code
// on a per-slot global workspace (`ws`, tail_layout(..., cap 0) bytes per
// slot), every run table in global scratch.
template <bool BIG>
__global__ __launch_bounds__(LM_TAIL_THREADS) void k_tail(const LmConst* __restrict__ Kp, int s0,
                                                          const uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes,
                                                          unsigned long long* __restrict__ tailmask,
                                                          unsigned* __restrict__ scratch, LmSlotOut* __restrict__ hdr,
                                                          long long* __restrict__ prof, uint8_t* __restrict__ ws,
                                                          int64_t ws_slot, const unsigned long long* __restrict__ keys,
                                                          const int32_t* __restrict__ n_pos) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smt_lds[];
#define TAIL_PROF(k) \
  if (prof && threadIdx.x == 0) prof[blockIdx.x * 16 + (k)] = clock64();
  TAIL_PROF(0)
  if (prof && threadIdx.x == 0) prof[blockIdx.x * 16 + 14] = wall_clock64();
  const LmConst& K = *Kp;
  const int slot = s0 + blockIdx.x;
  uint8_t* smt = BIG ? ws + (int64_t)slot * ws_slot : smt_lds;
  const int TW = K.tail_w, HB = K.tail_hb, HS = K.tail_hs, nb64 = (TW + 63) / 64;
  const int cap = BIG ? 0 : K.tail_cap, ntc = K.tail_ntc, ntrb = (HB + 31) / 32, ntrs = (HS + 31) / 32;
  const TailLayout L = tail_layout(TW, HB, HS, cap, ntc);
  int* rowoff = reinterpret_cast<int*>(smt + L.rowoff);
  int* colc = reinterpret_cast<int*>(smt + L.colc);
  unsigned long long* colm = reinterpret_cast<unsigned long long*>(smt + L.colm);
  unsigned long long* mask = reinterpret_cast<unsigned long long*>(smt + L.mask);
  unsigned long long* bm = reinterpret_cast<unsigned long long*>(smt + L.bm);
  unsigned* mb = reinterpret_cast<unsigned*>(smt + L.mb);
  unsigned* ms = reinterpret_cast<unsigned*>(smt + L.ms);
  const CCRuns<uint16_t> SL{reinterpret_cast<uint16_t*>(smt + L.rs), reinterpret_cast<uint16_t*>(smt + L.re),
                            reinterpret_cast<unsigned*>(smt + L.par), reinterpret_cast<unsigned*>(smt + L.area),
                            reinterpret_cast<unsigned*>(smt + L.key)};
  const int64_t capg = (int64_t)max(HB, HS) * ((TW + 1) / 2);  // at most ceil(TW/2) runs per row
  unsigned* gb = scratch + (int64_t)slot * 5 * capg;
  const CCRuns<unsigned> SG{gb, gb + capg, gb + 2 * capg, gb + 3 * capg, gb + 4 * capg};
  __shared__ unsigned long long s_red[LM_TAIL_THREADS / 64];
  __shared__ unsigned s_best;
  __shared__ int s_total, s_first, s_last;
  __shared__ int s_tx[LM_TAIL_SEGS];
  const int tid = threadIdx.x, nt = blockDim.x;
  const bool c8 = K.connectivity == 8;
  const bool lds_ok = TW <= 65535;
  const unsigned long long* __restrict__ binb =
      reinterpret_cast<const unsigned long long*>(tailbin + (int64_t)slot * tailbin_slot_bytes);
  const unsigned long long* __restrict__ bins = binb + (int64_t)HB * nb64;

  for (int i = tid; i < TW + 2; i += nt) colc[i] = 0;
  for (int i = tid; i < HB * nb64; i += nt) mask[i] = 0;
  for (int i = tid; i < LM_TAIL_SEGS * ntrb * ntc * 3; i += nt) mb[i] = 0;
  for (int i = tid; i < LM_TAIL_SEGS * ntrs * 2; i += nt) ms[i] = 0;
  if (tid == 0) {
    s_first = 0x7FFFFFFF;
    s_last = -1;
  }

  // ---- bottom: largest component, TAIL_MASK, column mask, segment moments
  cc_bitmap_bits(binb, HB, nb64, nullptr, bm, rowoff);
  TAIL_PROF(1)
  cc_wave0_scan(rowoff, HB, &s_total);
  int R = s_total;
  TAIL_PROF(2)
  const bool gb_b = !(lds_ok && R <= cap);
  if (!gb_b) cc_label<false>(SL, bm, nb64, TW, HB, R, rowoff, c8, s_red, &s_best);
  else cc_label<true>(SG, bm, nb64, TW, HB, R, rowoff, c8, s_red, &s_best);
  const unsigned best_b = s_best;
  TAIL_PROF(3)
  const bool have = best_b != 0xFFFFFFFFu;
  if (have) {
    if (!gb_b) tail_bottom_runs<false>(SL, R, rowoff, HB, best_b, nb64, mask, colc, &s_first, &s_last);
    else tail_bottom_runs<true>(SG, R, rowoff, HB, best_b, nb64, mask, colc, &s_first, &s_last);
  }
  __syncthreads();
  const int first = s_first, last = s_last;
  const int tail_width = have ? last - first : 0;  // :2677 (no +1)
  const int rem = tail_width % LM_TAIL_SEGS, reg = (tail_width - rem) / LM_TAIL_SEGS;
  if (have) {
    if (!gb_b) tail_bottom_moments<false>(SL, R, rowoff, HB, best_b, first, tail_width, rem, reg, mb, ntrb, ntc);
    else tail_bottom_moments<true>(SG, R, rowoff, HB, best_b, first, tail_width, rem, reg, mb, ntrb, ntc);
  }
  // column counts -> colmax bitmap (reduce(MAX, dim 0), :2615)
  if (tid < 64) {
    const int lane = tid;
    int carry = 0;
    for (int k = 0; k < nb64; ++k) {
      const int x = 64 * k + lane;
      int inc = x < TW ? colc[x] : 0;
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
      }
      const unsigned long long b = __ballot(x < TW && carry + inc > 0);
      if (lane == 0) colm[k] = b;
      carry += __shfl(inc, 63);
    }
  }
  __syncthreads();
  TAIL_PROF(4)
  unsigned long long* __restrict__ tm = tailmask + (int64_t)slot * HB * nb64;
  for (int i = tid; i < HB * nb64; i += nt) tm[i] = mask[i];
  // detectSideCandidates runs only when the bottom list of the feature is
  // non-empty after the TAIL_MASK filter (:820-833).  Decided here, from the
  // keys before k_nms stages any candidate over them: in k_nms the bottom
  // block of a (slot, feature) overwrites its own keys while the side block
  // would be reading them.
  for (int feat = 0; feat < LM_NFEAT; ++feat) {
    const LmDet& D = K.det[feat == 0 ? DET_PAW_B : DET_SNOUT_B];
    const unsigned long long* __restrict__ src = keys + (int64_t)slot * K.keys_per_slot + K.list_off[feat];
    const int n = n_pos[slot * LM_NLIST + feat];
    int keep = 0;
    for (int k = tid; k < n && !keep; k += nt) {
      const unsigned idx = key_lo(src[k]);
      const int y = idx / D.ow, x = idx - y * D.ow;
      keep = !(x < TW && y < HB && ((mask[y * nb64 + (x >> 6)] >> (x & 63)) & 1));
    }
    keep = __syncthreads_or(keep);
    if (tid == 0) hdr[slot].bottom_kept[feat] = keep != 0;
  }

  // ---- side: (tail_s > 0) & repeat(colmax) -> largest component
  cc_bitmap_bits(bins, HS, nb64, colm, bm, rowoff);
  TAIL_PROF(5)
  cc_wave0_scan(rowoff, HS, &s_total);
  R = s_total;
  const bool gb_s = !(lds_ok && R <= cap);
  if (!gb_s) cc_label<false>(SL, bm, nb64, TW, HS, R, rowoff, c8, s_red, &s_best);
  else cc_label<true>(SG, bm, nb64, TW, HS, R, rowoff, c8, s_red, &s_best);
  const unsigned best_s = s_best;
  TAIL_PROF(6)

  // track x, y per segment (moments of the bottom component, :2702-2725)
  if (tid < LM_TAIL_SEGS) {
    const int i = tid;
    int tx_ = -1, ty_ = -1;
    if (have) {
      const int sx = first + (i < rem ? i * (reg + 1) : rem * (reg + 1) + (i - rem) * reg);
      const int wseg = i < rem ? reg + 1 : reg;
      double m00 = 0, m10 = 0, m01 = 0;
      const double s = 1. / 255;
      const int nc = (wseg + 31) >> 5;
      for (int ty = 0; ty < ntrb; ++ty)
        for (int tx = 0; tx < nc; ++tx) {
          const unsigned* t = mb + ((i * ntrb + ty) * ntc + tx) * 3;
          const double mom0 = (double)(255u * t[0]) * s;
          const double mom1 = (double)(255u * t[1]) * s;
          const double mom2 = (double)(255u * t[2]) * s;
          const double xm = (double)(tx * 32) * mom0, ym = (double)(ty * 32) * mom0;
          m00 += mom0;
          m10 += mom1 + xm;
          m01 += mom2 + ym;
        }
      if (m00 > 0) {
        tx_ = (int)(m10 / m00) + sx;
        ty_ = (int)(m01 / m00) + 0;
      }
    }
    s_tx[i] = tx_;
    hdr[slot].tail[i] = tx_;
    hdr[slot].tail[LM_TAIL_SEGS + i] = ty_;
  }
  __syncthreads();
  TAIL_PROF(7)
  if (best_s != 0xFFFFFFFFu) {
    if (!gb_s) tail_side_moments<false>(SL, R, rowoff, HS, best_s, s_tx, ms, ntrs);
    else tail_side_moments<true>(SG, R, rowoff, HS, best_s, s_tx, ms, ntrs);
  }
  __syncthreads();
  TAIL_PROF(8)
  // track z (:2728-2737): the side moments of column x_i when x_i > 0
  if (tid < LM_TAIL_SEGS) {
    const int i = tid;
    int tz = -1;
    if (s_tx[i] > 0) {
      double m00 = 0, m01 = 0;
      const double s = 1. / 255;
      for (int ty = 0; ty < ntrs; ++ty) {
        const double mom0 = (double)(255u * ms[(i * ntrs + ty) * 2]) * s;
        const double mom2 = (double)(255u * ms[(i * ntrs + ty) * 2 + 1]) * s;
        const double ym = (double)(ty * 32) * mom0;
        m00 += mom0;
        m01 += mom2 + ym;
      }
      if (m00 > 0) tz = (int)(m01 / m00) + 0;
    }
    hdr[slot].tail[2 * LM_TAIL_SEGS + i] = tz;
  }
  if (prof && threadIdx.x == 0) {
    prof[blockIdx.x * 16 + 9] = clock64();
    prof[blockIdx.x * 16 + 13] = R;
    prof[blockIdx.x * 16 + 15] = wall_clock64();
  }
#undef TAIL_PROF
}

// ------------------------------------------------------------------- k_nms
// One 512-thread block per (frame, list).  Positive detections are filtered by
// TAIL_MASK (bottom lists), sorted by (score desc, row-major index asc) —
// equal to std::sort whenever scores are distinct; on an exact tie the list is
// re-sorted from row-major order with the libstdc++ introsort replica
// (lm_introsort.h) — then clustered: nmsMax for the bottom view,
// peakClustering for the side view.
#ifndef LM_NMS_THREADS
#define LM_NMS_THREADS 512
#endif
#define LM_GLOB_BLOCKS 16   // grid of the global-scratch (<true>) k_nms / k_post launches: one scratch region each
// The LDS instantiation at 36 KB and <= 64 VGPRs (8 waves per SIMD): four
// 512-thread blocks per CU, so a batch's 1,024 (slot, list) blocks are one
// round (at 2,048 entries / 48 KB and 75 VGPRs, three per CU): 67 -> 61 us per
// batch alone, +1 % frames/s with four contexts (profiles/r04/nms/)
#ifndef LM_NMS_CAP
#define LM_NMS_CAP 1536     // entries kept in LDS; larger lists use the global-memory path
#endif
#ifndef LM_NMS_RANKSORT
#define LM_NMS_RANKSORT 768  // up to this many entries: O(n^2/T) rank sort instead of bitonic
#endif
#ifndef LM_NMS_WPE
#define LM_NMS_WPE 8  // amdgpu_waves_per_eu minimum of the LDS instantiation
#endif
// nmsMax's "first earlier overlapping point": every (i < j) pair spread over
// the block (LM_NMS_PAIRPAR entries or fewer), or each j scanning its earlier
// points until its first hit.  All pairs balance a block's threads but test
// ~3x the pairs; with four blocks per CU that VALU time is taken from the
// other blocks and the correlation: the early-exit scan is 1-2 % more
// frames/s with four contexts (profiles/r04/nms/sweep.txt), so it is used.
#ifndef LM_NMS_PAIRPAR
#define LM_NMS_PAIRPAR 0
#endif
#ifndef LM_NMS_BRANCHLESS
#define LM_NMS_BRANCHLESS 1   // overlap test without branches (a zero factor when the rects do not intersect)
#endif


// in-place ascending bitonic sort of a[0..np), np a power of two, block-wide
DEV void bitonic_sort(unsigned long long* a, int np) {
  for (int k = 2; k <= np; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long x = a[i], y = a[ixj];
          const bool up = (i & k) == 0;
          if ((x > y) == up) {
            a[i] = y;
            a[ixj] = x;
          }
        }
      }
      __syncthreads();
    }
  }
}

// ascending sort of n DISTINCT keys by rank counting: every key's position is
// the number of smaller keys.  All lanes of a wave read the same a[i]
// (LDS broadcast), no barrier inside.  tmp holds n keys.
DEV void rank_sort(unsigned long long* a, unsigned long long* tmp, int n) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const unsigned long long key = a[k];
    int r = 0;
    int i = 0;
#pragma unroll 1  // (unrolled further, the loads in flight spill at 64 VGPRs)
    for (; i + 8 <= n; i += 8) {  // 4 x 16 B loads in flight per iteration
      const ulonglong2 q0 = *reinterpret_cast<const ulonglong2*>(a + i);
      const ulonglong2 q1 = *reinterpret_cast<const ulonglong2*>(a + i + 2);
      const ulonglong2 q2 = *reinterpret_cast<const ulonglong2*>(a + i + 4);
      const ulonglong2 q3 = *reinterpret_cast<const ulonglong2*>(a + i + 6);
      r += (q0.x < key) + (q0.y < key) + (q1.x < key) + (q1.y < key) + (q2.x < key) + (q2.y < key) +
           (q3.x < key) + (q3.y < key);
    }
    for (; i < n; ++i) r += a[i] < key;
    tmp[r] = key;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < n; k += blockDim.x) a[k] = tmp[k];
  __syncthreads();
}

// ascending sort of n <= blockDim.x DISTINCT keys (< ~0): every wave sorts
// its 64 keys in registers (bitonic network over lane shuffles), the sorted
// runs go back to a, and each key's position is its index in its run plus,
// for every other run, the count of smaller keys there (binary searches, the
// runs' probes interleaved).  A few shuffle and LDS latencies per step instead
// of rank_sort's n / 8 rounds of loads per key.  tmp holds n keys.
static_assert(LM_NMS_THREADS % 64 == 0 && LM_NMS_THREADS <= 512, "wave_merge_sort: up to 8 runs of 64");
DEV void wave_merge_sort(unsigned long long* a, unsigned long long* tmp, int n) {
  constexpr int NR = LM_NMS_THREADS / 64;  // runs
  const int t = threadIdx.x, lane = t & 63, run = t >> 6, nruns = (n + 63) >> 6;
  unsigned long long v = t < n ? a[t] : ~0ull;
  if (run < nruns) {
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        const unsigned long long p = __shfl_xor(v, j);
        const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
        v = keep_min ? (v < p ? v : p) : (v < p ? p : v);
      }
  }
  __syncthreads();  // every key of a has been read
  if (run < nruns) a[t] = v;  // sorted runs, padded with ~0 past n
  __syncthreads();
  if (t < n) {
    int lo[NR], rank = lane;
#pragma unroll
    for (int r = 0; r < NR; ++r) lo[r] = 0;
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1)
#pragma unroll
      for (int r = 0; r < NR; ++r)
        if (r < nruns && r != run && a[r * 64 + lo[r] + s - 1] < v) lo[r] += s;
#pragma unroll
    for (int r = 0; r < NR; ++r)
      if (r < nruns && r != run) rank += lo[r] + (a[r * 64 + lo[r]] < v ? 1 : 0);
    tmp[rank] = v;
  }
  __syncthreads();
  for (int k = t; k < n; k += blockDim.x) a[k] = tmp[k];
  __syncthreads();
}

struct ReplicaLess {  // compareCandidate on (idx << 32 | score bits) words
  DEV bool operator()(unsigned long long a, unsigned long long b) const {
    return __uint_as_float((unsigned)(a & 0xFFFFFFFFu)) > __uint_as_float((unsigned)(b & 0xFFFFFFFFu));
  }
};

// Rect overlap test of nmsMax / peakClustering (:1698-1709, :1833-1844) on
// packed x | y << 16: inter / (2wh - inter) > 0.5  <=>  3*inter > 2wh.  The two
// are equal for these integers: the margin of the double quotient over 0.5 is
// >= 1/(4wh), far above its rounding error.
DEV bool overlaps_xy(unsigned a, unsigned b, int bw, int bh) {
  const int dx = abs((int)(a & 0xFFFFu) - (int)(b & 0xFFFFu));
  const int dy = abs((int)(a >> 16) - (int)(b >> 16));
  if constexpr (LM_NMS_BRANCHLESS) {
    // no intersection (dx >= bw or dy >= bh) makes a factor 0: 0 > 2wh is false
    return 3 * max(bw - dx, 0) * max(bh - dy, 0) > 2 * bw * bh;
  } else {
    if (dx >= bw || dy >= bh) return false;  // R.area() == 0
    return 3 * (bw - dx) * (bh - dy) > 2 * bw * bh;
  }
}

// std::sort(compareCandidate) replica in level order (lm_introsort.h
// process_range / std_sort_levels; tests/cpp/introsort_check.cpp proves the
// level-order form equal to libstdc++).  Every range of a level is handled
// by one wave:
//  * median-of-3 to the front (lane 0), then libstdc++'s unguarded Hoare
//    partition computed in parallel: with f_k the k-th element from the left
//    that is !(a < pivot) and l_k the k-th from the right that is
//    !(pivot < a) (both in the range as it was before the loop), the loop
//    swaps a[f_k] <-> a[l_k] for k < K, K = first k with f_k >= l_k, and
//    returns min(f_K, l_{K-1}) (f_0 when K = 0);
//  * depth 0: heap sort by lane 0 (libstdc++'s fallback; never seen here);
//  * ranges of <= 64 elements: their whole subtree, leaves' insertion sorts
//    included, in one wave's registers (wave_subtree).  Partitioned level
//    by level down to the 16-element leaves, every level took ~5k cycles,
//    latency-bound (the LDS lists, three wave syncs, the level's two block
//    barriers), and a leaf phase another ~15k: ~64k cycles for a
//    350-element tie list (profiles/r04/nms/kprof_tie_levels.txt).
// q: two queues of qcap (first, last, depth); tf, tr: n ints.
// Lanes of one wave exchanging data through memory.  k_nms reaches its
// arrays through generic pointers (LDS, or global scratch for long lists), so
// the accesses are FLAT instructions, which complete out of order: a
// wavefront-scope fence alone emits no wait, and a lane could read a value
// another lane had stored but whose store had not landed (measured: rare
// wrong leaders in the tie sort and in peakClustering, more often when other
// kernels load the memory system).  Drain both counters, then a workgroup
// fence for the global-scratch case, then the wave barrier.
DEV void wave_sync() {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

DEV int wave_partition(unsigned long long* a, int F, int L, int* tf, int* tr) {
  const ReplicaLess comp;
  const int lane = threadIdx.x & 63;
  if (lane == 0) {
    const int mid = F + (L - F) / 2;
    lm_sort::move_median_to_first(a + F, a + F + 1, a + mid, a + L - 1, comp);
  }
  wave_sync();
  const unsigned long long pv = a[F];
  const int lo = F + 1, hi = L;
  // ranks of the stoppers; tf[lo + k] = f_k, tr[lo + k] = k-th R-stopper from the LEFT
  int nl = 0, nr = 0;
  for (int b = lo; b < hi; b += 64) {
    const int i = b + lane;
    bool lf = false, rf = false;
    if (i < hi) {
      const unsigned long long v = a[i];
      lf = !comp(v, pv);
      rf = !comp(pv, v);
    }
    const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
    const unsigned long long below = (1ull << lane) - 1;
    if (lf) tf[lo + nl + __popcll(ml & below)] = i;
    if (rf) tr[lo + nr + __popcll(mr & below)] = i;
    nl += __popcll(ml);
    nr += __popcll(mr);
  }
  wave_sync();
  // K: f_k < l_k holds for a prefix of k
  int K = 0;
  const int kmax = min(nl, nr);
  for (int b = 0; b < kmax; b += 64) {
    const int k = b + lane;
    const bool ok = k < kmax && tf[lo + k] < tr[lo + nr - 1 - k];
    const unsigned long long m = __ballot(ok);
    K += __popcll(m);
    if (m != ~0ull) break;
  }
  int cut;
  if (K == 0) cut = tf[lo];
  else cut = min(K < nl ? tf[lo + K] : 0x7fffffff, tr[lo + nr - K]);
  for (int k = lane; k < K; k += 64) {
    const int i = tf[lo + k], j = tr[lo + nr - 1 - k];
    const unsigned long long x = a[i], y = a[j];
    a[i] = y;
    a[j] = x;
  }
  wave_sync();
  return cut;
}

DEV unsigned long long readlane_u64(unsigned long long v, int l) {
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)v, l);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
  return ((unsigned long long)hi << 32) | lo;
}
DEV unsigned long long bpermute_u64(unsigned long long v, int src) {  // lane src's v
  const unsigned lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)v);
  const unsigned hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}
DEV unsigned long long permute_u64(unsigned long long v, int dst) {  // v to lane dst (a permutation)
  const unsigned lo = __builtin_amdgcn_ds_permute(dst << 2, (int)(unsigned)v);
  const unsigned hi = __builtin_amdgcn_ds_permute(dst << 2, (int)(unsigned)(v >> 32));
  return ((unsigned long long)hi << 32) | lo;
}
// position of the k-th (0-based) set bit of m counting from bit 0 (m must
// have more than k set bits)
DEV int nth_set_bit(unsigned long long m, int k) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const int c = __popcll((m >> pos) & ((1ull << w) - 1));
    if (k >= c) {
      k -= c;
      pos += w;
    }
  }
  return pos;
}

// One range [F, L) of <= 64 elements at depth d0, finished by one wave in
// registers (element F + i in lane i): every partition of its introsort
// subtree, then the final insertion sort of its leaves.  The ranges of the
// subtree are disjoint and what happens to a range depends on its contents
// and depth alone (lm_introsort.h, level-order formulation), so they are
// taken one at a time, lowest first: `bnd` marks where the ranges start,
// `pend` those of > kThreshold elements still to partition, lane s's `dep`
// the depth of the range starting at s.  A partition is wave_partition's
// (median of three to the front, then the k-th !(a < pivot) element from the
// left swapped with the k-th !(pivot < a) from the right while the first is
// left of the second) on ballots instead of LDS lists; a leaf's insertion
// sort is its stable sort (each element's place: the leaf's elements that
// compare before it, and the equal ones left of it).  No LDS round trip and
// no barrier except on the depth-0 heap-sort fallback.
DEV void wave_subtree(unsigned long long* a, int F, int L, int d0) {
  const ReplicaLess comp;
  constexpr int TH = lm_sort::kThreshold;
  const int lane = threadIdx.x & 63;
  const int m = L - F;
  unsigned long long v = lane < m ? a[F + lane] : 0ull;
  unsigned long long bnd = 1ull, pend = m > TH ? 1ull : 0ull;
  int dep = d0;
  const unsigned long long below = (1ull << lane) - 1;
  while (pend) {
    const int s = __builtin_ctzll(pend);  // s + TH < m <= 64
    pend &= pend - 1;
    const unsigned long long after = bnd & ~((2ull << s) - 1);
    const int e = after ? __builtin_ctzll(after) : m;
    const int d = __builtin_amdgcn_readlane(dep, s);
    if (d == 0) {  // depth limit: libstdc++'s heap sort, by lane 0 (never seen here)
      if (lane < m) a[F + lane] = v;
      wave_sync();
      if (lane == 0) lm_sort::partial_sort_full(a + F + s, a + F + e, comp);
      wave_sync();
      v = lane < m ? a[F + lane] : 0ull;
      continue;  // sorted: its leaf sort below leaves it as it is
    }
    // move_median_to_first(s, s + 1, mid, e - 1)
    const int mid = s + (e - s) / 2;
    const unsigned long long x = readlane_u64(v, s + 1), y = readlane_u64(v, mid), z = readlane_u64(v, e - 1);
    int ch;
    if (comp(x, y)) ch = comp(y, z) ? mid : comp(x, z) ? e - 1 : s + 1;
    else ch = comp(x, z) ? s + 1 : comp(y, z) ? e - 1 : mid;
    const unsigned long long vs = readlane_u64(v, s), pv = readlane_u64(v, ch);
    if (lane == s) v = pv;
    if (lane == ch) v = vs;
    const bool in = lane > s && lane < e;
    const bool lf = in && !comp(v, pv), rf = in && !comp(pv, v);
    const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
    const int nl = __popcll(ml), nr = __popcll(mr);
    const int fk = nth_set_bit(ml, lane);           // f_k, k = lane (lane < nl)
    const int lk = nth_set_bit(mr, nr - 1 - lane);  // l_k, k = lane (lane < nr)
    const int K = __popcll(__ballot(lane < nl && lane < nr && fk < lk));
    int cut;
    if (K == 0) {
      cut = __builtin_amdgcn_readlane(fk, 0);
    } else {
      cut = __builtin_amdgcn_readlane(lk, K - 1);
      if (K < nl) cut = min(cut, __builtin_amdgcn_readlane(fk, K));
    }
    // swap a[f_k] <-> a[l_k], k < K (no element is both an f_k and an l_k)
    const int rl = __popcll(ml & below), rr = __popcll(mr >> lane) - 1;
    const int from_l = __shfl(lk, rl), from_r = __shfl(fk, rr & 63);
    const int src = (lf && rl < K) ? from_l : (rf && rr < K) ? from_r : lane;
    v = bpermute_u64(v, src);
    if (lane == s || (lane == cut && cut < e)) dep = d - 1;
    if (cut < e) bnd |= 1ull << cut;
    if (cut - s > TH) pend |= 1ull << s;
    if (e - cut > TH) pend |= 1ull << cut;
  }
  // leaves: stable sort of each (a heap-sorted range keeps its order)
  const unsigned long long upto = lane == 63 ? ~0ull : (2ull << lane) - 1;
  const int ls = 63 - __builtin_clzll(bnd & upto);
  const unsigned long long aft = bnd & ~upto;
  const int le = aft ? __builtin_ctzll(aft) : m;
  const float sc = __uint_as_float((unsigned)v);
  int rk = 0;
#pragma unroll
  for (int j = 0; j < TH; ++j) {
    const int i = ls + j;
    const float sj = __shfl(sc, i & 63);
    if (i < le) rk += (sj > sc) || (i < lane && !(sc > sj));
  }
  const int dst = lane >= m ? lane : le - ls <= TH ? ls + rk : lane;
  v = permute_u64(v, dst);
  if (lane < m) a[F + lane] = v;
}

// wave_partition by the whole block: the stoppers' ranks come from per-wave
// ballot counts (s_w: 2 nw + 1 ints), the swaps are spread over the block.
DEV int block_partition(unsigned long long* a, int F, int L, int* tf, int* tr, int* s_w) {
  const ReplicaLess comp;
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6, nw = blockDim.x >> 6;
  if (t == 0) {
    const int mid = F + (L - F) / 2;
    lm_sort::move_median_to_first(a + F, a + F + 1, a + mid, a + L - 1, comp);
    s_w[2 * nw] = 0;
  }
  __syncthreads();
  const unsigned long long pv = a[F];
  const int lo = F + 1, hi = L;
  const unsigned long long below = (1ull << lane) - 1;
  int nl = 0, nr = 0;
  for (int b = lo; b < hi; b += blockDim.x) {
    const int i = b + t;
    bool lf = false, rf = false;
    if (i < hi) {
      const unsigned long long v = a[i];
      lf = !comp(v, pv);
      rf = !comp(pv, v);
    }
    const unsigned long long ml = __ballot(lf), mr = __ballot(rf);
    if (lane == 0) {
      s_w[wid] = __popcll(ml);
      s_w[nw + wid] = __popcll(mr);
    }
    __syncthreads();
    int bl = nl, br = nr, tl = 0, tr_ = 0;
    for (int w = 0; w < nw; ++w) {
      const int cl = s_w[w], cr = s_w[nw + w];
      if (w < wid) {
        bl += cl;
        br += cr;
      }
      tl += cl;
      tr_ += cr;
    }
    if (lf) tf[lo + bl + __popcll(ml & below)] = i;
    if (rf) tr[lo + br + __popcll(mr & below)] = i;
    nl += tl;
    nr += tr_;
    __syncthreads();  // the lists are complete, s_w free again
  }
  const int kmax = min(nl, nr);
  for (int k0 = 0; k0 < kmax; k0 += blockDim.x) {  // K: f_k < l_k holds for a prefix of k
    const int k = k0 + t;
    const unsigned long long m = __ballot(k < kmax && tf[lo + k] < tr[lo + nr - 1 - k]);
    if (lane == 0 && m) atomicAdd(&s_w[2 * nw], __popcll(m));
  }
  __syncthreads();
  const int K = s_w[2 * nw];
  int cut;
  if (K == 0) cut = tf[lo];
  else cut = min(K < nl ? tf[lo + K] : 0x7fffffff, tr[lo + nr - K]);
  for (int k = t; k < K; k += blockDim.x) {
    const int i = tf[lo + k], j = tr[lo + nr - 1 - k];
    const unsigned long long x = a[i], y = a[j];
    a[i] = y;
    a[j] = x;
  }
  __syncthreads();
  return cut;
}

// Ranges of <= 64 elements go to a list (`small`, packed first | size << 11
// | depth << 18) that the waves finish at the end with wave_subtree; the
// others are partitioned level by level, by the whole block when a level
// holds one range (the top levels, and the long chains of uneven partitions
// that exact ties produce), else one wave per range.
// prof (LM_KPROF=1, else null): [0] clock at the end of the levels, [1] the
// number of levels
DEV int small_range(int f, int l, int d) { return f | (l - f) << 11 | d << 18; }
DEV void std_sort_levels_dev(unsigned long long* a, int n, int* q, int qcap, int* small, int* tf, int* tr,
                             int* s_cnt, int* s_w, long long* prof = nullptr) {
  static_assert(LM_NMS_CAP <= 2048, "small_range packs first in 11 bits");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int* s_small = s_w + 2 * nw + 1;
  const ReplicaLess comp;
  if (threadIdx.x == 0) {
    const int d0 = 2 * lm_sort::lg_(n);
    s_cnt[0] = n > 64 ? 1 : 0;
    s_cnt[1] = 0;
    *s_small = 0;
    if (n > 64) {
      q[0] = 0;
      q[1] = n;
      q[2] = d0;
    } else if (n > 0) {
      small[0] = small_range(0, n, d0);
      *s_small = 1;
    }
  }
  __syncthreads();
  // children of a partitioned range: > 64 elements to the next level, the rest to `small`
  auto push = [&](int* nxt, int sel, int f, int l, int d) {
    if (l - f > 64) {
      const int k = atomicAdd(&s_cnt[1 - sel], 1);
      nxt[3 * k] = f;
      nxt[3 * k + 1] = l;
      nxt[3 * k + 2] = d;
    } else if (l > f) {
      small[atomicAdd(s_small, 1)] = small_range(f, l, d);
    }
  };
  int sel = 0;
  while (true) {
    const int qn = s_cnt[sel];
    if (qn == 0) break;
    const int* cur = q + sel * 3 * qcap;
    int* nxt = q + (1 - sel) * 3 * qcap;
    if (qn == 1 && cur[2] > 0) {
      const int f = cur[0], l = cur[1], d = cur[2];
      const int cut = block_partition(a, f, l, tf, tr, s_w);
      if (threadIdx.x == 0) {
        push(nxt, sel, f, cut, d - 1);
        push(nxt, sel, cut, l, d - 1);
      }
    } else {
      for (int r = wid; r < qn; r += nw) {
        const int f = cur[3 * r], l = cur[3 * r + 1], d = cur[3 * r + 2];
        if (d == 0) {
          if (lane == 0) lm_sort::partial_sort_full(a + f, a + l, comp);  // sorted: a leaf
        } else {
          const int cut = wave_partition(a, f, l, tf, tr);
          if (lane == 0) {
            push(nxt, sel, f, cut, d - 1);
            push(nxt, sel, cut, l, d - 1);
          }
        }
        wave_sync();
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_cnt[sel] = 0;
    sel = 1 - sel;
    __syncthreads();
    if (prof && threadIdx.x == 0) ++prof[1];
  }
  if (prof && threadIdx.x == 0) prof[0] = clock64();
  const int ns = *s_small;
  for (int r = wid; r < ns; r += nw) {  // the whole subtree and its leaves' insertion sorts
    const int e = small[r];
    const int f = e & 0x7FF;
    wave_subtree(a, f, f + ((e >> 11) & 0x7F), e >> 18);
  }
  __syncthreads();
}

// Enumerates the j in [0, n) with flag(j) in increasing order: out[r] = j.
// Returns their count.
template <class F>
DEV int block_compact(int n, F flag, int* out, int* s_wsum) {
  const int T = blockDim.x, chunk = (n + T - 1) / T;
  const int j0 = threadIdx.x * chunk, j1 = min(n, j0 + chunk);
  int c = 0;
  for (int j = j0; j < j1; ++j) c += flag(j);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int v = c;  // inclusive wave scan
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) s_wsum[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int w = 0; w < (T >> 6); ++w) {
      const int t = s_wsum[w];
      s_wsum[w] = acc;
      acc += t;
    }
    s_wsum[T >> 6] = acc;
  }
  __syncthreads();
  int r = s_wsum[wid] + v - c;
  for (int j = j0; j < j1; ++j)
    if (flag(j)) out[r++] = j;
  const int total = s_wsum[T >> 6];
  __syncthreads();
  return total;
}

DEV double readlane_f64(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// The body of k_nms on its working arrays: LDS (GLOB = false, every access a
// ds_* instruction) or per-block global scratch for lists above LM_NMS_CAP.
// Kept as two instantiations so the common case never goes through generic
// (FLAT) pointers, which cost several times the latency of LDS accesses.
// optional phase timestamps (LM_KPROF=1): clock64() of thread 0 per phase
#ifndef LM_NMS_PREHASH
#define LM_NMS_PREHASH 1
#endif
#ifndef LM_NMS_TIE_PRIO
#define LM_NMS_TIE_PRIO 3  // s_setprio of a tie block's waves (0: as every block)
#endif
#define NMS_PROF(k) \
  if (prof && threadIdx.x == 0) prof[(blockIdx.x * 2 + (blockIdx.y & 1)) * 16 + (k)] = clock64();
template <bool GLOB>
DEV auto nms_run(const LmConst& K, const LmDet& D, LmSlotOut* H, int slot, int list, int side, int feat, int n_in,
                 const unsigned long long* __restrict__ src, const unsigned long long* __restrict__ tailmask,
                 unsigned long long* a, int* assign, int* mlist, unsigned* xy, int* s_tmp, unsigned long long* stmp,
                 int qcap, int* s_stk, int* s_wsum,
                 int* s_n_, int* s_flag_, int* s_qcnt, int* s_part, unsigned long long* __restrict__ keys,
                 int32_t* __restrict__ err,
                 long long* __restrict__ prof) -> int {
  int& s_n = *s_n_;
  int& s_flag = *s_flag_;
  constexpr bool glob = GLOB;
  int* s_assign = assign;
  int* s_mlist = mlist;
  unsigned* s_xy = xy;
  if (threadIdx.x == 0) {
    s_n = 0;
    s_flag = 0;
  }
  __syncthreads();
  // load + TAIL_MASK filter (bottom: mask(BB_BOTTOM_TAIL).setTo(255, TAIL_MASK), :783)
  const int tnb = (K.tail_w + 63) / 64;  // TAIL_MASK bitmap words per row
  const unsigned long long* __restrict__ tm = tailmask + (int64_t)slot * K.tail_hb * tnb;
  for (int k = threadIdx.x; k < n_in; k += blockDim.x) {
    const unsigned long long v = src[k];
    bool keep = true;
    if (!side) {
      const unsigned idx = key_lo(v);
      const int y = idx / D.ow, x = idx - y * D.ow;
      if (x < K.tail_w && y < K.tail_hb && ((tm[y * tnb + (x >> 6)] >> (x & 63)) & 1)) keep = false;
    }
    if (keep) a[atomicAdd(&s_n, 1)] = v;
  }
  __syncthreads();
  NMS_PROF(1)
  const int n = s_n;
  if (prof && threadIdx.x == 0) prof[(blockIdx.x * 2 + (blockIdx.y & 1)) * 16 + 13] = n;
  int np = 1;
  while (np < n) np <<= 1;
  // Exact score ties, found before sorting (an LDS hash set of the score
  // bits, linear probing, at most half full): a tie list is re-sorted from
  // row-major order by the std::sort replica below, so its (score, index)
  // sort would be thrown away -- ~20k cycles of the slowest blocks.
  // The table is the next power of two >= 2n and lives in s_tmp
  // (LM_NMS_CAP ints), so it is used only when that power fits: n <= 512 at
  // LM_NMS_CAP = 1536 (2n <= CAP alone would let 513..768 keys write a
  // 2048-entry table past s_tmp).
  int tb = 64, lg = 6;
  while (tb < 2 * n) {
    tb <<= 1;
    ++lg;
  }
  const bool pre = LM_NMS_PREHASH && !glob && tb <= LM_NMS_CAP;
  if (pre) {
    unsigned* tab = reinterpret_cast<unsigned*>(s_tmp);
    for (int k = threadIdx.x; k < tb; k += blockDim.x) tab[k] = ~0u;  // empty: a NaN pattern no score has
    __syncthreads();
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const unsigned h = (unsigned)(a[k] >> 32);
      // Fibonacci hashing: the product's HIGH bits, which every bit of the
      // score feeds (scores of a smooth map often share their low mantissa
      // bits, and the low bits of the product only see those)
      unsigned sl = (h * 2654435761u) >> (32 - lg);
      while (true) {
        const unsigned old = atomicCAS(&tab[sl], ~0u, h);
        if (old == ~0u) break;
        if (old == h) {
          s_flag = 1;
          break;
        }
        sl = (sl + 1) & (unsigned)(tb - 1);
      }
    }
    __syncthreads();
  }
  if (!(pre && s_flag)) {
    if (!glob && n <= LM_NMS_THREADS) {
      wave_merge_sort(a, stmp, n);
    } else if (n <= LM_NMS_RANKSORT) {
      rank_sort(a, stmp, n);
    } else {
      for (int k = n + threadIdx.x; k < np; k += blockDim.x) a[k] = ~0ull;
      __syncthreads();
      bitonic_sort(a, np);
    }
  }
  NMS_PROF(2)
  if (!pre) {
    for (int k = threadIdx.x; k + 1 < n; k += blockDim.x)
      if ((a[k] >> 32) == (a[k + 1] >> 32)) s_flag = 1;
    __syncthreads();
  }
  const int tie = s_flag;
  if (tie) {  // (GLOB: the row-major re-sort below is the single-thread replica)
    // A tie block is the launch's slowest (the replica's levels, then the
    // same clustering as every block) and shares its CU with three others
    // that end far earlier: its waves take issue priority for the rest of
    // the block, so the span is more nearly its own length.
    __builtin_amdgcn_s_setprio(LM_NMS_TIE_PRIO);
    // exact score tie: std::sort from the row-major order nmsMax builds (:1638-1648)
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const unsigned long long v = a[k];
      a[k] = ((unsigned long long)key_lo(v) << 32) | (unsigned)(~(unsigned)(v >> 32));
    }
    // every key must be re-keyed before any thread ranks them (rank_sort reads
    // all n keys); without this barrier a lagging wave's old-format keys were
    // ranked among new-format ones -- duplicate ranks, unwritten slots, and
    // garbage candidates in rare tie blocks
    __syncthreads();
    NMS_PROF(8)
    if (!glob) {
      if (n <= LM_NMS_THREADS) {  // back to row-major order
        wave_merge_sort(a, stmp, n);
      } else if (n <= LM_NMS_RANKSORT) {
        rank_sort(a, stmp, n);
      } else {
        for (int k = n + threadIdx.x; k < np; k += blockDim.x) a[k] = ~0ull;
        __syncthreads();
        bitonic_sort(a, np);
      }
      NMS_PROF(9)
      std_sort_levels_dev(a, n, s_mlist, qcap, s_assign, reinterpret_cast<int*>(s_xy), s_tmp, s_qcnt, s_part,
                          prof ? prof + (blockIdx.x * 2 + (blockIdx.y & 1)) * 16 + 11 : nullptr);
      NMS_PROF(10)
    } else {  // rare and slow: one thread, explicit stack
      for (int k = n + threadIdx.x; k < np; k += blockDim.x) a[k] = ~0ull;
      __syncthreads();
      if (np > 1) bitonic_sort(a, np);
      if (threadIdx.x == 0) lm_sort::std_sort(a, a + n, ReplicaLess(), s_stk);
      __syncthreads();
    }
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      const unsigned long long v = a[k];
      a[k] = ((unsigned long long)(~(unsigned)(v & 0xFFFFFFFFu)) << 32) | (unsigned)(v >> 32);
    }
    __syncthreads();
  }
  // row-major index -> packed (x | y << 16), once per detection
  const int ow = D.ow, bw = D.box_w, bh = D.box_h;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const unsigned idx = key_lo(a[k]);
    const unsigned y = idx / ow, x = idx - y * ow;
    xy[k] = x | (y << 16);
  }
  for (int k = n + threadIdx.x; k < ((n + 15) & ~15); k += blockDim.x) xy[k] = 0;
  __syncthreads();
  NMS_PROF(3)
  if (!side) {
    // nmsMax: every point, suppressed or not, suppresses the later points it
    // overlaps (:1677-1720) => j belongs to the first i < j overlapping it;
    // maxima by pointer jumping.
    if (n <= LM_NMS_PAIRPAR) {
      // Every (i < j) pair tested once, spread evenly over the block: tile
      // (b, j) holds the pairs i in [16 b, min(16 b + 16, j)), tiles in (b, j)
      // order, a thread takes every blockDim-th one; its first hit goes to
      // assign[j] by an LDS atomicMin.  (Each j scanning its earlier points
      // until its first hit left the block waiting for the last maxima's full
      // scans: ~25k cycles at ~300 points.)
      for (int j = threadIdx.x; j < n; j += blockDim.x) assign[j] = j;
      __syncthreads();
      int b = 0, j = 1 + threadIdx.x;  // tile index threadIdx.x: row b = 0 holds j = 1 .. n - 1
      while (true) {
        while (b * 16 + 1 < n && j >= n) {  // past row b: into row b + 1 (j = 16 (b + 1) + 1 ..)
          const int over = j - n;
          ++b;
          j = 16 * b + 1 + over;
        }
        if (j >= n) break;
        const int i0 = 16 * b;
        unsigned v[16];
        *reinterpret_cast<uint4*>(v) = *reinterpret_cast<const uint4*>(xy + i0);
        *reinterpret_cast<uint4*>(v + 4) = *reinterpret_cast<const uint4*>(xy + i0 + 4);
        *reinterpret_cast<uint4*>(v + 8) = *reinterpret_cast<const uint4*>(xy + i0 + 8);
        *reinterpret_cast<uint4*>(v + 12) = *reinterpret_cast<const uint4*>(xy + i0 + 12);
        const unsigned xj = xy[j];
        unsigned hit = 0;
#pragma unroll
        for (int t = 0; t < 16; ++t) hit |= (unsigned)(i0 + t < j && overlaps_xy(v[t], xj, bw, bh)) << t;
        if (hit) atomicMin(&assign[j], i0 + __ffs(hit) - 1);
        j += blockDim.x;
      }
    } else {
      // long lists: each j scans the earlier points 16 at a time (4 x 16 B
      // loads in flight) and stops at its first hit
      for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const unsigned xj = xy[j];
        int as = j;
        for (int i0 = 0; i0 < j && as == j; i0 += 16) {
          unsigned v[16];
          *reinterpret_cast<uint4*>(v) = *reinterpret_cast<const uint4*>(xy + i0);
          *reinterpret_cast<uint4*>(v + 4) = *reinterpret_cast<const uint4*>(xy + i0 + 4);
          *reinterpret_cast<uint4*>(v + 8) = *reinterpret_cast<const uint4*>(xy + i0 + 8);
          *reinterpret_cast<uint4*>(v + 12) = *reinterpret_cast<const uint4*>(xy + i0 + 12);
          unsigned hit = 0;
#pragma unroll
          for (int t = 0; t < 16; ++t) hit |= (unsigned)(i0 + t < j && overlaps_xy(v[t], xj, bw, bh)) << t;
          if (hit) as = i0 + __ffs(hit) - 1;
        }
        assign[j] = as;
      }
    }
    __syncthreads();
    NMS_PROF(4)
    while (true) {
      if (threadIdx.x == 0) s_flag = 0;
      __syncthreads();
      for (int j = threadIdx.x; j < n; j += blockDim.x) {
        const int m = assign[j], mm = assign[m];
        if (mm != m) {
          assign[j] = mm;
          s_flag = 1;
        }
      }
      __syncthreads();
      const int again = s_flag;
      __syncthreads();
      if (!again) break;
    }
  } else if (threadIdx.x < 64) {
    // peakClustering: leaders in sorted order; each claims the undecided
    // points overlapping it (:1815-1850).  One wave, no block barriers:
    // assign[j] = leader, -1 undecided.
    const int lane = threadIdx.x;
    for (int j = lane; j < n; j += 64) assign[j] = -1;
    wave_sync();
    int lead = 0;
    while (lead < n) {
      const unsigned xl = xy[lead];
      if (lane == 0) assign[lead] = lead;
      int next = n;
      for (int b = lead + 1; b < n; b += 64) {
        const int j = b + lane;
        bool und = false;
        if (j < n && assign[j] < 0) {
          if (overlaps_xy(xl, xy[j], bw, bh)) assign[j] = lead;
          else und = true;
        }
        const unsigned long long m = __ballot(und);
        if (m && next == n) next = b + __ffsll((long long)m) - 1;
      }
      wave_sync();  // the next leader's sweep reads assign[] entries other lanes just wrote
      lead = next;
    }
  }
  __syncthreads();
  NMS_PROF(5)
  // maxima (leaders) in sorted order
  const int ncand = block_compact(n, [&](int j) { return assign[j] == j; }, mlist, s_wsum);
  LmCand* __restrict__ out = LM_CAND_STAGE(K, keys, slot, list);
  const bool fits = ncand <= K.list_cap[list] / 2;  // always: maxima are >= w/3 apart
  if (!fits && threadIdx.x == 0) atomicOr(err, 32);
  NMS_PROF(6)
  // weighted mean over each cluster's members in sorted order, in double
  // (:1731-1744 / :1865-1883).  One wave per cluster: members are found 64 at
  // a time with a ballot; the products x*s, y*s are exact in double, so they
  // are formed per lane and only the additions run in member order.
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int r = wid; r < ncand && fits; r += nw) {
    const int m = mlist[r];
    double wx = 0, wy = 0, ss = 0;
    int members = 0;
    for (int b = m; b < n; b += 64) {
      const int j = b + lane;
      bool mem = false;
      double px = 0, py = 0, ps = 0;
      if (j < n && assign[j] == m) {
        mem = true;
        const unsigned q = xy[j];
        ps = (double)key_score(a[j]);
        px = (double)(int)(q & 0xFFFFu) * ps;
        py = (double)(int)(q >> 16) * ps;
      }
      unsigned long long mask = __ballot(mem);
      members += __popcll(mask);
      while (mask) {
        const int sl = __ffsll((long long)mask) - 1;
        mask &= mask - 1;
        wx += readlane_f64(px, sl);
        wy += readlane_f64(py, sl);
        ss += readlane_f64(ps, sl);
      }
    }
    if (lane == 0) {
      const unsigned xm = xy[m];
      LmCand c;
      c.s = (double)key_score(a[m]);
      if (!side) {  // Point_<double> / double -> Point_<int>: cvRound (half even)
        c.x = (int)rint(wx / ss);
        c.y = (int)rint(wy / ss);
      } else if (members > 1) {  // std::round (half away from zero)
        c.x = (int)round(wx / ss);
        c.y = (int)round(wy / ss);
      } else {
        c.x = (int)(xm & 0xFFFFu);
        c.y = (int)(xm >> 16);
      }
      out[r] = c;
    }
  }
  NMS_PROF(7)
  if (prof && threadIdx.x == 0) prof[(blockIdx.x * 2 + (blockIdx.y & 1)) * 16 + 15] = wall_clock64();
  if (threadIdx.x == 0) {
    H->n_pos[list] = n;
    H->cand_cnt[list] = fits ? ncand : 0;
    H->ties[list] = tie;
  }
  return fits ? ncand : 0;
}

// One block per (slot, list): nmsMax for the bottom lists, peakClustering
// for the side lists.  detectSideCandidates runs only when the frame's
// bottom candidate list for the feature is non-empty (:820-833); nmsMax makes
// at least one candidate from any non-empty point list, so "is any bottom
// key left after the TAIL_MASK filter" decides it.  k_tail records that per
// (slot, feature) in the slot header (LmSlotOut::bottom_kept) before k_nms
// runs, so a side block neither waits for the bottom block nor reads the
// bottom keys the bottom block overwrites with its staged candidates.
// <false>: lists of at most LM_NMS_CAP positives, in LDS.  <true>: the
// longer lists, in global scratch (for_overflow_pairs, launched after
// <false>).

template <bool GLOB>
DEV void nms_block(int bx, int list, const LmConst* __restrict__ Kp, int s0, unsigned long long* __restrict__ keys,
                   const int32_t* __restrict__ n_pos, const unsigned long long* __restrict__ tailmask,
                   unsigned long long* __restrict__ gscratch, int64_t gscratch_slot, LmSlotOut* __restrict__ hdr,
                   int32_t* __restrict__ err, long long* __restrict__ prof_b, long long* __restrict__ prof_s) {
  constexpr int ACAP = GLOB ? 1 : LM_NMS_CAP;  // LDS array sizes
  const LmConst& K = *Kp;
  const int slot = s0 + bx;
  const int feat = list & 1, side = list >> 1;  // feat: 0 paw, 1 snout
  LmSlotOut* H = hdr + slot;
  // 16-byte aligned: the sorts and the nmsMax sweep read them with ds_read_b128
  __shared__ __attribute__((aligned(16))) unsigned long long s_keys[ACAP];
  __shared__ __attribute__((aligned(16))) int s_assign[ACAP];
  __shared__ int s_mlist[ACAP];
  __shared__ __attribute__((aligned(16))) unsigned s_xy[ACAP + 16];
  __shared__ int s_tmp[LM_NMS_CAP];
  __shared__ int s_stk[GLOB ? lm_sort::kStackInts : 1];
  __shared__ int s_wsum[LM_NMS_THREADS / 64 + 1];
  __shared__ int s_n, s_flag, s_qcnt[2];
  __shared__ int s_part[2 * (LM_NMS_THREADS / 64) + 2];  // block_partition's counts + the small-range count
  static_assert(LM_NMS_RANKSORT * 8 <= LM_NMS_CAP * 4, "s_assign holds the sorts' keys");
  const int64_t npg = gscratch_slot / 3;
  // <true>: the launch's block b works its pairs one after another in scratch region b
  unsigned long long* ga = gscratch + (int64_t)(GLOB ? blockIdx.x : 0) * gscratch_slot;
  int* gassign = reinterpret_cast<int*>(ga + npg);
  int* gmlist = gassign + npg;
  const int n_in = n_pos[slot * LM_NLIST + list];
  if (side && slot < 1) return;  // the previous frame (halo slot): bottom lists only
  if (GLOB != (n_in > LM_NMS_CAP)) return;  // the other instantiation's list
  const int det = side ? (feat == 0 ? DET_PAW_S : DET_SNOUT_S) : (feat == 0 ? DET_PAW_B : DET_SNOUT_B);
  const LmDet D = K.det[det];
  if (side) {
    if (!H->bottom_kept[feat]) {  // set by k_tail from the keys before any block stages candidates over them
      if (threadIdx.x == 0) {  // detectSideCandidates not run: an empty side list
        H->n_pos[list] = 0;
        H->cand_cnt[list] = 0;
        H->ties[list] = 0;
      }
      return;
    }
  }
  long long* prof = side ? prof_s : prof_b;
  NMS_PROF(0)
  if (prof && threadIdx.x == 0) prof[(blockIdx.x * 2 + (blockIdx.y & 1)) * 16 + 14] = wall_clock64();
  const unsigned long long* __restrict__ src = keys + (int64_t)slot * K.keys_per_slot + K.list_off[list];
  if constexpr (!GLOB)
    nms_run<false>(K, D, H, slot, list, side, feat, n_in, src, tailmask, s_keys, s_assign, s_mlist, s_xy, s_tmp,
                   reinterpret_cast<unsigned long long*>(s_assign), LM_NMS_CAP / 6, s_stk, s_wsum, &s_n, &s_flag, s_qcnt, s_part,
                   keys, err, prof);
  else
    nms_run<true>(K, D, H, slot, list, side, feat, n_in, src, tailmask, ga, gassign, gmlist,
                  reinterpret_cast<unsigned*>(gmlist + npg), s_tmp, reinterpret_cast<unsigned long long*>(gassign), 0,
                  s_stk, s_wsum, &s_n, &s_flag, s_qcnt, s_part, keys, err, prof);
}

// For the <true> (global-scratch) instantiations of k_nms / k_post: a small
// grid finds the (slot, feature) pairs that need it — every thread tests one
// pair, so the usual "none" costs one round of header reads — and the blocks
// share them out.  fn(pair) runs block-wide.
template <class Pred, class Fn>
DEV void for_overflow_pairs(int npairs, Pred overflow, Fn fn) {
  // every block must see the same list in the same order (block b takes
  // entries b, b + gridDim.x, ...): an order-preserving compaction, not
  // atomics (whose order differs between blocks: pairs were skipped or run
  // twice when several overflowed)
  __shared__ int s_list[1024], s_wsum[1024 / 64 + 1];
  for (int c0 = 0; c0 < npairs; c0 += 1024) {
    const int cnt = block_compact(min(npairs - c0, 1024), [&](int j) { return overflow(c0 + j) ? 1 : 0; }, s_list,
                                  s_wsum);
    for (int i = blockIdx.x; i < cnt; i += gridDim.x) {
      fn(c0 + s_list[i]);
      __syncthreads();  // the next pair reuses the block's shared variables
    }
    __syncthreads();
  }
}

// <false>: one block per (slot, feature), lists of at most LM_NMS_CAP
// positives in LDS.  <true>: the longer lists, from global scratch, by a
// small grid that walks all npairs (slot, feature) pairs — usually none
// qualifies, so it costs a launch and a few header reads.  One kernel
// holding both paths ran the common one slower (register allocation).
// LM_KPROF=1: clock64() of thread 0 per k_post phase (LDS instantiation),
// 16 per (frame, feature) block; null otherwise
#define POST_PROF(k)                                                                           \
  if (!G && threadIdx.x == 0) {                                                                \
    long long* pp_ = prof;                                                                     \
    if (pp_) pp_[(blockIdx.x * 2 + blockIdx.y) * 16 + (k)] = (k) >= 14 ? wall_clock64() : clock64(); \
  }
template <bool GLOB>
__global__ __launch_bounds__(LM_NMS_THREADS) __attribute__((amdgpu_waves_per_eu(GLOB ? 1 : LM_NMS_WPE, 8))) void k_nms(const LmConst* __restrict__ Kp, int s0, unsigned long long* __restrict__ keys,
                                                       const int32_t* __restrict__ n_pos, const unsigned long long* __restrict__ tailmask,
                                                       unsigned long long* __restrict__ gscratch, int64_t gscratch_slot,
                                                       LmSlotOut* __restrict__ hdr, int32_t* __restrict__ err,
                                                       long long* __restrict__ prof_b, long long* __restrict__ prof_s,
                                                       int npairs) {
  if constexpr (!GLOB)
    nms_block<false>(blockIdx.x, blockIdx.y, Kp, s0, keys, n_pos, tailmask, gscratch, gscratch_slot, hdr, err, prof_b,
                     prof_s);
  else
    for_overflow_pairs(
        npairs,  // (slot, list) pairs
        [&](int p) {
          const int slot = s0 + (p >> 2), list = p & 3;
          return n_pos[slot * LM_NLIST + list] > LM_NMS_CAP && (slot >= 1 || list < 2);
        },
        [&](int p) {
          nms_block<true>(p >> 2, p & 3, Kp, s0, keys, n_pos, tailmask, gscratch, gscratch_slot, hdr, err, nullptr,
                          nullptr);
        });
#undef NMS_PROF
}

// ------------------------------------------------------------------ k_post
#ifndef LM_POST_THREADS
#define LM_POST_THREADS 256
#endif
#define LM_POST_MAXC 512     // candidates per list handled in LDS
#define LM_POST_MAXOFF 2048  // CSC columns (Ni + Nong) + 1

// checkVelCriterion (:1256-1267): sum(sat_u8(I - I_prev) > 25) >= area*alpha,
// by one whole wave (called with every lane active, arguments wave-uniform):
// the rectangle's pixels are shared out over the lanes and counted with a
// ballot per round, so a check costs a few dependent load chains
// (calibration -> frame -> LUT) instead of one per pixel.
template <class FP>
DEV bool vel_criterion_wave(const LmConst& K, FP Fc, FP Fp, const uint8_t* bkg, const int32_t* cal,
                            const uint8_t* lutc, const uint8_t* lutp, const LmSlot& slc, const LmSlot& slp, int crop_x,
                            int crop_y, int crop_w, int crop_h, int bx, int by, int bwid, int bhei, int area,
                            double alpha, int32_t* err, int tag) {
  const int lane = threadIdx.x & 63;
  if (bx < 0 || by < 0 || bwid < 0 || bhei < 0 || bx + bwid > crop_w || by + bhei > crop_h) {
    if (lane == 0) {
      atomicOr(err, 4);  // cv::Mat ROI assertion in the reference
      if (atomicCAS(&err[1], 0, 1) == 0) {  // first offender, for the error message
        err[2] = tag;
        err[3] = bx;
        err[4] = by;
        err[5] = bwid;
        err[6] = bhei;
        err[7] = crop_w;
        err[8] = crop_h;
      }
    }
    return false;
  }
  const int n = bwid * bhei;
  int sum = 0;
  for (int p0 = 0; p0 < n; p0 += 64) {
    const int p = p0 + lane;
    bool hit = false;
    if (p < n) {
      const int r = p / bwid, c = p - r * bwid;
      const int R = crop_y + by + r, C = crop_x + bx + c;
      const int a = ipad_pixel_t(Fc, bkg, cal, lutc, K, slc, R, C);  // I_*_MOUSE_PAD
      const int b = ipad_pixel_t(Fp, bkg, cal, lutp, K, slp, R, C);  // I_*_MOUSE_PAD_PREV
      hit = (a > b ? a - b : 0) > 25;
    }
    sum += __popcll(__ballot(hit));
  }
  return (double)sum >= ((double)area) * alpha;
}

// Bump allocation of `amount` entries of arena k from sub-arena g (one
// thread): the offset, or -1 with the overflow flag set.
DEV int arena_alloc(LmArenaCtl* __restrict__ ctl, int k, int g, int amount) {
  const int part = ctl->cap[k] / ctl->nparts;
  const int b = atomicAdd(&ctl->sub[g][k], amount);
  if (b + amount > part) {
    atomicOr(&ctl->overflow, 1);
    return -1;
  }
  return g * part + b;
}

// The body of k_post on its working arrays: candidate copies and per-list
// state in LDS (G = false), or, for lists beyond the LDS capacity, the staged
// candidate lists themselves and per-block global scratch (G = true; the
// reference has no size limit).  Two instantiations, so the common case stays
// on ds_* instructions.
template <bool G>
DEV void post_run(const LmConst& K, const LmSlot* __restrict__ slots, const uint8_t* const* __restrict__ frame_ptr,
                  const uint8_t* __restrict__ bkg, const int32_t* __restrict__ cal, const uint8_t* __restrict__ luts,
                  LmSlotOut* H, int slot, int feat, int frame, int Nb, int Ns, int Ni, const LmCand* sb,
                  const LmCand* st, const LmCand* sp, int* s_off, int* s_mb, int* s_mt, float* s_bps, float* s_tpb,
                  int cap, int* s_base, int& s_any1, int& s_any0, LmP22D* __restrict__ arena_p22d,
                  int32_t* __restrict__ arena_side_y, double* __restrict__ arena_side_s, double* __restrict__ arena_unary,
                  int32_t* __restrict__ arena_jc, int32_t* __restrict__ arena_ir, double* __restrict__ arena_pr,
                  LmArenaCtl* __restrict__ ctl, int32_t* __restrict__ err, int sub,
                  long long* __restrict__ prof) {
  POST_PROF(14)
  POST_PROF(0)
  // ---------------- unary (unaryCostBox :1909-1952), column-major Nb x nprior
  const int nprior = feat == 0 ? 4 : 1;
  const int p0 = feat == 0 ? 0 : 4;
  if (threadIdx.x == 0) {
    s_base[0] = arena_alloc(ctl, AR_UNARY, sub, Nb * nprior);
  }
  __syncthreads();
  if (s_base[0] >= 0) {
    const double norm_fact = 1 / sqrt(2.0);
    for (int e = threadIdx.x; e < Nb * nprior; e += blockDim.x) {
      const int j = e / Nb, i = e % Nb;  // column-major: values[j*nrows + i]
      const double* pr = K.prior[p0 + j];
      const double cx = (double)sb[i].x / (double)K.bb_bottom_w, cy = (double)sb[i].y / (double)K.bb_bottom_h;
      const double ax = pr[3], aw = pr[4] - pr[3], ay = pr[5], ah = pr[6] - pr[5];
      double v = 0.0;
      if (ax <= cx && cx < ax + aw && ay <= cy && cy < ay + ah) {
        const double dx = cx - pr[0], dy = cy - pr[1];
        const double dd = __dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy));
        const double val = sqrt(dd) * norm_fact;
        if (val <= pr[2]) v = (1 - val) * sb[i].s;
      }
      arena_unary[s_base[0] + e] = v;
    }
  }
  if (threadIdx.x == 0) {
    H->unary_off[feat] = s_base[0];
    H->unary_cnt[feat] = Nb * nprior;
  }

  POST_PROF(1)
  // ---------------- pairwise (pairwisePotential :1954-2070) when frame > 0
  if (frame > 0) {
    const int Nong = K.ong_nx * K.ong_ny;
    const int ncols = Ni + Nong, nrows = Nb + Nong;
    const double gs = (double)K.ong_spacing_bottom, maxd = (double)K.max_displacement_bottom;
    const double alpha = K.alpha_vel_bottom, occ = K.pairwise_occluded_cost * alpha;
    auto ong_of = [&](const LmCand& c) {
      const int xc = (int)round((K.ong_br_x - (double)c.x) / gs);
      const int yc = (int)round((K.ong_br_y - (double)c.y) / gs);
      const int ox = xc < 0 ? 0 : (xc > K.ong_nx - 1 ? K.ong_nx - 1 : xc);
      const int oy = yc < 0 ? 0 : (yc > K.ong_ny - 1 ? K.ong_ny - 1 : yc);
      return oy * K.ong_nx + ox;
    };
    auto trans = [&](int i, int j) {  // D(j, i) candidate -> candidate
      const double dx = (double)sb[j].x - (double)sp[i].x, dy = (double)sb[j].y - (double)sp[i].y;
      const double dist = sqrt(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)));
      if (!(dist < maxd)) return 0.0;
      double inv = 1 - (dist / maxd);
      return inv * alpha;
    };
    // each bottom candidate's ONG node once (s_mb is free until the matching)
    int* s_ong = s_mb;
    for (int j = threadIdx.x; j < Nb; j += blockDim.x) s_ong[j] = ong_of(sb[j]);
    __syncthreads();
    // column counts -> Jc
    for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
      int cnt = 0;
      if (c < Ni) {
        for (int j = 0; j < Nb; ++j) cnt += trans(c, j) != 0.0;
        cnt += occ != 0.0;
      } else {
        const int q = c - Ni;
        if (Ni > 0 && occ != 0.0)
          for (int j = 0; j < Nb; ++j) cnt += s_ong[j] == q;
        cnt += occ != 0.0;
      }
      s_off[c] = cnt;
    }
    __syncthreads();
    // exclusive scan of the counts by the first wave, 64 columns a round
    if (threadIdx.x < 64) {
      const int lane = threadIdx.x;
      int carry = 0;
      for (int c0 = 0; c0 < ncols; c0 += 64) {
        const int c = c0 + lane;
        const int t = c < ncols ? s_off[c] : 0;
        int v = t;  // inclusive wave scan
        for (int o = 1; o < 64; o <<= 1) {
          const int u = __shfl_up(v, o);
          if (lane >= o) v += u;
        }
        if (c < ncols) s_off[c] = carry + v - t;
        carry += __shfl(v, 63);
      }
      if (lane == 0) s_off[ncols] = carry;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const int acc = s_off[ncols];
      const int bj = arena_alloc(ctl, AR_PWJC, sub, ncols + 1);
      const int bn = arena_alloc(ctl, AR_PWNZ, sub, acc);
      s_base[1] = bn < 0 ? -1 : bj;
      s_base[2] = bn;
    }
    __syncthreads();
    POST_PROF(2)
    const int bj = s_base[1], bn = s_base[2];
    if (bj >= 0) {
      for (int c = threadIdx.x; c <= ncols; c += blockDim.x) arena_jc[bj + c] = s_off[c];
      for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
        int o = bn + s_off[c];
        if (c < Ni) {
          for (int j = 0; j < Nb; ++j) {
            const double v = trans(c, j);
            if (v != 0.0) {
              arena_ir[o] = j;
              arena_pr[o] = v;
              ++o;
            }
          }
          if (occ != 0.0) {
            arena_ir[o] = Nb + ong_of(sp[c]);
            arena_pr[o] = occ;
            ++o;
          }
        } else {
          const int q = c - Ni;
          if (Ni > 0 && occ != 0.0)
            for (int j = 0; j < Nb; ++j)
              if (s_ong[j] == q) {
                arena_ir[o] = j;
                arena_pr[o] = occ;
                ++o;
              }
          if (occ != 0.0) {
            arena_ir[o] = Nb + q;
            arena_pr[o] = occ;
            ++o;
          }
        }
      }
    }
    if (threadIdx.x == 0) {
      H->pw_rows[feat] = nrows;
      H->pw_cols[feat] = ncols;
      H->pw_nnz[feat] = s_off[ncols];
      H->pw_jc_off[feat] = bj;
      H->pw_nz_off[feat] = bn;
    }
    __syncthreads();
  } else if (threadIdx.x == 0) {
    H->pw_rows[feat] = -1;
    H->pw_cols[feat] = -1;
    H->pw_nnz[feat] = 0;
    H->pw_jc_off[feat] = 0;
    H->pw_nz_off[feat] = 0;
  }

  POST_PROF(3)
  // ---------------- matching (:1023-1254)
  const int ovlp = (int)(K.size_b[feat][0] * (1 - K.side_bottom_min_overlap));
  const bool vel_check = frame > 0;
  if (threadIdx.x == 0) {
    s_any1 = 0;
    s_any0 = 0;
  }
  for (int k = threadIdx.x; k < cap; k += blockDim.x) {
    s_mb[k] = -1;
    s_mt[k] = -1;
    s_bps[k] = 0.f;
    s_tpb[k] = 0.f;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < Nb * Ns; e += blockDim.x) {
    const int i = e / Ns, j = e % Ns;
    if (abs(sb[i].x - st[j].x) <= ovlp) s_any1 = 1;
    else s_any0 = 1;
  }
  __syncthreads();
  const bool mixed = s_any1 && s_any0;  // normalize(NORM_MINMAX) all-equal -> all 0 (:1065)
  auto boolD = [&](int i, int j) { return mixed && abs(sb[i].x - st[j].x) <= ovlp; };
  for (int j = threadIdx.x; j < Ns; j += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < Nb; ++i) s += boolD(i, j) ? 1.f : 0.f;
    s_bps[j] = s;
  }
  for (int i = threadIdx.x; i < Nb; i += blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < Ns; ++j) s += boolD(i, j) ? 1.f : 0.f;
    s_tpb[i] = s;
  }
  __syncthreads();
  POST_PROF(4)
  // motion status where the reference evaluates it
  const LmSlot sl = slots[slot], slp = slots[slot - 1];
  const lm_gu8* Fc = as_global(frame_ptr[slot]);
  const lm_gu8* Fp = as_global(frame_ptr[slot - 1]);
  const uint8_t* lutc = luts + slot * 256;
  const uint8_t* lutp = luts + (slot - 1) * 256;
  const int* mbox = K.match_b[feat];
  const int* tbox = K.match_s[feat];
  if (vel_check) {
    // which candidates the reference tests (-2: pending), then one wave per test
    for (int i = threadIdx.x; i < Nb; i += blockDim.x) {
      bool need = false;
      for (int j = 0; j < Ns; ++j) need |= boolD(i, j) && s_bps[j] > 1;
      if (need) s_mb[i] = -2;
    }
    for (int j = threadIdx.x; j < Ns; j += blockDim.x) {
      bool need = false;
      if (s_bps[j] > 1)
        for (int i = 0; i < Nb; ++i) need |= boolD(i, j);
      if (need) s_mt[j] = -2;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int k = wid; k < Nb + Ns; k += nw) {
      if (k < Nb) {
        const int i = k;
        if (s_mb[i] != -2) continue;
        const bool m = vel_criterion_wave(K, Fc, Fp, bkg, cal, lutc, lutp, sl, slp, sl.crop_x[0], sl.crop_y[0], K.crop_w[0],
                                          K.crop_h[0], mbox[0] + sb[i].x + K.spre_b_w, mbox[1] + sb[i].y + K.spre_b_h,
                                          mbox[2], mbox[3], K.size_b[feat][0] * K.size_b[feat][1], 0.02, err,
                                          (slot << 16) | (feat << 12) | i);
        if (lane == 0) s_mb[i] = m;
      } else {
        const int j = k - Nb;
        if (s_mt[j] != -2) continue;
        const bool m = vel_criterion_wave(K, Fc, Fp, bkg, cal, lutc, lutp, sl, slp, sl.crop_x[1], sl.crop_y[1], K.crop_w[1],
                                          K.crop_h[1], tbox[0] + st[j].x + K.spre_t_w, tbox[1] + st[j].y + K.spre_t_h,
                                          tbox[2], tbox[3], K.size_s[feat][0] * K.size_s[feat][1], 0.05, err,
                                          (slot << 16) | (feat << 12) | 0x800 | j);
        if (lane == 0) s_mt[j] = m;
      }
    }
  }
  __syncthreads();
  POST_PROF(5)
  const double walpha = -(1. / (double)ovlp);
  auto matches = [&](int i, int j) {
    if (!boolD(i, j)) return false;
    if ((s_bps[j] > 1) & vel_check) return s_mb[i] == s_mt[j];
    return true;
  };
  // side entries per bottom candidate (>= 1: the "no match" entry)
  for (int i = threadIdx.x; i < Nb; i += blockDim.x) {
    int cnt = 0;
    if (Ns > 0 && s_tpb[i] != 0)
      for (int j = 0; j < Ns; ++j) cnt += matches(i, j);
    s_off[i] = cnt > 0 ? cnt : 1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int i = 0; i < Nb; ++i) {
      const int t = s_off[i];
      s_off[i] = acc;
      acc += t;
    }
    s_off[Nb] = acc;
    const int bp = arena_alloc(ctl, AR_P22D, sub, Nb);
    const int bs = arena_alloc(ctl, AR_SIDE, sub, acc);
    s_base[0] = bs < 0 ? -1 : bp;
    s_base[1] = bs;
  }
  __syncthreads();
  const int bp = s_base[0], bs = s_base[1];
  if (bp >= 0) {
    for (int i = threadIdx.x; i < Nb; i += blockDim.x) {
      const int o = bs + s_off[i];
      int cnt = 0;
      double st0 = -1;
      if (Ns > 0 && s_tpb[i] != 0) {
        for (int j = 0; j < Ns; ++j) {
          if (!matches(i, j)) continue;
          const double wgt = __dadd_rn(__dmul_rn((double)abs(sb[i].x - st[j].x), walpha), 1.0);
          const double sv = st[j].s * wgt;
          // P22D(C_b, C_temp) then add_side_candidate (Candidates.cpp:106-115)
          if (cnt == 0) {
            arena_side_y[o] = st[j].y;
            arena_side_s[o] = sv;
            st0 = sv;
            cnt = 1;
          } else if (st0 < 0) {
            arena_side_y[o] = st[j].y;
            arena_side_s[o] = sv;
            st0 = sv;
          } else {
            if (!(sv >= 0)) atomicOr(err, 16);  // CV_Assert(S >= 0)
            arena_side_y[o + cnt] = st[j].y;
            arena_side_s[o + cnt] = sv;
            ++cnt;
          }
        }
      }
      if (cnt == 0) {
        arena_side_y[o] = -1;  // Candidate(-1, -1, -1)
        arena_side_s[o] = -1;
        cnt = 1;
      }
      LmP22D p;
      p.bottom = sb[i];
      p.side_off = o;
      p.side_cnt = cnt;
      arena_p22d[bp + i] = p;
    }
  }
  POST_PROF(6)
  POST_PROF(15)
  if (threadIdx.x == 0) {
    H->p22d_off[feat] = bp;
    H->p22d_cnt[feat] = Nb;
    H->side_off[feat] = bs;
    H->side_cnt[feat] = s_off[Nb];
  }
}


// Two instantiations, launched back to back on the same grid: <false> takes
// the (slot, feature) blocks whose lists fit the LDS arrays, <true> the rest
// (global scratch).  One kernel holding both paths ran the common one 60 %
// slower (register allocation and code layout of the larger body).
#define LM_POST_ARGS                                                                                               \
  const LmConst *__restrict__ Kp, const LmSlot *__restrict__ slots, const uint8_t *const *__restrict__ frame_ptr,  \
      const uint8_t *__restrict__ bkg, const int32_t *__restrict__ cal, const uint8_t *__restrict__ luts,           \
      LmSlotOut *__restrict__ hdr, const unsigned long long *__restrict__ keys, LmP22D *__restrict__ arena_p22d,    \
      int32_t *__restrict__ arena_side_y, double *__restrict__ arena_side_s, double *__restrict__ arena_unary,      \
      int32_t *__restrict__ arena_jc, int32_t *__restrict__ arena_ir, double *__restrict__ arena_pr,                \
      LmArenaCtl *__restrict__ ctl, int32_t *__restrict__ err, unsigned long long *__restrict__ gscratch,          \
      int64_t gscratch_slot, long long *__restrict__ prof
#define LM_POST_PASS                                                                                                \
  Kp, slots, frame_ptr, bkg, cal, luts, hdr, keys, arena_p22d, arena_side_y, arena_side_s, arena_unary, arena_jc,    \
      arena_ir, arena_pr, ctl, err, gscratch, gscratch_slot, prof
template <bool GLOB>
DEV void post_block(int bx, int feat, LM_POST_ARGS) {
  const LmConst& K = *Kp;
  const int slot = 1 + bx;
  LmSlotOut* H = hdr + slot;
  const LmSlotOut* HP = hdr + slot - 1;
  const int frame = slots[slot].frame;
  __shared__ int s_any1, s_any0, s_base[4];
  const int Nb = H->cand_cnt[feat], Ns = H->cand_cnt[2 + feat];
  const int Ni = frame > 0 ? HP->cand_cnt[feat] : 0;
  const int Nong = K.ong_nx * K.ong_ny;
  const LmCand* cb = LM_CAND_STAGE(K, keys, slot, feat);
  const LmCand* ct = LM_CAND_STAGE(K, keys, slot, 2 + feat);
  const LmCand* cp = LM_CAND_STAGE(K, keys, slot - 1, feat);
  const bool fits = Nb <= LM_POST_MAXC && Ns <= LM_POST_MAXC && Ni <= LM_POST_MAXC && Ni + Nong + 1 <= LM_POST_MAXOFF;
  if (fits == GLOB) return;  // the other instantiation's block
  if constexpr (!GLOB) {
    __shared__ LmCand sb[LM_POST_MAXC], st[LM_POST_MAXC], sp[LM_POST_MAXC];
    __shared__ int s_off[LM_POST_MAXOFF];
    __shared__ int s_mb[LM_POST_MAXC], s_mt[LM_POST_MAXC];  // motion status (-1 unknown)
    __shared__ float s_bps[LM_POST_MAXC], s_tpb[LM_POST_MAXC];
    for (int k = threadIdx.x; k < Nb; k += blockDim.x) sb[k] = cb[k];
    for (int k = threadIdx.x; k < Ns; k += blockDim.x) st[k] = ct[k];
    for (int k = threadIdx.x; k < Ni; k += blockDim.x) sp[k] = cp[k];
    __syncthreads();
    post_run<false>(K, slots, frame_ptr, bkg, cal, luts, H, slot, feat, frame, Nb, Ns, Ni, sb, st, sp, s_off, s_mb, s_mt,
                    s_bps, s_tpb, LM_POST_MAXC, s_base, s_any1, s_any0, arena_p22d, arena_side_y, arena_side_s,
                    arena_unary, arena_jc, arena_ir, arena_pr, ctl, err, (2 * bx + feat) % ctl->nparts, prof);
  } else {  // long lists, in the block's global scratch region
    const int big = max(max(Nb, Ns), Ni);
    // the launch's block b works its pairs one after another in scratch region b
    int* g = reinterpret_cast<int*>(gscratch + (int64_t)blockIdx.x * gscratch_slot);
    int* g_off = g;                      // max(Ni + Nong, Nb) + 1
    int* g_mb = g_off + max(Ni + Nong, Nb) + 1;
    int* g_mt = g_mb + big;
    float* g_bps = reinterpret_cast<float*>(g_mt + big);
    float* g_tpb = g_bps + big;
    if ((int64_t)(reinterpret_cast<int*>(g_tpb + big) - g) > 2 * gscratch_slot) {  // the host sizes the scratch for it
      if (threadIdx.x == 0) atomicOr(err, 8);
      return;
    }
    post_run<true>(K, slots, frame_ptr, bkg, cal, luts, H, slot, feat, frame, Nb, Ns, Ni, cb, ct, cp, g_off, g_mb, g_mt,
                   g_bps, g_tpb, big, s_base, s_any1, s_any0, arena_p22d, arena_side_y, arena_side_s, arena_unary,
                   arena_jc, arena_ir, arena_pr, ctl, err, (2 * bx + feat) % ctl->nparts, prof);
  }
}

// <false>: one block per (slot, feature) whose lists fit the LDS arrays;
// <true>: the others, from global scratch, by a small grid walking all npairs
// (slot, feature) pairs (usually none).  Kept apart: one kernel holding both
// paths ran the common one 60 % slower.
template <bool GLOB>
__global__ __launch_bounds__(LM_POST_THREADS) void k_post(LM_POST_ARGS, int npairs) {
  if constexpr (!GLOB)
    post_block<false>(blockIdx.x, blockIdx.y, LM_POST_PASS);
  else
    for_overflow_pairs(
        npairs,
        [&](int p) {
          const int slot = 1 + (p >> 1), feat = p & 1;
          const LmSlotOut* H = hdr + slot;
          const int Nb = H->cand_cnt[feat], Ns = H->cand_cnt[2 + feat];
          const int Ni = slots[slot].frame > 0 ? hdr[slot - 1].cand_cnt[feat] : 0;
          return !(Nb <= LM_POST_MAXC && Ns <= LM_POST_MAXC && Ni <= LM_POST_MAXC &&
                   Ni + Kp->ong_nx * Kp->ong_ny + 1 <= LM_POST_MAXOFF);
        },
        [&](int p) { post_block<true>(p >> 1, p & 1, LM_POST_PASS); });
}

// ----------------------------------------------------------------- k_carry
// Copies the bottom candidate lists of the last slot of the previous batch
// (frame first-1) into slot 0's candidate staging, where k_post reads the
// previous frame's candidates (pairwisePotential, :896-919).  Runs first in a
// batch, before k_corr reuses the key areas of slots >= 1.
// k_carry (block 1 of k_prep's launch when the batch continues the lane's
// last one): the previous batch's last frame's bottom candidates into slot 0.
DEV void carry_block(const LmConst& K, unsigned long long* __restrict__ keys, const LmSlotOut* __restrict__ prev_hdr,
                     int prev_slot, LmSlotOut* __restrict__ hdr) {
  for (int l = 0; l < LM_NFEAT; ++l) {
    const int cnt = prev_hdr[prev_slot].cand_cnt[l];
    const LmCand* src = LM_CAND_STAGE(K, keys, prev_slot, l);
    LmCand* dst = LM_CAND_STAGE(K, keys, 0, l);
    for (int k = threadIdx.x; k < cnt; k += blockDim.x) dst[k] = src[k];
    if (threadIdx.x == 0) hdr[0].cand_cnt[l] = cnt;
  }
}

// ------------------------------------------------------------- k_prep / k_out
// The batch's only transfers between host and device memory are done by these
// two kernels through mapped pinned host memory, so a batch's stream holds
// nothing but kernels: 5 runtime copies/memsets and a second stream sync per
// batch are gone (the header and the packed results land in host memory in
// the same pass, the host reads them after one hipStreamSynchronize).
//
// k_prep: slots, frame pointers and the arena control block from host memory,
// candidate counters and error flags zeroed.  One block.
static_assert(4 * LM_TL_NC == 256, "k_prep zeroes the tile-list counters with its 256 threads");
__global__ __launch_bounds__(256) void k_prep(const LmSlot* __restrict__ h_slots, const uint8_t* const* __restrict__ h_fptr,
                                              const LmArenaCtl* __restrict__ h_ctl, int ns, LmSlot* __restrict__ slots,
                                              const uint8_t** __restrict__ fptr, LmArenaCtl* __restrict__ ctl,
                                              int32_t* __restrict__ npos, int32_t* __restrict__ err,
                                              const LmConst* __restrict__ Kp, unsigned long long* __restrict__ keys,
                                              const LmSlotOut* __restrict__ prev_hdr, int prev_slot,
                                              LmSlotOut* __restrict__ hdr, int32_t* __restrict__ dark_cnt) {
  if (blockIdx.x == 1) {
    carry_block(*Kp, keys, prev_hdr, prev_slot, hdr);
    return;
  }
  if (dark_cnt) dark_cnt[threadIdx.x] = 0;  // k_ingest's bright-tile counters (4 LM_TL_NC = blockDim.x)
  for (int i = threadIdx.x; i < ns; i += blockDim.x) {
    slots[i] = h_slots[i];
    fptr[i] = h_fptr[i];
  }
  for (int i = threadIdx.x; i < ns * LM_NLIST; i += blockDim.x) npos[i] = 0;
  if (threadIdx.x < 16) err[threadIdx.x] = 0;
  if (threadIdx.x < AR_COUNT) {
    ctl->used[threadIdx.x] = h_ctl->used[threadIdx.x];
    ctl->cap[threadIdx.x] = h_ctl->cap[threadIdx.x];
  }
  if (threadIdx.x == 0) {
    ctl->overflow = h_ctl->overflow;
    ctl->nparts = h_ctl->nparts;
    ctl->pack_dst = h_ctl->pack_dst;
    ctl->pack_cap = h_ctl->pack_cap;
  }
  for (int i = threadIdx.x; i < LM_SUBARENA * 32; i += blockDim.x) (&ctl->sub[0][0])[i] = 0;
}

// k_out: the pack header always, and when the batch succeeded and its packed
// results fit the host buffer, the results themselves -> mapped pinned host
// memory; then the next batch's previous frame (storePreviousImage,
// LocoMouse_class.cpp:1508-1513) -> the halo buffer.  Packed sizes and frame
// sizes are multiples of 16 bytes.
// h_pack == nullptr: the destination and its size are the batch's, in ctl
// (k_prep copied them from the lane's mapped control block).
__global__ __launch_bounds__(256) void k_out(const LmPackHdr* __restrict__ ph, LmPackHdr* __restrict__ h_ph,
                                             const uint8_t* __restrict__ pack, uint8_t* __restrict__ h_pack, int64_t h_cap,
                                             const LmArenaCtl* __restrict__ ctl,
                                             const uint8_t* __restrict__ halo_arg, const uint8_t* const* __restrict__ fptr,
                                             int fidx, uint8_t* __restrict__ halo_dst, int64_t halo_bytes) {
  if (!h_pack && ctl) {
    h_pack = ctl->pack_dst;
    h_cap = ctl->pack_cap;
  }
  // halo source: halo_arg, else the batch's frame pointer fptr[fidx] (device
  // array written by k_prep, so a captured graph replays with fresh frames)
  const uint8_t* __restrict__ halo_src = halo_arg ? halo_arg : (fptr ? fptr[fidx] : nullptr);
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, nth = (int64_t)gridDim.x * blockDim.x;
  if (tid == 0) *h_ph = *ph;
  const int64_t bytes = ph->bytes;
  if (ph->overflow || ph->err || bytes > h_cap) return;
  for (int64_t i = tid; i < bytes / 16; i += nth)
    reinterpret_cast<uint4*>(h_pack)[i] = reinterpret_cast<const uint4*>(pack)[i];
  if (halo_src) {
    for (int64_t i = tid; i < halo_bytes / 16; i += nth)
      reinterpret_cast<uint4*>(halo_dst)[i] = reinterpret_cast<const uint4*>(halo_src)[i];
    for (int64_t i = halo_bytes / 16 * 16 + tid; i < halo_bytes; i += nth) halo_dst[i] = halo_src[i];
  }
}

// ------------------------------------------------------------------ k_pack
// Packs the batch's results into lm_batch_result's layout (frame order) in one
// buffer: k_pack_scan computes every offset array (exclusive scans over the
// frames) and the totals, k_pack_copy moves each (frame, feature)'s data.
// Unit = one batch; a few KB per frame, launch-latency bound.
// All six offset arrays in one pass: each thread takes a contiguous run of
// frames, sums its frames' counts per array, one block-wide exclusive scan of
// the six sums (one pair of barriers instead of six), then the thread writes
// its frames' per-list offsets.  (Six scans one after the other cost six
// dependent load + barrier rounds: ~19 us per batch, launch-latency bound.)
__global__ __launch_bounds__(1024) void k_pack_scan(const LmSlotOut* __restrict__ hdr, int n,
                                                    const LmArenaCtl* __restrict__ ctl, const int32_t* __restrict__ err,
                                                    LmPackHdr* __restrict__ ph, uint8_t* __restrict__ pack, int64_t pack_cap,
                                                    int64_t* __restrict__ side_base) {
  constexpr int NA = 6;  // cand, p22d, unary, jc, nz, side
  __shared__ int64_t s_w[1024 / 64 + 1][NA];
  const int64_t zero[PK_COUNT] = {0, 0, 0, 0, 0, 0};
  const LmPackLayout L0 = lm_pack_layout(n, zero);  // offset arrays do not depend on the totals
  const LmSlotOut* H = hdr + 1;
  int64_t* outs[NA] = {reinterpret_cast<int64_t*>(pack + L0.cand_off), reinterpret_cast<int64_t*>(pack + L0.p22d_off),
                       reinterpret_cast<int64_t*>(pack + L0.unary_off), reinterpret_cast<int64_t*>(pack + L0.jc_off),
                       reinterpret_cast<int64_t*>(pack + L0.nz_off), side_base};
  const int per[NA] = {4, 2, 2, 2, 2, 2};  // entries per frame
  // count of array a, entry j of frame f
  auto count = [&](const LmSlotOut& h, int a, int j) -> int64_t {
    switch (a) {
      case 0: return h.cand_cnt[j];
      case 1: return h.p22d_cnt[j];
      case 2: return h.unary_cnt[j];
      case 3: return h.pw_rows[j] >= 0 ? (int64_t)h.pw_cols[j] + 1 : 0;
      case 4: return h.pw_rows[j] >= 0 ? (int64_t)h.pw_nnz[j] : 0;
      default: return h.side_cnt[j];
    }
  };
  const int T = blockDim.x, chunk = (n + T - 1) / T;
  const int f0 = threadIdx.x * chunk, f1 = min(n, f0 + chunk);
  int64_t c[NA] = {0, 0, 0, 0, 0, 0};
  for (int f = f0; f < f1; ++f) {
    const LmSlotOut& h = H[f];
#pragma unroll
    for (int a = 0; a < NA; ++a)
      for (int j = 0; j < per[a]; ++j) c[a] += count(h, a, j);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t v[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    v[a] = c[a];
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = __shfl_up(v[a], o);
      if (lane >= o) v[a] += u;
    }
  }
  if (lane == 63)
#pragma unroll
    for (int a = 0; a < NA; ++a) s_w[wid][a] = v[a];
  __syncthreads();
  if (threadIdx.x < NA) {
    const int a = threadIdx.x;
    int64_t acc = 0;
    for (int w = 0; w < (T >> 6); ++w) {
      const int64_t t = s_w[w][a];
      s_w[w][a] = acc;
      acc += t;
    }
    s_w[T >> 6][a] = acc;
  }
  __syncthreads();
  int64_t r[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) r[a] = s_w[wid][a] + v[a] - c[a];
  for (int f = f0; f < f1; ++f) {
    const LmSlotOut& h = H[f];
#pragma unroll
    for (int a = 0; a < NA; ++a)
      for (int j = 0; j < per[a]; ++j) {
        outs[a][per[a] * f + j] = r[a];
        r[a] += count(h, a, j);
      }
  }
  if (threadIdx.x < NA) outs[threadIdx.x][per[threadIdx.x] * n] = s_w[T >> 6][threadIdx.x];
  // the sub-arena counts, one load per thread (a serial loop over them by one
  // thread waited out 6 x 16 dependent L2 round trips)
  __shared__ int s_sub[AR_COUNT][LM_SUBARENA];
  const int nparts = ctl->nparts;
  if (threadIdx.x < AR_COUNT * LM_SUBARENA) {
    const int k = threadIdx.x / LM_SUBARENA, g = threadIdx.x % LM_SUBARENA;
    s_sub[k][g] = g < nparts ? ctl->sub[g][k] : 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t tot[PK_COUNT];
    tot[PK_CAND] = s_w[T >> 6][0];
    tot[PK_P22D] = s_w[T >> 6][1];
    tot[PK_UNARY] = s_w[T >> 6][2];
    tot[PK_JC] = s_w[T >> 6][3];
    tot[PK_NZ] = s_w[T >> 6][4];
    tot[PK_SIDE] = s_w[T >> 6][5];
    const LmPackLayout L = lm_pack_layout(n, tot);
    for (int k = 0; k < PK_COUNT; ++k) ph->tot[k] = tot[k];
    ph->bytes = L.bytes;
    ph->overflow = (L.bytes > pack_cap ? 1 : 0) | (ctl->overflow ? 2 : 0);
    ph->err = *err;
    for (int k = 0; k < AR_COUNT; ++k) {
      int m = 0;
      for (int g = 0; g < LM_SUBARENA; ++g) m = max(m, s_sub[k][g]);
      ph->used[k] = m * nparts;
    }
  }
}

__global__ __launch_bounds__(256) void k_pack_copy(const LmConst* __restrict__ Kp, const LmSlotOut* __restrict__ hdr, int n,
                                                   const unsigned long long* __restrict__ keys,
                                                   const LmP22D* __restrict__ arena_p22d, const int32_t* __restrict__ arena_side_y,
                                                   const double* __restrict__ arena_side_s, const double* __restrict__ arena_unary,
                                                   const int32_t* __restrict__ arena_jc, const int32_t* __restrict__ arena_ir,
                                                   const double* __restrict__ arena_pr, const LmPackHdr* __restrict__ ph,
                                                   uint8_t* __restrict__ pack, const int64_t* __restrict__ side_base) {
  const LmConst& K = *Kp;
  if (ph->overflow || ph->err) return;  // the host raises or reruns; offsets may be garbage
  const int f = blockIdx.x, feat = blockIdx.y, slot = 1 + f;
  const LmSlotOut& H = hdr[slot];
  int64_t tot[PK_COUNT];
  for (int k = 0; k < PK_COUNT; ++k) tot[k] = ph->tot[k];
  const LmPackLayout L = lm_pack_layout(n, tot);
  const int64_t* cand_off = reinterpret_cast<const int64_t*>(pack + L.cand_off);
  const int64_t* p22d_off = reinterpret_cast<const int64_t*>(pack + L.p22d_off);
  const int64_t* unary_off = reinterpret_cast<const int64_t*>(pack + L.unary_off);
  const int64_t* jc_off = reinterpret_cast<const int64_t*>(pack + L.jc_off);
  const int64_t* nz_off = reinterpret_cast<const int64_t*>(pack + L.nz_off);
  LmCand* cand = reinterpret_cast<LmCand*>(pack + L.cand);
  for (int l = feat; l < LM_NLIST; l += 2) {
    const LmCand* src = LM_CAND_STAGE(K, keys, slot, l);
    LmCand* dst = cand + cand_off[4 * f + l];
    for (int k = threadIdx.x; k < H.cand_cnt[l]; k += blockDim.x) dst[k] = src[k];
  }
  const int q = 2 * f + feat;
  const int64_t sb = side_base[q];
  LmP22D* p22d = reinterpret_cast<LmP22D*>(pack + L.p22d) + p22d_off[q];
  for (int k = threadIdx.x; k < H.p22d_cnt[feat]; k += blockDim.x) {
    LmP22D v = arena_p22d[H.p22d_off[feat] + k];
    v.side_off = (int32_t)(sb + (v.side_off - H.side_off[feat]));
    p22d[k] = v;
  }
  int32_t* side_y = reinterpret_cast<int32_t*>(pack + L.side_y) + sb;
  double* side_s = reinterpret_cast<double*>(pack + L.side_s) + sb;
  for (int k = threadIdx.x; k < H.side_cnt[feat]; k += blockDim.x) {
    side_y[k] = arena_side_y[H.side_off[feat] + k];
    side_s[k] = arena_side_s[H.side_off[feat] + k];
  }
  double* unary = reinterpret_cast<double*>(pack + L.unary) + unary_off[q];
  for (int k = threadIdx.x; k < H.unary_cnt[feat]; k += blockDim.x) unary[k] = arena_unary[H.unary_off[feat] + k];
  int32_t* dims = reinterpret_cast<int32_t*>(pack + L.pw_dims) + 3 * q;
  if (H.pw_rows[feat] >= 0) {
    int32_t* jc = reinterpret_cast<int32_t*>(pack + L.jc) + jc_off[q];
    int32_t* ir = reinterpret_cast<int32_t*>(pack + L.ir) + nz_off[q];
    double* pr = reinterpret_cast<double*>(pack + L.pr) + nz_off[q];
    for (int k = threadIdx.x; k <= H.pw_cols[feat]; k += blockDim.x) jc[k] = arena_jc[H.pw_jc_off[feat] + k];
    for (int k = threadIdx.x; k < H.pw_nnz[feat]; k += blockDim.x) {
      ir[k] = arena_ir[H.pw_nz_off[feat] + k];
      pr[k] = arena_pr[H.pw_nz_off[feat] + k];
    }
    if (threadIdx.x == 0) {
      dims[0] = H.pw_rows[feat];
      dims[1] = H.pw_cols[feat];
      dims[2] = H.pw_nnz[feat];
    }
  } else if (threadIdx.x == 0) {
    dims[0] = -1;
    dims[1] = -1;
    dims[2] = 0;
  }
  if (feat == 0) {
    int32_t* tail = reinterpret_cast<int32_t*>(pack + L.tail) + 45 * f;
    for (int k = threadIdx.x; k < 45; k += blockDim.x) tail[k] = H.tail[k];
  }
}

