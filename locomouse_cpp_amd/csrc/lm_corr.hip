// lm_corr.hip — the six filter2D detectors (its own translation unit; the
// runtime reaches it through the dispatch functions declared in lm_corr.h).
//
// cv::filter2D(I_VIEW_PAD, scores, CV_32F, W, Point(-1,-1), -rho, BORDER_CONSTANT)
// at LocoMouse_class.cpp:845, :860, :2575, :2576, restated as
//     acc = (float)(-rho);  for i in rows, j in cols: acc = acc (+) W[i][j] * I(y+i-kh/2, x+j-kw/2)
// with (+)* either one fused multiply-add per tap (OpenCV's AVX2 build,
// v_muladd -> vfmadd; the default) or a rounded multiply then a rounded add
// (OpenCV's scalar/SSE2 build; LM_FILTER_UNFUSED).  Taps are visited in
// row-major order, zero-padded taps add +0 (OpenCV skips zero taps; the sum is
// the same), so every score is bit-identical to the oracle's chain.
//
// Kernels:
//   k_corr_rw<KW, UNF>  width-specialised packed-FP32 kernel (every detector
//                       width of LM_KW_LIST, any height): one wave per 80 x 16
//                       output tile streaming its window through a private
//                       LDS ring; the production path.
//   k_corr_gen<UNF>     any width and height: taps in chunks of 4 columns and
//                       the tap rows in LDS-sized chunks (detectors larger than
//                       the LDS window, widths without an instantiation).
//   k_corr_f16<NCH>     NON-PARITY half-precision mode (LM_CORR_F16): f16
//                       weights, fp32 accumulation on the matrix cores.
//   k_corr_dbg<UNF>     raw scores straight from the ext crops in global memory
//                       (diagnostics: lm_debug_scores).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <type_traits>
#include <vector>

#include "lm_corr.h"

#define DEV __device__ __forceinline__

typedef float lm_f2 __attribute__((ext_vector_type(2)));

// One tap on a packed pair of accumulators (two vertically adjacent outputs of
// one column; both use the same weight).
template <bool UNF>
DEV lm_f2 corr_tap(lm_f2 acc, lm_f2 w2, lm_f2 p) {
  if constexpr (UNF) {
    const lm_f2 prod = w2 * p;  // v_pk_mul_f32 (-ffp-contract=off keeps mul and add apart)
    return acc + prod;          // v_pk_add_f32
  } else {
    return __builtin_elementwise_fma(w2, p, acc);  // v_pk_fma_f32
  }
}

template <bool UNF>
DEV float corr_tap1(float acc, float w, float p) {
  if constexpr (UNF) {
    const float prod = w * p;
    return acc + prod;
  } else {
    return __builtin_fmaf(w, p, acc);
  }
}

// Shared epilogue: point detectors apply the brightness mask of
// detectBottom/SideCandidates (threshold(25.5 -> 25, BINARY_INV), :782/:817;
// setTo(0, mask) :849/:864) and append every score > 0 as a sort key
// (~score_bits << 32 | row-major index) to the frame's list; tail detectors
// write the binarised map (threshold(>0) + convertTo 8U, :2593-2598).
// Two passes over a register bitmask keep the accumulators statically indexed.
template <int R_, int C_>
DEV void corr_epilogue(const LmConst& K, const LmDet& D, const float (&acc)[R_][C_], const float* lds, int stride, int ly,
                       int lx, int oy0, int ox0, int slot, unsigned long long* __restrict__ keys,
                       int32_t* __restrict__ n_pos, uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes, int* s_cnt,
                       int* s_base, const uint8_t* __restrict__ msrc, int mpitch, float* __restrict__ tile) {
  static_assert(R_ * C_ <= 32, "bitmask");
  if (D.kind != 0) {
    // the tile's bits gathered in LDS (rows of the <= 4 u32 words its LM_TW
    // columns touch; in the dead window once every wave is past its taps),
    // then ORed into the slot's zeroed bitmap; neighbouring tiles share the
    // boundary words
    unsigned* s_tb = reinterpret_cast<unsigned*>(tile);
    const int w0 = ox0 >> 5;
    __syncthreads();
    for (int i = threadIdx.x; i < LM_TH * 4; i += blockDim.x) s_tb[i] = 0u;
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R_; ++r)
#pragma unroll
      for (int c = 0; c < C_; ++c) {
        const int y = oy0 + ly * R_ + r, x = ox0 + lx * C_ + c;
        if (y < D.oh && x < D.ow && acc[r][c] > 0.0f) atomicOr(&s_tb[(ly * R_ + r) * 4 + (x >> 5) - w0], 1u << (x & 31));
      }
    __syncthreads();
    unsigned* __restrict__ tb = reinterpret_cast<unsigned*>(tailbin + (int64_t)slot * tailbin_slot_bytes) +
                                (D.list ? (int64_t)K.tail_hb * K.tail_nw : 0);
    for (int i = threadIdx.x; i < LM_TH * 4; i += blockDim.x) {
      const unsigned v = s_tb[i];
      const int y = oy0 + (i >> 2), gw = w0 + (i & 3);
      if (v && y < D.oh && gw < K.tail_nw) atomicOr(&tb[(int64_t)y * K.tail_nw + gw], v);
    }
    return;
  }
  unsigned bits = 0;
#pragma unroll
  for (int r = 0; r < R_; ++r)
#pragma unroll
    for (int c = 0; c < C_; ++c) {
      const int y = oy0 + ly * R_ + r, x = ox0 + lx * C_ + c;
      // the I_*_MOUSE pixel of this output: from the LDS tile when it holds it,
      // else (row-chunked generic kernel) from the ext crop
      const int pix = lds ? (int)lds[(ly * R_ + r + D.m_y - D.in_y) * stride + lx * C_ + c + D.m_x - D.in_x]
                          : (int)msrc[(int64_t)(ly * R_ + r) * mpitch + lx * C_ + c];
      if (y < D.oh && x < D.ow && pix > 25 && acc[r][c] > 0.0f) bits |= 1u << (r * C_ + c);
    }
  const int nk = __popc(bits);
  const int off = nk ? atomicAdd(s_cnt, nk) : 0;
  __syncthreads();
  if (threadIdx.x == 0) *s_base = *s_cnt ? atomicAdd(&n_pos[slot * LM_NLIST + D.list], *s_cnt) : 0;
  __syncthreads();
  unsigned long long* __restrict__ kl = keys + (int64_t)slot * K.keys_per_slot + K.list_off[D.list] + *s_base + off;
  int k = 0;
#pragma unroll
  for (int r = 0; r < R_; ++r)
#pragma unroll
    for (int c = 0; c < C_; ++c)
      if (bits & (1u << (r * C_ + c))) {
        const int y = oy0 + ly * R_ + r, x = ox0 + lx * C_ + c;
        kl[k++] = ((unsigned long long)(~__float_as_uint(acc[r][c])) << 32) | (unsigned)(y * D.ow + x);
      }
}

// Tile fill: u8 ext-crop window (rows x cols from src, row pitch ew) -> fp32
// LDS (row stride `stride`).  16-byte aligned vector loads, all of a round
// issued before any is consumed (a workgroup's fill is one or two load
// latencies, not one per 4 bytes), then unpacked with v_cvt_f32_ubyte*.
// ew and the ext-crop base are multiples of 16; src itself need not be.
// Reads up to 15 bytes past a row's last column (inside the padded row or the
// next; the ext buffer has slack after its last slot).
DEV void tile_fill_f32(float* __restrict__ lds, int stride, const uint8_t* __restrict__ src, int ew, int rows,
                       int cols) {
  const int mis = (int)((uintptr_t)src & 15);
  const uint8_t* __restrict__ a = src - mis;
  const int nch = (mis + cols + 15) >> 4;
  const int total = rows * nch;
  for (int e0 = 0; e0 < total; e0 += 4 * (int)blockDim.x) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * (int)blockDim.x + (int)threadIdx.x;
      if (e < total) {
        const int r = e / nch, ch = e - r * nch;
        v[u] = *reinterpret_cast<const uint4*>(a + (int64_t)r * ew + ch * 16);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * (int)blockDim.x + (int)threadIdx.x;
      if (e < total) {
        const int r = e / nch, ch = e - r * nch;
        const int c0 = ch * 16 - mis;
        float* __restrict__ o = lds + r * stride + c0;
        const unsigned w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        if (c0 >= 0 && c0 + 16 <= cols) {  // whole chunk inside the window: straight-line stores
#pragma unroll
          for (int k = 0; k < 16; ++k) o[k] = (float)((w[k >> 2] >> (8 * (k & 3))) & 0xFFu);
        } else {
#pragma unroll
          for (int k = 0; k < 16; ++k)
            if (c0 + k >= 0 && c0 + k < cols) o[k] = (float)((w[k >> 2] >> (8 * (k & 3))) & 0xFFu);
        }
      }
    }
  }
}

// Which detector of the group a block works on, and its tile origin.
struct CorrTile {
  int d, oy0, ox0;
};
DEV CorrTile corr_tile(const LmConst& K, const LmDetGroup& G) {
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const int lt = blockIdx.x - tb;
  const int tx = K.det[d].tiles_x;
  return CorrTile{d, (lt / tx) * K.det[d].tile_h, (lt % tx) * K.det[d].tile_w};
}

DEV const uint8_t* corr_src(const LmConst& K, const LmDet& D, const uint8_t* ext, int64_t ext_slot_bytes, int slot,
                            int oy0, int ox0) {
  return ext + (int64_t)slot * ext_slot_bytes + (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
         (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
}

// ---------------------------------------------------------------- k_corr_rw
// Packed-FP32 correlation.  gfx950 issues one v_fma_f32 (wave64) per 4 cycles
// per SIMD; v_pk_fma_f32 does two FMAs per lane in the same slot.  Each
// accumulator pair holds two vertically adjacent outputs (rows 2p, 2p+1) of
// one column: for tap (i, j) both use weight w[i][j] (SGPR, broadcast) and
// pixels (t, t+1) of one column, which one ds_read2_b32 loads into an aligned
// register pair.  A thread owns 5 columns x 4 rows (two row pairs sharing the
// pixel rows of a step with weight rows t and t - 2).  A wave is LM_RW_NQ
// independent sub-tiles of LM_FW x 8 outputs (round 4: four 40 x 8 quarters
// of 16 lanes, 8 x 2 threads; round 3: two 80 x 8 halves of 32 lanes), so
// the dark-tile skip works at LM_FW x 8 granularity (60-62 % of the
// synthetic point outputs in bright 40 x 8 tiles vs 72-73 % at 80 x 8), each
// streaming its own window through a private LDS ring of LM_RW_HSLOTS rows +
// 1 mirror row: at step t its 2 row groups read window rows t + 4 ly,
// t + 4 ly + 1 (rows t .. t + 5), the ring also holds the rows loaded ahead,
// and the mirror slot keeps a pair from wrapping.  Any kh fits, no wave waits
// for another and a wave's LDS operations execute in order, so the rings need
// no barrier.

// A ring wave's work (see rw_tile): LM_RW_NQ sub-tiles of LM_FW x LM_FH
// outputs -- LM_RW_NQ bright tiles from a segment of a dark-tile list (the
// entries at l), or the 8 parts of one 80 x 16 tile.
struct RwRun {
  const uint32_t* l;  // listed: the wave's first entry; nullptr: one 80 x 16 tile
  int nvalid;         // sub-tiles 0 .. nvalid - 1 hold a tile
  int ftx;            // listed: flag-grid columns of the view
  int slot, oy, ox;   // one tile: its slot and origin
  // list entry of sub-tile i (a valid one for i past the last)
  DEV uint32_t entry(int i) const { return l ? l[min(i, nvalid - 1)] : 0u; }
  // slot and output origin of sub-tile i (e: its entry)
  DEV void tile(int i, uint32_t e, int& s, int& y, int& x) const {
    if (l) {
      const int lt = (int)(e & 0xFFFFu);
      s = (int)(e >> 16);
      y = (lt / ftx) * LM_FH;
      x = (lt % ftx) * LM_FW;
    } else {
      s = slot;
      y = oy + (i / LM_RW_NQX) * LM_FH;
      x = ox + (i % LM_RW_NQX) * LM_FW;
    }
  }
};

// Wave g of a ring launch -> its detector and sub-tiles.  The batch's work
// is flattened detector-major (all slots of the group's first detector, then
// the next ...; the host puts the longest detectors first), so no wave idles
// at a frame's end.  With dark-tile lists (tl_cnt != nullptr) a point
// detector's waves take its view's bright LM_FW x LM_FH tiles LM_RW_NQ at a
// time from the list segments k_ingest filled (segment c: tl_cnt[view
// LM_TL_NC + c] tiles, ceil(/ LM_RW_NQ) waves), packed densely: a wave finds
// its segment with one scan over the 64 counters, one per lane.  The group's
// wave count is known on the device only, so the grid is sized for every
// 80 x 16 tile and the waves past the last group's count (whole workgroups
// at the grid's end) return.  Otherwise a wave takes the sub-tiles of one
// 80 x 16 tile (row-major per slot).  Called by every lane of the wave;
// false: past the last wave.
//
// Round 6 tried an arithmetic map instead (workgroup b -> the room of its
// slot group's segment, the counter and the entries read together: one
// dependent global read less per wave): 2-3 % fewer frames/s at 8 contexts
// (profiles/r06/corr_ab/).  The room-based layout puts a segment's working
// waves in whole workgroups, so every segment's last workgroup idles up to
// three wave slots while its LDS is held, and the empty workgroups sit
// between the working ones; the dense layout has neither.
static_assert(LM_TL_NC == 64, "one list counter per lane");
DEV bool corr_locate_rw(const LmConst& K, const LmDetGroup& G, int nslots, int s0, int g, const int32_t* tl_cnt,
                        const uint32_t* tl_list, int& d, RwRun& R) {
  constexpr int NQ = LM_RW_NQ;
  const int lane = threadIdx.x & 63;
  int base = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET; ++k) {
    if (k >= G.n) return false;
    const int dk = G.ids[k];
    const LmDet& D = K.det[dk];
    const int nt = G.tile_end[k] - (k ? G.tile_end[k - 1] : 0);
    if (tl_cnt != nullptr && D.kind == 0) {
      const int v = D.view;
      const int cn = tl_cnt[v * LM_TL_NC + lane];  // segment `lane`'s bright tiles
      const int wv = (cn + NQ - 1) / NQ;
      int P = wv;  // inclusive scan: waves of segments 0 .. lane
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(P, o);
        if (lane >= o) P += u;
      }
      const int cnt = __builtin_amdgcn_readlane(P, 63);  // (readlane: wave-uniform values stay scalar)
      if (g < base + cnt) {
        const int local = g - base;
        const int c = __builtin_amdgcn_readfirstlane(__ffsll((long long)__ballot(P > local)) - 1);
        const int w = local - (__builtin_amdgcn_readlane(P, c) - __builtin_amdgcn_readlane(wv, c));  // place in segment c
        const int ng = (nslots + LM_INGEST_FB - 1) / LM_INGEST_FB;
        d = dk;
        R = RwRun{tl_list + (int64_t)v * K.tl_stride + (int64_t)lm_tl_y0(c, ng) * LM_INGEST_FB * K.fl_tx[v] * K.fl_ty[v] +
                      NQ * w,
                  min(NQ, __builtin_amdgcn_readlane(cn, c) - NQ * w), K.fl_tx[v], 0, 0, 0};
        return true;
      }
      base += cnt;
    } else {
      const int cnt = nt * nslots;
      if (g < base + cnt) {
        const int local = g - base;
        const int tx = D.tiles_x;
        const int lt = local - (local / nt) * nt;
        d = dk;
        R = RwRun{nullptr, NQ, 0, s0 + local / nt, (lt / tx) * LM_RW_TH, (lt % tx) * LM_TW};
        return true;
      }
      base += cnt;
    }
  }
  return false;
}

// A workgroup tile of a point detector (k_corr_gen, k_corr_f16) whose flag
// tiles are all dark has no output that survives the mask.
DEV bool corr_tile_dark(const LmConst& K, const LmDet& D, const uint8_t* __restrict__ dark, int slot, int oy0, int ox0) {
  if (dark == nullptr || D.kind != 0) return false;
  const int v = D.view;
  const int ty0 = oy0 / LM_FH, ty1 = min(K.fl_ty[v] - 1, (oy0 + D.tile_h - 1) / LM_FH);
  const int tx0 = ox0 / LM_FW, tx1 = min(K.fl_tx[v] - 1, (ox0 + D.tile_w - 1) / LM_FW);
  const uint8_t* __restrict__ f = dark + (int64_t)slot * K.fl_slot + K.fl_off[v];
  for (int ty = ty0; ty <= ty1; ++ty)
    for (int tx = tx0; tx <= tx1; ++tx)
      if (f[ty * K.fl_tx[v] + tx]) return false;
  return true;
}

// Software pipeline of k_corr_rw's step: a detector row's taps in
// chunks (the first of 8 taps, the others of <= 12, every chunk starting on
// an even tap); while a chunk's FMAs run, the pixel pairs and weights of the
// next chunk (the next step's first chunk after the last) are already in
// flight, so a wave waits on LDS / scalar loads only when they are late, and
// at most 12 + 4 pairs are live.  Weights are read as 64-bit pairs (taps 2q,
// 2q + 1 of a row; rows are zero-padded to a multiple of 4) into aligned SGPR
// pairs, and each tap's v_pk_fma_f32 broadcasts its half of the pair with
// op_sel: with single-float weights the compiler copied every
// odd SGPR into an even one, and the copies of the next step's first chunk
// forced an lgkmcnt(0) wait right after that chunk's loads were issued.
#ifndef LM_RW_PMAX
#define LM_RW_PMAX 4
#endif
template <int KW>
struct RwPlan {
  static_assert(KW >= 10, "k_corr_rw pipeline: at least 10 taps per row");
  static constexpr int NP = (KW + 1) / 2;  // weight pairs per row (the last one half used when KW is odd)
  static constexpr int P0 = 4;             // pairs of the first chunk
  static constexpr int RP = NP - P0;
  static constexpr int PMAX = LM_RW_PMAX;  // weight pairs per chunk
  static constexpr int NR0 = (RP + PMAX - 1) / PMAX;
  static constexpr int NR = NR0 < 2 ? 2 : NR0;  // >= 3 chunks: the first chunk's pairs are dead by the last
  static constexpr int N = 1 + NR;
  static constexpr int qb(int c) { return c == 0 ? 0 : P0 + ((c - 1) * RP) / NR; }
  static constexpr int qe(int c) { return c == N - 1 ? NP : qb(c + 1); }
  static constexpr int beg(int c) { return 2 * qb(c); }
  static constexpr int end(int c) { return c == N - 1 ? KW : 2 * qe(c); }
  // pixel pairs a chunk needs that the previous chunk of its step did not load
  static constexpr int pbeg(int c) { return c == 0 ? 0 : beg(c) + PK_C - 1; }
  static constexpr int pend(int c) { return end(c) + PK_C - 1; }
};

template <int STRIDE, int Q>
DEV void lds_pair_nw(lm_f2& dst, unsigned base) {
  static_assert(Q + STRIDE <= 255, "ds_read2_b32 offset range");
  asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(dst) : "v"(base), "i"(Q), "i"(Q + STRIDE) : "memory");
}

// One tap on a packed pair of accumulators with weight half H of the SGPR
// pair w2.  Volatile, like the ds_read2_b32 that produce p: the taps stay
// behind the chunk's s_waitcnt.
template <bool UNF, int H>
DEV lm_f2 corr_tap_h(lm_f2 acc, lm_f2 w2, lm_f2 p) {
  if constexpr (UNF) {  // rounded product, then rounded sum (OpenCV's scalar / SSE2 build)
    lm_f2 prod;
    if constexpr (H == 0)
      asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(prod) : "s"(w2), "v"(p));
    else
      asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(prod) : "s"(w2), "v"(p));
    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc) : "v"(prod));
    return acc;
  } else if constexpr (H == 0) {
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc) : "s"(w2), "v"(p));
    return acc;
  } else {
    asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "s"(w2), "v"(p));
    return acc;
  }
}

// Both taps (halves 0 and 1) of one weight pair in ONE inline-asm block, for
// pair 0 (acc a, weights wa) and/or pair 1 (acc b, weights wb); px: the six
// pixel pairs p .. p + 5 the two taps read.  The compiler cannot see inside
// an asm statement, so it separates any two that touch the same registers by
// an s_nop (the wait states an MFMA result would need): one statement per
// tap put 30 s_nops into a kw-30 step, one per pair halves that.  Per
// accumulator the taps keep their order (half 0, then half 1).
#define LM_RWF(a, w, p, sel) "v_pk_fma_f32 %" #a ", %" #w ", %" #p ", %" #a " " sel "\n"
#define LM_RW_S0 "op_sel_hi:[0,1,1]"
#define LM_RW_S1 "op_sel:[1,0,0] op_sel_hi:[1,1,1]"
DEV void rw_pair_ab(lm_f2 (&a)[PK_C], lm_f2 (&b)[PK_C], lm_f2 wa, lm_f2 wb, const lm_f2* px) {
  static_assert(PK_C == 5, "the asm block is written for 5 columns");
  asm volatile(LM_RWF(0, 10, 12, LM_RW_S0) LM_RWF(1, 10, 13, LM_RW_S0) LM_RWF(2, 10, 14, LM_RW_S0)
                   LM_RWF(3, 10, 15, LM_RW_S0) LM_RWF(4, 10, 16, LM_RW_S0)
               LM_RWF(5, 11, 12, LM_RW_S0) LM_RWF(6, 11, 13, LM_RW_S0) LM_RWF(7, 11, 14, LM_RW_S0)
                   LM_RWF(8, 11, 15, LM_RW_S0) LM_RWF(9, 11, 16, LM_RW_S0)
               LM_RWF(0, 10, 13, LM_RW_S1) LM_RWF(1, 10, 14, LM_RW_S1) LM_RWF(2, 10, 15, LM_RW_S1)
                   LM_RWF(3, 10, 16, LM_RW_S1) LM_RWF(4, 10, 17, LM_RW_S1)
               LM_RWF(5, 11, 13, LM_RW_S1) LM_RWF(6, 11, 14, LM_RW_S1) LM_RWF(7, 11, 15, LM_RW_S1)
                   LM_RWF(8, 11, 16, LM_RW_S1) LM_RWF(9, 11, 17, LM_RW_S1)
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(b[0]), "+v"(b[1]), "+v"(b[2]),
                 "+v"(b[3]), "+v"(b[4])
               : "s"(wa), "s"(wb), "v"(px[0]), "v"(px[1]), "v"(px[2]), "v"(px[3]), "v"(px[4]), "v"(px[5]));
}
DEV void rw_pair_1(lm_f2 (&a)[PK_C], lm_f2 w, const lm_f2* px) {
  asm volatile(LM_RWF(0, 5, 6, LM_RW_S0) LM_RWF(1, 5, 7, LM_RW_S0) LM_RWF(2, 5, 8, LM_RW_S0)
                   LM_RWF(3, 5, 9, LM_RW_S0) LM_RWF(4, 5, 10, LM_RW_S0)
               LM_RWF(0, 5, 7, LM_RW_S1) LM_RWF(1, 5, 8, LM_RW_S1) LM_RWF(2, 5, 9, LM_RW_S1)
                   LM_RWF(3, 5, 10, LM_RW_S1) LM_RWF(4, 5, 11, LM_RW_S1)
               : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4])
               : "s"(w), "v"(px[0]), "v"(px[1]), "v"(px[2]), "v"(px[3]), "v"(px[4]), "v"(px[5]));
}
#undef LM_RWF
#undef LM_RW_S0
#undef LM_RW_S1

template <int KW, bool UNF>
struct RwPipe {
  using P = RwPlan<KW>;
  static constexpr int STR = rw_stride(KW);
  lm_f2 px[PK_C + KW - 1];
  lm_f2 acc[2][PK_C];
  lm_f2 wa[P::PMAX], wb[P::PMAX];  // weight pairs of the chunk being computed (rows t, t - 2)
  template <int Q0, int Q1>
  DEV void issue(unsigned base) {
    if constexpr (Q0 < Q1) {
      lds_pair_nw<STR, Q0>(px[Q0], base);
      issue<Q0 + 1, Q1>(base);
    }
  }
  // chunk C's weight pairs of rows ra (pair 0) and rb (pair 1) into na / nb
  template <int C>
  DEV void load_w(lm_f2 (&na)[P::PMAX], lm_f2 (&nb)[P::PMAX], const lm_f2* __restrict__ ra,
                  const lm_f2* __restrict__ rb) {
#pragma unroll
    for (int q = 0; q < P::qe(C) - P::qb(C); ++q) {
      na[q] = ra[P::qb(C) + q];
      nb[q] = rb[P::qb(C) + q];
    }
  }
  template <int J, int C, bool A, bool B>
  DEV void compute_from() {
    if constexpr (J < P::end(C) && !UNF && (J & 1) == 0 && J + 1 < P::end(C) &&
                  (A || B)) {
      constexpr int q = J / 2 - P::qb(C);
      if constexpr (A && B) rw_pair_ab(acc[0], acc[1], wa[q], wb[q], &px[J]);
      else if constexpr (A) rw_pair_1(acc[0], wa[q], &px[J]);
      else rw_pair_1(acc[1], wb[q], &px[J]);
      compute_from<J + 2, C, A, B>();
    } else if constexpr (J < P::end(C)) {
      constexpr int q = J / 2 - P::qb(C), h = J & 1;
      if constexpr (A) {
#pragma unroll
        for (int c = 0; c < PK_C; ++c) acc[0][c] = corr_tap_h<UNF, h>(acc[0][c], wa[q], px[c + J]);
      }
      if constexpr (B) {
#pragma unroll
        for (int c = 0; c < PK_C; ++c) acc[1][c] = corr_tap_h<UNF, h>(acc[1][c], wb[q], px[c + J]);
      }
      compute_from<J + 1, C, A, B>();
    }
  }
  // step t, chunk C onwards.  On entry chunk C's pairs and weights are in
  // flight; on exit the next step's first chunk is.  `base_n` addresses the
  // next step's pixel rows, rows_n its weight rows.
  // NEXT = false (a wave's last step): nothing is prefetched for a step that
  // does not come -- an LDS read whose result nobody uses leaves its
  // destination registers free to the compiler, which may write them before
  // the read returns and is overwritten by it.
  template <int C, bool A, bool B, bool NEXT = true, typename F>
  DEV void chunks(unsigned base, unsigned base_n, const lm_f2* __restrict__ ra, const lm_f2* __restrict__ rb,
                  const lm_f2* __restrict__ ra_n, const lm_f2* __restrict__ rb_n, F&& at_start) {
    // lgkmcnt(0) through the builtin (vmcnt / expcnt left at their maxima), so
    // the compiler's own wait insertion knows the scalar loads are done too
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (C == 0) at_start();
    lm_f2 na[P::PMAX], nb[P::PMAX];
    if constexpr (C + 1 < P::N) {
      load_w<C + 1>(na, nb, ra, rb);
      issue<P::pbeg(C + 1), P::pend(C + 1)>(base);
    } else if constexpr (NEXT) {
      load_w<0>(na, nb, ra_n, rb_n);
      issue<P::pbeg(0), P::pend(0)>(base_n);
    }
    __builtin_amdgcn_sched_barrier(0);
    compute_from<P::beg(C), C, A, B>();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (C + 1 < P::N || NEXT) {
#pragma unroll
      for (int q = 0; q < P::PMAX; ++q) {
        wa[q] = na[q];
        wb[q] = nb[q];
      }
    }
    if constexpr (C + 1 < P::N) chunks<C + 1, A, B, NEXT>(base, base_n, ra, rb, ra_n, rb_n, at_start);
  }
};

// The ring kernels' arguments, gathered for rw_tile.
struct RwArgs {
  const LmConst* K;
  LmDetGroup G;
  const uint8_t* ext;
  int64_t ext_slot_bytes;
  const float* weights;
  int32_t s0, nslots;
  unsigned long long* keys;
  int32_t* n_pos;
  uint8_t* tailbin;
  int64_t tailbin_slot_bytes;
  const int32_t* tl_cnt;
  const uint32_t* tl_list;
};

// One wave's work (the body of k_corr_rw and k_corr_rw_all): LM_RW_NQ
// sub-tiles of 40 x 4 outputs, 8 lanes each (lane 8 q + lx), each sub-tile
// streaming its window (kh + 3 rows of 40 + kw - 1 pixels) through its own
// LDS ring of 3 rows + 1 mirror.  Lane lx of sub-tile q owns 5 columns x 4
// rows as two packed row pairs; at step t (t = 0 .. kh + 1) it reads window
// rows t and t + 1 (pair 0 with weight row t, pair 1 with weight row t - 2);
// row t + 3 is stored at the end of step t into row t's slot, its global
// load issued two steps earlier.  A wave's LDS operations run in order, so
// no barrier anywhere.  The sub-tiles' row loads: load k of a lane is dword
// dk of sub-tile qk's window row (lane + 64 k = qk NL + dk).
template <int KW, bool UNF>
DEV __attribute__((always_inline)) void rw_tile(const RwArgs& A, int dix, const RwRun& R, float* ring) {
  constexpr int NQ = LM_RW_NQ, NQX = LM_RW_NQX;
  constexpr int QX = LM_FW / PK_C;  // lanes across a sub-tile
  static_assert(LM_FH == PK_R && QX * NQ == 64, "one row of 8 lanes per 40 x 4 sub-tile");
  constexpr int STR = rw_stride(KW);
  constexpr int QP = rw_qpitch(KW);
  constexpr int NL = (3 + LM_FW + KW - 1 + 3) / 4;  // dwords of a sub-tile's window row
  constexpr int NLD = (NQ * NL + 63) / 64;          // dwords a lane loads per row
  static_assert(NLD <= 4, "window rows wider than four loads per lane");
  constexpr int HS = LM_RW_HSLOTS;
  const LmConst& K = *A.K;
  const LmDet& D = K.det[dix];
  const int lane = threadIdx.x & 63;
  const int q = lane / QX, lx = lane % QX;
  const int kh = D.kh, kwp = D.kwp;
  // the host runs one-row detectors on k_corr_gen: without this the compiler
  // also lays out kh < 2 paths, on which a prefetched pixel pair could reach
  // the epilogue without its wait (infeasible, but the LDS-wait checker of
  // tests/test_kernel_resources.py cannot tell)
  __builtin_assume(kh >= 2);
  const int nrows = LM_RW_HTH + kh - 1;
  const int ew = K.ext_w[D.view];
  const int ew4 = ew >> 2;  // ext rows are padded to 16 bytes
  const uint8_t* __restrict__ vext = A.ext + (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0);
  // the ext crops start 256-byte aligned per slot, views and rows are
  // multiples of 16 bytes and tile origins of 4, so every window row starts
  // in_x & 3 bytes past a dword
  const int mis = D.in_x & 3;
  // the lane's sub-tile
  int slot, oy0, ox0;
  R.tile(q, R.entry(q), slot, oy0, ox0);
  const bool valid = q < R.nvalid;
  // row loads: load k of a lane is dword dk of sub-tile qk's window row
  // (e = lane + 64 k = qk NL + dk), stored at LDS byte address lo[k] of the rings.  They
  // are buffer loads from the wave's lowest slot: the base in a buffer
  // resource (SGPRs), the row offset a scalar, and a 32-bit byte offset per
  // lane, so no load needs vector address arithmetic.  A wave's sub-tiles
  // come from one list segment (the slots of one k_ingest workgroup per 64 of
  // them) or one slot, so the lane offsets stay far below 4 GiB.
  int smin = slot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) smin = min(smin, __shfl_xor(smin, o));
  smin = __builtin_amdgcn_readfirstlane(smin);
  const __amdgpu_buffer_rsrc_t wrsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(vext + (int64_t)smin * A.ext_slot_bytes), 0, (int)0xFFFFFFFF, 0x00020000);
  unsigned la[NLD];
  int lo[NLD];  // LDS byte address of the load's ring column (row 0)
  bool lk[NLD];
#pragma unroll
  for (int k = 0; k < NLD; ++k) {
    const int e = lane + 64 * k, qk = e / NL, dk = e - qk * NL;
    lk[k] = qk < R.nvalid;
    int sk, yk, xk;
    const int ik = min(qk, NQ - 1);  // lanes past the last sub-tile: a valid address, the value unused
    R.tile(ik, R.entry(ik), sk, yk, xk);
    la[k] = (unsigned)((int64_t)(sk - smin) * A.ext_slot_bytes + (int64_t)(D.in_y + yk) * ew + (D.in_x + xk - mis)) +
            4u * (unsigned)dk;
    lo[k] = (int)(unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)(ring + qk * QP + 4 * dk);
  }

  // brightness mask of the point detectors' outputs (crop pixel > 25), read
  // from the ext crop now so the loads are long done by the epilogue: per
  // output row the lane's 5 bytes, from the two aligned dwords they lie in
  unsigned mbits = 0;
  if (D.kind == 0 && valid) {
    const uint8_t* __restrict__ m =
        vext + (int64_t)slot * A.ext_slot_bytes + (int64_t)(D.m_y + oy0) * ew + (D.m_x + ox0 + lx * PK_C);
    const int mo = (int)((uintptr_t)m & 3);  // the same for every row (ew is a multiple of 16)
    const unsigned* __restrict__ m4 = reinterpret_cast<const unsigned*>(m - mo);
    unsigned mw[PK_R][2];
#pragma unroll
    for (int r = 0; r < PK_R; ++r) {
      mw[r][0] = m4[(int64_t)r * ew4];
      mw[r][1] = m4[(int64_t)r * ew4 + 1];
    }
#pragma unroll
    for (int r = 0; r < PK_R; ++r) {
      const unsigned long long row = ((unsigned long long)mw[r][1] << 32 | mw[r][0]) >> (8 * mo);
#pragma unroll
      for (int c = 0; c < PK_C; ++c) mbits |= (((unsigned)(row >> (8 * c)) & 0xFFu) > 25u ? 1u : 0u) << (r * PK_C + c);
    }
  }

  struct Row {
    unsigned v[NLD];
  };
  // Every lane loads unconditionally (rows past the window clamped to its
  // last, lanes without a sub-tile at a valid address; those values are never
  // stored), so the loads of a step are not behind branches and the compiler
  // can wait for the older row with vmcnt(NLD) while the newer one stays in
  // flight.
  auto load_row = [&](int r) -> Row {
    Row w;
    // the row offset is wave-uniform: keep it scalar (the compiler otherwise
    // forms it with 64-bit vector multiplies in every step)
    const int ro = __builtin_amdgcn_readfirstlane(min(r, nrows - 1) * ew);
#pragma unroll
    for (int k = 0; k < NLD; ++k) w.v[k] = __builtin_amdgcn_raw_buffer_load_b32(wrsrc, (int)la[k], ro, 0);
    return w;
  };
  auto store_row = [&](int r, Row w) {
    if (r >= nrows) return;
    const int s = r % HS;  // r is wave-uniform: scalar arithmetic
    // the slot's byte offset as one scalar (else the compiler adds two per store)
    const int so = __builtin_amdgcn_readfirstlane(s * STR * (int)sizeof(float));
#pragma unroll
    for (int k = 0; k < NLD; ++k)
      if (lk[k]) {
        const unsigned v = w.v[k];
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v f = {(float)(v & 0xFFu), (float)((v >> 8) & 0xFFu), (float)((v >> 16) & 0xFFu), (float)(v >> 24)};
        typedef __attribute__((address_space(3))) f4v lds_f4;
        *reinterpret_cast<lds_f4*>((uintptr_t)(unsigned)(lo[k] + so)) = f;
        if (s == 0) *reinterpret_cast<lds_f4*>((uintptr_t)(unsigned)(lo[k] + HS * STR * (int)sizeof(float))) = f;
      }
  };
  {
    Row v0[HS];
#pragma unroll
    for (int r = 0; r < HS; ++r) v0[r] = load_row(r);
#pragma unroll
    for (int r = 0; r < HS; ++r) store_row(r, v0[r]);
  }

  const lm_f2* __restrict__ W = reinterpret_cast<const lm_f2*>(A.weights + D.w_off);  // kwp is a multiple of 4
  const int kwp2 = kwp >> 1;
  const unsigned ring_base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)ring +
                             (unsigned)(q * QP * (int)sizeof(float));
  const unsigned lane_off = (unsigned)((lx * PK_C + mis) * (int)sizeof(float));
  const unsigned ring_lane = ring_base + lane_off;
  auto row_base = [&](int t) -> unsigned {  // the slot offset as one scalar: one vector add per row
    return ring_lane + (unsigned)__builtin_amdgcn_readfirstlane((t % HS) * STR * (int)sizeof(float));
  };
  RwPipe<KW, UNF> S;
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int c = 0; c < PK_C; ++c) S.acc[p][c] = (lm_f2){D.delta, D.delta};
  auto wrow = [&](int i) { return W + min(max(i, 0), kh - 1) * kwp2; };
  S.template load_w<0>(S.wa, S.wb, wrow(0), wrow(-2));
  S.template issue<RwPlan<KW>::pbeg(0), RwPlan<KW>::pend(0)>(row_base(0));
  using T1 = std::true_type;
  using F0 = std::false_type;
  // Step t reads ring rows t and t + 1 and prefetches step t + 1's pixel
  // pairs in its last chunk; at its end it stores row t + HS into the slot
  // of row t (dead by then: a wave's LDS operations run in order).  That
  // row's global load was issued at the start of step t - 1, so it has two
  // steps to land: step t loads row t + HS + 1 into one register set while
  // it stores the other (even steps store r0 and load r1, odd steps the
  // reverse -- the step loop is unrolled by two by hand, so no register copy
  // makes the wave wait for the load just issued).
  auto stepx = [&](int t, auto B0, auto B1, Row& st, Row& ld, auto N) {
    S.template chunks<0, decltype(B0)::value, decltype(B1)::value, decltype(N)::value>(
        row_base(t), row_base(t + 1), wrow(t), wrow(t - 2), wrow(t + 1), wrow(t - 1),
        [&]() { if constexpr (decltype(N)::value) ld = load_row(t + HS + 1); });
    if constexpr (decltype(N)::value) store_row(t + HS, st);  // the last step stores no row (t + HS >= nrows)
  };
  Row r0 = load_row(HS), r1;
  {  // kh >= 2: the host runs one-row detectors on k_corr_gen
    // pair 0 (tap row t) runs while t < kh, pair 1 (tap row t - 2) from t = 2
    stepx(0, T1{}, F0{}, r0, r1, T1{});
    stepx(1, T1{}, F0{}, r1, r0, T1{});
    int t = 2;
    for (; t + 1 < kh; t += 2) {
      stepx(t, T1{}, T1{}, r0, r1, T1{});
      stepx(t + 1, T1{}, T1{}, r1, r0, T1{});
    }
    if (t < kh) {
      stepx(t, T1{}, T1{}, r0, r1, T1{});
      stepx(kh, F0{}, T1{}, r1, r0, T1{});
      stepx(kh + 1, F0{}, T1{}, r0, r1, F0{});
    } else {
      stepx(kh, F0{}, T1{}, r0, r1, T1{});
      stepx(kh + 1, F0{}, T1{}, r1, r0, F0{});
    }
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);  // the last (unused) prefetch

  // epilogue (the ring is dead: this wave's reads were issued first)
  unsigned bits = 0;
  if (valid) {
#pragma unroll
    for (int p = 0; p < PK_R / 2; ++p)
#pragma unroll
      for (int c = 0; c < PK_C; ++c) {
        const int x = ox0 + lx * PK_C + c;
        const int y0 = oy0 + 2 * p;
        if (x < D.ow && y0 < D.oh && S.acc[p][c].x > 0.0f) bits |= 1u << ((2 * p) * PK_C + c);
        if (x < D.ow && y0 + 1 < D.oh && S.acc[p][c].y > 0.0f) bits |= 1u << ((2 * p + 1) * PK_C + c);
      }
  }
  if (D.kind != 0) {
    // tail map (the sub-tiles are one 80 x 16 tile with sub-tile 0 at its top
    // left): 16 rows x <= 4 u32 words (the tile's origin is a multiple of 80,
    // so 80 columns touch at most 4 words) = one word per lane, gathered in
    // the ring, then ORed into the slot's bitmap
    unsigned* s_tb = reinterpret_cast<unsigned*>(ring);
    const int w0 = (ox0 - (q % NQX) * LM_FW) >> 5;  // the tile's first word
    const int ty = (q / NQX) * LM_FH;               // the lane's first row in the tile
    s_tb[lane] = 0u;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < PK_R; ++r)
#pragma unroll
      for (int c = 0; c < PK_C; ++c)
        if (bits & (1u << (r * PK_C + c))) {
          const int x = ox0 + lx * PK_C + c;
          atomicOr(&s_tb[(ty + r) * 4 + (x >> 5) - w0], 1u << (x & 31));
        }
    __builtin_amdgcn_wave_barrier();
    const unsigned v = s_tb[lane];
    unsigned* __restrict__ tb = reinterpret_cast<unsigned*>(A.tailbin + (int64_t)slot * A.tailbin_slot_bytes) +
                                (D.list ? (int64_t)K.tail_hb * K.tail_nw : 0);
    const int y = oy0 - (q / NQX) * LM_FH + (lane >> 2), gw = w0 + (lane & 3);  // rows from the tile's top
    if (v && y < D.oh && gw < K.tail_nw) atomicOr(&tb[(int64_t)y * K.tail_nw + gw], v);
    return;
  }
  bits &= mbits;
  // keys: each lane's set bits at consecutive places after the lanes of its
  // sub-tile before it (popcount, then an inclusive scan over the sub-tile's
  // 8 lanes), one global atomic per sub-tile (keys are sorted later: their
  // order in the list does not matter)
  const int cnt = __popc(bits);
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < QX; o <<= 1) {
    const int u = __shfl_up(incl, o, QX);
    if (lx >= o) incl += u;
  }
  const int tot = __shfl(incl, QX - 1, QX);  // the sub-tile's count
  const int before = incl - cnt, lastl = (lane & ~(QX - 1)) + QX - 1;
  if (__ballot(tot != 0) == 0) return;
  int base_k = 0;
  if (lane == lastl && tot) base_k = atomicAdd(&A.n_pos[slot * LM_NLIST + D.list], tot);
  base_k = __shfl(base_k, lastl);
  unsigned long long* __restrict__ kl = A.keys + (int64_t)slot * K.keys_per_slot + K.list_off[D.list] + base_k + before;
  int pos = 0;
#pragma unroll
  for (int p = 0; p < PK_R / 2; ++p)
#pragma unroll
    for (int c = 0; c < PK_C; ++c)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int r = 2 * p + hh, k = r * PK_C + c;
        if (bits & (1u << k)) {
          const int y = oy0 + r, x = ox0 + lx * PK_C + c;
          const float sc = hh ? S.acc[p][c].y : S.acc[p][c].x;
          kl[pos++] = ((unsigned long long)(~__float_as_uint(sc)) << 32) | (unsigned)(y * D.ow + x);
        }
      }
}

// XCD-aware work order: workgroups are dispatched to the 8 XCDs round-robin
// (block b on XCD b mod 8), each XCD with its own L2.  Block b takes logical
// block xcd_block(b): the logical blocks come in runs of LM_RW_XCD
// consecutive ones, and each run goes to one XCD (runs dealt to the XCDs in
// turn, so the empty waves at the grid's end stay spread over all eight).
// Consecutive work items are neighbouring bright tiles of one frame, so the
// sub-tiles that re-read each other's window rows (the (kh - 1)-row vertical
// halo, the (kw - 1)-column horizontal one) fetch them from one L2.
#ifndef LM_RW_XCD
#define LM_RW_XCD 16  // run length in workgroups (0: the hardware order)
#endif
DEV int xcd_block(int b, int nb) {
#if LM_RW_XCD
  constexpr int C = LM_RW_XCD;
  const int full = nb / (8 * C) * (8 * C);
  if (b >= full) return b;  // the last partial round: hardware order
  const int k = b >> 3, x = b & 7;
  return (k / C) * (8 * C) + x * C + (k % C);
#else
  (void)nb;
  return b;
#endif
}

// One launch per width group (LM_KW_LIST widths).
// Waves per SIMD: the 40-column sub-tiles' rings allow 4 (80-column ones: 5
// at kw <= 32); the register budget is set to match.
#ifndef LM_RW_WPE
#define LM_RW_WPE (LM_FW == 40 ? 4 : 5)
#endif
template <int KW, bool UNF>
__global__ __launch_bounds__(LM_RW_THREADS) __attribute__((amdgpu_waves_per_eu(KW <= 32 ? LM_RW_WPE : 1, 8))) void k_corr_rw(
    const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext, int64_t ext_slot_bytes,
    const float* __restrict__ weights, int s0, int nslots, unsigned long long* __restrict__ keys,
    int32_t* __restrict__ n_pos, uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes,
    const int32_t* __restrict__ tl_cnt, const uint32_t* __restrict__ tl_list) {
  extern __shared__ uint4 lds_rw[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* ring = reinterpret_cast<float*>(lds_rw) + wave * rw_ring_floats(KW);
  const RwArgs a{Kp, G, ext, ext_slot_bytes, weights, s0, nslots, keys, n_pos, tailbin, tailbin_slot_bytes, tl_cnt, tl_list};
  int d;
  RwRun R;
  if (!corr_locate_rw(*a.K, a.G, a.nslots, a.s0, xcd_block(blockIdx.x, gridDim.x) * LM_RW_WAVES + wave, a.tl_cnt,
                      a.tl_list, d, R))
    return;
  rw_tile<KW, UNF>(a, d, R, ring);
}

// Every ring detector of the context in ONE launch (longest first), so the
// widths share the launch's tail instead of each ending its own; each wave
// branches to its width's body.  G.ring_floats: LDS floats per wave (the
// widest detector's rings and the tail scratch words).
template <bool UNF>
__global__ __launch_bounds__(LM_RW_THREADS) __attribute__((amdgpu_waves_per_eu(LM_RW_ALL_WPE, 8))) void k_corr_rw_all(
    const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext, int64_t ext_slot_bytes,
    const float* __restrict__ weights, int s0, int nslots, unsigned long long* __restrict__ keys,
    int32_t* __restrict__ n_pos, uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes,
    const int32_t* __restrict__ tl_cnt, const uint32_t* __restrict__ tl_list) {
  extern __shared__ uint4 lds_rw[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* ring = reinterpret_cast<float*>(lds_rw) + wave * G.ring_floats;
  const RwArgs a{Kp, G, ext, ext_slot_bytes, weights, s0, nslots, keys, n_pos, tailbin, tailbin_slot_bytes, tl_cnt, tl_list};
  int d;
  RwRun R;
  if (!corr_locate_rw(*a.K, a.G, a.nslots, a.s0, xcd_block(blockIdx.x, gridDim.x) * LM_RW_WAVES + wave, a.tl_cnt,
                      a.tl_list, d, R))
    return;
  switch (a.K->det[d].kw_ring) {
#define LM_KW_CASE(n)           \
  case n:                       \
    rw_tile<n, UNF>(a, d, R, ring); \
    break;
    LM_KW_LIST_RW_ALL(LM_KW_CASE)
#undef LM_KW_CASE
    default:
      break;
  }
}

// ---------------------------------------------------------------- k_corr_gen
// Any detector size.  Same thread shape and arithmetic as k_corr_pk, but the
// width is a runtime value (taps in chunks of LM_JC = 4 columns over the
// zero-padded row of kwp weights) and the detector rows are processed in
// chunks of D.chunk_rows, each with its own LDS window of 48 + chunk - 1 rows,
// so a detector of any height fits.  Each output still visits its taps in
// row-major order (chunks in order, rows in order, columns in order).
template <bool UNF>
__global__ __launch_bounds__(LM_CORR_THREADS) void k_corr_gen(const LmConst* __restrict__ Kp, const LmDetGroup G,
                                                              const uint8_t* __restrict__ ext, int64_t ext_slot_bytes,
                                                              const float* __restrict__ weights, int s0,
                                                              unsigned long long* __restrict__ keys,
                                                              int32_t* __restrict__ n_pos, uint8_t* __restrict__ tailbin,
                                                              int64_t tailbin_slot_bytes,
                                                              const uint8_t* __restrict__ dark) {
  const LmConst& K = *Kp;
  extern __shared__ float lds[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  const CorrTile T = corr_tile(K, G);
  const LmDet D = K.det[T.d];
  const int oy0 = T.oy0, ox0 = T.ox0;
  if (corr_tile_dark(K, D, dark, slot, oy0, ox0)) return;
  const int kh = D.kh, kwp = D.kwp, ch = D.chunk_rows;
  const int cols = LM_TW + kwp - 1, stride = pk_stride(cols);
  const int ew = K.ext_w[D.view];
  const uint8_t* __restrict__ src = corr_src(K, D, ext, ext_slot_bytes, slot, oy0, ox0);
  const float* __restrict__ W = weights + D.w_off;
  if (threadIdx.x == 0) s_cnt = 0;
  const int ly = threadIdx.x >> 4, lx = threadIdx.x & 15;
  lm_f2 acc[PK_R / 2][PK_C];
#pragma unroll
  for (int p = 0; p < PK_R / 2; ++p)
#pragma unroll
    for (int c = 0; c < PK_C; ++c) acc[p][c] = (lm_f2){D.delta, D.delta};
  for (int i0 = 0; i0 < kh; i0 += ch) {
    const int cn = min(ch, kh - i0);
    __syncthreads();  // the previous chunk's LDS reads are done
    tile_fill_f32(lds, stride, src + (int64_t)i0 * ew, ew, LM_TH + cn - 1, cols);
    __syncthreads();
    for (int t = 0; t < cn + PK_R - 2; ++t) {
      const float* p0 = lds + (ly * PK_R + t) * stride + lx * PK_C;
      for (int jc = 0; jc < kwp; jc += LM_JC) {
        lm_f2 px[PK_C + LM_JC - 1];
#pragma unroll
        for (int q = 0; q < PK_C + LM_JC - 1; ++q) px[q] = (lm_f2){p0[jc + q], p0[jc + q + stride]};
#pragma unroll
        for (int p = 0; p < PK_R / 2; ++p) {
          const int i = t - 2 * p;
          if (i >= 0 && i < cn) {
            const float* wr = W + (int64_t)(i0 + i) * kwp + jc;
#pragma unroll
            for (int j = 0; j < LM_JC; ++j) {
              const float w = wr[j];
              const lm_f2 w2 = (lm_f2){w, w};
#pragma unroll
              for (int c = 0; c < PK_C; ++c) acc[p][c] = corr_tap<UNF>(acc[p][c], w2, px[c + j]);
            }
          }
        }
      }
    }
  }
  float accf[PK_R][PK_C];
#pragma unroll
  for (int p = 0; p < PK_R / 2; ++p)
#pragma unroll
    for (int c = 0; c < PK_C; ++c) {
      accf[2 * p][c] = acc[p][c].x;
      accf[2 * p + 1][c] = acc[p][c].y;
    }
  // the mask pixels come from the ext crop (the LDS window holds only the last chunk)
  const uint8_t* msrc = ext + (int64_t)slot * ext_slot_bytes + (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                        (int64_t)(D.m_y + oy0) * ew + (D.m_x + ox0);
  corr_epilogue<PK_R, PK_C>(K, D, accf, nullptr, 0, ly, lx, oy0, ox0, slot, keys, n_pos, tailbin, tailbin_slot_bytes,
                            &s_cnt, &s_base, msrc, ew, lds);
}

// ---------------------------------------------------------------- k_corr_f16
// Non-parity half-precision mode (lm_setup.corr_precision = LM_CORR_F16,
// BASELINE config 5): u8 pixels (exact in f16) times f16 weights (each
// detector's scaled by a power of two, so the rounding is 2^-12 relative and
// nothing is subnormal), accumulated in fp32 by v_mfma_f32_32x32x16_f16.
// Kernel row i of a detector is a banded (Toeplitz) product
//     C[y][x] += sum_k A_i[y][k] * B_i[k][x],  A_i[y][k] = I(y + i, x0 + k),
//                                              B_i[k][x] = w[i][k - x] (0 off the band)
// over k < 16 * NCH (32 + kw - 1 rounded up to 16).  A fragments are aligned
// 16-byte reads of the f16 window in LDS (row stride = 8 mod 16 halfs: the
// 32 rows a read touches fall in distinct bank groups).  B fragments do not
// depend on the output tile: the host lays them out once per detector in the
// MFMA's lane order ([i][chunk][lane] x 8 halfs), and every wave loads row
// i + 1's fragments from global memory (the same NCH KiB for every workgroup:
// L1 / L2 hits) into registers while it multiplies with row i's, using each
// for its two 32 x 32 output tiles; the LDS holds only the window, and the
// row loop has no barrier.
// 2 x 2 waves: a 128 x 64 output tile per workgroup; each wave holds two
// 32 x 32 tiles side by side, which share their A fragments (tile 1 at
// window chunk m + 2 is tile 0 at chunk m: NCH + 2 LDS reads per detector row
// for 2 NCH MFMAs instead of 2 NCH) and every B fragment.
// Accumulator layout (32x32 MFMA): column = lane & 31, row = (reg & 3) +
// 8 (reg >> 2) + 4 (lane >> 5).
typedef _Float16 lm_h8 __attribute__((ext_vector_type(8)));
typedef float lm_f32x16 __attribute__((ext_vector_type(16)));

// u8 window -> f16 LDS: each thread converts 8 pixels per item (one 8-byte
// global load at any alignment, one 16-byte LDS store: the row stride is a
// multiple of 8 halfs); up to 7 columns past `cols` are written (inside the
// row's stride) and never read.
#ifndef LM_F16_FILLU
#define LM_F16_FILLU 4  // 8-byte window loads in flight per thread
#endif
DEV void tile_fill_f16(_Float16* __restrict__ lds, int stride, const uint8_t* __restrict__ src, int ew, int rows,
                       int cols) {
  constexpr int UF = LM_F16_FILLU;
  const int ng = (cols + 7) >> 3;
  const int total = rows * ng;
  for (int e0 = 0; e0 < total; e0 += UF * (int)blockDim.x) {
    uint2 v[UF];
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int e = e0 + u * (int)blockDim.x + (int)threadIdx.x;
      if (e < total) {
        const int r = e / ng, g = e - r * ng;
        __builtin_memcpy(&v[u], src + (int64_t)r * ew + 8 * g, 8);
      }
    }
#pragma unroll
    for (int u = 0; u < UF; ++u) {
      const int e = e0 + u * (int)blockDim.x + (int)threadIdx.x;
      if (e < total) {
        const int r = e / ng, g = e - r * ng;
        lm_h8 h;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          h[k] = (_Float16)(float)((v[u].x >> (8 * k)) & 0xFFu);
          h[4 + k] = (_Float16)(float)((v[u].y >> (8 * k)) & 0xFFu);
        }
        *reinterpret_cast<lm_h8*>(lds + r * stride + 8 * g) = h;
      }
    }
  }
}

template <int NCH>
__global__ __launch_bounds__(LM_F16_THREADS) __attribute__((amdgpu_waves_per_eu(NCH <= 7 ? 3 : 2))) void k_corr_f16(const LmConst* __restrict__ Kp, const LmDetGroup G,
                                                            const uint8_t* __restrict__ ext, int64_t ext_slot_bytes,
                                                            const uint4* __restrict__ bfrag, int s0,
                                                            unsigned long long* __restrict__ keys,
                                                            int32_t* __restrict__ n_pos, uint8_t* __restrict__ tailbin,
                                                            int64_t tailbin_slot_bytes,
                                                            const uint8_t* __restrict__ dark) {
  const LmConst& K = *Kp;
  // uint4: the dynamic area starts 16-byte aligned after the static variables
  // (with a float array it would start 8 bytes in, and every ds_read_b128 of
  // the window would be misaligned — an order of magnitude slower)
  extern __shared__ uint4 lds_f16[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  const CorrTile T = corr_tile(K, G);
  const LmDet D = K.det[T.d];
  const int oy0 = T.oy0, ox0 = T.ox0, kh = D.kh;
  if (corr_tile_dark(K, D, dark, slot, oy0, ox0)) return;
  constexpr int cols = f16_cols(NCH), STR = f16_stride(cols);
  const int rows = LM_F16_TH + kh - 1;
  _Float16* __restrict__ img = reinterpret_cast<_Float16*>(lds_f16);
  tile_fill_f16(img, STR, corr_src(K, D, ext, ext_slot_bytes, slot, oy0, ox0), K.ext_w[D.view], rows, cols);
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, r = lane & 31, h = lane >> 5;
  // 2 x 2 waves; wave (wx, wy) owns output columns 64 wx .. + 63 (two 32 x 32
  // accumulator tiles side by side) of rows 32 wy .. + 31.  Tile 1's A
  // fragment at window chunk m + 2 is tile 0's at chunk m, so a row's
  // NCH + 2 A fragments feed both tiles: A_m x B_m into tile 0 (m < NCH),
  // A_m x B_(m-2) into tile 1 (m >= 2).
  static_assert(LM_F16_WAVES == 4 && LM_F16_TW == 128 && LM_F16_TH == 64, "2 x 2 waves of two 32 x 32 tiles");
  const int wx = wave & 1, wy = wave >> 1;
  constexpr int NS = NCH + 2;  // A steps per detector row
  const float init = D.delta * D.wscale;
  lm_f32x16 acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[t][q] = init;
  const _Float16* __restrict__ arow = img + (32 * wy + r) * STR + 64 * wx + 8 * h;
  const lm_h8* __restrict__ bsrc = reinterpret_cast<const lm_h8*>(bfrag + D.w16_off) + lane;
  // Detector rows in groups of three, flattened to 3 NM (row, A step)
  // steps: step k's A fragment was read two steps earlier (a 3-deep register
  // ring), so an MFMA never waits on the LDS read issued right before it; B
  // fragments of row i + 3 load while rows i + 1, i + 2 multiply.  With the
  // group unrolled, every ring index is static.
  lm_h8 bf[3][NCH], ar[3];
  auto load_b = [&](lm_h8 (&b)[NCH], int i) {
#pragma unroll
    for (int c = 0; c < NCH; ++c) b[c] = bsrc[(int64_t)(i * NCH + c) * 64];
  };
  const int xb = ox0 + 64 * wx + r;  // tile t: column xb + 32 t
  const int yb = oy0 + 32 * wy;
  const _Float16* __restrict__ mrow = img + (D.m_y - D.in_y + 32 * wy) * STR + 64 * wx + r + (D.m_x - D.in_x);
  // tile t runs only when it holds an output (inside oh x ow) and, for a
  // point detector, some output whose mouse pixel is > 25 (the rest are
  // zeroed by the reference's mask and produce no key)
  bool on[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    bool any = false;
    if (xb + 32 * t < D.ow && yb < D.oh) {
      if (D.kind != 0) {
        any = true;
      } else {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int ly = 16 * h + q;
          any |= yb + ly < D.oh && (float)mrow[ly * STR + 32 * t] > 25.0f;
        }
      }
    }
    on[t] = __builtin_amdgcn_readfirstlane(__ballot(any) != 0 ? 1 : 0) != 0;
  }
  auto mma_all = [&](auto c0, auto c1) {
    constexpr bool ON0 = decltype(c0)::value, ON1 = decltype(c1)::value;
    constexpr int M0 = ON0 ? 0 : 2, M1 = ON1 ? NS : NCH;  // the A steps a row needs
    constexpr int NM = M1 - M0;
    auto load_a = [&](lm_h8& a, int i, int m) { a = *reinterpret_cast<const lm_h8*>(arow + min(i, kh - 1) * STR + 16 * (M0 + m)); };
    auto mma = [&](const lm_h8& a, lm_h8 (&b)[NCH], int m) {
      const int mm = M0 + m;
      if (ON0 && mm < NCH) acc[0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[mm < NCH ? mm : 0], acc[0], 0, 0, 0);
      if (ON1 && mm >= 2) acc[1] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b[mm >= 2 ? mm - 2 : 0], acc[1], 0, 0, 0);
    };
#pragma unroll
    for (int q = 0; q < 3; ++q)
      if (q < kh) load_b(bf[q], q);
    load_a(ar[0], 0, 0);
    load_a(ar[1], 1 / NM, 1 % NM);
    int i = 0;
    for (; i + 2 < kh; i += 3) {
#pragma unroll
      for (int k = 0; k < 3 * NM; ++k) {
        const int q = k / NM, m = k % NM, k2 = k + 2;
        load_a(ar[k2 % 3], i + k2 / NM, k2 % NM);
        __builtin_amdgcn_sched_barrier(0);
        mma(ar[k % 3], bf[q], m);
        if (m == NM - 1 && i + q + 3 < kh) load_b(bf[q], i + q + 3);
      }
    }
    // the last kh % 3 rows (their B fragments are in bf[0], bf[1])
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (i + q < kh)
#pragma unroll
        for (int m = 0; m < NM; ++m) {
          lm_h8 a;
          load_a(a, i + q, m);
          mma(a, bf[q], m);
        }
  };
  using T1 = std::true_type;
  using F0 = std::false_type;
  if (on[0] && on[1])
    mma_all(T1{}, T1{});
  else if (on[0])
    mma_all(T1{}, F0{});
  else if (on[1])
    mma_all(F0{}, T1{});

  if (D.kind != 0) {
    // bits straight from a ballot: this wave owns u32 words (ox0 / 32 + 2 wx + t)
    // of its rows (lanes 0-31: row y, lanes 32-63: row y + 4)
    unsigned* __restrict__ tb = reinterpret_cast<unsigned*>(tailbin + (int64_t)slot * tailbin_slot_bytes) +
                                (D.list ? (int64_t)K.tail_hb * K.tail_nw : 0);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int gw = (ox0 >> 5) + 2 * wx + t, x = xb + 32 * t;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int y = yb + (q & 3) + 8 * (q >> 2) + 4 * h;
        const unsigned long long m = __ballot(y < D.oh && x < D.ow && acc[t][q] > 0.0f);
        if ((lane & 31) == 0 && y < D.oh && gw < K.tail_nw) tb[(int64_t)y * K.tail_nw + gw] = (unsigned)(m >> (32 * h));
      }
    }
    return;
  }
  unsigned bits = 0;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ly = (q & 3) + 8 * (q >> 2) + 4 * h;
      const int y = yb + ly, x = xb + 32 * t;
      const float pix = (float)mrow[ly * STR + 32 * t];
      if (y < D.oh && x < D.ow && pix > 25.0f && acc[t][q] > 0.0f) bits |= 1u << (16 * t + q);
    }
  const int nk = __popc(bits);
  const int off = nk ? atomicAdd(&s_cnt, nk) : 0;
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&n_pos[slot * LM_NLIST + D.list], s_cnt) : 0;
  __syncthreads();
  unsigned long long* __restrict__ kl = keys + (int64_t)slot * K.keys_per_slot + K.list_off[D.list] + s_base + off;
  int k = 0;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (bits & (1u << (16 * t + q))) {
        const int y = yb + (q & 3) + 8 * (q >> 2) + 4 * h, x = xb + 32 * t;
        const float score = acc[t][q] * D.inv_wscale;
        kl[k++] = ((unsigned long long)(~__float_as_uint(score)) << 32) | (unsigned)(y * D.ow + x);
      }
}

// Debug copy of raw scores (lm_debug_scores): the same chain per output,
// computed straight from the ext crops in global memory (no LDS, any size).
template <bool UNF>
__global__ __launch_bounds__(256) void k_corr_dbg(const LmConst* __restrict__ Kp, const uint8_t* __restrict__ ext,
                                                  int64_t ext_slot_bytes, const float* __restrict__ weights, int s0,
                                                  float* __restrict__ dbg, const int64_t* __restrict__ dbg_off,
                                                  int64_t dbg_slot_floats) {
  const LmConst& K = *Kp;
  const int slot = s0 + blockIdx.y;
  const int d = blockIdx.z;
  const LmDet D = K.det[d];
  const int64_t n = (int64_t)D.oh * D.ow;
  const int ew = K.ext_w[D.view];
  const uint8_t* __restrict__ base =
      ext + (int64_t)slot * ext_slot_bytes + (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0);
  const float* __restrict__ W = weights + D.w_off;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int y = (int)(e / D.ow), x = (int)(e % D.ow);
    const uint8_t* src = base + (int64_t)(D.in_y + y) * ew + (D.in_x + x);
    float a = D.delta;
    for (int i = 0; i < D.kh; ++i)
      for (int j = 0; j < D.kw; ++j) a = corr_tap1<UNF>(a, W[i * D.kwp + j], (float)src[(int64_t)i * ew + j]);
    dbg[(int64_t)slot * dbg_slot_floats + dbg_off[d] + e] = a;
  }
}

// ---------------------------------------------------------------- dispatch
const void* corr_kernel_f16(int kw) {
  switch (f16_nch(kw)) {
    case 2: return (const void*)&k_corr_f16<2>;
    case 3: return (const void*)&k_corr_f16<3>;
    case 4: return (const void*)&k_corr_f16<4>;
    case 5: return (const void*)&k_corr_f16<5>;
    case 6: return (const void*)&k_corr_f16<6>;
    case 7: return (const void*)&k_corr_f16<7>;
    case 8: return (const void*)&k_corr_f16<8>;
    case 9: return (const void*)&k_corr_f16<9>;
    case 10: return (const void*)&k_corr_f16<10>;
    default: return nullptr;
  }
}

bool corr_ring(int kw) {
  switch (kw) {
#define LM_KW_CASE(n) case n:
    LM_KW_LIST(LM_KW_CASE)
#undef LM_KW_CASE
    return true;
    default:
      return false;
  }
}

const void* corr_kernel(int kw, bool unf) {
  switch (kw) {
#define LM_KW_CASE(n) \
  case n:             \
    return unf ? (const void*)&k_corr_rw<n, true> : (const void*)&k_corr_rw<n, false>;
    LM_KW_LIST(LM_KW_CASE)
#undef LM_KW_CASE
    default:
      return unf ? (const void*)&k_corr_gen<true> : (const void*)&k_corr_gen<false>;
  }
}

size_t corr_rw_lds(int kw) { return (size_t)LM_RW_WAVES * rw_ring_floats(kw) * sizeof(float); }

const void* corr_kernel_gen(bool unf) { return unf ? (const void*)&k_corr_gen<true> : (const void*)&k_corr_gen<false>; }

const void* corr_kernel_rw_all(bool unf) {
  return unf ? (const void*)&k_corr_rw_all<true> : (const void*)&k_corr_rw_all<false>;
}

hipError_t launch_corr(const void* fn, bool ring, dim3 grid, int threads, size_t lds, hipStream_t st, const LmConst* K,
                       const LmDetGroup& G, const uint8_t* ext, int64_t ext_slot_bytes, const void* weights, int s0,
                       unsigned long long* keys, int32_t* n_pos, uint8_t* tailbin, int64_t tailbin_slot_bytes,
                       const CorrDark& dk) {
  if (ring) {
    int nslots = (int)grid.y;
    const unsigned waves = (unsigned)(G.tile_end[G.n - 1] * nslots);  // every 80 x 16 tile (corr_locate_rw)
    void* args[] = {(void*)&K,       (void*)&G,    (void*)&ext,     (void*)&ext_slot_bytes,
                    (void*)&weights, (void*)&s0,   (void*)&nslots,  (void*)&keys,
                    (void*)&n_pos,   (void*)&tailbin, (void*)&tailbin_slot_bytes, (void*)&dk.cnt,
                    (void*)&dk.list};
    return hipLaunchKernel(fn, dim3((waves + LM_RW_WAVES - 1) / LM_RW_WAVES), dim3(LM_RW_THREADS), args, lds, st);
  }
  void* args[] = {(void*)&K,     (void*)&G,       (void*)&ext,     (void*)&ext_slot_bytes,           (void*)&weights,
                  (void*)&s0,    (void*)&keys,    (void*)&n_pos,   (void*)&tailbin, (void*)&tailbin_slot_bytes,
                  (void*)&dk.flags};
  return hipLaunchKernel(fn, grid, dim3(threads), args, lds, st);
}

hipError_t launch_corr_dbg(bool unf, dim3 grid, hipStream_t st, const LmConst* K, const uint8_t* ext,
                           int64_t ext_slot_bytes, const float* weights, int s0, float* dbg, const int64_t* dbg_off,
                           int64_t dbg_slot_floats) {
  if (unf)
    k_corr_dbg<true><<<grid, 256, 0, st>>>(K, ext, ext_slot_bytes, weights, s0, dbg, dbg_off, dbg_slot_floats);
  else
    k_corr_dbg<false><<<grid, 256, 0, st>>>(K, ext, ext_slot_bytes, weights, s0, dbg, dbg_off, dbg_slot_floats);
  return hipGetLastError();
}

