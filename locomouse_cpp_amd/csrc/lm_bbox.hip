// lm_bbox.hip — whole-video bounding-box pass, method 0, on gfx950
// (SURVEY.md §8(f) row 1): LocoMouse::computeBoundingBox
// (LocoMouse_class.cpp:579-653) with computeMouseBox (:948-997),
// largestBWAreaObject (:921-946), firstLastOverT (LocoMouse_class.hpp:411-440),
// computeMouseBoxSize (:1481-1506), medianvec / stdvec / vecmovingaverage
// (:1516-1608).  Its own translation unit of liblocomouse_hip.so; k_minmax /
// k_lut come from lm_kernels.hip through launch_minmax_lut (lm_host.h).
//
// Exact reformulation on 0/1 images.  medianBlur is a rank filter and the
// threshold after it (:955, v > 2.55 <=> v >= 3) is monotone, so
//     median(window) >= 3  <=>  #{x in window : x >= 3} >= (n + 1) / 2,  n = k^2.
// The zero-initialised border ring of I_median (:585-603) is rewritten by the
// in-place medianBlur every frame (:952) and read back by the next frame's
// filter; only its indicator [v >= 3] ever reaches a later threshold, so the
// ring is carried as 0/1 too.  The per-frame work becomes box counts over
// bytes (k_bb_center) plus a small sequential recurrence over the ring
// (k_bb_ring, one workgroup walking the batch's frames in order).
//
// Per batch of n frames:
//   k_minmax      \ normalize LUT per frame (shared with the detection path)
//   k_lut         /
//   k_bb_ingest   I_median centre indicator  M[f] = [corrected frame >= 3]
//   k_bb_bands    the border bands of M[f] in k_bb_ring's LDS layout
//   k_bb_ring     ring state recurrence; writes ring_{f-1} into M[f]
//   k_bb_center   11x11 (k x k) majority over M[f] -> thresholded image bin[f]
//   k_bb_cc       per (frame, view): largest component (row runs + union-find
//                 in LDS; per-pixel union-find in global memory when a view
//                 has too many runs), row/column counts, firstLastOverT
// The host turns the limits into computeMouseBox's six values and runs the
// whole-video post-processing in lm_bb_finish.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "locomouse_hip.h"
#include "lm_device.h"
#include "lm_dev_common.h"
#include "lm_host.h"
#include "lm_cc.h"

struct LmBBConst {
  int32_t n_rows, n_cols;  // corrected image
  int32_t p, hp, wp;       // median half-size; I_median rows / cols
  int32_t thr;             // ones needed in a window: (k*k + 1) / 2
  int32_t flip;
  int32_t view_y[2], view_h[2];  // 0 side, 1 bottom (x = 0, width = n_cols)
  int32_t conn, semantics, min_pixel_visible;
  int32_t ring_n;          // ring state bytes: top [p][wp] | bottom [p][wp] | left [n_rows][p] | right [n_rows][p]
  int32_t band_n;          // per-frame band bytes (k_bb_bands), multiple of 16
  int32_t bits_nw;         // bit-packed ring (p <= 7): words per band row; 0 = byte ring in M
  int32_t run_cap;         // k_bb_cc: runs per view held in LDS
  int64_t m_bytes;         // per-frame I_median indicator image (hp x wp)
  int64_t bin_bytes;       // per-frame thresholded image (n_rows x n_cols)
  int64_t cc_words;        // per-frame run tables for views with many runs (6 words per possible run)
};

// ---------------------------------------------------------------- k_bb_ingest
// readFrame(I_center) (:615, :1273-1333) fused with the indicator: 4 centre
// pixels per thread.
__global__ __launch_bounds__(256) void k_bb_ingest(const LmBBConst K, const uint8_t* const* __restrict__ frame_ptr,
                                                   const uint8_t* __restrict__ bkg, const int32_t* __restrict__ cal,
                                                   const uint8_t* __restrict__ luts, uint8_t* __restrict__ M) {
  const int f = blockIdx.y;
  __shared__ uint8_t lut[256];
  lut[threadIdx.x] = luts[f * 256 + threadIdx.x];
  __syncthreads();
  const lm_gu8* __restrict__ F = as_global(frame_ptr[f]);
  uint8_t* __restrict__ Mf = M + (int64_t)f * K.m_bytes;
  const int64_t np = (int64_t)K.n_rows * K.n_cols;
  const int64_t q0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t q = q0 + k;
    if (q >= np) break;
    const int r = (int)(q / K.n_cols), c = (int)(q % K.n_cols);
    const int cs = K.flip ? K.n_cols - 1 - c : c;
    const int idx = cal[(int64_t)r * K.n_cols + cs];
    const int fv = F[idx], bv = bkg[idx];
    Mf[(int64_t)(r + K.p) * K.wp + c + K.p] = lut[fv > bv ? fv - bv : 0] >= 3 ? 1 : 0;
  }
}

// ----------------------------------------------------------------- k_bb_bands
// Per frame, the 2p-wide bands of M[f] along the border in exactly the LDS
// layout k_bb_ring uses (top [2p][wp] | bottom [2p][wp] | left [hp][2p] |
// right [hp][2p]), so the sequential kernel fetches a frame with contiguous
// dword loads issued one frame ahead.  Ring positions are placeholders (the
// ring kernel overwrites them from its state).
__global__ __launch_bounds__(256) void k_bb_bands(const LmBBConst K, const uint8_t* __restrict__ M,
                                                  uint8_t* __restrict__ bands) {
  const int f = blockIdx.y, p2 = 2 * K.p, wp = K.wp, hp = K.hp;
  const uint8_t* __restrict__ Mf = M + (int64_t)f * K.m_bytes;
  const int q0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
  const int tb = p2 * wp, lb = hp * p2;
  uint32_t w = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int q = q0 + k;
    if (q >= 2 * tb + 2 * lb) break;
    int r, c;
    if (q < 2 * tb) {
      const int qq = q < tb ? q : q - tb;
      r = qq / wp;
      c = qq - r * wp;
      if (q >= tb) r += hp - p2;
    } else {
      const int qq = q - 2 * tb, side = qq >= lb, q2 = side ? qq - lb : qq;
      r = q2 / p2;
      c = q2 - r * p2 + (side ? wp - p2 : 0);
    }
    w |= (uint32_t)Mf[(int64_t)r * wp + c] << (8 * k);
  }
  if (q0 < K.band_n) *reinterpret_cast<uint32_t*>(bands + (int64_t)f * K.band_n + q0) = w;
}

// ------------------------------------------------------------------ k_bb_ring
// One 1024-thread workgroup; the ring state lives in LDS across the batch.
// For frame f: (1) copy the frame's bands (prefetched into registers during
// frame f-1) into LDS, put the ring state (= ring_{f-1}) over their ring
// positions and publish it into M[f]'s ring for k_bb_center; (2) horizontal
// clamped window counts; (3) vertical clamped counts at the ring pixels ->
// ring_f.  Clamping is medianBlur's BORDER_REPLICATE at the edges of
// I_median.  Counts run as sliding sums along rows / columns (segments per
// thread), so a frame costs O(band area) LDS byte operations.
// Workgroup barrier that waits for LDS traffic only: __syncthreads() would also
// drain the global prefetch of the next frame and the ring publish stores
// (s_waitcnt vmcnt(0)), exposing their latency at every barrier.
DEV void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

#define LM_BB_SEG 24   // horizontal segment per thread
#define LM_BB_VCH 16   // left/right ring rows per thread
#define LM_BB_BDW 16   // band dwords per thread (band_n <= 64 KiB)
__global__ __launch_bounds__(1024) void k_bb_ring(const LmBBConst K, uint8_t* __restrict__ M,
                                                  const uint8_t* __restrict__ bands, int n,
                                                  uint8_t* __restrict__ ring, unsigned long long* __restrict__ prof) {
  unsigned long long t_last = prof ? __builtin_amdgcn_s_memtime() : 0ull;
  auto tick = [&](int ph) {  // diagnostics (LM_BB_PROF=1): shader clocks per phase, thread 0
    if (prof && threadIdx.x == 0) {
      const unsigned long long t = __builtin_amdgcn_s_memtime();
      prof[ph] += t - t_last;
      t_last = t;
    }
  };
  extern __shared__ uint8_t sm[];
  const int p = K.p, p2 = 2 * p, hp = K.hp, wp = K.wp, nr = K.n_rows, thr = K.thr;
  const int tid = threadIdx.x, nt = blockDim.x;
  uint8_t* sT = sm;                          // [p][wp]
  uint8_t* sB = sT + p * wp;                 // [p][wp]
  uint8_t* sL = sB + p * wp;                 // [nr][p]
  uint8_t* sR = sL + nr * p;                 // [nr][p]
  uint8_t* bT = sm + ((K.ring_n + 15) & ~15);  // [2p][wp]  rows 0 .. 2p-1
  uint8_t* bB = bT + p2 * wp;                // [2p][wp]  rows hp-2p .. hp-1
  uint8_t* bL = bB + p2 * wp;                // [hp][2p]  cols 0 .. 2p-1
  uint8_t* bR = bL + hp * p2;                // [hp][2p]  cols wp-2p .. wp-1
  uint8_t* hT = bT + ((K.band_n + 15) & ~15);  // [2p][wp]
  uint8_t* hB = hT + p2 * wp;                // [2p][wp]
  uint8_t* hL = hB + p2 * wp;                // [hp][p]
  uint8_t* hR = hL + hp * p;                 // [hp][p]
  uint32_t* bT32 = reinterpret_cast<uint32_t*>(bT);
  const int nd = K.band_n >> 2;
  uint32_t cur[LM_BB_BDW], nxt[LM_BB_BDW];
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(bands);
#pragma unroll
    for (int k = 0; k < LM_BB_BDW; ++k) cur[k] = tid + k * nt < nd ? src[tid + k * nt] : 0u;
  }
  for (int i = tid; i < K.ring_n; i += nt) sm[i] = ring[i];
  lds_barrier();
  const int nseg = (wp + LM_BB_SEG - 1) / LM_BB_SEG;
  const int nhT = 2 * p2 * nseg;  // horizontal tasks, top + bottom bands
  const int nch = (nr + LM_BB_VCH - 1) / LM_BB_VCH;
  for (int f = 0; f < n; ++f) {
    uint8_t* __restrict__ Mf = M + (int64_t)f * K.m_bytes;
    if (f + 1 < n) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(bands + (int64_t)(f + 1) * K.band_n);
#pragma unroll
      for (int k = 0; k < LM_BB_BDW; ++k) nxt[k] = tid + k * nt < nd ? src[tid + k * nt] : 0u;
    }
#pragma unroll
    for (int k = 0; k < LM_BB_BDW; ++k)
      if (tid + k * nt < nd) bT32[tid + k * nt] = cur[k];
    // publish ring_{f-1} into M[f]
    for (int c = tid; c < wp; c += nt)
      for (int r = 0; r < p; ++r) {
        Mf[(int64_t)r * wp + c] = sT[r * wp + c];
        Mf[(int64_t)(hp - p + r) * wp + c] = sB[r * wp + c];
      }
    for (int i = tid; i < nr * p; i += nt) {
      const int r = i / p, j = i - r * p;
      Mf[(int64_t)(r + p) * wp + j] = sL[i];
      Mf[(int64_t)(r + p) * wp + wp - p + j] = sR[i];
    }
    lds_barrier();
    tick(0);
    // ring positions of the bands from the state
    for (int c = tid; c < wp; c += nt) {
      for (int r = 0; r < p; ++r) {
        bT[r * wp + c] = sT[r * wp + c];
        bB[(p + r) * wp + c] = sB[r * wp + c];
      }
      if (c < p || c >= wp - p) {
        const uint8_t* side = c < p ? sL + c : sR + c - (wp - p);
        for (int r = p; r < p2; ++r) {
          bT[r * wp + c] = side[(r - p) * p];                  // M row r
          bB[(r - p) * wp + c] = side[(hp - p2 + r - p - p) * p];  // M row hp-2p+(r-p)
        }
      }
    }
    for (int r = tid; r < hp; r += nt) {
      if (r < p || r >= hp - p) {
        const uint8_t* src = r < p ? sT + r * wp : sB + (r - (hp - p)) * wp;
        for (int j = 0; j < p2; ++j) {
          bL[r * p2 + j] = src[j];
          bR[r * p2 + j] = src[wp - p2 + j];
        }
      } else {
        for (int j = 0; j < p; ++j) {
          bL[r * p2 + j] = sL[(r - p) * p + j];
          bR[r * p2 + p + j] = sR[(r - p) * p + j];
        }
      }
    }
    lds_barrier();
    tick(1);
    // (2) horizontal counts: sliding sums over row segments
    for (int t = tid; t < nhT + 2 * hp; t += nt) {
      if (t < nhT) {
        const int band = t / (p2 * nseg), rem = t - band * (p2 * nseg);
        const int r = rem / nseg, c0 = (rem - r * nseg) * LM_BB_SEG, c1 = min(c0 + LM_BB_SEG, wp);
        const uint8_t* src = (band ? bB : bT) + r * wp;
        uint8_t* dst = (band ? hB : hT) + r * wp;
        int s = 0;
        for (int dc = -p; dc <= p; ++dc) s += src[min(max(c0 + dc, 0), wp - 1)];
        dst[c0] = (uint8_t)s;
        for (int c = c0 + 1; c < c1; ++c) {
          s += src[min(c + p, wp - 1)] - src[max(c - 1 - p, 0)];
          dst[c] = (uint8_t)s;
        }
      } else {
        const int q = t - nhT, side = q / hp, r = q - side * hp;
        if (side == 0) {  // ring cols 0..p-1: band cols [j-p, j+p] clamped at 0
          const uint8_t* src = bL + r * p2;
          int s = 0;
          for (int dc = -p; dc <= p; ++dc) s += src[max(dc, 0)];
          hL[r * p] = (uint8_t)s;
          for (int j = 1; j < p; ++j) {
            s += src[j + p] - src[max(j - 1 - p, 0)];
            hL[r * p + j] = (uint8_t)s;
          }
        } else {  // ring cols wp-p+j: band cols [j, 2p+j] clamped at 2p-1
          const uint8_t* src = bR + r * p2;
          int s = 0;
          for (int k = 0; k <= p2; ++k) s += src[min(k, p2 - 1)];
          hR[r * p] = (uint8_t)s;
          for (int j = 1; j < p; ++j) {
            s += src[p2 - 1] - src[j - 1];
            hR[r * p + j] = (uint8_t)s;
          }
        }
      }
    }
    lds_barrier();
    tick(2);
    // (3) vertical counts -> ring_f
    for (int t = tid; t < 2 * wp + 2 * p * nch; t += nt) {
      if (t < wp) {  // top ring column: rows [r-p, r+p] clamped at 0
        const int c = t;
        int s = (p + 1) * hT[c];
        for (int k = 1; k <= p; ++k) s += hT[k * wp + c];
        sT[c] = s >= thr ? 1 : 0;
        for (int r = 1; r < p; ++r) {
          s += hT[(r + p) * wp + c] - hT[max(r - 1 - p, 0) * wp + c];
          sT[r * wp + c] = s >= thr ? 1 : 0;
        }
      } else if (t < 2 * wp) {  // bottom ring column: band rows [i, 2p+i] clamped at 2p-1
        const int c = t - wp;
        int s = 0;
        for (int k = 0; k <= p2; ++k) s += hB[min(k, p2 - 1) * wp + c];
        sB[c] = s >= thr ? 1 : 0;
        for (int i = 1; i < p; ++i) {
          s += hB[(p2 - 1) * wp + c] - hB[(i - 1) * wp + c];
          sB[i * wp + c] = s >= thr ? 1 : 0;
        }
      } else {  // left / right ring: (side, column j, chunk of rows)
        const int q = t - 2 * wp, side = q / (p * nch), rem = q - side * (p * nch);
        const int j = rem / nch, r0 = (rem - j * nch) * LM_BB_VCH, r1 = min(r0 + LM_BB_VCH, nr);
        const uint8_t* h = side ? hR : hL;
        uint8_t* st = side ? sR : sL;
        int s = 0;
        for (int dr = -p; dr <= p; ++dr) s += h[(r0 + p + dr) * p + j];
        st[r0 * p + j] = s >= thr ? 1 : 0;
        for (int r = r0 + 1; r < r1; ++r) {
          s += h[(r + p + p) * p + j] - h[(r - 1) * p + j];
          st[r * p + j] = s >= thr ? 1 : 0;
        }
      }
    }
    lds_barrier();
    tick(3);
#pragma unroll
    for (int k = 0; k < LM_BB_BDW; ++k) cur[k] = nxt[k];
  }
  for (int i = tid; i < K.ring_n; i += nt) ring[i] = sm[i];
}

// ------------------------------------------------- bit-packed ring (p <= 7)
// The same recurrence on bitmaps: the 2p-row top/bottom bands as rows of
// 32-bit words, the 2p-column left/right bands as one word per I_median row.
// The ring state lives inside these bitmaps (ring positions), so a frame is:
// merge the frame's centre bits (prefetched one frame ahead) -> window counts
// by popcount of funnel-shifted words (top / bottom: one thread per column
// keeps its 2p counts in registers and forms the vertical counts there) ->
// new ring rows by wave ballots -> refresh corner duplicates and padding.
// k_bb_center reads ring_{f-1} from the published band words (rbits).
//
// Band word layout (per frame; also the global band / rbits buffers):
//   T  [2p][NW]  I_median rows 0 .. 2p-1, bit position = column + p; the p
//                positions on either side replicate columns 0 / wp-1
//                (BORDER_REPLICATE), so a window is one popcount
//   Bt [2p][NW]  rows hp-2p .. hp-1, same columns
//   L  [hp]      bit j = column j (j < 2p)
//   R  [hp]      bit j = column wp-2p+j
struct BBBits {
  int P, NW, hp, wp, nw;  // nw: words per frame
  DEV int t(int r) const { return r * NW; }
  DEV int b(int r) const { return (2 * P + r) * NW; }
  DEV int l(int r) const { return 4 * P * NW + r; }
  DEV int rr(int r) const { return 4 * P * NW + hp + r; }
};

DEV BBBits bb_bits(const LmBBConst& K) {
  BBBits B;
  B.P = K.p;
  B.NW = K.bits_nw;
  B.hp = K.hp;
  B.wp = K.wp;
  B.nw = 4 * K.p * K.bits_nw + 2 * K.hp;
  return B;
}

DEV bool bb_is_center(int P, int hp, int wp, int r, int c) { return r >= P && r < hp - P && c >= P && c < wp - P; }

// Centre bits of M[f] in the band word layout (ring and padding positions 0).
__global__ __launch_bounds__(256) void k_bb_bands_bits(const LmBBConst K, const uint8_t* __restrict__ M,
                                                       uint32_t* __restrict__ bands) {
  const BBBits B = bb_bits(K);
  const int f = blockIdx.y, w = blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= B.nw) return;
  const int P = B.P, hp = B.hp, wp = B.wp;
  const uint8_t* __restrict__ Mf = M + (int64_t)f * K.m_bytes;
  uint32_t v = 0;
  if (w < 4 * P * B.NW) {
    const int band = w / (2 * P * B.NW), q = w - band * 2 * P * B.NW;
    const int i = q / B.NW, k = q - i * B.NW;
    const int r = band ? hp - 2 * P + i : i;
    for (int j = 0; j < 32; ++j) {
      const int c = 32 * k + j - P;
      if (c >= 0 && c < wp && bb_is_center(P, hp, wp, r, c) && Mf[(int64_t)r * wp + c]) v |= 1u << j;
    }
  } else {
    const int q = w - 4 * P * B.NW, side = q >= hp, r = side ? q - hp : q;
    for (int j = 0; j < 2 * P; ++j) {
      const int c = side ? wp - 2 * P + j : j;
      if (bb_is_center(P, hp, wp, r, c) && Mf[(int64_t)r * wp + c]) v |= 1u << j;
    }
  }
  bands[(int64_t)f * B.nw + w] = v;
}

// Ones at positions [lo, lo + n) of a bitmap row (n <= 32).
DEV int bb_popc_range(const uint32_t* row, int lo, int n) {
  const int k = lo >> 5, s = lo & 31;
  const unsigned long long x = (((unsigned long long)row[k + 1] << 32) | row[k]) >> s;
  return __popcll(x & ((1ull << n) - 1));
}
DEV uint32_t bb_get_bits(const uint32_t* row, int lo, int n) {  // n <= 32
  const int k = lo >> 5, s = lo & 31;
  const unsigned long long x = (((unsigned long long)row[k + 1] << 32) | row[k]) >> s;
  return (uint32_t)(x & ((1ull << n) - 1));
}
DEV void bb_set_bits(uint32_t* row, int lo, int n, uint32_t v) {  // n <= 32, single writer
  const int k = lo >> 5, s = lo & 31;
  const unsigned long long m = ((1ull << n) - 1) << s, x = (unsigned long long)v << s;
  unsigned long long w = (((unsigned long long)row[k + 1] << 32) | row[k]);
  w = (w & ~m) | (x & m);
  row[k] = (uint32_t)w;
  row[k + 1] = (uint32_t)(w >> 32);
}
// Padding positions of a T/Bt row replicate columns 0 and wp-1.
DEV void bb_pad_row(uint32_t* row, int P, int wp) {
  bb_set_bits(row, 0, P, ((row[P >> 5] >> (P & 31)) & 1u) ? 0xFFFFFFFFu : 0u);
  const int q = wp - 1 + P;
  bb_set_bits(row, wp + P, P, ((row[q >> 5] >> (q & 31)) & 1u) ? 0xFFFFFFFFu : 0u);
}

template <int P>
__global__ __launch_bounds__(1024) void k_bb_ring_bits(const LmBBConst K, const uint32_t* __restrict__ bands, int n,
                                                       uint32_t* __restrict__ state, uint32_t* __restrict__ rbits) {
  extern __shared__ uint32_t smw[];
  const BBBits B = bb_bits(K);
  const int NW = B.NW, hp = B.hp, wp = B.wp, nw = B.nw, thr = K.thr;
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6;
  uint32_t* W = smw;                                  // [nw] band words
  uint32_t* HL = smw + nw;                            // [2][hp][HLW] packed byte counts
  constexpr int HLW = (P + 3) / 4;
  constexpr uint32_t PM = (1u << P) - 1, P2M = (1u << (2 * P)) - 1;
  const int npos = wp + P;  // column c sits at position c + P
  // per-thread word slots and their frame-invariant keep masks (non-centre bits)
  constexpr int SL = 4;
  uint32_t keep[SL];
  for (int k = 0; k < SL; ++k) {
    const int w = tid + k * nt;
    uint32_t m = 0xFFFFFFFFu;
    if (w < 4 * P * NW) {
      const int band = w / (2 * P * NW), q = w - band * 2 * P * NW;
      const int i = q / NW, kk = q - i * NW;
      const int r = band ? hp - 2 * P + i : i;
      for (int j = 0; j < 32; ++j) {
        const int c = 32 * kk + j - P;
        if (c >= 0 && c < wp && bb_is_center(P, hp, wp, r, c)) m &= ~(1u << j);
      }
    } else if (w < nw) {
      const int q = w - 4 * P * NW, side = q >= hp, r = side ? q - hp : q;
      m = (r < P || r >= hp - P) ? 0xFFFFFFFFu : (side ? ~(PM << P) : ~PM);
    }
    keep[k] = m;
  }
  for (int w = tid; w < nw; w += nt) W[w] = state[w];
  uint32_t cur[SL], nxt[SL];
#pragma unroll
  for (int k = 0; k < SL; ++k) cur[k] = tid + k * nt < nw ? bands[tid + k * nt] : 0u;
  lds_barrier();
  for (int f = 0; f < n; ++f) {
    if (f + 1 < n) {
#pragma unroll
      for (int k = 0; k < SL; ++k) nxt[k] = tid + k * nt < nw ? bands[(int64_t)(f + 1) * nw + tid + k * nt] : 0u;
    }
    // (A) merge the centre bits; publish ring_{f-1} + centre for k_bb_center
#pragma unroll
    for (int k = 0; k < SL; ++k) {
      const int w = tid + k * nt;
      if (w < nw) {
        const uint32_t v = (W[w] & keep[k]) | cur[k];
        W[w] = v;
        rbits[(int64_t)f * nw + w] = v;
      }
    }
    lds_barrier();
    // (B) top / bottom: thread per position, 2p window counts -> vertical counts in registers
    uint32_t ntop[2] = {0, 0}, nbot[2] = {0, 0};
    for (int cb = 0; cb < 2 && cb * nt < npos; ++cb) {
      const int c = cb * nt + tid - P;
      if (c >= 0 && c < wp) {
        int h[2 * P];
#pragma unroll
        for (int i = 0; i < 2 * P; ++i) h[i] = bb_popc_range(W + B.t(i), c, 2 * P + 1);
        int sacc = (P + 1) * h[0];
#pragma unroll
        for (int k = 1; k <= P; ++k) sacc += h[k];
        uint32_t bits = sacc >= thr ? 1u : 0u;
#pragma unroll
        for (int r = 1; r < P; ++r) {
          sacc += h[r + P] - h[r - 1 - P < 0 ? 0 : r - 1 - P];
          bits |= (sacc >= thr ? 1u : 0u) << r;
        }
        ntop[cb] = bits;
#pragma unroll
        for (int i = 0; i < 2 * P; ++i) h[i] = bb_popc_range(W + B.b(i), c, 2 * P + 1);
        sacc = 0;
#pragma unroll
        for (int k = 0; k <= 2 * P; ++k) sacc += h[k < 2 * P - 1 ? k : 2 * P - 1];
        bits = sacc >= thr ? 1u : 0u;
#pragma unroll
        for (int i = 1; i < P; ++i) {
          sacc += h[2 * P - 1] - h[i - 1];
          bits |= (sacc >= thr ? 1u : 0u) << i;
        }
        nbot[cb] = bits;
      }
    }
    // left / right: per row, p window counts (packed bytes) -> HL
    for (int q = tid; q < 2 * hp; q += nt) {
      const int side = q >= hp, r = side ? q - hp : q;
      const uint32_t word = W[side ? B.rr(r) : B.l(r)];
      uint32_t pk[HLW];
#pragma unroll
      for (int k = 0; k < HLW; ++k) pk[k] = 0;
#pragma unroll
      for (int j = 0; j < P; ++j) {
        int cnt;
        if (!side) {  // columns [j-p, j+p], clamped at 0
          cnt = __popc(word & ((2u << (j + P)) - 1)) + (P - j) * (int)(word & 1u);
        } else {      // band columns [j, 2p+j], clamped at 2p-1
          cnt = __popc(word & P2M & ~((1u << j) - 1)) + (j + 1) * (int)((word >> (2 * P - 1)) & 1u);
        }
        pk[j >> 2] |= (uint32_t)cnt << (8 * (j & 3));
      }
#pragma unroll
      for (int k = 0; k < HLW; ++k) HL[(side * hp + r) * HLW + k] = pk[k];
    }
    lds_barrier();
    // (C) new top / bottom ring rows by ballot (padding positions 0 for now);
    // left / right vertical counts -> new left / right ring bits
    for (int cb = 0; cb < 2 && cb * nt < npos; ++cb) {
      const int c = cb * nt + tid - P;
      const bool valid = c >= 0 && c < wp;
      const int wbase = (cb * nt + wave * 64) >> 5;
      const bool wr = lane == 0 && cb * nt + wave * 64 < npos + P;
#pragma unroll
      for (int r = 0; r < P; ++r) {
        const unsigned long long bt = __ballot(valid && ((ntop[cb] >> r) & 1u));
        const unsigned long long bb = __ballot(valid && ((nbot[cb] >> r) & 1u));
        if (wr) {
          W[B.t(r) + wbase] = (uint32_t)bt;
          W[B.t(r) + wbase + 1] = (uint32_t)(bt >> 32);
          W[B.b(P + r) + wbase] = (uint32_t)bb;
          W[B.b(P + r) + wbase + 1] = (uint32_t)(bb >> 32);
        }
      }
    }
    for (int q = tid; q < 2 * (hp - 2 * P); q += nt) {
      const int side = q >= hp - 2 * P, R = P + (side ? q - (hp - 2 * P) : q);
      uint32_t acc[HLW];
#pragma unroll
      for (int k = 0; k < HLW; ++k) acc[k] = 0;
#pragma unroll
      for (int d = -P; d <= P; ++d)
#pragma unroll
        for (int k = 0; k < HLW; ++k) acc[k] += HL[(side * hp + R + d) * HLW + k];  // bytes <= (2p+1)^2 <= 225
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < P; ++j) bits |= (((acc[j >> 2] >> (8 * (j & 3))) & 255u) >= (uint32_t)thr ? 1u : 0u) << j;
      if (!side) W[B.l(R)] = (W[B.l(R)] & ~PM) | bits;
      else W[B.rr(R)] = (W[B.rr(R)] & ~(PM << P)) | (bits << P);
    }
    lds_barrier();
    // (D) corner duplicates and padding: L/R rows of the top / bottom rings
    // from T/Bt; ring columns of T rows p..2p-1 and Bt rows 0..p-1 from L/R
    for (int q = tid; q < 4 * P; q += nt) {
      const int grp = q / P, i = q - grp * P;
      if (grp < 2) {  // top ring row i / bottom ring row hp-p+i (band row p+i)
        uint32_t* row = W + (grp == 0 ? B.t(i) : B.b(P + i));
        const int r = grp == 0 ? i : hp - P + i;
        bb_pad_row(row, P, wp);
        W[B.l(r)] = bb_get_bits(row, P, 2 * P);              // columns 0 .. 2p-1
        W[B.rr(r)] = bb_get_bits(row, wp - 2 * P + P, 2 * P);  // columns wp-2p .. wp-1
      } else {  // grp 2: T row p+i (I_median row p+i); grp 3: Bt row i (row hp-2p+i)
        const int r = grp == 2 ? P + i : hp - 2 * P + i;
        uint32_t* row = W + (grp == 2 ? B.t(P + i) : B.b(i));
        bb_set_bits(row, P, P, W[B.l(r)] & PM);                 // columns 0 .. p-1
        bb_set_bits(row, wp, P, (W[B.rr(r)] >> P) & PM);        // columns wp-p .. wp-1
        bb_pad_row(row, P, wp);
      }
    }
    lds_barrier();
#pragma unroll
    for (int k = 0; k < SL; ++k) cur[k] = nxt[k];
  }
  for (int w = tid; w < nw; w += nt) state[w] = W[w];
}

// ---------------------------------------------------------------- k_bb_center
// Majority filter over the centre: one 128 x 64 output tile per 256 threads.
// The (64+2p) x (128+2p) input window is staged in LDS; column counts run
// down the tile (thread per column), window counts slide along row segments
// (thread per 32 outputs), and the 0/1 tile leaves through coalesced dword
// stores.
#define LM_BB_TW 128
#define LM_BB_TH 64
__global__ __launch_bounds__(256) void k_bb_center(const LmBBConst K, const uint8_t* __restrict__ M,
                                                   const uint32_t* __restrict__ rbits, uint8_t* __restrict__ bin) {
  extern __shared__ uint8_t sm[];
  const int P = K.p, p2 = 2 * P, hp = K.hp, wp = K.wp;
  const int IW = LM_BB_TW + p2, IH = LM_BB_TH + p2;
  uint8_t* in = sm;                                        // [IH][IW], later the output tile [TH][TW]
  uint8_t* vs = sm + ((IH * IW + 15) & ~15);               // [TH][IW] column counts
  const int c0 = blockIdx.x * LM_BB_TW, r0 = blockIdx.y * LM_BB_TH, f = blockIdx.z, tid = threadIdx.x;
  const uint8_t* __restrict__ Mf = M + (int64_t)f * K.m_bytes;
  const BBBits Bb = bb_bits(K);
  const uint32_t* __restrict__ Rb = rbits + (int64_t)f * Bb.nw;
  for (int i = 0; i < IH; ++i) {
    const int rr = r0 + i;
    for (int j = tid; j < IW; j += blockDim.x) {
      const int cc = c0 + j;
      uint8_t v = 0;
      if (rr < hp && cc < wp) {
        if (K.bits_nw && (rr < P || rr >= hp - P || cc < P || cc >= wp - P)) {  // ring_{f-1} from the band bits
          uint32_t w;
          int bit;
          if (rr < P) {
            w = Rb[Bb.t(rr) + ((cc + P) >> 5)];
            bit = (cc + P) & 31;
          } else if (rr >= hp - P) {
            w = Rb[Bb.b(rr - (hp - 2 * P)) + ((cc + P) >> 5)];
            bit = (cc + P) & 31;
          } else if (cc < P) {
            w = Rb[Bb.l(rr)];
            bit = cc;
          } else {
            w = Rb[Bb.rr(rr)];
            bit = cc - (wp - 2 * P);
          }
          v = (uint8_t)((w >> bit) & 1u);
        } else {
          v = Mf[(int64_t)rr * wp + cc];
        }
      }
      in[i * IW + j] = v;
    }
  }
  __syncthreads();
  for (int j = tid; j < IW; j += blockDim.x) {
    int s = 0;
    for (int k = 0; k < p2; ++k) s += in[k * IW + j];
    for (int i = 0; i < LM_BB_TH; ++i) {
      s += in[(i + p2) * IW + j];
      vs[i * IW + j] = (uint8_t)s;
      s -= in[i * IW + j];
    }
  }
  __syncthreads();
  {
    constexpr int SEG = LM_BB_TW * LM_BB_TH / 256;  // 32 outputs per thread
    const int i = tid / (LM_BB_TW / SEG), cs = (tid % (LM_BB_TW / SEG)) * SEG;
    const uint8_t* v = vs + i * IW + cs;
    int s = 0;
    for (int k = 0; k <= p2; ++k) s += v[k];
    uint8_t* o = in + i * LM_BB_TW + cs;
    o[0] = s >= K.thr ? 1 : 0;
    for (int c = 1; c < SEG; ++c) {
      s += v[c + p2] - v[c - 1];
      o[c] = s >= K.thr ? 1 : 0;
    }
  }
  __syncthreads();
  uint8_t* __restrict__ B = bin + (int64_t)f * K.bin_bytes;
  const bool full = c0 + LM_BB_TW <= K.n_cols && (K.n_cols & 3) == 0;
  for (int q = tid; q < LM_BB_TH * (LM_BB_TW / 4); q += blockDim.x) {
    const int i = q / (LM_BB_TW / 4), c4 = (q % (LM_BB_TW / 4)) * 4, r = r0 + i;
    if (r >= K.n_rows) continue;
    if (full) {
      *reinterpret_cast<uint32_t*>(B + (int64_t)r * K.n_cols + c0 + c4) =
          *reinterpret_cast<const uint32_t*>(in + i * LM_BB_TW + c4);
    } else {
      for (int k = 0; k < 4; ++k)
        if (c0 + c4 + k < K.n_cols) B[(int64_t)r * K.n_cols + c0 + c4 + k] = in[i * LM_BB_TW + c4 + k];
    }
  }
}

// -------------------------------------------------------------------- k_bb_cc
// largestBWAreaObject + reduce + firstLastOverT for one (view, frame).  The
// largest area wins; equal areas go to the component OpenCV labels first
// (8-connectivity: Grana BBDT 2x2-block raster order of its first block;
// 4-connectivity: Wu pixel raster order).  Global-memory union-find tables
// are read with L1-bypassing loads so every wave sees the others' hooks.
// firstLastOverT's pass test on one row/column sum (LocoMouse_class.hpp:419-421).
DEV bool bb_pass(const LmBBConst& K, int count) {
  const int v = 255 * count;  // the mask is 0/255 (cv::compare, :945)
  if (K.semantics == LM_BB_FIRSTLAST_INTEGER) return v >= K.min_pixel_visible;
  return __int_as_float(v) >= (float)K.min_pixel_visible;  // CV_32S read through ptr<float>
}

// The largest component of one view (lm_cc.h: row runs + union-find, run
// table in LDS when a view has at most K.run_cap runs, else in the global
// scratch) and its per-column (difference array) and per-row pixel counts.
// Block-wide call.
template <bool G, class IX>
DEV void bb_cc_runs(const CCRuns<IX> S, const unsigned long long* bm, int nb64, int W, int H, int R,
                    const int* rowoff, bool c8, int* colc, int* rowc, unsigned long long* s_red, unsigned* s_best) {
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63;
  cc_label<G>(S, bm, nb64, W, H, R, rowoff, c8, s_red, s_best);
  const unsigned broot = *s_best;
  if (broot != 0xFFFFFFFFu)
    for (int i = tid; i < R; i += nt) {
      if (rld<G>(&S.par[i]) != broot) continue;
      const int x0 = (int)rld<G>(&S.rs[i]), x1 = (int)rld<G>(&S.re[i]);
      atomicAdd(&rowc[cc_row_of(rowoff, H, i)], x1 - x0 + 1);
      atomicAdd(&colc[x0], 1);
      atomicSub(&colc[x1 + 1], 1);
    }
  __syncthreads();
  // difference array -> per-column counts (inclusive scan by wave 0)
  if (tid < 64) {
    int carry = 0;
    for (int b = 0; b < W; b += 64) {
      const int i = b + lane;
      int inc = i < W ? colc[i] : 0;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      if (i < W) colc[i] = carry + inc;
      carry += __shfl(inc, 63);
    }
  }
  __syncthreads();
}

// LDS of k_bb_cc: counts, run offsets, the view bitmap (dead once the runs
// are extracted, so the union-find arrays reuse it), run columns.
struct BBCCLayout {
  int colc, rowc, rowoff, bm, par, area, key, rs, re, bytes;  // byte offsets
};
__host__ __device__ inline BBCCLayout bb_cc_layout(int W, int Hmax, int cap) {
  BBCCLayout L;
  int o = 0;
  L.colc = o;
  o += 4 * (W + 1);
  L.rowc = o;
  o += 4 * Hmax;
  L.rowoff = o;
  o += 4 * (Hmax + 1);
  o = (o + 7) & ~7;
  L.bm = o;
  L.par = o;
  L.area = o + 4 * cap;
  L.key = o + 8 * cap;
  const int bmb = 8 * Hmax * ((W + 63) / 64 + 1), ufb = 12 * cap;
  o += bmb > ufb ? bmb : ufb;
  L.rs = o;
  o += 2 * cap;
  L.re = o;
  o += 2 * cap;
  L.bytes = o;
  return L;
}

// largestBWAreaObject + reduce + firstLastOverT for one (view, frame).
__global__ __launch_bounds__(1024) void k_bb_cc(const LmBBConst K, const uint8_t* __restrict__ bin,
                                                unsigned* __restrict__ scratch, int32_t* __restrict__ lims) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smc[];
  const int v = blockIdx.x, f = blockIdx.y;
  const int W = K.n_cols, H = K.view_h[v], nb64 = (W + 63) / 64;
  const BBCCLayout L = bb_cc_layout(W, max(K.view_h[0], K.view_h[1]), K.run_cap);
  const uint8_t* __restrict__ Bv = bin + (int64_t)f * K.bin_bytes + (int64_t)K.view_y[v] * W;
  int* colc = reinterpret_cast<int*>(smc + L.colc);      // [W + 1]  Row_* (reduce over rows), difference array
  int* rowc = reinterpret_cast<int*>(smc + L.rowc);      // [H]      Col_*
  int* rowoff = reinterpret_cast<int*>(smc + L.rowoff);  // [H + 1]  run offsets per row
  unsigned long long* bm = reinterpret_cast<unsigned long long*>(smc + L.bm);  // [H][nb64 + 1]
  __shared__ unsigned long long s_red[16];
  __shared__ unsigned s_best;
  __shared__ int s_total;
  __shared__ int s_lim[2][3];  // (first, last, count) for Row, Col
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = nt >> 6;

  for (int i = tid; i < W + 1 + H + H + 1; i += nt) {
    if (i < W + 1) colc[i] = 0;
    else if (i < W + 1 + H) rowc[i - W - 1] = 0;
  }
  if (tid < 2) {
    s_lim[tid][0] = 0x7FFFFFFF;
    s_lim[tid][1] = -1;
    s_lim[tid][2] = 0;
  }
  if (tid == 0) s_best = 0xFFFFFFFFu;
  // view bitmap and run counts per row
  cc_bitmap_u8(Bv, W, W, H, nb64, (W & 15) == 0, nullptr, bm, rowoff);
  cc_wave0_scan(rowoff, H, &s_total);
  const int R = s_total;
  const bool c8 = K.conn == 8;
  if (R <= K.run_cap && W <= 65536) {
    const CCRuns<uint16_t> S{reinterpret_cast<uint16_t*>(smc + L.rs), reinterpret_cast<uint16_t*>(smc + L.re),
                             reinterpret_cast<unsigned*>(smc + L.par), reinterpret_cast<unsigned*>(smc + L.area),
                             reinterpret_cast<unsigned*>(smc + L.key)};
    bb_cc_runs<false>(S, bm, nb64, W, H, R, rowoff, c8, colc, rowc, s_red, &s_best);
  } else {
    const int64_t cap = (int64_t)H * ((W + 1) / 2);  // at most ceil(W/2) runs per row
    unsigned* b = scratch + (int64_t)f * K.cc_words + (v ? 5 * (int64_t)K.view_h[0] * ((W + 1) / 2) : 0);
    const CCRuns<unsigned> S{b, b + cap, b + 2 * cap, b + 3 * cap, b + 4 * cap};
    bb_cc_runs<true>(S, bm, nb64, W, H, R, rowoff, c8, colc, rowc, s_red, &s_best);
  }
  for (int i = tid; i < W + H; i += nt) {
    const int dd = i < W ? 0 : 1, idx = i < W ? i : i - W;
    if (bb_pass(K, i < W ? colc[i] : rowc[idx])) {
      atomicMin(&s_lim[dd][0], idx);
      atomicMax(&s_lim[dd][1], idx);
      atomicAdd(&s_lim[dd][2], 1);
    }
  }
  __syncthreads();
  if (tid < 2) {
    // first_last = {first, last}; {first, 0} when one entry passes; {-1, -1} when none.
    const int n = s_lim[tid][2];
    int32_t* o = lims + ((int64_t)f * 2 + v) * 4 + 2 * tid;
    o[0] = n ? s_lim[tid][0] : -1;
    o[1] = n == 0 ? -1 : (n == 1 ? 0 : s_lim[tid][1]);
  }
}

// ------------------------------------------------------------------- k_bb_de
// LocoMouse_TM_DE::computeMouseBox_DE (TM_DE.cpp:56-113), one workgroup per
// frame: histogram of the corrected side view -> imadjust_default LUT
// (LocoMouse_class.cpp:3244-3311, float cumulative sums, convertTo with float
// scale / shift), the hard-coded zero bands (only rows [100, 149) and columns
// [46, 760) survive), threshold(12.75) and CV_32F column sums, then
// firstLastOverT(th = 10) and bb_x = min(width - 1, last * 1.1).
__global__ __launch_bounds__(1024) void k_bb_de(const LmBBConst K, const uint8_t* const* __restrict__ frame_ptr,
                                                const uint8_t* __restrict__ bkg, const int32_t* __restrict__ cal,
                                                const uint8_t* __restrict__ luts, double* __restrict__ bbx) {
  extern __shared__ int colc[];  // [n_cols]
  __shared__ unsigned hist[16][256];
  __shared__ uint8_t lut[256], lut2[256];
  __shared__ float s_sf, s_hf;
  __shared__ int s_noscale, s_last, s_cnt;
  const int f = blockIdx.x, tid = threadIdx.x, nt = blockDim.x, wave = tid >> 6;
  const int NC = K.n_cols, vy = K.view_y[0], vh = K.view_h[0];
  const lm_gu8* __restrict__ F = as_global(frame_ptr[f]);
  if (tid < 256) lut[tid] = luts[f * 256 + tid];
  for (int i = tid; i < 16 * 256; i += nt) (&hist[0][0])[i] = 0;
  for (int i = tid; i < NC; i += nt) colc[i] = 0;
  if (tid == 0) {
    s_last = -1;
    s_cnt = 0;
  }
  __syncthreads();
  auto pix = [&](int r, int c) -> int {  // corrected image I(r, c) (readFrame, :1302-1327)
    const int cs = K.flip ? NC - 1 - c : c;
    const int idx = cal[(int64_t)r * NC + cs];
    const int fv = F[idx], bv = bkg[idx];
    return lut[fv > bv ? fv - bv : 0];
  };
  const int np = vh * NC;
  for (int q = tid; q < np; q += nt) {
    const int r = q / NC, c = q - r * NC;
    atomicAdd(&hist[wave][pix(vy + r, c)], 1u);
  }
  __syncthreads();
  if (tid < 256) {
    unsigned h = 0;
    for (int w = 1; w < 16; ++w) h += hist[w][tid];
    hist[0][tid] += h;
  }
  __syncthreads();
  if (tid == 0) {
    double sd = 0;
    for (int i = 0; i < 256; ++i) sd += (float)hist[0][i];
    const float sum_histf = (float)sd, min_tol = 0.01f, max_tol = 0.99f;
    float cum = 0;
    int idx0 = 0, idx1 = 0, imin = 0, imax = 0;
    bool cmin = true, cmax = true;
    for (int i = 0; i < 256; ++i) {
      cum = __fadd_rn(cum, (float)hist[0][i]);
      const float cn = __fdiv_rn(cum, sum_histf);
      if ((cn > min_tol) & cmin) {
        idx0 = i;
        cmin = false;
        imin = i;
      }
      if ((cn >= max_tol) & cmax) {
        idx1 = i;
        cmax = false;
        imax = i;
      }
      if (!(cmin || cmax)) break;
    }
    if (imin == imax) idx1 = 256;
    const float r0 = __fdiv_rn((float)idx0, 255.0f), r1 = __fdiv_rn((float)idx1, 255.0f);
    const double d = (double)__fsub_rn(r1, r0);
    const double inv = 1. / d;
    const double alpha = inv, beta = -(double)r0 * inv;
    s_noscale = fabs(alpha - 1) < 2.220446049250313e-16 && fabs(beta) < 2.220446049250313e-16;
    s_sf = (float)alpha;
    s_hf = (float)beta;
  }
  __syncthreads();
  if (tid < 256) {
    int v = tid;
    if (!s_noscale) {
      const float t = __fadd_rn(__fmul_rn((float)tid, s_sf), s_hf);
      const int iv = (int)rintf(t);
      v = iv < 0 ? 0 : (iv > 255 ? 255 : iv);
    }
    lut2[tid] = (uint8_t)v;
  }
  __syncthreads();
  const int r0 = 100, r1 = min(149, vh), c0 = 46, c1 = min(760, NC);
  const int bw = c1 - c0;
  for (int q = tid; q < (r1 - r0) * bw; q += nt) {
    const int r = r0 + q / bw, c = c0 + q % bw;
    if (lut2[pix(vy + r, c)] > 12) atomicAdd(&colc[c], 1);
  }
  __syncthreads();
  for (int i = tid; i < NC; i += nt)
    if ((float)colc[i] >= (float)10) {  // firstLastOverT(Row_side, N_COLS, lims, MIN_PIXEL_COUNT = 10)
      atomicMax(&s_last, i);
      atomicAdd(&s_cnt, 1);
    }
  __syncthreads();
  if (tid == 0) {
    const int last = s_cnt == 0 ? -1 : (s_cnt == 1 ? 0 : s_last);
    const double a = (double)(K.n_cols - 1), b = (double)last * 1.1;  // std::min(width - 1, last * WIDTH_MARGIN)
    bbx[f] = b < a ? b : a;
  }
}

// ================================================================ host side

struct lm_bb_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t s2 = nullptr;  // majority filter + components, overlapping the ring on `stream`
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  int max_batch = 0;
  int64_t npix = 0, frame_stride = 0;
  int view_y[2] = {0, 0};
  lm_bb_params P{};
  LmBBConst K{};
  size_t ring_lds = 0, center_lds = 0, cc_lds = 0;
  DevBuf<uint8_t> bkg, frames, luts, M, ring, bin, bands;
  DevBuf<unsigned> mm;  // k_minmax partial (min, max) pairs
  DevBuf<uint32_t> rbits;  // bit-packed ring: per-frame band words (published ring_{f-1})
  size_t ring_bits_lds = 0;
  DevBuf<unsigned long long> prof;  // LM_BB_PROF=1: k_bb_ring phase clocks
  DevBuf<int32_t> cal;
  DevBuf<unsigned> cc;
  HostBuf<const uint8_t*> fptr;
  HostBuf<int32_t> lims;
  HostBuf<double> bbx;  // method 2: per-frame bb_x
  int method = 0, side_h = 0, bottom_h = 0;
  int last_n = 0;
  std::vector<lm_bb_frame> per;
  std::vector<uint32_t> x_pos, yb_pos, ys_pos;
  ~lm_bb_ctx() {
    if (prof.p) {
      unsigned long long h[8];
      if (hipMemcpy(h, prof.p, sizeof h, hipMemcpyDeviceToHost) == hipSuccess)
        fprintf(stderr, "k_bb_ring phase clocks: %llu  %llu  %llu  %llu\n",
                h[0], h[1], h[2], h[3]);
    }
    if (stream) {
      (void)hipSetDevice(device);
      (void)hipStreamSynchronize(stream);
      if (s2) (void)hipStreamSynchronize(s2);
      for (hipEvent_t e : ev)
        if (e) (void)hipEventDestroy(e);
      if (s2) (void)hipStreamDestroy(s2);
      (void)hipStreamDestroy(stream);
    }
  }
};

namespace {

void bb_validate_and_build(lm_bb_ctx* c, const lm_setup* su, const lm_bb_params* bp) {
  if (!su || !bp) throw std::invalid_argument("null setup / params");
  const lm_bb_params& P = *bp;
  const int method = su->method;
  if (method < 0 || method > 2) throw std::invalid_argument("method must be 0, 1 or 2.");
  if (method == 1 && P.firstlast_semantics != LM_BB_FIRSTLAST_AS_EXECUTED)
    throw std::invalid_argument("lm_bb_*, method 1: only LM_BB_FIRSTLAST_AS_EXECUTED (the result then depends on "
                                "min_pixel_visible alone; bwAreaOpen / disk filter / imfill are not run).");
  if (P.conn_comp_connectivity != 4 && P.conn_comp_connectivity != 8)
    throw std::invalid_argument("Invalid configuration parameter: conn_comp_connectivity must be either 4 or 8.");
  if (P.median_filter_size % 2 == 0 || P.median_filter_size < 1 || P.median_filter_size > 63)
    throw std::invalid_argument("Invalid configuration parameter: median_filter_size must be odd (1..63 here).");
  if (P.min_pixel_visible < 0)
    throw std::invalid_argument("Invalid configuration parameter: min_pixel_visible must be non-negative.");
  if (P.moving_average_window % 2 == 0 || P.moving_average_window < 1)
    throw std::invalid_argument("Invalid configuration parameter: moving_average_window must be odd.");
  if (P.firstlast_semantics != LM_BB_FIRSTLAST_AS_EXECUTED && P.firstlast_semantics != LM_BB_FIRSTLAST_INTEGER)
    throw std::invalid_argument("firstlast_semantics must be LM_BB_FIRSTLAST_AS_EXECUTED or LM_BB_FIRSTLAST_INTEGER.");
  if (!su->background || !su->ind_warp_mapping) throw std::invalid_argument("background / calibration missing.");
  const int VR = su->video_rows, VC = su->video_cols, NR = su->calib_rows, NC = su->calib_cols;
  if (VR <= 0 || VC <= 0 || NR <= 0 || NC <= 0) throw std::invalid_argument("empty video or calibration.");
  const int64_t npix = (int64_t)VR * VC;
  for (int64_t i = 0; i < (int64_t)NR * NC; ++i)
    if (su->ind_warp_mapping[i] < 0 || su->ind_warp_mapping[i] >= npix)
      throw std::runtime_error("Calibration mapping indices out of range.");
  const lm_rect vw[2] = {su->view_box_side, su->view_box_bottom};
  for (int v = 0; v < 2; ++v) {
    if ((v == 0 || method == 0) && (vw[v].x != 0 || vw[v].width != NC))
      throw std::invalid_argument("BB pass: view boxes must span the corrected width (firstLastOverT reads N_COLS sums, :975-976).");
    if (vw[v].x < 0 || vw[v].y < 0 || vw[v].height <= 0 || vw[v].width <= 0 || vw[v].y + vw[v].height > NR ||
        vw[v].x + vw[v].width > NC)
      throw std::runtime_error("BB pass: view box outside the corrected image.");
  }
  if (method == 0) {
    if (NR < P.median_filter_size / 2 || NC < P.median_filter_size / 2)
      throw std::invalid_argument("BB pass: corrected image smaller than the median filter's half size.");
    if (vw[0].y < vw[1].y + vw[1].height && vw[1].y < vw[0].y + vw[0].height)
      throw std::invalid_argument("BB pass: overlapping side and bottom view boxes are not supported.");
  } else if (method == 1) {  // computeMouseBox_DD's colRange / rowRange bounds (TM.cpp:205-208)
    if (P.zero_col_pre < 0 || P.zero_col_post < 0 || P.zero_row_pre < 0 || P.zero_row_post < 0)
      throw std::invalid_argument("Invalid configuration parameter: zero_*_* parameters range from 0 to the relevant size of the image.");
    if (P.bb_width < 1 || P.bb_height_side < 1)
      throw std::invalid_argument("Invalid configuration parameter: bb_width / bb_height_side must be at least 1 pixel.");
    if (P.zero_col_pre > NC || P.zero_col_post > NC || P.zero_row_pre > vw[0].height || P.zero_row_post > vw[0].height)
      throw std::runtime_error("BB pass, method 1: zero_* ranges exceed the side view (cv::Mat::colRange/rowRange assert).");
  } else {  // computeMouseBox_DE's hard-coded ranges (TM_DE.cpp:69-72)
    if (760 > NC || 149 > vw[0].height)
      throw std::runtime_error("BB pass, method 2: the hard-coded zero ranges exceed the side view (cv::Mat::colRange/rowRange assert).");
  }
  c->method = method;
  c->side_h = vw[0].height;
  c->bottom_h = vw[1].height;
  c->P = P;
  c->npix = npix;
  c->frame_stride = (npix + 255) / 256 * 256;
  LmBBConst& K = c->K;
  K.n_rows = NR;
  K.n_cols = NC;
  K.p = P.median_filter_size / 2;
  K.hp = NR + 2 * K.p;
  K.wp = NC + 2 * K.p;
  K.thr = (P.median_filter_size * P.median_filter_size + 1) / 2;
  K.flip = su->flip ? 1 : 0;
  for (int v = 0; v < 2; ++v) {
    K.view_y[v] = vw[v].y;
    K.view_h[v] = vw[v].height;
    c->view_y[v] = vw[v].y;
  }
  K.conn = P.conn_comp_connectivity;
  K.semantics = P.firstlast_semantics;
  K.min_pixel_visible = P.min_pixel_visible;
  K.ring_n = 2 * K.p * K.wp + 2 * NR * K.p;
  K.m_bytes = ((int64_t)K.hp * K.wp + 255) / 256 * 256;
  K.bin_bytes = ((int64_t)NR * NC + 255) / 256 * 256;
  K.cc_words = 5 * (int64_t)((NC + 1) / 2) * (vw[0].height + vw[1].height);  // run tables of both views
  const int p = K.p, p2 = 2 * p;
  K.band_n = (2 * p2 * K.wp + 2 * K.hp * p2 + 15) & ~15;
  // bit-packed ring for p <= 7 (packed byte sums of (2p+1)^2 <= 255 window counts)
  K.bits_nw = 0;
  if (p >= 1 && p <= 7 && NR >= 2 * p && NC >= 2 * p && K.wp + 2 * p <= 2048) {
    const int nw_row = (K.wp + 2 * p + 63) / 64 * 2 + 1;  // ballot words up to the 64-aligned end, +1 for funnels
    const int nw = 4 * p * nw_row + 2 * K.hp;
    if (nw <= 4 * 1024) {
      K.bits_nw = nw_row;
      c->ring_bits_lds = 4 * ((size_t)nw + 2 * (size_t)K.hp * ((p + 3) / 4));
    }
  }
  c->ring_lds = (size_t)((K.ring_n + 15) & ~15) + (size_t)K.band_n + 2 * (size_t)p2 * K.wp + 2 * (size_t)K.hp * p;
  if (K.band_n > 4 * 1024 * LM_BB_BDW)
    throw std::invalid_argument("BB pass: frame size / median_filter_size exceed the ring kernel's band registers.");
  const int IW = LM_BB_TW + p2, IH = LM_BB_TH + p2;
  c->center_lds = (size_t)((IH * IW + 15) & ~15) + (size_t)LM_BB_TH * IW;
  const int hmax = std::max(vw[0].height, vw[1].height);
  {
    int cap = 16384;
    while (cap > 64 && bb_cc_layout(NC, hmax, cap).bytes > 160 * 1024) cap -= 64;
    K.run_cap = cap;
    c->cc_lds = (size_t)bb_cc_layout(NC, hmax, K.run_cap).bytes;
  }
  const size_t lds_max = 160 * 1024;
  if (c->ring_lds > lds_max || c->center_lds > lds_max || c->cc_lds > lds_max)
    throw std::invalid_argument("BB pass: frame size / median_filter_size exceed the 160 KiB LDS of one workgroup.");
  if ((int64_t)NC * std::max(vw[0].height, vw[1].height) >= (1ll << 31))
    throw std::invalid_argument("BB pass: view too large.");

  if (method != 0) {
    c->bkg.alloc((size_t)c->frame_stride);
    SET_SYNC(c->bkg.p, 0, c->bkg.n, c->stream);
    COPY_SYNC(c->bkg.p, su->background, (size_t)npix, hipMemcpyHostToDevice, c->stream);
    c->cal.alloc((size_t)NR * NC);
    COPY_SYNC(c->cal.p, su->ind_warp_mapping, sizeof(int32_t) * NR * NC, hipMemcpyHostToDevice, c->stream);
    if (method == 2) {
      c->frames.alloc((size_t)c->frame_stride * c->max_batch);
      c->luts.alloc((size_t)256 * c->max_batch);
      c->mm.alloc((size_t)2 * LM_MM_SPLIT * c->max_batch);
      c->fptr.alloc((size_t)c->max_batch);
      c->bbx.alloc((size_t)c->max_batch);
      HIPCHK(hipFuncSetAttribute((const void*)k_bb_de, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * NC));
    }
    return;
  }
  HIPCHK(hipFuncSetAttribute((const void*)k_bb_ring, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->ring_lds));
  HIPCHK(hipFuncSetAttribute((const void*)k_bb_center, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->center_lds));
  HIPCHK(hipFuncSetAttribute((const void*)k_bb_cc, hipFuncAttributeMaxDynamicSharedMemorySize, (int)c->cc_lds));

  const int B = c->max_batch;
  c->bkg.alloc((size_t)c->frame_stride);
  SET_SYNC(c->bkg.p, 0, c->bkg.n, c->stream);
  COPY_SYNC(c->bkg.p, su->background, (size_t)npix, hipMemcpyHostToDevice, c->stream);
  c->cal.alloc((size_t)NR * NC);
  COPY_SYNC(c->cal.p, su->ind_warp_mapping, sizeof(int32_t) * NR * NC, hipMemcpyHostToDevice, c->stream);
  c->frames.alloc((size_t)c->frame_stride * B);
  c->luts.alloc((size_t)256 * B);
  c->mm.alloc((size_t)2 * LM_MM_SPLIT * B);
  c->M.alloc((size_t)K.m_bytes * B);
  SET_SYNC(c->M.p, 0, c->M.n, c->stream);
  c->ring.alloc((size_t)std::max(K.ring_n, 1));
  SET_SYNC(c->ring.p, 0, c->ring.n, c->stream);  // I_median = zeros (:588)
  c->bin.alloc((size_t)K.bin_bytes * B);
  if (K.bits_nw) {
    const size_t nw = 4 * (size_t)K.p * K.bits_nw + 2 * (size_t)K.hp;
    c->bands.alloc(nw * 4 * B);
    c->rbits.alloc(nw * B);
    c->ring.alloc(nw * 4);
    SET_SYNC(c->ring.p, 0, c->ring.n, c->stream);  // I_median = zeros (:588)
  } else {
    c->bands.alloc((size_t)std::max(K.band_n, 16) * B);
    c->rbits.alloc(1);
  }
  if (dbg_env("LM_BB_PROF")) {
    c->prof.alloc(8);
    SET_SYNC(c->prof.p, 0, 8 * sizeof(unsigned long long), c->stream);
  }
  c->cc.alloc((size_t)K.cc_words * B);
  c->fptr.alloc((size_t)B);
  c->lims.alloc((size_t)8 * B);
}

// computeMouseBox's six values from the four limits of each view (:983-993)
// plus the bottom-view offset (:636).
lm_bb_frame bb_frame_values(const int32_t* l, int bottom_view_y) {
  const int32_t *ls = l, *lb = l + 4;  // {row first, row last, col first, col last}
  lm_bb_frame o;
  o.x = (lb[1] > ls[1]) ? (double)lb[1] : (double)ls[1];
  o.y_bottom = (double)lb[3];
  o.y_side = (double)ls[3];
  const unsigned wt = (unsigned)(ls[1] - ls[0]), wb = (unsigned)(lb[1] - lb[0]);
  o.width = wt > wb ? (double)wt : (double)wb;
  o.height_bottom = (double)(lb[3] - lb[2]);
  o.height_side = (double)(ls[3] - ls[2]);
  o.y_bottom += bottom_view_y;
  return o;
}

void bb_push(lm_bb_ctx* c, const uint8_t* frames, int64_t pitch, int n, bool device_frames, lm_bb_frame* out) {
  if (!frames) throw std::invalid_argument("frames is NULL");
  if (n < 1 || n > c->max_batch) throw std::invalid_argument("n must be in [1, max_batch]");
  if (pitch < c->npix) throw std::invalid_argument("frame_pitch smaller than one frame.");
  HIPCHK(hipSetDevice(c->device));
  const LmBBConst& K = c->K;
  hipStream_t s = c->stream;
  if (c->method == 1) {
    // computeMouseBox_DD: the as-executed result depends on min_pixel_visible
    // only (see lm_bb_create); the frames themselves are not read.
    lm_bb_frame o{};
    o.x = c->P.min_pixel_visible <= 0 ? (double)(K.n_cols - 1) : -1.0;  // firstLastOverT -> lims[1]
    o.y_bottom = (double)(K.n_rows - 1);
    o.y_side = 164.0;  // 165 - 1 (TM.cpp:141)
    c->last_n = n;
    for (int i = 0; i < n; ++i) {
      c->per.push_back(o);
      if (out) out[i] = o;
    }
    return;
  }
  // device frames are read in place when 16-byte aligned (k_minmax loads 16 B per lane)
  const bool direct = device_frames && ((((uintptr_t)frames | (uintptr_t)pitch) & 15) == 0);
  if (device_frames && !direct)
    HIPCHK(hipMemcpy2DAsync(c->frames.p, (size_t)c->frame_stride, frames, (size_t)pitch, (size_t)c->npix, (size_t)n,
                            hipMemcpyDeviceToDevice, s));
  for (int i = 0; i < n; ++i) {
    if (direct) {
      c->fptr.p[i] = frames + (int64_t)i * pitch;
    } else if (device_frames) {
      c->fptr.p[i] = c->frames.p + (int64_t)i * c->frame_stride;
    } else {
      uint8_t* dst = c->frames.p + (int64_t)i * c->frame_stride;
      HIPCHK(hipMemcpyAsync(dst, frames + (int64_t)i * pitch, (size_t)c->npix, hipMemcpyHostToDevice, s));
      c->fptr.p[i] = dst;
    }
  }
  const int64_t np = (int64_t)K.n_rows * K.n_cols;
  HIPCHK(launch_minmax_lut(c->fptr.d, c->bkg.p, (int)c->npix, 0, n, c->mm.p, nullptr, 0, c->luts.p, s));
  if (c->method == 2) {
    k_bb_de<<<n, 1024, 4 * K.n_cols, s>>>(K, c->fptr.d, c->bkg.p, c->cal.p, c->luts.p, c->bbx.d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    c->last_n = n;
    for (int i = 0; i < n; ++i) {
      lm_bb_frame o{};
      o.x = c->bbx.p[i];
      o.y_bottom = (double)(K.n_rows - 1);
      o.y_side = (double)(c->side_h - 1);
      c->per.push_back(o);
      if (out) out[i] = o;
    }
    return;
  }
  k_bb_ingest<<<dim3((unsigned)((np + 1023) / 1024), n), 256, 0, s>>>(K, c->fptr.d, c->bkg.p, c->cal.p, c->luts.p,
                                                                       c->M.p);
  // The ring recurrence (one workgroup) runs chunk by chunk on stream s; the
  // majority filter and components of chunk i follow on stream s2 as soon as
  // its ring is done, overlapping the ring of chunk i+1.
  static const int chunks = [] {
    const char* e = getenv("LM_BB_CHUNKS");
    return e ? std::max(1, std::min(4, atoi(e))) : 4;
  }();
  const int nch = K.p > 0 && n >= 16 ? chunks : 1;
  const int csz = (n + nch - 1) / nch;
  const dim3 cgrid((unsigned)((K.n_cols + LM_BB_TW - 1) / LM_BB_TW), (unsigned)((K.n_rows + LM_BB_TH - 1) / LM_BB_TH));
  const int nw = K.bits_nw ? 4 * K.p * K.bits_nw + 2 * K.hp : 0;
  uint32_t* bw = reinterpret_cast<uint32_t*>(c->bands.p);
  uint32_t* st = reinterpret_cast<uint32_t*>(c->ring.p);
  if (K.bits_nw) {
    k_bb_bands_bits<<<dim3((unsigned)((nw + 255) / 256), n), 256, 0, s>>>(K, c->M.p, bw);
  } else if (K.p > 0) {
    k_bb_bands<<<dim3((unsigned)((K.band_n / 4 + 255) / 256), n), 256, 0, s>>>(K, c->M.p, c->bands.p);
  }
  for (int ch = 0; ch < nch; ++ch) {
    const int f0 = ch * csz, m = std::min(csz, n - f0);
    if (m <= 0) break;
    if (K.bits_nw) {
      const uint32_t* bwc = bw + (int64_t)f0 * nw;
      uint32_t* rbc = c->rbits.p + (int64_t)f0 * nw;
      switch (K.p) {
#define LM_BB_RING_CASE(PP) \
  case PP: k_bb_ring_bits<PP><<<1, 1024, c->ring_bits_lds, s>>>(K, bwc, m, st, rbc); break;
        LM_BB_RING_CASE(1) LM_BB_RING_CASE(2) LM_BB_RING_CASE(3) LM_BB_RING_CASE(4) LM_BB_RING_CASE(5)
        LM_BB_RING_CASE(6) LM_BB_RING_CASE(7)
#undef LM_BB_RING_CASE
      }
    } else if (K.p > 0) {
      k_bb_ring<<<1, 1024, c->ring_lds, s>>>(K, c->M.p + (int64_t)f0 * K.m_bytes, c->bands.p + (int64_t)f0 * K.band_n, m,
                                             c->ring.p, c->prof.p);
    }
    HIPCHK(hipEventRecord(c->ev[ch], s));
    HIPCHK(hipStreamWaitEvent(c->s2, c->ev[ch], 0));
    k_bb_center<<<dim3(cgrid.x, cgrid.y, m), 256, c->center_lds, c->s2>>>(
        K, c->M.p + (int64_t)f0 * K.m_bytes, K.bits_nw ? c->rbits.p + (int64_t)f0 * nw : c->rbits.p,
        c->bin.p + (int64_t)f0 * K.bin_bytes);
    k_bb_cc<<<dim3(2, m), 1024, c->cc_lds, c->s2>>>(K, c->bin.p + (int64_t)f0 * K.bin_bytes,
                                                   c->cc.p + (int64_t)f0 * K.cc_words, c->lims.d + 8 * f0);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(c->s2));
  HIPCHK(hipStreamSynchronize(s));
  c->last_n = n;
  for (int i = 0; i < n; ++i) {
    const lm_bb_frame o = bb_frame_values(c->lims.p + 8 * i, c->view_y[1]);
    c->per.push_back(o);
    if (out) out[i] = o;
  }
}

// (uint32_t)double as the reference's x86-64 build evaluates it (cvttsd2si to
// 64 bits, low 32 bits kept): negative values wrap (-1.0 -> 4294967295).
uint32_t bb_u32(double d) {
  if (!(d > -9.2e18 && d < 9.2e18)) return 0;
  return (uint32_t)(uint64_t)(int64_t)d;
}

// medianvec (:1516-1533): sorts in place; the odd case returns v[N/2 - 1].
double bb_medianvec(std::vector<double>& v) {
  const int N = (int)v.size();
  if (N == 1) return v[0];
  std::sort(v.begin(), v.end());
  const int h = N / 2;
  return N % 2 == 0 ? (v[h - 1] + v[h]) / 2 : v[h - 1];
}

// stdvec (:1535-1556): sample standard deviation, accumulated in order.
double bb_stdvec(const std::vector<double>& v) {
  const int N = (int)v.size();
  if (N == 1) return 0.0;
  double sum = 0.0;
  for (double x : v) sum += x;
  const double mean = sum / N;
  double sq = 0.0;
  for (double x : v) {
    const double d = x - mean;
    sq = sq + d * d;
  }
  return std::sqrt(sq / (N - 1));
}

// vecmovingaverage (:1558-1608): centred window average, floor-rounded; the
// first N/2 and last N/2 + 1 samples are copied.
void bb_movavg(const std::vector<double>& v, std::vector<uint32_t>& out, int N) {
  const size_t n = v.size();
  out.assign(n, 0);
  if ((size_t)N >= n) {
    for (size_t i = 0; i < n; ++i) out[i] = bb_u32(v[i]);
    return;
  }
  const int h = N / 2;
  double cur = 0;
  for (int i = 0; i < h; ++i) out[i] = bb_u32(v[i]);
  for (int i = 0; i < N; ++i) cur += v[i];
  out[h] = bb_u32(std::floor(cur / N));
  for (size_t i = 0; i + N < n; ++i) {
    cur = cur - v[i] + v[i + N];
    out[h + 1 + i] = bb_u32(std::floor(cur / N));
  }
  for (size_t i = n - h - 1; i < n; ++i) out[i] = bb_u32(v[i]);
}

void bb_finish(lm_bb_ctx* c, lm_bb_result* out) {
  const size_t N = c->per.size();
  if (N == 0) throw std::invalid_argument("lm_bb_finish: no frame was pushed.");
  out->n_frames = (int32_t)N;
  out->reserved0 = 0;
  out->frames = c->per.data();
  if (c->method != 0) {  // TM.cpp:145-155, TM_DE.cpp:41-52
    std::vector<double> x(N);
    for (size_t i = 0; i < N; ++i) x[i] = c->per[i].x;
    bb_movavg(x, c->x_pos, c->P.moving_average_window);
    c->yb_pos.assign(N, (uint32_t)(c->K.n_rows - 1));
    c->ys_pos.assign(N, c->method == 1 ? 164u : (uint32_t)(c->side_h - 1));
    const int w = c->method == 1 ? c->P.bb_width : 400;
    out->bb_side_mouse = lm_rect{0, 0, w, c->method == 1 ? c->P.bb_height_side : c->side_h};
    out->bb_bottom_mouse = lm_rect{0, 0, w, c->bottom_h};
    out->x_pos = c->x_pos.data();
    out->y_bottom_pos = c->yb_pos.data();
    out->y_side_pos = c->ys_pos.data();
    return;
  }
  std::vector<double> x(N), yb(N), ys(N), w(N), hb(N), ht(N);
  for (size_t i = 0; i < N; ++i) {
    x[i] = c->per[i].x;
    yb[i] = c->per[i].y_bottom;
    ys[i] = c->per[i].y_side;
    w[i] = c->per[i].width;
    hb[i] = c->per[i].height_bottom;
    ht[i] = c->per[i].height_side;
  }
  // computeMouseBoxSize (:1481-1506)
  const double mw = bb_medianvec(w), mhb = bb_medianvec(hb), mht = bb_medianvec(ht);
  const double sw = bb_stdvec(w), shb = bb_stdvec(hb), sht = bb_stdvec(ht);
  const uint32_t w3 = bb_u32(mw + 3 * sw), hb3 = bb_u32(mhb + 3 * shb), ht3 = bb_u32(mht + 3 * sht);
  const uint32_t fw = ((double)w3 < w[N - 1]) ? w3 : bb_u32(w[N - 1]);
  const uint32_t fhb = ((double)hb3 < hb[N - 1]) ? hb3 : bb_u32(hb[N - 1]);
  const uint32_t fht = ((double)ht3 < ht[N - 1]) ? ht3 : bb_u32(ht[N - 1]);
  bb_movavg(x, c->x_pos, c->P.moving_average_window);
  bb_movavg(yb, c->yb_pos, c->P.moving_average_window);
  bb_movavg(ys, c->ys_pos, c->P.moving_average_window);
  out->n_frames = (int32_t)N;
  out->reserved0 = 0;
  out->bb_side_mouse = lm_rect{0, 0, (int32_t)fw, (int32_t)fht};
  out->bb_bottom_mouse = lm_rect{0, 0, (int32_t)fw, (int32_t)fhb};
  out->x_pos = c->x_pos.data();
  out->y_bottom_pos = c->yb_pos.data();
  out->y_side_pos = c->ys_pos.data();
  out->frames = c->per.data();
}

}  // namespace

LM_API lm_status lm_bb_create(int32_t device, const lm_setup* setup, const lm_bb_params* params, int32_t max_batch,
                              lm_bb_ctx** out) {
  if (!out) return fail(LM_ERR_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  if (max_batch <= 0) return fail(LM_ERR_INVALID_ARGUMENT, "max_batch must be > 0");
  lm_bb_ctx* c = new lm_bb_ctx();
  lm_status s = guarded([&] {
    int ndev = 0;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) throw HipError("invalid HIP device index");
    c->device = device;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->s2, hipStreamNonBlocking));
    for (hipEvent_t& e : c->ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->max_batch = max_batch;
    bb_validate_and_build(c, setup, params);
  });
  if (s != LM_OK) {
    delete c;
    return s;
  }
  *out = c;
  return LM_OK;
}

LM_API void lm_bb_destroy(lm_bb_ctx* ctx) { delete ctx; }

LM_API lm_status lm_bb_push(lm_bb_ctx* ctx, const uint8_t* frames, int64_t frame_pitch, int32_t n, lm_bb_frame* out) {
  if (!ctx) return fail(LM_ERR_INVALID_ARGUMENT, "null ctx");
  return guarded([&] { bb_push(ctx, frames, frame_pitch, n, false, out); });
}

LM_API lm_status lm_bb_push_device(lm_bb_ctx* ctx, const uint8_t* d_frames, int64_t frame_pitch, int32_t n,
                                   lm_bb_frame* out) {
  if (!ctx) return fail(LM_ERR_INVALID_ARGUMENT, "null ctx");
  return guarded([&] { bb_push(ctx, d_frames, frame_pitch, n, true, out); });
}

LM_API lm_status lm_bb_finish(lm_bb_ctx* ctx, lm_bb_result* out) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  return guarded([&] { bb_finish(ctx, out); });
}

LM_API lm_status lm_bb_debug_binary(lm_bb_ctx* ctx, int32_t f, uint8_t* out, int32_t rows, int32_t cols) {
  if (!ctx || !out) return fail(LM_ERR_INVALID_ARGUMENT, "null argument");
  if (ctx->method != 0) return fail(LM_ERR_INVALID_ARGUMENT, "debug binary images exist for method 0 only");
  if (f < 0 || f >= ctx->last_n) return fail(LM_ERR_INVALID_ARGUMENT, "index out of range");
  if (rows != ctx->K.n_rows || cols != ctx->K.n_cols) return fail(LM_ERR_INVALID_ARGUMENT, "shape mismatch");
  return guarded([&] {
    HIPCHK(hipSetDevice(ctx->device));
    COPY_SYNC(out, ctx->bin.p + (int64_t)f * ctx->K.bin_bytes, (size_t)rows * cols, hipMemcpyDeviceToHost, ctx->stream);
  });
}

LM_API void* lm_bb_stream(lm_bb_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }
