// lm_kernels.hip — gfx950 kernels of the LocoMouse per-frame detection path.
//
// Batch pipeline (one launch each, grid over frame slots; see lm_device.h):
//   k_minmax_lut  per-frame min/max of sat(F - BKG) -> normalize LUT (+ TM imadjust)
//                 LocoMouse_class.cpp:1304-1310, TM.cpp:247, :3204-3242
//   k_ingest      calibration gather + flip + LUT -> extended padded crops (u8)
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

#include <utility>

#include "lm_device.h"
#include "lm_introsort.h"

#define DEV __device__ __forceinline__

// ------------------------------------------------------------------ helpers

DEV uint8_t ipad_pixel(const uint8_t* __restrict__ F, const uint8_t* __restrict__ bkg,
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

DEV float wave_min_u32(unsigned v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, (unsigned)__shfl_xor((int)v, o));
  return v;
}

// ------------------------------------------------------------ k_minmax_lut
// One 1024-thread block per frame slot.  16-byte loads of frame and
// background; the per-frame LUT folds normalize(NORM_MINMAX) -> convertTo
// (sat_u8(cvRound((float)p*(float)scale + (float)shift)), OpenCV 3.x) and the
// LocoMouse_TM imadjust LUT.
__global__ __launch_bounds__(1024) void k_minmax_lut(const uint8_t* const* __restrict__ frame_ptr,
                                                     const uint8_t* __restrict__ bkg, int npix, int s0,
                                                     const uint8_t* __restrict__ adj, int use_adj,
                                                     uint8_t* __restrict__ luts) {
  const int slot = s0 + blockIdx.x;
  const uint8_t* __restrict__ F = frame_ptr[slot];
  unsigned mn = 255, mx = 0;
  const int nvec = npix >> 4;
  const uint4* F4 = reinterpret_cast<const uint4*>(F);
  const uint4* B4 = reinterpret_cast<const uint4*>(bkg);
  for (int i = threadIdx.x; i < nvec; i += blockDim.x) {
    uint4 f = F4[i];
    uint4 b = B4[i];
    unsigned fw[4] = {f.x, f.y, f.z, f.w}, bw[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        unsigned fv = (fw[q] >> (8 * k)) & 255u, bv = (bw[q] >> (8 * k)) & 255u;
        unsigned d = fv > bv ? fv - bv : 0u;
        mn = min(mn, d);
        mx = max(mx, d);
      }
    }
  }
  for (int i = (nvec << 4) + threadIdx.x; i < npix; i += blockDim.x) {
    unsigned fv = F[i], bv = bkg[i];
    unsigned d = fv > bv ? fv - bv : 0u;
    mn = min(mn, d);
    mx = max(mx, d);
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, (unsigned)__shfl_xor((int)mn, o));
    mx = max(mx, (unsigned)__shfl_xor((int)mx, o));
  }
  __shared__ unsigned smn[16], smx[16];
  const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) {
    smn[wid] = mn;
    smx[wid] = mx;
  }
  __syncthreads();
  if (threadIdx.x < 256) {
    unsigned a = 255, b = 0;
    const int nw = blockDim.x >> 6;
    for (int w = 0; w < nw; ++w) {
      a = min(a, smn[w]);
      b = max(b, smx[w]);
    }
    const double smin = (double)a, smax = (double)b, dmin = 0.0, dmax = 255.0;
    const double scale = (dmax - dmin) * (smax - smin > 2.220446049250313e-16 ? 1. / (smax - smin) : 0.0);
    const double shift = dmin - smin * scale;
    const int p = threadIdx.x;
    int v;
    if (fabs(scale - 1.0) < 2.220446049250313e-16 && fabs(shift) < 2.220446049250313e-16) {
      v = p;  // convertTo noScale -> copy
    } else {
      const float sf = (float)scale, hf = (float)shift;
      float t = __fmul_rn((float)p, sf);
      t = __fadd_rn(t, hf);
      int iv = (int)rintf(t);
      v = iv < 0 ? 0 : (iv > 255 ? 255 : iv);
    }
    if (use_adj) v = adj[v];
    luts[slot * 256 + p] = (uint8_t)v;
  }
}

// ---------------------------------------------------------------- k_ingest
// Builds the extended padded crops of both views for each slot: every I_PAD
// pixel any detector tap reads.  Each thread writes 4 consecutive bytes.
__global__ __launch_bounds__(256) void k_ingest(const LmConst* __restrict__ Kp, const uint8_t* const* __restrict__ frame_ptr,
                                                const uint8_t* __restrict__ bkg, const int32_t* __restrict__ cal,
                                                const uint8_t* __restrict__ luts, const LmSlot* __restrict__ slots,
                                                int s0, uint8_t* __restrict__ ext, int64_t ext_slot_bytes) {
  const LmConst& K = *Kp;
  const int slot = s0 + blockIdx.y;
  __shared__ uint8_t lut[256];
  lut[threadIdx.x] = luts[slot * 256 + threadIdx.x];
  __syncthreads();
  const uint8_t* __restrict__ F = frame_ptr[slot];
  const int64_t e0 = (int64_t)K.ext_h[0] * K.ext_w[0];
  const int64_t etot = e0 + (int64_t)K.ext_h[1] * K.ext_w[1];
  const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (q >= etot) return;
  const int v = q < e0 ? 0 : 1;
  const int64_t qq = v == 0 ? q : q - e0;
  const int er = (int)(qq / K.ext_w[v]);
  const int ec = (int)(qq % K.ext_w[v]);  // multiple of 4 (ext_w % 16 == 0)
  const LmSlot sl = slots[slot];
  const int R = sl.crop_y[v] + K.ext_oy[v] + er;
  const int C0 = sl.crop_x[v] + K.ext_ox[v] + ec;
  uint32_t word = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) word |= (uint32_t)ipad_pixel(F, bkg, cal, lut, K, R, C0 + k) << (8 * k);
  *reinterpret_cast<uint32_t*>(ext + (int64_t)slot * ext_slot_bytes + q) = word;
}

// ---------------------------------------------------------------- k_ingest_fb
// k_ingest for LM_INGEST_FB consecutive slots per thread: the calibration
// index and background byte of a crop pixel are loaded once and reused for
// every slot whose crop sits at the same place (always, with a provided
// bounding box); only the frame gather and the per-frame LUT are per slot.
#define LM_INGEST_FB 8
__global__ __launch_bounds__(256) void k_ingest_fb(const LmConst* __restrict__ Kp, const uint8_t* const* __restrict__ frame_ptr,
                                                   const uint8_t* __restrict__ bkg, const int32_t* __restrict__ cal,
                                                   const uint8_t* __restrict__ luts, const LmSlot* __restrict__ slots,
                                                   int s0, int s_end, int fb, uint8_t* __restrict__ ext,
                                                   int64_t ext_slot_bytes) {
  const LmConst& K = *Kp;
  const int sb = s0 + blockIdx.y * fb;
  const int nf = min(fb, s_end - sb);
  __shared__ uint8_t lut[LM_INGEST_FB][256];
  for (int i = threadIdx.x; i < nf * 256; i += blockDim.x) lut[i >> 8][i & 255] = luts[(sb + (i >> 8)) * 256 + (i & 255)];
  __syncthreads();
  const int64_t e0 = (int64_t)K.ext_h[0] * K.ext_w[0];
  const int64_t etot = e0 + (int64_t)K.ext_h[1] * K.ext_w[1];
  const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (q >= etot) return;
  const int v = q < e0 ? 0 : 1;
  const int64_t qq = v == 0 ? q : q - e0;
  const int er = (int)(qq / K.ext_w[v]);
  const int ec = (int)(qq % K.ext_w[v]);  // multiple of 4 (ext_w % 16 == 0)
  int idx[4] = {-1, -1, -1, -1}, bv[4] = {0, 0, 0, 0};  // defined before the first crop test
  int px = INT32_MIN, py = INT32_MIN;
  for (int f = 0; f < nf; ++f) {
    const int slot = sb + f;
    const LmSlot sl = slots[slot];
    if (sl.crop_x[v] != px || sl.crop_y[v] != py) {  // crop moved: recompute the gather indices
      px = sl.crop_x[v];
      py = sl.crop_y[v];
      const int R = py + K.ext_oy[v] + er - K.pad_pre_rows;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        int c = px + K.ext_ox[v] + ec + k - K.pad_pre_cols;
        if (R < 0 || R >= K.n_rows || c < 0 || c >= K.n_cols) {
          idx[k] = -1;
        } else {
          if (K.flip) c = K.n_cols - 1 - c;
          idx[k] = cal[R * K.n_cols + c];
          bv[k] = bkg[idx[k]];
        }
      }
    }
    const uint8_t* __restrict__ F = frame_ptr[slot];
    uint32_t word = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (idx[k] >= 0) {
        const int fv = F[idx[k]];
        word |= (uint32_t)lut[f][fv > bv[k] ? fv - bv[k] : 0] << (8 * k);
      }
    }
    *reinterpret_cast<uint32_t*>(ext + (int64_t)slot * ext_slot_bytes + q) = word;
  }
}

// ------------------------------------------------------------------ k_corr
// One block = one 80x48 output tile of one detector of one slot; 256 threads
// as 16x16, each LM_R rows x LM_C columns.  The input tile is staged in LDS as
// float.  For every output the taps are accumulated as
//     acc = (float)(-rho);  for i in rows, j in cols: acc = fmaf(w[i][j], I, acc)
// i.e. exactly cv::filter2D's row-major chain (zero-padded taps add +0).
// Pixel rows are walked once per thread (t = r + i), so a loaded row feeds all
// LM_R accumulator rows; weights are wave-uniform scalar loads.
#define LM_MAXK 64

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
                       int* s_base) {
  static_assert(R_ * C_ <= 32, "bitmask");
  const int my = D.m_y - D.in_y, mx = D.m_x - D.in_x;  // I_*_MOUSE pixel inside the LDS tile
  if (D.kind != 0) {
    uint8_t* __restrict__ tb = tailbin + (int64_t)slot * tailbin_slot_bytes + (D.list ? (int64_t)K.tail_hb * K.tail_w : 0);
#pragma unroll
    for (int r = 0; r < R_; ++r)
#pragma unroll
      for (int c = 0; c < C_; ++c) {
        const int y = oy0 + ly * R_ + r, x = ox0 + lx * C_ + c;
        if (y < D.oh && x < D.ow) tb[(int64_t)y * D.ow + x] = acc[r][c] > 0.0f ? 1 : 0;
      }
    return;
  }
  unsigned bits = 0;
#pragma unroll
  for (int r = 0; r < R_; ++r)
#pragma unroll
    for (int c = 0; c < C_; ++c) {
      const int y = oy0 + ly * R_ + r, x = ox0 + lx * C_ + c;
      const float pix = lds[(ly * R_ + r + my) * stride + lx * C_ + c + mx];
      if (y < D.oh && x < D.ow && pix > 25.0f && acc[r][c] > 0.0f) bits |= 1u << (r * C_ + c);
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

// LDS row stride of the packed kernel: == 4 (mod 8) so the two 16-lane row
// groups of a ds_read2_b32 (4 rows apart) hit disjoint bank halves.
__host__ __device__ inline int pk_stride(int cols) { return cols + ((4 - (cols & 7)) + 8) % 8; }

struct LmDetGroup {
  int32_t n;
  int32_t ids[LM_NDET];
  int32_t tile_end[LM_NDET];  // cumulative tile counts
  int32_t skip_taps;          // diagnostics (LM_CORR_SKIP=1): no FMAs, fill + epilogue only
};

__global__ __launch_bounds__(256) void k_corr(const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext,
                                              int64_t ext_slot_bytes, const float* __restrict__ weights, int s0,
                                              unsigned long long* __restrict__ keys, int32_t* __restrict__ n_pos,
                                              uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes) {
  const LmConst& K = *Kp;
  extern __shared__ float lds[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - tb;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1, cols = LM_TW + D.kwp - 1;
  int stride = cols;
  stride += (16 - (stride & 31) + 32) & 31;  // stride == 16 (mod 32): conflict-free row pairs
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  // stage: 4 bytes per thread-iteration (columns padded to a multiple of 4)
  const int cols4 = (cols + 3) >> 2;
  for (int e = threadIdx.x; e < rows * cols4; e += 256) {
    const int r = e / cols4, c4 = (e - r * cols4) << 2;
    const uint8_t* p = src + (int64_t)r * ew + c4;
    float* o = lds + r * stride + c4;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c4 + k < stride) o[k] = (float)p[k];
  }
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int ly = threadIdx.x >> 4, lx = threadIdx.x & 15;
  float acc[LM_R][LM_C];
#pragma unroll
  for (int r = 0; r < LM_R; ++r)
#pragma unroll
    for (int c = 0; c < LM_C; ++c) acc[r][c] = D.delta;
  const float* __restrict__ W = weights + D.w_off;
  const int kh = D.kh, kwp = D.kwp;
  for (int t = 0; t < LM_R + kh - 1; ++t) {
    const float* prow = lds + (ly * LM_R + t) * stride + lx * LM_C;
    for (int jc = 0; jc < kwp; jc += LM_JC) {
      float px[LM_C + LM_JC - 1];
#pragma unroll
      for (int q = 0; q < LM_C + LM_JC - 1; ++q) px[q] = prow[jc + q];
#pragma unroll
      for (int r = 0; r < LM_R; ++r) {
        const int i = t - r;
        if (i >= 0 && i < kh) {
          const float* wr = W + i * kwp + jc;
#pragma unroll
          for (int j = 0; j < LM_JC; ++j) {
            const float w = wr[j];
#pragma unroll
            for (int c = 0; c < LM_C; ++c) acc[r][c] = __builtin_fmaf(w, px[c + j], acc[r][c]);
          }
        }
      }
    }
  }

  corr_epilogue<LM_R, LM_C>(K, D, acc, lds, stride, ly, lx, oy0, ox0, slot, keys, n_pos, tailbin, tailbin_slot_bytes, &s_cnt, &s_base);
}

// k_corr_kw: k_corr specialised on the detector width KW (a weight row is
// fully unrolled: one scalar-load wait per detector row instead of one per
// 4 taps).  One launch covers the detectors of one width (ids in G).

template <int KW>
__global__ __launch_bounds__(256) void k_corr_kw(const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext,
                                                 int64_t ext_slot_bytes, const float* __restrict__ weights, int s0,
                                                 unsigned long long* __restrict__ keys, int32_t* __restrict__ n_pos,
                                                 uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes) {
  const LmConst& K = *Kp;
  extern __shared__ float lds[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - tb;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1, cols = LM_TW + KW - 1;
  int stride = cols;
  stride += (16 - (stride & 31) + 32) & 31;
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  const int cols4 = (cols + 3) >> 2;
  for (int e = threadIdx.x; e < rows * cols4; e += 256) {
    const int r = e / cols4, c4 = (e - r * cols4) << 2;
    const uint8_t* p = src + (int64_t)r * ew + c4;
    float* o = lds + r * stride + c4;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c4 + k < stride) o[k] = (float)p[k];
  }
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int ly = threadIdx.x >> 4, lx = threadIdx.x & 15;
  float acc[LM_R][LM_C];
#pragma unroll
  for (int r = 0; r < LM_R; ++r)
#pragma unroll
    for (int c = 0; c < LM_C; ++c) acc[r][c] = D.delta;
  const float* __restrict__ W = weights + D.w_off;
  const int kh = D.kh, kwp = D.kwp;
  for (int t = 0; t < LM_R + kh - 1; ++t) {
    const float* prow = lds + (ly * LM_R + t) * stride + lx * LM_C;
    float px[LM_C + KW - 1];
#pragma unroll
    for (int q = 0; q < LM_C + KW - 1; ++q) px[q] = prow[q];
#pragma unroll
    for (int r = 0; r < LM_R; ++r) {
      const int i = t - r;
      if (i >= 0 && i < kh) {
        const float* wr = W + i * kwp;
#pragma unroll
        for (int j = 0; j < KW; ++j) {
          const float w = wr[j];
#pragma unroll
          for (int c = 0; c < LM_C; ++c) acc[r][c] = __builtin_fmaf(w, px[c + j], acc[r][c]);
        }
      }
    }
  }

  corr_epilogue<LM_R, LM_C>(K, D, acc, lds, stride, ly, lx, oy0, ox0, slot, keys, n_pos, tailbin, tailbin_slot_bytes, &s_cnt, &s_base);
}

// k_corr_pk: packed-FP32 correlation.  gfx950 issues one v_fma_f32 (wave64)
// per 4 cycles per SIMD; v_pk_fma_f32 does two FMAs per lane in the same slot.
// Each accumulator pair holds two vertically adjacent outputs (rows 2p, 2p+1)
// of one column: for tap (i, j) both use weight w[i][j] (SGPR, broadcast) and
// pixels (t, t+1) of one column, which one ds_read2_b32 loads into an aligned
// register pair.  Every output still accumulates its taps in row-major order
// with single-rounding FMAs, so results are bit-identical to k_corr.
// 192 threads as 16 (x) x 12 (y), each 5 columns x 4 rows: the 80x48 tile.
#define PK_C 5
#define PK_R 4
#define PK_TY 12

typedef float lm_f2 __attribute__((ext_vector_type(2)));

// Pixel pairs (row t, row t+1) of one column straight into an aligned VGPR
// pair: ds_read2_b32 with offset1 = offset0 + STRIDE (dwords).  At most 15
// LDS reads in flight (lgkmcnt is 4 bits); one wait at the end.
constexpr int pk_stride_c(int cols) { return cols + ((4 - (cols & 7)) + 8) % 8; }

template <int STRIDE, int Q>
DEV void lds_pair(lm_f2& dst, unsigned base) {
  static_assert(Q + STRIDE <= 255, "ds_read2_b32 offset range");
  if constexpr (Q >= 15) asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory");
  asm volatile("ds_read2_b32 %0, %1 offset0:%2 offset1:%3" : "=v"(dst) : "v"(base), "i"(Q), "i"(Q + STRIDE) : "memory");
}

template <int STRIDE, int N, int... Qs>
DEV void lds_pairs_impl(lm_f2 (&px)[N], unsigned base, std::integer_sequence<int, Qs...>) {
  (lds_pair<STRIDE, Qs>(px[Qs], base), ...);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int STRIDE, int N>
DEV void lds_pairs(lm_f2 (&px)[N], unsigned base) {
  lds_pairs_impl<STRIDE, N>(px, base, std::make_integer_sequence<int, N>{});
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
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if (c0 + k >= 0 && c0 + k < cols) o[k] = (float)((w[k >> 2] >> (8 * (k & 3))) & 0xFFu);
      }
    }
  }
}

template <int KW, bool WLDS, bool ASMLD = false>
__global__ __launch_bounds__(192) void k_corr_pk(const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext,
                                                 int64_t ext_slot_bytes, const float* __restrict__ weights, int s0,
                                                 unsigned long long* __restrict__ keys, int32_t* __restrict__ n_pos,
                                                 uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes) {
  const LmConst& K = *Kp;
  // WLDS: detector weights staged in LDS (broadcast reads) instead of scalar
  // loads, so every lgkm wait is an in-order LDS wait the compiler can count.
  extern __shared__ float lds[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - tb;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1, cols = LM_TW + KW - 1;
  const int stride = pk_stride(cols);
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  tile_fill_f32(lds, stride, src, ew, rows, cols);
  float* wl = lds + ((rows * stride + 3) & ~3);
  if (WLDS)
    for (int e = threadIdx.x; e < D.kh * D.kwp; e += blockDim.x) wl[e] = weights[D.w_off + e];
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int ly = threadIdx.x >> 4, lx = threadIdx.x & 15;
  lm_f2 acc[PK_R / 2][PK_C];
#pragma unroll
  for (int p = 0; p < PK_R / 2; ++p)
#pragma unroll
    for (int c = 0; c < PK_C; ++c) acc[p][c] = (lm_f2){D.delta, D.delta};
  const float* __restrict__ W = weights + D.w_off;
  const int kh = D.kh, kwp = D.kwp;
  const int tend = (G.skip_taps & 1) ? 0 : kh + PK_R - 2;
  lm_f2 px[PK_C + KW - 1];
  for (int t = 0; t < tend; ++t) {
    const float* p0 = lds + (ly * PK_R + t) * stride + lx * PK_C;
    if ((G.skip_taps & 4) && t > 0) {
      // diagnostics: pixel pairs of row 0 reused (no LDS traffic in the loop)
    } else if constexpr (ASMLD) {
      constexpr int STR = pk_stride_c(LM_TW + KW - 1);
      const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)p0;
      lds_pairs<STR, PK_C + KW - 1>(px, base);
    } else {
#pragma unroll
      for (int q = 0; q < PK_C + KW - 1; ++q) px[q] = (lm_f2){p0[q], p0[q + stride]};
    }
#pragma unroll
    for (int p = 0; p < PK_R / 2; ++p) {
      const int i = t - 2 * p;
      if (i >= 0 && i < kh) {
        const float* wr = (WLDS ? wl : W) + ((G.skip_taps & 2) ? 0 : i * kwp);
#pragma unroll
        for (int j = 0; j < KW; ++j) {
          const float w = wr[j];
          const lm_f2 w2 = (lm_f2){w, w};
#pragma unroll
          for (int c = 0; c < PK_C; ++c) acc[p][c] = __builtin_elementwise_fma(w2, px[c + j], acc[p][c]);
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
  corr_epilogue<PK_R, PK_C>(K, D, accf, lds, stride, ly, lx, oy0, ox0, slot, keys, n_pos, tailbin, tailbin_slot_bytes,
                            &s_cnt, &s_base);
}

// k_corr_p2: one row-pair per thread, 10 columns wide (192 threads as 8 x 24:
// the same 80x48 tile).  Per input row-pair t only kernel row i = t is
// needed, so the next row's weights are prefetched into SGPRs one iteration
// ahead and the FMA block never waits on a scalar load.  LDS traffic: (KW+9)
// ds_read2 per 10*KW packed FMAs.
#define P2_C 10

template <int KW>
__global__ __launch_bounds__(192) void k_corr_p2(const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext,
                                                 int64_t ext_slot_bytes, const float* __restrict__ weights, int s0,
                                                 unsigned long long* __restrict__ keys, int32_t* __restrict__ n_pos,
                                                 uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes) {
  const LmConst& K = *Kp;
  extern __shared__ float lds[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - tb;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1, cols = LM_TW + KW - 1;
  const int stride = pk_stride(cols);
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  const int cols4 = (cols + 3) >> 2;
  for (int e = threadIdx.x; e < rows * cols4; e += blockDim.x) {
    const int r = e / cols4, c4 = (e - r * cols4) << 2;
    const uint8_t* p = src + (int64_t)r * ew + c4;
    float* o = lds + r * stride + c4;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c4 + k < stride) o[k] = (float)p[k];
  }
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int ly = threadIdx.x >> 3, lx = threadIdx.x & 7;
  lm_f2 acc[P2_C];
#pragma unroll
  for (int c = 0; c < P2_C; ++c) acc[c] = (lm_f2){D.delta, D.delta};
  const float* __restrict__ W = weights + D.w_off;
  const int kh = D.kh, kwp = D.kwp;
  float wc[KW];
#pragma unroll
  for (int j = 0; j < KW; ++j) wc[j] = W[j];
  constexpr int STR = pk_stride_c(LM_TW + KW - 1);
  for (int t = 0; t < kh; ++t) {
    const float* p0 = lds + (ly * 2 + t) * stride + lx * P2_C;
    lm_f2 px[P2_C + KW - 1];
    const unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)p0;
    lds_pairs<STR, P2_C + KW - 1>(px, base);
    const float* wnr = W + min(t + 1, kh - 1) * kwp;
    float wn[KW];
#pragma unroll
    for (int j = 0; j < KW; ++j) wn[j] = wnr[j];
    __builtin_amdgcn_sched_barrier(0);  // scalar loads of row t+1 issue before the FMAs of row t
#pragma unroll
    for (int j = 0; j < KW; ++j) {
      const lm_f2 w2 = (lm_f2){wc[j], wc[j]};
#pragma unroll
      for (int c = 0; c < P2_C; ++c) acc[c] = __builtin_elementwise_fma(w2, px[c + j], acc[c]);
    }
#pragma unroll
    for (int j = 0; j < KW; ++j) wc[j] = wn[j];
  }
  float accf[2][P2_C];
#pragma unroll
  for (int c = 0; c < P2_C; ++c) {
    accf[0][c] = acc[c].x;
    accf[1][c] = acc[c].y;
  }
  corr_epilogue<2, P2_C>(K, D, accf, lds, stride, ly, lx, oy0, ox0, slot, keys, n_pos, tailbin, tailbin_slot_bytes,
                         &s_cnt, &s_base);
}

// k_corr_db: k_corr_p2's shape with the LDS loads double-buffered.  Two
// pixel-pair buffers: while the FMAs of row-pair t run on one, the ds_read2
// loads of row-pair t+1 fill the other, so a wave waits on LDS only when its
// loads have not landed after a whole row of FMAs.  The detector weights of
// both rows of an iteration are scalar-loaded first and consumed by an empty
// asm statement, so the compiler's own lgkmcnt(0) for them comes before the
// pixel loads are issued and never drains the pixel queue.
template <int STRIDE, int... Qs>
DEV void db_issue(lm_f2 (&px)[sizeof...(Qs)], unsigned base, std::integer_sequence<int, Qs...>) {
  (lds_pair<STRIDE, Qs>(px[Qs], base), ...);
}

DEV void db_use_sgpr(float w) { asm volatile("; weight %0" ::"s"(w)); }

template <int N>
DEV void db_use_sgprs(const float (&w)[N]) {
#pragma unroll
  for (int i = 0; i < N; ++i) db_use_sgpr(w[i]);
}

template <int KW>
DEV void db_fma(lm_f2 (&acc)[P2_C], const lm_f2 (&px)[P2_C + KW - 1], const float (&w)[KW]) {
#pragma unroll
  for (int j = 0; j < KW; ++j) {
    const lm_f2 w2 = (lm_f2){w[j], w[j]};
#pragma unroll
    for (int c = 0; c < P2_C; ++c) acc[c] = __builtin_elementwise_fma(w2, px[c + j], acc[c]);
  }
}

template <int KW>
__global__ __launch_bounds__(192, 2) void k_corr_db(const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext,
                                                    int64_t ext_slot_bytes, const float* __restrict__ weights, int s0,
                                                    unsigned long long* __restrict__ keys, int32_t* __restrict__ n_pos,
                                                    uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes) {
  const LmConst& K = *Kp;
  constexpr int NQ = P2_C + KW - 1;
  constexpr int STR = pk_stride_c(LM_TW + KW - 1);
  extern __shared__ float lds[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - tb;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1, cols = LM_TW + KW - 1;
  const int stride = pk_stride(cols);
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  const int cols4 = (cols + 3) >> 2;
  for (int e = threadIdx.x; e < rows * cols4; e += blockDim.x) {
    const int r = e / cols4, c4 = (e - r * cols4) << 2;
    const uint8_t* p = src + (int64_t)r * ew + c4;
    float* o = lds + r * stride + c4;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c4 + k < stride) o[k] = (float)p[k];
  }
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int ly = threadIdx.x >> 3, lx = threadIdx.x & 7;
  lm_f2 acc[P2_C];
#pragma unroll
  for (int c = 0; c < P2_C; ++c) acc[c] = (lm_f2){D.delta, D.delta};
  const float* __restrict__ W = weights + D.w_off;
  const int kh = D.kh, kwp = D.kwp;
  const unsigned base0 =
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(lds + (ly * 2) * stride + lx * P2_C);
  const unsigned rstep = (unsigned)stride * 4u;
  lm_f2 pa[NQ], pb[NQ];
  db_issue<STR>(pa, base0, std::make_integer_sequence<int, NQ>{});
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  for (int t = 0; t < kh; t += 2) {
    const bool two = t + 1 < kh;
    float wa[KW], wb[KW];
#pragma unroll
    for (int j = 0; j < KW; ++j) wa[j] = W[t * kwp + j];
#pragma unroll
    for (int j = 0; j < KW; ++j) wb[j] = W[(two ? t + 1 : t) * kwp + j];
    db_use_sgprs<KW>(wa);  // the compiler's wait for the scalar loads lands here
    db_use_sgprs<KW>(wb);
    __builtin_amdgcn_sched_barrier(0);
    if (two) db_issue<STR>(pb, base0 + (unsigned)(t + 1) * rstep, std::make_integer_sequence<int, NQ>{});
    __builtin_amdgcn_sched_barrier(0);
    db_fma<KW>(acc, pa, wa);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (!two) break;
    if (t + 2 < kh) db_issue<STR>(pa, base0 + (unsigned)(t + 2) * rstep, std::make_integer_sequence<int, NQ>{});
    __builtin_amdgcn_sched_barrier(0);
    db_fma<KW>(acc, pb, wb);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
  float accf[2][P2_C];
#pragma unroll
  for (int c = 0; c < P2_C; ++c) {
    accf[0][c] = acc[c].x;
    accf[1][c] = acc[c].y;
  }
  corr_epilogue<2, P2_C>(K, D, accf, lds, stride, ly, lx, oy0, ox0, slot, keys, n_pos, tailbin, tailbin_slot_bytes,
                         &s_cnt, &s_base);
}

// k_corr_sp: software-pipelined packed correlation.  Thread shape of k_corr_p2
// (one row pair x 10 columns; 192 threads = 8 x 24 cover the 80x48 tile), one
// detector row per iteration t.  The loads for row pair t+1 are spread over
// row t's FMA stream: pixel pair q is dead once FMA block j = q is done
// (blocks run j = 0..KW-1 and block j reads pairs j..j+9), so its ds_read2 for
// t+1 is issued right after that block, into the same registers; the 9 pairs
// q >= KW follow the last block.  Row t+1's weights are scalar-loaded at the
// top of iteration t.  A wave therefore waits on LDS only for the last 9
// loads and never on the weights, instead of draining every load and scalar
// load before its FMAs (k_corr_pk / k_corr_p2).  Same fmaf chain per output
// (taps in row-major order from delta), so the scores stay bit-exact.
template <int STRIDE, int Q>
DEV void sp_load(lm_f2& dst, unsigned base) {
  static_assert(Q + STRIDE <= 255, "ds_read2_b32 offset range");
  asm volatile("s_waitcnt lgkmcnt(12)\n\tds_read2_b32 %0, %1 offset0:%2 offset1:%3"
               : "=v"(dst)
               : "v"(base), "i"(Q), "i"(Q + STRIDE)
               : "memory");
}

template <int KW, int STRIDE, int... Qs>
DEV void sp_tail(lm_f2 (&px)[P2_C + KW - 1], unsigned nbase, std::integer_sequence<int, Qs...>) {
  (sp_load<STRIDE, KW + Qs>(px[KW + Qs], nbase), ...);
}

template <int KW, int STRIDE, int J>
DEV void sp_block(lm_f2 (&acc)[P2_C], lm_f2 (&px)[P2_C + KW - 1], const float (&w)[KW], unsigned nbase) {
  const lm_f2 w2 = (lm_f2){w[J], w[J]};
#pragma unroll
  for (int c = 0; c < P2_C; ++c) acc[c] = __builtin_elementwise_fma(w2, px[c + J], acc[c]);
  __builtin_amdgcn_sched_barrier(0);
  sp_load<STRIDE, J>(px[J], nbase);  // pair J is dead for row t: refill it for row t+1
  if constexpr (J == KW - 1) sp_tail<KW, STRIDE>(px, nbase, std::make_integer_sequence<int, P2_C - 1>{});
  __builtin_amdgcn_sched_barrier(0);
}

template <int KW, int STRIDE, int... Js>
DEV void sp_row(lm_f2 (&acc)[P2_C], lm_f2 (&px)[P2_C + KW - 1], const float (&w)[KW], unsigned nbase,
                std::integer_sequence<int, Js...>) {
  (sp_block<KW, STRIDE, Js>(acc, px, w, nbase), ...);
}

template <int KW>
__global__ __launch_bounds__(192) void k_corr_sp(const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext,
                                                 int64_t ext_slot_bytes, const float* __restrict__ weights, int s0,
                                                 unsigned long long* __restrict__ keys, int32_t* __restrict__ n_pos,
                                                 uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes) {
  const LmConst& K = *Kp;
  constexpr int NQ = P2_C + KW - 1;
  constexpr int STR = pk_stride_c(LM_TW + KW - 1);
  extern __shared__ float lds[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - tb;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1, cols = LM_TW + KW - 1;
  const int stride = STR;
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  const int cols4 = (cols + 3) >> 2;
  for (int e = threadIdx.x; e < rows * cols4; e += blockDim.x) {
    const int r = e / cols4, c4 = (e - r * cols4) << 2;
    const uint8_t* p = src + (int64_t)r * ew + c4;
    float* o = lds + r * stride + c4;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c4 + k < stride) o[k] = (float)p[k];
  }
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int ly = threadIdx.x >> 3, lx = threadIdx.x & 7;
  lm_f2 acc[P2_C];
#pragma unroll
  for (int c = 0; c < P2_C; ++c) acc[c] = (lm_f2){D.delta, D.delta};
  const float* __restrict__ W = weights + D.w_off;
  const int kh = D.kh, kwp = D.kwp;
  unsigned base =
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(lds + (ly * 2) * stride + lx * P2_C);
  const unsigned rstep = (unsigned)stride * 4u;
  lm_f2 px[NQ];
  lds_pairs<STR, NQ>(px, base);  // row pair 0 (waits)
  float wc[KW];
#pragma unroll
  for (int j = 0; j < KW; ++j) wc[j] = W[j];
  for (int t = 0; t < kh; ++t) {
    // the last iteration loads a (dead) row pair kh: the LDS tile has 2 spare rows
    const float* wnr = W + min(t + 1, kh - 1) * kwp;
    float wn[KW];
#pragma unroll
    for (int j = 0; j < KW; ++j) wn[j] = wnr[j];
    __builtin_amdgcn_sched_barrier(0);  // row t+1's scalar loads issue before row t's FMAs
    base += rstep;
    sp_row<KW, STR>(acc, px, wc, base, std::make_integer_sequence<int, KW>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // row t+1's pairs (and weights) have landed
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < KW; ++j) wc[j] = wn[j];
  }
  float accf[2][P2_C];
#pragma unroll
  for (int c = 0; c < P2_C; ++c) {
    accf[0][c] = acc[c].x;
    accf[1][c] = acc[c].y;
  }
  corr_epilogue<2, P2_C>(K, D, accf, lds, stride, ly, lx, oy0, ox0, slot, keys, n_pos, tailbin, tailbin_slot_bytes,
                         &s_cnt, &s_base);
}

// k_corr_cb: column-block pairs.  A packed accumulator holds outputs
// (y, x) and (y, x + 40) of an 80 x 48 tile, so the two operands of every
// v_pk_fma_f32 are pixels 40 columns apart in the same row.  The tile is kept
// in LDS as float pairs LP[r][c] = (I[r][c], I[r][c + 40]), so each operand
// pair is one ds_read_b64 (2 LDS cycles per wave, 256 B/clk) where the
// row-pair kernels need a ds_read2_b32 (4 cycles, 128 B/clk): half the LDS
// time for the same FMA count.  Thread (lx, ly), 8 x 24 threads: outputs
// rows 2ly + {0, 1}, columns 5lx + {0..4} and 40 + 5lx + {0..4}.  Input row
// T = 2ly + t feeds output row r through detector row i = t - r, so each
// iteration uses weight rows t and t - 1.  Same fmaf chain per output (taps in
// row-major order from delta): bit-exact with the reference restatement.
#define CB_C 5
#define CB_H 40
constexpr int cb_stride_c(int kw) {  // pairs per LDS row: >= 40 + kw - 1 and == 4 or 12 (mod 16)
  int s = CB_H + kw - 1;
  while ((s & 7) != 4) ++s;
  return s;
}

template <int Q>
DEV void cb_load(lm_f2& dst, unsigned base) {
  if constexpr (Q >= 15) asm volatile("s_waitcnt lgkmcnt(14)" ::: "memory");
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(Q * 8) : "memory");
}

template <int N, int... Qs>
DEV void cb_loads_impl(lm_f2 (&px)[N], unsigned base, std::integer_sequence<int, Qs...>) {
  (cb_load<Qs>(px[Qs], base), ...);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int KW, bool WLDS = false>
__global__ __launch_bounds__(192) void k_corr_cb(const LmConst* __restrict__ Kp, const LmDetGroup G, const uint8_t* __restrict__ ext,
                                                 int64_t ext_slot_bytes, const float* __restrict__ weights, int s0,
                                                 unsigned long long* __restrict__ keys, int32_t* __restrict__ n_pos,
                                                 uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes) {
  const LmConst& K = *Kp;
  constexpr int NQ = CB_C + KW - 1;
  constexpr int S2 = cb_stride_c(KW);
  extern __shared__ lm_f2 lp[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - tb;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1;
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  constexpr int PC = CB_H + KW - 1;  // pair columns used
  for (int e = threadIdx.x; e < rows * PC; e += blockDim.x) {
    const int r = e / PC, c = e - r * PC;
    const uint8_t* p = src + (int64_t)r * ew + c;
    lp[r * S2 + c] = (lm_f2){(float)p[0], (float)p[CB_H]};
  }
  // WLDS: detector weights staged in LDS after the tile and read as broadcast
  // ds_reads (no scalar loads, whose waits also drain the LDS queue)
  float* wl = reinterpret_cast<float*>(lp + rows * S2);
  if (WLDS)
    for (int e = threadIdx.x; e < D.kh * D.kwp; e += blockDim.x) wl[e] = weights[D.w_off + e];
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int ly = threadIdx.x >> 3, lx = threadIdx.x & 7;
  lm_f2 acc[2][CB_C];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < CB_C; ++c) acc[r][c] = (lm_f2){D.delta, D.delta};
  const float* __restrict__ W = weights + D.w_off;
  const int kh = D.kh, kwp = D.kwp;
  const unsigned base0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) lm_f2*)(lp + (ly * 2) * S2 + lx * CB_C);
  for (int t = 0; t <= kh; ++t) {
    lm_f2 px[NQ];
    cb_loads_impl<NQ>(px, base0 + (unsigned)(t * S2 * 8), std::make_integer_sequence<int, NQ>{});
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = t - r;
      if (i >= 0 && i < kh) {
        const float* wr = (WLDS ? wl : W) + ((G.skip_taps & 2) ? 0 : i * kwp);
#pragma unroll
        for (int j = 0; j < KW; ++j) {
          const float w = wr[j];
          const lm_f2 w2 = (lm_f2){w, w};
#pragma unroll
          for (int c = 0; c < CB_C; ++c) acc[r][c] = __builtin_elementwise_fma(w2, px[c + j], acc[r][c]);
        }
      }
    }
  }
  // epilogue (see corr_epilogue): outputs (2ly + r, 5lx + c) in .x and (2ly + r, 40 + 5lx + c) in .y
  const int my = D.m_y - D.in_y, mx = D.m_x - D.in_x;
  if (D.kind != 0) {
    uint8_t* __restrict__ tbm = tailbin + (int64_t)slot * tailbin_slot_bytes + (D.list ? (int64_t)K.tail_hb * K.tail_w : 0);
#pragma unroll
    for (int r = 0; r < 2; ++r)
#pragma unroll
      for (int c = 0; c < CB_C; ++c)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int y = oy0 + ly * 2 + r, x = ox0 + h * CB_H + lx * CB_C + c;
          const float a = h ? acc[r][c].y : acc[r][c].x;
          if (y < D.oh && x < D.ow) tbm[(int64_t)y * D.ow + x] = a > 0.0f ? 1 : 0;
        }
    return;
  }
  unsigned bits = 0;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < CB_C; ++c) {
      const lm_f2 pix = lp[(ly * 2 + r + my) * S2 + lx * CB_C + c + mx];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int y = oy0 + ly * 2 + r, x = ox0 + h * CB_H + lx * CB_C + c;
        const float a = h ? acc[r][c].y : acc[r][c].x;
        const float pv = h ? pix.y : pix.x;
        if (y < D.oh && x < D.ow && pv > 25.0f && a > 0.0f) bits |= 1u << ((r * CB_C + c) * 2 + h);
      }
    }
  const int nk = __popc(bits);
  const int off = nk ? atomicAdd(&s_cnt, nk) : 0;
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&n_pos[slot * LM_NLIST + D.list], s_cnt) : 0;
  __syncthreads();
  unsigned long long* __restrict__ kl = keys + (int64_t)slot * K.keys_per_slot + K.list_off[D.list] + s_base + off;
  int k = 0;
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int c = 0; c < CB_C; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (bits & (1u << ((r * CB_C + c) * 2 + h))) {
          const int y = oy0 + ly * 2 + r, x = ox0 + h * CB_H + lx * CB_C + c;
          const float a = h ? acc[r][c].y : acc[r][c].x;
          kl[k++] = ((unsigned long long)(~__float_as_uint(a)) << 32) | (unsigned)(y * D.ow + x);
        }
}

// k_corr_c1: column-block pairs (as k_corr_cb) with one output row per
// thread: 384 threads = 8 x 48 cover the 80 x 48 tile, each owning columns
// 5lx+{0..4} and 40+5lx+{0..4} of row ly.  Twice the waves of the row-pair
// kernels for the same LDS (up to 6 waves/SIMD), one detector row per
// iteration, so row t+1's weights are scalar-loaded during row t, and row
// t+1's pixel pairs (ds_read_b64) are loaded into each register as soon as
// row t's FMA block j = q no longer needs pair q (as k_corr_sp).
template <int Q>
DEV void c1_load(lm_f2& dst, unsigned base) {
  asm volatile("s_waitcnt lgkmcnt(10)\n\tds_read_b64 %0, %1 offset:%2" : "=v"(dst) : "v"(base), "i"(Q * 8) : "memory");
}

template <int KW, int... Qs>
DEV void c1_tail(lm_f2 (&px)[CB_C + KW - 1], unsigned nbase, std::integer_sequence<int, Qs...>) {
  (c1_load<KW + Qs>(px[KW + Qs], nbase), ...);
}

template <int KW, int J>
DEV void c1_block(lm_f2 (&acc)[CB_C], lm_f2 (&px)[CB_C + KW - 1], const float (&w)[KW], unsigned nbase) {
  const lm_f2 w2 = (lm_f2){w[J], w[J]};
#pragma unroll
  for (int c = 0; c < CB_C; ++c) acc[c] = __builtin_elementwise_fma(w2, px[c + J], acc[c]);
  __builtin_amdgcn_sched_barrier(0);
  c1_load<J>(px[J], nbase);  // pair J is dead for row t: refill it for row t+1
  if constexpr (J == KW - 1) c1_tail<KW>(px, nbase, std::make_integer_sequence<int, CB_C - 1>{});
  __builtin_amdgcn_sched_barrier(0);
}

template <int KW, int... Js>
DEV void c1_row(lm_f2 (&acc)[CB_C], lm_f2 (&px)[CB_C + KW - 1], const float (&w)[KW], unsigned nbase,
                std::integer_sequence<int, Js...>) {
  (c1_block<KW, Js>(acc, px, w, nbase), ...);
}

template <int KW>
__global__ __launch_bounds__(384) void k_corr_c1(const LmConst* __restrict__ Kp, const LmDetGroup G,
                                                 const uint8_t* __restrict__ ext, int64_t ext_slot_bytes,
                                                 const float* __restrict__ weights, int s0,
                                                 unsigned long long* __restrict__ keys, int32_t* __restrict__ n_pos,
                                                 uint8_t* __restrict__ tailbin, int64_t tailbin_slot_bytes) {
  const LmConst& K = *Kp;
  constexpr int NQ = CB_C + KW - 1;
  constexpr int S2 = cb_stride_c(KW);
  extern __shared__ lm_f2 lp[];
  __shared__ int s_cnt, s_base;
  const int slot = s0 + blockIdx.y;
  int gi = 0, tb = 0;
#pragma unroll
  for (int k = 0; k < LM_NDET - 1; ++k)
    if (k + 1 < G.n && (int)blockIdx.x >= G.tile_end[k]) {
      gi = k + 1;
      tb = G.tile_end[k];
    }
  const int d = G.ids[gi];
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - tb;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1;
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  constexpr int PC = CB_H + KW - 1;
  for (int e = threadIdx.x; e < rows * PC; e += blockDim.x) {
    const int r = e / PC, c = e - r * PC;
    const uint8_t* p = src + (int64_t)r * ew + c;
    lp[r * S2 + c] = (lm_f2){(float)p[0], (float)p[CB_H]};
  }
  if (threadIdx.x == 0) s_cnt = 0;
  __syncthreads();

  const int ly = threadIdx.x >> 3, lx = threadIdx.x & 7;
  lm_f2 acc[CB_C];
#pragma unroll
  for (int c = 0; c < CB_C; ++c) acc[c] = (lm_f2){D.delta, D.delta};
  const float* __restrict__ W = weights + D.w_off;
  const int kh = D.kh, kwp = D.kwp;
  unsigned base = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) lm_f2*)(lp + ly * S2 + lx * CB_C);
  const unsigned rstep = (unsigned)S2 * 8u;
  lm_f2 px[NQ];
  cb_loads_impl<NQ>(px, base, std::make_integer_sequence<int, NQ>{});  // row 0 (waits)
  float wc[KW];
#pragma unroll
  for (int j = 0; j < KW; ++j) wc[j] = W[j];
  for (int t = 0; t < kh; ++t) {
    // the last iteration loads a (dead) row kh: the LDS tile has a spare row
    const float* wnr = W + min(t + 1, kh - 1) * kwp;
    float wn[KW];
#pragma unroll
    for (int j = 0; j < KW; ++j) wn[j] = wnr[j];
    __builtin_amdgcn_sched_barrier(0);  // row t+1's scalar loads issue before row t's FMAs
    base += rstep;
    c1_row<KW>(acc, px, wc, base, std::make_integer_sequence<int, KW>{});
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // row t+1's pairs (and weights) have landed
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < KW; ++j) wc[j] = wn[j];
  }
  // epilogue: outputs (ly, 5lx + c) in .x and (ly, 40 + 5lx + c) in .y
  const int my = D.m_y - D.in_y, mx = D.m_x - D.in_x;
  if (D.kind != 0) {
    uint8_t* __restrict__ tbm = tailbin + (int64_t)slot * tailbin_slot_bytes + (D.list ? (int64_t)K.tail_hb * K.tail_w : 0);
#pragma unroll
    for (int c = 0; c < CB_C; ++c)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int y = oy0 + ly, x = ox0 + h * CB_H + lx * CB_C + c;
        const float a = h ? acc[c].y : acc[c].x;
        if (y < D.oh && x < D.ow) tbm[(int64_t)y * D.ow + x] = a > 0.0f ? 1 : 0;
      }
    return;
  }
  unsigned bits = 0;
#pragma unroll
  for (int c = 0; c < CB_C; ++c) {
    const lm_f2 pix = lp[(ly + my) * S2 + lx * CB_C + c + mx];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int y = oy0 + ly, x = ox0 + h * CB_H + lx * CB_C + c;
      const float a = h ? acc[c].y : acc[c].x;
      const float pv = h ? pix.y : pix.x;
      if (y < D.oh && x < D.ow && pv > 25.0f && a > 0.0f) bits |= 1u << (c * 2 + h);
    }
  }
  const int nk = __popc(bits);
  const int off = nk ? atomicAdd(&s_cnt, nk) : 0;
  __syncthreads();
  if (threadIdx.x == 0) s_base = s_cnt ? atomicAdd(&n_pos[slot * LM_NLIST + D.list], s_cnt) : 0;
  __syncthreads();
  unsigned long long* __restrict__ kl = keys + (int64_t)slot * K.keys_per_slot + K.list_off[D.list] + s_base + off;
  int k = 0;
#pragma unroll
  for (int c = 0; c < CB_C; ++c)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (bits & (1u << (c * 2 + h))) {
        const int y = oy0 + ly, x = ox0 + h * CB_H + lx * CB_C + c;
        const float a = h ? acc[c].y : acc[c].x;
        kl[k++] = ((unsigned long long)(~__float_as_uint(a)) << 32) | (unsigned)(y * D.ow + x);
      }
}

// widths with a specialised kernel; others use the generic k_corr
#define LM_KW_LIST(X) \
  X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32)

// Correlation variants: 0 generic (runtime width), 1 width-specialised plain
// FMA (k_corr_kw), 2 packed FMA with compiler-scheduled LDS loads, 3 packed
// FMA with explicit (row t, row t+1) ds_read2_b32 pair loads (default).
enum {
  CORR_GENERIC = 0, CORR_KW = 1, CORR_PK = 2, CORR_PK_ASM = 3, CORR_P2 = 4, CORR_DB = 5, CORR_SP = 6, CORR_CB = 7,
  CORR_PK_WLDS = 8, CORR_CB_WLDS = 9, CORR_C1 = 10
};

template <int n>
static inline const void* corr_fn(int variant) {
  if (variant == CORR_C1) return (const void*)&k_corr_c1<n>;
  if (variant == CORR_CB_WLDS) return (const void*)&k_corr_cb<n, true>;
  if (variant == CORR_PK_WLDS) return (const void*)&k_corr_pk<n, true, true>;
  if (variant == CORR_CB) return (const void*)&k_corr_cb<n>;
  if (variant == CORR_SP) return (const void*)&k_corr_sp<n>;
  if (variant == CORR_DB) return (const void*)&k_corr_db<n>;
  if (variant == CORR_P2) return (const void*)&k_corr_p2<n>;
  if (variant == CORR_PK_ASM) return (const void*)&k_corr_pk<n, false, true>;
  if (variant == CORR_PK) return (const void*)&k_corr_pk<n, false, false>;
  return (const void*)&k_corr_kw<n>;
}

// wide detectors (the 1920x512 geometry of config C5: 44, 48, 52, 60) get the
// production variant only; other variants fall back to the generic kernel
#define LM_KW_WIDE_LIST(X) X(36) X(40) X(44) X(48) X(52) X(56) X(60) X(64)

template <int n>
static inline const void* corr_fn_wide(int variant) {
  if (variant == CORR_C1) return (const void*)&k_corr_c1<n>;
  if (variant == CORR_CB_WLDS) return (const void*)&k_corr_cb<n, true>;
  if (variant == CORR_PK_WLDS) return (const void*)&k_corr_pk<n, true, true>;
  if (variant == CORR_CB) return (const void*)&k_corr_cb<n>;
  if (variant == CORR_SP) return (const void*)&k_corr_sp<n>;
  return variant == CORR_PK_ASM ? (const void*)&k_corr_pk<n, false, true> : nullptr;
}

static inline const void* corr_kernel(int variant, int kw, int* threads) {
  if (variant == CORR_C1) *threads = 384;
  else *threads = (variant == CORR_PK || variant == CORR_PK_ASM || variant == CORR_P2 || variant == CORR_DB ||
              variant == CORR_SP || variant == CORR_CB || variant == CORR_PK_WLDS || variant == CORR_CB_WLDS)
                 ? 192
                 : 256;
  const void* fn = nullptr;
  if (variant != CORR_GENERIC) switch (kw) {
#define LM_KW_CASE(n) \
  case n:             \
    fn = corr_fn<n>(variant);  \
    break;
      LM_KW_LIST(LM_KW_CASE)
#undef LM_KW_CASE
#define LM_KW_CASE(n)             \
  case n:                         \
    fn = corr_fn_wide<n>(variant); \
    break;
      LM_KW_WIDE_LIST(LM_KW_CASE)
#undef LM_KW_CASE
      default:
        break;
    }
  if (fn) return fn;
  *threads = 256;
  return (const void*)&k_corr;
}

static inline hipError_t corr_set_lds(int variant, int kw, size_t lds) {
  int th;
  return hipFuncSetAttribute(corr_kernel(variant, kw, &th), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
}

// Launch the correlation for one detector group (all detectors of one width).
static inline hipError_t launch_corr(int variant, int kw, dim3 grid, size_t lds, hipStream_t st, const LmConst* K,
                                     const LmDetGroup& G, const uint8_t* ext, int64_t ext_slot_bytes,
                                     const float* weights, int s0, unsigned long long* keys, int32_t* n_pos,
                                     uint8_t* tailbin, int64_t tailbin_slot_bytes) {
  int th;
  const void* fn = corr_kernel(variant, kw, &th);
  void* args[] = {(void*)&K, (void*)&G, (void*)&ext, (void*)&ext_slot_bytes, (void*)&weights, (void*)&s0,
                  (void*)&keys, (void*)&n_pos, (void*)&tailbin, (void*)&tailbin_slot_bytes};
  return hipLaunchKernel(fn, grid, dim3(th), args, lds, st);
}


// Debug copy of raw scores: same arithmetic as k_corr, no compaction.
__global__ __launch_bounds__(256) void k_corr_dbg(const LmConst* __restrict__ Kp, const uint8_t* __restrict__ ext, int64_t ext_slot_bytes,
                                                  const float* __restrict__ weights, int s0, float* __restrict__ dbg,
                                                  const int64_t* __restrict__ dbg_off, int64_t dbg_slot_floats) {
  const LmConst& K = *Kp;
  extern __shared__ float lds[];
  const int slot = s0 + blockIdx.y;
  int d = 0;
#pragma unroll
  for (int k = 1; k < LM_NDET; ++k)
    if ((int)blockIdx.x >= K.det[k].tile_base) d = k;
  const LmDet D = K.det[d];
  const int lt = blockIdx.x - D.tile_base;
  const int oy0 = (lt / D.tiles_x) * LM_TH, ox0 = (lt % D.tiles_x) * LM_TW;
  const int rows = LM_TH + D.kh - 1, cols = LM_TW + D.kwp - 1;
  int stride = cols;
  stride += (16 - (stride & 31) + 32) & 31;
  const uint8_t* __restrict__ src = ext + (int64_t)slot * ext_slot_bytes +
                                    (D.view ? (int64_t)K.ext_h[0] * K.ext_w[0] : 0) +
                                    (int64_t)(D.in_y + oy0) * K.ext_w[D.view] + (D.in_x + ox0);
  const int ew = K.ext_w[D.view];
  const int cols4 = (cols + 3) >> 2;
  for (int e = threadIdx.x; e < rows * cols4; e += 256) {
    const int r = e / cols4, c4 = (e - r * cols4) << 2;
    const uint8_t* p = src + (int64_t)r * ew + c4;
    float* o = lds + r * stride + c4;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c4 + k < stride) o[k] = (float)p[k];
  }
  __syncthreads();
  const int ly = threadIdx.x >> 4, lx = threadIdx.x & 15;
  const float* __restrict__ W = weights + D.w_off;
  for (int r = 0; r < LM_R; ++r)
    for (int c = 0; c < LM_C; ++c) {
      const int y = oy0 + ly * LM_R + r, x = ox0 + lx * LM_C + c;
      if (y >= D.oh || x >= D.ow) continue;
      float a = D.delta;
      for (int i = 0; i < D.kh; ++i)
        for (int j = 0; j < D.kwp; ++j)
          a = __builtin_fmaf(W[i * D.kwp + j], lds[(ly * LM_R + r + i) * stride + lx * LM_C + c + j], a);
      dbg[(int64_t)slot * dbg_slot_floats + dbg_off[d] + (int64_t)y * D.ow + x] = a;
    }
}

// ------------------------------------------------------------------ k_tail
// Connected components by lock-free union-find (atomicMin hooking) over the
// compacted foreground of a tail binary map, in LDS.  The largest component
// wins; on equal areas the one OpenCV labels first (8-connectivity: Grana
// BBDT 2x2-block raster order; 4-connectivity: Wu pixel raster order).
#define LM_TAIL_FG_MAX 6144

struct CCWork {
  unsigned* fg;      // pixel index of each foreground element
  unsigned* parent;  // union-find forest over element ids
  unsigned* area;    // per root
  unsigned* key;     // per root: first-label key
};

DEV unsigned cc_find(unsigned* parent, unsigned a) {
  unsigned p = parent[a];
  while (p != a) {
    a = p;
    p = parent[a];
  }
  return a;
}

DEV void cc_union(unsigned* parent, unsigned a, unsigned b) {
  while (true) {
    a = cc_find(parent, a);
    b = cc_find(parent, b);
    if (a == b) return;
    if (a < b) {
      unsigned t = a;
      a = b;
      b = t;
    }
    // a > b: hook a under b
    unsigned old = atomicMin(&parent[a], b);
    if (old == a) return;
    a = old;
  }
}

// Labels the foreground (given as element list fg[0..n) with pixel indices
// into a rows x cols map where `is_fg(p)` tells membership and `id_of(p)`
// maps a foreground pixel to its element id).  Returns the chosen root (or
// 0xFFFFFFFF when n == 0) in *s_best.  Block-wide; all threads call.
template <class IsFg, class IdOf>
DEV void cc_largest(CCWork W, int n, int rows, int cols, int conn, IsFg is_fg, IdOf id_of, unsigned* s_best) {
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    W.parent[k] = k;
    W.area[k] = 0;
    W.key[k] = 0xFFFFFFFFu;
  }
  __syncthreads();
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const unsigned p = W.fg[k];
    const int y = p / cols, x = p % cols;
    if (x > 0 && is_fg(p - 1)) cc_union(W.parent, k, id_of(p - 1));
    if (y > 0) {
      if (is_fg(p - cols)) cc_union(W.parent, k, id_of(p - cols));
      if (conn == 8) {
        if (x > 0 && is_fg(p - cols - 1)) cc_union(W.parent, k, id_of(p - cols - 1));
        if (x + 1 < cols && is_fg(p - cols + 1)) cc_union(W.parent, k, id_of(p - cols + 1));
      }
    }
  }
  __syncthreads();
  const int nbx = (cols + 1) / 2;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    const unsigned root = cc_find(W.parent, k);
    const unsigned p = W.fg[k];
    const int y = p / cols, x = p % cols;
    const unsigned key = conn == 8 ? (unsigned)((y >> 1) * nbx + (x >> 1)) : p;
    atomicAdd(&W.area[root], 1u);
    atomicMin(&W.key[root], key);
  }
  __syncthreads();
  // max area, then min key
  unsigned long long best = 0;
  for (int k = threadIdx.x; k < n; k += blockDim.x) {
    if (W.parent[k] == (unsigned)k) {  // root (parents are final roots after find? roots satisfy parent==self)
      unsigned long long v = ((unsigned long long)W.area[k] << 32) | (0xFFFFFFFFu - W.key[k]);
      if (v > best) best = v;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long other = __shfl_xor(best, o);
    if (other > best) best = other;
  }
  __shared__ unsigned long long s_red[16];
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long b = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w)
      if (s_red[w] > b) b = s_red[w];
    unsigned chosen = 0xFFFFFFFFu;
    if (b) {
      // find the root with this (area, key): keys are unique per component
      const unsigned key = 0xFFFFFFFFu - (unsigned)(b & 0xFFFFFFFFu);
      for (int k = 0; k < n; ++k)
        if (W.parent[k] == (unsigned)k && W.key[k] == key) {
          chosen = k;
          break;
        }
    }
    *s_best = chosen;
  }
  __syncthreads();
}

__global__ __launch_bounds__(1024) void k_tail(const LmConst* __restrict__ Kp, int s0, const uint8_t* __restrict__ tailbin,
                                               int64_t tailbin_slot_bytes, uint8_t* __restrict__ tailmask,
                                               unsigned* __restrict__ scratch, int64_t scratch_slot_words,
                                               LmSlotOut* __restrict__ hdr, int32_t* __restrict__ err) {
  const LmConst& K = *Kp;
  const int slot = s0 + blockIdx.x;
  const int TW = K.tail_w, HB = K.tail_hb, HS = K.tail_hs;
  const uint8_t* __restrict__ binb = tailbin + (int64_t)slot * tailbin_slot_bytes;
  const uint8_t* __restrict__ bins = binb + (int64_t)HB * TW;
  uint8_t* __restrict__ mask = tailmask + (int64_t)slot * HB * TW;
  unsigned* __restrict__ idmap = scratch + (int64_t)slot * scratch_slot_words;  // [HB*TW] element ids

  __shared__ unsigned s_fg[LM_TAIL_FG_MAX], s_parent[LM_TAIL_FG_MAX], s_area[LM_TAIL_FG_MAX], s_key[LM_TAIL_FG_MAX];
  __shared__ int s_n;
  __shared__ unsigned s_best;
  __shared__ int s_first, s_last;
  __shared__ uint8_t s_col[1024];
  // moments accumulators: [segment 15][tile rows <= 16][tile cols <= 2] x (n, sx, sy)
  __shared__ unsigned s_mb[15][16][2][3];
  __shared__ unsigned s_ms[15][16][2];  // side: per track column, per tile row: (n, sy)

  CCWork Wk{s_fg, s_parent, s_area, s_key};
  const int conn = K.connectivity;

  // zero TAIL_MASK, column mask
  for (int p = threadIdx.x; p < HB * TW; p += blockDim.x) mask[p] = 0;
  for (int c = threadIdx.x; c < TW; c += blockDim.x) s_col[c] = 0;
  if (threadIdx.x == 0) {
    s_n = 0;
    s_first = 0x7FFFFFFF;
    s_last = -1;
  }
  for (int e = threadIdx.x; e < 15 * 16 * 2 * 3; e += blockDim.x) (&s_mb[0][0][0][0])[e] = 0;
  for (int e = threadIdx.x; e < 15 * 16 * 2; e += blockDim.x) (&s_ms[0][0][0])[e] = 0;
  __syncthreads();

  // ---- bottom: compact foreground
  for (int p = threadIdx.x; p < HB * TW; p += blockDim.x)
    if (binb[p]) {
      int k = atomicAdd(&s_n, 1);
      if (k < LM_TAIL_FG_MAX) {
        s_fg[k] = p;
        idmap[p] = k;
      }
    }
  __syncthreads();
  int n = s_n;
  if (n > LM_TAIL_FG_MAX) {
    if (threadIdx.x == 0) atomicOr(err, 2);  // tail foreground exceeds the LDS capacity
    return;
  }
  cc_largest(Wk, n, HB, TW, conn, [&](unsigned p) { return binb[p] != 0; }, [&](unsigned p) { return idmap[p]; }, &s_best);
  const unsigned best_b = s_best;
  if (best_b != 0xFFFFFFFFu) {
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      if (cc_find(s_parent, k) == best_b) {
        const unsigned p = s_fg[k];
        mask[p] = 255;
        const int x = p % TW;
        s_col[x] = 255;
        atomicMin(&s_first, x);
        atomicMax(&s_last, x);
      }
    }
  }
  __syncthreads();
  const int first = s_first, last = s_last;
  const bool have = best_b != 0xFFFFFFFFu;
  // segment geometry (:2677-2685)
  const int tail_width = have ? last - first : 0;
  const int rem = tail_width % 15, reg = (tail_width - rem) / 15;
  // bottom segment moments: per selected pixel, integer per-tile sums
  if (have) {
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      if (cc_find(s_parent, k) != best_b) continue;
      const unsigned p = s_fg[k];
      const int y = p / TW, x = p % TW;
      if (x < first || x >= first + tail_width) continue;  // segments cover [first, last)
      const int rx = x - first;
      int seg, sx;
      if (rx < rem * (reg + 1)) {
        seg = rx / (reg + 1);
        sx = seg * (reg + 1);
      } else {
        seg = rem + (rx - rem * (reg + 1)) / reg;
        sx = rem * (reg + 1) + (seg - rem) * reg;
      }
      const int lxs = rx - sx;  // x inside the segment ROI
      const int ty = y >> 5, tx = lxs >> 5;
      atomicAdd(&s_mb[seg][ty][tx][0], 1u);
      atomicAdd(&s_mb[seg][ty][tx][1], (unsigned)(lxs & 31));
      atomicAdd(&s_mb[seg][ty][tx][2], (unsigned)(y & 31));
    }
  }
  __syncthreads();

  // ---- side: (tail_s > 0) & repeat(colmax) -> largest component
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  for (int p = threadIdx.x; p < HS * TW; p += blockDim.x)
    if (bins[p] && s_col[p % TW]) {
      int k = atomicAdd(&s_n, 1);
      if (k < LM_TAIL_FG_MAX) {
        s_fg[k] = p;
        idmap[p] = k;
      }
    }
  __syncthreads();
  n = s_n;
  if (n > LM_TAIL_FG_MAX) {
    if (threadIdx.x == 0) atomicOr(err, 2);
    return;
  }
  auto side_fg = [&](unsigned p) { return bins[p] != 0 && s_col[p % TW] != 0; };
  cc_largest(Wk, n, HS, TW, conn, side_fg, [&](unsigned p) { return idmap[p]; }, &s_best);
  const unsigned best_s = s_best;

  // track x (per segment) — needed to know which side columns to measure
  __shared__ int s_tx[15];
  if (threadIdx.x < 15) {
    const int i = threadIdx.x;
    int tx_ = -1, ty_ = -1;
    if (have) {
      const int sx = first + (i < rem ? i * (reg + 1) : rem * (reg + 1) + (i - rem) * reg);
      const int wseg = i < rem ? reg + 1 : reg;
      double m00 = 0, m10 = 0, m01 = 0;
      const double s = 1. / 255;
      const int ntr = (HB + 31) >> 5, ntc = (wseg + 31) >> 5;
      for (int ty = 0; ty < ntr; ++ty)
        for (int tx = 0; tx < ntc; ++tx) {
          const unsigned cnt = s_mb[i][ty][tx][0];
          const double mom0 = (double)(255u * cnt) * s;
          const double mom1 = (double)(255u * s_mb[i][ty][tx][1] + 0u) * s;
          const double mom2 = (double)(255u * s_mb[i][ty][tx][2]) * s;
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
    hdr[slot].tail[15 + i] = ty_;
  }
  __syncthreads();
  if (best_s != 0xFFFFFFFFu) {
    for (int k = threadIdx.x; k < n; k += blockDim.x) {
      if (cc_find(s_parent, k) != best_s) continue;
      const unsigned p = s_fg[k];
      const int y = p / TW, x = p % TW;
      for (int i = 0; i < 15; ++i)
        if (s_tx[i] > 0 && s_tx[i] == x) {
          atomicAdd(&s_ms[i][y >> 5][0], 1u);
          atomicAdd(&s_ms[i][y >> 5][1], (unsigned)(y & 31));
        }
    }
  }
  __syncthreads();
  if (threadIdx.x < 15) {
    const int i = threadIdx.x;
    int tz = -1;
    if (s_tx[i] > 0) {
      double m00 = 0, m01 = 0;
      const double s = 1. / 255;
      const int ntr = (HS + 31) >> 5;
      for (int ty = 0; ty < ntr; ++ty) {
        const double mom0 = (double)(255u * s_ms[i][ty][0]) * s;
        const double mom2 = (double)(255u * s_ms[i][ty][1]) * s;
        const double xm = 0.0 * mom0, ym = (double)(ty * 32) * mom0;
        (void)xm;
        m00 += mom0;
        m01 += mom2 + ym;
      }
      if (m00 > 0) tz = (int)(m01 / m00) + 0;
    }
    hdr[slot].tail[30 + i] = tz;
  }
}

// ------------------------------------------------------------------- k_nms
// One 512-thread block per (frame, list).  Positive detections are filtered by
// TAIL_MASK (bottom lists), sorted by (score desc, row-major index asc) —
// equal to std::sort whenever scores are distinct; on an exact tie the list is
// re-sorted from row-major order with the libstdc++ introsort replica
// (lm_introsort.h) — then clustered: nmsMax for the bottom view,
// peakClustering for the side view.
#define LM_NMS_THREADS 512
#define LM_NMS_CAP 2048     // entries kept in LDS; larger lists use the global-memory path
#define LM_NMS_RANKSORT 1024  // up to this many entries: O(n^2/T) rank sort instead of bitonic

DEV float key_score(unsigned long long k) { return __uint_as_float(~(unsigned)(k >> 32)); }
DEV unsigned key_lo(unsigned long long k) { return (unsigned)(k & 0xFFFFFFFFu); }

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
  if (dx >= bw || dy >= bh) return false;  // R.area() == 0
  return 3 * (bw - dx) * (bh - dy) > 2 * bw * bh;
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
//  * leaves (<= 16 elements): the final insertion sort is a stable sort of
//    each leaf, done in registers by one thread per leaf.
// q: two queues of qcap (first, last, depth); leaf: n flags; tf, tr: n ints.
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

DEV void std_sort_levels_dev(unsigned long long* a, int n, int* q, int qcap, int* leaf, int* tf, int* tr, int* s_cnt) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int i = threadIdx.x; i < n; i += blockDim.x) leaf[i] = 0;
  if (threadIdx.x == 0) {
    q[0] = 0;
    q[1] = n;
    q[2] = 2 * lm_sort::lg_(n);
    s_cnt[0] = n > 0 ? 1 : 0;
    s_cnt[1] = 0;
  }
  __syncthreads();
  int sel = 0;
  while (true) {
    const int qn = s_cnt[sel];
    if (qn == 0) break;
    const int* cur = q + sel * 3 * qcap;
    int* nxt = q + (1 - sel) * 3 * qcap;
    for (int r = wid; r < qn; r += nw) {
      const int f = cur[3 * r], l = cur[3 * r + 1], d = cur[3 * r + 2];
      if (l - f <= lm_sort::kThreshold) {
        if (lane == 0) leaf[f] = 1;
      } else if (d == 0) {
        if (lane == 0) {
          lm_sort::partial_sort_full(a + f, a + l, ReplicaLess());
          leaf[f] = 2;  // sorted; its insertion sort is a no-op
        }
      } else {
        const int cut = wave_partition(a, f, l, tf, tr);
        if (lane == 0) {
          const int k = atomicAdd(&s_cnt[1 - sel], 2);
          nxt[3 * k] = f;
          nxt[3 * k + 1] = cut;
          nxt[3 * k + 2] = d - 1;
          nxt[3 * k + 3] = cut;
          nxt[3 * k + 4] = l;
          nxt[3 * k + 5] = d - 1;
        }
      }
      wave_sync();
    }
    __syncthreads();
    if (threadIdx.x == 0) s_cnt[sel] = 0;
    sel = 1 - sel;
    __syncthreads();
  }
  // final insertion sort == stable sort of each leaf (<= 16 elements)
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    if (leaf[i] != 1) continue;
    int e = i + 1;
    while (e < n && e - i < lm_sort::kThreshold && !leaf[e]) ++e;
    const int m = e - i;
    unsigned long long v[lm_sort::kThreshold];
    float sc[lm_sort::kThreshold];
#pragma unroll
    for (int t = 0; t < lm_sort::kThreshold; ++t) {
      v[t] = t < m ? a[i + t] : 0ull;
      sc[t] = __uint_as_float((unsigned)(v[t] & 0xFFFFFFFFu));
    }
#pragma unroll
    for (int t = 0; t < lm_sort::kThreshold; ++t) {
      if (t >= m) break;
      int r = 0;
#pragma unroll
      for (int u = 0; u < lm_sort::kThreshold; ++u)
        if (u < m) r += (sc[u] > sc[t]) || (u < t && !(sc[t] > sc[u]));
      a[i + r] = v[t];
    }
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

__global__ __launch_bounds__(LM_NMS_THREADS) void k_nms(const LmConst* __restrict__ Kp, int s0, int side, unsigned long long* __restrict__ keys,
                                                       const int32_t* __restrict__ n_pos, const uint8_t* __restrict__ tailmask,
                                                       unsigned long long* __restrict__ gscratch, int64_t gscratch_slot,
                                                       LmSlotOut* __restrict__ hdr, int32_t* __restrict__ err,
                                                       long long* __restrict__ prof) {
  const LmConst& K = *Kp;
  const int slot = s0 + blockIdx.x;
  const int feat = blockIdx.y;  // 0 paw, 1 snout
  // optional phase timestamps (LM_KPROF=1): clock64() of thread 0 per phase
#define NMS_PROF(k) \
  if (prof && threadIdx.x == 0) prof[(blockIdx.x * 2 + blockIdx.y) * 16 + (k)] = clock64();
  NMS_PROF(0)
  if (prof && threadIdx.x == 0) prof[(blockIdx.x * 2 + blockIdx.y) * 16 + 14] = wall_clock64();
  const int list = side ? 2 + feat : feat;
  const int det = side ? (feat == 0 ? DET_PAW_S : DET_SNOUT_S) : (feat == 0 ? DET_PAW_B : DET_SNOUT_B);
  const LmDet D = K.det[det];
  LmSlotOut* H = hdr + slot;
  __shared__ unsigned long long s_keys[LM_NMS_CAP];
  __shared__ int s_assign[LM_NMS_CAP], s_mlist[LM_NMS_CAP];
  __shared__ unsigned s_xy[LM_NMS_CAP + 16];
  __shared__ int s_tmp[LM_NMS_CAP];
  __shared__ int s_stk[lm_sort::kStackInts];
  __shared__ int s_wsum[LM_NMS_THREADS / 64 + 1];
  __shared__ int s_n, s_flag, s_qcnt[2];

  if (side && H->cand_cnt[feat] == 0) {  // detectSideCandidates skips (:820-833)
    if (threadIdx.x == 0) {
      H->n_pos[list] = 0;
      H->cand_cnt[list] = 0;
      H->ties[list] = 0;
    }
    return;
  }
  const int n_in = n_pos[slot * LM_NLIST + list];
  const unsigned long long* __restrict__ src = keys + (int64_t)slot * K.keys_per_slot + K.list_off[list];
  unsigned long long* a = s_keys;
  int* assign = s_assign;
  int* mlist = s_mlist;
  unsigned* xy = s_xy;
  const bool glob = n_in > LM_NMS_CAP;
  if (glob) {  // rare: most of the crop positive; same algorithm in global scratch
    const int64_t npg = gscratch_slot / 3;
    a = gscratch + (int64_t)(blockIdx.y + 2 * blockIdx.x) * gscratch_slot;
    assign = reinterpret_cast<int*>(a + npg);
    mlist = assign + npg;
    xy = reinterpret_cast<unsigned*>(mlist + npg);
  }
  if (threadIdx.x == 0) {
    s_n = 0;
    s_flag = 0;
  }
  __syncthreads();
  // load + TAIL_MASK filter (bottom: mask(BB_BOTTOM_TAIL).setTo(255, TAIL_MASK), :783)
  const uint8_t* __restrict__ tm = tailmask + (int64_t)slot * K.tail_hb * K.tail_w;
  for (int k = threadIdx.x; k < n_in; k += blockDim.x) {
    const unsigned long long v = src[k];
    bool keep = true;
    if (!side) {
      const unsigned idx = key_lo(v);
      const int y = idx / D.ow, x = idx - y * D.ow;
      if (x < K.tail_w && y < K.tail_hb && tm[y * K.tail_w + x]) keep = false;
    }
    if (keep) a[atomicAdd(&s_n, 1)] = v;
  }
  __syncthreads();
  NMS_PROF(1)
  const int n = s_n;
  if (prof && threadIdx.x == 0) prof[(blockIdx.x * 2 + blockIdx.y) * 16 + 13] = n;
  int np = 1;
  while (np < n) np <<= 1;
  if (n <= LM_NMS_RANKSORT) {
    rank_sort(a, reinterpret_cast<unsigned long long*>(s_assign), n);  // s_assign: 8 KB = 1024 keys
  } else {
    for (int k = n + threadIdx.x; k < np; k += blockDim.x) a[k] = ~0ull;
    __syncthreads();
    bitonic_sort(a, np);
  }
  NMS_PROF(2)
  for (int k = threadIdx.x; k + 1 < n; k += blockDim.x)
    if ((a[k] >> 32) == (a[k + 1] >> 32)) s_flag = 1;
  __syncthreads();
  const int tie = s_flag;
  if (tie) {
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
    if (!glob) {
      if (n <= LM_NMS_RANKSORT) {  // back to row-major order
        rank_sort(a, reinterpret_cast<unsigned long long*>(s_assign), n);
      } else {
        for (int k = n + threadIdx.x; k < np; k += blockDim.x) a[k] = ~0ull;
        __syncthreads();
        bitonic_sort(a, np);
      }
      std_sort_levels_dev(a, n, s_mlist, LM_NMS_CAP / 6, s_assign, reinterpret_cast<int*>(s_xy), s_tmp, s_qcnt);
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
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
      const unsigned xj = xy[j];
      int as = j;
      for (int i0 = 0; i0 < j && as == j; i0 += 16) {  // 4 x 16 B loads in flight
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
  if (prof && threadIdx.x == 0) prof[(blockIdx.x * 2 + blockIdx.y) * 16 + 15] = wall_clock64();
  if (threadIdx.x == 0) {
    H->n_pos[list] = n;
    H->cand_cnt[list] = fits ? ncand : 0;
    H->ties[list] = tie;
  }
#undef NMS_PROF
}

// ------------------------------------------------------------------ k_post
#define LM_POST_THREADS 256
#define LM_POST_MAXC 512     // candidates per list handled in LDS
#define LM_POST_MAXOFF 2048  // CSC columns (Ni + Nong) + 1

DEV bool vel_criterion(const LmConst& K, const uint8_t* Fc, const uint8_t* Fp, const uint8_t* bkg, const int32_t* cal,
                       const uint8_t* lutc, const uint8_t* lutp, int crop_x, int crop_y, int crop_w, int crop_h,
                       int bx, int by, int bwid, int bhei, int area, double alpha, int32_t* err, int tag) {
  // checkVelCriterion (:1256-1267): sum(sat_u8(I - I_prev) > 25) >= area*alpha
  if (bx < 0 || by < 0 || bwid < 0 || bhei < 0 || bx + bwid > crop_w || by + bhei > crop_h) {
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
    return false;
  }
  int sum = 0;
  for (int r = 0; r < bhei; ++r)
    for (int c = 0; c < bwid; ++c) {
      const int R = crop_y + by + r, C = crop_x + bx + c;
      const int a = ipad_pixel(Fc, bkg, cal, lutc, K, R, C);
      const int b = ipad_pixel(Fp, bkg, cal, lutp, K, R, C);
      const int s = a > b ? a - b : 0;
      sum += s > 25;
    }
  return (double)sum >= ((double)area) * alpha;
}

__global__ __launch_bounds__(LM_POST_THREADS) void k_post(const LmConst* __restrict__ Kp, const LmSlot* __restrict__ slots,
                                                         const uint8_t* const* __restrict__ frame_ptr,
                                                         const uint8_t* __restrict__ bkg, const int32_t* __restrict__ cal,
                                                         const uint8_t* __restrict__ luts, LmSlotOut* __restrict__ hdr,
                                                         const unsigned long long* __restrict__ keys, LmP22D* __restrict__ arena_p22d,
                                                         int32_t* __restrict__ arena_side_y, double* __restrict__ arena_side_s,
                                                         double* __restrict__ arena_unary, int32_t* __restrict__ arena_jc,
                                                         int32_t* __restrict__ arena_ir, double* __restrict__ arena_pr,
                                                         LmArenaCtl* __restrict__ ctl, int32_t* __restrict__ err) {
  const LmConst& K = *Kp;
  const int slot = 1 + blockIdx.x;
  const int feat = blockIdx.y;
  LmSlotOut* H = hdr + slot;
  const LmSlotOut* HP = hdr + slot - 1;
  const int frame = slots[slot].frame;
  __shared__ LmCand sb[LM_POST_MAXC], st[LM_POST_MAXC], sp[LM_POST_MAXC];
  __shared__ int s_off[LM_POST_MAXOFF];
  __shared__ int s_mb[LM_POST_MAXC], s_mt[LM_POST_MAXC];  // motion status (-1 unknown)
  __shared__ float s_bps[LM_POST_MAXC], s_tpb[LM_POST_MAXC];
  __shared__ int s_all_equal, s_any1, s_any0, s_base[4];
  const int Nb = H->cand_cnt[feat], Ns = H->cand_cnt[2 + feat];
  const int Ni = frame > 0 ? HP->cand_cnt[feat] : 0;
  if (Nb > LM_POST_MAXC || Ns > LM_POST_MAXC || Ni > LM_POST_MAXC || Ni + K.ong_nx * K.ong_ny + 1 > LM_POST_MAXOFF) {
    if (threadIdx.x == 0) atomicOr(err, 8);
    return;
  }
  const LmCand* cb = LM_CAND_STAGE(K, keys, slot, feat);
  const LmCand* ct = LM_CAND_STAGE(K, keys, slot, 2 + feat);
  const LmCand* cp = LM_CAND_STAGE(K, keys, slot - 1, feat);
  for (int k = threadIdx.x; k < Nb; k += blockDim.x) sb[k] = cb[k];
  for (int k = threadIdx.x; k < Ns; k += blockDim.x) st[k] = ct[k];
  for (int k = threadIdx.x; k < Ni; k += blockDim.x) sp[k] = cp[k];
  __syncthreads();

  // ---------------- unary (unaryCostBox :1909-1952), column-major Nb x nprior
  const int nprior = feat == 0 ? 4 : 1;
  const int p0 = feat == 0 ? 0 : 4;
  if (threadIdx.x == 0) {
    int b = atomicAdd(&ctl->used[AR_UNARY], Nb * nprior);
    if (b + Nb * nprior > ctl->cap[AR_UNARY]) {
      atomicOr(&ctl->overflow, 1);
      b = -1;
    }
    s_base[0] = b;
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
    // column counts -> Jc
    for (int c = threadIdx.x; c < ncols; c += blockDim.x) {
      int cnt = 0;
      if (c < Ni) {
        for (int j = 0; j < Nb; ++j) cnt += trans(c, j) != 0.0;
        cnt += occ != 0.0;
      } else {
        const int q = c - Ni;
        if (Ni > 0)
          for (int j = 0; j < Nb; ++j) cnt += (ong_of(sb[j]) == q && occ != 0.0);
        cnt += occ != 0.0;
      }
      s_off[c] = cnt;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0;
      for (int c = 0; c < ncols; ++c) {
        const int t = s_off[c];
        s_off[c] = acc;
        acc += t;
      }
      s_off[ncols] = acc;
      int bj = atomicAdd(&ctl->used[AR_PWJC], ncols + 1);
      int bn = atomicAdd(&ctl->used[AR_PWNZ], acc);
      if (bj + ncols + 1 > ctl->cap[AR_PWJC] || bn + acc > ctl->cap[AR_PWNZ]) {
        atomicOr(&ctl->overflow, 1);
        bj = -1;
      }
      s_base[1] = bj;
      s_base[2] = bn;
    }
    __syncthreads();
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
              if (ong_of(sb[j]) == q) {
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

  // ---------------- matching (:1023-1254)
  const int ovlp = (int)(K.size_b[feat][0] * (1 - K.side_bottom_min_overlap));
  const bool vel_check = frame > 0;
  if (threadIdx.x == 0) {
    s_any1 = 0;
    s_any0 = 0;
  }
  for (int k = threadIdx.x; k < LM_POST_MAXC; k += blockDim.x) {
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
  // motion status where the reference evaluates it
  const LmSlot sl = slots[slot];
  const uint8_t* Fc = frame_ptr[slot];
  const uint8_t* Fp = frame_ptr[slot - 1];
  const uint8_t* lutc = luts + slot * 256;
  const uint8_t* lutp = luts + (slot - 1) * 256;
  const int* mbox = K.match_b[feat];
  const int* tbox = K.match_s[feat];
  if (vel_check) {
    for (int i = threadIdx.x; i < Nb; i += blockDim.x) {
      bool need = false;
      for (int j = 0; j < Ns; ++j) need |= boolD(i, j) && s_bps[j] > 1;
      if (need)
        s_mb[i] = vel_criterion(K, Fc, Fp, bkg, cal, lutc, lutp, sl.crop_x[0], sl.crop_y[0], K.crop_w[0], K.crop_h[0],
                                mbox[0] + sb[i].x + K.spre_b_w, mbox[1] + sb[i].y + K.spre_b_h, mbox[2], mbox[3],
                                K.size_b[feat][0] * K.size_b[feat][1], 0.02, err, (slot << 16) | (feat << 12) | i);
    }
    for (int j = threadIdx.x; j < Ns; j += blockDim.x) {
      bool need = false;
      if (s_bps[j] > 1)
        for (int i = 0; i < Nb; ++i) need |= boolD(i, j);
      if (need)
        s_mt[j] = vel_criterion(K, Fc, Fp, bkg, cal, lutc, lutp, sl.crop_x[1], sl.crop_y[1], K.crop_w[1], K.crop_h[1],
                                tbox[0] + st[j].x + K.spre_t_w, tbox[1] + st[j].y + K.spre_t_h, tbox[2], tbox[3],
                                K.size_s[feat][0] * K.size_s[feat][1], 0.05, err, (slot << 16) | (feat << 12) | 0x800 | j);
    }
  }
  __syncthreads();
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
    int bp = atomicAdd(&ctl->used[AR_P22D], Nb);
    int bs = atomicAdd(&ctl->used[AR_SIDE], acc);
    if (bp + Nb > ctl->cap[AR_P22D] || bs + acc > ctl->cap[AR_SIDE]) {
      atomicOr(&ctl->overflow, 1);
      bp = -1;
    }
    s_base[0] = bp;
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
  if (threadIdx.x == 0) {
    H->p22d_off[feat] = bp;
    H->p22d_cnt[feat] = Nb;
    H->side_off[feat] = bs;
    H->side_cnt[feat] = s_off[Nb];
  }
}

// ----------------------------------------------------------------- k_carry
// Copies the bottom candidate lists of the last slot of the previous batch
// (frame first-1) into slot 0's candidate staging, where k_post reads the
// previous frame's candidates (pairwisePotential, :896-919).  Runs first in a
// batch, before k_corr reuses the key areas of slots >= 1.
__global__ void k_carry(const LmConst* __restrict__ Kp, unsigned long long* __restrict__ keys, const LmSlotOut* __restrict__ prev_hdr,
                        int prev_slot, LmSlotOut* __restrict__ hdr) {
  const LmConst& K = *Kp;
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
__global__ __launch_bounds__(256) void k_prep(const LmSlot* __restrict__ h_slots, const uint8_t* const* __restrict__ h_fptr,
                                              const LmArenaCtl* __restrict__ h_ctl, int ns, LmSlot* __restrict__ slots,
                                              const uint8_t** __restrict__ fptr, LmArenaCtl* __restrict__ ctl,
                                              int32_t* __restrict__ npos, int32_t* __restrict__ err) {
  for (int i = threadIdx.x; i < ns; i += blockDim.x) {
    slots[i] = h_slots[i];
    fptr[i] = h_fptr[i];
  }
  for (int i = threadIdx.x; i < ns * LM_NLIST; i += blockDim.x) npos[i] = 0;
  if (threadIdx.x < 16) err[threadIdx.x] = 0;
  if (threadIdx.x == 0) *ctl = *h_ctl;
}

// k_out: the pack header always, and when the batch succeeded and its packed
// results fit the host buffer, the results themselves -> mapped pinned host
// memory; then the next batch's previous frame (storePreviousImage,
// LocoMouse_class.cpp:1508-1513) -> the halo buffer.  Packed sizes and frame
// sizes are multiples of 16 bytes.
__global__ __launch_bounds__(256) void k_out(const LmPackHdr* __restrict__ ph, LmPackHdr* __restrict__ h_ph,
                                             const uint8_t* __restrict__ pack, uint8_t* __restrict__ h_pack, int64_t h_cap,
                                             const uint8_t* __restrict__ halo_arg, const uint8_t* const* __restrict__ fptr,
                                             int fidx, uint8_t* __restrict__ halo_dst, int64_t halo_bytes) {
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
template <class F>
DEV int64_t block_exscan64(int L, F count, int64_t* out, int64_t* s_w) {
  const int T = blockDim.x, chunk = (L + T - 1) / T;
  const int i0 = threadIdx.x * chunk, i1 = min(L, i0 + chunk);
  int64_t c = 0;
  for (int i = i0; i < i1; ++i) c += count(i);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int64_t v = c;
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
  if (lane == 63) s_w[wid] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t acc = 0;
    for (int w = 0; w < (T >> 6); ++w) {
      const int64_t t = s_w[w];
      s_w[w] = acc;
      acc += t;
    }
    s_w[T >> 6] = acc;
  }
  __syncthreads();
  int64_t r = s_w[wid] + v - c;
  for (int i = i0; i < i1; ++i) {
    out[i] = r;
    r += count(i);
  }
  const int64_t total = s_w[T >> 6];
  if (threadIdx.x == 0) out[L] = total;
  __syncthreads();
  return total;
}

__global__ __launch_bounds__(1024) void k_pack_scan(const LmSlotOut* __restrict__ hdr, int n,
                                                    const LmArenaCtl* __restrict__ ctl, const int32_t* __restrict__ err,
                                                    LmPackHdr* __restrict__ ph, uint8_t* __restrict__ pack, int64_t pack_cap,
                                                    int64_t* __restrict__ side_base) {
  __shared__ int64_t s_w[1024 / 64 + 1];
  const int64_t zero[PK_COUNT] = {0, 0, 0, 0, 0, 0};
  const LmPackLayout L0 = lm_pack_layout(n, zero);  // offset arrays do not depend on the totals
  const LmSlotOut* H = hdr + 1;
  int64_t tot[PK_COUNT];
  tot[PK_CAND] = block_exscan64(4 * n, [&](int i) { return (int64_t)H[i >> 2].cand_cnt[i & 3]; },
                                reinterpret_cast<int64_t*>(pack + L0.cand_off), s_w);
  tot[PK_P22D] = block_exscan64(2 * n, [&](int i) { return (int64_t)H[i >> 1].p22d_cnt[i & 1]; },
                                reinterpret_cast<int64_t*>(pack + L0.p22d_off), s_w);
  tot[PK_UNARY] = block_exscan64(2 * n, [&](int i) { return (int64_t)H[i >> 1].unary_cnt[i & 1]; },
                                 reinterpret_cast<int64_t*>(pack + L0.unary_off), s_w);
  tot[PK_JC] = block_exscan64(2 * n, [&](int i) {
    const LmSlotOut& h = H[i >> 1];
    return h.pw_rows[i & 1] >= 0 ? (int64_t)h.pw_cols[i & 1] + 1 : (int64_t)0;
  }, reinterpret_cast<int64_t*>(pack + L0.jc_off), s_w);
  tot[PK_NZ] = block_exscan64(2 * n, [&](int i) {
    const LmSlotOut& h = H[i >> 1];
    return h.pw_rows[i & 1] >= 0 ? (int64_t)h.pw_nnz[i & 1] : (int64_t)0;
  }, reinterpret_cast<int64_t*>(pack + L0.nz_off), s_w);
  tot[PK_SIDE] = block_exscan64(2 * n, [&](int i) { return (int64_t)H[i >> 1].side_cnt[i & 1]; }, side_base, s_w);
  if (threadIdx.x == 0) {
    const LmPackLayout L = lm_pack_layout(n, tot);
    for (int k = 0; k < PK_COUNT; ++k) ph->tot[k] = tot[k];
    ph->bytes = L.bytes;
    ph->overflow = (L.bytes > pack_cap ? 1 : 0) | (ctl->overflow ? 2 : 0);
    ph->err = *err;
    for (int k = 0; k < AR_COUNT; ++k) ph->used[k] = ctl->used[k];
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

