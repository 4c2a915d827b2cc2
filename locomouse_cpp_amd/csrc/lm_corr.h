// lm_corr.h — the correlation (filter2D) kernels' shared constants and the
// host-side dispatch that lm_corr.hip (its own translation unit) exports to
// the runtime (lm_runtime.hip).  See lm_corr.hip for the kernels.
#ifndef LM_CORR_H
#define LM_CORR_H

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "lm_device.h"

#define LM_CORR_THREADS 192
#define PK_C 5  // columns per thread
#define PK_R 4  // rows per thread (two packed row pairs)

// LDS row stride: == 4 (mod 8) so the two 16-lane row groups of a
// ds_read2_b32 (4 rows apart) hit disjoint bank halves.
__host__ __device__ constexpr int pk_stride(int cols) { return cols + ((4 - (cols & 7)) + 8) % 8; }

struct LmDetGroup {
  int32_t n;
  int32_t ids[LM_NDET];
  int32_t tile_end[LM_NDET];  // cumulative tile counts
  int32_t ring_floats;        // k_corr_rw_all: LDS floats per wave (the widest detector's rings)
};

// Widths with a width-specialised k_corr_rw (any height); every other
// detector runs k_corr_gen.
#ifdef LM_KW_ONLY  // experiment builds: one ring width
#define LM_KW_LIST(X) X(LM_KW_ONLY)
#elif defined(LM_KW_C3)  // experiment builds: the synthetic C3 widths only (fast compiles)
#define LM_KW_LIST(X) X(22) X(24) X(26) X(30)
#else
#define LM_KW_LIST(X)                                                                                             \
  X(16) X(17) X(18) X(19) X(20) X(21) X(22) X(23) X(24) X(25) X(26) X(27) X(28) X(29) X(30) X(31) X(32) X(36) \
      X(40) X(44) X(48) X(52) X(56) X(60) X(64)
#endif
// widths of the merged launch (k_corr_rw_all): the even widths up to 40.  The
// merged kernel's register need grows with every width it holds (all bodies
// inlined behind one switch): 16..32 all, 36, 40 took 168 VGPRs and spilled
// with 40 x 4 sub-tiles; the even ones take 151 (three waves per SIMD, no
// spill).  Other widths run their per-width kernels in either plan.
#if defined(LM_KW_ONLY) || defined(LM_KW_C3)
#define LM_KW_LIST_RW_ALL LM_KW_LIST
#else
#define LM_KW_LIST_RW_ALL(X) X(16) X(18) X(20) X(22) X(24) X(26) X(28) X(30) X(32) X(36) X(40)
#endif
__host__ __device__ constexpr bool rw_all_width(int kw) {
  return kw % 2 == 0 && kw >= 16 && (kw <= 32 || kw == 36 || kw == 40);
}

// k_corr_rw: one wave per LM_RW_NQ sub-tiles of LM_FW x LM_FH outputs (or one
// 80 x 16 tile split into them), LM_RW_WAVES waves per workgroup
#ifndef LM_RW_WAVES
#define LM_RW_WAVES 4
#endif
#define LM_RW_THREADS (64 * LM_RW_WAVES)
#ifndef LM_RW_ALL_WPE
#define LM_RW_ALL_WPE 4  // waves per SIMD of the merged launch (k_corr_rw_all)
#endif
#define LM_RW_TH 16     // output rows of a wave's 80 x 16 tile (tail detectors)
#define LM_RW_HTH LM_FH  // output rows per sub-tile (the dark-tile grid's rows)
#ifndef LM_RW_HSLOTS
// ring rows per sub-tile (+ 1 mirror).  Row t + HSLOTS is loaded at the start
// of step t and stored at its end into row t's slot, after the step's last
// chunk has issued step t + 1's first reads: 8-row sub-tiles (two row groups
// 4 rows apart) read rows t + 1 .. t + 6 then, so 7 suffice (80-column
// sub-tiles: 8 measured 1-2 % faster, profiles/r04/ring7; 40-column: 7 keeps
// four waves per SIMD); 4-row sub-tiles read t + 1, t + 2: 3 suffice.
#define LM_RW_HSLOTS (LM_FH == 4 ? 3 : LM_RW_NQ == 4 ? 7 : 8)
#endif
static_assert(LM_RW_HSLOTS >= (LM_FH == 4 ? 3 : 7), "k_corr_rw ring: rows live during a step");

// window row of a sub-tile: LM_FW + KW - 1 columns plus up to 3 before them
// (the loads start on a 4-byte boundary), rounded to float4 stores (a lane
// group's reads all hit one row of each sub-tile: the stride does not enter
// the bank mapping)
__host__ __device__ constexpr int rw_stride(int kw) { return (LM_FW + kw - 1 + 3 + 3) / 4 * 4; }
// floats per sub-tile ring: == LM_FW / 5 (mod 32).  A ds_read_b32 lane
// group (32 lanes) holds one row group of 32 / (LM_FW / 5) sub-tiles; a
// sub-tile's LM_FW / 5 lanes of a row group read columns 5 lx (mod 32) of one
// ring row, and rings that start LM_FW / 5 floats apart (mod 32) put the
// group's 32 reads on 32 banks (rw_tile).
__host__ __device__ constexpr int rw_qpitch(int kw) {
  return (LM_RW_HSLOTS + 1) * rw_stride(kw) +
         ((LM_FW / 5 - ((LM_RW_HSLOTS + 1) * rw_stride(kw)) % 32) + 32) % 32;
}
__host__ __device__ constexpr int rw_ring_floats(int kw) { return LM_RW_NQ * rw_qpitch(kw); }
// LDS of one ring workgroup at width kw (defined in lm_corr.hip, so it
// follows the LM_RW_WAVES that the ring kernels were built with)
size_t corr_rw_lds(int kw);

// k_corr_f16 (non-parity LM_CORR_F16 mode): 2 x 2 waves per workgroup, each
// with two 32 x 32 accumulator tiles side by side -> a 128 x 64 output tile
// (round 4: 5 waves of 32 columns, -4 % k_corr at C5 but fewer frames/s;
// four 32-row tiles per wave, 130k vs 150k C5 frames/s at two waves per SIMD)
#define LM_F16_WAVES 4
#define LM_F16_TW 128
#define LM_F16_TH 64
#define LM_F16_THREADS (64 * LM_F16_WAVES)
#define LM_F16_MAX_NCH 10

__host__ __device__ constexpr int f16_nch(int kw) { return (kw + 31 + 15) / 16; }
__host__ __device__ constexpr int f16_cols(int nch) { return LM_F16_TW - 32 + 16 * nch; }
__host__ __device__ constexpr int f16_stride(int cols) { return (cols + 7) / 16 * 16 + 8; }
__host__ __device__ constexpr size_t f16_lds_bytes(int nch, int kh) {
  // the f16 window (the B fragments come from global memory)
  (void)nch;
  return (size_t)(LM_F16_TH + kh - 1) * f16_stride(f16_cols(nch)) * 2;
}
// Host: the B fragment of (row i, chunk c) for lane l, element j (0 off the band).
static inline float f16_bfrag_weight(const double* w, int kw, int i, int c, int l, int j) {
  const int r = l & 31, h = l >> 5, jj = 16 * c + 8 * h + j - r;
  return (jj >= 0 && jj < kw) ? (float)w[(size_t)i * kw + jj] : 0.0f;
}

// ---- host dispatch (defined in lm_corr.hip)
// k_corr_rw's ring does not depend on the detector height: every width of
// LM_KW_LIST, any kh; other widths run k_corr_gen
bool corr_ring(int kw);
const void* corr_kernel(int kw, bool unf);     // k_corr_rw<kw> or k_corr_gen
const void* corr_kernel_gen(bool unf);         // k_corr_gen (any size)
const void* corr_kernel_rw_all(bool unf);      // every ring width in one launch
const void* corr_kernel_f16(int kw);           // nullptr when kw is too wide
// Dark tiles of a batch (written by k_ingest, lm_kernels.hip): flag bytes
// per (slot, view, tile), the bright tiles' list per view and their counts.
// All null: every tile is computed (LM_CORR_DARK=0).
struct CorrDark {
  uint8_t* flags = nullptr;
  int32_t* cnt = nullptr;
  uint32_t* list = nullptr;
};
// Launch the correlation for one detector group (`weights`: the fp32 rows, or
// the f16 B fragments for k_corr_f16).  Ring kernels take one wave per tile
// with the batch's tiles flattened (grid.y = slot count; with dark-tile lists
// the point detectors' waves are their bright tiles only); the others one
// workgroup per (tile, slot), dark workgroups returning at once.
hipError_t launch_corr(const void* fn, bool ring, dim3 grid, int threads, size_t lds, hipStream_t st, const LmConst* K,
                       const LmDetGroup& G, const uint8_t* ext, int64_t ext_slot_bytes, const void* weights, int s0,
                       unsigned long long* keys, int32_t* n_pos, uint8_t* tailbin, int64_t tailbin_slot_bytes,
                       const CorrDark& dark);
// Diagnostics: raw scores of every detector of slots s0 .. s0 + grid.y - 1.
hipError_t launch_corr_dbg(bool unf, dim3 grid, hipStream_t st, const LmConst* K, const uint8_t* ext,
                           int64_t ext_slot_bytes, const float* weights, int s0, float* dbg, const int64_t* dbg_off,
                           int64_t dbg_slot_floats);

#endif  // LM_CORR_H
