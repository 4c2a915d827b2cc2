// lm_cc.h — largest connected component of a binary map by row runs, shared by
// k_tail (selectLargestRegion, LocoMouse_class.cpp:2744-2767, called at :2604
// and :2626) and k_bb_cc (largestBWAreaObject, :921-946).
//
// cv::connectedComponentsWithStats labels 8-connected components in Grana's
// BBDT 2x2-block raster order and 4-connected ones in Wu/SAUF pixel raster
// order; the reference keeps the largest area with a strict '>' scan over the
// labels, so on equal areas the component OpenCV labels first wins.  Here:
//   1. the map is staged as a bitmap (64 columns per word, one spare zero word
//      per row) with per-row run counts; an exclusive scan gives run offsets;
//   2. runs (maximal horizontal stretches) are read off the words;
//   3. each run is linked to the overlapping runs of the row above (columns
//      within +-1 for 8-connectivity) in a union-find forest over runs
//      (atomicMin hooking of the larger root under the smaller, so a root is
//      its component's first run in raster order);
//   4. per root: area and first-label key (8-conn: (y/2)*ceil(W/2) + x/2 of
//      its first block; 4-conn: y*W + x of its first pixel); the largest area,
//      then the smallest key, wins.
// The run table lives in LDS when it fits (cap runs), else in per-frame global
// scratch, read with L1-bypassing loads so every wave sees the others' hooks.
// There is no size limit: a map has at most H * ceil(W/2) runs.
#ifndef LM_CC_H
#define LM_CC_H

DEV unsigned cc_ld(const unsigned* a) { return __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
DEV void cc_st(unsigned* a, unsigned v) { __hip_atomic_store(a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Run table: start / end column (u16 in LDS, u32 in global memory),
// union-find parent, area and first-label key per run; a run's row is found
// by binary search in the per-row run offsets.
template <class IX>
struct CCRuns {
  IX *rs, *re;
  unsigned *par, *area, *key;
};

template <bool G, class T>
DEV unsigned rld(const T* a) {
  if constexpr (G) return cc_ld(reinterpret_cast<const unsigned*>(a));
  else return (unsigned)*a;
}
template <bool G, class T>
DEV void rst(T* a, unsigned v) {
  if constexpr (G) cc_st(reinterpret_cast<unsigned*>(a), v);
  else *a = (T)v;
}
template <bool G>
DEV unsigned rfind(const unsigned* par, unsigned a) {
  unsigned q = rld<G>(&par[a]);
  while (q != a) {
    a = q;
    q = rld<G>(&par[a]);
  }
  return a;
}
template <bool G>
DEV void runion(unsigned* par, unsigned a, unsigned b) {
  while (true) {
    a = rfind<G>(par, a);
    b = rfind<G>(par, b);
    if (a == b) return;
    if (a < b) {
      const unsigned t = a;
      a = b;
      b = t;
    }
    const unsigned old = atomicMin(&par[a], b);
    if (old == a) return;
    a = old;
  }
}

// Exclusive scan of v[0..n) in place by wave 0; the total goes to *total.
// Block-wide call.
DEV void cc_wave0_scan(int* v, int n, int* total) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    int carry = 0;
    for (int b = 0; b < n; b += 64) {
      const int i = b + lane;
      const int x = i < n ? v[i] : 0;
      int inc = x;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
      }
      if (i < n) v[i] = carry + inc - x;
      carry += __shfl(inc, 63);
    }
    if (lane == 0) *total = carry;
  }
  __syncthreads();
}

// Row of run i: the last y with rowoff[y] <= i (rowoff exclusive offsets).
DEV int cc_row_of(const int* rowoff, int H, int i) {
  int lo = 0, hi = H;  // first y with rowoff[y] > i, minus one
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (rowoff[mid] <= i) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

// Bit i (0..3) = byte i of w is nonzero: bit 7 of each byte set by
// (w | ((w & 0x7F..) + 0x7F..)), then the four bits gathered by one multiply
// (the partial products land on distinct bits, so nothing carries into 28-31).
DEV unsigned cc_nonzero_bytes(unsigned w) {
  const unsigned t = ((w | ((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu)) & 0x80808080u) >> 7;
  return (t * 0x10204080u) >> 28;
}

// Bitmap of a u8 map (nonzero = foreground; H rows of W bytes at `pitch`)
// into bm[y][0..nb64] (the last word of a row stays zero), optionally ANDed
// with a column mask (colm[nb64] words, bit x = column x), and the number of
// runs of each row into rowoff[y].  Every thread takes 16-column pieces of
// any row, twelve pieces' loads in flight before any is used (16-byte loads when
// `vec`: W % 16 == 0 and 16-byte aligned rows), so the map streams in at a
// few load latencies instead of one per row; then one thread per row counts
// the run starts.  Block-wide call (ends with a barrier).
DEV void cc_bitmap_u8(const uint8_t* __restrict__ src, int64_t pitch, int W, int H, int nb64, bool vec,
                      const unsigned long long* colm, unsigned long long* bm, int* rowoff) {
  const int npc = 4 * (nb64 + 1);  // 16-bit pieces per bitmap row (incl. the spare word)
  const int total = H * npc;
  constexpr int U = 12;  // pieces per thread per round: a tail map is one or two load latencies
  for (int e0 = 0; e0 < total; e0 += U * (int)blockDim.x) {
    uint4 q[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * (int)blockDim.x + (int)threadIdx.x;
      const int y = e / npc, x = 16 * (e - y * npc);
      if (vec && e < total && x < W) q[u] = *reinterpret_cast<const uint4*>(src + (int64_t)y * pitch + x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * (int)blockDim.x + (int)threadIdx.x;
      if (e >= total) continue;
      const int y = e / npc, pc = e - y * npc, x = 16 * pc;
      unsigned m = 0;
      if (x < W) {
        if (vec) {
          const unsigned w4[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) m |= cc_nonzero_bytes(w4[k]) << (4 * k);
        } else {
          const uint8_t* row = src + (int64_t)y * pitch;
          for (int k = 0; k < 16 && x + k < W; ++k) m |= (row[x + k] ? 1u : 0u) << k;
        }
        if (colm) m &= (unsigned)(colm[x >> 6] >> (x & 63)) & 0xFFFFu;
      }
      reinterpret_cast<uint16_t*>(bm + (int64_t)y * (nb64 + 1))[pc] = (uint16_t)m;
    }
  }
  __syncthreads();
  for (int y = threadIdx.x; y < H; y += blockDim.x) {
    const unsigned long long* row = bm + (int64_t)y * (nb64 + 1);
    unsigned long long carry = 0;
    int n = 0;
    for (int k = 0; k < nb64; ++k) {
      const unsigned long long bits = row[k];
      n += __popcll(bits & ~((bits << 1) | carry));
      carry = bits >> 63;
    }
    rowoff[y] = n;
  }
  __syncthreads();
}

// The same staging from a bitmap already in memory (H rows of nb64 u64 words,
// bit x = column x; k_corr writes the tail maps this way), optionally ANDed
// with the column mask.  Block-wide call (ends with a barrier).
DEV void cc_bitmap_bits(const unsigned long long* __restrict__ src, int H, int nb64, const unsigned long long* colm,
                        unsigned long long* bm, int* rowoff) {
  const int total = H * (nb64 + 1);
  for (int e = threadIdx.x; e < total; e += blockDim.x) {
    const int y = e / (nb64 + 1), k = e - y * (nb64 + 1);
    unsigned long long w = 0;
    if (k < nb64) {
      w = src[(int64_t)y * nb64 + k];
      if (colm) w &= colm[k];
    }
    bm[e] = w;
  }
  __syncthreads();
  for (int y = threadIdx.x; y < H; y += blockDim.x) {
    const unsigned long long* row = bm + (int64_t)y * (nb64 + 1);
    unsigned long long carry = 0;
    int n = 0;
    for (int k = 0; k < nb64; ++k) {
      const unsigned long long bits = row[k];
      n += __popcll(bits & ~((bits << 1) | carry));
      carry = bits >> 63;
    }
    rowoff[y] = n;
  }
  __syncthreads();
}

// Labels the runs of a bitmap (rows bm[y][0..nb64], R runs at offsets rowoff)
// and picks the largest component (ties: first OpenCV label).  On return
// S.par[i] is the root of run i for every run and *s_best the chosen root
// (0xFFFFFFFF when there is no foreground).  The LDS union-find arrays may
// overlay the bitmap: it is dead once the runs are read.  Block-wide call.
template <bool G, class IX>
DEV void cc_label(const CCRuns<IX> S, const unsigned long long* bm, int nb64, int W, int H, int R, const int* rowoff,
                  bool c8, unsigned long long* s_red, unsigned* s_best) {
  const int tid = threadIdx.x, nt = blockDim.x, lane = tid & 63, wave = tid >> 6, nw = nt >> 6;
  const unsigned nbx = (unsigned)(W + 1) / 2;
  if (tid == 0) *s_best = 0xFFFFFFFFu;
  // Runs: one (row, word) per thread.  Runs are numbered in raster order, so
  // the starts (ends) in word k of a row are numbered after the starts (ends)
  // in the row's earlier words: popcounts of those words give the offsets.
  {
    const int items = H * nb64;
    for (int e = tid; e < items; e += nt) {
      const int y = e / nb64, k = e - y * nb64;
      const unsigned long long* row = bm + (int64_t)y * (nb64 + 1);
      const unsigned long long bits = row[k];
      const unsigned long long prev = k ? row[k - 1] >> 63 : 0ull, nxt = row[k + 1] & 1ull;
      unsigned long long st = bits & ~((bits << 1) | prev);
      unsigned long long en = bits & ~((bits >> 1) | (nxt << 63));
      if (!(st | en)) continue;
      int ns = rowoff[y], ne = ns;
      for (int q = 0; q < k; ++q) {
        const unsigned long long b = row[q], pb = q ? row[q - 1] >> 63 : 0ull, nb = row[q + 1] & 1ull;
        ns += __popcll(b & ~((b << 1) | pb));
        ne += __popcll(b & ~((b >> 1) | (nb << 63)));
      }
      for (; st; st &= st - 1) rst<G>(&S.rs[ns++], (unsigned)(64 * k + __ffsll((long long)st) - 1));
      for (; en; en &= en - 1) rst<G>(&S.re[ne++], (unsigned)(64 * k + __ffsll((long long)en) - 1));
    }
  }
  __syncthreads();  // the LDS union-find arrays overlay the bitmap
  for (int i = tid; i < R; i += nt) {
    rst<G>(&S.par[i], (unsigned)i);
    rst<G>(&S.area[i], 0u);
    rst<G>(&S.key[i], 0xFFFFFFFFu);
  }
  __syncthreads();
  const int d = c8 ? 1 : 0;
  for (int i = tid; i < R; i += nt) {
    const int y = cc_row_of(rowoff, H, i);
    if (y == 0) continue;
    const int a0 = (int)rld<G>(&S.rs[i]) - d, a1 = (int)rld<G>(&S.re[i]) + d;
    int lo = rowoff[y - 1], hi = rowoff[y];
    while (lo < hi) {  // first run of row y-1 ending at or after a0
      const int mid = (lo + hi) >> 1;
      if ((int)rld<G>(&S.re[mid]) < a0) lo = mid + 1; else hi = mid;
    }
    for (int j = lo; j < rowoff[y] && (int)rld<G>(&S.rs[j]) <= a1; ++j) runion<G>(S.par, i, j);
  }
  __syncthreads();
  for (int i = tid; i < R; i += nt) {
    const unsigned root = rfind<G>(S.par, i);
    const unsigned y = (unsigned)cc_row_of(rowoff, H, i), x = rld<G>(&S.rs[i]);
    atomicAdd(&S.area[root], rld<G>(&S.re[i]) - x + 1);
    atomicMin(&S.key[root], c8 ? (y >> 1) * nbx + (x >> 1) : y * (unsigned)W + x);
    rst<G>(&S.par[i], root);
  }
  __syncthreads();
  unsigned long long best = 0;
  for (int i = tid; i < R; i += nt) {
    if (rld<G>(&S.par[i]) != (unsigned)i) continue;
    const unsigned long long val = ((unsigned long long)rld<G>(&S.area[i]) << 32) | (0xFFFFFFFFu - rld<G>(&S.key[i]));
    best = val > best ? val : best;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long other = __shfl_xor(best, o);
    best = other > best ? other : best;
  }
  if (lane == 0) s_red[wave] = best;
  __syncthreads();
  best = 0;
  for (int w = 0; w < nw; ++w) best = s_red[w] > best ? s_red[w] : best;
  if (best) {
    const unsigned barea = (unsigned)(best >> 32), bkey = 0xFFFFFFFFu - (unsigned)best;
    for (int i = tid; i < R; i += nt)
      if (rld<G>(&S.par[i]) == (unsigned)i && rld<G>(&S.area[i]) == barea && rld<G>(&S.key[i]) == bkey) *s_best = i;
  }
  __syncthreads();
}

#endif  // LM_CC_H
