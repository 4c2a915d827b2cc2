// Compares lm_sort::std_sort (locomouse_cpp_amd/csrc/lm_introsort.h) with
// libstdc++ std::sort on tie-heavy inputs.  Test infrastructure.
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

#include "lm_introsort.h"

struct Cand {
  int x, y;
  double s;
};

static uint64_t sm(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Host emulation of k_nms's tie sort as the device runs it
// (lm_kernels.hip std_sort_levels_dev + wave_subtree): level order for
// ranges of more than 64 elements, each smaller range finished by "one wave"
// (64 lanes emulated as arrays) with ballot-style partitions and a stable
// leaf sort.  Checks the formulation, not the device intrinsics.
template <class T, class Less>
static void emu_wave_subtree(T* a, int m, int d0, Less comp) {
  const int TH = lm_sort::kThreshold;
  uint64_t bnd = 1, pend = m > TH ? 1 : 0;
  int dep[64];
  for (int i = 0; i < 64; ++i) dep[i] = d0;
  auto nth = [](uint64_t msk, int k) {  // k-th set bit from bit 0
    for (int p = 0; p < 64; ++p)
      if ((msk >> p) & 1) {
        if (k == 0) return p;
        --k;
      }
    return 64;
  };
  while (pend) {
    const int s = __builtin_ctzll(pend);
    pend &= pend - 1;
    const uint64_t after = bnd & ~((2ull << s) - 1);
    const int e = after ? __builtin_ctzll(after) : m;
    const int d = dep[s];
    if (d == 0) {
      lm_sort::partial_sort_full(a + s, a + e, comp);
      continue;
    }
    const int mid = s + (e - s) / 2;
    int ch;
    if (comp(a[s + 1], a[mid])) ch = comp(a[mid], a[e - 1]) ? mid : comp(a[s + 1], a[e - 1]) ? e - 1 : s + 1;
    else ch = comp(a[s + 1], a[e - 1]) ? s + 1 : comp(a[mid], a[e - 1]) ? e - 1 : mid;
    std::swap(a[s], a[ch]);
    const T pv = a[s];
    uint64_t ml = 0, mr = 0;
    for (int i = s + 1; i < e; ++i) {
      if (!comp(a[i], pv)) ml |= 1ull << i;
      if (!comp(pv, a[i])) mr |= 1ull << i;
    }
    const int nl = __builtin_popcountll(ml), nr = __builtin_popcountll(mr);
    int K = 0;
    while (K < nl && K < nr && nth(ml, K) < nth(mr, nr - 1 - K)) ++K;
    int cut = K == 0 ? nth(ml, 0) : nth(mr, nr - K);
    if (K > 0 && K < nl) cut = std::min(cut, nth(ml, K));
    for (int k = 0; k < K; ++k) std::swap(a[nth(ml, k)], a[nth(mr, nr - 1 - k)]);
    dep[s] = d - 1;
    if (cut < e) {
      dep[cut] = d - 1;
      bnd |= 1ull << cut;
    }
    if (cut - s > TH) pend |= 1ull << s;
    if (e - cut > TH) pend |= 1ull << cut;
  }
  std::vector<T> out(a, a + m);
  for (int i = 0; i < m; ++i) {
    int ls = i;
    while (!((bnd >> ls) & 1)) --ls;
    int le = i + 1;
    while (le < m && !((bnd >> le) & 1)) ++le;
    if (le - ls > TH) continue;
    int rk = 0;
    for (int j = ls; j < le; ++j) rk += comp(a[j], a[i]) || (j < i && !comp(a[i], a[j]));
    out[ls + rk] = a[i];
  }
  std::copy(out.begin(), out.end(), a);
}

template <class T, class Less>
static void emu_device_sort(T* a, int n, Less comp, int depth0 = -1) {
  if (n <= 0) return;
  // ranges of <= 64 elements are finished after the levels, in reverse order
  // (any order gives the same result: the ranges are disjoint)
  std::vector<int> cur = {0, n, depth0 >= 0 ? depth0 : 2 * lm_sort::lg_(n)}, nxt, small;
  while (!cur.empty()) {
    nxt.clear();
    for (size_t r = 0; r < cur.size(); r += 3) {
      const int f = cur[r], l = cur[r + 1], d = cur[r + 2];
      int cut = 0;
      if (l - f <= 64) small.insert(small.end(), {f, l, d});
      else if (d == 0) lm_sort::partial_sort_full(a + f, a + l, comp);
      else if (lm_sort::process_range(a, f, l, d, comp, &cut)) nxt.insert(nxt.end(), {f, cut, d - 1, cut, l, d - 1});
    }
    cur.swap(nxt);
  }
  for (size_t r = small.size(); r >= 3; r -= 3) emu_wave_subtree(a + small[r - 3], small[r - 2] - small[r - 3], small[r - 1], comp);
}

int main() {
  auto cmp = [](const Cand& a, const Cand& b) { return a.s > b.s; };
  long cases = 0, fails = 0;
  for (int n : {0, 1, 2, 3, 5, 15, 16, 17, 31, 32, 33, 64, 100, 255, 256, 257, 1000, 4097, 20000}) {
    for (int levels : {1, 2, 3, 7, 50, 1000000}) {
      for (int pattern = 0; pattern < 4; ++pattern) {
        std::vector<Cand> a(n);
        for (int i = 0; i < n; ++i) {
          uint64_t r = sm((uint64_t)n * 7919 + (uint64_t)levels * 104729 + pattern * 13 + i);
          double s;
          if (pattern == 0) s = (double)(r % levels);
          else if (pattern == 1) s = (double)((n - i) % levels);     // descending runs
          else if (pattern == 2) s = (double)(i % levels);           // ascending runs
          else s = (double)((i / 8) % levels) + (r % 2) * 0.5;       // blocky
          a[i] = Cand{i, 0, (float)s};
        }
        std::vector<Cand> b = a, c = a, w = a;
        std::sort(a.begin(), a.end(), cmp);
        lm_sort::std_sort(b.data(), b.data() + n, cmp);
        lm_sort::std_sort_levels(c.data(), n, cmp);
        emu_device_sort(w.data(), n, cmp);
        ++cases;
        for (int i = 0; i < n; ++i)
          if (a[i].x != b[i].x || a[i].x != c[i].x || a[i].x != w[i].x) {
            ++fails;
            std::printf("MISMATCH n=%d levels=%d pattern=%d at %d (%s)\n", n, levels, pattern, i,
                        a[i].x != b[i].x ? "replica" : a[i].x != c[i].x ? "level-order" : "wave subtree");
            break;
          }
      }
    }
  }
  // depth-limit exhaustion (heap-sort fallback): drive libstdc++'s internal
  // __introsort_loop with small depth limits and compare.
  for (int n : {17, 40, 64, 65, 200, 3000}) {
    for (int depth : {0, 1, 2, 3}) {
      std::vector<Cand> a(n);
      for (int i = 0; i < n; ++i) a[i] = Cand{i, 0, (double)(sm(i * 31 + n) % 9)};
      std::vector<Cand> b = a, c = a, w = a;
      lm_sort::std_sort_levels(c.data(), n, cmp, depth);
      emu_device_sort(w.data(), n, cmp, depth);
      std::__introsort_loop(a.begin(), a.end(), (long)depth, __gnu_cxx::__ops::__iter_comp_iter(cmp));
      std::__final_insertion_sort(a.begin(), a.end(), __gnu_cxx::__ops::__iter_comp_iter(cmp));
      int stk[lm_sort::kStackInts];
      lm_sort::introsort_loop(b.data(), 0, n, depth, cmp, stk);
      lm_sort::final_insertion_sort(b.data(), b.data() + n, cmp);
      ++cases;
      for (int i = 0; i < n; ++i)
        if (a[i].x != b[i].x || a[i].x != c[i].x || a[i].x != w[i].x) {
          ++fails;
          std::printf("HEAP MISMATCH n=%d depth=%d at %d\n", n, depth, i);
          break;
        }
    }
  }
  std::printf("cases=%ld fails=%ld\n", cases, fails);
  return fails ? 1 : 0;
}
