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
        std::vector<Cand> b = a, c = a;
        std::sort(a.begin(), a.end(), cmp);
        lm_sort::std_sort(b.data(), b.data() + n, cmp);
        lm_sort::std_sort_levels(c.data(), n, cmp);
        ++cases;
        for (int i = 0; i < n; ++i)
          if (a[i].x != b[i].x || a[i].x != c[i].x) {
            ++fails;
            std::printf("MISMATCH n=%d levels=%d pattern=%d at %d (%s)\n", n, levels, pattern, i,
                        a[i].x != b[i].x ? "replica" : "level-order");
            break;
          }
      }
    }
  }
  // depth-limit exhaustion (heap-sort fallback): drive libstdc++'s internal
  // __introsort_loop with small depth limits and compare.
  for (int n : {17, 40, 200, 3000}) {
    for (int depth : {0, 1, 2, 3}) {
      std::vector<Cand> a(n);
      for (int i = 0; i < n; ++i) a[i] = Cand{i, 0, (double)(sm(i * 31 + n) % 9)};
      std::vector<Cand> b = a, c = a;
      lm_sort::std_sort_levels(c.data(), n, cmp, depth);
      std::__introsort_loop(a.begin(), a.end(), (long)depth, __gnu_cxx::__ops::__iter_comp_iter(cmp));
      std::__final_insertion_sort(a.begin(), a.end(), __gnu_cxx::__ops::__iter_comp_iter(cmp));
      int stk[lm_sort::kStackInts];
      lm_sort::introsort_loop(b.data(), 0, n, depth, cmp, stk);
      lm_sort::final_insertion_sort(b.data(), b.data() + n, cmp);
      ++cases;
      for (int i = 0; i < n; ++i)
        if (a[i].x != b[i].x || a[i].x != c[i].x) {
          ++fails;
          std::printf("HEAP MISMATCH n=%d depth=%d at %d\n", n, depth, i);
          break;
        }
    }
  }
  std::printf("cases=%ld fails=%ld\n", cases, fails);
  return fails ? 1 : 0;
}
