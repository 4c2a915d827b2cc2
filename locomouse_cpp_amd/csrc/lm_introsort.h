/*
 * lm_introsort.h — exact replica of libstdc++'s std::sort (GCC 11, the
 * toolchain of this image and of the GPU box) for device code.
 *
 * Why: nmsMax / peakClustering sort their positive detections with
 * std::sort(compareCandidate) (LocoMouse_class.cpp:1658, :1800;
 * Candidates.cpp:33-36: a.s > b.s).  std::sort is unstable, so when two
 * detections have exactly equal scores their relative order — and therefore
 * cluster membership and candidate order — is whatever libstdc++'s
 * introsort produces from the row-major input order.  The GPU path sorts with
 * a bitonic network keyed (score desc, row-major index asc); that equals
 * std::sort whenever all scores are distinct.  When a tie is detected the
 * list is re-sorted with this replica from row-major order.
 *
 * Restated from the published libstdc++ algorithm (bits/stl_algo.h
 * __introsort_loop / __unguarded_partition_pivot / __move_median_to_first /
 * __final_insertion_sort with _S_threshold = 16, and bits/stl_heap.h
 * __make_heap / __adjust_heap / __push_heap / __pop_heap / __sort_heap for
 * the depth-limit fallback).  Every comparison and move happens in the same
 * order as libstdc++, which is what makes the permutation identical.
 * tests/test_introsort.py checks it against std::sort on tie-heavy inputs.
 */
#ifndef LM_INTROSORT_H
#define LM_INTROSORT_H

#if defined(__HIPCC__)
#define LM_HD __host__ __device__
#else
#define LM_HD
#endif

namespace lm_sort {

template <class T, class Less>
LM_HD inline void iter_swap_(T* a, T* b) {
  T t = *a;
  *a = *b;
  *b = t;
}

template <class T, class Less>
LM_HD inline void move_median_to_first(T* result, T* a, T* b, T* c, Less comp) {
  if (comp(*a, *b)) {
    if (comp(*b, *c)) iter_swap_<T, Less>(result, b);
    else if (comp(*a, *c)) iter_swap_<T, Less>(result, c);
    else iter_swap_<T, Less>(result, a);
  } else if (comp(*a, *c)) {
    iter_swap_<T, Less>(result, a);
  } else if (comp(*b, *c)) {
    iter_swap_<T, Less>(result, c);
  } else {
    iter_swap_<T, Less>(result, b);
  }
}

template <class T, class Less>
LM_HD inline T* unguarded_partition(T* first, T* last, T* pivot, Less comp) {
  while (true) {
    while (comp(*first, *pivot)) ++first;
    --last;
    while (comp(*pivot, *last)) --last;
    if (!(first < last)) return first;
    iter_swap_<T, Less>(first, last);
    ++first;
  }
}

template <class T, class Less>
LM_HD inline T* unguarded_partition_pivot(T* first, T* last, Less comp) {
  T* mid = first + (last - first) / 2;
  move_median_to_first<T, Less>(first, first + 1, mid, last - 1, comp);
  return unguarded_partition<T, Less>(first + 1, last, first, comp);
}

// ---- heap (stl_heap.h), used when the depth limit is exhausted
template <class T, class Less>
LM_HD inline void push_heap_(T* first, long hole, long top, T value, Less comp) {
  long parent = (hole - 1) / 2;
  while (hole > top && comp(first[parent], value)) {
    first[hole] = first[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  first[hole] = value;
}

template <class T, class Less>
LM_HD inline void adjust_heap(T* first, long hole, long len, T value, Less comp) {
  const long top = hole;
  long second = hole;
  while (second < (len - 1) / 2) {
    second = 2 * (second + 1);
    if (comp(first[second], first[second - 1])) second--;
    first[hole] = first[second];
    hole = second;
  }
  if ((len & 1) == 0 && second == (len - 2) / 2) {
    second = 2 * (second + 1);
    first[hole] = first[second - 1];
    hole = second - 1;
  }
  push_heap_<T, Less>(first, hole, top, value, comp);
}

template <class T, class Less>
LM_HD inline void make_heap_(T* first, T* last, Less comp) {
  const long len = last - first;
  if (len < 2) return;
  long parent = (len - 2) / 2;
  while (true) {
    T value = first[parent];
    adjust_heap<T, Less>(first, parent, len, value, comp);
    if (parent == 0) return;
    parent--;
  }
}

template <class T, class Less>
LM_HD inline void pop_heap_(T* first, T* last, T* result, Less comp) {
  T value = *result;
  *result = *first;
  adjust_heap<T, Less>(first, 0, (long)(last - first), value, comp);
}

template <class T, class Less>
LM_HD inline void partial_sort_full(T* first, T* last, Less comp) {
  // __heap_select(first, last, last) == __make_heap; then __sort_heap
  make_heap_<T, Less>(first, last, comp);
  while (last - first > 1) {
    --last;
    pop_heap_<T, Less>(first, last, last, comp);
  }
}

// ---- insertion sorts
template <class T, class Less>
LM_HD inline void unguarded_linear_insert(T* last, Less comp) {
  T val = *last;
  T* next = last - 1;
  while (comp(val, *next)) {
    *last = *next;
    last = next;
    --next;
  }
  *last = val;
}

template <class T, class Less>
LM_HD inline void insertion_sort(T* first, T* last, Less comp) {
  if (first == last) return;
  for (T* i = first + 1; i != last; ++i) {
    if (comp(*i, *first)) {
      T val = *i;
      for (T* p = i; p != first; --p) *p = *(p - 1);  // move_backward
      *first = val;
    } else {
      unguarded_linear_insert<T, Less>(i, comp);
    }
  }
}

enum { kThreshold = 16 };

template <class T, class Less>
LM_HD inline void final_insertion_sort(T* first, T* last, Less comp) {
  if (last - first > kThreshold) {
    insertion_sort<T, Less>(first, first + kThreshold, comp);
    for (T* i = first + kThreshold; i != last; ++i) unguarded_linear_insert<T, Less>(i, comp);
  } else {
    insertion_sort<T, Less>(first, last, comp);
  }
}

LM_HD inline int lg_(long n) {
  int r = 0;
  while (n > 1) {
    n >>= 1;
    ++r;
  }
  return r;  // floor(log2 n) == std::__lg
}

// __introsort_loop without recursion: the recursive call on [cut, last) is
// pushed on an explicit stack and processed before the loop continues on
// [first, cut) — the same visiting order as the recursive original.  The
// stack (kStackInts ints: first, last, depth, cut per frame; depth <=
// 2*lg(n)+1 <= 64 frames) is caller-provided so device code can keep it in
// LDS instead of per-lane scratch.
enum { kStackFrames = 66, kStackInts = 4 * kStackFrames };

template <class T, class Less>
LM_HD inline void introsort_loop(T* base, int first, int last, int depth_limit, Less comp, int* stk) {
  int sp = 0;
  auto push = [&](int f, int l, int d) {
    stk[4 * sp + 0] = f;
    stk[4 * sp + 1] = l;
    stk[4 * sp + 2] = d;
    stk[4 * sp + 3] = -1;  // cut (set once the frame partitions)
    ++sp;
  };
  push(first, last, depth_limit);
  while (sp > 0) {
    int* fr = stk + 4 * (sp - 1);
    if (fr[3] >= 0) {  // returned from the recursive call on [cut, last)
      fr[1] = fr[3];   // __last = __cut
      fr[3] = -1;
    }
    if (fr[1] - fr[0] > kThreshold) {
      if (fr[2] == 0) {
        partial_sort_full<T, Less>(base + fr[0], base + fr[1], comp);
        --sp;
        continue;
      }
      --fr[2];
      T* cut = unguarded_partition_pivot<T, Less>(base + fr[0], base + fr[1], comp);
      fr[3] = (int)(cut - base);
      push(fr[3], fr[1], fr[2]);
    } else {
      --sp;
    }
  }
}

template <class T, class Less>
LM_HD inline void std_sort(T* first, T* last, Less comp, int* stk) {
  if (first != last) {
    introsort_loop<T, Less>(first, 0, (int)(last - first), lg_((long)(last - first)) * 2, comp, stk);
    final_insertion_sort<T, Less>(first, last, comp);
  }
}

template <class T, class Less>
inline void std_sort(T* first, T* last, Less comp) {  // host convenience
  int stk[kStackInts];
  std_sort<T, Less>(first, last, comp, stk);
}

// ---- level-order formulation (for parallel execution)
//
// __introsort_loop only ever works on disjoint sub-ranges, and what it does to
// a range depends on the range's contents and depth alone, so the ranges can
// be processed level by level (in any order within a level) with the same
// result.  The final insertion sort never moves an element across the
// boundary of a leaf range (partitioning leaves every left-part element
// !(right < left)), so it equals an insertion sort of each leaf on its own.
// A leaf is a range of <= kThreshold elements or one heap-sorted at depth 0.
//
// process_range: returns true and the cut when the range was partitioned
// (children [first, cut) and [cut, last), both with depth - 1), false when it
// is a leaf.
template <class T, class Less>
LM_HD inline bool process_range(T* base, int first, int last, int depth, Less comp, int* cut) {
  if (last - first <= kThreshold) return false;
  if (depth == 0) {
    partial_sort_full<T, Less>(base + first, base + last, comp);
    return false;
  }
  *cut = (int)(unguarded_partition_pivot<T, Less>(base + first, base + last, comp) - base);
  return true;
}

template <class T, class Less>
inline void std_sort_levels(T* a, int n, Less comp, int depth0 = -1) {  // host reference of the level-order form
  if (n <= 0) return;
  int cur[3 * 4096], nxt[3 * 4096];
  static thread_local unsigned char leaf[1 << 20];
  for (int i = 0; i < n; ++i) leaf[i] = 0;
  int qn = 1;
  cur[0] = 0;
  cur[1] = n;
  cur[2] = depth0 >= 0 ? depth0 : 2 * lg_(n);
  while (qn > 0) {
    int nn = 0;
    for (int r = qn - 1; r >= 0; --r) {  // any order within a level
      int cut = 0;
      if (process_range<T, Less>(a, cur[3 * r], cur[3 * r + 1], cur[3 * r + 2], comp, &cut)) {
        const int d = cur[3 * r + 2] - 1;
        nxt[3 * nn] = cur[3 * r];
        nxt[3 * nn + 1] = cut;
        nxt[3 * nn + 2] = d;
        nxt[3 * nn + 3] = cut;
        nxt[3 * nn + 4] = cur[3 * r + 1];
        nxt[3 * nn + 5] = d;
        nn += 2;
      } else {
        leaf[cur[3 * r]] = 1;
      }
    }
    for (int k = 0; k < 3 * nn; ++k) cur[k] = nxt[k];
    qn = nn;
  }
  for (int i = n - 1; i >= 0; --i)  // leaves in any order
    if (leaf[i]) {
      int e = i + 1;
      while (e < n && !leaf[e]) ++e;
      insertion_sort<T, Less>(a + i, a + e, comp);
    }
}

}  // namespace lm_sort

#endif  // LM_INTROSORT_H
