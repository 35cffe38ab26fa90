// Go 1.16 `sort.Sort` ordering, reproduced for placement parity.
//
// The reference scheduler (Go 1.16 toolchain, reference Dockerfile:1) orders
// candidate devices with `sort.Sort(SortableGPUs)` (reference
// pkg/dealer/rater.go:80-89, 133-142). `sort.Sort` is NOT stable: for n <= 12
// it runs one gap-6 pass followed by insertion sort, and for larger n an
// introsort (median-of-three / Tukey ninther pivot, heapsort fallback).  The
// exact permutation decides which device wins a tie, so parity mode
// (`compat=go116`) must reproduce it bit for bit; SURVEY.md Appendix B.2 gives
// the worked example where a stable sort picks a different GPU.
//
// The algorithm below is written against the documented behaviour of the
// Go 1.16 standard library (BSD-licensed), expressed over index callbacks so
// the same code sorts device arrays and demand arrays.
#pragma once

#include <cstddef>

namespace nanogpu {
namespace gosort {

template <class Less, class Swap>
struct Sorter {
  Less less;
  Swap swap;

  void insertion(int a, int b) {
    for (int i = a + 1; i < b; ++i)
      for (int j = i; j > a && less(j, j - 1); --j) swap(j, j - 1);
  }

  void sift_down(int lo, int hi, int first) {
    int root = lo;
    for (;;) {
      int child = 2 * root + 1;
      if (child >= hi) return;
      if (child + 1 < hi && less(first + child, first + child + 1)) ++child;
      if (!less(first + root, first + child)) return;
      swap(first + root, first + child);
      root = child;
    }
  }

  void heap(int a, int b) {
    const int first = a, hi = b - a;
    for (int i = (hi - 1) / 2; i >= 0; --i) sift_down(i, hi, first);
    for (int i = hi - 1; i >= 0; --i) {
      swap(first, first + i);
      sift_down(0, i, first);
    }
  }

  void median3(int m1, int m0, int m2) {
    if (less(m1, m0)) swap(m1, m0);
    if (less(m2, m1)) {
      swap(m2, m1);
      if (less(m1, m0)) swap(m1, m0);
    }
  }

  void pivot(int lo, int hi, int* midlo, int* midhi) {
    const int m = static_cast<int>(static_cast<unsigned>(lo + hi) >> 1);
    if (hi - lo > 40) {
      const int s = (hi - lo) / 8;
      median3(lo, lo + s, lo + 2 * s);
      median3(m, m - s, m + s);
      median3(hi - 1, hi - 1 - s, hi - 1 - 2 * s);
    }
    median3(lo, m, hi - 1);

    const int p = lo;
    int a = lo + 1, c = hi - 1;
    while (a < c && less(a, p)) ++a;
    int b = a;
    for (;;) {
      while (b < c && !less(p, b)) ++b;
      while (b < c && less(p, c - 1)) --c;
      if (b >= c) break;
      swap(b, c - 1);
      ++b;
      --c;
    }
    bool protect = hi - c < 5;
    if (!protect && hi - c < (hi - lo) / 4) {
      int dups = 0;
      if (!less(p, hi - 1)) {
        swap(c, hi - 1);
        ++c;
        ++dups;
      }
      if (!less(b - 1, p)) {
        --b;
        ++dups;
      }
      if (!less(m, p)) {
        swap(m, b - 1);
        --b;
        ++dups;
      }
      protect = dups > 1;
    }
    if (protect) {
      for (;;) {
        while (a < b && !less(b - 1, p)) --b;
        while (a < b && less(a, p)) ++a;
        if (a >= b) break;
        swap(a, b - 1);
        ++a;
        --b;
      }
    }
    swap(p, b - 1);
    *midlo = b - 1;
    *midhi = c;
  }

  void quick(int a, int b, int depth) {
    while (b - a > 12) {
      if (depth == 0) {
        heap(a, b);
        return;
      }
      --depth;
      int mlo, mhi;
      pivot(a, b, &mlo, &mhi);
      if (mlo - a < b - mhi) {
        quick(a, mlo, depth);
        a = mhi;
      } else {
        quick(mhi, b, depth);
        b = mlo;
      }
    }
    if (b - a > 1) {
      for (int i = a + 6; i < b; ++i)
        if (less(i, i - 6)) swap(i, i - 6);
      insertion(a, b);
    }
  }
};

// Sorts positions [0, n) using the caller's less(i, j) / swap(i, j).
template <class Less, class Swap>
inline void sort(int n, Less less, Swap swap) {
  int depth = 0;
  for (int i = n; i > 0; i >>= 1) ++depth;
  Sorter<Less, Swap> s{less, swap};
  s.quick(0, n, depth * 2);
}

}  // namespace gosort
}  // namespace nanogpu
