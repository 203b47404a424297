// The permutation of std::sort, computed on several threads.
//
// Tie resolution needs the order in which the reference's std::sort (an
// introsort, not stable) leaves equally scored lowest-resolution candidates
// (fast_correlative_scan_matcher_2d.cc:276-312, sorted with
// std::greater<Candidate2D>). That order depends on every partition step, so
// the sort cannot be swapped for another algorithm; but the two sides of a
// partition are sorted independently of each other, so they can be sorted on
// different threads without changing a single comparison.
//
// IntroSort restates libstdc++'s std::sort (GCC 11, bits/stl_algo.h:
// __introsort_loop, __unguarded_partition_pivot, __final_insertion_sort):
// median of (first + 1, middle, last - 1) moved to first, unguarded Hoare
// partition, ranges of <= 16 left to the final insertion sort, heap sort
// (std::partial_sort over the whole range) once the depth limit 2 lg n is
// spent. tests/cpp/parallel_sort_test.cc checks it against std::sort.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstddef>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace csm {
namespace sort_detail {

constexpr std::ptrdiff_t kThreshold = 16;      // _S_threshold
constexpr std::ptrdiff_t kParallelGrain = 1 << 14;  // smallest range handed to another thread

template <typename T, typename Comp>
void MedianToFirst(T* result, T* a, T* b, T* c, Comp& comp) {
  if (comp(*a, *b)) {
    if (comp(*b, *c)) std::iter_swap(result, b);
    else if (comp(*a, *c)) std::iter_swap(result, c);
    else std::iter_swap(result, a);
  } else if (comp(*a, *c)) {
    std::iter_swap(result, a);
  } else if (comp(*b, *c)) {
    std::iter_swap(result, c);
  } else {
    std::iter_swap(result, b);
  }
}

template <typename T, typename Comp>
T* PartitionPivot(T* first, T* last, Comp& comp) {
  MedianToFirst(first, first + 1, first + (last - first) / 2, last - 1, comp);
  T* pivot = first;
  T* lo = first + 1;
  T* hi = last;
  while (true) {
    while (comp(*lo, *pivot)) ++lo;
    --hi;
    while (comp(*pivot, *hi)) --hi;
    if (!(lo < hi)) return lo;
    std::iter_swap(lo, hi);
    ++lo;
  }
}

template <typename T, typename Comp>
void IntroLoop(T* first, T* last, long depth, Comp& comp) {
  while (last - first > kThreshold) {
    if (depth == 0) {
      std::partial_sort(first, last, last, comp);
      return;
    }
    --depth;
    T* cut = PartitionPivot(first, last, comp);
    IntroLoop(cut, last, depth, comp);
    last = cut;
  }
}

// The sequential loop's steps for [first, last) on a pool of threads: a
// range above the grain is cut, its right side queued for any idle thread and
// its left side cut again here; ranges at or below the grain (or out of
// depth) finish with IntroLoop. Each range sees exactly the partitions the
// sequential recursion applies to it, whichever thread runs them.
template <typename T, typename Comp>
void IntroTask(T* first, T* last, long depth, Comp comp, int threads) {
  struct Range {
    T* first;
    T* last;
    long depth;
  };
  if (threads <= 1) {
    IntroLoop(first, last, depth, comp);
    return;
  }
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Range> queue{{first, last, depth}};
  int pending = 1;  // ranges queued or in progress
  auto work = [&] {
    Comp c = comp;
    std::unique_lock<std::mutex> lock(mu);
    while (true) {
      cv.wait(lock, [&] { return !queue.empty() || pending == 0; });
      if (queue.empty()) return;
      Range r = queue.back();
      queue.pop_back();
      lock.unlock();
      while (r.depth > 0 && r.last - r.first > kParallelGrain) {
        --r.depth;
        T* cut = PartitionPivot(r.first, r.last, c);
        {
          std::lock_guard<std::mutex> g(mu);
          queue.push_back({cut, r.last, r.depth});
          ++pending;
        }
        cv.notify_one();
        r.last = cut;
      }
      IntroLoop(r.first, r.last, r.depth, c);
      lock.lock();
      if (--pending == 0) cv.notify_all();
    }
  };
  std::vector<std::thread> pool;
  for (int i = 1; i < threads; ++i) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
}

template <typename T, typename Comp>
void LinearInsert(T* last, Comp& comp) {
  T val = std::move(*last);
  T* next = last - 1;
  while (comp(val, *next)) {
    *last = std::move(*next);
    last = next;
    --next;
  }
  *last = std::move(val);
}

template <typename T, typename Comp>
void InsertionSort(T* first, T* last, Comp& comp) {
  if (first == last) return;
  for (T* i = first + 1; i != last; ++i) {
    if (comp(*i, *first)) {
      T val = std::move(*i);
      std::move_backward(first, i, i + 1);
      *first = std::move(val);
    } else {
      LinearInsert(i, comp);
    }
  }
}

}  // namespace sort_detail

// fn(lo, hi) over [0, n) in up to `threads` contiguous pieces, one thread each.
template <typename Fn>
void ParallelRanges(std::ptrdiff_t n, int threads, Fn fn) {
  const std::ptrdiff_t pieces =
      std::max<std::ptrdiff_t>(1, std::min<std::ptrdiff_t>(threads, n / sort_detail::kParallelGrain));
  if (pieces <= 1) {
    fn(std::ptrdiff_t{0}, n);
    return;
  }
  std::vector<std::thread> pool;
  for (std::ptrdiff_t p = 1; p < pieces; ++p) pool.emplace_back(fn, n * p / pieces, n * (p + 1) / pieces);
  fn(std::ptrdiff_t{0}, n / pieces);
  for (auto& t : pool) t.join();
}

// Sorts [first, last) into exactly the order std::sort(first, last, comp)
// gives, using up to `threads` threads.
template <typename T, typename Comp>
void IntroSort(T* first, T* last, Comp comp, int threads = 1) {
  using namespace sort_detail;
  const std::ptrdiff_t n = last - first;
  if (n == 0) return;
  long lg = 0;
  while ((std::ptrdiff_t{1} << (lg + 1)) <= n) ++lg;  // std::__lg(n)
  IntroTask(first, last, 2 * lg, comp, std::max(threads, 1));
  // __final_insertion_sort, on one thread (a linear pass: every element is
  // within its <= 16-element range of its place).
  if (n > kThreshold) {
    InsertionSort(first, first + kThreshold, comp);
    for (T* i = first + kThreshold; i != last; ++i) LinearInsert(i, comp);
  } else {
    InsertionSort(first, last, comp);
  }
}

}  // namespace csm
