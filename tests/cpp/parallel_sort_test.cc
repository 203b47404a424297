// csm::IntroSort (cartographer-1_amd/csrc/parallel_sort.h) against std::sort:
// the same permutation, element for element, for the lists tie resolution
// sorts (float scores with many exact ties, int32 indices, descending) and
// for adversarial shapes (sorted, reversed, constant, organ pipe, sawtooth),
// on 1 to 16 threads. Prints "parallel_sort OK" on success.
#include "../../cartographer-1_amd/csrc/parallel_sort.h"

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

using Elem = std::pair<float, int32_t>;

static bool Check(const std::vector<float>& keys, int threads, const char* what) {
  const size_t n = keys.size();
  std::vector<Elem> a(n), b;
  for (size_t i = 0; i < n; ++i) a[i] = {keys[i], static_cast<int32_t>(i)};
  b = a;
  auto comp = [](const Elem& x, const Elem& y) { return x.first > y.first; };
  std::sort(a.begin(), a.end(), comp);
  csm::IntroSort(b.data(), b.data() + n, comp, threads);
  for (size_t i = 0; i < n; ++i) {
    if (a[i].second != b[i].second) {
      std::printf("MISMATCH %s n=%zu threads=%d at %zu: %d vs %d\n", what, n, threads, i,
                  a[i].second, b[i].second);
      return false;
    }
  }
  return true;
}

int main() {
  std::mt19937 rng(12345);
  int cases = 0;
  bool ok = true;
  const size_t sizes[] = {0, 1, 2, 15, 16, 17, 33, 100, 1000, 16385, 70000, 300000, 800000};
  for (size_t n : sizes) {
    for (int levels : {1, 3, 40, 1000, 0}) {  // distinct score values (0: continuous)
      std::vector<float> k(n);
      std::uniform_int_distribution<int> u(0, std::max(levels - 1, 0));
      std::uniform_real_distribution<float> f(0.f, 1.f);
      for (auto& v : k) v = levels ? 0.1f + 0.8f * u(rng) / std::max(levels, 1) : f(rng);
      for (int threads : {1, 2, 3, 8, 16}) {
        ok &= Check(k, threads, "random");
        ++cases;
      }
    }
    // Shapes that stress the pivot choice.
    std::vector<std::vector<float>> shapes(5, std::vector<float>(n));
    for (size_t i = 0; i < n; ++i) {
      shapes[0][i] = static_cast<float>(i);
      shapes[1][i] = static_cast<float>(n - i);
      shapes[2][i] = 0.5f;
      shapes[3][i] = static_cast<float>(std::min(i, n - i));
      shapes[4][i] = static_cast<float>(i % 64);
    }
    for (auto& s : shapes)
      for (int threads : {1, 8}) {
        ok &= Check(s, threads, "shape");
        ++cases;
      }
  }
  // Timing at the size tie resolution meets (768k top-level candidates).
  {
    const size_t n = 768000;
    std::vector<Elem> a(n);
    std::uniform_int_distribution<int> u(0, 2000);
    for (size_t i = 0; i < n; ++i) a[i] = {u(rng) / 2000.f, static_cast<int32_t>(i)};
    auto comp = [](const Elem& x, const Elem& y) { return x.first > y.first; };
    for (int threads : {1, 8}) {
      auto b = a;
      const auto t0 = std::chrono::steady_clock::now();
      csm::IntroSort(b.data(), b.data() + n, comp, threads);
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      std::printf("n=%zu threads=%d: %.2f ms\n", n, threads, ms);
    }
  }
  if (!ok) return 1;
  std::printf("parallel_sort OK (%d cases)\n", cases);
  return 0;
}
