// Option A's call pattern in C++: T threads call
// csm_fast2d_match_full_submap on shared matchers concurrently, as the
// reference's ThreadPool runs one MatchFullSubmap task per (node, submap) pair
// (constraint_builder_2d.cc:100-111, :213-215). The C2 world (500 nodes x 50
// submaps of 400 x 400 cells, 1080 beams, bench.py's seed), pyramids built
// once. Prints one JSON line: pairs/s per thread count, without the Python
// GIL that bounds bench.py's threaded leg.
//   built by cartographer-1_amd/csrc/Makefile (tools target)
//   usage: dropin_threads [calls] [min_score] [--check]
// --check: the threading contract test (tests/test_threading_gpu.py): 200
// pairs matched on one thread, then the same pairs from 16 threads at once
// (each pair twice); every concurrent result must equal the single-threaded
// one bit for bit. Exit status 1 on any difference.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "csm_amd.h"
#include "csm_synth.h"

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 2000;
  const float min_score = argc > 2 ? static_cast<float>(std::atof(argv[2])) : 0.55f;
  csm_synth2d_config cfg;
  csm_synth2d_default_config(&cfg);  // 500 nodes, 50 submaps, 400 cells, 1080 beams, seed 20250127
  csm_synth2d* w = nullptr;
  if (csm_synth2d_create(&cfg, &w) != 0) return 2;
  const int nodes = csm_synth2d_num_nodes(w), submaps = csm_synth2d_num_submaps(w);
  const int64_t* off = csm_synth2d_point_offsets(w);
  const float* pts = csm_synth2d_points(w);
  const double* smax = csm_synth2d_submap_max(w);
  const uint16_t* cells = csm_synth2d_submap_cells(w);
  csm_context* ctx = nullptr;
  if (csm_context_create(0, &ctx) != CSM_OK) return 3;
  // bench.py's C2 options: FastCorrelativeScanMatcherOptions2D(7.0, 30 deg, 7).
  const csm_fast2d_options opts{7.0, 30.0 * M_PI / 180.0, 7, 0};
  const float min_cost = 1.f - 0.9f, max_cost = 1.f - 0.1f;  // kMin/kMaxCorrespondenceCost
  std::vector<csm_fast2d*> m(submaps, nullptr);
  const int c = cfg.submap_cells;
  for (int s = 0; s < submaps; ++s) {
    const csm_map_limits lim{cfg.resolution, smax[2 * s], smax[2 * s + 1], c, c};
    if (csm_fast2d_create(ctx, &lim, cells + static_cast<size_t>(s) * c * c, min_cost, max_cost,
                          &opts, &m[s]) != CSM_OK)
      return 4;
  }
  auto run = [&](int threads, int n) {
    std::atomic<int> next{0}, errors{0};
    std::vector<std::thread> pool;
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t)
      pool.emplace_back([&] {
        for (int j; (j = next.fetch_add(1)) < n;) {
          const int node = j % nodes;
          float score = 0.f;
          csm_pose2d pose{};
          const int rc = csm_fast2d_match_full_submap(
              m[j % submaps], pts + 3 * off[node], static_cast<int32_t>(off[node + 1] - off[node]),
              min_score, &score, &pose);
          if (rc < 0) errors.fetch_add(1);
        }
      });
    for (auto& th : pool) th.join();
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return std::make_pair(n / s, errors.load());
  };
  if (argc > 3 && std::string(argv[3]) == "--check") {
    struct R {
      int rc;
      float score;
      csm_pose2d pose;
    };
    const int n = 200;
    auto one = [&](int j) {
      const int node = (7 * j) % nodes;
      R r{0, 0.f, {0., 0., 0.}};
      r.rc = csm_fast2d_match_full_submap(m[j % submaps], pts + 3 * off[node],
                                          static_cast<int32_t>(off[node + 1] - off[node]), min_score,
                                          &r.score, &r.pose);
      return r;
    };
    std::vector<R> ref(n);
    for (int j = 0; j < n; ++j) ref[j] = one(j);
    std::atomic<int> next{0}, bad{0}, matched{0};
    std::vector<std::thread> pool;
    for (int t = 0; t < 16; ++t)
      pool.emplace_back([&] {
        for (int k; (k = next.fetch_add(1)) < 2 * n;) {
          const int j = k % n;
          const R r = one(j);
          if (r.rc == CSM_OK) matched.fetch_add(1);
          if (r.rc != ref[j].rc || (r.rc == CSM_OK && (r.score != ref[j].score || r.pose.x != ref[j].pose.x ||
                                                      r.pose.y != ref[j].pose.y ||
                                                      r.pose.theta != ref[j].pose.theta)))
            bad.fetch_add(1);
        }
      });
    for (auto& th : pool) th.join();
    std::printf("{\"check_pairs\": %d, \"concurrent_calls\": %d, \"matched\": %d, \"mismatches\": %d}\n", n,
                2 * n, matched.load(), bad.load());
    for (csm_fast2d* x : m) csm_fast2d_destroy(x);
    csm_context_destroy(ctx);
    csm_synth2d_destroy(w);
    return bad.load() == 0 && matched.load() > 0 ? 0 : 1;
  }
  std::printf("{\"calls\": %d, \"pairs_per_s\": {", calls);
  bool first = true;
  for (int threads : {1, 2, 4, 8, 16}) {
    run(threads, 4 * threads);  // warm-up: one call context per thread
    const auto r = run(threads, calls);
    std::printf("%s\"%d\": %.1f", first ? "" : ", ", threads, r.first);
    first = false;
    if (r.second) std::fprintf(stderr, "dropin_threads: %d errors at %d threads\n", r.second, threads);
  }
  std::printf("}, \"world\": \"C2 (500 nodes x 50 submaps, 400 x 400 cells)\", \"min_score\": %.2f}\n",
              min_score);
  for (csm_fast2d* x : m) csm_fast2d_destroy(x);
  csm_context_destroy(ctx);
  csm_synth2d_destroy(w);
  return 0;
}
