// Option A in 3D from C++ threads: T threads call
// csm_fast3d_match_full_submap on shared matchers concurrently, as the
// reference's ThreadPool runs one MatchFullSubmap task per (node, submap)
// pair (constraint_builder_3d.cc:200-230, :239-241). A slice of the C5 world
// (bench.py's seed + 5, pose_graph.lua's 3D options, min_score 0.6), grids
// and pyramids built once. Prints one JSON line: pairs/s per thread count
// (no Python GIL, which bounds bench.py's threaded leg), the same pairs'
// batch rate (csm_fast3d_match_batch) and the number of single-call results
// that differ from the batch's (must be 0).
//   built by cartographer-1_amd/csrc/Makefile
//   usage: dropin_threads3d [calls] [submaps] [nodes]
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "csm_amd.h"
#include "csm_synth.h"

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 4000;
  csm_synth3d_config cfg;
  csm_synth3d_default_config(&cfg);
  cfg.seed = 20250127 + 5;
  cfg.num_submaps = argc > 2 ? std::atoi(argv[2]) : 8;
  cfg.num_nodes = argc > 3 ? std::atoi(argv[3]) : 200;
  csm_synth3d* w = nullptr;
  if (csm_synth3d_create(&cfg, &w) != 0) return 2;
  const int S = cfg.num_submaps, N = cfg.num_nodes, H = cfg.histogram_size;
  csm_context* ctx = nullptr;
  if (csm_context_create(0, &ctx) != CSM_OK) return 3;
  // FastCorrelativeScanMatcherOptions3D as bench.py's C5 (pose_graph.lua).
  const csm_fast3d_options o{8, 3, 0.77, 0.55, 5.0, 1.0, 15.0 * M_PI / 180.0};
  std::vector<csm_hybrid_grid*> grids;
  std::vector<csm_fast3d*> m(S, nullptr);
  for (int s = 0; s < S; ++s) {
    csm_hybrid_grid* g[2] = {nullptr, nullptr};
    for (int k = 0; k < 2; ++k) {
      const int64_t n = csm_synth3d_grid(w, s, k, nullptr, nullptr, 0);
      std::vector<int32_t> ijk(3 * n);
      std::vector<uint16_t> v(n);
      csm_synth3d_grid(w, s, k, ijk.data(), v.data(), n);
      const float res = static_cast<float>(k == 0 ? cfg.high_resolution : cfg.low_resolution);
      if (csm_hybrid_grid_create(ctx, res, ijk.data(), v.data(), n, 0, &g[k]) != CSM_OK) return 4;
      grids.push_back(g[k]);
    }
    std::vector<float> hist(H);
    csm_synth3d_submap_histogram(w, s, hist.data());
    if (csm_fast3d_create(ctx, g[0], g[1], hist.data(), H, &o, &m[s]) != CSM_OK) return 5;
  }
  std::vector<std::vector<float>> hi(N), lo(N), hist(N);
  std::vector<csm_node3d> nodes(N);
  std::vector<std::array<double, 4>> rot(N);
  const double* poses = csm_synth3d_node_poses(w);
  for (int i = 0; i < N; ++i) {
    for (int k = 1; k <= 2; ++k) {
      auto& c = k == 1 ? hi[i] : lo[i];
      c.resize(3 * csm_synth3d_cloud(w, i, k, nullptr, 0));
      csm_synth3d_cloud(w, i, k, c.data(), static_cast<int64_t>(c.size() / 3));
    }
    hist[i].resize(H);
    csm_synth3d_node_histogram(w, i, hist[i].data());
    nodes[i] = csm_node3d{hi[i].data(), static_cast<int32_t>(hi[i].size() / 3), lo[i].data(),
                          static_cast<int32_t>(lo[i].size() / 3), hist[i].data(), H,
                          {1.0, 0.0, 0.0, 0.0}};
    const double yaw = poses[4 * i + 3];
    rot[i] = {std::cos(0.5 * yaw), 0.0, 0.0, std::sin(0.5 * yaw)};  // SyntheticWorld3D.node_rotation
  }
  const double ident[4] = {1.0, 0.0, 0.0, 0.0};
  const float min_score = 0.6f;
  std::vector<int> ps(calls), pn(calls);
  unsigned seed = 3;
  for (int j = 0; j < calls; ++j) {
    seed = seed * 1103515245u + 12345u;
    ps[j] = static_cast<int>((seed >> 8) % S);
    seed = seed * 1103515245u + 12345u;
    pn[j] = static_cast<int>((seed >> 8) % N);
  }
  // The same pairs as one batch: the reference results and the batch rate.
  std::vector<csm_pair3d> pairs(calls);
  for (int j = 0; j < calls; ++j) {
    csm_pair3d& p = pairs[j];
    std::memset(&p, 0, sizeof(p));
    p.submap = ps[j];
    p.node = pn[j];
    p.full_submap = 1;
    p.min_score = min_score;
    for (int k = 0; k < 4; ++k) {
      p.node_pose.q[k] = rot[pn[j]][k];
      p.submap_pose.q[k] = ident[k];
    }
  }
  std::vector<csm_result3d> ref(calls);
  if (csm_fast3d_match_batch(ctx, m.data(), S, nodes.data(), N, pairs.data(), calls, ref.data()) < 0)
    return 6;
  const auto b0 = std::chrono::steady_clock::now();
  if (csm_fast3d_match_batch(ctx, m.data(), S, nodes.data(), N, pairs.data(), calls, ref.data()) < 0)
    return 6;
  const double batch_rate =
      calls / std::chrono::duration<double>(std::chrono::steady_clock::now() - b0).count();
  std::atomic<int> mism{0};
  auto run = [&](int threads, int n, bool check) {
    std::atomic<int> next{0};
    std::vector<std::thread> pool;
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t)
      pool.emplace_back([&] {
        for (int j; (j = next.fetch_add(1)) < n;) {
          csm_result3d r{};
          const int rc = csm_fast3d_match_full_submap(m[ps[j]], rot[pn[j]].data(), ident, &nodes[pn[j]],
                                                      min_score, &r);
          if (!check) continue;
          const csm_result3d& e = ref[j];
          bool same = rc == e.status;
          if (same && rc == CSM_OK)
            same = r.score == e.score && r.rotational_score == e.rotational_score &&
                   r.low_resolution_score == e.low_resolution_score &&
                   std::memcmp(&r.pose, &e.pose, sizeof(r.pose)) == 0;
          if (!same) mism.fetch_add(1);
        }
      });
    for (auto& th : pool) th.join();
    return n / std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  };
  std::printf("{\"calls\": %d, \"pairs_per_s\": {", calls);
  bool first = true;
  for (int threads : {1, 4, 8, 16, 32}) {
    run(threads, 4 * threads, false);  // warm-up: call contexts
    const double r = run(threads, threads == 1 ? calls / 8 : calls, true);
    std::printf("%s\"%d\": %.1f", first ? "" : ", ", threads, r);
    first = false;
  }
  std::printf("}, \"batch_pairs_per_s\": %.1f, \"mismatches_vs_batch\": %d, \"world\": "
              "\"C5 slice (%d nodes x %d submaps), min_score 0.6\"}\n",
              batch_rate, mism.load(), N, S);
  for (csm_fast3d* x : m) csm_fast3d_destroy(x);
  for (csm_hybrid_grid* g : grids) csm_hybrid_grid_destroy(g);
  csm_context_destroy(ctx);
  csm_synth3d_destroy(w);
  return mism.load() == 0 ? 0 : 1;
}
