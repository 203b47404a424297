// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// extern "C" surface of the oracle for tests/ (ctypes) and bench.py's
// cpu_baseline leg. Mirrors the product C-ABI (include/csm_amd.h) argument by
// argument so parity tests call both the same way.
//
// oracle_fast2d_match_pairs() is the CPU baseline: one (node, submap) pair
// per task on a pool of T std::threads that pull tasks in FIFO order, as
// ConstraintBuilder2D schedules one Task per pair on common::ThreadPool
// (constraint_builder_2d.cc:102-111, thread_pool.cc:80-106).

#include <atomic>
#include <cmath>
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

#include "csm_oracle.h"

using namespace oracle;

namespace {
PointCloud ToCloud(const float* xyz, int32_t n) {
  PointCloud c(static_cast<size_t>(n));
  for (int32_t i = 0; i < n; ++i) c[i] = Vec3f{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
  return c;
}
MapLimits ToLimits(double res, double max_x, double max_y, int nx, int ny) {
  MapLimits l;
  l.resolution = res;
  l.max_x = max_x;
  l.max_y = max_y;
  l.cells = CellLimits{nx, ny};
  return l;
}
}  // namespace

extern "C" {

int oracle_version() { return 1; }

void* oracle_fast2d_create(double res, double max_x, double max_y, int32_t nx,
                           int32_t ny, const uint16_t* cells, double lin,
                           double ang, int32_t depth) {
  const MapLimits l = ToLimits(res, max_x, max_y, nx, ny);
  ProbabilityGrid g(l, std::vector<uint16_t>(cells, cells + static_cast<size_t>(nx) * ny));
  FastOptions2D o;
  o.linear_search_window = lin;
  o.angular_search_window = ang;
  o.branch_and_bound_depth = depth;
  return new FastCorrelativeScanMatcher2D(g, o);
}

void oracle_fast2d_destroy(void* h) { delete static_cast<FastCorrelativeScanMatcher2D*>(h); }

// Copies precomputation level d (uint8, wide grid) into out (may be null to
// query the size). Returns wide nx * ny.
int64_t oracle_fast2d_level(void* h, int32_t d, uint8_t* out, int32_t* wide_nx,
                            int32_t* wide_ny) {
  const auto* m = static_cast<FastCorrelativeScanMatcher2D*>(h);
  const PrecomputationGrid2D& g = m->Level(d);
  *wide_nx = g.wide_limits().num_x_cells;
  *wide_ny = g.wide_limits().num_y_cells;
  if (out) std::copy(g.cells().begin(), g.cells().end(), out);
  return static_cast<int64_t>(g.cells().size());
}

static void FillStats(const MatchStats2D& s, int64_t* stats) {
  if (!stats) return;
  stats[0] = s.lookups;
  stats[1] = s.num_scans;
  stats[2] = s.lowest_resolution_candidates;
  for (int i = 0; i < 13; ++i) stats[3 + i] = s.candidates_per_level[i];
}

// pose_out: x, y, theta. stats (optional, 16 int64): lookups, num_scans,
// lowest-resolution candidates, candidates scored per level 0..12.
int32_t oracle_fast2d_match_full_submap(void* h, const float* xyz, int32_t n,
                                        float min_score, float* score,
                                        double* pose_out, int64_t* stats) {
  const auto* m = static_cast<FastCorrelativeScanMatcher2D*>(h);
  Rigid2d pose;
  MatchStats2D s;
  const bool ok = m->MatchFullSubmap(ToCloud(xyz, n), min_score, score, &pose, &s);
  FillStats(s, stats);
  if (ok) {
    pose_out[0] = pose.tx;
    pose_out[1] = pose.ty;
    pose_out[2] = pose.angle;
  }
  return ok ? 0 : 1;
}

int32_t oracle_fast2d_match(void* h, const double* initial, const float* xyz,
                            int32_t n, float min_score, float* score,
                            double* pose_out, int64_t* stats) {
  const auto* m = static_cast<FastCorrelativeScanMatcher2D*>(h);
  Rigid2d init;
  init.tx = initial[0];
  init.ty = initial[1];
  init.angle = initial[2];
  Rigid2d pose;
  MatchStats2D s;
  const bool ok = m->Match(init, ToCloud(xyz, n), min_score, score, &pose, &s);
  FillStats(s, stats);
  if (ok) {
    pose_out[0] = pose.tx;
    pose_out[1] = pose.ty;
    pose_out[2] = pose.angle;
  }
  return ok ? 0 : 1;
}

// Level-d score of one candidate exactly as ScoreCandidates computes it
// (integer sum + ToScore), for tie checks: the candidate is given by its
// window (full_submap or initial pose), rotation index and offsets.
int32_t oracle_fast2d_score_candidate(void* h, int32_t full_submap,
                                      const double* initial, double lin,
                                      double ang, const float* xyz, int32_t n,
                                      int32_t scan_index, int32_t x_off,
                                      int32_t y_off, int32_t depth,
                                      int32_t* sum_out, float* score_out) {
  const auto* m = static_cast<FastCorrelativeScanMatcher2D*>(h);
  const MapLimits& l = m->limits();
  const PointCloud cloud = ToCloud(xyz, n);
  Rigid2d init;
  if (full_submap) {
    lin = 1e6 * l.resolution;
    ang = M_PI;
    const double half = 0.5 * l.resolution;
    init.tx = l.max_x - half * l.cells.num_y_cells;
    init.ty = l.max_y - half * l.cells.num_x_cells;
  } else {
    init.tx = initial[0];
    init.ty = initial[1];
    init.angle = initial[2];
  }
  SearchParameters sp(lin, ang, cloud, l.resolution);
  if (scan_index < 0 || scan_index >= sp.num_scans) return -1;
  Rigid3f pre;
  pre.q = QuatFromAngleAxisF(static_cast<float>(init.angle), 0.f, 0.f, 1.f);
  const auto rotated = GenerateRotatedScans(TransformPointCloud(cloud, pre), sp);
  const auto d = DiscretizeScans(l, rotated, static_cast<float>(init.tx),
                                 static_cast<float>(init.ty));
  const PrecomputationGrid2D& g = m->Level(depth);
  int sum = 0;
  for (const Idx2& xy : d[scan_index]) sum += g.GetValue(Idx2{xy.x + x_off, xy.y + y_off});
  *sum_out = sum;
  *score_out = g.ToScore(sum / static_cast<float>(d[scan_index].size()));
  return 0;
}

// Tie statistics (tests/tools only): the leaves tied at the maximum score
// (up to max_out, as scan, x_off, y_off triples) and the reference's pick.
// Returns the number of tied leaves (0: no match above min_score).
int32_t oracle_fast2d_tie_leaves(void* h, int32_t full_submap, const double* initial,
                                 const float* xyz, int32_t n, float min_score,
                                 int32_t max_out, int32_t* leaves, int32_t* picked) {
  const auto* m = static_cast<FastCorrelativeScanMatcher2D*>(h);
  Rigid2d init;
  if (initial) {
    init.tx = initial[0];
    init.ty = initial[1];
    init.angle = initial[2];
  }
  std::array<int, 3> pick{0, 0, 0};
  const auto ties = m->TiedMaxLeaves(full_submap != 0, init, ToCloud(xyz, n), min_score,
                                     static_cast<size_t>(max_out), &pick);
  for (size_t i = 0; i < ties.size(); ++i)
    for (int k = 0; k < 3; ++k) leaves[3 * i + k] = ties[i][k];
  for (int k = 0; k < 3; ++k) picked[k] = pick[k];
  return static_cast<int32_t>(ties.size());
}

// CPU baseline: pairs (submap index, node index) matched with
// MatchFullSubmap on `threads` workers pulling pairs FIFO. Returns wall
// seconds; matched[i] = 1 on success.
// oracle_fast2d_match_pairs_stats: the same, and per pair (when stats is
// not null) the 16 counters of oracle_fast2d_match_full_submap: lookups
// (GetValue calls, fast_correlative_scan_matcher_2d.cc:319-330), scans,
// lowest-resolution candidates, candidates scored per level 0..12 — the
// reference's work per pair, next to the GPU search's (bench.py work_ratio).
double oracle_fast2d_match_pairs_stats(void* const* submaps, const float* points,
                                       const int64_t* point_offsets,
                                       const int32_t* pair_submap,
                                       const int32_t* pair_node, int64_t num_pairs,
                                       int32_t threads, float min_score, float* scores,
                                       double* poses, int32_t* matched, double* task_seconds,
                                       int64_t* stats) {
  std::vector<PointCloud> clouds;
  // Clouds are materialised per task (TrajectoryNode::Data holds them
  // already in the reference; conversion is outside the timed region).
  int32_t max_node = -1;
  for (int64_t i = 0; i < num_pairs; ++i) max_node = std::max(max_node, pair_node[i]);
  clouds.resize(static_cast<size_t>(max_node + 1));
  for (int32_t n = 0; n <= max_node; ++n)
    clouds[n] = ToCloud(points + 3 * point_offsets[n],
                        static_cast<int32_t>(point_offsets[n + 1] - point_offsets[n]));
  std::atomic<int64_t> next{0};
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (int t = 0; t < std::max(1, threads); ++t)
    pool.emplace_back([&] {
      for (int64_t i = next++; i < num_pairs; i = next++) {
        const auto* m = static_cast<const FastCorrelativeScanMatcher2D*>(submaps[pair_submap[i]]);
        Rigid2d pose;
        float score = 0.f;
        const auto ts = std::chrono::steady_clock::now();
        MatchStats2D st;
        const bool ok = m->MatchFullSubmap(clouds[pair_node[i]], min_score, &score, &pose,
                                           stats ? &st : nullptr);
        if (stats) FillStats(st, stats + 16 * i);
        if (task_seconds)  // per-task time, for the baseline's confidence interval
          task_seconds[i] =
              std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
        matched[i] = ok ? 1 : 0;
        scores[i] = ok ? score : 0.f;
        poses[3 * i] = pose.tx;
        poses[3 * i + 1] = pose.ty;
        poses[3 * i + 2] = pose.angle;
      }
    });
  for (auto& th : pool) th.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

double oracle_fast2d_match_pairs(void* const* submaps, const float* points,
                                 const int64_t* point_offsets,
                                 const int32_t* pair_submap,
                                 const int32_t* pair_node, int64_t num_pairs,
                                 int32_t threads, float min_score, float* scores,
                                 double* poses, int32_t* matched, double* task_seconds) {
  return oracle_fast2d_match_pairs_stats(submaps, points, point_offsets, pair_submap, pair_node,
                                         num_pairs, threads, min_score, scores, poses, matched,
                                         task_seconds, nullptr);
}

// RealTimeCorrelativeScanMatcher2D::Match over a probability grid.
double oracle_rt2d_match(double res, double max_x, double max_y, int32_t nx,
                         int32_t ny, const uint16_t* cells, double lin,
                         double ang, double wt, double wr, const double* initial,
                         const float* xyz, int32_t n, double* pose_out,
                         int64_t* num_candidates) {
  const MapLimits l = ToLimits(res, max_x, max_y, nx, ny);
  ProbabilityGrid g(l, std::vector<uint16_t>(cells, cells + static_cast<size_t>(nx) * ny));
  RealTimeOptions o;
  o.linear_search_window = lin;
  o.angular_search_window = ang;
  o.translation_delta_cost_weight = wt;
  o.rotation_delta_cost_weight = wr;
  Rigid2d init;
  init.tx = initial[0];
  init.ty = initial[1];
  init.angle = initial[2];
  Rigid2d pose;
  const double s = RealTimeCorrelativeScanMatcher2D(o).Match(init, ToCloud(xyz, n), g, &pose,
                                                             num_candidates);
  pose_out[0] = pose.tx;
  pose_out[1] = pose.ty;
  pose_out[2] = pose.angle;
  return s;
}

// Timed RTCSM2D: `reps` Match() calls on one thread; returns seconds per call.
double oracle_rt2d_time(double res, double max_x, double max_y, int32_t nx,
                        int32_t ny, const uint16_t* cells, double lin, double ang,
                        double wt, double wr, const double* initial,
                        const float* xyz, int32_t n, int32_t reps) {
  const MapLimits l = ToLimits(res, max_x, max_y, nx, ny);
  ProbabilityGrid g(l, std::vector<uint16_t>(cells, cells + static_cast<size_t>(nx) * ny));
  RealTimeOptions o;
  o.linear_search_window = lin;
  o.angular_search_window = ang;
  o.translation_delta_cost_weight = wt;
  o.rotation_delta_cost_weight = wr;
  Rigid2d init;
  init.tx = initial[0];
  init.ty = initial[1];
  init.angle = initial[2];
  const PointCloud cloud = ToCloud(xyz, n);
  const RealTimeCorrelativeScanMatcher2D m(o);
  Rigid2d pose;
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; ++r) m.Match(init, cloud, g, &pose);
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() /
         std::max(1, reps);
}

// Discretized scans for (initial pose, search window) — used by tests to
// check the GPU's discretization bit-for-bit. out: num_scans * n int32 pairs.
int32_t oracle_discretize(double res, double max_x, double max_y, int32_t nx,
                          int32_t ny, const double* initial, double lin,
                          double ang, const float* xyz, int32_t n,
                          int32_t sp_from_rotated, int32_t* num_scans,
                          int32_t* bounds, int32_t* out, int64_t out_capacity,
                          double* step) {
  const MapLimits l = ToLimits(res, max_x, max_y, nx, ny);
  const PointCloud cloud = ToCloud(xyz, n);
  Rigid3f pre;
  pre.q = QuatFromAngleAxisF(static_cast<float>(initial[2]), 0.f, 0.f, 1.f);
  const PointCloud rotated = TransformPointCloud(cloud, pre);
  // FastCSM builds SearchParameters from the input cloud (:202-204), RTCSM
  // from the pre-rotated one (real_time_correlative_scan_matcher_2d.cc:128).
  SearchParameters sp(lin, ang, sp_from_rotated ? rotated : cloud, res);
  const auto scans = GenerateRotatedScans(rotated, sp);
  const auto d = DiscretizeScans(l, scans, static_cast<float>(initial[0]),
                                 static_cast<float>(initial[1]));
  *num_scans = sp.num_scans;
  *step = sp.angular_perturbation_step_size;
  if (out == nullptr) return 0;
  if (static_cast<int64_t>(sp.num_scans) * n * 2 > out_capacity) return -1;
  SearchParameters shrunk = sp;
  shrunk.ShrinkToFit(d, l.cells);
  for (int s = 0; s < sp.num_scans; ++s) {
    bounds[4 * s] = shrunk.linear_bounds[s].min_x;
    bounds[4 * s + 1] = shrunk.linear_bounds[s].max_x;
    bounds[4 * s + 2] = shrunk.linear_bounds[s].min_y;
    bounds[4 * s + 3] = shrunk.linear_bounds[s].max_y;
    for (int i = 0; i < n; ++i) {
      out[2 * (static_cast<int64_t>(s) * n + i)] = d[s][i].x;
      out[2 * (static_cast<int64_t>(s) * n + i) + 1] = d[s][i].y;
    }
  }
  return 0;
}

// ---- correlative_scan_matcher_2d.h helpers (checkers for the csm_search_*,
// csm_generate_rotated_scans, csm_discretize_scans and
// csm_rt2d_score_candidates exports) -----------------------------------------

// SearchParameters(lin, ang, cloud, res): num_angular, step, num_scans and
// the first scan's bounds (all scans start equal).
int32_t oracle_search_parameters(double lin, double ang, const float* xyz, int32_t n, double res,
                                 int32_t* num_angular, double* step, int32_t* num_scans,
                                 int32_t* bounds4) {
  const SearchParameters sp(lin, ang, ToCloud(xyz, n), res);
  *num_angular = sp.num_angular_perturbations;
  *step = sp.angular_perturbation_step_size;
  *num_scans = sp.num_scans;
  bounds4[0] = sp.linear_bounds[0].min_x;
  bounds4[1] = sp.linear_bounds[0].max_x;
  bounds4[2] = sp.linear_bounds[0].min_y;
  bounds4[3] = sp.linear_bounds[0].max_y;
  return 0;
}

// GenerateRotatedScans with the testing SearchParameters constructor;
// out: num_scans * n * 3 floats.
int32_t oracle_generate_rotated_scans(const float* xyz, int32_t n, int32_t num_linear,
                                      int32_t num_angular, double step, double res, float* out) {
  const SearchParameters sp(num_linear, num_angular, step, res);
  const auto scans = GenerateRotatedScans(ToCloud(xyz, n), sp);
  for (int s = 0; s < sp.num_scans; ++s)
    for (int i = 0; i < n; ++i) {
      float* o = out + 3 * (static_cast<int64_t>(s) * n + i);
      o[0] = scans[s][i].x;
      o[1] = scans[s][i].y;
      o[2] = scans[s][i].z;
    }
  return sp.num_scans;
}

// DiscretizeScans of num_scans given clouds (scan-major); out: (x, y) pairs.
int32_t oracle_discretize_scans(double res, double max_x, double max_y, int32_t nx, int32_t ny,
                                const float* rotated, int32_t n, int32_t num_scans, float tx,
                                float ty, int32_t* out) {
  std::vector<PointCloud> scans(static_cast<size_t>(num_scans));
  for (int s = 0; s < num_scans; ++s) scans[s] = ToCloud(rotated + 3 * static_cast<int64_t>(s) * n, n);
  const auto d = DiscretizeScans(ToLimits(res, max_x, max_y, nx, ny), scans, tx, ty);
  for (int s = 0; s < num_scans; ++s)
    for (int i = 0; i < n; ++i) {
      out[2 * (static_cast<int64_t>(s) * n + i)] = d[s][i].x;
      out[2 * (static_cast<int64_t>(s) * n + i) + 1] = d[s][i].y;
    }
  return 0;
}

// RealTimeCorrelativeScanMatcher2D::ScoreCandidates over a probability grid.
// discrete: num_scans * n (x, y); cands: (scan, x_off, y_off) triples;
// sp given as (num_angular, step, res) through the testing constructor.
int32_t oracle_rt2d_score_candidates(double res, double max_x, double max_y, int32_t nx,
                                     int32_t ny, const uint16_t* cells, double wt, double wr,
                                     const int32_t* discrete, int32_t num_scans, int32_t n,
                                     int32_t num_angular, double step, const int32_t* cands,
                                     int64_t count, float* out) {
  const MapLimits l = ToLimits(res, max_x, max_y, nx, ny);
  ProbabilityGrid g(l, std::vector<uint16_t>(cells, cells + static_cast<size_t>(nx) * ny));
  RealTimeOptions o;
  o.translation_delta_cost_weight = wt;
  o.rotation_delta_cost_weight = wr;
  std::vector<DiscreteScan2D> scans(static_cast<size_t>(num_scans));
  for (int s = 0; s < num_scans; ++s)
    for (int i = 0; i < n; ++i) {
      const int64_t k = static_cast<int64_t>(s) * n + i;
      scans[s].push_back(Idx2{discrete[2 * k], discrete[2 * k + 1]});
    }
  const SearchParameters sp(0, num_angular, step, res);
  std::vector<Candidate2D> c;
  for (int64_t i = 0; i < count; ++i) c.emplace_back(cands[3 * i], cands[3 * i + 1], cands[3 * i + 2], sp);
  RealTimeCorrelativeScanMatcher2D(o).ScoreCandidates(g, scans, &c);
  for (int64_t i = 0; i < count; ++i) out[i] = c[i].score;
  return 0;
}

}  // extern "C"

// ---- test-grid construction (the reference tests build grids through the
// real inserter, fast_correlative_scan_matcher_2d_test.cc:160-172) -----------
extern "C" {

void* oracle_grid_create(double res, double max_x, double max_y, int32_t nx, int32_t ny) {
  return new ProbabilityGrid(ToLimits(res, max_x, max_y, nx, ny));
}
void oracle_grid_destroy(void* g) { delete static_cast<ProbabilityGrid*>(g); }

void oracle_grid_insert(void* g, float hit_p, float miss_p, int32_t insert_free,
                        const float* origin, const float* returns, int32_t n) {
  RangeData rd;
  rd.origin = Vec3f{origin[0], origin[1], origin[2]};
  rd.returns = ToCloud(returns, n);
  ProbabilityGridInserter2D(hit_p, miss_p, insert_free != 0)
      .Insert(rd, static_cast<ProbabilityGrid*>(g));
}

void oracle_grid_set_probability(void* g, int32_t x, int32_t y, float p) {
  static_cast<ProbabilityGrid*>(g)->SetProbability(Idx2{x, y}, p);
}

// Submap2D::Finish (submap_2d.cc:146-150): replaces the grid by
// ComputeCroppedGrid(), cropped to the known box its updates tracked.
void oracle_grid_crop(void* g) {
  ProbabilityGrid* grid = static_cast<ProbabilityGrid*>(g);
  *grid = grid->ComputeCroppedGrid();
}

// info: resolution, max_x, max_y; cells: nx, ny.
void oracle_grid_info(void* g, double* info, int32_t* cells) {
  const MapLimits& l = static_cast<ProbabilityGrid*>(g)->limits();
  info[0] = l.resolution;
  info[1] = l.max_x;
  info[2] = l.max_y;
  cells[0] = l.cells.num_x_cells;
  cells[1] = l.cells.num_y_cells;
}

void oracle_grid_cells(void* g, uint16_t* out) {
  const auto& c = static_cast<ProbabilityGrid*>(g)->cells();
  std::copy(c.begin(), c.end(), out);
}

// Pose helpers matching the reference tests' float transforms.
void oracle_transform_cloud_2d(const float* pose_f, const float* in, int32_t n, float* out) {
  Rigid2f r;
  r.tx = pose_f[0];
  r.ty = pose_f[1];
  r.angle = pose_f[2];
  const PointCloud c = TransformPointCloud(ToCloud(in, n), Embed3D(r));
  for (int32_t i = 0; i < n; ++i) {
    out[3 * i] = c[i].x;
    out[3 * i + 1] = c[i].y;
    out[3 * i + 2] = c[i].z;
  }
}

}  // extern "C"
