// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// 2D correlative scan matching restated from
//   mapping/internal/2d/scan_matching/correlative_scan_matcher_2d.cc
//   mapping/internal/2d/scan_matching/fast_correlative_scan_matcher_2d.cc
//   mapping/internal/2d/scan_matching/real_time_correlative_scan_matcher_2d.cc
// keeping the reference's data structures (vector<Candidate2D>, std::sort,
// recursive branch and bound, per-lookup bounds checks) so that it is also a
// faithful CPU baseline.

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>

#include "csm_oracle.h"

#define ORACLE_CHECK(cond)                                              \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "oracle CHECK failed %s:%d: %s\n", __FILE__, \
                   __LINE__, #cond);                                    \
      std::abort();                                                     \
    }                                                                   \
  } while (0)

namespace oracle {

// correlative_scan_matcher_2d.cc:27-55
SearchParameters::SearchParameters(double linear_search_window,
                                   double angular_search_window,
                                   const PointCloud& cloud, double res)
    : resolution(res) {
  // 'float max_scan_range = 3.f * resolution' narrows a double product.
  float max_scan_range = 3.f * res;
  for (const Vec3f& p : cloud) {
    const float range = std::sqrt(p.x * p.x + p.y * p.y);
    max_scan_range = std::max(range, max_scan_range);
  }
  const double kSafetyMargin = 1. - 1e-3;
  // common::Pow2 on the float range is a float product.
  const float range_sq = max_scan_range * max_scan_range;
  angular_perturbation_step_size =
      kSafetyMargin * std::acos(1. - (res * res) / (2. * range_sq));
  num_angular_perturbations =
      static_cast<int>(std::ceil(angular_search_window /
                                 angular_perturbation_step_size));
  num_scans = 2 * num_angular_perturbations + 1;
  const int n_lin = static_cast<int>(std::ceil(linear_search_window / res));
  linear_bounds.assign(num_scans, LinearBounds{-n_lin, n_lin, -n_lin, n_lin});
}

// correlative_scan_matcher_2d.cc:57-71
SearchParameters::SearchParameters(int num_linear_perturbations,
                                   int num_angular, double step, double res)
    : num_angular_perturbations(num_angular),
      angular_perturbation_step_size(step),
      resolution(res),
      num_scans(2 * num_angular + 1) {
  const int n = num_linear_perturbations;
  linear_bounds.assign(num_scans, LinearBounds{-n, n, -n, n});
}

// correlative_scan_matcher_2d.cc:73-91
void SearchParameters::ShrinkToFit(const std::vector<DiscreteScan2D>& scans,
                                   const CellLimits& cl) {
  ORACLE_CHECK(static_cast<int>(scans.size()) == num_scans);
  for (int i = 0; i < num_scans; ++i) {
    int lo_x = 0, lo_y = 0, hi_x = 0, hi_y = 0;
    for (const Idx2& xy : scans[i]) {
      lo_x = std::min(lo_x, -xy.x);
      lo_y = std::min(lo_y, -xy.y);
      hi_x = std::max(hi_x, cl.num_x_cells - 1 - xy.x);
      hi_y = std::max(hi_y, cl.num_y_cells - 1 - xy.y);
    }
    LinearBounds& b = linear_bounds[i];
    b.min_x = std::max(b.min_x, lo_x);
    b.max_x = std::min(b.max_x, hi_x);
    b.min_y = std::max(b.min_y, lo_y);
    b.max_y = std::min(b.max_y, hi_y);
  }
}

// correlative_scan_matcher_2d.cc:93-109 — the angle is accumulated in double
// and narrowed to float by Eigen::AngleAxisf.
std::vector<PointCloud> GenerateRotatedScans(const PointCloud& cloud,
                                             const SearchParameters& sp) {
  std::vector<PointCloud> out;
  out.reserve(sp.num_scans);
  double theta = -sp.num_angular_perturbations * sp.angular_perturbation_step_size;
  for (int s = 0; s < sp.num_scans; ++s, theta += sp.angular_perturbation_step_size) {
    Rigid3f rot;
    rot.q = QuatFromAngleAxisF(static_cast<float>(theta), 0.f, 0.f, 1.f);
    out.push_back(TransformPointCloud(cloud, rot));
  }
  return out;
}

// correlative_scan_matcher_2d.cc:111-127 — Affine2f(translation) * p is
// t + (1*x + 0*y) in float; then MapLimits::GetCellIndex in double.
std::vector<DiscreteScan2D> DiscretizeScans(const MapLimits& limits,
                                            const std::vector<PointCloud>& scans,
                                            float tx, float ty) {
  std::vector<DiscreteScan2D> out;
  out.reserve(scans.size());
  for (const PointCloud& scan : scans) {
    out.emplace_back();
    out.back().reserve(scan.size());
    for (const Vec3f& p : scan)
      out.back().push_back(limits.GetCellIndex(tx + p.x, ty + p.y));
  }
  return out;
}

// correlative_scan_matcher_2d.h:75-85
Candidate2D::Candidate2D(int si, int xo, int yo, const SearchParameters& sp)
    : scan_index(si),
      x_index_offset(xo),
      y_index_offset(yo),
      x(-yo * sp.resolution),
      y(-xo * sp.resolution),
      orientation((si - sp.num_angular_perturbations) *
                  sp.angular_perturbation_step_size) {}

// ---------------------------------------------------------------------------
// fast_correlative_scan_matcher_2d.cc:41-74 — a monotone deque holding the
// non-ascending maxima of the current window.
namespace {
class WindowMax {
 public:
  void Push(float v) {
    while (!q_.empty() && v > q_.back()) q_.pop_back();
    q_.push_back(v);
  }
  void Pop(float v) {
    if (v == q_.front()) q_.pop_front();
  }
  float Max() const { return q_.front(); }
  bool Empty() const { return q_.empty(); }

 private:
  std::deque<float> q_;
};
}  // namespace

// fast_correlative_scan_matcher_2d.cc:91-161: row pass then column pass.
// Cell (x0, y0) of the wide grid holds the max over the window
// [x0-(w-1), x0] x [y0-(w-1), y0] of the source grid (clipped to it).
PrecomputationGrid2D::PrecomputationGrid2D(const ProbabilityGrid& grid,
                                           const CellLimits& limits, int width,
                                           std::vector<float>* scratch)
    : offset_x_(-width + 1),
      offset_y_(-width + 1),
      wide_{limits.num_x_cells + width - 1, limits.num_y_cells + width - 1},
      min_score_(1.f - grid.max_correspondence_cost()),
      max_score_(1.f - grid.min_correspondence_cost()),
      cells_(static_cast<size_t>(wide_.num_x_cells) * wide_.num_y_cells) {
  ORACLE_CHECK(width >= 1 && limits.num_x_cells >= 1 && limits.num_y_cells >= 1);
  const int nx = limits.num_x_cells, ny = limits.num_y_cells;
  const int stride = wide_.num_x_cells;
  auto prob = [&grid](int x, int y) {
    return 1.f - std::abs(grid.GetCorrespondenceCost(Idx2{x, y}));
  };
  std::vector<float>& mid = *scratch;
  mid.resize(static_cast<size_t>(stride) * ny);
  for (int y = 0; y < ny; ++y) {
    WindowMax win;
    // Output column xw covers source columns [xw-(w-1), xw].
    int next_in = 0;  // next source column to enter the window
    for (int xw = 0; xw < stride; ++xw) {
      if (next_in < nx && next_in <= xw) win.Push(prob(next_in++, y));
      mid[xw + y * stride] = win.Max();
      const int out_col = xw - (width - 1);
      if (out_col >= 0) win.Pop(prob(out_col, y));
    }
    ORACLE_CHECK(win.Empty());
  }
  for (int x = 0; x < stride; ++x) {
    WindowMax win;
    int next_in = 0;
    for (int yw = 0; yw < wide_.num_y_cells; ++yw) {
      if (next_in < ny && next_in <= yw) win.Push(mid[x + next_in++ * stride]);
      cells_[x + yw * stride] = ComputeCellValue(win.Max());
      const int out_row = yw - (width - 1);
      if (out_row >= 0) win.Pop(mid[x + out_row * stride]);
    }
    ORACLE_CHECK(win.Empty());
  }
}

// fast_correlative_scan_matcher_2d.cc:163-169
uint8_t PrecomputationGrid2D::ComputeCellValue(float probability) const {
  const int v =
      RoundToIntF((probability - min_score_) * (255.f / (max_score_ - min_score_)));
  ORACLE_CHECK(v >= 0 && v <= 255);
  return static_cast<uint8_t>(v);
}

// fast_correlative_scan_matcher_2d.cc:171-194
FastCorrelativeScanMatcher2D::FastCorrelativeScanMatcher2D(
    const ProbabilityGrid& grid, const FastOptions2D& options)
    : options_(options), limits_(grid.limits()) {
  ORACLE_CHECK(options.branch_and_bound_depth >= 1);
  std::vector<float> scratch;
  grids_.reserve(options.branch_and_bound_depth);
  for (int i = 0; i < options.branch_and_bound_depth; ++i)
    grids_.emplace_back(grid, grid.limits().cells, 1 << i, &scratch);
}

// fast_correlative_scan_matcher_2d.cc:198-208
bool FastCorrelativeScanMatcher2D::Match(const Rigid2d& initial,
                                         const PointCloud& cloud,
                                         float min_score, float* score,
                                         Rigid2d* pose,
                                         MatchStats2D* stats) const {
  const SearchParameters sp(options_.linear_search_window,
                            options_.angular_search_window, cloud,
                            limits_.resolution);
  return MatchWithSearchParameters(sp, initial, cloud, min_score, score, pose,
                                   stats);
}

// fast_correlative_scan_matcher_2d.cc:210-225 — note (num_y, num_x) order.
bool FastCorrelativeScanMatcher2D::MatchFullSubmap(const PointCloud& cloud,
                                                   float min_score,
                                                   float* score, Rigid2d* pose,
                                                   MatchStats2D* stats) const {
  const SearchParameters sp(1e6 * limits_.resolution, M_PI, cloud,
                            limits_.resolution);
  const double half = 0.5 * limits_.resolution;
  Rigid2d center;
  center.tx = limits_.max_x - half * limits_.cells.num_y_cells;
  center.ty = limits_.max_y - half * limits_.cells.num_x_cells;
  center.angle = 0.;
  return MatchWithSearchParameters(sp, center, cloud, min_score, score, pose,
                                   stats);
}

// fast_correlative_scan_matcher_2d.cc:227-262
bool FastCorrelativeScanMatcher2D::MatchWithSearchParameters(
    SearchParameters sp, const Rigid2d& initial, const PointCloud& cloud,
    float min_score, float* score, Rigid2d* pose, MatchStats2D* stats) const {
  ORACLE_CHECK(score != nullptr && pose != nullptr);
  Rigid3f pre;
  pre.q = QuatFromAngleAxisF(static_cast<float>(initial.angle), 0.f, 0.f, 1.f);
  const PointCloud rotated = TransformPointCloud(cloud, pre);
  const std::vector<PointCloud> rotated_scans = GenerateRotatedScans(rotated, sp);
  const std::vector<DiscreteScan2D> discrete =
      DiscretizeScans(limits_, rotated_scans, static_cast<float>(initial.tx),
                      static_cast<float>(initial.ty));
  sp.ShrinkToFit(discrete, limits_.cells);
  std::vector<Candidate2D> lowest = GenerateLowestResolutionCandidates(sp);
  if (stats) {
    stats->num_scans = sp.num_scans;
    stats->lowest_resolution_candidates = static_cast<int64_t>(lowest.size());
  }
  ScoreCandidates(grids_[max_depth()], discrete, &lowest, stats);
  if (stats) stats->candidates_per_level[max_depth()] += lowest.size();
  const Candidate2D best =
      BranchAndBound(discrete, sp, lowest, max_depth(), min_score, stats);
  if (best.score > min_score) {
    *score = best.score;
    pose->tx = initial.tx + best.x;
    pose->ty = initial.ty + best.y;
    pose->angle = initial.angle + best.orientation;
    return true;
  }
  return false;
}

// fast_correlative_scan_matcher_2d.cc:276-312
std::vector<Candidate2D>
FastCorrelativeScanMatcher2D::GenerateLowestResolutionCandidates(
    const SearchParameters& sp) const {
  const int step = 1 << max_depth();
  size_t n = 0;
  for (int s = 0; s < sp.num_scans; ++s) {
    const LinearBounds& b = sp.linear_bounds[s];
    n += static_cast<size_t>((b.max_x - b.min_x + step) / step) *
         ((b.max_y - b.min_y + step) / step);
  }
  std::vector<Candidate2D> out;
  out.reserve(n);
  for (int s = 0; s < sp.num_scans; ++s) {
    const LinearBounds& b = sp.linear_bounds[s];
    for (int xo = b.min_x; xo <= b.max_x; xo += step)
      for (int yo = b.min_y; yo <= b.max_y; yo += step)
        out.emplace_back(s, xo, yo, sp);
  }
  ORACLE_CHECK(out.size() == n);
  return out;
}

// fast_correlative_scan_matcher_2d.cc:314-333 — integer sum, mean, sort.
void FastCorrelativeScanMatcher2D::ScoreCandidates(
    const PrecomputationGrid2D& grid, const std::vector<DiscreteScan2D>& scans,
    std::vector<Candidate2D>* candidates, MatchStats2D* stats) const {
  for (Candidate2D& c : *candidates) {
    int sum = 0;
    const DiscreteScan2D& scan = scans[c.scan_index];
    for (const Idx2& xy : scan)
      sum += grid.GetValue(Idx2{xy.x + c.x_index_offset, xy.y + c.y_index_offset});
    c.score = grid.ToScore(sum / static_cast<float>(scan.size()));
    if (stats) stats->lookups += static_cast<int64_t>(scan.size());
  }
  std::sort(candidates->begin(), candidates->end(), std::greater<Candidate2D>());
}

// fast_correlative_scan_matcher_2d.cc:335-378
Candidate2D FastCorrelativeScanMatcher2D::BranchAndBound(
    const std::vector<DiscreteScan2D>& scans, const SearchParameters& sp,
    const std::vector<Candidate2D>& candidates, int depth, float min_score,
    MatchStats2D* stats) const {
  if (depth == 0) return candidates.front();
  Candidate2D best(0, 0, 0, sp);
  best.score = min_score;
  const int half = 1 << (depth - 1);
  for (const Candidate2D& c : candidates) {
    if (c.score <= min_score) break;
    std::vector<Candidate2D> children;
    const LinearBounds& b = sp.linear_bounds[c.scan_index];
    for (int dx : {0, half}) {
      if (c.x_index_offset + dx > b.max_x) break;
      for (int dy : {0, half}) {
        if (c.y_index_offset + dy > b.max_y) break;
        children.emplace_back(c.scan_index, c.x_index_offset + dx,
                              c.y_index_offset + dy, sp);
      }
    }
    ScoreCandidates(grids_[depth - 1], scans, &children, stats);
    if (stats) stats->candidates_per_level[depth - 1] += children.size();
    best = std::max(best, BranchAndBound(scans, sp, children, depth - 1,
                                         best.score, stats));
  }
  return best;
}

// Test-only tie enumeration (not part of the reference): the same window,
// discretization and lowest-resolution candidates as MatchWithSearchParameters
// (fast_correlative_scan_matcher_2d.cc:227-262), BranchAndBound for the
// maximum, then a second walk that keeps every node whose bound reaches that
// maximum and collects the leaves scoring exactly it. Equal float scores are
// equal integer sums (ToScore is strictly monotone, SURVEY §8a hazard 13).
std::vector<std::array<int, 3>> FastCorrelativeScanMatcher2D::TiedMaxLeaves(
    bool full_submap, const Rigid2d& initial_in, const PointCloud& cloud,
    float min_score, size_t max_out, std::array<int, 3>* picked) const {
  Rigid2d initial = initial_in;
  double lin = options_.linear_search_window, ang = options_.angular_search_window;
  if (full_submap) {
    lin = 1e6 * limits_.resolution;
    ang = M_PI;
    const double half = 0.5 * limits_.resolution;
    initial.tx = limits_.max_x - half * limits_.cells.num_y_cells;
    initial.ty = limits_.max_y - half * limits_.cells.num_x_cells;
    initial.angle = 0.;
  }
  SearchParameters sp(lin, ang, cloud, limits_.resolution);
  Rigid3f pre;
  pre.q = QuatFromAngleAxisF(static_cast<float>(initial.angle), 0.f, 0.f, 1.f);
  const std::vector<PointCloud> rotated_scans =
      GenerateRotatedScans(TransformPointCloud(cloud, pre), sp);
  const std::vector<DiscreteScan2D> discrete =
      DiscretizeScans(limits_, rotated_scans, static_cast<float>(initial.tx),
                      static_cast<float>(initial.ty));
  sp.ShrinkToFit(discrete, limits_.cells);
  std::vector<Candidate2D> lowest = GenerateLowestResolutionCandidates(sp);
  ScoreCandidates(grids_[max_depth()], discrete, &lowest, nullptr);
  const Candidate2D best = BranchAndBound(discrete, sp, lowest, max_depth(), min_score, nullptr);
  std::vector<std::array<int, 3>> out;
  if (!(best.score > min_score)) return out;
  *picked = {best.scan_index, best.x_index_offset, best.y_index_offset};
  CollectTies(discrete, sp, lowest, max_depth(), best.score, max_out, &out);
  return out;
}

void FastCorrelativeScanMatcher2D::CollectTies(
    const std::vector<DiscreteScan2D>& scans, const SearchParameters& sp,
    const std::vector<Candidate2D>& candidates, int depth, float best, size_t max_out,
    std::vector<std::array<int, 3>>* out) const {
  for (const Candidate2D& c : candidates) {
    if (c.score < best || out->size() >= max_out) break;  // sorted, descending
    if (depth == 0) {
      out->push_back({c.scan_index, c.x_index_offset, c.y_index_offset});
      continue;
    }
    std::vector<Candidate2D> children;
    const LinearBounds& b = sp.linear_bounds[c.scan_index];
    const int half = 1 << (depth - 1);
    for (int dx : {0, half}) {
      if (c.x_index_offset + dx > b.max_x) break;
      for (int dy : {0, half}) {
        if (c.y_index_offset + dy > b.max_y) break;
        children.emplace_back(c.scan_index, c.x_index_offset + dx, c.y_index_offset + dy, sp);
      }
    }
    ScoreCandidates(grids_[depth - 1], scans, &children, nullptr);
    CollectTies(scans, sp, children, depth - 1, best, max_out, out);
  }
}

// ---------------------------------------------------------------------------
// real_time_correlative_scan_matcher_2d.cc:81-115
std::vector<Candidate2D>
RealTimeCorrelativeScanMatcher2D::GenerateExhaustiveSearchCandidates(
    const SearchParameters& sp) const {
  size_t n = 0;
  for (int s = 0; s < sp.num_scans; ++s) {
    const LinearBounds& b = sp.linear_bounds[s];
    n += static_cast<size_t>(b.max_x - b.min_x + 1) * (b.max_y - b.min_y + 1);
  }
  std::vector<Candidate2D> out;
  out.reserve(n);
  for (int s = 0; s < sp.num_scans; ++s) {
    const LinearBounds& b = sp.linear_bounds[s];
    for (int xo = b.min_x; xo <= b.max_x; ++xo)
      for (int yo = b.min_y; yo <= b.max_y; ++yo) out.emplace_back(s, xo, yo, sp);
  }
  return out;
}

// real_time_correlative_scan_matcher_2d.cc:117-149
double RealTimeCorrelativeScanMatcher2D::Match(const Rigid2d& initial,
                                               const PointCloud& cloud,
                                               const ProbabilityGrid& grid,
                                               Rigid2d* pose,
                                               int64_t* num_candidates) const {
  ORACLE_CHECK(pose != nullptr);
  Rigid3f pre;
  pre.q = QuatFromAngleAxisF(static_cast<float>(initial.angle), 0.f, 0.f, 1.f);
  const PointCloud rotated = TransformPointCloud(cloud, pre);
  const SearchParameters sp(options_.linear_search_window,
                            options_.angular_search_window, rotated,
                            grid.limits().resolution);
  const std::vector<PointCloud> rotated_scans = GenerateRotatedScans(rotated, sp);
  const std::vector<DiscreteScan2D> discrete = DiscretizeScans(
      grid.limits(), rotated_scans, static_cast<float>(initial.tx),
      static_cast<float>(initial.ty));
  std::vector<Candidate2D> candidates = GenerateExhaustiveSearchCandidates(sp);
  if (num_candidates) *num_candidates = static_cast<int64_t>(candidates.size());
  ScoreCandidates(grid, discrete, &candidates);
  const Candidate2D& best = *std::max_element(candidates.begin(), candidates.end());
  pose->tx = initial.tx + best.x;
  pose->ty = initial.ty + best.y;
  pose->angle = initial.angle + best.orientation;
  return best.score;
}

// real_time_correlative_scan_matcher_2d.cc:61-75, 151-176 (probability grid).
void RealTimeCorrelativeScanMatcher2D::ScoreCandidates(
    const ProbabilityGrid& grid, const std::vector<DiscreteScan2D>& scans,
    std::vector<Candidate2D>* candidates) const {
  for (Candidate2D& c : *candidates) {
    const DiscreteScan2D& scan = scans[c.scan_index];
    float s = 0.f;
    for (const Idx2& xy : scan)
      s += grid.GetProbability(Idx2{xy.x + c.x_index_offset, xy.y + c.y_index_offset});
    s /= static_cast<float>(scan.size());
    ORACLE_CHECK(s > 0.f);
    const double pen = std::hypot(c.x, c.y) * options_.translation_delta_cost_weight +
                       std::abs(c.orientation) * options_.rotation_delta_cost_weight;
    c.score = s;
    c.score *= std::exp(-(pen * pen));
  }
}

}  // namespace oracle
