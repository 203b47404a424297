// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// Pins the oracle: every known-answer / property check the reference's own
// unit tests make on this path, restated against the oracle. Each TEST names
// the reference test it restates (file:line). Exit status 0 = all passed.
//
// Random inputs use the same libstdc++ engines as the reference tests
// (std::mt19937 + uniform distributions), so the draws follow the same
// generator; the checks are the reference's checks and tolerances.

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <functional>
#include <limits>
#include <random>
#include <string>
#include <vector>

#include "csm_oracle.h"
#include "oracle3d.h"

using namespace oracle;

namespace {

int g_failures = 0;
int g_checks = 0;
const char* g_test = "";

#define EXPECT(cond)                                                       \
  do {                                                                     \
    ++g_checks;                                                            \
    if (!(cond)) {                                                         \
      ++g_failures;                                                        \
      std::fprintf(stderr, "[%s] FAILED %s:%d: %s\n", g_test, __FILE__,    \
                   __LINE__, #cond);                                       \
    }                                                                      \
  } while (0)
#define EXPECT_NEAR(a, b, tol) EXPECT(std::abs((double)(a) - (double)(b)) <= (tol))

struct TestCase {
  const char* name;
  std::function<void()> fn;
};
std::vector<TestCase>& Registry() {
  static std::vector<TestCase> r;
  return r;
}
struct Registrar {
  Registrar(const char* n, std::function<void()> f) {
    Registry().push_back({n, std::move(f)});
  }
};
#define TEST(name)                                   \
  void name();                                       \
  Registrar reg_##name(#name, name);                 \
  void name()

bool SameIdx(const Idx2& a, int x, int y) { return a.x == x && a.y == y; }

MapLimits Limits(double res, double mx, double my, int nx, int ny) {
  MapLimits l;
  l.resolution = res;
  l.max_x = mx;
  l.max_y = my;
  l.cells = CellLimits{nx, ny};
  return l;
}

// ----------------------------------------------------------------- 2D ------
// correlative_scan_matcher_test.cc:26-40
TEST(SearchParametersConstruction) {
  const SearchParameters sp(4, 5, 0.03, 0.05);
  EXPECT(sp.num_angular_perturbations == 5);
  EXPECT_NEAR(sp.angular_perturbation_step_size, 0.03, 1e-9);
  EXPECT_NEAR(sp.resolution, 0.05, 1e-9);
  EXPECT(sp.num_scans == 11);
  EXPECT(sp.linear_bounds.size() == 11u);
  for (const LinearBounds& b : sp.linear_bounds)
    EXPECT(b.min_x == -4 && b.max_x == 4 && b.min_y == -4 && b.max_y == 4);
}

// correlative_scan_matcher_test.cc:42-56
TEST(CandidateConstruction) {
  const SearchParameters sp(4, 5, 0.03, 0.05);
  const Candidate2D c(3, 4, -5, sp);
  EXPECT(c.scan_index == 3 && c.x_index_offset == 4 && c.y_index_offset == -5);
  EXPECT_NEAR(c.x, 0.25, 1e-9);
  EXPECT_NEAR(c.y, -0.2, 1e-9);
  EXPECT_NEAR(c.orientation, -0.06, 1e-9);
  EXPECT_NEAR(c.score, 0., 1e-9);
  Candidate2D bigger(3, 4, 5, sp);
  bigger.score = 1.f;
  EXPECT(c < bigger);
}

// correlative_scan_matcher_test.cc:58-70
TEST(GenerateRotatedScansTest) {
  PointCloud cloud{{-1.f, 1.f, 0.f}};
  const auto scans = GenerateRotatedScans(cloud, SearchParameters(0, 1, M_PI / 2., 0.));
  EXPECT(scans.size() == 3u);
  EXPECT_NEAR(scans[0][0].x, 1., 1e-6);
  EXPECT_NEAR(scans[0][0].y, 1., 1e-6);
  EXPECT_NEAR(scans[1][0].x, -1., 1e-6);
  EXPECT_NEAR(scans[1][0].y, 1., 1e-6);
  EXPECT_NEAR(scans[2][0].x, -1., 1e-6);
  EXPECT_NEAR(scans[2][0].y, -1., 1e-6);
}

PointCloud SevenPointCloud() {
  return PointCloud{{0.025f, 0.175f, 0.f},  {-0.025f, 0.175f, 0.f},
                    {-0.075f, 0.175f, 0.f}, {-0.125f, 0.175f, 0.f},
                    {-0.125f, 0.125f, 0.f}, {-0.125f, 0.075f, 0.f},
                    {-0.125f, 0.025f, 0.f}};
}

// correlative_scan_matcher_test.cc:72-96 — exact cell indices.
TEST(DiscretizeScansTest) {
  const MapLimits limits = Limits(0.05, 0.05, 0.25, 6, 6);
  const auto scans = GenerateRotatedScans(SevenPointCloud(), SearchParameters(0, 0, 0., 0.));
  const auto d = DiscretizeScans(limits, scans, 0.f, 0.f);
  EXPECT(d.size() == 1u);
  EXPECT(d[0].size() == 7u);
  const int expect[7][2] = {{1, 0}, {1, 1}, {1, 2}, {1, 3}, {2, 3}, {3, 3}, {4, 3}};
  for (int i = 0; i < 7; ++i) EXPECT(SameIdx(d[0][i], expect[i][0], expect[i][1]));
}

void PrecomputationCheck(const MapLimits& limits, int x0, int y0,
                         const std::vector<int>& widths) {
  std::mt19937 prng(42);
  std::uniform_int_distribution<int> distribution(0, 255);
  ProbabilityGrid grid(limits);
  std::vector<float> scratch;
  PrecomputationGrid2D dummy(grid, grid.limits().cells, 1, &scratch);
  for (int y = y0; y < limits.cells.num_y_cells; ++y)
    for (int x = x0; x < limits.cells.num_x_cells; ++x)
      grid.SetProbability(Idx2{x, y}, dummy.ToScore(distribution(prng)));
  scratch.clear();
  for (int width : widths) {
    PrecomputationGrid2D pg(grid, grid.limits().cells, width, &scratch);
    for (int y = 0; y < limits.cells.num_y_cells; ++y)
      for (int x = 0; x < limits.cells.num_x_cells; ++x) {
        float max_score = -std::numeric_limits<float>::infinity();
        for (int dy = 0; dy < width; ++dy)
          for (int dx = 0; dx < width; ++dx)
            max_score = std::max(max_score, grid.GetProbability(Idx2{x + dx, y + dy}));
        EXPECT_NEAR(max_score, pg.ToScore(pg.GetValue(Idx2{x, y})), 1e-4);
      }
  }
}

// fast_correlative_scan_matcher_2d_test.cc:37-77 (cells (50..249)^2 set).
TEST(PrecomputationGridCorrectValues) {
  PrecomputationCheck(Limits(0.05, 5., 5., 250, 250), 50, 50, {1, 2, 3, 8});
}

// fast_correlative_scan_matcher_2d_test.cc:79-117 (window wider than grid).
TEST(PrecomputationGridTinyProbabilityGrid) {
  PrecomputationCheck(Limits(0.05, 0.1, 0.1, 4, 4), 0, 0, {1, 2, 3, 8, 200});
}

// fast_correlative_scan_matcher_2d_test.cc:144-192
TEST(FastCorrelativeScanMatcherCorrectPose) {
  std::mt19937 prng(42);
  std::uniform_real_distribution<float> distribution(-1.f, 1.f);
  const ProbabilityGridInserter2D inserter(0.7f, 0.4f, true);
  constexpr float kMinScore = 0.1f;
  FastOptions2D options;
  options.linear_search_window = 3.;
  options.angular_search_window = 1.;
  options.branch_and_bound_depth = 3;
  const PointCloud cloud{{-2.5f, 0.5f, 0.f}, {-2.f, 0.5f, 0.f}, {0.f, -0.5f, 0.f},
                         {0.5f, -1.6f, 0.f}, {2.5f, 0.5f, 0.f}, {2.5f, 1.7f, 0.f}};
  for (int i = 0; i < 50; ++i) {
    Rigid2f expected;
    expected.tx = 2.f * distribution(prng);
    expected.ty = 2.f * distribution(prng);
    expected.angle = static_cast<float>(0.5 * distribution(prng));
    ProbabilityGrid grid(Limits(0.05, 5., 5., 200, 200));
    RangeData rd;
    rd.origin = Vec3f{expected.tx, expected.ty, 0.f};
    rd.returns = TransformPointCloud(cloud, Embed3D(expected));
    inserter.Insert(rd, &grid);
    grid.FinishUpdate();
    FastCorrelativeScanMatcher2D matcher(grid, options);
    Rigid2d pose;
    float score = 0.f;
    EXPECT(matcher.Match(Rigid2d{}, cloud, kMinScore, &score, &pose));
    EXPECT(kMinScore < score);
    const Rigid2f posef{static_cast<float>(pose.tx), static_cast<float>(pose.ty),
                        static_cast<float>(pose.angle)};
    EXPECT(IsNearly2D(expected, posef, 0.03f));
  }
}

// fast_correlative_scan_matcher_2d_test.cc:194-246
TEST(FastCorrelativeScanMatcherFullSubmapMatching) {
  std::mt19937 prng(42);
  std::uniform_real_distribution<float> distribution(-1.f, 1.f);
  const ProbabilityGridInserter2D inserter(0.7f, 0.4f, true);
  constexpr float kMinScore = 0.1f;
  FastOptions2D options;
  options.linear_search_window = 3.;
  options.angular_search_window = 1.;
  options.branch_and_bound_depth = 6;
  const PointCloud unperturbed{{-2.5f, 0.5f, 0.f}, {-2.25f, 0.5f, 0.f},
                               {0.f, 0.5f, 0.f},   {0.25f, 1.6f, 0.f},
                               {2.5f, 0.5f, 0.f},  {2.f, 1.8f, 0.f}};
  for (int i = 0; i < 20; ++i) {
    Rigid2f perturbation;
    perturbation.tx = 10.f * distribution(prng);
    perturbation.ty = 10.f * distribution(prng);
    perturbation.angle = static_cast<float>(1.6 * distribution(prng));
    const PointCloud cloud = TransformPointCloud(unperturbed, Embed3D(perturbation));
    Rigid2f local;
    local.tx = 2.f * distribution(prng);
    local.ty = 2.f * distribution(prng);
    local.angle = static_cast<float>(0.5 * distribution(prng));
    const Rigid2f expected = Mul(local, Inverse(perturbation));
    ProbabilityGrid grid(Limits(0.05, 5., 5., 200, 200));
    RangeData rd;
    const Rigid3f origin = Embed3D(Mul(expected, perturbation));
    rd.origin = origin.t;
    rd.returns = TransformPointCloud(cloud, Embed3D(expected));
    inserter.Insert(rd, &grid);
    grid.FinishUpdate();
    FastCorrelativeScanMatcher2D matcher(grid, options);
    Rigid2d pose;
    float score = 0.f;
    EXPECT(matcher.MatchFullSubmap(cloud, kMinScore, &score, &pose));
    EXPECT(kMinScore < score);
    const Rigid2f posef{static_cast<float>(pose.tx), static_cast<float>(pose.ty),
                        static_cast<float>(pose.angle)};
    EXPECT(IsNearly2D(expected, posef, 0.03f));
  }
}

ProbabilityGrid SevenPointGrid() {
  ProbabilityGrid grid(Limits(0.05, 0.05, 0.25, 6, 6));
  const ProbabilityGridInserter2D inserter(0.7f, 0.4f, true);
  RangeData rd;
  rd.origin = Vec3f{0.f, 0.f, 0.f};
  rd.returns = SevenPointCloud();
  inserter.Insert(rd, &grid);
  grid.FinishUpdate();
  return grid;
}

RealTimeOptions RtTestOptions() {
  RealTimeOptions o;
  o.linear_search_window = 0.6;
  o.angular_search_window = 0.16;
  o.translation_delta_cost_weight = 0.;
  o.rotation_delta_cost_weight = 0.;
  return o;
}

// real_time_correlative_scan_matcher_2d_test.cc:125-141
TEST(RealTimeScorePerfectHighResolutionCandidateProbabilityGrid) {
  const ProbabilityGrid grid = SevenPointGrid();
  const SearchParameters sp(0, 0, 0., 0.);
  const auto d = DiscretizeScans(grid.limits(), GenerateRotatedScans(SevenPointCloud(), sp), 0.f, 0.f);
  std::vector<Candidate2D> c{Candidate2D(0, 0, 0, sp)};
  RealTimeCorrelativeScanMatcher2D(RtTestOptions()).ScoreCandidates(grid, d, &c);
  EXPECT(c[0].scan_index == 0 && c[0].x_index_offset == 0 && c[0].y_index_offset == 0);
  EXPECT_NEAR(c[0].score, 0.7, 1e-2);
}

// real_time_correlative_scan_matcher_2d_test.cc:161-178
TEST(RealTimeScorePartiallyCorrectHighResolutionCandidateProbabilityGrid) {
  const ProbabilityGrid grid = SevenPointGrid();
  const SearchParameters sp(0, 0, 0., 0.);
  const auto d = DiscretizeScans(grid.limits(), GenerateRotatedScans(SevenPointCloud(), sp), 0.f, 0.f);
  std::vector<Candidate2D> c{Candidate2D(0, 0, 1, sp)};
  RealTimeCorrelativeScanMatcher2D(RtTestOptions()).ScoreCandidates(grid, d, &c);
  EXPECT(c[0].scan_index == 0 && c[0].x_index_offset == 0 && c[0].y_index_offset == 1);
  EXPECT(0.7 * 3. / 7. < c[0].score);
  EXPECT(0.7 > c[0].score);
}

// ray_to_pixel_mask_test.cc:34-140 (unit-scale cases).
bool RayIs(const std::vector<Idx2>& r, const std::vector<std::pair<int, int>>& e) {
  if (r.size() != e.size()) return false;
  for (size_t i = 0; i < r.size(); ++i)
    if (r[i].x != e[i].first || r[i].y != e[i].second) return false;
  return true;
}
TEST(RayToPixelMaskCases) {
  EXPECT(RayIs(RayToPixelMask({1, 1}, {1, 1}, 1), {{1, 1}}));
  EXPECT(RayIs(RayToPixelMask({1, 1}, {3, 1}, 1), {{1, 1}, {2, 1}, {3, 1}}));
  EXPECT(RayIs(RayToPixelMask({3, 1}, {1, 1}, 1), {{1, 1}, {2, 1}, {3, 1}}));
  EXPECT(RayIs(RayToPixelMask({1, 1}, {1, 3}, 1), {{1, 1}, {1, 2}, {1, 3}}));
  EXPECT(RayIs(RayToPixelMask({1, 3}, {1, 1}, 1), {{1, 1}, {1, 2}, {1, 3}}));
  EXPECT(RayIs(RayToPixelMask({1, 1}, {3, 3}, 1), {{1, 1}, {2, 2}, {3, 3}}));
  EXPECT(RayIs(RayToPixelMask({3, 3}, {1, 1}, 1), {{1, 1}, {2, 2}, {3, 3}}));
  EXPECT(RayIs(RayToPixelMask({1, 3}, {3, 1}, 1), {{1, 3}, {2, 2}, {3, 1}}));
  EXPECT(RayIs(RayToPixelMask({3, 1}, {1, 3}, 1), {{1, 3}, {2, 2}, {3, 1}}));
  EXPECT(RayIs(RayToPixelMask({1, 1}, {2, 5}, 1),
               {{1, 1}, {1, 2}, {1, 3}, {2, 3}, {2, 4}, {2, 5}}));
  EXPECT(RayIs(RayToPixelMask({1, 1}, {2, 4}, 1), {{1, 1}, {1, 2}, {2, 3}, {2, 4}}));
  EXPECT(RayIs(RayToPixelMask({1, 1}, {5, 2}, 1),
               {{1, 1}, {2, 1}, {3, 1}, {3, 2}, {4, 2}, {5, 2}}));
  EXPECT(RayIs(RayToPixelMask({1, 1}, {4, 2}, 1), {{1, 1}, {2, 1}, {3, 2}, {4, 2}}));
}

// ray_to_pixel_mask_test.cc:142-165 (MultiScaleAxisAlignedX).
TEST(RayToPixelMaskMultiScale) {
  for (int scale = 1; scale < 10000; scale *= 2) {
    const MapLimits l = Limits(0.1 / scale, 1.0, 1.0, 20 * scale, 20 * scale);
    const Idx2 b = l.GetCellIndex(0.05f, 0.05f);
    const Idx2 e = l.GetCellIndex(0.35f, 0.05f);
    EXPECT(RayIs(RayToPixelMask(b, e, scale), {{9, 6}, {9, 7}, {9, 8}, {9, 9}}));
  }
  const MapLimits l1 = Limits(0.1, 1.0, 1.0, 20, 20);
  EXPECT(RayIs(RayToPixelMask(l1.GetCellIndex(0.01f, 0.09f), l1.GetCellIndex(0.21f, 0.19f), 1),
               {{8, 7}, {8, 8}, {9, 8}, {9, 9}}));
}

// probability_values_test.cc:25-40
TEST(ProbabilityValuesOdds) {
  EXPECT_NEAR(ProbabilityFromOdds(Odds(kMinProbability)), kMinProbability, 1e-6);
  EXPECT_NEAR(ProbabilityFromOdds(Odds(kMaxProbability)), kMaxProbability, 1e-6);
  EXPECT_NEAR(ProbabilityFromOdds(Odds(0.5f)), 0.5, 1e-6);
  EXPECT_NEAR(1.f - ProbabilityFromOdds(Odds(1.f - kMaxCorrespondenceCost)),
              kMaxCorrespondenceCost, 1e-6);
}

// probability_values_test.cc:64-71 and :73-110 (first part).
TEST(ProbabilityValuesTables) {
  const auto& vp = ValueToProbabilityTable();
  const auto& vc = ValueToCorrespondenceCostTable();
  EXPECT_NEAR(vp[0], 1.f - vc[0], 1e-6);
  int bad = 0;
  for (int i = 1; i < 32768; ++i)
    if (std::abs(vp[i] - vc[i]) > 1e-6) ++bad;
  EXPECT(bad == 0);
  const auto pt = LookupTableToApplyOdds(Odds(0.9f));
  const auto ct = LookupTableToApplyCorrespondenceCostOdds(Odds(0.9f));
  EXPECT_NEAR(vp[pt[0]], 1.f - vc[ct[0]], 1e-6);
  int bad2 = 0;
  for (int i = 0; i < 5000; ++i) {
    const float p = (static_cast<float>(i) / 5000.f) * (kMaxProbability - kMinProbability) +
                    kMinProbability;
    const uint16_t pv = ProbabilityToValue(p);
    const uint16_t cv = CorrespondenceCostToValue(1.f - p);
    if (std::abs(int(pv) - (32768 - int(cv))) > 1) ++bad2;
    if (std::abs(vp[pt[pv]] - (1.f - vc[ct[cv]])) > 5e-5) ++bad2;
  }
  EXPECT(bad2 == 0);
}

// transform::IsNearly (rigid_transform_test_helpers.h:42-46) for Rigid2d:
// Eigen's isApprox of the 3x3 affine matrices, |A - B|_F^2 <= eps^2 *
// min(|A|_F^2, |B|_F^2).
bool IsNearly2D(const double a[3], const double b[3], double eps) {
  auto mat = [](const double p[3], double m[9]) {
    const double c = std::cos(p[2]), s = std::sin(p[2]);
    const double v[9] = {c, -s, p[0], s, c, p[1], 0., 0., 1.};
    for (int k = 0; k < 9; ++k) m[k] = v[k];
  };
  double ma[9], mb[9], d = 0., na = 0., nb = 0.;
  mat(a, ma);
  mat(b, mb);
  for (int k = 0; k < 9; ++k) {
    d += (ma[k] - mb[k]) * (ma[k] - mb[k]);
    na += ma[k] * ma[k];
    nb += mb[k] * mb[k];
  }
  return d <= eps * eps * std::min(na, nb);
}

// ceres_scan_matcher_2d_test.cc:35-96 — one occupied cell at (-3.5, 2.5),
// one point at (-3, 2): from four initial poses the solver reaches
// Translation(-0.5, 0.5) within 1e-2 with final_cost ~ 0 (EXPECT_NEAR 1e-2).
// Options as the test's Lua dictionary: occupied_space_weight 1,
// translation_weight 0.1, rotation_weight 1.5, max_num_iterations 50.
TEST(CeresScanMatcher2DTest) {
  ProbabilityGrid grid(Limits(1., 10., 10., 20, 20));
  grid.SetProbability(grid.limits().GetCellIndex(-3.5f, 2.5f), kMaxProbability);
  const std::vector<Vec2d> cloud{{-3., 2.}};
  CeresOptions2D o;
  o.occupied_space_weight = 1.;
  o.translation_weight = 0.1;
  o.rotation_weight = 1.5;
  o.max_num_iterations = 50;
  const double starts[4][2] = {{-0.5, 0.5}, {-0.3, 0.5}, {-0.45, 0.3}, {-0.3, 0.3}};
  for (const auto& st : starts) {
    const double initial[3] = {st[0], st[1], 0.};
    double pose[3], final_cost = -1.;
    CeresMatch2D(grid.limits(), grid.cells(), grid.min_correspondence_cost(),
                 grid.max_correspondence_cost(), o, st, initial, cloud, pose, &final_cost);
    EXPECT_NEAR(0., final_cost, 1e-2);
    const double expected[3] = {-0.5, 0.5, 0.};
    EXPECT(IsNearly2D(pose, expected, 1e-2));
  }
}

// occupied_space_cost_function_2d_test.cc:30-47 — an all-unknown 2x2 grid:
// the residual of one point at the origin is kMaxProbability (DoubleEq,
// 4 ulps).
TEST(OccupiedSpaceCostFunction2DSmokeTest) {
  ProbabilityGrid grid(Limits(1., 1., 1., 2, 2));
  const std::vector<Vec2d> cloud{{0., 0.}};
  const double pose[3] = {0., 0., 0.};
  const std::vector<double> r =
      OccupiedSpaceResiduals2D(grid.limits(), grid.cells(), grid.min_correspondence_cost(),
                               grid.max_correspondence_cost(), 1., cloud, pose);
  EXPECT(r.size() == 1u);
  const double want = static_cast<double>(kMaxProbability);
  EXPECT(std::abs(r[0] - want) <= 4. * std::numeric_limits<double>::epsilon() * want);
}

}  // namespace

int RunRefTests3D(int* checks);    // ref_tests_3d.cc
int RunRefTestsTSDF(int* checks);  // ref_tests_tsdf.cc
int RunRefTestsVoxel(int* checks);  // ref_tests_voxel.cc
int RunRefTestsGrids(int* checks);  // ref_tests_grids.cc

int main() {
  for (const TestCase& t : Registry()) {
    g_test = t.name;
    const int before = g_failures;
    t.fn();
    std::printf("%-70s %s\n", t.name, g_failures == before ? "OK" : "FAILED");
  }
  int checks3d = 0, checks_tsdf = 0, checks_voxel = 0, checks_grids = 0;
  const int failures3d = RunRefTests3D(&checks3d);
  const int failures_tsdf = RunRefTestsTSDF(&checks_tsdf);
  const int failures_voxel = RunRefTestsVoxel(&checks_voxel);
  const int failures_grids = RunRefTestsGrids(&checks_grids);
  const int failures = g_failures + failures3d + failures_tsdf + failures_voxel + failures_grids;
  std::printf("checks: %d (2D) + %d (3D) + %d (TSDF) + %d (voxel filter) + %d (grids), failures: %d\n",
              g_checks, checks3d, checks_tsdf, checks_voxel, checks_grids, failures);
  return failures == 0 ? 0 : 1;
}
