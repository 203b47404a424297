// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// The reference's 3D scan-matching unit tests, restated against the oracle
// (same libstdc++ engines and distributions, same checks and tolerances).
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "oracle3d.h"

using namespace oracle;

namespace {

int g_fail = 0, g_checks = 0;
const char* g_name = "";
#define CHECK3(cond)                                                                \
  do {                                                                              \
    ++g_checks;                                                                     \
    if (!(cond)) {                                                                  \
      ++g_fail;                                                                     \
      std::fprintf(stderr, "[%s] FAILED %s:%d: %s\n", g_name, __FILE__, __LINE__, #cond); \
    }                                                                               \
  } while (0)

// rigid_transform_test_helpers.h:37-46 — Eigen isApprox on the 4x4 affine
// matrices: ||a - b||² <= eps² · min(||a||², ||b||²).
void Matrix(const Vec3d& t, const Quatd& q, double m[16]) {
  const double x = q.x, y = q.y, z = q.z, w = q.w;
  const double tx = 2 * x, ty = 2 * y, tz = 2 * z;
  const double twx = tx * w, twy = ty * w, twz = tz * w, txx = tx * x, txy = ty * x,
               txz = tz * x, tyy = ty * y, tyz = tz * y, tzz = tz * z;
  const double r[9] = {1 - (tyy + tzz), txy - twz, txz + twy, txy + twz, 1 - (txx + tzz),
                       tyz - twx,       txz - twy, tyz + twx, 1 - (txx + tyy)};
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) m[i * 4 + j] = r[i * 3 + j];
  }
  m[3] = t.x;
  m[7] = t.y;
  m[11] = t.z;
  m[12] = m[13] = m[14] = 0;
  m[15] = 1;
}

bool IsNearly3D(const Rigid3d& a, const Rigid3d& b, double eps) {
  double ma[16], mb[16];
  Matrix(a.t, a.q, ma);
  Matrix(b.t, b.q, mb);
  double d = 0, na = 0, nb = 0;
  for (int i = 0; i < 16; ++i) {
    d += (ma[i] - mb[i]) * (ma[i] - mb[i]);
    na += ma[i] * ma[i];
    nb += mb[i] * mb[i];
  }
  return d <= eps * eps * std::min(na, nb);
}

Rigid3d ToD(const Rigid3f& a) {
  return Rigid3d{Vec3d{a.t.x, a.t.y, a.t.z}, Quatd{a.q.w, a.q.x, a.q.y, a.q.z}};
}

// ------------------------------------------------------------------ RTCSM3D --
// real_time_correlative_scan_matcher_3d_test.cc:34-117
void RealTimeCorrelativeScanMatcher3DTests() {
  g_name = "RealTimeCorrelativeScanMatcher3DTest.*";
  HybridGrid grid(0.1f);
  const Rigid3d expected{Vec3d{-1., 0., 0.}, Quatd{1., 0., 0., 0.}};
  const Rigid3f expected_f{Vec3f{-1.f, 0.f, 0.f}, Quatf{1.f, 0.f, 0.f, 0.f}};
  PointCloud cloud;
  for (const Vec3f& p : {Vec3f{-3.f, 2.f, 0.f}, Vec3f{-4.f, 2.f, 0.f}, Vec3f{-5.f, 2.f, 0.f},
                         Vec3f{-6.f, 2.f, 0.f}, Vec3f{-6.f, 3.f, 1.f}, Vec3f{-6.f, 4.f, 2.f},
                         Vec3f{-7.f, 3.f, 1.f}}) {
    cloud.push_back(p);
    grid.SetProbability(grid.GetCellIndex(Apply3(expected_f, p)), 1.f);
  }
  RtOptions3D o;
  o.linear_search_window = 0.3;
  o.angular_search_window = 1. * M_PI / 180.;  // math.rad(1.)
  o.translation_delta_cost_weight = 1e-1;
  o.rotation_delta_cost_weight = 1.;
  auto from = [&](const Rigid3d& initial) {
    const Rt3dResult r = RealTimeMatch3D(o, initial, cloud, grid);
    CHECK3(IsNearly3D(r.pose, expected, 1e-3));
  };
  // Eigen::Quaterniond(Eigen::AngleAxisd(angle, axis)) with the axis as given:
  // the test's (0, 1, 1) is not normalized, so that quaternion is not unit.
  auto aa = [](double angle, double ax, double ay, double az) {
    const double s = std::sin(0.5 * angle);
    return Quatd{std::cos(0.5 * angle), s * ax, s * ay, s * az};
  };
  from(Rigid3d{Vec3d{-1., 0., 0.}, Quatd{1, 0, 0, 0}});     // PerfectEstimate
  from(Rigid3d{Vec3d{-0.8, 0., 0.}, Quatd{1, 0, 0, 0}});    // AlongX
  from(Rigid3d{Vec3d{-1., 0., -0.2}, Quatd{1, 0, 0, 0}});   // AlongZ
  from(Rigid3d{Vec3d{-0.9, -0.2, 0.2}, Quatd{1, 0, 0, 0}}); // AlongXYZ
  from(Rigid3d{Vec3d{-1., 0., 0.}, aa(0.8 / 180. * M_PI, 1., 0., 0.)});  // RotationAroundX
  from(Rigid3d{Vec3d{-1., 0., 0.}, aa(0.8 / 180. * M_PI, 0., 1., 0.)});  // RotationAroundY
  from(Rigid3d{Vec3d{-1., 0., 0.}, aa(0.8 / 180. * M_PI, 0., 1., 1.)});  // RotationAroundYZ
}

// ---------------------------------------------------- PrecomputationGrid3D --
// precomputation_grid_3d_test.cc:31-77
void PrecomputationGrid3DTest() {
  g_name = "PrecomputedGridGenerator3DTest.TestAgainstNaiveAlgorithm";
  HybridGrid grid(2.f);
  std::mt19937 rng(23847);
  std::uniform_int_distribution<int> coord(-50, 49);
  std::uniform_real_distribution<float> value(kMinProbability, kMaxProbability);
  for (int i = 0; i < 1000; ++i) {
    const int x = coord(rng);
    const int y = coord(rng);
    const int z = coord(rng);
    grid.SetProbability(Idx3{x, y, z}, value(rng));
  }
  std::vector<std::unique_ptr<PrecomputationGrid3D>> levels;
  for (int depth = 0; depth <= 3; ++depth) {
    if (depth == 0) {
      levels.push_back(ConvertToPrecomputationGrid(grid));
    } else {
      const int s = 1 << (depth - 1);
      levels.push_back(PrecomputeGrid(*levels.back(), false, Idx3{s, s, s}));
    }
    const int width = 1 << depth;
    for (int i = 0; i < 100; ++i) {
      const int x = coord(rng);
      const int y = coord(rng);
      const int z = coord(rng);
      float max_probability = 0.f;
      for (int dx = 0; dx < width; ++dx)
        for (int dy = 0; dy < width; ++dy)
          for (int dz = 0; dz < width; ++dz)
            max_probability =
                std::max(max_probability, grid.GetProbability(Idx3{x + dx, y + dy, z + dz}));
      CHECK3(std::abs(max_probability -
                      ToProbability3D(levels.back()->value(Idx3{x, y, z}))) <= 1e-2);
    }
  }
}

// --------------------------------------------------- RotationalScanMatcher --
// rotational_scan_matcher_test.cc:28-67
void RotationalScanMatcherTests() {
  g_name = "RotationalScanMatcher3DTest.OnlySameHistogramIsScoreOne";
  {
    const std::vector<float> h = {1.f, 43.f, 0.5f, 0.3123f, 23.f, 42.f, 0.f};
    const std::vector<float> s = RotationalMatch(h, h, 0.f, {0.f, 1.f});
    CHECK3(s.size() == 2);
    CHECK3(std::abs(1.f - s[0]) <= 1e-6);
    CHECK3(1.f > s[1]);
  }
  g_name = "RotationalScanMatcher3DTest.InterpolatesAsExpected";
  {
    constexpr int kNumBuckets = 10;
    constexpr float kAnglePerBucket = M_PI / kNumBuckets;
    auto unit = [](int i) {
      std::vector<float> v(kNumBuckets, 0.f);
      v[i] = 1.f;
      return v;
    };
    const std::vector<float> submap = unit(3);
    for (float t = 0.f; t < 1.f; t += 0.1f) {
      const float expected = t / std::hypot(t, 1 - t);
      std::vector<float> s = RotationalMatch(submap, unit(2), 0.f, {t * kAnglePerBucket});
      CHECK3(s.size() == 1 && std::abs(expected - s[0]) <= 1e-6);
      s = RotationalMatch(submap, unit(2), 0.f, {(2 - t) * kAnglePerBucket});
      CHECK3(s.size() == 1 && std::abs(expected - s[0]) <= 1e-6);
      s = RotationalMatch(submap, unit(4), 0.f, {-t * kAnglePerBucket, (t - 2) * kAnglePerBucket});
      CHECK3(s.size() == 2 && std::abs(expected - s[0]) <= 1e-6 &&
             std::abs(expected - s[1]) <= 1e-6);
    }
  }
}

// --------------------------------------------- FastCorrelativeScanMatcher3D --
// fast_correlative_scan_matcher_3d_test.cc:36-204
struct Fast3dFixture {
  std::mt19937 prng{42};
  std::uniform_real_distribution<float> dist{-1.f, 1.f};
  RangeDataInserter3D inserter{0.7f, 0.4f, 5};
  FastCsm3dOptions options;
  PointCloud cloud;
  std::vector<float> histogram = std::vector<float>(10, 0.f);
  std::unique_ptr<HybridGrid> grid;

  Fast3dFixture() {
    options.branch_and_bound_depth = 6;
    options.full_resolution_depth = 6;
    options.min_rotational_score = 0.1;
    options.min_low_resolution_score = 0.15;
    options.linear_xy_search_window = 0.8;
    options.linear_z_search_window = 0.8;
    options.angular_search_window = 0.3;
    for (const Vec3f& p : {Vec3f{4.f, 0.f, 0.f}, Vec3f{4.5f, 0.f, 0.f}, Vec3f{5.f, 0.f, 0.f},
                           Vec3f{5.5f, 0.f, 0.f}, Vec3f{0.f, 4.f, 0.f}, Vec3f{0.f, 4.5f, 0.f},
                           Vec3f{0.f, 5.f, 0.f}, Vec3f{0.f, 5.5f, 0.f}, Vec3f{0.f, 0.f, 4.f},
                           Vec3f{0.f, 0.f, 4.5f}, Vec3f{0.f, 0.f, 5.f}, Vec3f{0.f, 0.f, 5.5f}})
      cloud.push_back(p);
  }
  Rigid3f RandomPose() {
    const float x = 0.7f * dist(prng);
    const float y = 0.7f * dist(prng);
    const float z = 0.7f * dist(prng);
    const float theta = 0.2f * dist(prng);
    return Mul3(Rigid3f{Vec3f{x, y, z}, Quatf{1.f, 0.f, 0.f, 0.f}},
                Rigid3f{Vec3f{0.f, 0.f, 0.f}, QuatFromAngleAxisF(theta, 0.f, 0.f, 1.f)});
  }
  std::unique_ptr<FastCorrelativeScanMatcher3D> Matcher(const Rigid3f& pose) {
    grid.reset(new HybridGrid(0.05f));
    inserter.Insert(pose.t, TransformPointCloud(cloud, pose), grid.get());
    grid->FinishUpdate();
    return std::unique_ptr<FastCorrelativeScanMatcher3D>(
        new FastCorrelativeScanMatcher3D(*grid, grid.get(), &histogram, options));
  }
  NodeData3D Node(const PointCloud& low) const {
    NodeData3D n;
    n.high_resolution_point_cloud = cloud;
    n.low_resolution_point_cloud = low;
    n.rotational_scan_matcher_histogram = histogram;
    return n;
  }
};

void FastCorrelativeScanMatcher3DTests() {
  constexpr float kMinScore = 0.1f;
  const PointCloud far = {Vec3f{42.f, 42.f, 42.f}};
  g_name = "FastCorrelativeScanMatcher3DTest.CorrectPoseForMatch";
  {
    Fast3dFixture f;
    for (int i = 0; i != 20; ++i) {
      const Rigid3f expected = f.RandomPose();
      auto m = f.Matcher(expected);
      const Rigid3d id;
      const Fast3dResult r = m->Match(id, id, f.Node(f.cloud), kMinScore);
      CHECK3(r.matched);
      CHECK3(kMinScore < r.score);
      CHECK3(0.09f < r.rotational_score);
      CHECK3(0.14f < r.low_resolution_score);
      CHECK3(IsNearly3D(ToD(expected), r.pose, 0.05));
      const Fast3dResult low = m->Match(id, id, f.Node(far), kMinScore);
      CHECK3(!low.matched);
    }
  }
  g_name = "FastCorrelativeScanMatcher3DTest.CorrectPoseForMatchFullSubmap";
  {
    Fast3dFixture f;
    const Rigid3f expected = f.RandomPose();
    auto m = f.Matcher(expected);
    const Quatd id{1., 0., 0., 0.};
    const Fast3dResult r = m->MatchFullSubmap(id, id, f.Node(f.cloud), kMinScore);
    CHECK3(r.matched);
    CHECK3(kMinScore < r.score);
    CHECK3(0.09f < r.rotational_score);
    CHECK3(0.14f < r.low_resolution_score);
    CHECK3(IsNearly3D(ToD(expected), r.pose, 0.05));
    const Fast3dResult low = m->MatchFullSubmap(id, id, f.Node(far), kMinScore);
    CHECK3(!low.matched);
  }
}

// Eigen SSE quaternion product vs the textbook formula: same rotation.
void QuaternionSanity() {
  g_name = "Eigen float helpers";
  const Quatf a = QuatNormalizedSse(Quatf{0.9f, 0.1f, -0.3f, 0.2f});
  const Quatf b = QuatNormalizedSse(Quatf{0.5f, -0.5f, 0.4f, 0.1f});
  const Quatf p = QuatMulSse(a, b);
  const Quatf g = QuatMul(a, b);
  CHECK3(std::abs(p.w - g.w) < 1e-6f && std::abs(p.x - g.x) < 1e-6f &&
         std::abs(p.y - g.y) < 1e-6f && std::abs(p.z - g.z) < 1e-6f);
  const float v[11] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
  CHECK3(ReduxSumSse(v, 11) == 66.f);
}

}  // namespace

namespace {

Quatd AngleAxisQ(double angle, double ax, double ay, double az) {
  const double n = std::sqrt(ax * ax + ay * ay + az * az);
  const double s = std::sin(0.5 * angle) / n;
  return Quatd{std::cos(0.5 * angle), ax * s, ay * s, az * s};
}
Quatd Mul(const Quatd& a, const Quatd& b) {
  return Quatd{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z,
               a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
               a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x,
               a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w};
}
double RotationDeltaSquaredCost(const Quatd& rotation, double scale, const Quatd& target) {
  const double q[4] = {rotation.w, rotation.x, rotation.y, rotation.z};
  const double t[4] = {target.w, target.x, target.y, target.z};
  double r[3];
  RotationDeltaResiduals3D(scale, t, q, r);
  return r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
}

// rotation_delta_cost_functor_3d_test.cc:50-83 (kPrecision 1e-8).
void RotationDeltaCostFunctor3DTests() {
  const Quatd id{1., 0., 0., 0.};
  CHECK3(std::abs(RotationDeltaSquaredCost(id, 1.0, id)) <= 1e-8);
  const Quatd rot = AngleAxisQ(0.9, 0.2, 0.1, 0.3);
  CHECK3(std::abs(RotationDeltaSquaredCost(rot, 1.0, rot)) <= 1e-8);
  const double scaling = 1.2, angle = 0.8;
  const Quatd rotation = AngleAxisQ(angle, 0.2, 0.1, 0.8);
  const Quatd target = AngleAxisQ(0.2, -0.5, 0.3, 0.4);
  const double expected = std::pow(scaling * std::sin(angle / 2.0), 2);
  CHECK3(std::abs(expected - RotationDeltaSquaredCost(rotation, scaling, id)) <= 1e-8);
  CHECK3(std::abs(expected - RotationDeltaSquaredCost(Mul(target, rotation), scaling, target)) <=
         1e-8);
  CHECK3(std::abs(expected - RotationDeltaSquaredCost(Mul(rotation, target), scaling, target)) <=
         1e-8);
}

// ceres_scan_matcher_3d_test.cc (the upstream test the fork keeps as
// ceres_scan_matcher_3d_test.cc.bak:34-136): seven points set to probability
// 1 in a 1 m HybridGrid at expected_pose = Translation(-1, 0, 0) * point;
// occupied_space_weight_0 = 1, translation_weight 0.01, rotation_weight 0.1,
// use_nonmonotonic_steps, max_num_iterations 10; final_cost ~ 0 (1e-2) and
// IsNearly(expected, 3e-2) from five initial poses. The test's intensity
// block (IntensityHybridGrid, weight 0.5) is left out: ConstraintBuilder3D
// passes no intensity grid (constraint_builder_3d.cc:267-274), so neither
// the oracle nor the device path carries that cost.
void CeresScanMatcher3DTests() {
  HybridGrid grid(1.f);
  std::vector<Vec3f> cloud;
  const float pts[7][3] = {{-3.f, 2.f, 0.f}, {-4.f, 2.f, 0.f}, {-5.f, 2.f, 0.f}, {-6.f, 2.f, 0.f},
                           {-6.f, 3.f, 1.f}, {-6.f, 4.f, 2.f}, {-7.f, 3.f, 1.f}};
  for (const auto& p : pts) {
    cloud.push_back(Vec3f{p[0], p[1], p[2]});
    grid.SetProbability(grid.GetCellIndex(Vec3f{p[0] + -1.f, p[1], p[2]}), 1.f);
  }
  CeresOptions3D o;
  o.w0 = 1.;
  o.w1 = 0.;  // one (cloud, grid) pair in the test: the second block is inert
  o.wt = 0.01;
  o.wr = 0.1;
  o.max_num_iterations = 10;
  o.use_nonmonotonic_steps = true;
  auto run = [&](const std::vector<Vec3f>& c, const Rigid3d& initial, const Rigid3d& expected) {
    const double t0[3] = {initial.t.x, initial.t.y, initial.t.z};
    const double q0[4] = {initial.q.w, initial.q.x, initial.q.y, initial.q.z};
    double t[3], q[4], final_cost = -1.;
    CeresMatch3D(grid, grid, c, c, o, t0, t0, q0, t, q, &final_cost);
    CHECK3(std::abs(final_cost) <= 1e-2);
    CHECK3(IsNearly3D(Rigid3d{Vec3d{t[0], t[1], t[2]}, Quatd{q[0], q[1], q[2], q[3]}}, expected,
                      3e-2));
  };
  const Quatd id{1., 0., 0., 0.};
  const Rigid3d expected{Vec3d{-1., 0., 0.}, id};
  run(cloud, Rigid3d{Vec3d{-1., 0., 0.}, id}, expected);     // PerfectEstimate
  run(cloud, Rigid3d{Vec3d{-0.8, 0., 0.}, id}, expected);    // AlongX
  run(cloud, Rigid3d{Vec3d{-1., 0., -0.2}, id}, expected);   // AlongZ
  run(cloud, Rigid3d{Vec3d{-0.9, -0.2, 0.2}, id}, expected); // AlongXYZ
  // FullPoseCorrection: the cloud rotated by 0.05 about z; expected pose
  // expected * additional^-1; start rotated about x.
  const Quatd add = AngleAxisQ(0.05, 0., 0., 1.);
  std::vector<Vec3f> turned;
  for (const Vec3f& p : cloud) {
    const double c = std::cos(0.05), s = std::sin(0.05);
    turned.push_back(Vec3f{static_cast<float>(c * p.x - s * p.y),
                           static_cast<float>(s * p.x + c * p.y), p.z});
  }
  const Rigid3d expected2{Vec3d{-1., 0., 0.}, Quatd{add.w, -add.x, -add.y, -add.z}};
  run(turned, Rigid3d{Vec3d{-0.95, -0.05, 0.05}, AngleAxisQ(0.05, 1., 0., 0.)}, expected2);
}

}  // namespace

int RunRefTests3D(int* checks) {
  const int before = g_fail;
  struct {
    const char* name;
    void (*fn)();
  } tests[] = {{"RealTimeCorrelativeScanMatcher3DTest (7 cases)", RealTimeCorrelativeScanMatcher3DTests},
               {"PrecomputedGridGenerator3DTest.TestAgainstNaiveAlgorithm", PrecomputationGrid3DTest},
               {"RotationalScanMatcher3DTest (2 cases)", RotationalScanMatcherTests},
               {"FastCorrelativeScanMatcher3DTest (Match, MatchFullSubmap)", FastCorrelativeScanMatcher3DTests},
               {"Eigen float helpers (SSE product, redux)", QuaternionSanity},
               {"RotationDeltaCostFunctor3DTest (2 cases)", RotationDeltaCostFunctor3DTests},
               {"CeresScanMatcher3DTest (5 cases, no intensity block)", CeresScanMatcher3DTests}};
  for (auto& t : tests) {
    const int b = g_fail;
    t.fn();
    std::printf("%-70s %s\n", t.name, g_fail == b ? "OK" : "FAILED");
  }
  *checks = g_checks;
  return g_fail - before;
}
