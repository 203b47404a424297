// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// The reference's TSDF2D unit tests, restated against the oracle with the
// reference's inputs, checks and tolerances. Each block cites the test it
// restates (mapping/internal/2d/*_test.cc and
// mapping/internal/2d/scan_matching/real_time_correlative_scan_matcher_2d_test.cc).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

#include "oracle_tsdf.h"

using namespace oracle;

namespace {

int g_fail = 0, g_checks = 0;
const char* g_name = "";
#define CHECKT(cond)                                                                \
  do {                                                                              \
    ++g_checks;                                                                     \
    if (!(cond)) {                                                                  \
      ++g_fail;                                                                     \
      std::fprintf(stderr, "[%s] FAILED %s:%d: %s\n", g_name, __FILE__, __LINE__, #cond); \
    }                                                                               \
  } while (0)
#define NEART(a, b, tol) CHECKT(std::abs((double)(a) - (double)(b)) <= (tol))

double NormalizeAngleDifferenceD(double d) {
  while (d > M_PI) d -= 2. * M_PI;
  while (d < -M_PI) d += 2. * M_PI;
  return d;
}

// tsd_value_converter_test.cc:27-121
void TSDValueConverterTests() {
  const float trunc = 0.1f, max_w = 10.0f;
  const TSDValueConverter c(trunc, max_w);
  CHECKT(c.min_tsd() == -trunc && c.max_tsd() == trunc);
  CHECKT(c.min_weight() == 0.f && c.max_weight() == max_w);
  int bad = 0;
  for (int i = 1; i < 32768; ++i) {
    if (c.TSDToValue(c.ValueToTSD(i)) != i) ++bad;
    if (c.TSDToValue(c.ValueToTSD(i + 32768)) != i) ++bad;
    if (c.WeightToValue(c.ValueToWeight(i)) != i) ++bad;
    if (c.WeightToValue(c.ValueToWeight(i + 32768)) != i) ++bad;
  }
  CHECKT(bad == 0);
  const int num_samples = 1000;
  for (int i = 0; i < num_samples; ++i) {
    const float s = -trunc + i * 2.f * trunc / num_samples;
    NEART(c.ValueToTSD(c.TSDToValue(s)), s, trunc * 2.f / 32767.f);
    const float w = i * max_w / num_samples;
    NEART(c.ValueToWeight(c.WeightToValue(w)), w, max_w / 32767.f);
  }
  NEART(c.ValueToWeight(c.WeightToValue(2.f * max_w)), max_w, max_w / 32767.f);
  NEART(c.ValueToWeight(c.WeightToValue(-max_w)), 0.f, max_w / 32767.f);
  NEART(c.ValueToTSD(c.TSDToValue(2.f * trunc)), trunc, trunc * 2.f / 32767.f);
  NEART(c.ValueToTSD(c.TSDToValue(-2.f * trunc)), -trunc, trunc * 2.f / 32767.f);
}

MapLimits Limits(double res, double mx, double my, int nx, int ny) {
  MapLimits l;
  l.resolution = res;
  l.max_x = mx;
  l.max_y = my;
  l.cells = CellLimits{nx, ny};
  return l;
}

// tsdf_2d_test.cc:77-142 (GetCellIndex, WriteRead), :144-166 (CorrectCropping)
void TSDF2DTests() {
  {
    TSDF2D t(Limits(2., 8., 14., 14, 8), 1.f, 10.f);
    const MapLimits& l = t.limits();
    auto is = [&](float x, float y, int ix, int iy) {
      const Idx2 i = l.GetCellIndex(x, y);
      return i.x == ix && i.y == iy;
    };
    CHECKT(is(7.f, 13.f, 0, 0));
    CHECKT(is(7.f, -13.f, 13, 0));
    CHECKT(is(-7.f, 13.f, 0, 7));
    CHECKT(is(-7.f, -13.f, 13, 7));
    CHECKT(is(0.5f, 0.5f, 6, 3));
    CHECKT(is(1.5f, 1.5f, 6, 3));
    CHECKT(is(0.5f, -0.5f, 7, 3));
    CHECKT(is(-0.5f, 0.5f, 6, 4));
    CHECKT(is(-0.5f, -0.5f, 7, 4));
  }
  {
    const float trunc = 1.f, max_w = 10.f;
    TSDF2D t(Limits(1., 1., 2., 2, 2), trunc, max_w);
    std::mt19937 rng(42);
    std::uniform_real_distribution<float> td(-trunc, trunc);
    std::uniform_real_distribution<float> wd(0.f, max_w);
    const float tsd = td(rng), w = wd(rng);
    const Idx2 i = t.limits().GetCellIndex(-0.5f, 0.5f);
    t.SetCell(i, tsd, w);
    NEART(t.GetTSDAndWeight(i).first, tsd, 2.f * trunc / 32768.f);
    NEART(t.GetTSDAndWeight(i).second, w, max_w / 32768.f);
    NEART(t.GetTSD(i), tsd, 2.f * trunc / 32768.f);
    NEART(t.GetWeight(i), w, max_w / 32768.f);
    for (const Idx2& k : {t.limits().GetCellIndex(-0.5f, 1.5f), t.limits().GetCellIndex(0.5f, 0.5f),
                          t.limits().GetCellIndex(0.5f, 1.5f)}) {
      CHECKT(t.limits().Contains(k));
      CHECKT(!t.IsKnown(k));
    }
  }
  {
    const float trunc = 1.f, max_w = 10.f;
    std::mt19937 rng(42);
    std::uniform_real_distribution<float> td(-trunc, trunc);
    std::uniform_real_distribution<float> wd(0.f, max_w);
    TSDF2D t(Limits(0.05, 10., 10., 400, 400), trunc, max_w);
    // XYIndexRangeIterator(min, max) walks x fastest.
    for (int y = 100; y <= 299; ++y)
      for (int x = 100; x <= 299; ++x) {
        const float a = td(rng);
        const float b = wd(rng);
        t.SetCell(Idx2{x, y}, a, b);
      }
    Idx2 off;
    CellLimits cl;
    t.ComputeCroppedLimits(&off, &cl);
    CHECKT(off.x == 100 && off.y == 100);
    CHECKT(cl.num_x_cells == 200 && cl.num_y_cells == 200);
  }
}

// normal_estimation_2d_test.cc:32-140
void NormalEstimationTests() {
  NormalEstimationOptions2D o;
  o.num_normal_samples = 2;
  o.sample_radius = 10.f;
  const size_t num_angles = 100;
  {
    RangeData rd;
    rd.origin = Vec3f{0.f, 0.f, 0.f};
    for (size_t a = 0; a < num_angles; ++a) {
      const double angle = static_cast<double>(a) / static_cast<double>(num_angles) * 2. * M_PI - M_PI;
      rd.returns = {Vec3f{static_cast<float>(std::cos(angle)), static_cast<float>(std::sin(angle)), 0.f}};
      const std::vector<float> n = EstimateNormals(rd, o);
      NEART(NormalizeAngleDifferenceD(angle - n[0] - M_PI), 0.0, 2.0 * M_PI / num_angles + 1e-4);
    }
  }
  {
    RangeData rd;
    rd.origin = Vec3f{0.f, 0.f, 0.f};
    rd.returns = {{-1.f, 1.f, 0.f}, {0.f, 1.f, 0.f}, {1.f, 1.f, 0.f}};
    for (float n : EstimateNormals(rd, o)) NEART(n, -M_PI_2, 1e-4);
    rd.returns = {{1.f, 1.f, 0.f}, {1.f, 0.f, 0.f}, {1.f, -1.f, 0.f}};
    for (float n : EstimateNormals(rd, o)) NEART(std::abs(n), M_PI, 1e-4);
    rd.returns = {{1.f, -1.f, 0.f}, {0.f, -1.f, 0.f}, {-1.f, -1.f, 0.f}};
    for (float n : EstimateNormals(rd, o)) NEART(n, M_PI_2, 1e-4);
    rd.returns = {{-1.f, -1.f, 0.f}, {-1.f, 0.f, 0.f}, {-1.f, 1.f, 0.f}};
    for (float n : EstimateNormals(rd, o)) NEART(n, 0, 1e-4);
  }
  for (int param : {1, 2, 4, 5, 8}) {
    NormalEstimationOptions2D op;
    op.num_normal_samples = param;
    op.sample_radius = 10.f;
    RangeData rd;
    rd.origin = Vec3f{0.f, 0.f, 0.f};
    for (size_t a = 0; a < num_angles; ++a) {
      const double angle = static_cast<double>(a) / static_cast<double>(num_angles) * 2. * M_PI - M_PI;
      rd.returns.push_back(Vec3f{static_cast<float>(std::cos(angle)), static_cast<float>(std::sin(angle)), 0.f});
    }
    const std::vector<float> n = EstimateNormals(rd, op);
    for (size_t a = 0; a < num_angles; ++a) {
      const double angle = static_cast<double>(a) / static_cast<double>(num_angles) * 2. * M_PI;
      NEART(NormalizeAngleDifferenceD(n[a] - angle), 0.0, 2.0 * M_PI / num_angles * param / 2.0 + 1e-4);
    }
  }
}

// tsdf_range_data_inserter_2d_test.cc:28-62 fixture.
TSDFInserterOptions2D FixtureOptions() {
  TSDFInserterOptions2D o;
  o.truncation_distance = 2.0;
  o.maximum_weight = 10.;
  o.update_free_space = false;
  o.normal_estimation.num_normal_samples = 2;
  o.normal_estimation.sample_radius = 10.f;
  o.project_sdf_distance_to_scan_normal = false;
  o.update_weight_range_exponent = 0;
  o.update_weight_angle_scan_normal_to_ray_kernel_bandwidth = 0;
  o.update_weight_distance_cell_to_hit_kernel_bandwidth = 0;
  return o;
}
TSDF2D FixtureGrid() { return TSDF2D(Limits(1., 1., 7., 8, 1), 2.0f, 10.0f); }
void InsertPoint(const TSDFRangeDataInserter2D& ins, TSDF2D* t) {
  RangeData rd;
  rd.returns.push_back(Vec3f{-0.5f, 3.5f, 0.f});
  rd.origin = Vec3f{-0.5f, -0.5f, 0.f};
  ins.Insert(rd, t);
  t->FinishUpdate();
}
// EqualCellProperties (:80-88)
bool Cell(const TSDF2D& t, float x, float y, bool known, float tsd, float w) {
  const Idx2 i = t.limits().GetCellIndex(x, y);
  return t.IsKnown(i) == known && std::abs(tsd - t.GetTSD(i)) < 1e-4 &&
         std::abs(w - t.GetWeight(i)) < 1e-2;
}

// tsdf_range_data_inserter_2d_test.cc:90-347
void TSDFInserterTests() {
  const float trunc = 2.0f, max_w = 10.f;
  for (bool free_space : {false, true}) {  // InsertPoint, InsertPointWithFreeSpaceUpdate
    TSDFInserterOptions2D o = FixtureOptions();
    o.update_free_space = free_space;
    const TSDFRangeDataInserter2D ins(o);
    TSDF2D t = FixtureGrid();
    InsertPoint(ins, &t);
    for (float y = free_space ? -0.5f : 1.5f; y < 6.; ++y) {
      CHECKT(Cell(t, -0.5f, y, true, std::max(std::min(3.5f - y, trunc), -trunc), 1.f));
      CHECKT(Cell(t, 0.5f, y, false, -trunc, 0.f));
      CHECKT(Cell(t, 1.5f, y, false, -trunc, 0.f));
    }
    CHECKT(Cell(t, free_space ? -0.5f : 0.5f, 6.5f, false, -trunc, 0.f));
    CHECKT(Cell(t, -0.5f, -1.5f, false, -trunc, 0.f));
    for (int i = 0; i < 1000; ++i) InsertPoint(ins, &t);
    for (float y = free_space ? -0.5f : 1.5f; y < 6.; ++y)
      CHECKT(Cell(t, -0.5f, y, true, std::max(std::min(3.5f - y, trunc), -trunc), max_w));
  }
  for (int exponent : {1, 2}) {  // InsertPointLinearWeight, InsertPointQuadraticWeight
    TSDFInserterOptions2D o = FixtureOptions();
    o.update_weight_range_exponent = exponent;
    const TSDFRangeDataInserter2D ins(o);
    TSDF2D t = FixtureGrid();
    InsertPoint(ins, &t);
    for (float y = 1.5f; y < 6.; ++y)
      CHECKT(Cell(t, -0.5f, y, true, std::max(std::min(3.5f - y, trunc), -trunc),
                  exponent == 1 ? 1.f / 4.f : 1.f / std::pow(4.f, 2)));
  }
  {  // InsertSmallAnglePointWithoutNormalProjection
    const TSDFRangeDataInserter2D ins(FixtureOptions());
    TSDF2D t = FixtureGrid();
    RangeData rd;
    rd.returns = {{-0.5f, 3.5f, 0.f}, {5.5f, 3.5f, 0.f}, {10.5f, 3.5f, 0.f}};
    rd.origin = Vec3f{-0.5f, -0.5f, 0.f};
    ins.Insert(rd, &t);
    t.FinishUpdate();
    const float x = 4.5f, y = 2.5f;
    const float rx = -0.5f - 5.5f, ry = -0.5f - 3.5f;
    const float ray_length = std::sqrt(rx * rx + ry * ry);
    const float ox = x + 0.5f, oy = y + 0.5f;
    const float expected = ray_length - std::sqrt(ox * ox + oy * oy);
    CHECKT(Cell(t, x, y, true, expected, 1.f));
  }
  {  // InsertSmallAnglePointWitNormalProjection
    TSDFInserterOptions2D o = FixtureOptions();
    o.project_sdf_distance_to_scan_normal = true;
    const TSDFRangeDataInserter2D ins(o);
    TSDF2D t = FixtureGrid();
    RangeData rd;
    rd.returns = {{-0.5f, 3.5f, 0.f}, {5.5f, 3.5f, 0.f}};
    rd.origin = Vec3f{-0.5f, -0.5f, 0.f};
    ins.Insert(rd, &t);
    t.FinishUpdate();
    CHECKT(Cell(t, 4.5f, 2.5f, true, 1.f, 1.f));
    CHECKT(Cell(t, 6.5f, 4.5f, true, -1.f, 1.f));
  }
  {  // InsertPointsWithAngleScanNormalToRayWeight
    const float bw = 10.f;
    TSDFInserterOptions2D o = FixtureOptions();
    o.update_weight_angle_scan_normal_to_ray_kernel_bandwidth = bw;
    const TSDFRangeDataInserter2D ins(o);
    TSDF2D t = FixtureGrid();
    RangeData rd;
    rd.returns = {{-0.5f, 3.5f, 0.f}, {5.5f, 3.5f, 0.f}};
    rd.origin = Vec3f{-0.5f, -0.5f, 0.f};
    ins.Insert(rd, &t);
    t.FinishUpdate();
    float expected = 1.f / (std::sqrt(2 * M_PI) * bw);
    NEART(expected, t.GetWeight(t.limits().GetCellIndex(-0.5f, 3.5f)), 1e-3);
    NEART(expected, t.GetWeight(t.limits().GetCellIndex(6.5f, 4.5f)), 1e-3);
    const float angle = std::atan(7.f / 5.f);
    expected = 1.f / (std::sqrt(2 * M_PI) * bw) * std::exp(angle * angle / (2 * std::pow(bw, 2)));
    NEART(expected, t.GetWeight(t.limits().GetCellIndex(6.5f, 4.5f)), 1e-3);
  }
  {  // InsertPointsWithDistanceCellToHit
    const float bw = 10.f;
    TSDFInserterOptions2D o = FixtureOptions();
    o.update_weight_distance_cell_to_hit_kernel_bandwidth = bw;
    const TSDFRangeDataInserter2D ins(o);
    TSDF2D t = FixtureGrid();
    InsertPoint(ins, &t);
    for (float y = 1.5f; y < 6.; ++y) {
      const float e_tsd = std::max(std::min(3.5f - y, trunc), -trunc);
      const float e_w = 1.f / (std::sqrt(2 * M_PI) * bw) * std::exp(std::pow(e_tsd, 2) / (2 * std::pow(bw, 2)));
      CHECKT(Cell(t, -0.5f, y, true, e_tsd, e_w));
    }
  }
}

// real_time_correlative_scan_matcher_2d_test.cc:54-92, 143-159, 180-198
PointCloud SevenPoints() {
  return {{0.025f, 0.175f, 0.f},  {-0.025f, 0.175f, 0.f}, {-0.075f, 0.175f, 0.f},
          {-0.125f, 0.175f, 0.f}, {-0.125f, 0.125f, 0.f}, {-0.125f, 0.075f, 0.f},
          {-0.125f, 0.025f, 0.f}};
}
void RealTimeTSDFTests() {
  TSDF2D t(Limits(0.05, 0.3, 0.5, 20, 20), 0.3f, 1.0f);
  TSDFInserterOptions2D o;
  o.truncation_distance = 0.3;
  o.maximum_weight = 10.;
  o.update_free_space = false;
  o.normal_estimation.num_normal_samples = 4;
  o.normal_estimation.sample_radius = 0.5f;
  o.project_sdf_distance_to_scan_normal = true;
  o.update_weight_range_exponent = 0;
  o.update_weight_angle_scan_normal_to_ray_kernel_bandwidth = 0.5;
  o.update_weight_distance_cell_to_hit_kernel_bandwidth = 0.5;
  RangeData rd;
  rd.origin = Vec3f{0.5f, -0.5f, 0.f};
  rd.returns = SevenPoints();
  TSDFRangeDataInserter2D(o).Insert(rd, &t);
  t.FinishUpdate();
  RealTimeOptions ro;
  ro.linear_search_window = 0.6;
  ro.angular_search_window = 0.16;
  ro.translation_delta_cost_weight = 0.;
  ro.rotation_delta_cost_weight = 0.;
  const SearchParameters sp(0, 0, 0., 0.);
  const auto d = DiscretizeScans(t.limits(), GenerateRotatedScans(SevenPoints(), sp), 0.f, 0.f);
  {
    std::vector<Candidate2D> c{Candidate2D(0, 0, 0, sp)};
    RealTimeScoreCandidatesTSDF(ro, t, d, &c);
    CHECKT(c[0].scan_index == 0 && c[0].x_index_offset == 0 && c[0].y_index_offset == 0);
    NEART(c[0].score, 1.0, 1e-1);
    CHECKT(0.95 < c[0].score);
  }
  {
    std::vector<Candidate2D> c{Candidate2D(0, 0, 1, sp)};
    RealTimeScoreCandidatesTSDF(ro, t, d, &c);
    CHECKT(c[0].scan_index == 0 && c[0].x_index_offset == 0 && c[0].y_index_offset == 1);
    CHECKT(1.0 - 4. / (7. * 6.) < c[0].score);
    CHECKT(1.0 > c[0].score);
  }
}

}  // namespace

int RunRefTestsTSDF(int* checks) {
  const int before = g_fail;
  struct {
    const char* name;
    void (*fn)();
  } tests[] = {{"TSDValueConverterTest (9 cases)", TSDValueConverterTests},
               {"TSDF2DTest (GetCellIndex, WriteRead, CorrectCropping)", TSDF2DTests},
               {"NormalEstimation2DTest + CircularGeometry2DTest {1,2,4,5,8}", NormalEstimationTests},
               {"RangeDataInserterTest2DTSDF (8 cases)", TSDFInserterTests},
               {"RealTimeCorrelativeScanMatcherTest TSDF (2 cases)", RealTimeTSDFTests}};
  for (auto& t : tests) {
    g_name = t.name;
    const int b = g_fail;
    t.fn();
    std::printf("%-70s %s\n", t.name, g_fail == b ? "OK" : "FAILED");
  }
  *checks = g_checks;
  return g_fail - before;
}
