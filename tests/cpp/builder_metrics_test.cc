// The drop-ins' observability (constraint_builder_2d.cc:46-53, :239,
// :260-300, :318-343; constraint_builder_3d.cc:46-59, :257-259, :284-386):
// metric families through an in-memory FamilyFactory, the score histograms
// and the log_matches lines. Driven by tests/test_builder_metrics.py:
//   builder_metrics_test hist v1 v2 ...   ScoreHistogram::ToString(10) (CPU)
//   builder_metrics_test sweep            a scripted 2D and 3D sweep (GPU),
//                                         printed as one JSON object
// The Python mirror runs the same script; the test compares the two and
// checks the counts against the script.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "cartographer_amd/constraint_builder_2d.h"
#include "cartographer_amd/constraint_builder_3d.h"

using namespace cartographer_amd;

static std::string Quote(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '"' || c == '\\') o += '\\', o += c;
    else if (c == '\n') o += "\\n";
    else if (c == '\t') o += "\\t";
    else o += c;
  }
  return o + "\"";
}

static std::string Num(double v) {
  char b[64];
  std::snprintf(b, sizeof(b), "%.17g", v);
  return b;
}

// The scripted 2D world (tests/test_builder_metrics.py sweep_world_2d): an
// 80 x 80 grid at 5 cm, a square ring of occupied cells (index 20 and 60)
// around free cells, unknown outside.
static std::vector<uint16_t> SweepCells() {
  std::vector<uint16_t> cells(80 * 80, 0);
  for (int y = 20; y <= 60; ++y)
    for (int x = 20; x <= 60; ++x)
      cells[y * 80 + x] = (x == 20 || x == 60 || y == 20 || y == 60) ? 1 : 32767;
  return cells;
}

// Node k: 40 points on the ring and 5 k interior points (cell centres).
static PointCloud SweepCloud(int k) {
  PointCloud c;
  auto coord = [](int i) { return static_cast<float>(2.0 - (i + 0.5) * 0.05); };
  for (int j = 0; j < 10; ++j) {
    const int i = 22 + 4 * j;
    c.push_back(coord(20), coord(i), 0.f);
    c.push_back(coord(60), coord(i), 0.f);
    c.push_back(coord(i), coord(20), 0.f);
    c.push_back(coord(i), coord(60), 0.f);
  }
  for (int j = 0; j < 5 * k; ++j) c.push_back(coord(30 + (j * 7) % 21), coord(30 + (j * 3) % 19), 0.f);
  return c;
}

static std::string HistJson(const metrics::InMemoryFamilyFactory& f, const std::string& name,
                            const metrics::Labels& labels) {
  const metrics::BucketHistogram* h = f.histogram(name, labels);
  if (!h) return "null";
  std::string o = "[";
  const auto c = h->counts();
  for (size_t i = 0; i < c.size(); ++i) o += (i ? "," : "") + std::to_string(c[i]);
  return o + "]";
}

static void Sweep() {
  metrics::InMemoryFamilyFactory factory;
  ConstraintBuilder2D::RegisterMetrics(&factory);
  ConstraintBuilder3D::RegisterMetrics(&factory);
  std::vector<std::string> log;
  const std::string m2 = "mapping_constraints_constraint_builder_2d_";
  const std::string m3 = "mapping_constraints_constraint_builder_3d_";
  auto counter = [&](const std::string& name, const char* region, const char* what) {
    const metrics::ValueCounter* c = factory.counter(name, {{"search_region", region}, {"matcher", what}});
    return c ? c->value() : -1.;
  };
  auto gauge = [&](const std::string& name) {
    const metrics::ValueGauge* g = factory.gauge(name);
    return g ? g->value() : -1.;
  };
  std::string out = "{";

  // ---- 2D: two submaps, local pairs of nodes 0..5, global pairs of even nodes,
  // one pair past max_constraint_distance (filtered before the queue).
  {
    ConstraintBuilderOptions o;
    o.sampling_ratio = 1.;
    o.min_score = 0.3f;
    o.global_localization_min_score = 0.35f;
    o.refine_with_ceres = std::getenv("CSM_TEST_NO_REFINE") == nullptr;
    ConstraintBuilder2D b(o);
    b.set_log_sink([&](const std::string& line) { log.push_back("2d " + line); });
    const std::vector<uint16_t> cells = SweepCells();
    Submap2DView s0, s1;
    for (Submap2DView* s : {&s0, &s1}) {
      s->grid.resolution = 0.05;
      s->grid.max_x = 2.;
      s->grid.max_y = 2.;
      s->grid.num_x_cells = 80;
      s->grid.num_y_cells = 80;
      s->grid.cells = cells.data();
    }
    s0.local_pose = Rigid2d{0., 0., 0.};
    s1.local_pose = Rigid2d{0.3, -0.2, 0.1};
    std::vector<PointCloud> clouds;
    for (int k = 0; k < 6; ++k) clouds.push_back(SweepCloud(k));
    for (int k = 0; k < 6; ++k) {
      b.MaybeAddConstraint({0, 0}, &s0, {0, k}, &clouds[k], Rigid2d{0.02 * k, -0.01 * k, 0.01});
      b.MaybeAddConstraint({0, 1}, &s1, {0, k}, &clouds[k],
                           Compose(Inverse(s1.local_pose), Rigid2d{0.03, 0.02 * k, -0.02}));
      if (k % 2 == 0) b.MaybeAddGlobalConstraint({0, 1}, &s1, {0, k}, &clouds[k]);
      b.NotifyEndOfNode();
    }
    b.MaybeAddConstraint({0, 0}, &s0, {0, 9}, &clouds[0], Rigid2d{20., 0., 0.});  // filtered
    out += "\"queue_2d\":" + Num(gauge(m2 + "queue_length"));
    out += ",\"matchers_2d\":" + Num(gauge(m2 + "num_submap_scan_matchers"));
    std::string cons = "[";
    b.WhenDone([&](const ConstraintBuilder2D::Result& r) {
      for (size_t i = 0; i < r.size(); ++i)
        cons += std::string(i ? "," : "") + "[" + std::to_string(r[i].submap_id.submap_index) +
                "," + std::to_string(r[i].node_id.node_index) + "," + Num(r[i].score) + "," +
                Num(r[i].relative_pose.x) + "," + Num(r[i].relative_pose.y) + "," +
                Num(r[i].relative_pose.theta) + "]";
    });
    out += ",\"constraints_2d\":" + cons + "]";
    out += ",\"queue_2d_after\":" + Num(gauge(m2 + "queue_length"));
    b.DeleteScanMatcher({0, 0});
    out += ",\"matchers_2d_after_delete\":" + Num(gauge(m2 + "num_submap_scan_matchers"));
    out += ",\"counters_2d\":[" + Num(counter(m2 + "constraints", "local", "searched")) + "," +
           Num(counter(m2 + "constraints", "local", "found")) + "," +
           Num(counter(m2 + "constraints", "global", "searched")) + "," +
           Num(counter(m2 + "constraints", "global", "found")) + "]";
    out += ",\"hist_2d_local\":" + HistJson(factory, m2 + "scores", {{"search_region", "local"}});
    out += ",\"hist_2d_global\":" + HistJson(factory, m2 + "scores", {{"search_region", "global"}});
    out += ",\"tostring_2d\":" + Quote(b.score_histogram().ToString(10));
  }
  // ---- 3D: ConstraintBuilder3DTest.FindsConstraints' inputs (an empty
  // submap, one point), two rounds.
  {
    ConstraintBuilderOptions o;
    o.sampling_ratio = 1.;
    o.min_score = 0.f;
    o.global_localization_min_score = 0.f;
    o.fast_correlative_scan_matcher_options_3d.min_rotational_score = 0.;
    o.fast_correlative_scan_matcher_options_3d.min_low_resolution_score = 0.;
    ConstraintBuilder3D b(o);
    b.set_log_sink([&](const std::string& line) { log.push_back("3d " + line); });
    Submap3DView submap;
    submap.high_resolution_hybrid_grid.resolution = 0.1f;
    submap.low_resolution_hybrid_grid.resolution = 0.1f;
    submap.rotational_scan_matcher_histogram.assign(3, 0.f);
    TrajectoryNodeData3D node;
    node.high_resolution_point_cloud.push_back(0.1f, 0.2f, 0.3f);
    node.low_resolution_point_cloud.push_back(0.1f, 0.2f, 0.3f);
    node.rotational_scan_matcher_histogram.assign(3, 0.f);
    for (int round = 0; round < 2; ++round) {
      for (int j = 0; j < 2; ++j)
        b.MaybeAddConstraint({0, 1}, &submap, {0, 0}, &node, Rigid3d::Identity(), Rigid3d::Identity());
      b.MaybeAddGlobalConstraint({0, 1}, &submap, {0, 0}, &node, Quaterniond::Identity(),
                                 Quaterniond::Identity());
      b.NotifyEndOfNode();
      if (round == 0) out += ",\"queue_3d\":" + Num(gauge(m3 + "queue_length"));
      b.WhenDone([](const ConstraintBuilder3D::Result&) {});
    }
    out += ",\"queue_3d_after\":" + Num(gauge(m3 + "queue_length"));
    out += ",\"counters_3d\":[" + Num(counter(m3 + "constraints", "local", "searched")) + "," +
           Num(counter(m3 + "constraints", "local", "found")) + "," +
           Num(counter(m3 + "constraints", "global", "searched")) + "," +
           Num(counter(m3 + "constraints", "global", "found")) + "]";
    for (const char* region : {"local", "global"})
      for (const char* kind : {"score", "rotational_score", "low_resolution_score"})
        out += std::string(",\"hist_3d_") + region + "_" + kind + "\":" +
               HistJson(factory, m3 + "scores", {{"search_region", region}, {"kind", kind}});
  }
  out += ",\"log\":[";
  for (size_t i = 0; i < log.size(); ++i) out += (i ? "," : "") + Quote(log[i]);
  out += "]}";
  std::printf("%s\n", out.c_str());
}

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "hist") {
    ScoreHistogram h;
    for (int i = 2; i < argc; ++i) h.Add(std::strtof(argv[i], nullptr));
    std::printf("%s", h.ToString(10).c_str());
    return 0;
  }
  if (argc >= 2 && std::string(argv[1]) == "sweep") {
    Sweep();
    return 0;
  }
  std::fprintf(stderr, "usage: builder_metrics_test hist v... | sweep\n");
  return 2;
}
