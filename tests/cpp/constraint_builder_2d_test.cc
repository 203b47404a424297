// C++ restatement of ConstraintBuilder2DTest (reference
// mapping/internal/constraints/constraint_builder_2d_test.cc:58-128) against
// the drop-in headers. Exits 0 when every check holds; prints the failing
// check otherwise. Compiled by tests/test_constraint_builder.py (CPU) and run
// there on the GPU.
#include <cstdio>
#include <vector>

#include "cartographer_amd/constraint_builder_2d.h"

using namespace cartographer_amd;

static int failures = 0;
#define EXPECT(cond)                                                  \
  do {                                                                \
    if (!(cond)) {                                                    \
      std::fprintf(stderr, "%s:%d: EXPECT(%s)\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                     \
    }                                                                 \
  } while (0)

static ConstraintBuilderOptions TestOptions() {
  ConstraintBuilderOptions o;  // pose_graph.lua defaults, then the test's overrides
  o.sampling_ratio = 1;
  o.min_score = 0;
  o.global_localization_min_score = 0;
  return o;
}

static void CallsBack() {
  ConstraintBuilder2D builder(TestOptions());
  EXPECT(builder.GetNumFinishedNodes() == 0);
  builder.NotifyEndOfNode();
  size_t n = 99;
  builder.WhenDone([&](const ConstraintBuilder2D::Result& r) { n = r.size(); });
  EXPECT(n == 0);
  EXPECT(builder.GetNumFinishedNodes() == 1);
}

static void FindsConstraints() {
  ConstraintBuilder2D builder(TestOptions());
  PointCloud cloud;
  cloud.push_back(0.1f, 0.2f, 0.3f);
  // MapLimits(1., (2., 3.), CellLimits(100, 110)), all cells unknown.
  std::vector<uint16_t> cells(100 * 110, 0);
  Submap2DView submap;
  submap.grid.resolution = 1.;
  submap.grid.max_x = 2.;
  submap.grid.max_y = 3.;
  submap.grid.num_x_cells = 100;
  submap.grid.num_y_cells = 110;
  submap.grid.cells = cells.data();
  submap.local_pose = Rigid2d{4., 5., 0.};  // Submap2D origin (4, 5)
  const SubmapId submap_id{0, 1};
  int expected_nodes = 0;
  for (int i = 0; i < 2; ++i) {
    EXPECT(builder.GetNumFinishedNodes() == expected_nodes);
    for (int j = 0; j < 2; ++j)
      builder.MaybeAddConstraint(submap_id, &submap, NodeId{0, 0}, &cloud, Rigid2d::Identity());
    builder.MaybeAddGlobalConstraint(submap_id, &submap, NodeId{0, 0}, &cloud);
    builder.NotifyEndOfNode();
    EXPECT(builder.GetNumFinishedNodes() == ++expected_nodes);
    builder.NotifyEndOfNode();
    EXPECT(builder.GetNumFinishedNodes() == ++expected_nodes);
    ConstraintBuilder2D::Result result;
    builder.WhenDone([&](const ConstraintBuilder2D::Result& r) { result = r; });
    EXPECT(result.size() == 3);
    for (const Constraint& c : result) EXPECT(c.tag == Constraint::INTER_SUBMAP);
    // The constraints' poses, compared with the oracle by the Python runner
    // (tests/test_constraint_builder.py): every leaf ties on this grid.
    if (i == 0)
      for (const Constraint& c : result)
        std::printf("FINDS_CONSTRAINTS %.17g %.17g %.17g %.9g\n", c.relative_pose.x,
                    c.relative_pose.y, c.relative_pose.theta, c.score);
    builder.DeleteScanMatcher(submap_id);
  }
  EXPECT(builder.constraints_searched == 4 && builder.constraints_found == 4);
  EXPECT(builder.global_constraints_searched == 2 && builder.global_constraints_found == 2);
}

// A cloud past the device path's limit (more than 16448 points: CSM_ERANGE)
// is skipped and counted; the other pairs of the flush still produce their
// constraints and the process does not abort.
static void SkipsUnsearchablePairs() {
  ConstraintBuilder2D builder(TestOptions());
  PointCloud small, huge;
  small.push_back(0.1f, 0.2f, 0.3f);
  for (int i = 0; i < 16449; ++i) huge.push_back(0.001f * (i % 100), 0.001f * (i / 100), 0.f);
  std::vector<uint16_t> cells(100 * 110, 0);
  Submap2DView submap;
  submap.grid.resolution = 1.;
  submap.grid.max_x = 2.;
  submap.grid.max_y = 3.;
  submap.grid.num_x_cells = 100;
  submap.grid.num_y_cells = 110;
  submap.grid.cells = cells.data();
  submap.local_pose = Rigid2d{4., 5., 0.};
  const SubmapId submap_id{0, 1};
  builder.MaybeAddGlobalConstraint(submap_id, &submap, NodeId{0, 0}, &small);
  builder.MaybeAddGlobalConstraint(submap_id, &submap, NodeId{0, 1}, &huge);
  builder.NotifyEndOfNode();
  ConstraintBuilder2D::Result result;
  builder.WhenDone([&](const ConstraintBuilder2D::Result& r) { result = r; });
  EXPECT(result.size() == 1);
  EXPECT(result.size() == 1 && result[0].node_id.node_index == 0);
  EXPECT(builder.constraints_failed == 1 && builder.last_error == CSM_ERANGE);
  EXPECT(builder.global_constraints_searched == 1 && builder.global_constraints_found == 1);
}

// Node clouds stay resident across flushes (csm_scan_set_append). A node
// whose cloud changes between flushes is searched with the new points: the
// second flush of a long-lived builder equals a fresh builder's result.
static void ReusesResidentCloudsAcrossFlushes() {
  std::vector<uint16_t> cells(100 * 110, 0);
  // An L of occupied cells (correspondence cost value 1: probability 0.9).
  for (int x = 10; x <= 14; ++x) cells[20 * 100 + x] = 1;
  for (int y = 21; y <= 23; ++y) cells[y * 100 + 10] = 1;
  Submap2DView submap;
  submap.grid.resolution = 1.;
  submap.grid.max_x = 2.;
  submap.grid.max_y = 3.;
  submap.grid.num_x_cells = 100;
  submap.grid.num_y_cells = 110;
  submap.grid.cells = cells.data();
  submap.local_pose = Rigid2d{0., 0., 0.};
  // The L's cell centres in the submap frame (x from the cell row, y from
  // the column), then the same points shifted 3 m.
  PointCloud first, shifted;
  for (int x = 10; x <= 14; ++x) first.push_back(2.f - 20.5f, 3.f - (x + 0.5f), 0.f);
  for (int y = 21; y <= 23; ++y) first.push_back(2.f - (y + 0.5f), 3.f - 10.5f, 0.f);
  for (size_t i = 0; i < first.size(); ++i)
    shifted.push_back(first.xyz[3 * i] + 3.f, first.xyz[3 * i + 1], 0.f);
  const SubmapId submap_id{0, 0};
  ConstraintBuilder2D kept(TestOptions());
  ConstraintBuilder2D::Result r1, r2, fresh;
  kept.MaybeAddGlobalConstraint(submap_id, &submap, NodeId{0, 7}, &first);
  kept.NotifyEndOfNode();
  kept.WhenDone([&](const ConstraintBuilder2D::Result& r) { r1 = r; });
  kept.MaybeAddGlobalConstraint(submap_id, &submap, NodeId{0, 7}, &shifted);  // changed cloud
  kept.MaybeAddGlobalConstraint(submap_id, &submap, NodeId{0, 8}, &first);    // new node
  kept.NotifyEndOfNode();
  kept.WhenDone([&](const ConstraintBuilder2D::Result& r) { r2 = r; });
  ConstraintBuilder2D once(TestOptions());
  once.MaybeAddGlobalConstraint(submap_id, &submap, NodeId{0, 7}, &shifted);
  once.MaybeAddGlobalConstraint(submap_id, &submap, NodeId{0, 8}, &first);
  once.NotifyEndOfNode();
  once.WhenDone([&](const ConstraintBuilder2D::Result& r) { fresh = r; });
  EXPECT(r1.size() == 1 && r2.size() == 2 && fresh.size() == 2);
  if (r1.size() != 1 || r2.size() != 2 || fresh.size() != 2) return;
  for (int k = 0; k < 2; ++k) {
    EXPECT(r2[k].score == fresh[k].score);
    EXPECT(r2[k].relative_pose.x == fresh[k].relative_pose.x &&
           r2[k].relative_pose.y == fresh[k].relative_pose.y &&
           r2[k].relative_pose.theta == fresh[k].relative_pose.theta);
  }
  // The shifted cloud matched elsewhere than the first (not a stale copy),
  // and node 8's copy of the first cloud matched where node 7's first did.
  EXPECT(r2[0].relative_pose.x != r1[0].relative_pose.x ||
         r2[0].relative_pose.y != r1[0].relative_pose.y ||
         r2[0].relative_pose.theta != r1[0].relative_pose.theta);
  EXPECT(r2[1].score == r1[0].score && r2[1].relative_pose.x == r1[0].relative_pose.x &&
         r2[1].relative_pose.y == r1[0].relative_pose.y);
}

// Submaps with an L of occupied cells at a per-submap offset, and the L's
// points (submap 0's cell centres) as a cloud.
struct LWorld {
  std::vector<std::vector<uint16_t>> cells;
  std::vector<Submap2DView> submaps;
  PointCloud cloud;
  explicit LWorld(int n) : cells(n), submaps(n) {
    for (int s = 0; s < n; ++s) {
      cells[s].assign(100 * 110, 0);
      const int ox = s % 7, oy = (s / 7) % 5;
      for (int x = 10; x <= 14 + s % 3; ++x) cells[s][(20 + oy) * 100 + x + ox] = 1;
      for (int y = 21; y <= 23 + s % 4; ++y) cells[s][(y + oy) * 100 + 10 + ox] = 1;
      Submap2DView& v = submaps[s];
      v.grid.resolution = 1.;
      v.grid.max_x = 2.;
      v.grid.max_y = 3.;
      v.grid.num_x_cells = 100;
      v.grid.num_y_cells = 110;
      v.grid.cells = cells[s].data();
      v.local_pose = Rigid2d{0.5 * s, -0.25 * s, 0.01 * s};
    }
    for (int x = 10; x <= 14; ++x) cloud.push_back(2.f - 20.5f, 3.f - (x + 0.5f), 0.f);
    for (int y = 21; y <= 23; ++y) cloud.push_back(2.f - (y + 0.5f), 3.f - 10.5f, 0.f);
  }
};

static ConstraintBuilder2D::Result Sweep(ConstraintBuilder2D* b, LWorld* w, int nodes) {
  ConstraintBuilder2D::Result all;
  for (int n = 0; n < nodes; ++n) {
    for (size_t s = 0; s < w->submaps.size(); ++s)
      b->MaybeAddGlobalConstraint(SubmapId{0, static_cast<int>(s)}, &w->submaps[s], NodeId{0, n},
                                  &w->cloud);
    b->NotifyEndOfNode();
  }
  b->WhenDone([&](const ConstraintBuilder2D::Result& r) { all = r; });
  return all;
}

// The matcher cache under a device budget of 5 matchers: LRU matchers are
// dropped and rebuilt, each flush is cut into sub-batches that fit, and the
// constraints are the unbounded builder's, in the same order.
static void BudgetedMatcherCache() {
  LWorld w(40);
  ConstraintBuilderOptions unbounded = TestOptions();
  unbounded.matcher_cache_bytes = 0;
  ConstraintBuilder2D ref(unbounded);
  const ConstraintBuilder2D::Result expected = Sweep(&ref, &w, 3);
  EXPECT(ref.num_submap_scan_matchers() == 40 && ref.matcher_evictions() == 0);
  const int64_t one = ref.matcher_cache_bytes() / 40;
  ConstraintBuilderOptions small = TestOptions();
  small.matcher_cache_bytes = 5 * one;
  ConstraintBuilder2D b(small);
  const ConstraintBuilder2D::Result got = Sweep(&b, &w, 3);
  EXPECT(b.matcher_evictions() > 0 && b.matcher_builds() > 40);
  EXPECT(b.matcher_cache_bytes() <= 5 * one && b.num_submap_scan_matchers() <= 5);
  EXPECT(got.size() == expected.size() && !got.empty());
  for (size_t k = 0; k < got.size() && k < expected.size(); ++k) {
    EXPECT(got[k].submap_id.submap_index == expected[k].submap_id.submap_index &&
           got[k].node_id.node_index == expected[k].node_id.node_index);
    EXPECT(got[k].score == expected[k].score);
    EXPECT(got[k].relative_pose.x == expected[k].relative_pose.x &&
           got[k].relative_pose.y == expected[k].relative_pose.y &&
           got[k].relative_pose.theta == expected[k].relative_pose.theta);
  }
}

// One PointCloud object refilled for the same node with other points of the
// same count: the resident copy is stale and the new points are searched.
static void RefilledCloudIsUploadedAgain() {
  LWorld w(1);
  PointCloud cloud = w.cloud;
  ConstraintBuilder2D b(TestOptions());
  ConstraintBuilder2D::Result r1, r2;
  b.MaybeAddGlobalConstraint(SubmapId{0, 0}, &w.submaps[0], NodeId{0, 3}, &cloud);
  b.NotifyEndOfNode();
  b.WhenDone([&](const ConstraintBuilder2D::Result& r) { r1 = r; });
  for (size_t i = 0; i < cloud.size(); ++i) cloud.xyz[3 * i] += 3.f;  // same object, same size
  b.MaybeAddGlobalConstraint(SubmapId{0, 0}, &w.submaps[0], NodeId{0, 3}, &cloud);
  b.NotifyEndOfNode();
  b.WhenDone([&](const ConstraintBuilder2D::Result& r) { r2 = r; });
  EXPECT(r1.size() == 1 && r2.size() == 1);
  if (r1.size() == 1 && r2.size() == 1)
    EXPECT(r1[0].relative_pose.x != r2[0].relative_pose.x ||
           r1[0].relative_pose.y != r2[0].relative_pose.y);
}

// DeleteScanMatcher drops the submap's pending pairs: no constraint, no
// rebuild from a view the caller is trimming.
static void DeleteDropsPendingPairs() {
  LWorld w(2);
  ConstraintBuilderOptions o = TestOptions();
  o.flush_pairs = 1000;  // nothing is searched before WhenDone
  ConstraintBuilder2D b(o);
  for (int s = 0; s < 2; ++s)
    b.MaybeAddGlobalConstraint(SubmapId{0, s}, &w.submaps[s], NodeId{0, 0}, &w.cloud);
  b.NotifyEndOfNode();
  b.DeleteScanMatcher(SubmapId{0, 1});
  ConstraintBuilder2D::Result r;
  b.WhenDone([&](const ConstraintBuilder2D::Result& res) { r = res; });
  EXPECT(r.size() == 1 && r[0].submap_id.submap_index == 0);
  EXPECT(b.global_constraints_searched == 1);
}

int main() {
  CallsBack();
  FindsConstraints();
  SkipsUnsearchablePairs();
  ReusesResidentCloudsAcrossFlushes();
  BudgetedMatcherCache();
  RefilledCloudIsUploadedAgain();
  DeleteDropsPendingPairs();
  if (failures) return 1;
  std::printf("constraint_builder_2d_test: OK\n");
  return 0;
}
