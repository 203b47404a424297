// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
// C API of the 3D restatement, for tests/oracle_lib.py.
#include <atomic>
#include <chrono>
#include <cstring>
#include <thread>

#include "oracle3d.h"

using namespace oracle;

namespace {
PointCloud Cloud(const float* xyz, int n) {
  PointCloud c(n);
  for (int i = 0; i < n; ++i) c[i] = Vec3f{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
  return c;
}
Rigid3d Pose(const double* p) {  // t[3], q[4] (w, x, y, z)
  return Rigid3d{Vec3d{p[0], p[1], p[2]}, Quatd{p[3], p[4], p[5], p[6]}};
}
void PutPose(const Rigid3d& r, double* out) {
  out[0] = r.t.x;
  out[1] = r.t.y;
  out[2] = r.t.z;
  out[3] = r.q.w;
  out[4] = r.q.x;
  out[5] = r.q.y;
  out[6] = r.q.z;
}
struct Fast3dHandle {
  std::unique_ptr<FastCorrelativeScanMatcher3D> m;
  std::vector<float> histogram;
};
}  // namespace

extern "C" {

void* oracle_hgrid_create(float resolution) { return new HybridGrid(resolution); }
void oracle_hgrid_destroy(void* g) { delete static_cast<HybridGrid*>(g); }
void oracle_hgrid_set_probability(void* g, int x, int y, int z, float p) {
  static_cast<HybridGrid*>(g)->SetProbability(Idx3{x, y, z}, p);
}
void oracle_hgrid_set_values(void* g, const int32_t* ijk, const uint16_t* values, int64_t n) {
  auto* h = static_cast<HybridGrid*>(g);
  for (int64_t i = 0; i < n; ++i)
    *h->mutable_value(Idx3{ijk[3 * i], ijk[3 * i + 1], ijk[3 * i + 2]}) = values[i];
}
void oracle_hgrid_insert(void* g, float hit, float miss, int num_free_space_voxels,
                         const float* origin, const float* xyz, int n) {
  RangeDataInserter3D ins(hit, miss, num_free_space_voxels);
  ins.Insert(Vec3f{origin[0], origin[1], origin[2]}, Cloud(xyz, n), static_cast<HybridGrid*>(g));
}
// Non-zero cells in iterator order. Returns the count; writes when capacity allows.
int64_t oracle_hgrid_cells(void* g, int32_t* ijk, uint16_t* values, int64_t capacity) {
  int64_t n = 0;
  static_cast<HybridGrid*>(g)->ForEach([&](const Idx3& i, uint16_t v) {
    if (n < capacity) {
      ijk[3 * n] = i.x;
      ijk[3 * n + 1] = i.y;
      ijk[3 * n + 2] = i.z;
      values[n] = v;
    }
    ++n;
  });
  return n;
}
int oracle_hgrid_grid_size(void* g) { return static_cast<HybridGrid*>(g)->grid_size(); }
// InterpolatedProbabilityGrid::GetInterpolatedValue at n points (x, y, z).
void oracle_hgrid_interpolate(void* g, const double* xyz, int64_t n, double* out) {
  const auto* h = static_cast<HybridGrid*>(g);
  for (int64_t i = 0; i < n; ++i)
    out[i] = Interpolate(*h, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], nullptr);
}
// HybridGridBase::GetCellIndex (float division, lround) of n points.
void oracle_hgrid_cell_index(void* g, const float* xyz, int64_t n, int32_t* out) {
  const auto* h = static_cast<HybridGrid*>(g);
  for (int64_t i = 0; i < n; ++i) {
    const Idx3 c = h->GetCellIndex(Vec3f{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]});
    out[3 * i] = c.x;
    out[3 * i + 1] = c.y;
    out[3 * i + 2] = c.z;
  }
}
float oracle_hgrid_probability(void* g, int x, int y, int z) {
  return static_cast<HybridGrid*>(g)->GetProbability(Idx3{x, y, z});
}

void oracle_histogram(const float* xyz, int n, int size, float* out) {
  const std::vector<float> h = ComputeHistogram(Cloud(xyz, n), size);
  std::memcpy(out, h.data(), sizeof(float) * size);
}
void oracle_rotational_match(const float* submap_hist, const float* hist, int size,
                             float initial_angle, const float* angles, int n, float* out) {
  const std::vector<float> s(submap_hist, submap_hist + size), h(hist, hist + size);
  const std::vector<float> a(angles, angles + n);
  const std::vector<float> r = RotationalMatch(s, h, initial_angle, a);
  std::memcpy(out, r.data(), sizeof(float) * n);
}

// options: bb_depth, full_res_depth, min_rot, min_low_res, lin_xy, lin_z, ang.
void* oracle_fast3d_create(void* high, void* low, const float* histogram, int hsize,
                           const double* options) {
  auto* h = new Fast3dHandle;
  h->histogram.assign(histogram, histogram + hsize);
  FastCsm3dOptions o;
  o.branch_and_bound_depth = static_cast<int>(options[0]);
  o.full_resolution_depth = static_cast<int>(options[1]);
  o.min_rotational_score = options[2];
  o.min_low_resolution_score = options[3];
  o.linear_xy_search_window = options[4];
  o.linear_z_search_window = options[5];
  o.angular_search_window = options[6];
  h->m.reset(new FastCorrelativeScanMatcher3D(*static_cast<HybridGrid*>(high),
                                              static_cast<HybridGrid*>(low), &h->histogram, o));
  return h;
}
void oracle_fast3d_destroy(void* h) { delete static_cast<Fast3dHandle*>(h); }

// Level d as a list of non-zero cells (iterator order). Returns the count.
int64_t oracle_fast3d_level(void* h, int d, int32_t* ijk, uint8_t* values, int64_t capacity) {
  int64_t n = 0;
  static_cast<Fast3dHandle*>(h)->m->level(d).ForEach([&](const Idx3& i, uint8_t v) {
    if (n < capacity) {
      ijk[3 * n] = i.x;
      ijk[3 * n + 1] = i.y;
      ijk[3 * n + 2] = i.z;
      values[n] = v;
    }
    ++n;
  });
  return n;
}

// result: matched, score, rotational_score, low_resolution_score (floats as
// doubles), pose t[3] q[4], lookups, low_resolution_checks, num_discrete_scans.
static void PutResult(const Fast3dResult& r, double* out) {
  out[0] = r.matched ? 1. : 0.;
  out[1] = r.score;
  out[2] = r.rotational_score;
  out[3] = r.low_resolution_score;
  PutPose(r.pose, out + 4);
  out[11] = static_cast<double>(r.lookups);
  out[12] = static_cast<double>(r.low_resolution_checks);
  out[13] = r.num_discrete_scans;
}

static const double kIdentityQ[4] = {1., 0., 0., 0.};

static NodeData3D Node(const float* high, int nh, const float* low, int nl, const float* hist,
                       int hsize, const double* gravity_q) {
  NodeData3D n;
  n.high_resolution_point_cloud = Cloud(high, nh);
  n.low_resolution_point_cloud = Cloud(low, nl);
  n.rotational_scan_matcher_histogram.assign(hist, hist + hsize);
  n.gravity_alignment = Quatd{gravity_q[0], gravity_q[1], gravity_q[2], gravity_q[3]};
  return n;
}

void oracle_fast3d_match(void* h, const double* node_pose, const double* submap_pose,
                         const float* high, int nh, const float* low, int nl, const float* hist,
                         int hsize, const double* gravity_q, float min_score, double* out) {
  const Fast3dResult r = static_cast<Fast3dHandle*>(h)->m->Match(
      Pose(node_pose), Pose(submap_pose), Node(high, nh, low, nl, hist, hsize, gravity_q),
      min_score);
  PutResult(r, out);
}

void oracle_fast3d_match_full_submap(void* h, const double* node_q, const double* submap_q,
                                     const float* high, int nh, const float* low, int nl,
                                     const float* hist, int hsize, const double* gravity_q,
                                     float min_score, double* out) {
  const Fast3dResult r = static_cast<Fast3dHandle*>(h)->m->MatchFullSubmap(
      Quatd{node_q[0], node_q[1], node_q[2], node_q[3]},
      Quatd{submap_q[0], submap_q[1], submap_q[2], submap_q[3]},
      Node(high, nh, low, nl, hist, hsize, gravity_q), min_score);
  PutResult(r, out);
}

// Tie checks: evaluates the leaf behind `pose` (t[3], q[4]); returns 1 if found.
int oracle_fast3d_evaluate_leaf(void* h, int full_submap, const double* node_pose,
                                const double* submap_pose, const float* high, int nh,
                                const float* low, int nl, const float* hist, int hsize,
                                const double* gravity_q, const double* pose, double* out) {
  Fast3dResult r;
  const bool ok = static_cast<Fast3dHandle*>(h)->m->EvaluateLeaf(
      full_submap != 0, Pose(node_pose), Pose(submap_pose),
      Node(high, nh, low, nl, hist, hsize, gravity_q), Pose(pose), &r);
  PutResult(r, out);
  return ok ? 1 : 0;
}

// options: lin, ang, wt, wr. out: score, pose t[3] q[4], best_index, candidates.
void oracle_rt3d_match(void* g, const double* options, const double* initial, const float* xyz,
                       int n, double* out) {
  RtOptions3D o;
  o.linear_search_window = options[0];
  o.angular_search_window = options[1];
  o.translation_delta_cost_weight = options[2];
  o.rotation_delta_cost_weight = options[3];
  const Rt3dResult r = RealTimeMatch3D(o, Pose(initial), Cloud(xyz, n), *static_cast<HybridGrid*>(g));
  out[0] = r.score;
  PutPose(r.pose, out + 1);
  out[8] = static_cast<double>(r.best_index);
  out[9] = static_cast<double>(r.candidates);
}

float oracle_rt3d_score(void* g, const double* options, const double* initial, const float* xyz,
                        int n, int64_t index, double* pose_out) {
  RtOptions3D o;
  o.linear_search_window = options[0];
  o.angular_search_window = options[1];
  o.translation_delta_cost_weight = options[2];
  o.rotation_delta_cost_weight = options[3];
  Rigid3f c;
  const float s = RealTimeScore3D(o, Pose(initial), Cloud(xyz, n), *static_cast<HybridGrid*>(g),
                                  index, &c);
  if (pose_out)
    PutPose(Rigid3d{Vec3d{c.t.x, c.t.y, c.t.z}, Quatd{c.q.w, c.q.x, c.q.y, c.q.z}}, pose_out);
  return s;
}

void oracle_rt3d_window(const double* options, float resolution, const float* xyz, int n,
                        int* linear_window, float* angular_step, int* angular_window) {
  RtOptions3D o;
  o.linear_search_window = options[0];
  o.angular_search_window = options[1];
  RealTime3DWindow(o, resolution, Cloud(xyz, n), linear_window, angular_step, angular_window);
}


// CPU baseline (bench.py): MatchFullSubmap over (submap, node) pairs on
// `threads` host threads, one pair per task like ConstraintBuilder3D's pool.
// nodes: packed clouds with offsets; rotations (w,x,y,z) per node. Returns
// wall seconds; matched[i] = 1 when a Result was returned.
double oracle_fast3d_match_pairs(void** submaps, const float* high, const int64_t* high_off,
                                 const float* low, const int64_t* low_off, const float* hists,
                                 int hsize, const double* node_q, const int32_t* pair_submap,
                                 const int32_t* pair_node, int64_t num_pairs, int threads,
                                 float min_score, int32_t* matched, double* results,
                                 double* task_seconds) {
  std::atomic<int64_t> next{0};
  const auto t0 = std::chrono::steady_clock::now();
  auto work = [&]() {
    for (int64_t i = next++; i < num_pairs; i = next++) {
      const int n = pair_node[i];
      const NodeData3D node =
          Node(high + 3 * high_off[n], static_cast<int>(high_off[n + 1] - high_off[n]),
               low + 3 * low_off[n], static_cast<int>(low_off[n + 1] - low_off[n]),
               hists + static_cast<int64_t>(hsize) * n, hsize, kIdentityQ);
      const double* q = node_q + 4 * n;
      const auto ts = std::chrono::steady_clock::now();
      const Fast3dResult r = static_cast<Fast3dHandle*>(submaps[pair_submap[i]])->m->MatchFullSubmap(
          Quatd{q[0], q[1], q[2], q[3]}, Quatd{1., 0., 0., 0.}, node, min_score);
      matched[i] = r.matched ? 1 : 0;
      if (results) PutResult(r, results + 14 * i);  // score, poses: the bench's parity sample
      if (task_seconds)
        task_seconds[i] = std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// CPU baseline for RTCSM3D: seconds to score `count` candidates spread over
// the search (indices i * stride), single-threaded like Match.
double oracle_rt3d_time(void* g, const double* options, const double* initial, const float* xyz,
                        int n, int64_t count, int64_t stride) {
  RtOptions3D o;
  o.linear_search_window = options[0];
  o.angular_search_window = options[1];
  o.translation_delta_cost_weight = options[2];
  o.rotation_delta_cost_weight = options[3];
  float sink = 0.f;
  return RealTimeTime3D(o, Pose(initial), Cloud(xyz, n), *static_cast<HybridGrid*>(g), count,
                        stride, &sink);
}

}  // extern "C"
