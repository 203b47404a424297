// C++ drop-in shim over the csm_amd 3D C-ABI, source-compatible with the call
// sites of Cartographer's 3D scan matchers:
//   constraint_builder_3d.cc:190-193  FastCorrelativeScanMatcher3D(high, &low,
//                                       &histogram, options)
//   constraint_builder_3d.cc:221-223  MatchFullSubmap(node_rot, submap_rot, data, min)
//   constraint_builder_3d.cc:239-241  Match(node_pose, submap_pose, data, min)
//   local_trajectory_builder_3d.cc:481  RealTimeCorrelativeScanMatcher3D::Match
//
// The reference types (HybridGrid, TrajectoryNode::Data, transform::Rigid3d,
// Eigen::Quaterniond, the option protos) are represented by the POD views
// below (INTEGRATION.md shows the adapter). As in scan_matching.h, negative
// return codes abort like the reference's CHECKs.
#ifndef CARTOGRAPHER_AMD_SCAN_MATCHING_3D_H_
#define CARTOGRAPHER_AMD_SCAN_MATCHING_3D_H_

#include <cmath>
#include <cstdint>
#include <memory>
#include <vector>

#include "scan_matching.h"

namespace cartographer_amd {

// Eigen::Quaterniond (w, x, y, z).
struct Quaterniond {
  double w = 1., x = 0., y = 0., z = 0.;
  static Quaterniond Identity() { return Quaterniond{}; }
};

// transform::Rigid3d.
struct Rigid3d {
  double t[3] = {0., 0., 0.};
  Quaterniond rotation;
  static Rigid3d Identity() { return Rigid3d{}; }
  static Rigid3d Rotation(const Quaterniond& q) {
    Rigid3d r;
    r.rotation = q;
    return r;
  }
  csm_pose3d ToC() const {
    return csm_pose3d{{t[0], t[1], t[2]}, {rotation.w, rotation.x, rotation.y, rotation.z}};
  }
  static Rigid3d FromC(const csm_pose3d& p) {
    Rigid3d r;
    for (int i = 0; i < 3; ++i) r.t[i] = p.t[i];
    r.rotation = Quaterniond{p.q[0], p.q[1], p.q[2], p.q[3]};
    return r;
  }
};

// A HybridGrid as its iterator yields it (hybrid_grid.h:530-541): known cells'
// indices and uint16 probability values, plus DynamicGrid::grid_size()
// (0 = derive from the indices).
struct HybridGridView {
  float resolution = 0.1f;
  std::vector<int32_t> xyz;     // 3 per cell
  std::vector<uint16_t> values;
  int32_t grid_size = 0;
};

// Device copy of a HybridGrid (owned; csm_hybrid_grid).
class HybridGrid3D {
 public:
  explicit HybridGrid3D(const HybridGridView& v, csm_context* context = nullptr) {
    csm_hybrid_grid* h = nullptr;
    CheckOk(csm_hybrid_grid_create(context ? context : ThreadContext(), v.resolution,
                                   v.xyz.data(), v.values.data(),
                                   static_cast<int64_t>(v.values.size()), v.grid_size, &h),
            "HybridGrid");
    handle_ = h;
  }
  ~HybridGrid3D() { csm_hybrid_grid_destroy(handle_); }
  HybridGrid3D(const HybridGrid3D&) = delete;
  HybridGrid3D& operator=(const HybridGrid3D&) = delete;
  const csm_hybrid_grid* handle() const { return handle_; }
  int64_t device_bytes() const { return csm_hybrid_grid_device_bytes(handle_); }

 private:
  csm_hybrid_grid* handle_ = nullptr;
};

// proto::FastCorrelativeScanMatcherOptions3D, pose_graph.lua:40-48 defaults.
struct FastCorrelativeScanMatcherOptions3D {
  int branch_and_bound_depth = 8;
  int full_resolution_depth = 3;
  double min_rotational_score = 0.77;
  double min_low_resolution_score = 0.55;
  double linear_xy_search_window = 5.;
  double linear_z_search_window = 1.;
  double angular_search_window = 15. * M_PI / 180.;
};

// The TrajectoryNode::Data fields the 3D matcher reads (trajectory_node.h:45-63).
struct TrajectoryNodeData3D {
  PointCloud high_resolution_point_cloud;
  PointCloud low_resolution_point_cloud;
  std::vector<float> rotational_scan_matcher_histogram;
  Quaterniond gravity_alignment;
  csm_node3d ToC() const {
    csm_node3d n{};
    n.high_resolution_xyz = high_resolution_point_cloud.xyz.data();
    n.num_high_resolution = static_cast<int32_t>(high_resolution_point_cloud.size());
    n.low_resolution_xyz = low_resolution_point_cloud.xyz.data();
    n.num_low_resolution = static_cast<int32_t>(low_resolution_point_cloud.size());
    n.histogram = rotational_scan_matcher_histogram.data();
    n.histogram_size = static_cast<int32_t>(rotational_scan_matcher_histogram.size());
    n.gravity_alignment[0] = gravity_alignment.w;
    n.gravity_alignment[1] = gravity_alignment.x;
    n.gravity_alignment[2] = gravity_alignment.y;
    n.gravity_alignment[3] = gravity_alignment.z;
    return n;
  }
};

// fast_correlative_scan_matcher_3d.h:66-158
class FastCorrelativeScanMatcher3D {
 public:
  // FastCorrelativeScanMatcher3D::Result (.h:68-73).
  struct Result {
    float score = 0.f;
    Rigid3d pose_estimate;
    float rotational_score = 0.f;
    float low_resolution_score = 0.f;
  };

  // As the reference keeps a raw pointer to the low-resolution grid (.h:150),
  // `low_resolution_hybrid_grid` must outlive the matcher.
  FastCorrelativeScanMatcher3D(const HybridGrid3D& hybrid_grid,
                               const HybridGrid3D* low_resolution_hybrid_grid,
                               const std::vector<float>* rotational_scan_matcher_histogram,
                               const FastCorrelativeScanMatcherOptions3D& options,
                               csm_context* context = nullptr) {
    const csm_fast3d_options o{options.branch_and_bound_depth, options.full_resolution_depth,
                               options.min_rotational_score, options.min_low_resolution_score,
                               options.linear_xy_search_window, options.linear_z_search_window,
                               options.angular_search_window};
    csm_fast3d* h = nullptr;
    CheckOk(csm_fast3d_create(context ? context : ThreadContext(), hybrid_grid.handle(),
                              low_resolution_hybrid_grid->handle(),
                              rotational_scan_matcher_histogram->data(),
                              static_cast<int32_t>(rotational_scan_matcher_histogram->size()), &o,
                              &h),
            "FastCorrelativeScanMatcher3D");
    handle_ = h;
  }
  ~FastCorrelativeScanMatcher3D() { csm_fast3d_destroy(handle_); }
  FastCorrelativeScanMatcher3D(const FastCorrelativeScanMatcher3D&) = delete;
  FastCorrelativeScanMatcher3D& operator=(const FastCorrelativeScanMatcher3D&) = delete;

  // .h:89-92; nullptr when no candidate scores above min_score.
  std::unique_ptr<Result> Match(const Rigid3d& global_node_pose,
                                const Rigid3d& global_submap_pose,
                                const TrajectoryNodeData3D& constant_data,
                                float min_score) const {
    const csm_pose3d np = global_node_pose.ToC(), sp = global_submap_pose.ToC();
    const csm_node3d node = constant_data.ToC();
    csm_result3d r{};
    const int rc = csm_fast3d_match(handle_, &np, &sp, &node, min_score, &r);
    CheckOk(rc, "FastCorrelativeScanMatcher3D::Match");
    return Convert(rc, r);
  }

  // .h:98-101
  std::unique_ptr<Result> MatchFullSubmap(const Quaterniond& global_node_rotation,
                                          const Quaterniond& global_submap_rotation,
                                          const TrajectoryNodeData3D& constant_data,
                                          float min_score) const {
    const double nq[4] = {global_node_rotation.w, global_node_rotation.x,
                          global_node_rotation.y, global_node_rotation.z};
    const double sq[4] = {global_submap_rotation.w, global_submap_rotation.x,
                          global_submap_rotation.y, global_submap_rotation.z};
    const csm_node3d node = constant_data.ToC();
    csm_result3d r{};
    const int rc = csm_fast3d_match_full_submap(handle_, nq, sq, &node, min_score, &r);
    CheckOk(rc, "FastCorrelativeScanMatcher3D::MatchFullSubmap");
    return Convert(rc, r);
  }

  csm_fast3d* handle() const { return handle_; }
  int64_t device_bytes() const { return csm_fast3d_device_bytes(handle_); }

  static std::unique_ptr<Result> Convert(int rc, const csm_result3d& r) {
    if (rc != CSM_OK || r.status != CSM_OK) return nullptr;
    std::unique_ptr<Result> out(new Result);
    out->score = r.score;
    out->pose_estimate = Rigid3d::FromC(r.pose);
    out->rotational_score = r.rotational_score;
    out->low_resolution_score = r.low_resolution_score;
    return out;
  }

 private:
  csm_fast3d* handle_ = nullptr;
};

// real_time_correlative_scan_matcher_3d.h:33-62
class RealTimeCorrelativeScanMatcher3D {
 public:
  explicit RealTimeCorrelativeScanMatcher3D(const RealTimeCorrelativeScanMatcherOptions& o)
      : options_{o.linear_search_window, o.angular_search_window,
                 o.translation_delta_cost_weight, o.rotation_delta_cost_weight} {}

  float Match(const Rigid3d& initial_pose_estimate, const PointCloud& point_cloud,
              const HybridGrid3D& hybrid_grid, Rigid3d* pose_estimate) const {
    const csm_pose3d init = initial_pose_estimate.ToC();
    csm_pose3d out{};
    float score = 0.f;
    CheckOk(csm_rt3d_match(ThreadContext(), &options_, hybrid_grid.handle(), &init,
                           point_cloud.xyz.data(), static_cast<int32_t>(point_cloud.size()),
                           &score, &out),
            "RealTimeCorrelativeScanMatcher3D::Match");
    *pose_estimate = Rigid3d::FromC(out);
    return score;
  }

 private:
  csm_rt_options options_;
};

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_SCAN_MATCHING_3D_H_
