// Types shared by the ConstraintBuilder2D / 3D drop-ins: ids, the
// ConstraintBuilderOptions proto (one proto carries both scan-matcher
// configurations, constraint_builder_options.proto:24-59) and
// common::FixedRatioSampler.
#ifndef CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_COMMON_H_
#define CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_COMMON_H_

#include <cstdint>

#include "scan_matching.h"
#include "scan_matching_3d.h"

namespace cartographer_amd {

struct SubmapId {
  int trajectory_id = 0, submap_index = 0;
  bool operator<(const SubmapId& o) const {
    return trajectory_id != o.trajectory_id ? trajectory_id < o.trajectory_id
                                            : submap_index < o.submap_index;
  }
};
struct NodeId {
  int trajectory_id = 0, node_index = 0;
  bool operator<(const NodeId& o) const {
    return trajectory_id != o.trajectory_id ? trajectory_id < o.trajectory_id
                                            : node_index < o.node_index;
  }
};

// proto::ConstraintBuilderOptions (constraint_builder_options.proto:24-59),
// defaults from configuration_files/pose_graph.lua:17-29.
struct ConstraintBuilderOptions {
  double sampling_ratio = 0.3;
  double max_constraint_distance = 15.;
  float min_score = 0.55f;
  float global_localization_min_score = 0.6f;
  double loop_closure_translation_weight = 1.1e4;
  double loop_closure_rotation_weight = 1e5;
  FastCorrelativeScanMatcherOptions2D fast_correlative_scan_matcher_options;
  FastCorrelativeScanMatcherOptions3D fast_correlative_scan_matcher_options_3d;
  int flush_pairs = 0;  // 0: search each node's pairs when the node ends
  // ceres_scan_matcher (pose_graph.lua:30-39): accepted 2D matches are refined
  // with CeresScanMatcher2D (constraint_builder_2d.cc:245-249).
  csm_ceres2d_options ceres_scan_matcher_options{20., 10., 1., 10, /*nonmonotonic=*/1};
  // ceres_scan_matcher_3d (pose_graph.lua:49-60), ConstraintBuilder3D (:264-275).
  csm_ceres3d_options ceres_scan_matcher_options_3d{5., 30., 10., 1., 10, /*nonmonotonic=*/0};
  bool refine_with_ceres = true;
  // Node clouds stay on the device across flushes (a node's cloud is uploaded
  // once); past this many resident points the 2D builder starts a new set.
  int64_t scan_cache_points = int64_t{1} << 25;
};

// common/fixed_ratio_sampler.cc:32-39
class FixedRatioSampler {
 public:
  explicit FixedRatioSampler(double ratio) : ratio_(ratio) {}
  bool Pulse() {
    ++num_pulses_;
    if (static_cast<double>(num_samples_) / num_pulses_ < ratio_) {
      ++num_samples_;
      return true;
    }
    return false;
  }

 private:
  double ratio_;
  int64_t num_pulses_ = 0, num_samples_ = 0;
};

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_COMMON_H_
