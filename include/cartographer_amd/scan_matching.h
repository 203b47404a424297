// C++ drop-in shim over the csm_amd C-ABI, source-compatible with the call
// sites of Cartographer's scan matchers:
//   constraint_builder_2d.cc:179-181  FastCorrelativeScanMatcher2D(grid, options)
//   constraint_builder_2d.cc:213-215  MatchFullSubmap(cloud, min_score, &score, &pose)
//   constraint_builder_2d.cc:226-228  Match(initial, cloud, min_score, &score, &pose)
//   local_trajectory_builder_2d.cc:78-80  RealTimeCorrelativeScanMatcher2D::Match
//
// The reference types (Grid2D, sensor::PointCloud, transform::Rigid2d, the
// option protos) are represented by the small POD views below; a maintainer
// adapts them in one place (INTEGRATION.md shows the adapter). Negative return
// codes abort, like the reference's glog CHECKs
// (fast_correlative_scan_matcher_2d.cc:232-233, real_time_..._2d.cc:73).
#ifndef CARTOGRAPHER_AMD_SCAN_MATCHING_H_
#define CARTOGRAPHER_AMD_SCAN_MATCHING_H_

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <vector>

#include "../csm_amd.h"

namespace cartographer_amd {

inline void CheckOk(int code, const char* what) {
  if (code < 0) {
    std::fprintf(stderr, "F %s: %s (%d)\n", what, csm_strerror(code), code);
    std::abort();
  }
}

// transform::Rigid2d (translation + angle).
struct Rigid2d {
  double x = 0., y = 0., theta = 0.;
  static Rigid2d Identity() { return Rigid2d{}; }
};

// sensor::PointCloud: RangefinderPoint positions, xyz floats.
struct PointCloud {
  std::vector<float> xyz;  // 3 floats per point
  size_t size() const { return xyz.size() / 3; }
  void push_back(float x, float y, float z) {
    xyz.push_back(x);
    xyz.push_back(y);
    xyz.push_back(z);
  }
};

// Grid2D view: MapLimits + uint16 correspondence-cost cells (x fastest).
struct Grid2DView {
  // Grid2D::GetGridType() (grid_2d.h:32): which cells the view carries.
  enum class GridType { PROBABILITY_GRID, TSDF };
  GridType grid_type = GridType::PROBABILITY_GRID;
  double resolution = 0.05;
  double max_x = 0., max_y = 0.;
  int num_x_cells = 0, num_y_cells = 0;
  const uint16_t* cells = nullptr;       // correspondence_cost_cells() (TSD values for a TSDF)
  // kMinCorrespondenceCost = 1.f - kMaxProbability and kMaxCorrespondenceCost =
  // 1.f - kMinProbability, in float (probability_values.h:32-36): 0.100000024f
  // and 0.9f (-truncation / truncation for a TSDF).
  float min_correspondence_cost = 1.f - (1.f - 0.1f);
  float max_correspondence_cost = 1.f - 0.1f;
  // TSDF2D only (tsdf_2d.h:55-60): weight_cells_ and TSDValueConverter's max weight.
  const uint16_t* weight_cells = nullptr;
  float max_weight = 0.f;
};

// proto::FastCorrelativeScanMatcherOptions2D (pose_graph.lua:25-29 defaults).
struct FastCorrelativeScanMatcherOptions2D {
  double linear_search_window = 7.;
  double angular_search_window = 30. * M_PI / 180.;
  int branch_and_bound_depth = 7;
};

// proto::RealTimeCorrelativeScanMatcherOptions (trajectory_builder_2d.lua:38-43).
struct RealTimeCorrelativeScanMatcherOptions {
  double linear_search_window = 0.1;
  double angular_search_window = 20. * M_PI / 180.;
  double translation_delta_cost_weight = 1e-1;
  double rotation_delta_cost_weight = 1e-1;
};

// One device context per thread (the C-ABI serialises calls per context).
inline csm_context* ThreadContext(int device = 0) {
  thread_local std::unique_ptr<csm_context, void (*)(csm_context*)> ctx(nullptr,
                                                                        csm_context_destroy);
  if (!ctx) {
    csm_context* c = nullptr;
    CheckOk(csm_context_create(device, &c), "csm_context_create");
    ctx.reset(c);
  }
  return ctx.get();
}

// fast_correlative_scan_matcher_2d.h:112-164
class FastCorrelativeScanMatcher2D {
 public:
  FastCorrelativeScanMatcher2D(const Grid2DView& grid,
                               const FastCorrelativeScanMatcherOptions2D& options,
                               csm_context* context = nullptr) {
    const csm_map_limits limits{grid.resolution, grid.max_x, grid.max_y, grid.num_x_cells,
                                grid.num_y_cells};
    const csm_fast2d_options o{options.linear_search_window, options.angular_search_window,
                               options.branch_and_bound_depth, 0};
    csm_fast2d* h = nullptr;
    CheckOk(csm_fast2d_create(context ? context : ThreadContext(), &limits, grid.cells,
                              grid.min_correspondence_cost, grid.max_correspondence_cost, &o, &h),
            "FastCorrelativeScanMatcher2D");
    handle_ = h;
  }
  ~FastCorrelativeScanMatcher2D() { csm_fast2d_destroy(handle_); }
  FastCorrelativeScanMatcher2D(const FastCorrelativeScanMatcher2D&) = delete;
  FastCorrelativeScanMatcher2D& operator=(const FastCorrelativeScanMatcher2D&) = delete;

  bool Match(const Rigid2d& initial_pose_estimate, const PointCloud& point_cloud,
             float min_score, float* score, Rigid2d* pose_estimate) const {
    const csm_pose2d init{initial_pose_estimate.x, initial_pose_estimate.y,
                          initial_pose_estimate.theta};
    csm_pose2d out{};
    const int rc = csm_fast2d_match(handle_, &init, point_cloud.xyz.data(),
                                    static_cast<int32_t>(point_cloud.size()), min_score, score, &out);
    CheckOk(rc, "FastCorrelativeScanMatcher2D::Match");
    if (rc == CSM_OK) *pose_estimate = Rigid2d{out.x, out.y, out.theta};
    return rc == CSM_OK;
  }

  bool MatchFullSubmap(const PointCloud& point_cloud, float min_score, float* score,
                       Rigid2d* pose_estimate) const {
    csm_pose2d out{};
    const int rc = csm_fast2d_match_full_submap(handle_, point_cloud.xyz.data(),
                                                static_cast<int32_t>(point_cloud.size()),
                                                min_score, score, &out);
    CheckOk(rc, "FastCorrelativeScanMatcher2D::MatchFullSubmap");
    if (rc == CSM_OK) *pose_estimate = Rigid2d{out.x, out.y, out.theta};
    return rc == CSM_OK;
  }

  csm_fast2d* handle() const { return handle_; }
  int64_t device_bytes() const { return csm_fast2d_device_bytes(handle_); }

 private:
  csm_fast2d* handle_ = nullptr;
};

// real_time_correlative_scan_matcher_2d.h:53-85
class RealTimeCorrelativeScanMatcher2D {
 public:
  explicit RealTimeCorrelativeScanMatcher2D(const RealTimeCorrelativeScanMatcherOptions& o)
      : options_{o.linear_search_window, o.angular_search_window,
                 o.translation_delta_cost_weight, o.rotation_delta_cost_weight} {}

  double Match(const Rigid2d& initial_pose_estimate, const PointCloud& point_cloud,
               const Grid2DView& grid, Rigid2d* pose_estimate) const {
    const csm_map_limits limits{grid.resolution, grid.max_x, grid.max_y, grid.num_x_cells,
                                grid.num_y_cells};
    const csm_pose2d init{initial_pose_estimate.x, initial_pose_estimate.y,
                          initial_pose_estimate.theta};
    csm_pose2d out{};
    double score = 0.;
    // ScoreCandidates switches on grid.GetGridType() (.cc:155-168).
    if (grid.grid_type == Grid2DView::GridType::TSDF)
      CheckOk(csm_rt2d_match_tsdf(ThreadContext(), &options_, &limits, grid.cells,
                                  grid.weight_cells, grid.max_correspondence_cost, grid.max_weight,
                                  &init, point_cloud.xyz.data(),
                                  static_cast<int32_t>(point_cloud.size()), &score, &out),
              "RealTimeCorrelativeScanMatcher2D::Match");
    else
      CheckOk(csm_rt2d_match(ThreadContext(), &options_, &limits, grid.cells,
                             grid.min_correspondence_cost, grid.max_correspondence_cost, &init,
                             point_cloud.xyz.data(), static_cast<int32_t>(point_cloud.size()),
                             &score, &out),
              "RealTimeCorrelativeScanMatcher2D::Match");
    *pose_estimate = Rigid2d{out.x, out.y, out.theta};
    return score;
  }

 private:
  csm_rt_options options_;
};

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_SCAN_MATCHING_H_
