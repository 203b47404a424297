// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h). 3D restatement.
//
// Follows, line by line:
//   mapping/3d/hybrid_grid.h                       (HybridGrid, Dynamic/Nested/FlatGrid)
//   mapping/3d/range_data_inserter_3d.cc           (test-fixture grids)
//   mapping/internal/3d/scan_matching/precomputation_grid_3d.{h,cc}
//   mapping/internal/3d/scan_matching/rotational_scan_matcher.cc
//   mapping/internal/3d/scan_matching/low_resolution_matcher.cc
//   mapping/internal/3d/scan_matching/fast_correlative_scan_matcher_3d.cc
//   mapping/internal/3d/scan_matching/real_time_correlative_scan_matcher_3d.cc
//
// Eigen float arithmetic: x86-64 builds vectorize with SSE2, so Quaternionf
// products use Eigen 3.3's Geometry_SSE.h quat_product and dynamic-size
// reductions (VectorXf dot/norm) use the packet order of Redux.h
// (two 4-wide accumulators, then (a0+a2)+(a1+a3), then scalar tail).
#ifndef CSM_ORACLE3D_H_
#define CSM_ORACLE3D_H_

#include <array>
#include <cstdint>
#include <limits>
#include <memory>
#include <vector>

#include "csm_oracle.h"

namespace oracle {

// ---------------------------------------------------------------------------
// hybrid_grid.h:38-52
inline int ToFlatIndex3(const Idx3& i, int bits) {
  return (((i.z << bits) + i.y) << bits) + i.x;
}
inline Idx3 To3DIndex(int index, int bits) {
  const int mask = (1 << bits) - 1;
  return Idx3{index & mask, (index >> bits) & mask, (index >> bits) >> bits};
}

// FlatGrid<T, 3> (hybrid_grid.h:66-137): 8^3 values.
template <typename T>
struct FlatGrid3 {
  std::array<T, 512> cells{};
};

// NestedGrid<FlatGrid<T,3>,3> (:141-241): 8^3 lazily allocated flat grids.
template <typename T>
struct NestedGrid3 {
  std::array<std::unique_ptr<FlatGrid3<T>>, 512> meta{};
};

// DynamicGrid<NestedGrid<FlatGrid<T,3>,3>> + HybridGridBase (:246-461).
// Index range [-grid_size/2, grid_size/2) per axis; grows by doubling.
template <typename T>
class HybridGridBase3 {
 public:
  explicit HybridGridBase3(float resolution) : resolution_(resolution), meta_(8) {}
  float resolution() const { return resolution_; }
  int grid_size() const { return 64 << bits_; }
  int bits() const { return bits_; }

  // hybrid_grid.h:428-433 — float division, lround per axis.
  Idx3 GetCellIndex(const Vec3f& p) const {
    return Idx3{RoundToIntF(p.x / resolution_), RoundToIntF(p.y / resolution_),
                RoundToIntF(p.z / resolution_)};
  }

  T value(const Idx3& index) const {
    const int half = grid_size() >> 1;
    const Idx3 s{index.x + half, index.y + half, index.z + half};
    const unsigned gs = static_cast<unsigned>(grid_size());
    if (static_cast<unsigned>(s.x) >= gs || static_cast<unsigned>(s.y) >= gs ||
        static_cast<unsigned>(s.z) >= gs)
      return T();
    const Idx3 m{s.x / 64, s.y / 64, s.z / 64};
    const NestedGrid3<T>* nested = meta_[ToFlatIndex3(m, bits_)].get();
    if (!nested) return T();
    const Idx3 in{s.x - m.x * 64, s.y - m.y * 64, s.z - m.z * 64};
    const Idx3 f{in.x / 8, in.y / 8, in.z / 8};
    const FlatGrid3<T>* flat = nested->meta[ToFlatIndex3(f, 3)].get();
    if (!flat) return T();
    return flat->cells[ToFlatIndex3(Idx3{in.x - f.x * 8, in.y - f.y * 8, in.z - f.z * 8}, 3)];
  }

  T* mutable_value(const Idx3& index) {
    for (;;) {
      const int half = grid_size() >> 1;
      const Idx3 s{index.x + half, index.y + half, index.z + half};
      const unsigned gs = static_cast<unsigned>(grid_size());
      if (static_cast<unsigned>(s.x) >= gs || static_cast<unsigned>(s.y) >= gs ||
          static_cast<unsigned>(s.z) >= gs) {
        Grow();
        continue;
      }
      const Idx3 m{s.x / 64, s.y / 64, s.z / 64};
      auto& nested = meta_[ToFlatIndex3(m, bits_)];
      if (!nested) nested.reset(new NestedGrid3<T>());
      const Idx3 in{s.x - m.x * 64, s.y - m.y * 64, s.z - m.z * 64};
      const Idx3 f{in.x / 8, in.y / 8, in.z / 8};
      auto& flat = nested->meta[ToFlatIndex3(f, 3)];
      if (!flat) flat.reset(new FlatGrid3<T>());
      return &flat->cells[ToFlatIndex3(Idx3{in.x - f.x * 8, in.y - f.y * 8, in.z - f.z * 8}, 3)];
    }
  }

  // Iteration over non-default cells in the reference's iterator order
  // (meta cells z-major, then nested, then flat).
  template <typename F>
  void ForEach(F&& f) const {
    const int n = 1 << bits_;
    for (int mi = 0; mi < n * n * n; ++mi) {
      const NestedGrid3<T>* nested = meta_[mi].get();
      if (!nested) continue;
      const Idx3 m = To3DIndex(mi, bits_);
      for (int ni = 0; ni < 512; ++ni) {
        const FlatGrid3<T>* flat = nested->meta[ni].get();
        if (!flat) continue;
        const Idx3 nn = To3DIndex(ni, 3);
        for (int ci = 0; ci < 512; ++ci) {
          const T v = flat->cells[ci];
          if (v == T()) continue;
          const Idx3 c = To3DIndex(ci, 3);
          const int half = (1 << (bits_ - 1)) * 64;
          f(Idx3{m.x * 64 + nn.x * 8 + c.x - half, m.y * 64 + nn.y * 8 + c.y - half,
                 m.z * 64 + nn.z * 8 + c.z - half},
            v);
        }
      }
    }
  }

 private:
  // hybrid_grid.h:384-399
  void Grow() {
    const int new_bits = bits_ + 1;
    std::vector<std::unique_ptr<NestedGrid3<T>>> next(8 * meta_.size());
    for (int z = 0; z != (1 << bits_); ++z)
      for (int y = 0; y != (1 << bits_); ++y)
        for (int x = 0; x != (1 << bits_); ++x) {
          const Idx3 o{x, y, z};
          const int h = 1 << (bits_ - 1);
          next[ToFlatIndex3(Idx3{x + h, y + h, z + h}, new_bits)] =
              std::move(meta_[ToFlatIndex3(o, bits_)]);
        }
    meta_ = std::move(next);
    bits_ = new_bits;
  }

  float resolution_;
  int bits_ = 1;
  std::vector<std::unique_ptr<NestedGrid3<T>>> meta_;
};

// HybridGrid (hybrid_grid.h:463-545): uint16 probability values.
class HybridGrid : public HybridGridBase3<uint16_t> {
 public:
  explicit HybridGrid(float resolution) : HybridGridBase3<uint16_t>(resolution) {}
  void SetProbability(const Idx3& i, float p) { *mutable_value(i) = ProbabilityToValue(p); }
  float GetProbability(const Idx3& i) const { return ValueToProbabilityTable()[value(i)]; }
  bool ApplyLookupTable(const Idx3& i, const std::vector<uint16_t>& table);
  void FinishUpdate();

 private:
  std::vector<uint16_t*> update_indices_;
};

// InterpolatedProbabilityGrid::GetInterpolatedValue (interpolated_grid.h:48-105)
// and its gradient (grad may be null); ceres3d.cc.
double Interpolate(const HybridGrid& g, double x, double y, double z, double grad[3]);

// range_data_inserter_3d.cc:100-136 (hits, then the last num_free_space_voxels
// misses of every ray).
class RangeDataInserter3D {
 public:
  RangeDataInserter3D(float hit_probability, float miss_probability, int num_free_space_voxels);
  void Insert(const Vec3f& origin, const PointCloud& returns, HybridGrid* grid) const;

 private:
  int num_free_space_voxels_;
  std::vector<uint16_t> hit_table_, miss_table_;
};

// precomputation_grid_3d.{h,cc}
typedef HybridGridBase3<uint8_t> PrecomputationGrid3D;
inline float ToProbability3D(float value) {  // precomputation_grid_3d.h:32-35
  return kMinProbability + value * ((kMaxProbability - kMinProbability) / 255.f);
}
std::unique_ptr<PrecomputationGrid3D> ConvertToPrecomputationGrid(const HybridGrid& grid);
std::unique_ptr<PrecomputationGrid3D> PrecomputeGrid(const PrecomputationGrid3D& grid,
                                                     bool half_resolution, const Idx3& shift);

// ---------------------------------------------------------------------------
// Eigen float helpers with the SSE evaluation order.
Quatf QuatMulSse(const Quatf& a, const Quatf& b);      // Geometry_SSE.h quat_product
Quatf QuatNormalizedSse(const Quatf& q);               // (x²+z²)+(y²+w²)
Quatf QuatInverseSse(const Quatf& q);                  // conjugate / squaredNorm
Quatf QuatConjugateF(const Quatf& q);
float ReduxSumSse(const float* v, int n);              // Redux.h packet order
float DotSse(const std::vector<float>& a, const std::vector<float>& b);
float NormSse(const std::vector<float>& a);
Vec3f Rotate3(const Quatf& q, const Vec3f& v);         // _transformVector
Rigid3f Mul3(const Rigid3f& a, const Rigid3f& b);      // rigid_transform.h:183-188
Rigid3f Inverse3(const Rigid3f& a);                    // rigid_transform.h:159-163
Vec3f Apply3(const Rigid3f& r, const Vec3f& p);        // rigid_transform.h:191-196
float NormF(const Vec3f& v);                           // sqrt((x²+y²)+z²)
// transform.h:86-100 (float): scale = sin(norm/2.)/norm in double.
Quatf AngleAxisVectorToRotationQuaternionF(const Vec3f& angle_axis);
float GetAngleF(const Quatf& q);                       // transform.h:34-37
float GetYawF(const Quatf& q);                         // transform.h:43-47

// ---------------------------------------------------------------------------
// rotational_scan_matcher.cc
std::vector<float> RotateHistogram(const std::vector<float>& histogram, float angle);
std::vector<float> ComputeHistogram(const PointCloud& cloud, int histogram_size);
float MatchHistograms(const std::vector<float>& submap, const std::vector<float>& scan);
std::vector<float> RotationalMatch(const std::vector<float>& submap_histogram,
                                   const std::vector<float>& histogram, float initial_angle,
                                   const std::vector<float>& angles);

// low_resolution_matcher.cc:23-35
float LowResolutionScore(const HybridGrid& grid, const PointCloud& points, const Rigid3f& pose);

// ---------------------------------------------------------------------------
// fast_correlative_scan_matcher_3d.{h,cc}
struct FastCsm3dOptions {
  int branch_and_bound_depth = 8;
  int full_resolution_depth = 3;
  double min_rotational_score = 0.77;
  double min_low_resolution_score = 0.55;
  double linear_xy_search_window = 5.;
  double linear_z_search_window = 1.;
  double angular_search_window = 15. * 3.14159265358979323846 / 180.;
};

struct NodeData3D {
  PointCloud high_resolution_point_cloud;
  PointCloud low_resolution_point_cloud;
  std::vector<float> rotational_scan_matcher_histogram;
  Quatd gravity_alignment{1, 0, 0, 0};
};

struct Fast3dResult {
  bool matched = false;
  float score = 0.f;
  Rigid3d pose;
  float rotational_score = 0.f;
  float low_resolution_score = 0.f;
  int64_t lookups = 0;             // precomputation-grid value() calls
  int64_t low_resolution_checks = 0;
  int num_discrete_scans = 0;
};

class FastCorrelativeScanMatcher3D {
 public:
  FastCorrelativeScanMatcher3D(const HybridGrid& hybrid_grid,
                               const HybridGrid* low_resolution_grid,
                               const std::vector<float>* histogram,
                               const FastCsm3dOptions& options);
  Fast3dResult Match(const Rigid3d& global_node_pose, const Rigid3d& global_submap_pose,
                     const NodeData3D& node, float min_score) const;
  Fast3dResult MatchFullSubmap(const Quatd& global_node_rotation,
                               const Quatd& global_submap_rotation, const NodeData3D& node,
                               float min_score) const;
  // Test hook (tie checks): the leaf whose GetPoseFromCandidate equals `pose`
  // exactly, if any, with its score, rotational and low-resolution scores.
  bool EvaluateLeaf(bool full_submap, const Rigid3d& global_node_pose,
                    const Rigid3d& global_submap_pose, const NodeData3D& node,
                    const Rigid3d& pose, Fast3dResult* out) const;
  const PrecomputationGrid3D& level(int d) const { return *levels_.at(d); }
  int num_levels() const { return static_cast<int>(levels_.size()); }
  int width_in_voxels() const { return width_in_voxels_; }

  struct SearchParameters {
    int linear_xy_window_size, linear_z_window_size;
    double angular_search_window;
  };
  struct DiscreteScan3D {
    Rigid3f pose;
    std::vector<std::vector<Idx3>> cell_indices_per_depth;
    float rotational_score;
  };
  struct Candidate3D {
    int scan_index = 0;
    Idx3 offset{0, 0, 0};
    float score = -std::numeric_limits<float>::infinity();  // (fast_correlative_scan_matcher_3d.cc:104)
    float low_resolution_score = 0.f;
  };
  std::vector<DiscreteScan3D> GenerateDiscreteScans(const SearchParameters& sp,
                                                    const PointCloud& cloud,
                                                    const std::vector<float>& histogram,
                                                    const Quatd& gravity_alignment,
                                                    const Rigid3f& global_node_pose,
                                                    const Rigid3f& global_submap_pose) const;

 private:
  void Setup(bool full_submap, const Rigid3d& node_pose, const Rigid3d& submap_pose,
             const NodeData3D& node, SearchParameters* sp, Rigid3f* np, Rigid3f* spf) const;
  Fast3dResult MatchWithSearchParameters(const SearchParameters& sp,
                                         const Rigid3f& global_node_pose,
                                         const Rigid3f& global_submap_pose,
                                         const NodeData3D& node, float min_score) const;
  DiscreteScan3D DiscretizeScan(const SearchParameters& sp, const PointCloud& cloud,
                                const Rigid3f& pose, float rotational_score) const;
  void ScoreCandidates(int depth, const std::vector<DiscreteScan3D>& scans,
                       std::vector<Candidate3D>* candidates, int64_t* lookups) const;
  Candidate3D BranchAndBound(const SearchParameters& sp,
                             const std::vector<DiscreteScan3D>& scans,
                             const std::vector<Candidate3D>& candidates, int depth,
                             float min_score, const NodeData3D& node, Fast3dResult* stats) const;
  Rigid3f GetPoseFromCandidate(const std::vector<DiscreteScan3D>& scans,
                               const Candidate3D& c) const;

  FastCsm3dOptions options_;
  float resolution_;
  int width_in_voxels_;
  std::vector<std::unique_ptr<PrecomputationGrid3D>> levels_;
  const HybridGrid* low_resolution_grid_;
  const std::vector<float>* histogram_;
};

// ---------------------------------------------------------------------------
// real_time_correlative_scan_matcher_3d.cc
struct RtOptions3D {
  double linear_search_window = 0.15;
  double angular_search_window = 1. * 3.14159265358979323846 / 180.;
  double translation_delta_cost_weight = 1e-1;
  double rotation_delta_cost_weight = 1e-1;
};
struct Rt3dResult {
  float score = -1.f;
  Rigid3d pose;
  int64_t candidates = 0;
  int64_t best_index = -1;  // linear (z, y, x, rz, ry, rx) index of the winner
};
// Exhaustive search exactly as the reference orders it (first strict max).
// `max_candidates` bounds the work (0 = no bound; larger searches abort).
Rt3dResult RealTimeMatch3D(const RtOptions3D& options, const Rigid3d& initial,
                           const PointCloud& cloud, const HybridGrid& grid);
// CPU baseline timing: seconds for `count` candidates (indices i * stride),
// each transformed and scored the way Match does it.
double RealTimeTime3D(const RtOptions3D& options, const Rigid3d& initial, const PointCloud& cloud,
                      const HybridGrid& grid, int64_t count, int64_t stride, float* sink);
// Search-space geometry (for tests/bench): linear window size, angular step
// and window size.
void RealTime3DWindow(const RtOptions3D& options, float resolution, const PointCloud& cloud,
                      int* linear_window, float* angular_step, int* angular_window);
// Score of one candidate (linear index in the reference's loop order).
float RealTimeScore3D(const RtOptions3D& options, const Rigid3d& initial,
                      const PointCloud& cloud, const HybridGrid& grid, int64_t index,
                      Rigid3f* candidate_out);

// mapping/internal/3d/scan_matching/ceres_scan_matcher_3d.cc (ceres3d.cc).
struct CeresOptions3D {
  double w0 = 5., w1 = 30., wt = 10., wr = 1.;
  int max_num_iterations = 10;
  bool use_nonmonotonic_steps = false;
};
int CeresMatch3D(const HybridGrid& high, const HybridGrid& low, const std::vector<Vec3f>& high_cloud,
                 const std::vector<Vec3f>& low_cloud, const CeresOptions3D& o,
                 const double target[3], const double initial_t[3], const double initial_q[4],
                 double out_t[3], double out_q[4], double* final_cost);
// RotationDeltaCostFunctor3D residuals (rotation_delta_cost_functor_3d.h):
// scale * vec(target^-1 * q), quaternions (w, x, y, z).
void RotationDeltaResiduals3D(double scale, const double target_q[4], const double q[4],
                              double out[3]);

}  // namespace oracle

#endif  // CSM_ORACLE3D_H_
