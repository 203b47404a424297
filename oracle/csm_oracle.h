// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of Cartographer's correlative scan matching hot path
// (reference: juwangvsu/cartographer-1 @ /root/reference). It is the checker
// for the MI355X product in cartographer-1_amd/, never the thing measured or
// shipped: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load it.
//
// Parity pinning: the reference C++ cannot be compiled in this image (it needs
// Eigen, absl, glog, Ceres, Lua, protobuf, PCL — see DESIGN.md), and it holds
// no Python implementation. The restatement is therefore pinned by every
// known-answer / property test the reference's own unit tests hold for this
// path, restated in oracle/ref_tests.cc (see DESIGN.md "Oracle").
//
// Eigen arithmetic (quaternion rotation, Affine2f translation) is restated
// from Eigen 3.3's Quaternion.h / OrthoMethods.h / Transform.h formulas with
// the exact float/double operation order, since the x86-64 reference build
// (-O3, no -march) never contracts to FMA.

#ifndef CSM_ORACLE_H_
#define CSM_ORACLE_H_

#include <cstdint>
#include <array>
#include <vector>

namespace oracle {

// ---------------------------------------------------------------------------
// common/port.h:40-42 — RoundToInt is std::lround (half away from zero).
int RoundToInt(double x);
int RoundToIntF(float x);

// ---------------------------------------------------------------------------
// Small POD math (stand-ins for the Eigen types the reference uses).
struct Vec2f { float x, y; };
struct Vec3f { float x, y, z; };
struct Vec2d { double x, y; };
struct Vec3d { double x, y, z; };
struct Idx2 { int x, y; };
struct Idx3 { int x, y, z; };
struct Quatf { float w, x, y, z; };
struct Quatd { double w, x, y, z; };

// Eigen::Quaternion<float>(Eigen::AngleAxisf(angle, axis)):
//   w = cos(0.5f*angle), vec = sin(0.5f*angle) * axis.
Quatf QuatFromAngleAxisF(float angle, float ax, float ay, float az);
Quatd QuatFromAngleAxisD(double angle, double ax, double ay, double az);
// QuaternionBase::_transformVector (Eigen 3.3 Quaternion.h):
//   uv = q.vec x v; uv += uv; return v + q.w*uv + q.vec x uv.
Vec3f Rotate(const Quatf& q, const Vec3f& v);
Vec3d Rotate(const Quatd& q, const Vec3d& v);
Quatf QuatMul(const Quatf& a, const Quatf& b);
Quatd QuatMul(const Quatd& a, const Quatd& b);
Quatf QuatNormalized(const Quatf& q);
Quatd QuatNormalized(const Quatd& q);
Quatd QuatConjugate(const Quatd& q);

// transform/rigid_transform.h:33-107 — Rigid2 with an (unnormalized) angle.
struct Rigid2d {
  double tx = 0, ty = 0, angle = 0;
};
struct Rigid2f {
  float tx = 0, ty = 0, angle = 0;
};
Rigid2d Mul(const Rigid2d& a, const Rigid2d& b);
Rigid2f Mul(const Rigid2f& a, const Rigid2f& b);
Rigid2f Inverse(const Rigid2f& a);
Rigid2d Inverse(const Rigid2d& a);

// transform/rigid_transform.h:109-196 — Rigid3.
struct Rigid3f {
  Vec3f t{0, 0, 0};
  Quatf q{1, 0, 0, 0};
};
struct Rigid3d {
  Vec3d t{0, 0, 0};
  Quatd q{1, 0, 0, 0};
};
Vec3f Apply(const Rigid3f& r, const Vec3f& p);
Vec3d Apply(const Rigid3d& r, const Vec3d& p);
Rigid3f Mul(const Rigid3f& a, const Rigid3f& b);  // normalizes (:183-188)
Rigid3d Mul(const Rigid3d& a, const Rigid3d& b);
Rigid3d Inverse(const Rigid3d& a);
Rigid3f CastF(const Rigid3d& a);
// transform/transform.h:103-115
Rigid3f Embed3D(const Rigid2f& r);
Rigid3d Embed3D(const Rigid2d& r);

typedef std::vector<Vec3f> PointCloud;
// sensor/point_cloud.cc:56-64
PointCloud TransformPointCloud(const PointCloud& cloud, const Rigid3f& r);

// rigid_transform_test_helpers.h — IsNearly via Eigen isApprox on the 3x3
// homogeneous matrices: ||a-b||_F <= eps * min(||a||_F, ||b||_F).
bool IsNearly2D(const Rigid2f& a, const Rigid2f& b, float eps);

// ---------------------------------------------------------------------------
// mapping/probability_values.{h,cc}, value_conversion_tables.cc
constexpr float kMinProbability = 0.1f;
constexpr float kMaxProbability = 1.f - kMinProbability;
constexpr float kMinCorrespondenceCost = 1.f - kMaxProbability;
constexpr float kMaxCorrespondenceCost = 1.f - kMinProbability;
constexpr uint16_t kUnknownValue = 0;
constexpr uint16_t kUpdateMarker = 1u << 15;

float Odds(float p);
float ProbabilityFromOdds(float odds);
uint16_t BoundedFloatToValue(float v, float lo, float hi);
uint16_t CorrespondenceCostToValue(float cc);
uint16_t ProbabilityToValue(float p);
// 65536-entry tables: value (bit 15 masked) -> float, 0 -> unknown_result.
const std::vector<float>& ValueToCorrespondenceCostTable();
const std::vector<float>& ValueToProbabilityTable();
std::vector<float> MakeConversionTable(float unknown_result, float lo, float hi);
std::vector<uint16_t> LookupTableToApplyCorrespondenceCostOdds(float odds);
std::vector<uint16_t> LookupTableToApplyOdds(float odds);

// ---------------------------------------------------------------------------
// mapping/2d/map_limits.h, xy_index.h
struct CellLimits {
  int num_x_cells = 0;
  int num_y_cells = 0;
};

struct MapLimits {
  double resolution = 0.05;
  double max_x = 0, max_y = 0;
  CellLimits cells;
  // map_limits.h:69-75 (double arithmetic, lround)
  Idx2 GetCellIndex(float px, float py) const;
  bool Contains(const Idx2& i) const;
};

// mapping/2d/probability_grid.{h,cc} + grid_2d.{h,cc} (probability grid only).
class ProbabilityGrid {
 public:
  explicit ProbabilityGrid(const MapLimits& limits);
  ProbabilityGrid(const MapLimits& limits, std::vector<uint16_t> cells);

  const MapLimits& limits() const { return limits_; }
  const std::vector<uint16_t>& cells() const { return cells_; }
  std::vector<uint16_t>* mutable_cells() { return &cells_; }
  float min_correspondence_cost() const { return kMinCorrespondenceCost; }
  float max_correspondence_cost() const { return kMaxCorrespondenceCost; }

  int FlatIndex(const Idx2& i) const;
  float GetCorrespondenceCost(const Idx2& i) const;
  float GetProbability(const Idx2& i) const;
  bool IsKnown(const Idx2& i) const;
  void SetProbability(const Idx2& i, float p);
  bool ApplyLookupTable(const Idx2& i, const std::vector<uint16_t>& table);
  void FinishUpdate();
  void GrowLimits(float px, float py);
  void ComputeCroppedLimits(Idx2* offset, CellLimits* limits) const;
  ProbabilityGrid ComputeCroppedGrid() const;

 private:
  MapLimits limits_;
  std::vector<uint16_t> cells_;
  std::vector<int> update_indices_;
  bool box_empty_ = true;
  int box_min_x_ = 0, box_min_y_ = 0, box_max_x_ = 0, box_max_y_ = 0;
  void ExtendBox(const Idx2& i);
};

// mapping/internal/2d/ray_to_pixel_mask.cc
std::vector<Idx2> RayToPixelMask(Idx2 scaled_begin, Idx2 scaled_end,
                                 int subpixel_scale);

// mapping/2d/probability_grid_range_data_inserter_2d.cc
struct RangeData {
  Vec3f origin;
  PointCloud returns;
  PointCloud misses;
};
class ProbabilityGridInserter2D {
 public:
  ProbabilityGridInserter2D(float hit_probability, float miss_probability,
                            bool insert_free_space);
  void Insert(const RangeData& range_data, ProbabilityGrid* grid) const;

 private:
  bool insert_free_space_;
  std::vector<uint16_t> hit_table_, miss_table_;
};

// ---------------------------------------------------------------------------
// mapping/internal/2d/scan_matching/correlative_scan_matcher_2d.{h,cc}
typedef std::vector<Idx2> DiscreteScan2D;

struct LinearBounds {
  int min_x, max_x, min_y, max_y;
};

struct SearchParameters {
  SearchParameters(double linear_search_window, double angular_search_window,
                   const PointCloud& cloud, double resolution);
  SearchParameters(int num_linear_perturbations, int num_angular_perturbations,
                   double angular_perturbation_step_size, double resolution);
  void ShrinkToFit(const std::vector<DiscreteScan2D>& scans,
                   const CellLimits& cell_limits);

  int num_angular_perturbations;
  double angular_perturbation_step_size;
  double resolution;
  int num_scans;
  std::vector<LinearBounds> linear_bounds;
};

std::vector<PointCloud> GenerateRotatedScans(const PointCloud& cloud,
                                             const SearchParameters& sp);
std::vector<DiscreteScan2D> DiscretizeScans(const MapLimits& limits,
                                            const std::vector<PointCloud>& scans,
                                            float tx, float ty);

struct Candidate2D {
  Candidate2D(int scan_index, int x_off, int y_off, const SearchParameters& sp);
  int scan_index = 0;
  int x_index_offset = 0;
  int y_index_offset = 0;
  double x = 0., y = 0., orientation = 0.;
  float score = 0.f;
  bool operator<(const Candidate2D& o) const { return score < o.score; }
  bool operator>(const Candidate2D& o) const { return score > o.score; }
};

// mapping/internal/2d/scan_matching/fast_correlative_scan_matcher_2d.{h,cc}
class PrecomputationGrid2D {
 public:
  PrecomputationGrid2D(const ProbabilityGrid& grid, const CellLimits& limits,
                       int width, std::vector<float>* scratch);
  int GetValue(const Idx2& xy) const {
    const int lx = xy.x - offset_x_, ly = xy.y - offset_y_;
    if (static_cast<unsigned>(lx) >= static_cast<unsigned>(wide_.num_x_cells) ||
        static_cast<unsigned>(ly) >= static_cast<unsigned>(wide_.num_y_cells))
      return 0;
    return cells_[lx + ly * wide_.num_x_cells];
  }
  float ToScore(float value) const {
    return min_score_ + value * ((max_score_ - min_score_) / 255.f);
  }
  const std::vector<uint8_t>& cells() const { return cells_; }
  const CellLimits& wide_limits() const { return wide_; }
  int offset_x() const { return offset_x_; }
  int offset_y() const { return offset_y_; }

 private:
  uint8_t ComputeCellValue(float probability) const;
  int offset_x_, offset_y_;
  CellLimits wide_;
  float min_score_, max_score_;
  std::vector<uint8_t> cells_;
};

struct FastOptions2D {
  double linear_search_window = 7.;
  double angular_search_window = 30. * 3.14159265358979323846 / 180.;
  int branch_and_bound_depth = 7;
};

// Counters for §8d (reporting only): lookups and candidates per level.
struct MatchStats2D {
  int64_t lookups = 0;
  int64_t candidates_per_level[16] = {0};
  int num_scans = 0;
  int64_t lowest_resolution_candidates = 0;
};

class FastCorrelativeScanMatcher2D {
 public:
  FastCorrelativeScanMatcher2D(const ProbabilityGrid& grid,
                               const FastOptions2D& options);
  bool Match(const Rigid2d& initial, const PointCloud& cloud, float min_score,
             float* score, Rigid2d* pose, MatchStats2D* stats = nullptr) const;
  bool MatchFullSubmap(const PointCloud& cloud, float min_score, float* score,
                       Rigid2d* pose, MatchStats2D* stats = nullptr) const;
  const PrecomputationGrid2D& Level(int i) const { return grids_[i]; }
  // Test-only (tie statistics): every leaf {scan_index, x_off, y_off} whose
  // score equals the maximum leaf score, when that maximum beats min_score
  // (the set the reference's DFS picks its first-visited member from), and
  // the reference's own pick in *picked. Empty if nothing beats min_score.
  std::vector<std::array<int, 3>> TiedMaxLeaves(bool full_submap, const Rigid2d& initial,
                                                const PointCloud& cloud, float min_score,
                                                size_t max_out,
                                                std::array<int, 3>* picked) const;
  int max_depth() const { return static_cast<int>(grids_.size()) - 1; }
  const MapLimits& limits() const { return limits_; }

 private:
  bool MatchWithSearchParameters(SearchParameters sp, const Rigid2d& initial,
                                 const PointCloud& cloud, float min_score,
                                 float* score, Rigid2d* pose,
                                 MatchStats2D* stats) const;
  std::vector<Candidate2D> GenerateLowestResolutionCandidates(
      const SearchParameters& sp) const;
  void ScoreCandidates(const PrecomputationGrid2D& grid,
                       const std::vector<DiscreteScan2D>& scans,
                       std::vector<Candidate2D>* candidates,
                       MatchStats2D* stats) const;
  void CollectTies(const std::vector<DiscreteScan2D>& scans, const SearchParameters& sp,
                   const std::vector<Candidate2D>& candidates, int depth, float best,
                   size_t max_out, std::vector<std::array<int, 3>>* out) const;
  Candidate2D BranchAndBound(const std::vector<DiscreteScan2D>& scans,
                             const SearchParameters& sp,
                             const std::vector<Candidate2D>& candidates,
                             int depth, float min_score,
                             MatchStats2D* stats) const;

  FastOptions2D options_;
  MapLimits limits_;
  std::vector<PrecomputationGrid2D> grids_;
};

// mapping/internal/2d/scan_matching/real_time_correlative_scan_matcher_2d.cc
struct RealTimeOptions {
  double linear_search_window = 0.1;
  double angular_search_window = 20. * 3.14159265358979323846 / 180.;
  double translation_delta_cost_weight = 1e-1;
  double rotation_delta_cost_weight = 1e-1;
};

class RealTimeCorrelativeScanMatcher2D {
 public:
  explicit RealTimeCorrelativeScanMatcher2D(const RealTimeOptions& o)
      : options_(o) {}
  double Match(const Rigid2d& initial, const PointCloud& cloud,
               const ProbabilityGrid& grid, Rigid2d* pose,
               int64_t* num_candidates = nullptr) const;
  void ScoreCandidates(const ProbabilityGrid& grid,
                       const std::vector<DiscreteScan2D>& scans,
                       std::vector<Candidate2D>* candidates) const;
  std::vector<Candidate2D> GenerateExhaustiveSearchCandidates(
      const SearchParameters& sp) const;

 private:
  RealTimeOptions options_;
};

// mapping/internal/2d/scan_matching/ceres_scan_matcher_2d.cc (ceres2d.cc)
struct CeresOptions2D {
  double occupied_space_weight = 20., translation_weight = 10., rotation_weight = 1.;
  int max_num_iterations = 10;
  bool use_nonmonotonic_steps = true;
};
int CeresMatch2D(const MapLimits& limits, const std::vector<uint16_t>& cells, float min_cc,
                 float max_cc, const CeresOptions2D& o, const double target[2],
                 const double initial[3], const std::vector<Vec2d>& points, double pose[3],
                 double* final_cost);
std::vector<double> OccupiedSpaceResiduals2D(const MapLimits& limits,
                                             const std::vector<uint16_t>& cells, float min_cc,
                                             float max_cc, double weight,
                                             const std::vector<Vec2d>& points,
                                             const double pose[3]);

}  // namespace oracle

#endif  // CSM_ORACLE_H_
