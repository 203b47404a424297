// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// TSDF2D grids and RealTimeCorrelativeScanMatcher2D scoring over them,
// restated from the reference:
//   mapping/internal/2d/tsd_value_converter.{h,cc}
//   mapping/internal/2d/tsdf_2d.{h,cc}
//   mapping/internal/2d/normal_estimation_2d.cc
//   mapping/internal/2d/tsdf_range_data_inserter_2d.cc
//   mapping/internal/2d/scan_matching/real_time_correlative_scan_matcher_2d.cc:38-59
// The inserter and normal estimation only rebuild the grids the reference's
// own tests score against; the scan matcher consumes the uint16 cells.

#ifndef CSM_ORACLE_TSDF_H_
#define CSM_ORACLE_TSDF_H_

#include <cstdint>
#include <utility>
#include <vector>

#include "csm_oracle.h"

namespace oracle {

// tsd_value_converter.{h,cc}
class TSDValueConverter {
 public:
  TSDValueConverter(float max_tsd, float max_weight);
  uint16_t TSDToValue(float tsd) const;
  uint16_t WeightToValue(float weight) const;
  float ValueToTSD(uint16_t v) const { return value_to_tsd_[v]; }
  float ValueToWeight(uint16_t v) const { return value_to_weight_[v]; }
  float max_tsd() const { return max_tsd_; }
  float min_tsd() const { return min_tsd_; }
  float max_weight() const { return max_weight_; }
  float min_weight() const { return 0.f; }
  const std::vector<float>& tsd_table() const { return value_to_tsd_; }
  const std::vector<float>& weight_table() const { return value_to_weight_; }

 private:
  float max_tsd_, min_tsd_, max_weight_, tsd_resolution_, weight_resolution_;
  std::vector<float> value_to_tsd_, value_to_weight_;
};

// tsdf_2d.{h,cc} on top of grid_2d.{h,cc}: correspondence-cost cells hold the
// TSD values, min/max correspondence cost = -/+ truncation distance.
class TSDF2D {
 public:
  TSDF2D(const MapLimits& limits, float truncation_distance, float max_weight);
  TSDF2D(const MapLimits& limits, float truncation_distance, float max_weight,
         std::vector<uint16_t> tsd_cells, std::vector<uint16_t> weight_cells);

  const MapLimits& limits() const { return limits_; }
  const std::vector<uint16_t>& tsd_cells() const { return tsd_cells_; }
  const std::vector<uint16_t>& weight_cells() const { return weight_cells_; }
  const TSDValueConverter& converter() const { return conv_; }
  float GetMaxCorrespondenceCost() const { return conv_.max_tsd(); }

  bool CellIsUpdated(const Idx2& i) const;
  void SetCell(const Idx2& i, float tsd, float weight);
  float GetTSD(const Idx2& i) const;
  float GetWeight(const Idx2& i) const;
  std::pair<float, float> GetTSDAndWeight(const Idx2& i) const;
  bool IsKnown(const Idx2& i) const;
  void FinishUpdate();
  void GrowLimits(float px, float py);
  void ComputeCroppedLimits(Idx2* offset, CellLimits* limits) const;

 private:
  int FlatIndex(const Idx2& i) const;
  MapLimits limits_;
  TSDValueConverter conv_;
  std::vector<uint16_t> tsd_cells_, weight_cells_;
  std::vector<int> update_indices_;
  bool box_empty_ = true;
  int box_min_x_ = 0, box_min_y_ = 0, box_max_x_ = 0, box_max_y_ = 0;
};

// normal_estimation_2d.cc
struct NormalEstimationOptions2D {
  int num_normal_samples = 4;
  float sample_radius = 0.5f;
};
std::vector<float> EstimateNormals(const RangeData& range_data,
                                   const NormalEstimationOptions2D& options);

// tsdf_range_data_inserter_2d.cc
struct TSDFInserterOptions2D {
  double truncation_distance = 0.3;
  double maximum_weight = 10.;
  bool update_free_space = false;
  NormalEstimationOptions2D normal_estimation;
  bool project_sdf_distance_to_scan_normal = true;
  int update_weight_range_exponent = 0;
  double update_weight_angle_scan_normal_to_ray_kernel_bandwidth = 0.5;
  double update_weight_distance_cell_to_hit_kernel_bandwidth = 0.5;
};

class TSDFRangeDataInserter2D {
 public:
  explicit TSDFRangeDataInserter2D(const TSDFInserterOptions2D& o) : options_(o) {}
  void Insert(const RangeData& range_data, TSDF2D* tsdf) const;

 private:
  void InsertHit(const Vec2f& hit, const Vec2f& origin, float normal,
                 TSDF2D* tsdf) const;
  void UpdateCell(const Idx2& cell, float update_sdf, float update_weight,
                  TSDF2D* tsdf) const;
  TSDFInserterOptions2D options_;
};

// real_time_correlative_scan_matcher_2d.cc:38-59, 117-176 over a TSDF2D.
double RealTimeMatchTSDF(const RealTimeOptions& options, const Rigid2d& initial,
                         const PointCloud& cloud, const TSDF2D& tsdf,
                         Rigid2d* pose, int64_t* num_candidates = nullptr);
void RealTimeScoreCandidatesTSDF(const RealTimeOptions& options,
                                 const TSDF2D& tsdf,
                                 const std::vector<DiscreteScan2D>& scans,
                                 std::vector<Candidate2D>* candidates);

}  // namespace oracle

#endif  // CSM_ORACLE_TSDF_H_
