// Host-side search-window arithmetic of the 2D correlative scan matchers,
// with the reference's exact float/double semantics. Shared by the batch
// path, the single-call path and the real-time matcher.
#ifndef CSM_SEARCH_WINDOW_H_
#define CSM_SEARCH_WINDOW_H_

#include <cstdint>
#include <vector>

namespace csm {

// correlative_scan_matcher_2d.cc:27-55 (SearchParameters ctor).
struct SearchWindow2D {
  int num_angular_perturbations = 0;
  double angular_perturbation_step_size = 0.;
  int num_scans = 0;
  int num_linear_perturbations = 0;  // before ShrinkToFit
};

// Eigen Quaternion(AngleAxisf(angle, UnitZ)) as (w, s): w = cos(0.5f*a),
// s = sin(0.5f*a) (Eigen Quaternion.h operator=(AngleAxis)).
struct ZRot {
  float w, s;
};
ZRot MakeZRot(float angle);
// QuaternionBase::_transformVector specialised to a z-axis quaternion, in
// the exact operation order (see DESIGN.md "Bitwise discretization").
void RotateZ(const ZRot& q, float x, float y, float* ox, float* oy);

// max_scan_range over the cloud (optionally pre-rotated by `pre`), then the
// step/count formulas. `rotate_first` selects RTCSM semantics (window built
// on the pre-rotated cloud, real_time_correlative_scan_matcher_2d.cc:128-130)
// versus FastCSM (input cloud, fast_correlative_scan_matcher_2d.cc:202-204).
SearchWindow2D MakeSearchWindow2D(double linear_window, double angular_window,
                                  const float* xyz, int32_t n, double resolution,
                                  const ZRot* pre);

// GenerateRotatedScans angles (correlative_scan_matcher_2d.cc:99-106): theta
// accumulated in double, narrowed to float, turned into (w, s) pairs.
void RotationTable(const SearchWindow2D& w, std::vector<ZRot>* out);

// PrecomputationGrid2D::ComputeCellValue applied to 1 - |cc(value)| for all
// 32768 masked cell values (fast_correlative_scan_matcher_2d.cc:163-169 with
// Grid2D::GetCorrespondenceCost's table, value_conversion_tables.cc:28-52).
// Returns false if a value falls outside [0, 255] (the reference CHECKs).
bool QuantizationTable(float min_cc, float max_cc, uint8_t* out32768);

// Probability table for RTCSM: 1 - kValueToCorrespondenceCost[v]
// (probability_grid.cc:78-82, probability_values.cc:26-66).
void ProbabilityTable(float* out32768);
// ValueConversionTables::GetConversionTable(unknown, lower, upper)
// (value_conversion_tables.cc:28-52) over the 32768 unmarked values.
void ConversionTable(float unknown_result, float lower, float upper, float* out32768);

// PrecomputationGrid2D::ToScore(sum / float(n)) (fast_correlative_scan_
// matcher_2d.h:74-76, .cc:328-329).
float SumToScore(int64_t sum, int32_t n, float min_s, float max_s);
// Largest integer sum whose score is <= min_score (-1 if none): a candidate
// with bound sum <= this value is pruned / rejected exactly as the
// reference's `score <= min_score` tests (.cc:253, :348).
int64_t MaxRejectedSum(float min_score, int32_t n, float min_s, float max_s);

}  // namespace csm

#endif  // CSM_SEARCH_WINDOW_H_
