// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// extern "C" surface for TSDF2D: building TSDF grids with the restated
// TSDFRangeDataInserter2D (test fixtures) and RealTimeCorrelativeScanMatcher2D
// over a TSDF2D (the checker for csm_rt2d_match_tsdf).

#include <algorithm>
#include <cstdint>
#include <vector>

#include "oracle_tsdf.h"

using namespace oracle;

namespace {
MapLimits ToLimitsT(double res, double max_x, double max_y, int nx, int ny) {
  MapLimits l;
  l.resolution = res;
  l.max_x = max_x;
  l.max_y = max_y;
  l.cells = CellLimits{nx, ny};
  return l;
}
}  // namespace

extern "C" {

void* oracle_tsdf_create(double res, double max_x, double max_y, int32_t nx, int32_t ny,
                         float truncation_distance, float max_weight) {
  return new TSDF2D(ToLimitsT(res, max_x, max_y, nx, ny), truncation_distance, max_weight);
}

void oracle_tsdf_destroy(void* h) { delete static_cast<TSDF2D*>(h); }

// opts: truncation_distance, maximum_weight, update_free_space,
// num_normal_samples, sample_radius, project_sdf_distance_to_scan_normal,
// update_weight_range_exponent, angle bandwidth, distance bandwidth.
void oracle_tsdf_insert(void* h, const double* opts, const float* origin, const float* xyz,
                        int32_t n) {
  TSDFInserterOptions2D o;
  o.truncation_distance = opts[0];
  o.maximum_weight = opts[1];
  o.update_free_space = opts[2] != 0.;
  o.normal_estimation.num_normal_samples = static_cast<int>(opts[3]);
  o.normal_estimation.sample_radius = static_cast<float>(opts[4]);
  o.project_sdf_distance_to_scan_normal = opts[5] != 0.;
  o.update_weight_range_exponent = static_cast<int>(opts[6]);
  o.update_weight_angle_scan_normal_to_ray_kernel_bandwidth = opts[7];
  o.update_weight_distance_cell_to_hit_kernel_bandwidth = opts[8];
  RangeData rd;
  rd.origin = Vec3f{origin[0], origin[1], origin[2]};
  rd.returns.resize(static_cast<size_t>(n));
  for (int32_t i = 0; i < n; ++i) rd.returns[i] = Vec3f{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
  TSDFRangeDataInserter2D(o).Insert(rd, static_cast<TSDF2D*>(h));
}

void oracle_tsdf_info(void* h, double* limits3, int32_t* cells2) {
  const MapLimits& l = static_cast<TSDF2D*>(h)->limits();
  limits3[0] = l.resolution;
  limits3[1] = l.max_x;
  limits3[2] = l.max_y;
  cells2[0] = l.cells.num_x_cells;
  cells2[1] = l.cells.num_y_cells;
}

void oracle_tsdf_cells(void* h, uint16_t* tsd, uint16_t* weight) {
  const TSDF2D* t = static_cast<TSDF2D*>(h);
  std::copy(t->tsd_cells().begin(), t->tsd_cells().end(), tsd);
  std::copy(t->weight_cells().begin(), t->weight_cells().end(), weight);
}

// RealTimeCorrelativeScanMatcher2D::Match over a TSDF2D.
double oracle_rt2d_match_tsdf(double res, double max_x, double max_y, int32_t nx, int32_t ny,
                              const uint16_t* tsd, const uint16_t* weight,
                              float truncation_distance, float max_weight, double lin, double ang,
                              double wt, double wr, const double* initial, const float* xyz,
                              int32_t n, double* pose_out, int64_t* num_candidates) {
  const size_t cells = static_cast<size_t>(nx) * ny;
  const TSDF2D t(ToLimitsT(res, max_x, max_y, nx, ny), truncation_distance, max_weight,
                 std::vector<uint16_t>(tsd, tsd + cells), std::vector<uint16_t>(weight, weight + cells));
  RealTimeOptions o;
  o.linear_search_window = lin;
  o.angular_search_window = ang;
  o.translation_delta_cost_weight = wt;
  o.rotation_delta_cost_weight = wr;
  Rigid2d init;
  init.tx = initial[0];
  init.ty = initial[1];
  init.angle = initial[2];
  PointCloud cloud(static_cast<size_t>(n));
  for (int32_t i = 0; i < n; ++i) cloud[i] = Vec3f{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]};
  Rigid2d pose;
  const double s = RealTimeMatchTSDF(o, init, cloud, t, &pose, num_candidates);
  pose_out[0] = pose.tx;
  pose_out[1] = pose.ty;
  pose_out[2] = pose.angle;
  return s;
}

// RealTimeScoreCandidatesTSDF (ScoreCandidates over a TSDF2D), arguments as
// oracle_rt2d_score_candidates.
int32_t oracle_rt2d_score_candidates_tsdf(double res, double max_x, double max_y, int32_t nx,
                                          int32_t ny, const uint16_t* tsd, const uint16_t* weight,
                                          float truncation_distance, float max_weight, double wt,
                                          double wr, const int32_t* discrete, int32_t num_scans,
                                          int32_t n, int32_t num_angular, double step,
                                          const int32_t* cands, int64_t count, float* out) {
  const size_t cells = static_cast<size_t>(nx) * ny;
  const TSDF2D t(ToLimitsT(res, max_x, max_y, nx, ny), truncation_distance, max_weight,
                 std::vector<uint16_t>(tsd, tsd + cells), std::vector<uint16_t>(weight, weight + cells));
  RealTimeOptions o;
  o.translation_delta_cost_weight = wt;
  o.rotation_delta_cost_weight = wr;
  std::vector<DiscreteScan2D> scans(static_cast<size_t>(num_scans));
  for (int s = 0; s < num_scans; ++s)
    for (int i = 0; i < n; ++i) {
      const int64_t k = static_cast<int64_t>(s) * n + i;
      scans[s].push_back(Idx2{discrete[2 * k], discrete[2 * k + 1]});
    }
  const SearchParameters sp(0, num_angular, step, res);
  std::vector<Candidate2D> c;
  for (int64_t i = 0; i < count; ++i) c.emplace_back(cands[3 * i], cands[3 * i + 1], cands[3 * i + 2], sp);
  RealTimeScoreCandidatesTSDF(o, t, scans, &c);
  for (int64_t i = 0; i < count; ++i) out[i] = c[i].score;
  return 0;
}

}  // extern "C"
