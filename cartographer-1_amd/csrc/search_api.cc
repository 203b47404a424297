// C-ABI of the search-space helpers in correlative_scan_matcher_2d.{h,cc}
// (SearchParameters, ShrinkToFit, GenerateRotatedScans, DiscretizeScans):
// host-side, with the reference's float/double arithmetic — the same
// functions (search_window.cc) the device path uses for its windows and
// rotation tables, and the same GetCellIndex arithmetic as its kernels.
#include <algorithm>
#include <cmath>
#include <vector>

#include "../../include/csm_amd.h"
#include "search_window.h"

namespace {

bool ValidSp(const csm_search_parameters* sp) {
  return sp && sp->num_scans >= 1 && sp->num_scans == 2 * sp->num_angular_perturbations + 1 &&
         sp->num_linear_perturbations >= 0 && sp->resolution >= 0.;
}

}  // namespace

extern "C" {

int csm_search_parameters_init(double linear_search_window, double angular_search_window,
                               const float* points_xyz, int32_t n, double resolution,
                               csm_search_parameters* out) {
  if (!out || n < 0 || (n > 0 && !points_xyz) || !(resolution > 0.) ||
      !(linear_search_window >= 0.) || !(angular_search_window >= 0.))
    return CSM_EINVAL;
  const csm::SearchWindow2D w = csm::MakeSearchWindow2D(
      linear_search_window, angular_search_window, points_xyz, n, resolution, nullptr);
  if (w.num_scans < 1 || w.num_angular_perturbations > (1 << 24)) return CSM_ERANGE;
  out->num_angular_perturbations = w.num_angular_perturbations;
  out->angular_perturbation_step_size = w.angular_perturbation_step_size;
  out->resolution = resolution;
  out->num_scans = w.num_scans;
  out->num_linear_perturbations = w.num_linear_perturbations;
  return CSM_OK;
}

int csm_search_parameters_init_for_testing(int32_t num_linear_perturbations,
                                           int32_t num_angular_perturbations,
                                           double angular_perturbation_step_size,
                                           double resolution, csm_search_parameters* out) {
  if (!out || num_linear_perturbations < 0 || num_angular_perturbations < 0 ||
      num_angular_perturbations > (1 << 24))
    return CSM_EINVAL;
  out->num_angular_perturbations = num_angular_perturbations;
  out->angular_perturbation_step_size = angular_perturbation_step_size;
  out->resolution = resolution;
  out->num_scans = 2 * num_angular_perturbations + 1;
  out->num_linear_perturbations = num_linear_perturbations;
  return CSM_OK;
}

int csm_search_parameters_shrink_to_fit(const csm_search_parameters* sp,
                                        const int32_t* discrete_xy, int32_t points_per_scan,
                                        int32_t num_x_cells, int32_t num_y_cells,
                                        csm_linear_bounds* bounds) {
  if (!ValidSp(sp) || !bounds || points_per_scan < 0 || (points_per_scan > 0 && !discrete_xy))
    return CSM_EINVAL;
  for (int32_t s = 0; s < sp->num_scans; ++s) {
    // min_bound / max_bound start at zero (.cc:74-75).
    int min_x = 0, min_y = 0, max_x = 0, max_y = 0;
    const int32_t* d = discrete_xy + 2 * static_cast<int64_t>(s) * points_per_scan;
    for (int32_t i = 0; i < points_per_scan; ++i) {
      min_x = std::min(min_x, -d[2 * i]);
      min_y = std::min(min_y, -d[2 * i + 1]);
      max_x = std::max(max_x, num_x_cells - 1 - d[2 * i]);
      max_y = std::max(max_y, num_y_cells - 1 - d[2 * i + 1]);
    }
    csm_linear_bounds& b = bounds[s];
    b.min_x = std::max(b.min_x, min_x);
    b.max_x = std::min(b.max_x, max_x);
    b.min_y = std::max(b.min_y, min_y);
    b.max_y = std::min(b.max_y, max_y);
  }
  return CSM_OK;
}

int csm_generate_rotated_scans(const float* points_xyz, int32_t n,
                               const csm_search_parameters* sp, float* out_xyz) {
  if (!ValidSp(sp) || n < 0 || (n > 0 && (!points_xyz || !out_xyz))) return CSM_EINVAL;
  csm::SearchWindow2D w;
  w.num_angular_perturbations = sp->num_angular_perturbations;
  w.angular_perturbation_step_size = sp->angular_perturbation_step_size;
  w.num_scans = sp->num_scans;
  std::vector<csm::ZRot> table;
  csm::RotationTable(w, &table);
  for (int32_t s = 0; s < sp->num_scans; ++s) {
    float* o = out_xyz + 3 * static_cast<int64_t>(s) * n;
    for (int32_t i = 0; i < n; ++i) {
      // Rigid3f::Rotation(AngleAxisf(theta, UnitZ)) * p: z is unchanged.
      csm::RotateZ(table[s], points_xyz[3 * i], points_xyz[3 * i + 1], &o[3 * i], &o[3 * i + 1]);
      o[3 * i + 2] = points_xyz[3 * i + 2];
    }
  }
  return CSM_OK;
}

int csm_discretize_scans(const csm_map_limits* limits, const float* rotated_xyz, int32_t n,
                         int32_t num_scans, float initial_x, float initial_y, int32_t* out_xy) {
  if (!limits || !(limits->resolution > 0.) || n < 0 || num_scans < 0 ||
      (n > 0 && num_scans > 0 && (!rotated_xyz || !out_xy)))
    return CSM_EINVAL;
  const int64_t total = static_cast<int64_t>(num_scans) * n;
  for (int64_t k = 0; k < total; ++k) {
    // Affine2f(translation) * p in float, then GetCellIndex (map_limits.h:69-75).
    const float px = initial_x + rotated_xyz[3 * k];
    const float py = initial_y + rotated_xyz[3 * k + 1];
    const double cx = std::round((limits->max_y - static_cast<double>(py)) / limits->resolution - 0.5);
    const double cy = std::round((limits->max_x - static_cast<double>(px)) / limits->resolution - 0.5);
    if (!(std::fabs(cx) < 2147483647.) || !(std::fabs(cy) < 2147483647.)) return CSM_ERANGE;
    out_xy[2 * k] = static_cast<int32_t>(cx);
    out_xy[2 * k + 1] = static_cast<int32_t>(cy);
  }
  return CSM_OK;
}

}  // extern "C"
