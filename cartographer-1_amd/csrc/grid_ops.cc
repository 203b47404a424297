// Submap grid formats on the host side of the boundary: Submap2D::Finish's
// crop (submap_2d.cc:146-150 -> ProbabilityGrid::ComputeCroppedGrid,
// probability_grid.cc:91-106, Grid2D::ComputeCroppedLimits, grid_2d.cc:110-120).
//
// The crop is a bounding box and a copy, done once per finished submap before
// csm_fast2d_create uploads the cells, so it stays on the host. A grid that
// crosses the boundary carries no known_cells_box; every update the inserter
// makes leaves a nonzero value (kUnknownCorrespondenceValue is 0 and the
// update tables never produce it), so the box is the bounding box of the
// nonzero cells. ComputeCroppedGrid copies each known cell through
// SetProbability(GetProbability(v)); that float round trip returns every value
// 1..32767 unchanged (tests/test_grid_ops.py checks all of them against the
// oracle), so the copy is exact.
#include <cstdint>
#include <cstring>

#include "../../include/csm_amd.h"

extern "C" {

int csm_grid2d_cropped_limits(const csm_map_limits* limits, const uint16_t* cells,
                              int32_t* offset_xy, csm_map_limits* cropped) {
  if (!limits || !cropped || !offset_xy) return CSM_EINVAL;
  const int nx = limits->num_x_cells, ny = limits->num_y_cells;
  if (nx < 0 || ny < 0 || (nx > 0 && ny > 0 && !cells)) return CSM_EINVAL;
  int min_x = nx, min_y = ny, max_x = -1, max_y = -1;
  for (int y = 0; y < ny; ++y) {
    const uint16_t* row = cells + static_cast<int64_t>(y) * nx;
    int first = -1, last = -1;
    for (int x = 0; x < nx; ++x)
      if (row[x] != 0) {
        if (first < 0) first = x;
        last = x;
      }
    if (first < 0) continue;
    min_x = first < min_x ? first : min_x;
    max_x = last > max_x ? last : max_x;
    min_y = y < min_y ? y : min_y;
    max_y = y;
  }
  *cropped = *limits;
  if (max_x < 0) {  // known_cells_box_.isEmpty(): offset 0, CellLimits(1, 1)
    offset_xy[0] = offset_xy[1] = 0;
    cropped->num_x_cells = cropped->num_y_cells = 1;
    return CSM_OK;
  }
  offset_xy[0] = min_x;
  offset_xy[1] = min_y;
  cropped->num_x_cells = max_x - min_x + 1;
  cropped->num_y_cells = max_y - min_y + 1;
  // max = limits().max() - resolution * Vector2d(offset.y(), offset.x())
  cropped->max_x = limits->max_x - limits->resolution * static_cast<double>(min_y);
  cropped->max_y = limits->max_y - limits->resolution * static_cast<double>(min_x);
  return CSM_OK;
}

int csm_grid2d_crop(const csm_map_limits* limits, const uint16_t* cells,
                    csm_map_limits* cropped, uint16_t* cropped_cells, int64_t capacity) {
  int32_t off[2];
  const int rc = csm_grid2d_cropped_limits(limits, cells, off, cropped);
  if (rc != CSM_OK) return rc;
  const int64_t cnx = cropped->num_x_cells, cny = cropped->num_y_cells;
  if (!cropped_cells || capacity < cnx * cny) return CSM_EINVAL;
  bool any = false;  // an empty known box crops to one unknown cell
  const int64_t n = static_cast<int64_t>(limits->num_x_cells) * limits->num_y_cells;
  for (int64_t i = 0; i < n && !any; ++i) any = cells[i] != 0;
  if (!any) {
    cropped_cells[0] = 0;
    return CSM_OK;
  }
  // SetProbability(GetProbability(v)) keeps every value; the update marker
  // (bit 15) is not part of a value (the conversion table masks it).
  for (int64_t y = 0; y < cny; ++y)
    for (int64_t x = 0; x < cnx; ++x)
      cropped_cells[y * cnx + x] =
          cells[(y + off[1]) * limits->num_x_cells + (x + off[0])] & 0x7fff;
  return CSM_OK;
}

}  // extern "C"
