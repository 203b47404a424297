// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
// HybridGrid updates, the 3D range-data inserter and PrecomputationGrid3D.
#include <algorithm>
#include <cstdlib>

#include "oracle3d.h"

namespace oracle {

// hybrid_grid.h:497-521
bool HybridGrid::ApplyLookupTable(const Idx3& i, const std::vector<uint16_t>& table) {
  uint16_t* const cell = mutable_value(i);
  if (*cell >= kUpdateMarker) return false;
  update_indices_.push_back(cell);
  *cell = table[*cell];
  return true;
}

void HybridGrid::FinishUpdate() {
  while (!update_indices_.empty()) {
    *update_indices_.back() -= kUpdateMarker;
    update_indices_.pop_back();
  }
}

// range_data_inserter_3d.cc:100-108
RangeDataInserter3D::RangeDataInserter3D(float hit_probability, float miss_probability,
                                         int num_free_space_voxels)
    : num_free_space_voxels_(num_free_space_voxels),
      hit_table_(LookupTableToApplyOdds(Odds(hit_probability))),
      miss_table_(LookupTableToApplyOdds(Odds(miss_probability))) {}

// range_data_inserter_3d.cc:110-136 and InsertMissesIntoGrid :44-74.
void RangeDataInserter3D::Insert(const Vec3f& origin, const PointCloud& returns,
                                 HybridGrid* grid) const {
  for (const Vec3f& hit : returns) grid->ApplyLookupTable(grid->GetCellIndex(hit), hit_table_);
  const Idx3 o = grid->GetCellIndex(origin);
  for (const Vec3f& hit : returns) {
    const Idx3 h = grid->GetCellIndex(hit);
    const Idx3 d{h.x - o.x, h.y - o.y, h.z - o.z};
    const int num_samples = std::max(std::abs(d.x), std::max(std::abs(d.y), std::abs(d.z)));
    for (int position = std::max(0, num_samples - num_free_space_voxels_);
         position < num_samples; ++position) {
      // Eigen Array3i: delta * position / num_samples, C++ integer division.
      const Idx3 miss{o.x + d.x * position / num_samples, o.y + d.y * position / num_samples,
                      o.z + d.z * position / num_samples};
      grid->ApplyLookupTable(miss, miss_table_);
    }
  }
  grid->FinishUpdate();
}

// precomputation_grid_3d.cc:49-61
std::unique_ptr<PrecomputationGrid3D> ConvertToPrecomputationGrid(const HybridGrid& grid) {
  std::unique_ptr<PrecomputationGrid3D> result(new PrecomputationGrid3D(grid.resolution()));
  const std::vector<float>& table = ValueToProbabilityTable();
  grid.ForEach([&](const Idx3& index, uint16_t value) {
    const int cell_value = RoundToIntF((table[value] - kMinProbability) *
                                       (255.f / (kMaxProbability - kMinProbability)));
    *result->mutable_value(index) = static_cast<uint8_t>(cell_value);
  });
  return result;
}

// precomputation_grid_3d.cc:63-81 (>> 1 rounds toward -inf, :34-36).
std::unique_ptr<PrecomputationGrid3D> PrecomputeGrid(const PrecomputationGrid3D& grid,
                                                     bool half_resolution, const Idx3& shift) {
  std::unique_ptr<PrecomputationGrid3D> result(new PrecomputationGrid3D(grid.resolution()));
  grid.ForEach([&](const Idx3& index, uint8_t value) {
    for (int i = 0; i != 8; ++i) {
      const Idx3 o{(i & 1) ? 1 : 0, (i & 2) ? 1 : 0, (i & 4) ? 1 : 0};  // GetOctant
      Idx3 c{index.x - shift.x * o.x, index.y - shift.y * o.y, index.z - shift.z * o.z};
      if (half_resolution) c = Idx3{c.x >> 1, c.y >> 1, c.z >> 1};
      uint8_t* const v = result->mutable_value(c);
      *v = std::max(value, *v);
    }
  });
  return result;
}

}  // namespace oracle
