// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
// sensor/internal/voxel_filter.{h,cc} restated (voxel_filter.cc cites inside).
#ifndef ORACLE_VOXEL_H_
#define ORACLE_VOXEL_H_

#include <cstdint>
#include <vector>

#include "csm_oracle.h"

namespace oracle {

// proto::AdaptiveVoxelFilterOptions (sensor/proto/adaptive_voxel_filter_options.proto):
// all three fields are floats.
struct AdaptiveVoxelFilterOptions {
  float max_length = 1.f;
  float min_num_points = 2.f;
  float max_range = 3.f;
};

uint64_t GetVoxelCellIndex(float px, float py, float pz, float resolution);
std::vector<bool> RandomizedVoxelFilterIndices(const std::vector<Vec3f>& cloud, float resolution);
// The kept points in order; kept_index (optional) receives their indices.
std::vector<Vec3f> VoxelFilter(const std::vector<Vec3f>& cloud, float resolution,
                               std::vector<int>* kept_index = nullptr);
// Indices (into cloud) of AdaptiveVoxelFilter(cloud, options), in order.
std::vector<int> AdaptiveVoxelFilterIndices(const std::vector<Vec3f>& cloud,
                                            const AdaptiveVoxelFilterOptions& options);

}  // namespace oracle

#endif  // ORACLE_VOXEL_H_
