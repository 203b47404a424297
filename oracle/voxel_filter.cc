// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h). Never linked into
// libcsm_amd.so; used by tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg as the checker for csm_voxel_filter / csm_adaptive_voxel_filter.
//
// Restates sensor/internal/voxel_filter.cc (the reference fork's version):
//   GetVoxelCellIndex                      :79-86
//   RandomizedVoxelFilterIndices           :136-162
//   VoxelFilter(const PointCloud&, float)  :212-232 (and the overloads :205-251)
//   FilterByMaxRange                       :31-36
//   AdaptivelyVoxelFiltered                :38-76
//   AdaptiveVoxelFilter                    :263-268
//
// The reservoir sampling draws come from a fresh std::minstd_rand0 (seed 1)
// per VoxelFilter call and std::uniform_int_distribution<>(1, count), both
// from libstdc++ exactly as the reference uses them. Which point a voxel keeps
// depends only on the draws, consumed in point order; the map's iteration
// order (absl::flat_hash_map in the reference) only decides the order in which
// points_used is set, not its contents, so std::unordered_map is equivalent.
#include <cmath>
#include <cstdint>
#include <random>
#include <unordered_map>
#include <utility>
#include <vector>

#include "oracle_voxel.h"

namespace oracle {

uint64_t GetVoxelCellIndex(float px, float py, float pz, float resolution) {
  // point.array() / resolution: one IEEE float division per coordinate, then
  // common::RoundToInt (std::lround, narrowed to int) and a sign-extending
  // conversion to uint64_t.
  const float ix = px / resolution, iy = py / resolution, iz = pz / resolution;
  const uint64_t x = static_cast<uint64_t>(static_cast<int64_t>(static_cast<int>(std::lround(ix))));
  const uint64_t y = static_cast<uint64_t>(static_cast<int64_t>(static_cast<int>(std::lround(iy))));
  const uint64_t z = static_cast<uint64_t>(static_cast<int64_t>(static_cast<int>(std::lround(iz))));
  return (x << 42) + (y << 21) + z;
}

std::vector<bool> RandomizedVoxelFilterIndices(const std::vector<Vec3f>& cloud, float resolution) {
  std::minstd_rand0 generator;
  std::unordered_map<uint64_t, std::pair<int, int>> voxel_count_and_point_index;
  for (size_t i = 0; i < cloud.size(); i++) {
    auto& voxel = voxel_count_and_point_index[GetVoxelCellIndex(cloud[i].x, cloud[i].y, cloud[i].z,
                                                                resolution)];
    voxel.first++;
    if (voxel.first == 1) {
      voxel.second = static_cast<int>(i);
    } else {
      std::uniform_int_distribution<> distribution(1, voxel.first);
      if (distribution(generator) == voxel.first) voxel.second = static_cast<int>(i);
    }
  }
  std::vector<bool> points_used(cloud.size(), false);
  for (const auto& voxel_and_index : voxel_count_and_point_index)
    points_used[voxel_and_index.second.second] = true;
  return points_used;
}

std::vector<Vec3f> VoxelFilter(const std::vector<Vec3f>& cloud, float resolution,
                               std::vector<int>* kept_index) {
  const std::vector<bool> used = RandomizedVoxelFilterIndices(cloud, resolution);
  std::vector<Vec3f> out;
  if (kept_index) kept_index->clear();
  for (size_t i = 0; i < cloud.size(); ++i)
    if (used[i]) {
      out.push_back(cloud[i]);
      if (kept_index) kept_index->push_back(static_cast<int>(i));
    }
  return out;
}

// Vector3f::norm(): Eigen's unrolled 3-element sum is x0 + (x1 + x2).
static float Norm3f(const Vec3f& p) { return std::sqrt(p.x * p.x + (p.y * p.y + p.z * p.z)); }

std::vector<int> AdaptiveVoxelFilterIndices(const std::vector<Vec3f>& cloud,
                                            const AdaptiveVoxelFilterOptions& options) {
  // FilterByMaxRange (:31-36): copy_if keeps the original order.
  std::vector<Vec3f> ranged;
  std::vector<int> ranged_index;
  for (size_t i = 0; i < cloud.size(); ++i)
    if (Norm3f(cloud[i]) <= options.max_range) {
      ranged.push_back(cloud[i]);
      ranged_index.push_back(static_cast<int>(i));
    }
  auto lift = [&](const std::vector<int>& local) {
    std::vector<int> out;
    out.reserve(local.size());
    for (int k : local) out.push_back(ranged_index[k]);
    return out;
  };
  // AdaptivelyVoxelFiltered (:38-76). min_num_points is a float proto field,
  // so every size comparison is done in float.
  if (static_cast<float>(ranged.size()) <= options.min_num_points) return ranged_index;
  std::vector<int> result;
  VoxelFilter(ranged, options.max_length, &result);
  if (static_cast<float>(result.size()) >= options.min_num_points) return lift(result);
  for (float high_length = options.max_length; high_length > 1e-2f * options.max_length;
       high_length /= 2.f) {
    float low_length = high_length / 2.f;
    VoxelFilter(ranged, low_length, &result);
    if (static_cast<float>(result.size()) >= options.min_num_points) {
      while ((high_length - low_length) / low_length > 1e-1f) {
        const float mid_length = (low_length + high_length) / 2.f;
        std::vector<int> candidate;
        VoxelFilter(ranged, mid_length, &candidate);
        if (static_cast<float>(candidate.size()) >= options.min_num_points) {
          low_length = mid_length;
          result = candidate;
        } else {
          high_length = mid_length;
        }
      }
      return lift(result);
    }
  }
  return lift(result);
}

}  // namespace oracle

using namespace oracle;

extern "C" {

// keep[i] = 1 when point i of cloud c survives VoxelFilter(cloud c, resolution).
// Clouds are consecutive in xyz, cloud c = [offsets[c], offsets[c+1]).
// Returns the total number of kept points.
int64_t oracle_voxel_filter(const float* xyz, const int64_t* offsets, int32_t num_clouds,
                            float resolution, uint8_t* keep) {
  int64_t total = 0;
  for (int32_t c = 0; c < num_clouds; ++c) {
    std::vector<Vec3f> cloud;
    for (int64_t i = offsets[c]; i < offsets[c + 1]; ++i)
      cloud.push_back(Vec3f{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]});
    const std::vector<bool> used = RandomizedVoxelFilterIndices(cloud, resolution);
    for (size_t i = 0; i < used.size(); ++i) {
      keep[offsets[c] + static_cast<int64_t>(i)] = used[i] ? 1 : 0;
      total += used[i];
    }
  }
  return total;
}

// AdaptiveVoxelFilter(cloud c, {max_length, min_num_points, max_range}).
int64_t oracle_adaptive_voxel_filter(const float* xyz, const int64_t* offsets, int32_t num_clouds,
                                     float max_length, float min_num_points, float max_range,
                                     uint8_t* keep) {
  const AdaptiveVoxelFilterOptions o{max_length, min_num_points, max_range};
  int64_t total = 0;
  for (int32_t c = 0; c < num_clouds; ++c) {
    std::vector<Vec3f> cloud;
    for (int64_t i = offsets[c]; i < offsets[c + 1]; ++i) {
      cloud.push_back(Vec3f{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]});
      keep[i] = 0;
    }
    for (int k : AdaptiveVoxelFilterIndices(cloud, o)) {
      keep[offsets[c] + k] = 1;
      ++total;
    }
  }
  return total;
}

}  // extern "C"
