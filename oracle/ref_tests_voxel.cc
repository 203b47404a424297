// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// sensor/internal/voxel_filter_test.cc restated against the oracle with the
// reference's inputs and checks.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "oracle_voxel.h"

using namespace oracle;

namespace {

int g_fail = 0, g_checks = 0;
const char* g_name = "";
#define CHECKV(cond)                                                                \
  do {                                                                              \
    ++g_checks;                                                                     \
    if (!(cond)) {                                                                  \
      ++g_fail;                                                                     \
      std::fprintf(stderr, "[%s] FAILED %s:%d: %s\n", g_name, __FILE__, __LINE__, #cond); \
    }                                                                               \
  } while (0)

bool Same(const Vec3f& a, const Vec3f& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }
bool Contains(const std::vector<Vec3f>& v, const Vec3f& p) {
  return std::any_of(v.begin(), v.end(), [&](const Vec3f& q) { return Same(p, q); });
}

// voxel_filter_test.cc:30-41 ReturnsOnePointInEachVoxel
void ReturnsOnePointInEachVoxel() {
  g_name = "VoxelFilterTest.ReturnsOnePointInEachVoxel";
  const std::vector<Vec3f> cloud{{0.f, 0.f, 0.f}, {0.1f, -0.1f, 0.1f}, {0.3f, -0.1f, 0.f},
                                 {0.f, 0.f, 0.1f}};
  const std::vector<Vec3f> result = VoxelFilter(cloud, 0.3f);
  CHECKV(result.size() == 2);
  if (result.size() != 2) return;
  CHECKV(Contains(cloud, result[0]));
  CHECKV(Contains(cloud, result[1]));
  CHECKV(Contains(result, cloud[2]));
}

// voxel_filter_test.cc:43-62 CorrectIntensities: the kept intensities are
// those of the kept points (the kept index drives both).
void CorrectIntensities() {
  g_name = "VoxelFilterTest.CorrectIntensities";
  std::vector<Vec3f> cloud;
  std::vector<float> intensities;
  for (int i = 0; i < 100; ++i) {
    const float value = 0.1f * i;
    cloud.push_back({-100.f, 0.3f, value});
    intensities.push_back(value);
  }
  std::vector<int> kept;
  const std::vector<Vec3f> result = VoxelFilter(cloud, 0.3f, &kept);
  CHECKV(kept.size() == result.size());
  for (size_t i = 0; i < result.size(); ++i)
    CHECKV(std::abs(result[i].z - intensities[kept[i]]) <= 1e-6);
}

// voxel_filter_test.cc:64-74 HandlesLargeCoordinates
void HandlesLargeCoordinates() {
  g_name = "VoxelFilterTest.HandlesLargeCoordinates";
  const std::vector<Vec3f> cloud{{100000.f, 0.f, 0.f},
                                 {100000.001f, -0.0001f, 0.0001f},
                                 {100000.003f, -0.0001f, 0.f},
                                 {-200000.f, 0.f, 0.f}};
  const std::vector<Vec3f> result = VoxelFilter(cloud, 0.01f);
  CHECKV(result.size() == 2);
  CHECKV(Contains(result, cloud[3]));
}

// voxel_filter_test.cc:76-84 IgnoresTime (the time field does not enter the key)
void IgnoresTime() {
  g_name = "VoxelFilterTest.IgnoresTime";
  std::vector<Vec3f> cloud(100, Vec3f{-100.f, 0.3f, 0.4f});
  const std::vector<Vec3f> result = VoxelFilter(cloud, 0.3f);
  CHECKV(result.size() == 1);
  if (!result.empty()) CHECKV(Contains(cloud, result[0]));
}

}  // namespace

int RunRefTestsVoxel(int* checks) {
  ReturnsOnePointInEachVoxel();
  CorrectIntensities();
  HandlesLargeCoordinates();
  IgnoresTime();
  std::printf("%-70s %s\n", "VoxelFilterTest (4 cases)", g_fail == 0 ? "OK" : "FAILED");
  *checks = g_checks;
  return g_fail;
}
