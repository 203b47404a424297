// Device-side data layout of the 3D path (HybridGrid bricks, FastCSM3D
// pyramid levels, per-pair / per-yaw work descriptors). Shared by
// kernels3d.hip and host3d.cc.
#ifndef CSM_DEVICE3D_H_
#define CSM_DEVICE3D_H_

#include <cstdint>

namespace csm {

constexpr int kMaxLevels3d = 12;
constexpr int kExtraLevels3d = 2;       // coarser levels above the reference's stack (roots only)
constexpr int kRootTarget3d = 64;        // a pair's roots start at the lowest level with <= this many
constexpr int kTiny3dPoints = 512;       // cloud capacity (LDS) of the tiny-cloud build (24 KiB, 5 per CU)
constexpr int kSmall3dPoints = 2048;      // cloud capacity (LDS) of the 4-workgroups-per-CU build
constexpr int kMax3dPoints = 8192;        // of the large-cloud build (2 per CU); more: CSM_ERANGE
constexpr int kTopLds3d = 6 * 1024;       // top pyramid level cached in LDS when it fits
constexpr int kRootChunk3d = 128;         // roots fed to the DFS stack at a time
constexpr int kRootScore3d = 256;         // roots scored at a time (one per lane)
constexpr int kTopCells3d = 512;          // distinct top-level cells of a cloud (LDS list)
constexpr int kBatch3d = 16;              // DFS nodes scored per step (16 lanes each; small, large builds)
constexpr int kTinyBatch3d = 32;          // of the tiny-cloud build (8 lanes each)
constexpr int kMax3dTop = 1 << 20;        // top-level candidates per yaw
constexpr int kTieCap3d = 4096;           // tied leaves recorded per pair (collect search)
constexpr int kWalkStack3d = 128;         // ordered-walk stack: 1 + 7 x depth entries at most
constexpr int kStack3d = 1024;            // DFS stack entries per workgroup in LDS (small, large builds)
constexpr int kTinyStack3d = 512;        // of the tiny-cloud build
constexpr int kDfsCap3d = 4096;           // DFS stack entries per workgroup, LDS + global spill
constexpr int kStat3dHighWater = 14;      // stats word: DFS stack high-water (max over workgroups)
constexpr int kMax3dYaws = 1 << 16;
constexpr int kMax3dWindow = 1 << 14;
constexpr int kSearch3dThreads = 256;
constexpr int kSearch3dBlocksPerCuTiny = 5;   // resident workgroups per CU, tiny-cloud build
constexpr int kSearch3dBlocksPerCu = 4;       // small-cloud build
constexpr int kSearch3dBlocksPerCuLarge = 2;  // large-cloud build
// Octet loads a lane of the tiny build keeps in flight: 8 fit its 96 VGPRs
// (16 spill 13); the small and large builds keep 16.
constexpr int kTinyInflight3d = 8;
// Search builds by cloud size: 0 tiny, 1 small, 2 large.
constexpr int kSearch3dTiers = 3;
constexpr int Search3dTier(int num_points) {
  return num_points <= kTiny3dPoints ? 0 : num_points <= kSmall3dPoints ? 1 : 2;
}
constexpr int kSearch3dBlocksPerCuMax = kSearch3dBlocksPerCuTiny > kSearch3dBlocksPerCu
                                            ? kSearch3dBlocksPerCuTiny : kSearch3dBlocksPerCu;
constexpr int kCellLimit3d = 16000;       // |cell index| kept in int16 in LDS
// Per pair: key = sum << key_shift | ~leaf_id, leaf_id = ((yaw << bxy | x) << bxy
// | y) << bz | z with x = ox + wxy etc.; the host sizes the fields so that
// sum and id fit 64 bits (else CSM_ERANGE).

// A dense brick over the bounding box of a sparse grid's known cells:
// value(i) = data[((i.z - oz) * ny + (i.y - oy)) * nx + (i.x - ox)], and the
// grid's default outside the box.
struct Brick3 {
  int32_t ox, oy, oz;
  int32_t nx, ny, nz;
  int64_t offset;  // byte offset of this brick in its allocation
};

// One HybridGrid of a batched grid build (csm_hybrid_grid_create_batch): its
// cell list (device), the dense value brick it is scattered into and the
// float probability brick made from it (n cells each).
struct GridJob3 {
  const int32_t* ijk;
  const uint16_t* vals;
  int64_t count;
  Brick3 b;
  uint16_t* values;
  float* prob;
  int64_t n;
};

// One output brick of a batched pyramid build (csm_fast3d_create_batch):
// source brick -> output brick, as level_gather (shift h, half) or
// octet_build (h) do it. `lds`: the job's staged-rows bytes.
struct RowJob3 {
  const uint8_t* src;
  void* out;
  Brick3 sb, ob;
  int32_t h, lds;
};

// One level-0 conversion of a batched build (brick_from_values' qtab path).
struct ValueJob3 {
  const uint16_t* values;
  uint8_t* level0;
  int64_t n;
};

// One FastCSM3D submap (csm_fast3d): pyramid levels (uint8 bricks in one
// allocation) and the low-resolution HybridGrid (float probability brick).
struct Submap3Desc {
  const uint8_t* levels;  // base of the level allocation
  int32_t levels_bytes;   // its size (< 2^31: one buffer resource spans it)
  Brick3 level[kMaxLevels3d];
  int32_t num_levels;     // branch_and_bound_depth
  // Levels built: num_levels plus up to kExtraLevels3d coarser ones with the
  // same recurrence. A node of level L + 1 bounds its (up to) 8 children of
  // level L exactly as within the reference's stack, so rooting a search
  // there reaches the same top-level candidates (the children past the
  // window are dropped) while scoring far fewer roots.
  int32_t search_levels;
  int32_t full_resolution_depth;
  float resolution;
  // Octet layout of levels 0..num_levels-2 (the DFS child levels): one
  // uint64 per cell c packs the 8 values at c + H*(x, y, z), x, y, z in {0,1},
  // byte (z << 2 | y << 1 | x); H = 2^L below full_resolution_depth, else
  // 2^(full_resolution_depth - 1). Boxes are the level's box grown by H
  // towards -inf so that every cell with a child inside is present.
  const uint8_t* octs;
  int32_t octs_bytes;  // < 2^31 (0: octets disabled, byte path)
  Brick3 oct[kMaxLevels3d];
  int32_t oct_h[kMaxLevels3d];
  const float* low_prob;  // low-resolution grid probabilities
  Brick3 low;
  float low_resolution;
};

// One (submap, node) pair.
struct Pair3Desc {
  int32_t submap;
  int32_t num_points;       // high-resolution points
  int64_t point_offset;     // into the high-resolution point buffer (xyz)
  int32_t num_low;          // low-resolution points
  int64_t low_offset;
  int32_t yaw_begin, num_yaws;
  int32_t wxy, wz;          // linear window sizes (voxels)
  int32_t root_level;       // level the pair's roots are generated and scored at
  int32_t top_nx, top_ny, top_nz;  // roots per axis at root_level
  int32_t min_sum;          // smallest sum whose score exceeds min_score
  float min_low_resolution_score;
  int32_t key_shift, bits_xy, bits_z;  // leaf key layout
  // Tie resolution (host3d.cc ResolveTies3d): a collect search records every
  // leaf that passes the low-resolution check with sum == collect_sum.
  int32_t collect, collect_sum;
};

// Ordered walk (host3d.cc ResolveTies3d, pairs whose passing tied leaves
// overflow the collect record; kernels3d.hip fast3d_walk).
struct Walk3Job {
  int32_t pair;        // device pair index
  int32_t target_sum;  // the pair's best passing leaf sum
  int32_t top_level;   // max_depth
  int32_t top_first;   // sorted lowest-resolution entries (yaw, x | y << 16, z, sum), sum >= target
  int32_t top_count;
  int32_t pad[3];
};

// One discrete scan (yaw) of a pair: the pose the cloud is discretized with,
// the normalized rotation of leaf poses (GetPoseFromCandidate), and its
// rotational score.
struct Yaw3Desc {
  float qw, qx, qy, qz;     // DiscreteScan3D::pose rotation (not normalized)
  float nw, nx, ny, nz;     // normalized (identity * q).normalized()
  float tx, ty, tz;
  float rotational_score;
  int32_t pair;
  int32_t yaw_id;           // index among the pair's discrete scans
};

}  // namespace csm

#endif  // CSM_DEVICE3D_H_
