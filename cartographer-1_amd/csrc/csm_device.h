// Structures shared between the host runtime and the gfx950 kernels.
#ifndef CSM_DEVICE_H_
#define CSM_DEVICE_H_

#include <cstdint>

#if defined(__HIPCC__)
#define CSM_HD __host__ __device__
#else
#define CSM_HD
#endif

namespace csm {

constexpr int kMaxLevels = 12;
constexpr int kNumXcd = 8;           // MI355X: 8 XCDs, 32 CUs each
constexpr int kSearchThreads = 256;  // 4 waves per workgroup
constexpr int kWaves = kSearchThreads / 64;
constexpr int kStackCap = 160;       // per-wave DFS stack entries
constexpr int kTopChunk = 64;        // top-level candidates per DFS chunk
constexpr int kMaxPoints = 16448;    // 22-bit sum field: 16448 * 255 < 2^22
constexpr int kIndexLimit = 16383;   // |discretized cell index| bound
constexpr int kOffsetLimit = 8191;   // |candidate offset| bound (14-bit field)
constexpr int kMaxRotations = 16383; // 14-bit field
constexpr int16_t kSentinel = -32768;

// Device pyramid of one submap (PrecomputationGridStack2D): level d is a
// (nx + 2^d - 1) x (ny + 2^d - 1) uint8 wide grid, x fastest, followed by one
// zero byte used as the target of out-of-grid lookups.
struct SubmapDesc {
  double max_x, max_y, resolution;
  int32_t nx, ny;
  int32_t levels;       // search pyramid depth
  int32_t pad0;
  const uint8_t* level[kMaxLevels];
  int32_t wide_nx[kMaxLevels];
  int32_t wide_ny[kMaxLevels];
  int32_t zero_index[kMaxLevels];  // index of the trailing zero byte
  // Quad layout of level d (h = 2^d, search kernel v4): dword (X', Y'),
  // X' < quad_w = wide_nx + h, Y' < quad_h = wide_ny + h, packs the values
  // of the 2x2 children whose child (0,0) is at wide cell (X' - h, Y' - h):
  // byte0 (0,0), byte1 (0,h), byte2 (h,0), byte3 (h,h); 0 outside the grid.
  const uint32_t* quad[kMaxLevels];
  const uint8_t* pyramid_base;      // one allocation: row-major + quad levels
  int32_t pyramid_bytes;
  int32_t quad_off[kMaxLevels];     // byte offset of quad level d from the base
  int32_t quad_pws[kMaxLevels];     // polyphase plane row stride (dwords)
  int32_t quad_pph[kMaxLevels];     // polyphase plane rows
  int32_t quad_w[kMaxLevels];
  int32_t quad_h[kMaxLevels];
  int32_t quad_bytes[kMaxLevels];
  // Scan clustering per child level (DESIGN.md §5 "Clustered entries"):
  // quad level d holds M_d(c) = max of level 0 over [c, c + 2^d + k - 1)
  // per axis, k = 2^cshift[d], so one entry per occupied k x k cluster of
  // scan cells (weighted by its point count) bounds every point in it.
  // k = 1 at level 0 (exact leaf scores). Quad index X' = cell + offset +
  // quad_bias[d], quad_bias = (2^d - 1) + (k - 1) + 2^d.
  int32_t cshift[kMaxLevels];
  int32_t quad_bias[kMaxLevels];
  // Plane kind per level: entry bytes 4 = quad (above), 16 = hex, 0 = none.
  // Hex layout (search kernel v5): a node of a level L >= 2 in hex_mask
  // scores its 16 grandchildren at level c = L - 2, offsets (a h, b h),
  // a, b in 0..3, h = 2^c, from ONE 16-byte entry: dword a, byte b =
  // M_c(X + a h, Y + b h), X' = cell + offset + quad_bias[c] with quad_bias =
  // (h - 1) + (k - 1) + 3h, polyphase with period P = 4h (the lattice nodes of
  // level c + 2 sit on). Only the levels the node chain reaches get a plane
  // (virtual roots at levels: quad into levels - 1; then L -> L - 2 for hex
  // levels, L -> L - 1 otherwise).
  int32_t quad_es[kMaxLevels];
  int32_t hex_mask;  // bit L: nodes of level L expand two levels at once (0: v4)
};

constexpr int kMaxClusterShift = 3;  // clusters of 1, 2, 4, 8 cells per side

constexpr int kHexEntryBytes = 16;  // one hex entry: 16 uint8 grandchild values

// One (node, submap) search.
struct PairDesc {
  int32_t submap;
  int32_t num_points;
  int64_t point_offset;     // into the scan set's packed xyz floats (points)
  int32_t rot_offset;       // into the rotation table (w, s pairs)
  int32_t num_scans;
  int32_t num_linear;       // linear window in cells before ShrinkToFit
  int32_t max_rejected_sum; // prune / reject sums <= this value
  float tx, ty;             // initial translation, narrowed to float
  float pre_w, pre_s;       // initial rotation quaternion (z axis)
  int32_t collect;          // 1: tie enumeration, record every leaf with sum collect_sum
  int32_t collect_sum;
};

// Tie resolution (csm_host.cc ResolveTies): one workgroup per (pair,
// rotation) scores `count` queries (level, x_off, y_off) at queries[first..].
struct ScoreJob {
  int32_t pair, rot, first, count;
};
constexpr int kTieCap = 4096;  // tied leaves recorded per pair

// Ordered walk (csm_host.cc ResolveTies, pairs with more tied leaves than the
// collect pass records): one workgroup per job follows the reference's
// visiting order from the sorted lowest-resolution list down to the first
// leaf at the maximum (fast_correlative_scan_matcher_2d.cc:335-378).
struct WalkJob2 {
  int32_t pair;          // into the collect launch's pair descriptors
  int32_t target_sum;    // the pair's maximum leaf sum
  int32_t top_level;     // branch_and_bound_depth - 1
  int32_t top_first;     // sorted lowest-resolution entries (rot, x, y, sum), sum >= target
  int32_t top_count;
  int32_t bounds_first;  // ShrinkToFit bounds of rotation r at bounds_first + r
  float min_s, max_s;    // the submap's score range (SumToScore)
};
constexpr int kWalkStack = 64;  // 1 + 3 x depth entries at most

// Per-XCD work queues over rotation chunks of pairs.
struct WorkQueues {
  const int32_t* pair_order;      // pairs, grouped by queue
  const int64_t* chunk_prefix;    // per entry of pair_order: first chunk id
  int32_t queue_begin[kNumXcd + 1];
  int64_t queue_chunks[kNumXcd];  // chunks per queue
  int32_t rot_chunk;              // rotations per chunk
};

// v2 work queues: chunks of `rot_chunk` rotations of a pair; a chunk id
// decodes to its pair in O(1) through a per-64-chunk block table.
struct WorkQueues2 {
  const int32_t* pair_order;    // pairs, grouped by queue
  const int64_t* chunk_prefix;  // size |pair_order|+1, cumulative chunks
  const int32_t* block_first;   // per queue block of 64 chunks: pair_order index
  int32_t block_offset[kNumXcd];
  int32_t queue_begin[kNumXcd + 1];
  int64_t queue_chunks[kNumXcd];
  int32_t rot_chunk;
};

// Rotations per v4/v5 search item at most (per-rotation LDS tables are sized
// for it; the host clamps CSM_ROT_CHUNK to it).
#ifndef CSM_MAX_ROT_CHUNK
#define CSM_MAX_ROT_CHUNK 16
#endif
constexpr int kV4MaxRotChunk = CSM_MAX_ROT_CHUNK;

constexpr int kStack2 = 1024;   // v4 per-workgroup DFS stack entries in LDS
constexpr int kSpill2 = 7168;   // further entries per workgroup in global memory
constexpr int kBatchNodes = 64; // nodes expanded per batch (256 children; hex: 1024)

// Best leaf per pair, packed for a 64-bit atomicMax:
//   [63:42] level-0 integer sum (22 bits)
//   [41:0]  ~(rotation << 28 | (x_off + 8192) << 14 | (y_off + 8192))
// so the max key is the max sum, ties to the smallest (rotation, x, y).
constexpr int kSumShift = 42;
constexpr uint64_t kTieMask = (uint64_t(1) << kSumShift) - 1;

CSM_HD inline uint64_t PackLeafKey(uint32_t sum, int rot, int xo, int yo) {
  const uint64_t idx = (uint64_t(rot) << 28) | (uint64_t(xo + 8192) << 14) |
                       uint64_t(yo + 8192);
  return (uint64_t(sum) << kSumShift) | (~idx & kTieMask);
}
// The same leaf as (sum, index) with the index NOT inverted: the per-pair
// atomicMax of these keeps the tied maximum with the largest index, so a pair
// has more than one maximal leaf iff its two keys differ.
CSM_HD inline uint64_t HighLeafKey(uint64_t key) {
  return (key & ~kTieMask) | (~key & kTieMask);
}
CSM_HD inline void UnpackLeafKey(uint64_t key, uint32_t* sum, int* rot, int* xo, int* yo) {
  *sum = static_cast<uint32_t>(key >> kSumShift);
  const uint64_t idx = ~key & kTieMask;
  *rot = static_cast<int>(idx >> 28);
  *xo = static_cast<int>((idx >> 14) & 0x3fff) - 8192;
  *yo = static_cast<int>(idx & 0x3fff) - 8192;
}

// Search statistics words (csm_host.cc reads them back): [0] candidates,
// [1] lookups, [2, 2 + L) candidates per child level, [2 + L, 2 + 2L)
// batches per level, 4 CSM_KPROF phase counters, the DFS stack high-water
// mark (max over workgroups, entries).
constexpr int kStatHighWater = 2 + 2 * kMaxLevels + 4;
// CSM_KPROF builds: distinct 128-byte lines, gather instructions and quad
// lines (distinct lines summed over the 4-lane groups) per child level (the
// texture path's cost model).
constexpr int kStatLines = kStatHighWater + 1;
constexpr int kStatsWords = kStatLines + 5 * kMaxLevels;  // + active and out-of-range lanes

// Per-pair status written by the search kernel (0 = ok).
constexpr int32_t kStatusRange = 1;

}  // namespace csm

#endif  // CSM_DEVICE_H_
