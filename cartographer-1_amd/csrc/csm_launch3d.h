// Host-callable launchers of the kernels in kernels3d.hip.
#ifndef CSM_LAUNCH3D_H_
#define CSM_LAUNCH3D_H_

#include <hip/hip_runtime.h>

#include "csm_device3d.h"

namespace csm {

constexpr int kRt3dThreads = 384;  // translations per RTCSM3D launch

// Pyramid row builds (kernels3d.hip BrickRows): bytes per staged source row
// of W positions (the dwords holding them, which may start up to 3 bytes
// early), and the dynamic LDS of a workgroup (4 source rows, 16 for a
// half-resolution level).
constexpr int BrickRowsPitch(int W) { return ((W + 3) & ~3) + 4; }
constexpr int BrickRowsLds(int nx, int h, bool half) {
  return (half ? 16 : 4) * BrickRowsPitch(half ? 2 * nx + h : nx + h);
}

hipError_t LaunchBrickFromValues(const uint16_t* values, int64_t n, const float* ptab,
                                 const uint8_t* qtab, float* prob, uint8_t* level0,
                                 hipStream_t st);
hipError_t LaunchBrickScatter(const int32_t* ijk, const uint16_t* values, int64_t count,
                              const Brick3& b, uint16_t* out, hipStream_t st);
// Batched grid builds (csm_hybrid_grid_create_batch): every job's value
// brick zeroed, its cells scattered, its probabilities made; blockIdx.y =
// job, max_n / max_count over the jobs.
hipError_t LaunchGridBuildBatch(const GridJob3* jobs, int num_jobs, int64_t max_n, int64_t max_count,
                                const float* ptab, hipStream_t st);
hipError_t LaunchLevelGather(const uint8_t* prev, const Brick3& pb, uint8_t* out, const Brick3& ob,
                             int shift, int half, hipStream_t st);
hipError_t LaunchOctetBuild(const uint8_t* level, const Brick3& lb, int h, uint64_t* out,
                            const Brick3& ob, hipStream_t st);
// Batched builds (csm_fast3d_create_batch): one launch per level for all
// jobs (device arrays); max_rows / max_lds over the jobs (lds <= 64 KiB).
hipError_t LaunchBrickRowsBatch(const RowJob3* jobs, int num_jobs, int max_rows, int max_lds,
                                bool octet, bool half, hipStream_t st);
hipError_t LaunchValuesToLevel0Batch(const ValueJob3* jobs, int num_jobs, int64_t max_n,
                                     const uint8_t* qtab, hipStream_t st);
hipError_t LaunchRt3dScore(int num_rot, hipStream_t st, const float* prob, const Brick3& gb,
                           float res, const float* points, int n, const float4* rot,
                           const float* rot_angle, const float4* trans, int num_trans, int t_base,
                           double wt, double wr, unsigned long long* best);
// rt3d_score2 over a brick padded by one 0.1 cell per side (LaunchPadProbBrick
// builds it); gb is the unpadded brick. num_trans <= kRt3dThreads.
hipError_t LaunchPadProbBrick(const float* prob, const Brick3& gb, float* out, hipStream_t st);
hipError_t LaunchRt3dScore2( int num_rot, hipStream_t st, const float* pad,
                            const Brick3& gb, float res, const float* points, int n,
                            const float4* rot, const float* rot_angle, const float4* trans,
                            int num_trans, int t_base, double wt, double wr,
                            unsigned long long* best, float* scores = nullptr,
                            int scores_pitch = 0);
// rt3d_score3 (same padded brick; byte offsets below 2^24): pre-scaled points
// and translations, eps = bound on the fast cell coordinate's error.
hipError_t LaunchRt3dScore3(int num_rot, hipStream_t st, const float* pad, const Brick3& gb,
                            float res, float eps, const float* points, int n, const float4* rot,
                            const float* rot_angle, const float4* trans, int num_trans, int t_base,
                            double wt, double wr, unsigned long long* best, float* scores,
                            int scores_pitch);
// rt3d_score4: lanes = 64 rotations of a 4 x 4 x 4 block of the angular
// lattice (rot / rot_index in block order, index -1 for holes), waves =
// translations. `pad` is the brick padded by P cells per side (LaunchPadProbBrick
// with P); points whose scaled rotation lies outside [safe_lo, safe_hi] take
// the clamped path.
constexpr int kRt4Waves = 8, kRt4Tw = 2, kRt4Tile = 32;
hipError_t LaunchPadProbBrickP(const float* prob, const Brick3& gb, int P, float* out,
                               hipStream_t st);
hipError_t LaunchRt3dScore4(int num_blocks, hipStream_t st, const float* pad, const Brick3& gb,
                            int P, float res, float eps, float4 safe_lo, float4 safe_hi,
                            const float* points, int n, const float4* rot, const int* rot_index,
                            const float* rot_angle, const float4* trans, int num_trans,
                            int num_rot, double wt, double wr, unsigned long long* best,
                            float* scores, int scores_pitch);
// rt3d_score5: v4's rotation blocks, one wave per (x, y) column of the
// translation lattice (nl = 2L + 1 in {3, 5, ..., 15} z steps), over the brick
// padded by P and stored z fastest (LaunchPadProbBrickZ). col_t0[c] = the
// scaled translation of step 0 of column c, col_thr[c] = per-axis rounding
// thresholds of the column test.
hipError_t LaunchPadProbBrickZ(const float* prob, const Brick3& gb, int P, float* out,
                               hipStream_t st);
hipError_t LaunchRt3dScore5(int nl, int num_blocks, hipStream_t st, const float* col,
                            const Brick3& gb, int P, float res, float eps, float4 safe_lo,
                            float4 safe_hi, const float* points, int n, const float4* rot,
                            const int* rot_index, const float* rot_angle, const float4* trans,
                            const float4* col_t0, const float4* col_thr, int num_rot, double wt,
                            double wr, unsigned long long* best, float* scores, int scores_pitch);
// Items [item_begin, item_begin + num_items) of the yaw list; `tier`
// (Search3dTier of the items' cloud size) selects the build.
hipError_t LaunchFast3dSearch(int tier, int grid, hipStream_t st, const Submap3Desc* submaps,
                              const Pair3Desc* pairs, const Yaw3Desc* yaws, int item_begin,
                              int num_items, const float* points, const float* low_points,
                              unsigned* counter, unsigned long long* best, int32_t* status,
                              unsigned long long* stats, int4* spill, unsigned long long* best_hi,
                              uint4* ties, int32_t* tie_count);
// Tie resolution: the reference's ScoreCandidates sum (fast_correlative_scan_
// matcher_3d.cc:332-352) of (depth, x, y, z offset) queries; one workgroup per
// job = (yaw item, queries[first, first + count)).
struct Score3Job {
  int32_t item, first, count, pad;
};
hipError_t LaunchFast3dScoreQueries(int num_jobs, hipStream_t st, const Submap3Desc* submaps,
                                    const Pair3Desc* pairs, const Yaw3Desc* yaws,
                                    const float* points, const Score3Job* jobs,
                                    const int4* queries, int32_t* sums);
// Ordered walks to the reference's pick among tied maxima (ResolveTies3d):
// out[2 j] = (yaw, x, y, z), out[2 j + 1].x = found.
hipError_t LaunchFast3dWalk(int num_jobs, hipStream_t st, const Submap3Desc* submaps,
                            const Pair3Desc* pairs, const Yaw3Desc* yaws, const float* points,
                            const float* low_points, const Walk3Job* jobs, const int4* top,
                            int4* out);
// Up to kSegs3 device segments (4-byte multiples) in one launch: copied
// back to back into `out` (PackSegments: one readback instead of one copy
// per buffer) or zeroed (ZeroSegments, out null: one launch instead of one
// memset per buffer).
constexpr int kSegs3 = 8;
struct Segs3 {
  void* ptr[kSegs3];
  int64_t bytes[kSegs3];
  int n;
};
hipError_t LaunchSegments(const Segs3& segs, void* out, hipStream_t st);
hipError_t LaunchFast3dFinalize(int num_pairs, hipStream_t st, const Submap3Desc* submaps,
                                const Pair3Desc* pairs, const Yaw3Desc* yaws,
                                const float* low_points, const unsigned long long* best,
                                float* low_score);

// Rotational scores of every (pair, yaw); `pairs` points to RotPair3 records
// (kernels3d.hip): {node_hist, submap_hist, size, window, step, yaw0, out}.
struct RotPair3Host {
  int32_t node_hist, submap_hist, size, window;
  float step, yaw0;
  int64_t out;
  double min_score;
};
constexpr int kMaxHistogram = 512;
hipError_t LaunchRotScores(const void* pairs, int num_pairs, int max_yaws, const float* hists,
                           float* out, hipStream_t st);
// Passing yaws of each pair (k, score), compacted: range[p] = {offset, count}
// at a global cursor (zeroed by the caller).
hipError_t LaunchYawCompact(const void* pairs, int num_pairs, const float* scores,
                            unsigned* cursor, int2* range, int32_t* out_k, float* out_s,
                            hipStream_t st);

// Discrete-scan poses of the passing yaws (GenerateDiscreteScans :277-294),
// one record per device pair (in device pair order): the pair's fixed
// rotations and translation, the angular step and window, where its passing
// (k, score) lists start in the compacted arrays, and where its Yaw3Desc
// records go.
struct YawBuild3 {
  float siw, six, siy, siz;  // submap_pose.rotation().inverse()
  float nqw, nqx, nqy, nqz;  // node_pose.rotation()
  float tx, ty, tz;          // (submap^-1 * node).translation()
  float astep;
  int32_t window, src, yaw_begin, num;
};
// A yaw whose float sin/cos rounding the device cannot decide: the host
// rebuilds it with the reference's libm.
struct YawFlag3 {
  int32_t dp, j, k;
  float score;
};
constexpr int kYawFlagCap = 4096;
hipError_t LaunchYawBuild(const YawBuild3* items, int num_pairs, const int32_t* k, const float* s,
                          Yaw3Desc* out, unsigned* flag_count, YawFlag3* flags, hipStream_t st);

}  // namespace csm

#endif  // CSM_LAUNCH3D_H_
