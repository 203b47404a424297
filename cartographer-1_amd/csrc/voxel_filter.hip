// Batched voxel filters on gfx950: sensor::VoxelFilter and
// sensor::AdaptiveVoxelFilter (reference sensor/internal/voxel_filter.cc), the
// filters that turn a node's range data into the clouds the scan matchers
// search with (local_trajectory_builder_2d.cc:61-62 and :229-231,
// local_trajectory_builder_3d.cc:682-683 and :735-748).
//
// One workgroup per cloud. The reference keeps, per voxel, the point chosen by
// reservoir sampling with draws from a fresh std::minstd_rand0 consumed in
// point order (RandomizedVoxelFilterIndices, voxel_filter.cc:136-162). The
// result is a function of the draws alone, so the workgroup reproduces it
// without a hash map:
//   1. voxel keys (GetVoxelCellIndex, :79-86: float division, lround, the
//      same wrapping 64-bit key) for the cloud's points, sorted in LDS by
//      (key, point index) with a bitonic network;
//   2. each point's rank within its voxel (segmented max-scan of the sorted
//      run heads); a point of rank r > 0 makes one uniform_int_distribution
//      (1, r + 1) draw, and its position in the generator's stream is the
//      exclusive prefix count of such points (a block scan);
//   3. each thread jumps the LCG to its chunk's first position
//      (16807^pos mod 2^31 - 1) and draws sequentially; libstdc++'s
//      downscaling rejects an output >= past and draws again, which shifts
//      every later draw (first at draw 1310 of a stream), so if any draw is
//      rejected the workgroup redoes the stream in order on one lane;
//   4. a voxel keeps its last successful point, or its first point when no
//      draw succeeded (per-voxel atomicMax in LDS).
// AdaptiveVoxelFilter adds FilterByMaxRange (:31-36) and the edge-length
// search of AdaptivelyVoxelFiltered (:38-76), whose float arithmetic it
// repeats; every VoxelFilter call of that search runs in the same workgroup
// on LDS-resident keys.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "csm_internal.h"

namespace csm {
namespace {

constexpr int kVfThreads = 256;
constexpr int kVfMaxPoints = 8192;  // LDS: 14 B per slot, 112 KiB at 8192
constexpr uint16_t kPad = 0xffff;
constexpr uint32_t kMinstdM = 2147483647u;  // std::minstd_rand0: x <- 16807 x mod (2^31 - 1)
constexpr uint32_t kMinstdA = 16807u;
// uniform_int_distribution's __urngrange = max() - min() for minstd_rand0.
constexpr uint32_t kUrngRange = 2147483645u;

__device__ __forceinline__ uint32_t MulMod(uint32_t a, uint32_t b) {
  const uint64_t p = static_cast<uint64_t>(a) * b;  // < 2^62
  uint64_t r = (p & kMinstdM) + (p >> 31);          // < 2^32
  r = (r & kMinstdM) + (r >> 31);                   // <= 2^31
  return static_cast<uint32_t>(r >= kMinstdM ? r - kMinstdM : r);
}

// State of a seed-1 minstd_rand0 after e draws.
__device__ uint32_t MinstdJump(uint32_t e) {
  uint32_t result = 1u, base = kMinstdA;
  while (e) {
    if (e & 1u) result = MulMod(result, base);
    base = MulMod(base, base);
    e >>= 1;
  }
  return result;
}

// One uniform_int_distribution<>(1, k) draw from output x (no rejection):
// returns 1 when the draw equals k, 0 otherwise, 2 when x is rejected.
__device__ __forceinline__ int Draw(uint32_t x, uint32_t k) {
  const uint32_t scaling = kUrngRange / k;
  const uint32_t past = k * scaling;
  const uint32_t ret = x - 1u;  // __urng() - __urngmin
  if (ret >= past) return 2;
  return (ret / scaling + 1u == k) ? 1 : 0;
}

// GetVoxelCellIndex (voxel_filter.cc:79-86).
__device__ __forceinline__ uint64_t VoxelKeyCoord(float v, float resolution) {
  const float q = __fdiv_rn(v, resolution);
  // common::RoundToInt = std::lround narrowed to int, then widened to uint64_t.
  const int i = static_cast<int>(static_cast<long long>(roundf(q)));
  return static_cast<uint64_t>(static_cast<int64_t>(i));
}
__device__ __forceinline__ uint64_t VoxelKey(float x, float y, float z, float resolution) {
  return (VoxelKeyCoord(x, resolution) << 42) + (VoxelKeyCoord(y, resolution) << 21) +
         VoxelKeyCoord(z, resolution);
}

struct VfLds {
  uint64_t* key;   // [M] sort keys; after sorting, overlaid by seg / rank / aux
  uint16_t* seg;   // [M] sorted position -> position of its voxel's first entry
  uint16_t* rank;  // [M] compacted point -> rank within its voxel
  int32_t* aux;    // [M] voxel head position -> chosen sorted position
  uint16_t* sidx;  // [M] sorted position -> compacted point (kPad past the end)
  uint16_t* vidx;  // [M] compacted point -> point of the cloud
  uint8_t* cur;    // [M] current filter's keep mask (compacted)
  uint8_t* res;    // [M] accepted result (compacted)
  int M, E;        // slots, slots per thread
};

// Exclusive block scans over one value per thread (4 waves).
__device__ int BlockExclusiveSum(int v, int* total, int* tmp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) tmp[w] = x;
  __syncthreads();
  int off = 0, tot = 0;
  for (int i = 0; i < kVfThreads / 64; ++i) {
    if (i < w) off += tmp[i];
    tot += tmp[i];
  }
  __syncthreads();
  *total = tot;
  return off + x - v;
}

__device__ int BlockExclusiveMax(int v, int* tmp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(x, d, 64);
    if (lane >= d) x = max(x, y);
  }
  int ex = __shfl_up(x, 1, 64);
  if (lane == 0) ex = -1;
  if (lane == 63) tmp[w] = x;
  __syncthreads();
  for (int i = 0; i < w; ++i) ex = max(ex, tmp[i]);
  __syncthreads();
  return ex;
}

__device__ __forceinline__ bool SortLess(uint64_t ka, uint16_t ia, uint64_t kb, uint16_t ib) {
  if (ia == kPad) return false;
  if (ib == kPad) return true;
  return ka < kb || (ka == kb && ia < ib);
}

// VoxelFilter over the m compacted points at edge length `resolution`:
// L.cur[j] = 1 for kept points; returns the number kept (all threads).
__device__ int VoxelFilterPass(const float* __restrict__ xyz, const VfLds& L, int m,
                               float resolution, int* tmp, int* flag) {
  const int t = threadIdx.x;
  int mp = 1;
  while (mp < m) mp <<= 1;
  for (int j = t; j < L.M; j += kVfThreads) {
    if (j < m) {
      const int i = L.vidx[j];
      L.key[j] = VoxelKey(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], resolution);
      L.sidx[j] = static_cast<uint16_t>(j);
    } else {
      L.key[j] = ~0ull;
      L.sidx[j] = kPad;
    }
  }
  __syncthreads();
  // Bitonic sort of [0, mp) by (key, index); pads sort last.
  for (int k = 2; k <= mp; k <<= 1) {
    for (int jj = k >> 1; jj > 0; jj >>= 1) {
      for (int i = t; i < mp; i += kVfThreads) {
        const int l = i ^ jj;
        if (l > i) {
          const uint64_t ka = L.key[i], kb = L.key[l];
          const uint16_t ia = L.sidx[i], ib = L.sidx[l];
          const bool asc = (i & k) == 0;
          if (asc ? SortLess(kb, ib, ka, ia) : SortLess(ka, ia, kb, ib)) {
            L.key[i] = kb;
            L.key[l] = ka;
            L.sidx[i] = ib;
            L.sidx[l] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  // Run heads over this thread's chunk of sorted positions [s0, s0 + E).
  const int s0 = t * L.E;
  uint32_t heads = 0;
  {
    uint64_t prev = s0 > 0 ? L.key[s0 - 1] : 0;
    bool prev_valid = s0 > 0 && s0 - 1 < m;
    for (int e = 0; e < L.E; ++e) {
      const int s = s0 + e;
      const uint64_t kk = L.key[s];
      const bool valid = s < m;
      if (valid && (!prev_valid || kk != prev)) heads |= 1u << e;
      prev = kk;
      prev_valid = valid;
    }
  }
  __syncthreads();  // keys are dead from here; seg / rank / aux overlay them
  const int last_head = heads ? s0 + 31 - __clz(heads) : -1;
  int start = BlockExclusiveMax(last_head, tmp);
  for (int e = 0; e < L.E; ++e) {
    const int s = s0 + e;
    if (s >= m) break;
    if (heads & (1u << e)) start = s;
    L.seg[s] = static_cast<uint16_t>(start);
    L.rank[L.sidx[s]] = static_cast<uint16_t>(s - start);
  }
  int nvox = 0;
  (void)BlockExclusiveSum(__popc(heads), &nvox, tmp);  // also orders the rank writes
  // Stream positions: points of rank > 0 in compacted order draw once each.
  const int j0 = t * L.E;
  int draws = 0;
  for (int e = 0; e < L.E; ++e) {
    const int j = j0 + e;
    if (j < m && L.rank[j] > 0) ++draws;
  }
  int total_draws = 0;
  const int pos0 = BlockExclusiveSum(draws, &total_draws, tmp);
  if (t == 0) *flag = 0;
  __syncthreads();
  bool rejected = false;
  if (draws > 0) {
    uint32_t state = MinstdJump(static_cast<uint32_t>(pos0));
    for (int e = 0; e < L.E; ++e) {
      const int j = j0 + e;
      if (j >= m) break;
      const int r = L.rank[j];
      uint8_t ok = 0;
      if (r > 0) {
        state = MulMod(state, kMinstdA);
        const int d = Draw(state, static_cast<uint32_t>(r + 1));
        rejected |= d == 2;
        ok = d == 1;
      }
      L.cur[j] = ok;
    }
  } else {
    for (int e = 0; e < L.E; ++e) {
      const int j = j0 + e;
      if (j < m) L.cur[j] = 0;
    }
  }
  if (rejected) *flag = 1;
  __syncthreads();
  if (*flag) {
    // A rejected output consumed an extra draw: replay the stream in order.
    if (t == 0) {
      uint32_t state = 1u;
      for (int j = 0; j < m; ++j) {
        const int r = L.rank[j];
        if (r == 0) {
          L.cur[j] = 0;
          continue;
        }
        int d;
        do {
          state = MulMod(state, kMinstdA);
          d = Draw(state, static_cast<uint32_t>(r + 1));
        } while (d == 2);
        L.cur[j] = d == 1;
      }
    }
    __syncthreads();
  }
  // Each voxel keeps its last successful point, else its first.
  for (int s = t; s < m; s += kVfThreads)
    if (L.seg[s] == s) L.aux[s] = -1;
  __syncthreads();
  for (int s = t; s < m; s += kVfThreads) {
    const int j = L.sidx[s];
    if (L.rank[j] == 0 || L.cur[j]) atomicMax(&L.aux[L.seg[s]], s);
  }
  __syncthreads();
  for (int j = t; j < m; j += kVfThreads) L.cur[j] = 0;
  __syncthreads();
  for (int s = t; s < m; s += kVfThreads)
    if (L.seg[s] == s) L.cur[L.sidx[L.aux[s]]] = 1;
  __syncthreads();
  return nvox;
}

__device__ void CopyMask(const VfLds& L, int m) {
  for (int j = threadIdx.x; j < m; j += kVfThreads) L.res[j] = L.cur[j];
  __syncthreads();
}

// mode 0: VoxelFilter(cloud, p0). mode 1: AdaptiveVoxelFilter(cloud,
// {max_length = p0, min_num_points = p1, max_range = p2}).
__global__ void __launch_bounds__(kVfThreads)
voxel_filter_batch(const float* __restrict__ points, const int64_t* __restrict__ offsets, int mode,
                   float p0, float p1, float p2, int M, uint8_t* __restrict__ keep,
                   int32_t* __restrict__ counts) {
  extern __shared__ __align__(16) unsigned char lds[];
  __shared__ int tmp[kVfThreads / 64];
  __shared__ int flag;
  VfLds L;
  L.M = M;
  L.E = M / kVfThreads;
  L.key = reinterpret_cast<uint64_t*>(lds);
  L.seg = reinterpret_cast<uint16_t*>(lds);
  L.rank = reinterpret_cast<uint16_t*>(lds + 2 * M);
  L.aux = reinterpret_cast<int32_t*>(lds + 4 * M);
  L.sidx = reinterpret_cast<uint16_t*>(lds + 8 * M);
  L.vidx = reinterpret_cast<uint16_t*>(lds + 10 * M);
  L.cur = lds + 12 * M;
  L.res = lds + 13 * M;

  const int c = blockIdx.x;
  const int64_t begin = offsets[c];
  const int n = static_cast<int>(offsets[c + 1] - begin);
  const float* xyz = points + 3 * begin;
  const int t = threadIdx.x;

  int m = n;
  if (mode == 1) {
    // FilterByMaxRange: ||p|| <= max_range, Eigen's x0 + (x1 + x2) order.
    const int i0 = t * L.E;
    uint32_t pass = 0;
    for (int e = 0; e < L.E; ++e) {
      const int i = i0 + e;
      if (i < n) {
        const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        const float norm = sqrtf(__fadd_rn(__fmul_rn(x, x), __fadd_rn(__fmul_rn(y, y), __fmul_rn(z, z))));
        if (norm <= p2) pass |= 1u << e;
      }
    }
    int total = 0;
    int j = BlockExclusiveSum(__popc(pass), &total, tmp);
    for (int e = 0; e < L.E; ++e)
      if (pass & (1u << e)) L.vidx[j++] = static_cast<uint16_t>(i0 + e);
    m = total;
  } else {
    for (int j = t; j < n; j += kVfThreads) L.vidx[j] = static_cast<uint16_t>(j);
  }
  __syncthreads();

  int kept;
  if (mode == 0) {
    kept = VoxelFilterPass(xyz, L, m, p0, tmp, &flag);
    CopyMask(L, m);
  } else if (static_cast<float>(m) <= p1) {
    for (int j = t; j < m; j += kVfThreads) L.res[j] = 1;
    __syncthreads();
    kept = m;
  } else {
    // AdaptivelyVoxelFiltered (voxel_filter.cc:38-76), float arithmetic as written.
    const float max_length = p0, min_num_points = p1;
    kept = VoxelFilterPass(xyz, L, m, max_length, tmp, &flag);
    CopyMask(L, m);
    if (!(static_cast<float>(kept) >= min_num_points)) {
      for (float high_length = max_length; high_length > __fmul_rn(1e-2f, max_length);
           high_length = __fdiv_rn(high_length, 2.f)) {
        float low_length = __fdiv_rn(high_length, 2.f);
        kept = VoxelFilterPass(xyz, L, m, low_length, tmp, &flag);
        CopyMask(L, m);
        if (static_cast<float>(kept) >= min_num_points) {
          while (__fdiv_rn(__fsub_rn(high_length, low_length), low_length) > 1e-1f) {
            const float mid_length = __fdiv_rn(__fadd_rn(low_length, high_length), 2.f);
            const int cand = VoxelFilterPass(xyz, L, m, mid_length, tmp, &flag);
            if (static_cast<float>(cand) >= min_num_points) {
              low_length = mid_length;
              kept = cand;
              CopyMask(L, m);
            } else {
              high_length = mid_length;
            }
          }
          break;
        }
      }
    }
  }
  // Scatter the compacted result back to the cloud's points, coalesced write.
  for (int i = t; i < n; i += kVfThreads) L.cur[i] = 0;
  __syncthreads();
  for (int j = t; j < m; j += kVfThreads) L.cur[L.vidx[j]] = L.res[j];
  __syncthreads();
  for (int i = t; i < n; i += kVfThreads) keep[begin + i] = L.cur[i];
  if (t == 0 && counts) counts[c] = kept;
}

int SlotsFor(int max_points) {
  int M = kVfThreads;
  while (M < max_points) M <<= 1;
  return M;
}

int LaunchVoxelFilter(csm_context* ctx, const float* d_xyz, const int64_t* d_offsets,
                      int32_t num_clouds, int32_t max_points, int mode, float p0, float p1,
                      float p2, uint8_t* d_keep, int32_t* d_counts) {
  if (!ctx || num_clouds < 0 || max_points < 0) return CSM_EINVAL;
  if (max_points > kVfMaxPoints) return CSM_ERANGE;
  if (num_clouds == 0) return CSM_OK;
  if (!d_xyz || !d_offsets || !d_keep) return CSM_EINVAL;
  const int M = SlotsFor(max_points);
  const size_t lds = static_cast<size_t>(14) * M;
  if (lds > 64 * 1024)
    CSM_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&voxel_filter_batch),
                                hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  hipLaunchKernelGGL(voxel_filter_batch, dim3(num_clouds), dim3(kVfThreads), lds, ctx->stream,
                     d_xyz, d_offsets, mode, p0, p1, p2, M, d_keep, d_counts);
  CSM_HIP(hipGetLastError());
  return CSM_OK;
}

int HostVoxelFilter(csm_context* ctx, const float* xyz, const int64_t* offsets, int32_t num_clouds,
                    int mode, float p0, float p1, float p2, uint8_t* keep, int32_t* counts) {
  if (!ctx || num_clouds < 0 || (num_clouds > 0 && (!offsets || !keep))) return CSM_EINVAL;
  if (num_clouds == 0) return CSM_OK;
  int64_t max_points = 0;
  for (int32_t c = 0; c < num_clouds; ++c) {
    const int64_t n = offsets[c + 1] - offsets[c];
    if (n < 0) return CSM_EINVAL;
    max_points = std::max(max_points, n);
  }
  if (max_points > kVfMaxPoints) return CSM_ERANGE;
  const int64_t total = offsets[num_clouds] - offsets[0];
  if (total > 0 && !xyz) return CSM_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  // Rebase the offsets so the device copy starts at point 0.
  std::vector<int64_t> rebased(static_cast<size_t>(num_clouds) + 1);
  for (int32_t c = 0; c <= num_clouds; ++c) rebased[c] = offsets[c] - offsets[0];
  int rc;
  if ((rc = ctx->vf_points.Reserve(sizeof(float) * 3 * std::max<int64_t>(total, 1)))) return rc;
  if ((rc = ctx->vf_offsets.Reserve(sizeof(int64_t) * rebased.size()))) return rc;
  if ((rc = ctx->vf_keep.Reserve(std::max<int64_t>(total, 1)))) return rc;
  if ((rc = ctx->vf_counts.Reserve(sizeof(int32_t) * num_clouds))) return rc;
  hipStream_t st = ctx->stream;
  if (total > 0)
    CSM_HIP(hipMemcpyAsync(ctx->vf_points.ptr, xyz + 3 * offsets[0], sizeof(float) * 3 * total,
                           hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(ctx->vf_offsets.ptr, rebased.data(), sizeof(int64_t) * rebased.size(),
                         hipMemcpyHostToDevice, st));
  if ((rc = LaunchVoxelFilter(ctx, ctx->vf_points.as<float>(), ctx->vf_offsets.as<int64_t>(),
                              num_clouds, static_cast<int32_t>(max_points), mode, p0, p1, p2,
                              ctx->vf_keep.as<uint8_t>(), ctx->vf_counts.as<int32_t>())))
    return rc;
  if (total > 0)
    CSM_HIP(hipMemcpyAsync(keep + offsets[0], ctx->vf_keep.ptr, total, hipMemcpyDeviceToHost, st));
  if (counts)
    CSM_HIP(hipMemcpyAsync(counts, ctx->vf_counts.ptr, sizeof(int32_t) * num_clouds,
                           hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  return CSM_OK;
}

}  // namespace
}  // namespace csm

extern "C" {

int csm_voxel_filter(csm_context* ctx, const float* xyz, const int64_t* offsets,
                     int32_t num_clouds, float resolution, uint8_t* keep, int32_t* counts) {
  if (!(resolution > 0.f)) return CSM_EINVAL;
  return csm::HostVoxelFilter(ctx, xyz, offsets, num_clouds, 0, resolution, 0.f, 0.f, keep,
                              counts);
}

int csm_adaptive_voxel_filter(csm_context* ctx, const float* xyz, const int64_t* offsets,
                              int32_t num_clouds, const csm_adaptive_voxel_filter_options* options,
                              uint8_t* keep, int32_t* counts) {
  if (!options || !(options->max_length > 0.f)) return CSM_EINVAL;
  return csm::HostVoxelFilter(ctx, xyz, offsets, num_clouds, 1, options->max_length,
                              options->min_num_points, options->max_range, keep, counts);
}

int csm_voxel_filter_device(csm_context* ctx, const float* d_xyz, const int64_t* d_offsets,
                            int32_t num_clouds, int32_t max_points, float resolution,
                            uint8_t* d_keep, int32_t* d_counts) {
  if (!(resolution > 0.f)) return CSM_EINVAL;
  return csm::LaunchVoxelFilter(ctx, d_xyz, d_offsets, num_clouds, max_points, 0, resolution, 0.f,
                                0.f, d_keep, d_counts);
}

int csm_adaptive_voxel_filter_device(csm_context* ctx, const float* d_xyz,
                                     const int64_t* d_offsets, int32_t num_clouds,
                                     int32_t max_points,
                                     const csm_adaptive_voxel_filter_options* options,
                                     uint8_t* d_keep, int32_t* d_counts) {
  if (!options || !(options->max_length > 0.f)) return CSM_EINVAL;
  return csm::LaunchVoxelFilter(ctx, d_xyz, d_offsets, num_clouds, max_points, 1,
                                options->max_length, options->min_num_points, options->max_range,
                                d_keep, d_counts);
}

}  // extern "C"
