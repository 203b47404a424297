// gfx950 kernels of the correlative scan matcher.
//
//   K1  pyramid_level0 / pyramid_double — PrecomputationGridStack2D
//       (fast_correlative_scan_matcher_2d.cc:91-186) built on the device.
//   K2-K4 fast2d_search — per (pair, rotation chunk): discretize the rotated
//       scan slice into LDS (correlative_scan_matcher_2d.cc:93-127 +
//       map_limits.h:69-75), ShrinkToFit (:73-91), score the top-level lattice
//       (fast_correlative_scan_matcher_2d.cc:264-333) and run an exact
//       depth-first branch and bound per wave (:335-378) against a per-pair
//       incumbent shared through a 64-bit atomicMax.
// (RealTimeCorrelativeScanMatcher2D's kernels are in rt2d.hip.)
//
// Built with -ffp-contract=off; the discretization additionally uses the
// explicit round-to-nearest intrinsics so no multiply-add is ever fused:
// the x86-64 reference build has no FMA (DESIGN.md "Bitwise discretization").

#include <hip/hip_runtime.h>

#include <algorithm>

#include "csm_device.h"
#include "geom2d_dev.h"

namespace csm {

// ---------------------------------------------------------------- helpers ---

__device__ __forceinline__ int WaveSum(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
__device__ __forceinline__ int WaveMin(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = min(v, __shfl_xor(v, m, 64));
  return v;
}
__device__ __forceinline__ int WaveMax(int v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = max(v, __shfl_xor(v, m, 64));
  return v;
}
__device__ __forceinline__ int Uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Wave-wide max / sum without the LDS crossbar: DPP within each 16-lane row
// (quad perms, half-row and row mirrors), then the four row results through
// readlane. Every lane gets the result.
template <typename Op>
__device__ __forceinline__ int DppReduce(int v, Op op) {
  v = op(v, __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
  v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
  v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x141, 0xF, 0xF, false));  // row_half_mirror
  v = op(v, __builtin_amdgcn_update_dpp(v, v, 0x140, 0xF, 0xF, false));  // row_mirror
  const int r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
  const int r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
  return op(op(r0, r1), op(r2, r3));
}
__device__ __forceinline__ int DppMax(int v) {
  return DppReduce(v, [](int a, int b) { return max(a, b); });
}
__device__ __forceinline__ int DppSum(int v) {
  return DppReduce(v, [](int a, int b) { return a + b; });
}

__device__ __forceinline__ uint64_t LoadBest(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- K1 -------

// Level 0: quantized probability of every cell (ComputeCellValue of
// 1 - |cc|); the table is computed on the host with the reference's float
// arithmetic. The trailing byte of every level is a zero sentinel.
__global__ void pyramid_level0(const uint16_t* __restrict__ cells,
                               const uint8_t* __restrict__ qtab,
                               uint8_t* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = qtab[cells[i] & 0x7fff];
  if (i == n) out[n] = 0;
}

// Level d from level d-1 (h = 2^(d-1)): wide cell l covers source cells
// [l - 2h + 1, l] = cover(l - h) u cover(l) of level d-1, per axis; an empty
// cover contributes 0, which never changes a max of uint8 values.
__global__ void pyramid_double(const uint8_t* __restrict__ prev, int pnx, int pny,
                               uint8_t* __restrict__ next, int nnx, int nny, int h) {
  const int lx = blockIdx.x * blockDim.x + threadIdx.x;
  const int ly = blockIdx.y;
  if (ly == 0 && lx == 0) next[static_cast<size_t>(nnx) * nny] = 0;
  if (lx >= nnx || ly >= nny) return;
  int v = 0;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int my = ly - a * h;
    if (my < 0 || my >= pny) continue;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int mx = lx - b * h;
      if (mx < 0 || mx >= pnx) continue;
      v = max(v, static_cast<int>(prev[static_cast<size_t>(my) * pnx + mx]));
    }
  }
  next[static_cast<size_t>(ly) * nnx + lx] = static_cast<uint8_t>(v);
}

// ---------------------------------------------------------------- K2-K4 ----

struct LevelView {
  const uint8_t* data;
  int wnx, wny, zero, bias;  // local index = cell + bias, bias = 2^d - 1
};

__device__ __forceinline__ LevelView MakeView(const SubmapDesc& s, int d) {
  LevelView v;
  v.data = s.level[d];
  v.wnx = s.wide_nx[d];
  v.wny = s.wide_ny[d];
  v.zero = s.zero_index[d];
  v.bias = (1 << d) - 1;
  return v;
}

// Scores the (up to) four children (xo + {0,h}) x (yo + {0,h}) of one node
// at level view L. Lanes walk the rotation's discretized points (packed
// int16 pairs in LDS, padded with sentinels to a multiple of 64).
__device__ __forceinline__ void ScoreChildren(const uint32_t* __restrict__ pts,
                                              int npad, const LevelView& L,
                                              int xo, int yo, int h, int out[4]) {
  const int lane = threadIdx.x & 63;
  int a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  const int hw = h * L.wnx;
  // npad is a multiple of 64; take 4 points per lane per iteration so 16
  // byte loads are in flight before any is consumed.
  int i = lane;
  for (; i + 192 < npad; i += 256) {
    int ad[16];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t p = pts[i + 64 * u];
      const int lx = static_cast<int>(static_cast<int16_t>(p & 0xffff)) + xo + L.bias;
      const int lyy = (static_cast<int>(p) >> 16) + yo + L.bias;
      const bool vx0 = static_cast<unsigned>(lx) < static_cast<unsigned>(L.wnx);
      const bool vx1 = static_cast<unsigned>(lx + h) < static_cast<unsigned>(L.wnx);
      const bool vy0 = static_cast<unsigned>(lyy) < static_cast<unsigned>(L.wny);
      const bool vy1 = static_cast<unsigned>(lyy + h) < static_cast<unsigned>(L.wny);
      const int base = lyy * L.wnx + lx;
      ad[4 * u + 0] = (vx0 && vy0) ? base : L.zero;
      ad[4 * u + 1] = (vx0 && vy1) ? base + hw : L.zero;
      ad[4 * u + 2] = (vx1 && vy0) ? base + h : L.zero;
      ad[4 * u + 3] = (vx1 && vy1) ? base + hw + h : L.zero;
    }
    int v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = L.data[ad[u]];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a0 += v[4 * u]; a1 += v[4 * u + 1]; a2 += v[4 * u + 2]; a3 += v[4 * u + 3];
    }
  }
  for (; i < npad; i += 64) {
    const uint32_t p = pts[i];
    const int lx = static_cast<int>(static_cast<int16_t>(p & 0xffff)) + xo + L.bias;
    const int ly = static_cast<int>(p) >> 16;
    const int lyy = ly + yo + L.bias;
    const bool vx0 = static_cast<unsigned>(lx) < static_cast<unsigned>(L.wnx);
    const bool vx1 = static_cast<unsigned>(lx + h) < static_cast<unsigned>(L.wnx);
    const bool vy0 = static_cast<unsigned>(lyy) < static_cast<unsigned>(L.wny);
    const bool vy1 = static_cast<unsigned>(lyy + h) < static_cast<unsigned>(L.wny);
    const int base = lyy * L.wnx + lx;
    a0 += L.data[(vx0 && vy0) ? base : L.zero];
    a1 += L.data[(vx0 && vy1) ? base + hw : L.zero];
    a2 += L.data[(vx1 && vy0) ? base + h : L.zero];
    a3 += L.data[(vx1 && vy1) ? base + hw + h : L.zero];
  }
  out[0] = WaveSum(a0);  // (xo,     yo)
  out[1] = WaveSum(a1);  // (xo,     yo + h)
  out[2] = WaveSum(a2);  // (xo + h, yo)
  out[3] = WaveSum(a3);  // (xo + h, yo + h)
}

// Scores one candidate at level view L.
__device__ __forceinline__ int ScoreOne(const uint32_t* __restrict__ pts, int npad,
                                        const LevelView& L, int xo, int yo) {
  const int lane = threadIdx.x & 63;
  int acc = 0;
  int i = lane;
  for (; i + 448 < npad; i += 512) {
    int ad[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint32_t p = pts[i + 64 * u];
      const int lx = static_cast<int>(static_cast<int16_t>(p & 0xffff)) + xo + L.bias;
      const int ly = (static_cast<int>(p) >> 16) + yo + L.bias;
      const bool v = static_cast<unsigned>(lx) < static_cast<unsigned>(L.wnx) &&
                     static_cast<unsigned>(ly) < static_cast<unsigned>(L.wny);
      ad[u] = v ? ly * L.wnx + lx : L.zero;
    }
    int val[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) val[u] = L.data[ad[u]];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += val[u];
  }
  for (; i < npad; i += 64) {
    const uint32_t p = pts[i];
    const int lx = static_cast<int>(static_cast<int16_t>(p & 0xffff)) + xo + L.bias;
    const int ly = (static_cast<int>(p) >> 16) + yo + L.bias;
    const bool v = static_cast<unsigned>(lx) < static_cast<unsigned>(L.wnx) &&
                   static_cast<unsigned>(ly) < static_cast<unsigned>(L.wny);
    acc += L.data[v ? ly * L.wnx + lx : L.zero];
  }
  return WaveSum(acc);
}

struct RotInfo {
  int min_x, max_x, min_y, max_y;  // ShrinkToFit bounds
  int top_begin;                   // prefix of top-level candidates
  int top_nx, top_ny;
  int pad;
};

// Stack entry: w0 = (uint16 xo) | (yo << 16); w1 = sum | rot << 22 | level << 27.
__device__ __forceinline__ uint2 MakeEntry(int xo, int yo, int sum, int rot, int level) {
  return make_uint2((static_cast<uint32_t>(xo) & 0xffff) | (static_cast<uint32_t>(yo) << 16),
                    static_cast<uint32_t>(sum) | (static_cast<uint32_t>(rot) << 22) |
                        (static_cast<uint32_t>(level) << 27));
}

__global__ void __launch_bounds__(kSearchThreads)
fast2d_search(const SubmapDesc* __restrict__ submaps,
              const PairDesc* __restrict__ pairs,
              const float* __restrict__ points,        // xyz
              const float2* __restrict__ rot_table,    // (w, s)
              WorkQueues queues,
              unsigned long long* __restrict__ counters,  // kNumXcd claim counters
              uint64_t* __restrict__ best,            // per pair leaf key
              int32_t* __restrict__ status,            // per pair
              unsigned long long* __restrict__ stats)  // [0] candidates scored, [1] lookups
{
  extern __shared__ __align__(16) uint32_t lds_pts[];  // rot_chunk * npad_max
  __shared__ RotInfo rinfo[32];
  __shared__ uint2 stack[kWaves][kStackCap];
  __shared__ uint32_t top_xy[kWaves][kTopChunk];
  __shared__ int top_meta[kWaves][kTopChunk];  // sum | rot << 22
  __shared__ int s_item_pair, s_item_chunk, s_total_top, s_next_chunk, s_queue;
  __shared__ int s_mm[32][4];

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int rc = queues.rot_chunk;
  unsigned long long local_cands = 0, local_lookups = 0;

  if (tid == 0) s_queue = blockIdx.x % kNumXcd;
  __syncthreads();
  int tries = 0;
  for (;;) {
    // ---- claim a work item (pair, rotation chunk) from an XCD queue ------
    if (tid == 0) {
      int q = s_queue;
      int pair = -1, chunk = 0;
      while (tries < kNumXcd) {
        const int64_t item = static_cast<int64_t>(atomicAdd(&counters[q], 1ull));
        if (item < queues.queue_chunks[q]) {
          // Binary search the pair whose chunk range holds `item`.
          int lo = queues.queue_begin[q], hi = queues.queue_begin[q + 1] - 1;
          const int64_t base = queues.chunk_prefix[queues.queue_begin[q]];
          while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (queues.chunk_prefix[mid] - base <= item) lo = mid; else hi = mid - 1;
          }
          pair = queues.pair_order[lo];
          chunk = static_cast<int>(item - (queues.chunk_prefix[lo] - base));
          break;
        }
        q = (q + 1) % kNumXcd;  // own queue drained: help the next XCD's queue
        ++tries;
      }
      s_queue = q;
      s_item_pair = pair;
      s_item_chunk = chunk;
    }
    __syncthreads();
    const int pair_index = Uniform(s_item_pair);
    if (pair_index < 0) break;
    const PairDesc pd = pairs[pair_index];
    const SubmapDesc& sm = submaps[pd.submap];
    const int rot0 = Uniform(s_item_chunk) * rc;
    const int nrot = min(rc, pd.num_scans - rot0);
    const int n = pd.num_points;
    const int npad = (n + 63) & ~63;

    // ---- K2: discretize the chunk's rotated scans into LDS --------------
    bool range_error = false;
    for (int r = 0; r < nrot; ++r) {
      const float2 q = rot_table[pd.rot_offset + rot0 + r];
      int mnx = 0x7fffffff, mxx = -0x7fffffff, mny = 0x7fffffff, mxy = -0x7fffffff;
      for (int i = tid; i < npad; i += kSearchThreads) {
        uint32_t packed = (static_cast<uint32_t>(static_cast<uint16_t>(kSentinel))) |
                          (static_cast<uint32_t>(static_cast<uint16_t>(kSentinel)) << 16);
        if (i < n) {
          const float* p = points + 3 * (pd.point_offset + i);
          float x, y;
          RotateZDev(pd.pre_w, pd.pre_s, p[0], p[1], &x, &y);
          RotateZDev(q.x, q.y, x, y, &x, &y);
          // Eigen::Affine2f(translation) * p == t + (1*x + 0*y) in float.
          const float px = __fadd_rn(pd.tx, x);
          const float py = __fadd_rn(pd.ty, y);
          const double cx = CellCoord(sm.max_y, py, sm.resolution);
          const double cy = CellCoord(sm.max_x, px, sm.resolution);
          int ix = 0, iy = 0;
          if (fabs(cx) > kIndexLimit || fabs(cy) > kIndexLimit) {
            range_error = true;
          } else {
            ix = static_cast<int>(cx);
            iy = static_cast<int>(cy);
          }
          mnx = min(mnx, ix); mxx = max(mxx, ix);
          mny = min(mny, iy); mxy = max(mxy, iy);
          packed = (static_cast<uint32_t>(ix) & 0xffff) | (static_cast<uint32_t>(iy) << 16);
        }
        lds_pts[r * npad + i] = packed;
      }
      mnx = WaveMin(mnx); mxx = WaveMax(mxx);
      mny = WaveMin(mny); mxy = WaveMax(mxy);
      if (lane == 0) {
        if (wave == 0) { s_mm[r][0] = mnx; s_mm[r][1] = mxx; s_mm[r][2] = mny; s_mm[r][3] = mxy; }
      }
      __syncthreads();
      if (lane == 0 && wave != 0) {
        atomicMin(&s_mm[r][0], mnx); atomicMax(&s_mm[r][1], mxx);
        atomicMin(&s_mm[r][2], mny); atomicMax(&s_mm[r][3], mxy);
      }
    }
    if (range_error) atomicOr(&status[pair_index], kStatusRange);
    __syncthreads();

    // ---- ShrinkToFit + top-level lattice sizes -------------------------
    const int top_level = sm.levels - 1;
    const int step = 1 << top_level;
    if (tid == 0) {
      int total = 0;
      for (int r = 0; r < nrot; ++r) {
        RotInfo ri;
        const int lo_x = min(0, -s_mm[r][1]), hi_x = max(0, sm.nx - 1 - s_mm[r][0]);
        const int lo_y = min(0, -s_mm[r][3]), hi_y = max(0, sm.ny - 1 - s_mm[r][2]);
        ri.min_x = max(-pd.num_linear, lo_x);
        ri.max_x = min(pd.num_linear, hi_x);
        ri.min_y = max(-pd.num_linear, lo_y);
        ri.max_y = min(pd.num_linear, hi_y);
        if (n == 0) { ri.min_x = ri.max_x = ri.min_y = ri.max_y = 0; }
        ri.top_nx = (ri.max_x - ri.min_x + step) / step;
        ri.top_ny = (ri.max_y - ri.min_y + step) / step;
        ri.top_begin = total;
        total += ri.top_nx * ri.top_ny;
        rinfo[r] = ri;
      }
      s_total_top = total;
      s_next_chunk = 0;
    }
    __syncthreads();

    // ---- K3 + K4: top-level chunks, then depth-first branch and bound ---
    const int total_top = s_total_top;
    const int s_min = pd.max_rejected_sum;
    uint64_t* pair_best = best + pair_index;
    uint64_t cached = LoadBest(pair_best);
    for (;;) {
      int chunk = 0;
      if (lane == 0) chunk = atomicAdd(&s_next_chunk, 1);
      chunk = Uniform(chunk);
      const int begin = chunk * kTopChunk;
      if (begin >= total_top) break;
      const int count = min(kTopChunk, total_top - begin);
      const LevelView top = MakeView(sm, top_level);
      // Score the chunk's candidates one after another (lanes = points).
      for (int j = 0; j < count; ++j) {
        const int t = begin + j;
        int r = 0;
        while (r + 1 < nrot && rinfo[r + 1].top_begin <= t) ++r;
        const RotInfo& ri = rinfo[r];
        const int k = t - ri.top_begin;
        const int xo = ri.min_x + (k / ri.top_ny) * step;
        const int yo = ri.min_y + (k % ri.top_ny) * step;
        const int sum = ScoreOne(lds_pts + r * npad, npad, top, xo, yo);
        if (lane == 0) {
          top_xy[wave][j] = (static_cast<uint32_t>(xo) & 0xffff) | (static_cast<uint32_t>(yo) << 16);
          top_meta[wave][j] = sum | (r << 22);
        }
      }
      local_cands += count;
      local_lookups += static_cast<unsigned long long>(count) * n;
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      const uint32_t best_sum = static_cast<uint32_t>(cached >> kSumShift);
      // Keep candidates above min_score and not below the incumbent; sort
      // them by bound, best on top of the stack.
      int meta = lane < count ? top_meta[wave][lane] : 0;
      int sum = meta & 0x3fffff;
      const bool keep = lane < count && sum > s_min && static_cast<uint32_t>(sum) >= best_sum;
      if (top_level == 0) {
        // Depth-1 search: the top level is the leaf level.
        uint64_t key = 0;
        if (keep) {
          const uint32_t xy = top_xy[wave][lane];
          const int xo = static_cast<int16_t>(xy & 0xffff), yo = static_cast<int>(xy) >> 16;
          key = PackLeafKey(sum, rot0 + (meta >> 22), xo, yo);
        }
        for (int m = 32; m >= 1; m >>= 1) {
          const uint64_t o = __shfl_xor(key, m, 64);
          key = o > key ? o : key;
        }
        if (key > cached) {
          uint64_t old = 0;
          if (lane == 0) old = atomicMax(reinterpret_cast<unsigned long long*>(pair_best), key);
          old = __shfl(old, 0, 64);
          cached = key > old ? key : old;
        }
        continue;
      }
      // Bitonic sort (descending) of (sum << 8 | lane) over the wave.
      uint32_t skey = keep ? ((static_cast<uint32_t>(sum) << 8) | static_cast<uint32_t>(lane)) : 0u;
      for (int k = 2; k <= 64; k <<= 1) {
        for (int jj = k >> 1; jj >= 1; jj >>= 1) {
          const uint32_t other = __shfl_xor(skey, jj, 64);
          const bool up = ((lane & k) == 0);
          const bool lower = ((lane & jj) == 0);
          const uint32_t hi_v = skey > other ? skey : other;
          const uint32_t lo_v = skey > other ? other : skey;
          skey = (lower == up) ? hi_v : lo_v;
        }
      }
      const int kept = __popcll(__ballot(keep));
      int sp = 0;
      if (lane < kept) {
        const int j = skey & 0xff;
        const uint32_t xy = top_xy[wave][j];
        const int m2 = top_meta[wave][j];
        // Largest sum at the highest stack slot.
        stack[wave][kept - 1 - lane] =
            make_uint2(xy, static_cast<uint32_t>(m2 & 0x3fffff) |
                               (static_cast<uint32_t>(m2 >> 22) << 22) |
                               (static_cast<uint32_t>(top_level) << 27));
      }
      sp = kept;
      __builtin_amdgcn_wave_barrier();

      // Depth-first branch and bound over this wave's stack.
      int iter = 0;
      while (sp > 0) {
        --sp;
        const uint2 e = stack[wave][sp];
        const uint32_t e0 = Uniform(e.x), e1 = Uniform(e.y);
        const int xo = static_cast<int16_t>(e0 & 0xffff);
        const int yo = static_cast<int>(e0) >> 16;
        const uint32_t bound = e1 & 0x3fffff;
        const int r = (e1 >> 22) & 0x1f;
        const int d = e1 >> 27;
        if ((++iter & 7) == 0) {
          uint64_t fresh = 0;
          if (lane == 0) fresh = LoadBest(pair_best);
          fresh = __shfl(fresh, 0, 64);
          cached = fresh > cached ? fresh : cached;
        }
        if (bound < static_cast<uint32_t>(cached >> kSumShift)) continue;
        const int h = 1 << (d - 1);
        const RotInfo& ri = rinfo[r];
        const bool hx = xo + h <= ri.max_x;
        const bool hy = yo + h <= ri.max_y;
        int sums[4];
        const LevelView L = MakeView(sm, d - 1);
        ScoreChildren(lds_pts + r * npad, npad, L, xo, yo, h, sums);
        const int nchild = 1 + (hx ? 1 : 0) + (hy ? 1 : 0) + ((hx && hy) ? 1 : 0);
        local_cands += nchild;
        local_lookups += static_cast<unsigned long long>(nchild) * n;
        const int cxo[4] = {xo, xo, xo + h, xo + h};
        const int cyo[4] = {yo, yo + h, yo, yo + h};
        const bool exists[4] = {true, hy, hx, hx && hy};
        const uint32_t cur = static_cast<uint32_t>(cached >> kSumShift);
        if (d - 1 == 0) {
          uint64_t key = 0;
          bool range_bad = false;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if (!exists[c] || sums[c] <= s_min || static_cast<uint32_t>(sums[c]) < cur) continue;
            if (cxo[c] < -kOffsetLimit || cxo[c] > kOffsetLimit || cyo[c] < -kOffsetLimit ||
                cyo[c] > kOffsetLimit) { range_bad = true; continue; }
            const uint64_t k2 = PackLeafKey(sums[c], rot0 + r, cxo[c], cyo[c]);
            key = k2 > key ? k2 : key;
          }
          if (range_bad && lane == 0) atomicOr(&status[pair_index], kStatusRange);
          if (key > cached) {
            uint64_t old = 0;
            if (lane == 0) old = atomicMax(reinterpret_cast<unsigned long long*>(pair_best), key);
            old = __shfl(old, 0, 64);
            cached = key > old ? key : old;
          }
        } else {
          // Push surviving children, ascending by bound (best popped first).
          int order[4];
          int m = 0;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (exists[c] && sums[c] > s_min && static_cast<uint32_t>(sums[c]) >= cur) order[m++] = c;
          for (int a = 1; a < m; ++a) {  // insertion sort, ascending
            const int v = order[a];
            int b = a - 1;
            while (b >= 0 && sums[order[b]] > sums[v]) { order[b + 1] = order[b]; --b; }
            order[b + 1] = v;
          }
          if (lane < m) {
            const int c = order[lane];
            stack[wave][sp + lane] = MakeEntry(cxo[c], cyo[c], sums[c], r, d - 1);
          }
          sp += m;
          __builtin_amdgcn_wave_barrier();
        }
      }
    }
    __syncthreads();
  }
  if (stats && lane == 0) {
    atomicAdd(&stats[0], local_cands);
    atomicAdd(&stats[1], local_lookups);
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t LevelRsrc(const uint8_t* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), 0, bytes, 0x00020000);
}

// DFS stack entry word 1: bound sum (22 bits) | level << 27.
__device__ __forceinline__ uint32_t V2Entry1(int sum, int level) {
  return static_cast<uint32_t>(sum) | (static_cast<uint32_t>(level) << 27);
}

constexpr int kRootChunk = 192;  // virtual roots pushed at a time

// ---------------------------------------------------------------- K1c ------

// Quad layout of level d (h = 2^d) for scan clusters of k = km1 + 1 cells
// per side: M(c) = max of level 0 over [c, c + h + km1) per axis = the max of
// G_d at c and c + km1 (km1 <= h). M's wide index is m = c + (h - 1) + km1.
// The dword for quad cell (X', Y'), X' < qw = wnx + km1 + h, Y' < qh, packs
// the children values of a node whose child (0,0) sits at M-wide cell
// (X, Y) = (X' - h, Y' - h): byte0 M(X, Y), byte1 M(X, Y+h), byte2 M(X+h, Y),
// byte3 M(X+h, Y+h); 0 outside. Cells are stored polyphase with period
// P = 2h: plane (X' mod P, Y' mod P), entry (X' / P, Y' / P), row stride
// pws, plane size pws * pph dwords. Same-level nodes of one rotation sit on
// one P-lattice, so one point's lookups by sibling nodes are adjacent dwords.
__global__ void pyramid_quad(const uint8_t* __restrict__ level, int wnx, int wny, int log_h, int km1,
                             uint32_t* __restrict__ out, int qw, int qh, int pws, int pph,
                             int total) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= total) return;
  const int h = 1 << log_h;
  const int s = log_h + 1, p = 2 * h;
  const int ps = pws * pph;
  const int pi = o / ps, k = o - pi * ps;
  const int fx = pi & (p - 1), fy = pi >> s;
  const int ky = k / pws, kx = k - ky * pws;
  const int xq = (kx << s) + fx, yq = (ky << s) + fy;
  uint32_t v = 0;
  if (xq < qw && yq < qh) {
    const int X = xq - h, Y = yq - h;
    auto g = [&](int a, int b) -> uint32_t {
      return (a >= 0 && b >= 0 && a < wnx && b < wny) ? level[static_cast<size_t>(b) * wnx + a] : 0u;
    };
    // G_d wide index of M-wide cell m is m - km1.
    auto m = [&](int a, int b) -> uint32_t {
      a -= km1;
      b -= km1;
      return max(max(g(a, b), g(a + km1, b)), max(g(a, b + km1), g(a + km1, b + km1)));
    };
    v = m(X, Y) | (m(X, Y + h) << 8) | (m(X + h, Y) << 16) | (m(X + h, Y + h) << 24);
  }
  out[o] = v;
}

// The widened level M (row-major, mw = wnx + km1 by mh = wny + km1): M-wide
// cell (X, Y) is the max of G_d at wide cells {X - km1, X} x {Y - km1, Y}
// (level 0 over [c, c + h + km1) per axis), 0 outside. Input of pyramid_hex.
__global__ void pyramid_widen(const uint8_t* __restrict__ level, int wnx, int wny, int km1,
                              uint8_t* __restrict__ out, int mw, int mh) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= mw || y >= mh) return;
  auto g = [&](int a, int b) -> uint32_t {
    return (a >= 0 && b >= 0 && a < wnx && b < wny) ? level[static_cast<size_t>(b) * wnx + a] : 0u;
  };
  const int a = x - km1, b = y - km1;
  out[static_cast<size_t>(y) * mw + x] =
      static_cast<uint8_t>(max(max(g(a, b), g(a + km1, b)), max(g(a, b + km1), g(a + km1, b + km1))));
}

// Hex layout of level d (h = 2^d, search kernel v5): the 16-byte entry for
// hex cell (X', Y'), X' < qw = mw + 3h, packs the 16 grandchildren values of a
// level-(d + 2) node whose child (0,0) sits at M-wide cell (X, Y) =
// (X' - 3h, Y' - 3h): dword a, byte b = M(X + a h, Y + b h); 0 outside.
// Polyphase with period P = 4h: plane (X' mod P, Y' mod P), entry
// (X' / P, Y' / P), so sibling nodes' lookups of one point are adjacent
// entries.
__global__ void pyramid_hex(const uint8_t* __restrict__ mlev, int mw, int mh, int log_h,
                            void* __restrict__ out, int qw, int qh, int pws, int pph, int total) {
  const int o = blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= total) return;
  const int h = 1 << log_h;
  const int s = log_h + 2, p = 4 * h;
  const int ps = pws * pph;
  const int pi = o / ps, k = o - pi * ps;
  const int fx = pi & (p - 1), fy = pi >> s;
  const int ky = k / pws, kx = k - ky * pws;
  const int xq = (kx << s) + fx, yq = (ky << s) + fy;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  if (xq < qw && yq < qh) {
    const int X = xq - 3 * h, Y = yq - 3 * h;
    auto m = [&](int a, int b) -> uint32_t {
      return (a >= 0 && b >= 0 && a < mw && b < mh) ? mlev[static_cast<size_t>(b) * mw + a] : 0u;
    };
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int xa = X + a * h;
      w[a] = m(xa, Y) | (m(xa, Y + h) << 8) | (m(xa, Y + 2 * h) << 16) | (m(xa, Y + 3 * h) << 24);
    }
  }
  static_cast<uint4*>(out)[o] = make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------- K2-K4 v4 -
//
// A workgroup (4 waves) searches a chunk of R rotations of one pair at once.
// Each rotation's discretized scan becomes up to four entry lists: runs of
// consecutive points in one cell (k = 1) and runs of consecutive points in
// one k x k cluster (k = 2, 4, 8), each entry weighted by its point count.
// A node at level d scores its 2x2 children at level d - 1 over the list of
// that level's cluster size against quad level d - 1, whose values are
// widened by k - 1 cells (SubmapDesc::cshift): every point of a cluster lies
// in [q, q + k), so the cluster's count times the widened max bounds the
// points' own terms. Leaves (level 0) use k = 1 and the exact values. The
// bounds are looser than the reference's at coarse levels, so more inner
// nodes survive, but every leaf that can reach the best sum is still scored
// exactly: the result is unchanged.
//
// The DFS stack mixes the chunk's rotations; a batch pops up to 64 nodes
// (deepest level first, best bound first): a thread takes one node and a
// strided subset of that node's list (flat lanes, below), and per entry issues
// ONE dword load from the quad layout that returns all four children's
// values. The threads' sums meet in LDS; all waves combine, prune and push
// survivors sorted (best on top), wave 0 pops the next batch. Roots are
// virtual nodes one level above the top lattice.

#ifndef CSM_U_QUAD
#define CSM_U_QUAD 8  // quad gathers in flight per lane (V4Score)
#endif
#ifndef CSM_U_HEX
#define CSM_U_HEX 4   // hex gathers in flight per lane (V4ScoreHex)
#endif
// Scoring lanes (V4Score, V4ScoreHex): the 4 waves' 256 threads take (node,
// chunk) pairs, node = t mod nodes, chunk = t / nodes, and chunk c of C =
// 256 / nodes walks entries c, c + C, ... of the node's list (a batch of 36
// nodes issues 7 chunks' worth of lanes instead of 4 waves x 36 lanes); the
// sums meet through LDS atomics (C3 launch 571.4 -> 569.0 ms, profiles/r5ba).
constexpr int kMaxRotChunk = kV4MaxRotChunk;
constexpr int kLists = kMaxClusterShift + 1;

// kKids: children sums per node, 4 (quad batches only, v4) or 16 (v5: hex
// batches, and the virtual roots' quad batches in the first 4 columns).
template <int kKids>
struct V4Shared {
  // LDS part of the DFS stack (v5: a quarter, so 6 workgroups fit a CU's
  // LDS with their 16-child sums); the rest spills to global memory.
  static constexpr int kStackLds = kKids == 16 ? kStack2 / 4 : kStack2;
  static constexpr int kStackCapacity = kStackLds + kSpill2;
  uint2 stack[kStackLds];  // w0: xo | yo << 16; w1: sum | rot << 22 | level << 27
  int part[kBatchNodes][kKids];  // children sums, accumulated by the 4 waves (LDS atomics)
  int batch_hex;                 // the batch's nodes score 16 grandchildren (v5)
  int head;                      // FIFO: LDS ring position of the oldest entry
  int ovf;                       // FIFO: entries in the global overflow stack
  int list_off[kMaxRotChunk][kLists];  // entry list (rotation, cluster shift): first entry
  int list_len[kMaxRotChunk][kLists];  // and length; a list that did not fit aliases a finer one
  int node_xo[kBatchNodes], node_yo[kBatchNodes], node_rot[kBatchNodes], node_level[kBatchNodes];
  int node_off[kBatchNodes], node_len[kBatchNodes];  // the node's children-level list
  int nodes, done, batch_len, batch_entries;
  int tie_sum;  // a sum the pair's witness keys already show two leaves at (-1: none)
  int item_pair, item_chunk, queue;
  int sp;
  uint64_t best;
  int mm[kMaxRotChunk][4];
  int bounds[kMaxRotChunk][4];
  int vny[kMaxRotChunk];
  int root_prefix[kMaxRotChunk + 1];
  int vnext;
  int range_error, batch_no, high_water, long_runs;
  // The submap's per-level quad layout (SubmapDesc), cached per item so the
  // batch loop reads LDS, not lane-divergent global loads: quad_w, quad_h,
  // quad_off, 4 * quad_pws, plane bytes, quad_bias, cshift.
  int lv[kMaxLevels][8];
#ifdef CSM_KPROF
  unsigned long long kp_lines[kMaxLevels], kp_instr[kMaxLevels], kp_qlines[kMaxLevels];
  unsigned long long kp_active[kMaxLevels], kp_oob[kMaxLevels];
#endif
};

// The DFS stack: entries [0, kStackLds) in LDS, [kStackLds, kStackLds + kSpill2)
// in the workgroup's spill region (global memory; the workgroup's own waves
// write and read it, ordered by the __syncthreads between phases).
template <typename Shared>
__device__ __forceinline__ uint2 StackGet(const Shared& sh, const uint2* spill, int i) {
  return i < Shared::kStackLds ? sh.stack[i] : spill[i - Shared::kStackLds];
}
template <typename Shared>
__device__ __forceinline__ void StackPut(Shared& sh, uint2* spill, int i, uint2 v) {
  if (i < Shared::kStackLds) sh.stack[i] = v; else spill[i - Shared::kStackLds] = v;
}

#ifdef CSM_KPROF
// Distinct 128-byte lines among the executing lanes' in-range addresses of
// one gather (instrumentation only: 63 shuffles).
template <typename Shared>
__device__ void CountLines(Shared& sh, int level, int ad, int oob) {
  const int lane = threadIdx.x & 63;
  const bool valid = ad != oob;
  const int line = valid ? (ad >> 7) : -1 - lane;
  bool first = valid;
  for (int j = 1; j < 64; ++j) {
    const int o = __shfl(line, (lane + 64 - j) & 63, 64);
    if (lane >= j && o == line) first = false;
  }
  // First lane of its line within its 4-lane group.
  bool qfirst = valid;
  for (int j = 1; j < 4; ++j) {
    const int o = __shfl(line, (lane & ~3) | ((lane - j) & 3), 64);
    if ((lane & 3) >= j && o == line) qfirst = false;
  }
  const int n = __popcll(__ballot(first));
  const int nq = __popcll(__ballot(qfirst));
  const int na = __popcll(__ballot(true));
  const int no = __popcll(__ballot(!valid));
  const int lv = __builtin_amdgcn_readfirstlane(level);
  if (__builtin_amdgcn_readfirstlane(lane) == lane) {
    atomicAdd(&sh.kp_lines[lv], static_cast<unsigned long long>(n));
    atomicAdd(&sh.kp_instr[lv], 1ull);
    atomicAdd(&sh.kp_qlines[lv], static_cast<unsigned long long>(nq));
    atomicAdd(&sh.kp_active[lv], static_cast<unsigned long long>(na));
    atomicAdd(&sh.kp_oob[lv], static_cast<unsigned long long>(no));
  }
}
#define CSM_COUNT_LINES(lvl, ad, oob) CountLines(sh, (lvl), (ad), (oob))
#else
#define CSM_COUNT_LINES(lvl, ad, oob)
#endif

// Scores the children of the batch's nodes: lane (node, group) walks entries
// g, g + groups, ... of the node's list (cells, counts). A child's sum is
// sum_k cnt[k] * value over the list: the reference's per-point sum
// regrouped at level 0, an upper bound of it at coarser levels.
template <typename Shared>
__device__ __forceinline__ void V4Score(Shared& sh, const uint32_t* cells, const uint8_t* cnts,
                                        int raw_end, const SubmapDesc& sm) {
  const int nodes = Uniform(sh.nodes);
  // Thread -> (node, chunk); chunk g of `groups` walks entries g, g + groups, ...
  const int groups = kSearchThreads / nodes;
  const int g = static_cast<int>(threadIdx.x) / nodes;
  const bool active = g < groups;
  const int node = active ? static_cast<int>(threadIdx.x) - g * nodes : 0;
  // Each node scores its children at its own child level: one descriptor
  // spans the whole pyramid, the level is a per-lane byte offset.
  const int level = sh.node_level[node] - 1;
  const int* L = sh.lv[level];
  const int qw = L[0], qh = L[1], qoff = L[2], pws4 = L[3], ps4 = L[4];
  const int sft = level + 1, pmask = (2 << level) - 1;
  const __amdgpu_buffer_rsrc_t rsrc = LevelRsrc(sm.pyramid_base, Uniform(sm.pyramid_bytes));
  const int off = sh.node_off[node], len = sh.node_len[node];
  const uint32_t* P = cells + off;
  // Raw scans (cells [0, raw_end)) weigh every entry 1 and store no counts;
  // cluster lists keep theirs at cnts[offset - raw_end].
  const bool raw = off < raw_end;
  const uint8_t* Cn = cnts + (raw ? 0 : off - raw_end);
  const int cx = sh.node_xo[node] + L[5];
  const int cy = sh.node_yo[node] + L[5];
  const int blen = Uniform(sh.batch_len);
  // Entry indices i + g for i = 0, groups, ... up to the batch's longest list.
  const int s = 0, e = Uniform((blen + groups - 1) / groups * groups);
  constexpr int kOOB = 0x7ffffff0;
  constexpr int U = CSM_U_QUAD;
  uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
  auto address = [&](uint32_t p, bool in) {
    const int X = static_cast<int16_t>(p & 0xffff) + cx;
    const int Y = (static_cast<int>(p) >> 16) + cy;
    const bool valid = in && static_cast<unsigned>(X) < static_cast<unsigned>(qw) &&
                       static_cast<unsigned>(Y) < static_cast<unsigned>(qh);
    const int a = __umul24((((Y & pmask) << sft) | (X & pmask)), ps4) + qoff;
    const int b = __umul24(Y >> sft, pws4) + a;
    return valid ? ((X >> sft) << 2) + b : kOOB;
  };
  // v_dot4_u32_u8 with the entry's count in one byte of the weight
  // multiplies that child's byte by the count and accumulates.
  auto accumulate = [&](uint32_t v, uint32_t c) {
    a0 = __builtin_amdgcn_udot4(v, c, a0, false);
    a1 = __builtin_amdgcn_udot4(v, c << 8, a1, false);
    a2 = __builtin_amdgcn_udot4(v, c << 16, a2, false);
    a3 = __builtin_amdgcn_udot4(v, c << 24, a3, false);
  };
  // U entries per lane in flight, then the remainder one at a time: every
  // issued load costs texture-path cycles even when its lanes are out of
  // range, so the tail issues no more loads than it needs.
  if (active) {  // the missing nodes' lanes issue no loads
    int i = s;
    for (; i + U * groups <= e; i += U * groups) {
      int ad[U];
      uint32_t c[U];
  #pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = i + u * groups + g;
        const bool in = idx < len;
        const int j = in ? idx : 0;
        ad[u] = address(P[j], in);
        c[u] = in ? (raw ? 1u : Cn[j]) : 0u;
      }
      for (int u = 0; u < U; ++u) CSM_COUNT_LINES(level, ad[u], kOOB);
      uint32_t v[U];
  #pragma unroll
      for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, ad[u], 0, 0);
  #pragma unroll
      for (int u = 0; u < U; ++u) accumulate(v[u], c[u]);
    }
    for (; i < e; i += groups) {
      const int idx = i + g;
      const bool in = idx < e && idx < len;
      const int j = in ? idx : 0;
      const uint32_t vv = __builtin_amdgcn_raw_buffer_load_b32(rsrc, address(P[j], in), 0, 0);
      accumulate(vv, in ? (raw ? 1u : Cn[j]) : 0u);
    }
  }
  if (active && (a0 | a1 | a2 | a3) != 0u) {
    atomicAdd(&sh.part[node][0], static_cast<int>(a0));  // (xo,     yo)
    atomicAdd(&sh.part[node][1], static_cast<int>(a1));  // (xo,     yo + h)
    atomicAdd(&sh.part[node][2], static_cast<int>(a2));  // (xo + h, yo)
    atomicAdd(&sh.part[node][3], static_cast<int>(a3));  // (xo + h, yo + h)
  }
}

// Hex batches (v5): a node at level L scores its 16 grandchildren at level
// c = L - 2, (xo + a h, yo + b h), a, b in 0..3, h = 2^c, over the list of
// level c's cluster size, with ONE 16-byte load per entry from level c's hex
// plane (dword a, byte b). The intermediate level's pruning is skipped: its
// bounds are only ever >= the grandchildren's, so the search still visits
// every leaf that can reach the best sum.
template <typename Shared>
__device__ __forceinline__ void V4ScoreHex(Shared& sh, const uint32_t* cells, const uint8_t* cnts,
                                           int raw_end, const SubmapDesc& sm) {
  const int nodes = Uniform(sh.nodes);
  const int groups = kSearchThreads / nodes;  // as V4Score
  const int g = static_cast<int>(threadIdx.x) / nodes;
  const bool active = g < groups;
  const int node = active ? static_cast<int>(threadIdx.x) - g * nodes : 0;
  const int level = sh.node_level[node] - 2;
  const int* L = sh.lv[level];
  const int qw = L[0], qh = L[1], qoff = L[2], pws16 = L[3], ps16 = L[4];
  const int sft = level + 2, pmask = (4 << level) - 1;
  const __amdgpu_buffer_rsrc_t rsrc = LevelRsrc(sm.pyramid_base, Uniform(sm.pyramid_bytes));
  const int off = sh.node_off[node], len = sh.node_len[node];
  const uint32_t* P = cells + off;
  // Raw scans (cells [0, raw_end)) weigh every entry 1 and store no counts;
  // cluster lists keep theirs at cnts[offset - raw_end].
  const bool raw = off < raw_end;
  const uint8_t* Cn = cnts + (raw ? 0 : off - raw_end);
  const int cx = sh.node_xo[node] + L[5];
  const int cy = sh.node_yo[node] + L[5];
  const int blen = Uniform(sh.batch_len);
  const int s = 0, e = Uniform((blen + groups - 1) / groups * groups);
  constexpr int kOOB = 0x7ffffff0;
  constexpr int U = CSM_U_HEX;
  uint32_t acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0u;
  auto address = [&](uint32_t p, bool in) {
    const int X = static_cast<int16_t>(p & 0xffff) + cx;
    const int Y = (static_cast<int>(p) >> 16) + cy;
    const bool valid = in && static_cast<unsigned>(X) < static_cast<unsigned>(qw) &&
                       static_cast<unsigned>(Y) < static_cast<unsigned>(qh);
    const int a = __umul24((((Y & pmask) << sft) | (X & pmask)), ps16) + qoff;
    const int b = __umul24(Y >> sft, pws16) + a;
    return valid ? ((X >> sft) << 4) + b : kOOB;
  };
  using HexVec = decltype(__builtin_amdgcn_raw_buffer_load_b128(rsrc, 0, 0, 0));
  auto hload = [&](int ad) { return __builtin_amdgcn_raw_buffer_load_b128(rsrc, ad, 0, 0); };
  // Child (a, b) accumulates byte b of dword a times the entry's count.
  auto accumulate = [&](const HexVec& v, uint32_t c) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        acc[4 * a + b] = __builtin_amdgcn_udot4(v[a], c << (8 * b), acc[4 * a + b], false);
    }
  };
  if (active) {  // the missing nodes' lanes issue no loads
    int i = s;
    for (; i + U * groups <= e; i += U * groups) {
      int ad[U];
      uint32_t c[U];
  #pragma unroll
      for (int u = 0; u < U; ++u) {
        const int idx = i + u * groups + g;
        const bool in = idx < len;
        const int j = in ? idx : 0;
        ad[u] = address(P[j], in);
        c[u] = in ? (raw ? 1u : Cn[j]) : 0u;
      }
      for (int u = 0; u < U; ++u) CSM_COUNT_LINES(level, ad[u], kOOB);
      HexVec v[U];
  #pragma unroll
      for (int u = 0; u < U; ++u) v[u] = hload(ad[u]);
  #pragma unroll
      for (int u = 0; u < U; ++u) accumulate(v[u], c[u]);
    }
    for (; i < e; i += groups) {
      const int idx = i + g;
      const bool in = idx < e && idx < len;
      const int j = in ? idx : 0;
      const HexVec vv = hload(address(P[j], in));
      accumulate(vv, in ? (raw ? 1u : Cn[j]) : 0u);
    }
  }
  if (active) {
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (acc[j] != 0u) atomicAdd(&sh.part[node][j], static_cast<int>(acc[j]));
  }
}

// Cluster key of a packed cell (int16 x | int16 y << 16): both coordinates
// rounded down to a multiple of 2^shift.
__device__ __forceinline__ uint32_t ClusterKey(uint32_t p, int shift) {
  const int x = (static_cast<int16_t>(p & 0xffff) >> shift) << shift;
  const int y = ((static_cast<int>(p) >> 16) >> shift) << shift;
  return (static_cast<uint32_t>(x) & 0xffff) | (static_cast<uint32_t>(y) << 16);
}

// One wave sweeps the n raw cells of a rotation (src) and makes its run list
// at cluster mask `mask` (both cell coordinates rounded down to a multiple
// of k = 2^sl: the cell word with the low sl bits of each half cleared):
// consecutive points with the same key become one entry, the key and the
// number of points (<= 255: a longer run splits at multiples of 255 from its
// start). kWrite = false only counts. Writing in place (P == src, mask all
// ones) is safe: entry k <= point i, and a block's cells are in registers
// before any write. Per block: one compare and ballot for the run heads, the
// entry index by mbcnt, the count as the distance to the next head; the
// 255-split scan runs only in blocks a run can reach 255 in.
template <bool kWrite>
__device__ int RunList(const uint32_t* src, int n, uint32_t mask, uint32_t* P, uint8_t* C) {
  const int lane = threadIdx.x & 63;
  const unsigned long long upto = (2ull << lane) - 1;  // lanes <= this one (lane 63: all)
  int out = 0, run_start = 0, open_k = -1, open_pos = 0;
  uint32_t last = 0;
  uint32_t nextv = lane < n ? src[lane] : 0u;  // the next block's cells, loaded a block ahead
  for (int base = 0; base < n; base += 64) {
    const int i = base + lane;
    const bool in = i < n;
    const uint32_t v = nextv;
    nextv = i + 64 < n ? src[i + 64] : 0u;
    uint32_t prev = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(
        0, static_cast<int>(v), 0x138, 0xF, 0xF, false));  // wave_shr:1
    if (lane == 0) prev = last;
    const bool head0 = in && (i == 0 || ((v ^ prev) & mask) != 0u);
    const unsigned long long h0 = __ballot(head0);
    unsigned long long hm = h0;
    if (base + 63 - run_start >= 255) {  // a run may pass 255 points in this block
      const unsigned long long mine = h0 & upto;
      const int rs = mine ? base + 63 - __clzll(mine) : run_start;
      hm = __ballot(head0 || (in && i > rs && (i - rs) % 255 == 0));
    }
    if (kWrite) {
      if (open_k >= 0 && hm) {  // close the entry left open by the previous block
        if (lane == 0) C[open_k] = static_cast<uint8_t>(base + __ffsll(static_cast<long long>(hm)) - 1 - open_pos);
        open_k = -1;
      }
      if ((hm >> lane) & 1ull) {
        const int k = out + static_cast<int>(__builtin_amdgcn_mbcnt_hi(
                                static_cast<uint32_t>(hm >> 32),
                                __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(hm), 0u)));
        P[k] = v & mask;
        const unsigned long long rest = lane < 63 ? hm >> (lane + 1) : 0ull;
        if (rest) C[k] = static_cast<uint8_t>(__ffsll(static_cast<long long>(rest)));
      }
      if (hm) {
        open_k = out + __popcll(hm) - 1;
        open_pos = base + 63 - __clzll(hm);
      }
    }
    out += __popcll(hm);
    if (h0) run_start = base + 63 - __clzll(h0);
    last = __builtin_amdgcn_readlane(v, 63);
  }
  if (kWrite && open_k >= 0 && lane == 0) C[open_k] = static_cast<uint8_t>(n - open_pos);
  return out;
}

__device__ __forceinline__ uint32_t ClusterMask(int sl) {
  const uint32_t h = (0xffffu << sl) & 0xffffu;
  return h | (h << 16);
}

// kHex = false: v4 (every node scores its 4 children from the quad planes).
// kHex = true: v5 (nodes of the levels in SubmapDesc::hex_mask score their
// 16 grandchildren from hex planes, the others their 4 children from quad
// planes; a batch holds one kind).
//
// kFifo = false: the stack is LIFO with the deepest level on top (depth-first,
// early leaves). kFifo = true: a FIFO ring (level by level: batches fill up
// with the whole frontier of a level; leaves come last).
#ifndef CSM_BEST_REFRESH
#define CSM_BEST_REFRESH 1  // batches between reads of the pair's global best (power of 2; profiles/r3ap)
#endif
#ifndef CSM_LIFO_LEVEL
#define CSM_LIFO_LEVEL 2  // FIFO order: levels pushed depth-first (0: none; profiles/r3an)
#endif
#ifndef CSM_XFAST
// Children and roots enter the stack x-fastest, so consecutive lanes of the
// next batch score nodes adjacent in x: adjacent entries of a polyphase plane
// (DESIGN.md §5).
#define CSM_XFAST 1
#endif
#ifndef CSM_ORIGIN_ALIGN
// The node lattice of a rotation starts at its ShrinkToFit corner (b0, b2)
// rounded down to a multiple of this power of two (>= the largest cluster,
// 2^kMaxClusterShift), and nodes wholly below the corner are dropped, so the
// leaves are still exactly the reference's [b0, b1] x [b2, b3]. Every node's
// offset is then a multiple of 8 at levels >= 3, and a cluster entry's cell
// a multiple of its cluster size, so the plane entries a level's cluster
// lists can address lie in one residue class: 1/16 of the level-2..4 planes
// and 1/64 of the level-6 hex plane, the same class for every pair and
// rotation, instead of all of them across a chunk's items. The planes'
// touched footprint shrinks to what one XCD's L2 holds. 1: the reference's
// corner (no alignment).
#define CSM_ORIGIN_ALIGN 8
#endif
static_assert((CSM_ORIGIN_ALIGN & (CSM_ORIGIN_ALIGN - 1)) == 0, "CSM_ORIGIN_ALIGN: a power of two");
#ifndef CSM_TIE_PRUNE
// 1: the main search stops expanding nodes bounded by a sum its witness keys
// already show tied (FindsConstraints-like inputs: every leaf ties).
#define CSM_TIE_PRUNE 1
#endif
#ifndef CSM_V4_WAVES
// Waves per SIMD the register budget targets: 6 workgroups per CU (v5 with
// its 256-entry LDS ring fits 6 in LDS too; measured best).
#define CSM_V4_WAVES 6
#endif
// kCollect: the tie-enumeration launch (PairDesc::collect_sum, csm_host.cc
// ResolveTies), its own symbol so profiles tell it from the search.
template <bool kHex, bool kFifo, bool kCollect>
__global__ void __launch_bounds__(kSearchThreads) __attribute__((amdgpu_waves_per_eu(CSM_V4_WAVES)))
fast2d_search_v4(const SubmapDesc* __restrict__ submaps,
                 const PairDesc* __restrict__ pairs,
                 const float* __restrict__ points,
                 const float2* __restrict__ rot_table,
                 WorkQueues2 queues,
                 unsigned long long* __restrict__ counters,
                 uint64_t* __restrict__ best,
                 int32_t* __restrict__ status,
                 unsigned long long* __restrict__ stats,
                 uint2* __restrict__ spill_base, int npad, int capc,
                 uint64_t* __restrict__ best_hi, uint2* __restrict__ ties,
                 int32_t* __restrict__ tie_count) {
  // Dynamic LDS: cells, rc * (npad + capc) words, then the cluster lists'
  // counts, rc * capc bytes. Rotation r's raw cells at r * npad; its cluster
  // lists packed in [rc * npad + r * capc, + capc).
  constexpr int kKids = kHex ? 16 : 4;
  extern __shared__ __align__(16) uint32_t cells[];
  __shared__ V4Shared<kKids> sh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rc = queues.rot_chunk;
  // Counts of the cluster lists only (the raw scans weigh 1): entry at cell
  // offset o has its count at cnts[o - rc * npad].
  uint8_t* cnts = reinterpret_cast<uint8_t*>(cells + rc * (npad + capc));
  const int raw_end = rc * npad;
  uint2* spill = spill_base + static_cast<size_t>(blockIdx.x) * kSpill2;
  for (int k = tid; k < kBatchNodes * kKids; k += kSearchThreads) sh.part[k / kKids][k % kKids] = 0;
  if (tid == 0) sh.batch_hex = 0;
  if (tid == 0) sh.high_water = 0;
  unsigned long long local_cands = 0, local_lookups = 0;
#ifdef CSM_KPROF
  long long kprof[4] = {0, 0, 0, 0};  // thread 0: setup, control, score cycles; lists (part of setup)
#endif
  if (tid == 0) sh.queue = blockIdx.x % kNumXcd;
  unsigned long long lv_cands = 0, lv_batches = 0;  // wave 0, lane l: child level l
#ifdef CSM_KPROF
  if (tid < kMaxLevels) {
    sh.kp_lines[tid] = 0; sh.kp_instr[tid] = 0; sh.kp_qlines[tid] = 0;
    sh.kp_active[tid] = 0; sh.kp_oob[tid] = 0;
  }
#endif
  int tries = 0;
  __syncthreads();
  for (;;) {
    // ---- claim (pair, rotation chunk) from an XCD-affine queue ------------
    if (tid == 0) {
      int q = sh.queue, pair = -1, chunk = 0;
      while (tries < kNumXcd) {
        const int64_t item = static_cast<int64_t>(atomicAdd(&counters[q], 1ull));
        if (item < queues.queue_chunks[q]) {
          const int64_t gch = queues.chunk_prefix[queues.queue_begin[q]] + item;
          int e = queues.block_first[queues.block_offset[q] + static_cast<int>(item >> 6)];
          while (queues.chunk_prefix[e + 1] <= gch) ++e;
          pair = queues.pair_order[e];
          chunk = static_cast<int>(gch - queues.chunk_prefix[e]);
          break;
        }
        q = (q + 1) % kNumXcd;
        ++tries;
      }
      sh.queue = q;
      sh.item_pair = pair;
      sh.item_chunk = chunk;
    }
    __syncthreads();
    const int pair_index = Uniform(sh.item_pair);
    if (pair_index < 0) break;
    const PairDesc pd = pairs[pair_index];
    const SubmapDesc& sm = submaps[pd.submap];
    const int n = pd.num_points;
    const int s_min = pd.max_rejected_sum;
    const int collect_sum = kCollect ? pd.collect_sum : -1;
    uint64_t* pair_best = best + pair_index;
    const int rot0 = Uniform(sh.item_chunk) * rc;
    const int nrot = min(rc, pd.num_scans - rot0);
    const int top_level = sm.levels - 1;
    const int step = 1 << top_level;
    const uint32_t hex_mask = kHex ? static_cast<uint32_t>(Uniform(sm.hex_mask)) : 0u;

    // ---- K2: discretize the chunk's rotated scans into LDS ----------------
#ifdef CSM_KPROF
    long long t_mark = clock64();
#endif
    if (tid < kMaxRotChunk * 4) sh.mm[tid >> 2][tid & 3] = (tid & 1) ? -0x7fffffff : 0x7fffffff;
    if (tid == 0) sh.range_error = 0;
    if (tid < sm.levels) {
      const int d = tid;
      sh.lv[d][0] = sm.quad_w[d];
      sh.lv[d][1] = sm.quad_h[d];
      sh.lv[d][2] = sm.quad_off[d];
      sh.lv[d][3] = sm.quad_pws[d] * sm.quad_es[d];
      sh.lv[d][4] = sm.quad_pws[d] * sm.quad_pph[d] * sm.quad_es[d];
      sh.lv[d][5] = sm.quad_bias[d];
      sh.lv[d][6] = sm.cshift[d];
    }
    __syncthreads();
    const double inv_res = 1.0 / sm.resolution;  // CellCoordFast
    bool range_error = false;
    for (int r = 0; r < nrot; ++r) {
      const float2 q = rot_table[pd.rot_offset + rot0 + r];
      int mnx = 0x7fffffff, mxx = -0x7fffffff, mny = 0x7fffffff, mxy = -0x7fffffff;
      for (int i = tid; i < n; i += kSearchThreads) {
        const float* p = points + 3 * (pd.point_offset + i);
        float x, y;
        RotateZDev(pd.pre_w, pd.pre_s, p[0], p[1], &x, &y);
        RotateZDev(q.x, q.y, x, y, &x, &y);
        const float px = __fadd_rn(pd.tx, x);
        const float py = __fadd_rn(pd.ty, y);
        const double cx = CellCoordFast(sm.max_y, py, sm.resolution, inv_res);
        const double cy = CellCoordFast(sm.max_x, px, sm.resolution, inv_res);
        int ix = 0, iy = 0;
        if (fabs(cx) > kIndexLimit || fabs(cy) > kIndexLimit) {
          range_error = true;
        } else {
          ix = static_cast<int>(cx);
          iy = static_cast<int>(cy);
        }
        mnx = min(mnx, ix); mxx = max(mxx, ix);
        mny = min(mny, iy); mxy = max(mxy, iy);
        cells[r * npad + i] = (static_cast<uint32_t>(ix) & 0xffff) | (static_cast<uint32_t>(iy) << 16);
      }
      mnx = WaveMin(mnx); mxx = WaveMax(mxx); mny = WaveMin(mny); mxy = WaveMax(mxy);
      if (lane == 0) {
        atomicMin(&sh.mm[r][0], mnx); atomicMax(&sh.mm[r][1], mxx);
        atomicMin(&sh.mm[r][2], mny); atomicMax(&sh.mm[r][3], mxy);
      }
    }
    if (range_error) sh.range_error = 1;
#ifdef CSM_DBG
    if (range_error) printf("discretize range\n");
#endif
    __syncthreads();
    // ---- Entry lists: k = 1 is the discretized scan itself (one point per
    // entry; it scores the leaves only), k = 2, 4, 8 are run lists of cluster
    // keys. All threads count the runs of all three; the lists are packed
    // into the rotation's capc region coarsest first (one that does not fit
    // aliases the next finer list); then one wave per (rotation, list) sweep
    // writes them -------------------------------------------------------------
    {
#ifdef CSM_KPROF
      const long long t_lists = clock64();
#endif
      // A rotation whose coarsest keys repeat 255 points apart may hold a run
      // past 255 points (split entries): its lists are counted by a sweep.
      if (tid < nrot * kLists) sh.list_len[tid / kLists][tid % kLists] = tid % kLists == 0 ? n : 0;
      if (tid == 0) sh.long_runs = 0;
      __syncthreads();
      for (int r = 0; r < nrot; ++r) {
        const uint32_t* raw = cells + r * npad;
        uint32_t c1 = 0, c23 = 0;  // run heads of k = 2 | k = 4, k = 8 (16-bit fields)
        bool long_run = false;
        for (int i = tid; i < n; i += kSearchThreads) {
          const uint32_t v = raw[i];
          const uint32_t d = i == 0 ? 0xffffffffu : v ^ raw[i - 1];
          c1 += (d & ClusterMask(1)) != 0u;
          c23 += ((d & ClusterMask(2)) != 0u) | (static_cast<uint32_t>((d & ClusterMask(3)) != 0u) << 16);
          long_run |= i >= 255 && ((v ^ raw[i - 255]) & ClusterMask(kMaxClusterShift)) == 0u;
        }
        c1 = DppSum(c1);
        c23 = DppSum(c23);
        if (lane == 0) {
          atomicAdd(&sh.list_len[r][1], static_cast<int>(c1));
          atomicAdd(&sh.list_len[r][2], static_cast<int>(c23 & 0xffff));
          atomicAdd(&sh.list_len[r][3], static_cast<int>(c23 >> 16));
        }
        if (__ballot(long_run) && lane == 0) atomicOr(&sh.long_runs, 1 << r);
      }
      __syncthreads();
      if (const int lr = sh.long_runs) {
        for (int t = wave; t < nrot * kMaxClusterShift; t += kWaves) {
          const int r = t / kMaxClusterShift, sl = 1 + t % kMaxClusterShift;
          if (lr >> r & 1) {
            const int len = RunList<false>(cells + r * npad, n, ClusterMask(sl), nullptr, nullptr);
            if (lane == 0) sh.list_len[r][sl] = len;
          }
        }
        __syncthreads();
      }
      // The cluster sizes some level scores with (SubmapDesc::cshift); an
      // unused list is not written and aliases the next finer one.
      uint32_t used_sl = 0;
      for (int d = 0; d < sm.levels; ++d) used_sl |= 1u << sh.lv[d][6];
      if (tid < nrot) {
        const int r = tid;
        sh.list_off[r][0] = r * npad;
        int used = 0;
        int off[kLists] = {r * npad, -1, -1, -1};
        for (int sl = kMaxClusterShift; sl >= 1; --sl)
          if ((used_sl >> sl & 1u) && used + sh.list_len[r][sl] <= capc) {
            off[sl] = rc * npad + r * capc + used;
            used += sh.list_len[r][sl];
          }
        for (int sl = 1; sl < kLists; ++sl) {
          if (off[sl] >= 0) {
            sh.list_off[r][sl] = off[sl];
          } else {  // does not fit: the finer list bounds this level too
            sh.list_off[r][sl] = sh.list_off[r][sl - 1];
            sh.list_len[r][sl] = sh.list_len[r][sl - 1] | (1 << 30);
          }
        }
      }
      __syncthreads();
      // Tasks (rotation, used list) dealt to the waves.
      const int nused = __popc(used_sl & 0xeu);
      for (int t = wave; t < nrot * nused; t += kWaves) {
        const int r = t / nused;
        int sl = 0;
        for (int k = t % nused, m = used_sl & 0xe; k >= 0; --k) {
          sl = __ffs(m) - 1;
          m &= m - 1;
        }
        if (!(sh.list_len[r][sl] & (1 << 30)))
          RunList<true>(cells + r * npad, n, ClusterMask(sl), cells + sh.list_off[r][sl],
                        cnts + (sh.list_off[r][sl] - raw_end));
      }
      __syncthreads();
      if (tid < nrot * kLists) sh.list_len[tid / kLists][tid % kLists] &= ~(1 << 30);
      __syncthreads();
#ifdef CSM_KPROF
      if (tid == 0) kprof[3] += clock64() - t_lists;
#endif
    }
    // ---- ShrinkToFit per rotation; root counts ------------------------------
    if (tid < nrot) {
      const int r = tid;
      const int lo_x = min(0, -sh.mm[r][1]), hi_x = max(0, sm.nx - 1 - sh.mm[r][0]);
      const int lo_y = min(0, -sh.mm[r][3]), hi_y = max(0, sm.ny - 1 - sh.mm[r][2]);
      const int b0 = max(-pd.num_linear, lo_x), b1 = min(pd.num_linear, hi_x);
      const int b2 = max(-pd.num_linear, lo_y), b3 = min(pd.num_linear, hi_y);
      sh.bounds[r][0] = b0; sh.bounds[r][1] = b1; sh.bounds[r][2] = b2; sh.bounds[r][3] = b3;
      const int a0 = b0 & -CSM_ORIGIN_ALIGN, a2 = b2 & -CSM_ORIGIN_ALIGN;  // lattice origin
      const int tnx = (b1 - a0 + step) / step, tny = (b3 - a2 + step) / step;
      sh.vny[r] = (tny + 1) >> 1;
      sh.root_prefix[r + 1] = ((tnx + 1) >> 1) * sh.vny[r];
    }
    __syncthreads();
    if (tid == 0) {
      if (sh.range_error) atomicOr(&status[pair_index], kStatusRange);
      sh.root_prefix[0] = 0;
      for (int r = 0; r < nrot; ++r) sh.root_prefix[r + 1] += sh.root_prefix[r];
      sh.vnext = 0;
      sh.sp = 0;
      sh.ovf = 0;
      sh.head = 0;
      sh.best = LoadBest(pair_best);
      sh.tie_sum = -1;
      sh.batch_no = 0;
      sh.nodes = 0;
      sh.done = 0;
    }
    __syncthreads();
    const int vtotal = Uniform(sh.root_prefix[nrot]);
#ifdef CSM_KPROF
    if (tid == 0) {
      const long long now = clock64();
      kprof[0] += now - t_mark;
      t_mark = now;
    }
#endif

    // ---- K3/K4: batched best-first DFS over the chunk -----------------------
    for (;;) {
      {
        // (a) Combine the previous batch: prune, record leaves, push survivors.
        // 16 nodes' children per pass (one per lane); the waves take the
        // passes in parallel and claim stack space atomically.
        // Hex batches: 4 nodes' 16 grandchildren per pass, child c = (a, b)
        // at (xo + a h, yo + b h), a = c >> 2, b = c & 3.
        const int pn = sh.nodes;
        const bool hexb = kHex && sh.batch_hex;
        const int lk = hexb ? 4 : 2;  // log2 children per node
        const int per_pass = 64 >> lk;
        for (int pass = wave; pass * per_pass < pn; pass += kWaves) {
          const int nd = pass * per_pass + (lane >> lk), cl = lane & ((1 << lk) - 1);
          // Child c = (a, b) at (xo + a h, yo + b h) sits in lane (b, a)
          // order when CSM_XFAST (x fastest), else (a, b).
          const int hb = lk >> 1;
          const int c = CSM_XFAST ? (((cl & ((1 << hb) - 1)) << hb) | (cl >> hb)) : cl;
          int sum = 0, xo = 0, yo = 0, r = 0, clvl = 0;
          bool exists = false;
          if (nd < pn) {
            clvl = sh.node_level[nd] - (hexb ? 2 : 1);
            const int h = 1 << clvl;
            sum = sh.part[nd][c];
            sh.part[nd][c] = 0;
            r = sh.node_rot[nd];
            xo = sh.node_xo[nd] + (c >> (lk >> 1)) * h;
            yo = sh.node_yo[nd] + (c & ((1 << (lk >> 1)) - 1)) * h;
            // Inside the window: not past (b1, b3), and not wholly below
            // (b0, b2), which only the aligned origin's nodes can be.
            exists = xo <= sh.bounds[r][1] && yo <= sh.bounds[r][3] &&
                     xo + h > sh.bounds[r][0] && yo + h > sh.bounds[r][2];
          }
          const uint64_t cur = sh.best;
          const uint32_t cur_sum = static_cast<uint32_t>(cur >> kSumShift);
          const bool keep = exists && sum > s_min && static_cast<uint32_t>(sum) >= cur_sum;
          // Leaves (child level 0) update the incumbent.
          uint64_t key = 0;
          if (keep && clvl == 0) {
            if (xo < -kOffsetLimit || xo > kOffsetLimit || yo < -kOffsetLimit || yo > kOffsetLimit) {
              atomicOr(&status[pair_index], kStatusRange);
#ifdef CSM_DBG
              printf("leaf range xo %d yo %d\n", xo, yo);
#endif
            }
            else
              key = PackLeafKey(sum, rot0 + r, xo, yo);
            // Tie enumeration: every leaf at the pair's maximum sum.
            if (collect_sum >= 0 && key != 0 && sum == collect_sum) {
              const int slot = atomicAdd(&tie_count[pair_index], 1);
              if (slot < kTieCap)
                ties[static_cast<size_t>(pair_index) * kTieCap + slot] = make_uint2(
                    static_cast<uint32_t>(rot0 + r),
                    (static_cast<uint32_t>(xo) & 0xffff) | (static_cast<uint32_t>(yo) << 16));
            }
          }
          if (__ballot(key != 0)) {  // wave-uniform: any leaf this pass
            uint64_t hi = key ? HighLeafKey(key) : 0;
            for (int m = 32; m >= 1; m >>= 1) {
              const uint64_t o = __shfl_xor(key, m, 64);
              key = o > key ? o : key;
              const uint64_t oh = __shfl_xor(hi, m, 64);
              hi = oh > hi ? oh : hi;
            }
            if (lane == 0 && key > cur) {
              atomicMax(reinterpret_cast<unsigned long long*>(pair_best), key);
              atomicMax(reinterpret_cast<unsigned long long*>(&sh.best), key);
            }
            // Two leaves at the pass's largest sum, or one at the best sum
            // other than the best's: the pair ties there, so nodes bounded by
            // that sum need not be expanded (sh.tie_sum; tie resolution
            // searches those leaves again, ResolveTies).
            // Only a real incumbent (cur != 0) can be the second leaf: with
            // none yet, cur_sum is 0 and a single leaf at sum 0 (reachable
            // when min_score lets sum 0 pass) would look tied.
            if (CSM_TIE_PRUNE && !kCollect && lane == 0) {
              const uint32_t ks = static_cast<uint32_t>(key >> kSumShift);
              if (ks >= cur_sum &&
                  (hi != HighLeafKey(key) ||
                   (cur != 0 && key != cur && static_cast<uint32_t>(cur >> kSumShift) == ks)))
                atomicMax(&sh.tie_sum, static_cast<int>(ks));
            }
            // The largest-index leaf at the running maximum: a second maximal
            // leaf shows as a different index at the final sum (ResolveTies).
            if (lane == 0 && static_cast<uint32_t>(hi >> kSumShift) >= cur_sum)
              atomicMax(reinterpret_cast<unsigned long long*>(best_hi + pair_index), hi);
          }
          // Inner survivors: deepest level on top (the batch pop takes the
          // top 64 entries at once, so order within a level is immaterial
          // there). Rank = survivors of deeper levels + same-level survivors
          // in lower lanes; one ballot per distinct level (usually one).
          const bool push = keep && clvl > 0;
          // FIFO: nodes at levels <= CSM_LIFO_LEVEL go to the overflow stack,
          // popped first and deepest first, so an item reaches its leaves
          // (and an incumbent) early while the upper levels keep full
          // level-by-level batches.
          const bool deep = kFifo && push && clvl <= CSM_LIFO_LEVEL;
          const unsigned long long pm = __ballot(push && !deep);
          const int kept = __popcll(pm);
          int rank = 0;
          if (kFifo) rank = __popcll(pm & ((1ull << lane) - 1));
          for (unsigned long long rem = kFifo ? 0ull : pm; rem;) {
            const int l0 = __builtin_amdgcn_readlane(clvl, static_cast<int>(__ffsll(static_cast<long long>(rem))) - 1);
            const unsigned long long same = __ballot(push && clvl == l0);
            if (push) rank += clvl > l0 ? __popcll(same) : (clvl == l0 ? __popcll(same & ((1ull << lane) - 1)) : 0);
            rem &= ~same;
          }
          int sp = 0;
          if (lane == 0 && kept > 0) {
            sp = atomicAdd(&sh.sp, kept);
            atomicMax(&sh.high_water, sp + kept);
          }
          sp = __shfl(sp, 0, 64);
          const uint2 entry = make_uint2(
              (static_cast<uint32_t>(xo) & 0xffff) | (static_cast<uint32_t>(yo) << 16),
              static_cast<uint32_t>(sum) | (static_cast<uint32_t>(r) << 22) |
                  (static_cast<uint32_t>(clvl) << 27));
          if (kFifo) {
            // Ring slots past the LDS ring's capacity go to the workgroup's
            // overflow stack in global memory (popped when the ring is
            // empty); past that the pair is flagged.
            constexpr int kRing = decltype(sh)::kStackLds;
            const int slot = sp + rank;
            if (push && !deep && slot < kRing) sh.stack[(sh.head + slot) & (kRing - 1)] = entry;
            const bool over = (push && !deep && slot >= kRing) || deep;
            const unsigned long long om = __ballot(over);
            if (om) {
              int ob = 0;
              if (lane == 0) ob = atomicAdd(&sh.ovf, __popcll(om));
              ob = __shfl(ob, 0, 64) + __popcll(om & ((1ull << lane) - 1));
              if (over && ob < kSpill2) spill[ob] = entry;
              if (over && ob >= kSpill2) atomicOr(&status[pair_index], kStatusRange);
#ifdef CSM_DBG
              if (over && ob >= kSpill2 && (lane == 0 || ob == kSpill2)) printf("ovf overflow ob %d sp %d kept %d head %d\n", ob, sp, kept, sh.head);
#endif
            }
          } else {
            // Entries past the LDS stack go to this workgroup's spill region
            // in global memory (StackPut); past that the pair is flagged.
            if (push && sp + kept <= sh.kStackCapacity) StackPut(sh, spill, sp + kept - 1 - rank, entry);
            if (lane == 0 && sp + kept > sh.kStackCapacity) atomicOr(&status[pair_index], kStatusRange);
          }
        }
      }
      __syncthreads();
      if (wave == 0) {
        // (b) Refill roots when the stack is empty. (An overflowed stack has
        // flagged the pair; its result is discarded.)
        constexpr int kRing = decltype(sh)::kStackLds;
        int sp = min(sh.sp, kFifo ? kRing : sh.kStackCapacity);
        int ovf = kFifo ? min(sh.ovf, kSpill2) : 0;
        // The collect pass abandons a pair once its tied leaves overflow the
        // record: the host resolves it with the ordered walk (fast2d_walk).
        const bool abandon =
            kCollect && Uniform(static_cast<int>(
                            *reinterpret_cast<volatile int32_t*>(tie_count + pair_index) > kTieCap)) != 0;
        if (abandon) {
          sp = 0;
          ovf = 0;
          if (lane == 0) sh.vnext = vtotal;
        }
        if (!abandon && sp == 0 && ovf == 0 && sh.vnext < vtotal) {
          const int v0 = sh.vnext, vc = min(kRootChunk, vtotal - v0);
          if (kFifo && lane == 0) sh.head = 0;  // empty ring: restart at slot 0
          for (int k = lane; k < vc; k += 64) {
            const int v = kFifo ? v0 + k : v0 + vc - 1 - k;  // lowest root index first
            int r = 0;
            while (sh.root_prefix[r + 1] <= v) ++r;
            const int lv = v - sh.root_prefix[r];
            int xi = lv / sh.vny[r], yi = lv % sh.vny[r];
            if (CSM_XFAST) {
              const int vnx = (sh.root_prefix[r + 1] - sh.root_prefix[r]) / sh.vny[r];
              xi = lv % vnx;
              yi = lv / vnx;
            }
            const int xo = (sh.bounds[r][0] & -CSM_ORIGIN_ALIGN) + xi * 2 * step;
            const int yo = (sh.bounds[r][2] & -CSM_ORIGIN_ALIGN) + yi * 2 * step;
            sh.stack[k] = make_uint2((static_cast<uint32_t>(xo) & 0xffff) | (static_cast<uint32_t>(yo) << 16),
                                     0x3fffffu | (static_cast<uint32_t>(r) << 22) |
                                         (static_cast<uint32_t>(top_level + 1) << 27));
          }
          sp = vc;
          if (lane == 0) sh.vnext = v0 + vc;
        }
        // (c) Pop the next batch: up to 64 nodes, best first.
        if (lane == 0 && (sh.batch_no++ & (CSM_BEST_REFRESH - 1)) == 0) {
          // Every 8th batch also reads the tie witness: once it shows two
          // leaves at the best sum, the search only has to find a larger sum,
          // so nodes bounded by that sum are pruned (tie resolution searches
          // those leaves again, ResolveTies).
          const uint64_t fresh = LoadBest(pair_best);
          if (fresh > sh.best) sh.best = fresh;
        }
        const uint32_t cur_sum = static_cast<uint32_t>(sh.best >> kSumShift);
        const int tie_sum = Uniform(sh.tie_sum);
        int nodes = 0, blen = 0, bent = 0;
        if (sp > 0 || ovf > 0) {
          // Up to 64 entries from the top (any level); expand a power of two
          // of the unpruned ones, discard pruned ones passed over. FIFO: from
          // the overflow stack's top while it holds entries (the deepest ones:
          // depth-first until it drains, which bounds the frontier the way
          // the LIFO order does), else from the ring's head.
          uint2 ent = make_uint2(0, 0);
          const bool from_ring = !kFifo || ovf == 0;
          bool in = lane < kBatchNodes && lane < (from_ring ? sp : ovf);
          const int head = kFifo ? Uniform(sh.head) : 0;
          if (in) {
            if (!kFifo)
              ent = StackGet(sh, spill, sp - 1 - lane);
            else if (from_ring)
              ent = sh.stack[(head + lane) & (kRing - 1)];
            else
              ent = spill[ovf - 1 - lane];
          }
          bool hexb = false;
          if (kHex) {
            // One kind per batch: the entries down to the first of the other
            // kind (quad vs hex node level, SubmapDesc::hex_mask) than the top
            // entry.
            const bool hx = (hex_mask >> (ent.y >> 27)) & 1;
            const bool top_hx = __builtin_amdgcn_readlane(static_cast<int>(hx), 0) != 0;
            const unsigned long long other = __ballot(in && hx != top_hx);
            if (other) in = in && lane < static_cast<int>(__ffsll(static_cast<long long>(other))) - 1;
            hexb = top_hx;
          }
          const unsigned long long inm = __ballot(in);
          // A node bounded by a sum the witness keys already show tied
          // (sh.tie_sum) is not expanded: only a larger sum can change the
          // maximum.
          const bool expandable = in && (ent.y & 0x3fffff) >= cur_sum &&
                                  static_cast<int>(ent.y & 0x3fffff) > tie_sum;
          const unsigned long long em = __ballot(expandable);
          const int ne = __popcll(em);
          int take = __popcll(inm);
          if (ne > 0) {
            nodes = ne;  // every expandable entry among the next 64 (profiles/r3y)
            const int rank = __popcll(em & ((1ull << lane) - 1));
            // Entries up to the nodes-th expandable one are taken.
            take = static_cast<int>(__ffsll(static_cast<long long>(
                __ballot(expandable && rank == nodes - 1))));
            int len = 0;
            const bool took = expandable && lane < take;
            if (took) {
              const int r = (ent.y >> 22) & 0x1f, lvl = static_cast<int>(ent.y >> 27);
              const int sl = sh.lv[lvl - (hexb ? 2 : 1)][6];
              len = sh.list_len[r][sl];
              sh.node_xo[rank] = static_cast<int16_t>(ent.x & 0xffff);
              sh.node_yo[rank] = static_cast<int>(ent.x) >> 16;
              sh.node_rot[rank] = r;
              sh.node_level[rank] = lvl;
              sh.node_off[rank] = sh.list_off[r][sl];
              sh.node_len[rank] = len;
            }
            blen = DppMax(len);
            bent = DppSum(len);
            // Per child level: candidates scored and batches (lane l counts
            // level l; one pass per distinct level, usually one).
            const int cl = static_cast<int>(ent.y >> 27) - (hexb ? 2 : 1);
            for (unsigned long long tm = __ballot(took); tm;) {
              const int l0 = __builtin_amdgcn_readlane(cl, static_cast<int>(__ffsll(static_cast<long long>(tm))) - 1);
              const unsigned long long same = __ballot(took && cl == l0);
              if (lane == l0) {
                lv_cands += static_cast<unsigned long long>((hexb ? 16 : 4) * __popcll(same));
                lv_batches += 1;
              }
              tm &= ~same;
            }
          }
          if (from_ring) sp -= take; else ovf -= take;
          if (kHex && lane == 0) sh.batch_hex = hexb ? 1 : 0;
          if (kFifo && from_ring && lane == 0) sh.head = (head + take) & (kRing - 1);
        }
        if (lane == 0) {
          sh.sp = sp;
          sh.nodes = nodes;
          sh.batch_len = blen;
          sh.batch_entries = bent;
          if (kFifo) sh.ovf = ovf;
          sh.done = (nodes == 0 && sp == 0 && ovf == 0 && sh.vnext >= vtotal) ? 1 : 0;
        }
      }
      __syncthreads();
#ifdef CSM_KPROF
      if (tid == 0) {
        const long long now = clock64();
        kprof[1] += now - t_mark;
        t_mark = now;
      }
#endif
      const int nodes = Uniform(sh.nodes);
      const int done = Uniform(sh.done);
      if (done) break;
      if (nodes > 0) {
        // Algorithmic bytes: 4 per quad-dword gather, 16 per hex gather.
        const bool hexb = kHex && Uniform(sh.batch_hex);
        if (hexb)
          V4ScoreHex(sh, cells, cnts, raw_end, sm);
        else
          V4Score(sh, cells, cnts, raw_end, sm);
        const int kids = hexb ? 16 : 4;
        local_cands += kids * nodes;
        local_lookups += static_cast<unsigned long long>(hexb ? kHexEntryBytes : 4) *
                         static_cast<unsigned>(Uniform(sh.batch_entries));
      }
      __syncthreads();
#ifdef CSM_KPROF
      if (tid == 0) {
        const long long now = clock64();
        kprof[2] += now - t_mark;
        t_mark = now;
      }
#endif
    }
  }
  if (stats && tid == 0) {
    atomicAdd(&stats[0], local_cands);
    atomicAdd(&stats[1], local_lookups);
#ifdef CSM_KPROF
    for (int k = 0; k < 4; ++k) atomicAdd(&stats[2 + 2 * kMaxLevels + k], static_cast<unsigned long long>(kprof[k]));
#endif
  }
  if (stats && tid < kMaxLevels) {  // wave 0's lane l: level l
    atomicAdd(&stats[2 + tid], lv_cands);
    atomicAdd(&stats[2 + kMaxLevels + tid], lv_batches);
  }
  if (stats && tid == 0) atomicMax(&stats[kStatHighWater], static_cast<unsigned long long>(sh.high_water));
#ifdef CSM_KPROF
  if (stats && tid < kMaxLevels) {
    atomicAdd(&stats[kStatLines + tid], sh.kp_lines[tid]);
    atomicAdd(&stats[kStatLines + kMaxLevels + tid], sh.kp_instr[tid]);
    atomicAdd(&stats[kStatLines + 2 * kMaxLevels + tid], sh.kp_qlines[tid]);
    atomicAdd(&stats[kStatLines + 3 * kMaxLevels + tid], sh.kp_active[tid]);
    atomicAdd(&stats[kStatLines + 4 * kMaxLevels + tid], sh.kp_oob[tid]);
  }
#endif
}

// One rotation of a pair's scan discretized into LDS exactly as the search
// discretizes it (padding cells lie off every level). The caller
// synchronizes before reading `cells`.
__device__ void DiscretizeRotation(uint32_t* __restrict__ cells, int npad, const PairDesc& pd,
                                   const SubmapDesc& sm, float2 q,
                                   const float* __restrict__ points) {
  const double inv_res = 1.0 / sm.resolution;  // CellCoordFast
  for (int i = threadIdx.x; i < npad; i += blockDim.x) {
    uint32_t c = 0x80008000u;  // (-32768, -32768): outside every level
    if (i < pd.num_points) {
      const float* p = points + 3 * (pd.point_offset + i);
      float x, y;
      RotateZDev(pd.pre_w, pd.pre_s, p[0], p[1], &x, &y);
      RotateZDev(q.x, q.y, x, y, &x, &y);
      const float px = __fadd_rn(pd.tx, x);
      const float py = __fadd_rn(pd.ty, y);
      const double cx = CellCoordFast(sm.max_y, py, sm.resolution, inv_res);
      const double cy = CellCoordFast(sm.max_x, px, sm.resolution, inv_res);
      if (fabs(cx) <= kIndexLimit && fabs(cy) <= kIndexLimit)
        c = (static_cast<uint32_t>(static_cast<int>(cx)) & 0xffff) |
            (static_cast<uint32_t>(static_cast<int>(cy)) << 16);
    }
    cells[i] = c;
  }
}

// Tie resolution (csm_host.cc ResolveTies): exact level-d sums of listed
// candidates, ScoreCandidates' integer sums (fast_correlative_scan_matcher_2d.cc
// :314-333) over the row-major levels. One workgroup per (pair, rotation)
// job: the rotation's scan is discretized into LDS, then each wave sums its
// queries (level, x_off, y_off) over the points.
__global__ void __launch_bounds__(256)
fast2d_score_queries(const SubmapDesc* __restrict__ submaps, const PairDesc* __restrict__ pairs,
                     const float* __restrict__ points, const float2* __restrict__ rot_table,
                     const ScoreJob* __restrict__ jobs, const int4* __restrict__ queries,
                     int32_t* __restrict__ sums, int npad) {
  extern __shared__ __align__(16) uint32_t cells[];
  const ScoreJob job = jobs[blockIdx.x];
  const PairDesc pd = pairs[job.pair];
  const SubmapDesc& sm = submaps[pd.submap];
  DiscretizeRotation(cells, npad, pd, sm, rot_table[pd.rot_offset + job.rot], points);
  __syncthreads();
  for (int k = threadIdx.x >> 6; k < job.count; k += blockDim.x >> 6) {
    const int4 qu = queries[job.first + k];
    const int s = ScoreOne(cells, npad, MakeView(sm, qu.x), qu.y, qu.z);
    if ((threadIdx.x & 63) == 0) sums[job.first + k] = s;
  }
}

// ScoreCandidates' score (fast_correlative_scan_matcher_2d.cc:330-332,
// PrecomputationGrid2D::ToScore) with the host's float operations
// (search_window.cc SumToScore): the children's visiting order compares it.
__device__ __forceinline__ float SumToScoreDev(int sum, int n, float min_s, float max_s) {
  const float mean = __fdiv_rn(static_cast<float>(sum), static_cast<float>(n));
  return __fadd_rn(min_s, __fmul_rn(mean, __fdiv_rn(__fsub_rn(max_s, min_s), 255.f)));
}

// Ordered walk to the reference's pick among exactly tied maxima, for pairs
// whose tied leaves overflow the collect pass (csm_host.cc ResolveTies). The
// reference's BranchAndBound (fast_correlative_scan_matcher_2d.cc:335-378)
// visits the sorted lowest-resolution list in order, each node's <= 4
// children (x, then y; a child past the rotation's ShrinkToFit bound ends
// its loop) by descending score with equal scores in generation order, and
// keeps the first leaf at the maximum: before it is reached the incumbent is
// below the maximum, so every node whose sum reaches the maximum is visited,
// and nodes below it cannot hold that leaf. One workgroup per job walks that
// order depth-first over nodes whose exact sum is >= target, one child per
// wave, and stops at the first leaf whose sum is the target.
__global__ void __launch_bounds__(256)
fast2d_walk(const SubmapDesc* __restrict__ submaps, const PairDesc* __restrict__ pairs,
            const float* __restrict__ points, const float2* __restrict__ rot_table,
            const WalkJob2* __restrict__ jobs, const int4* __restrict__ top,
            const int4* __restrict__ bounds, int4* __restrict__ out, int npad) {
  extern __shared__ __align__(16) uint32_t cells[];
  __shared__ int4 stk[kWalkStack];
  __shared__ int sp;
  __shared__ int csum[4];
  __shared__ int4 res;
  const int tid = threadIdx.x, wave = tid >> 6;
  const WalkJob2 job = jobs[blockIdx.x];
  const PairDesc pd = pairs[job.pair];
  const SubmapDesc& sm = submaps[pd.submap];
  const int target = job.target_sum;
  if (tid == 0) res = make_int4(0, 0, 0, 0);
  __syncthreads();
  int cur_rot = -1;
  for (int ti = 0; ti < job.top_count; ++ti) {
    const int4 te = top[job.top_first + ti];  // (rot, x, y, sum), uniform
    if (job.top_level == 0) {                 // the list holds the leaves
      if (te.w == target) {
        if (tid == 0) res = make_int4(te.x, te.y, te.z, 1);
        break;
      }
      continue;
    }
    if (te.x != cur_rot) {
      __syncthreads();  // the previous rotation's readers are done
      DiscretizeRotation(cells, npad, pd, sm, rot_table[pd.rot_offset + te.x], points);
      cur_rot = te.x;
    }
    const int4 b = bounds[job.bounds_first + te.x];
    __syncthreads();  // every wave has read the previous walk's empty stack
    if (tid == 0) {
      stk[0] = make_int4(job.top_level, te.y, te.z, 0);
      sp = 1;
    }
    for (;;) {
      __syncthreads();  // cells, the stack and res are visible
      const int s = sp;
      if (s == 0 || res.w) break;
      const int4 nd = stk[s - 1];
      const int d = nd.x, hw = 1 << (d - 1);
      // Children in generation order (:353-366).
      int cxs[4], cys[4], nc = 0;
      for (int a = 0; a < 2; ++a) {
        const int xo = nd.y + a * hw;
        if (xo > b.y) break;
        for (int c = 0; c < 2; ++c) {
          const int yo = nd.z + c * hw;
          if (yo > b.w) break;
          cxs[nc] = xo;
          cys[nc] = yo;
          ++nc;
        }
      }
      int mx = 0, my = 0;
      for (int c = 0; c < 4; ++c)
        if (c == wave && c < nc) { mx = cxs[c]; my = cys[c]; }
      if (wave < nc) {
        const int sum = ScoreOne(cells, npad, MakeView(sm, d - 1), mx, my);
        if ((tid & 63) == 0) csum[wave] = sum;
      }
      __syncthreads();
      if (tid == 0) {
        // Stable descending order by score (std::sort on <= 16 elements is
        // libstdc++'s insertion sort).
        int ord[4];
        float sc[4];
        for (int c = 0; c < nc; ++c) {
          ord[c] = c;
          sc[c] = SumToScoreDev(csum[c], pd.num_points, job.min_s, job.max_s);
        }
        for (int i = 1; i < nc; ++i) {
          const int k = ord[i];
          int j = i - 1;
          while (j >= 0 && sc[k] > sc[ord[j]]) {
            ord[j + 1] = ord[j];
            --j;
          }
          ord[j + 1] = k;
        }
        int top_sp = s - 1;
        if (d == 1) {  // leaves: BranchAndBound(depth 0) returns the first (:339-341)
          if (nc > 0 && csum[ord[0]] == target) res = make_int4(te.x, cxs[ord[0]], cys[ord[0]], 1);
        } else {
          for (int i = nc - 1; i >= 0; --i)
            if (csum[ord[i]] >= target && top_sp < kWalkStack)
              stk[top_sp++] = make_int4(d - 1, cxs[ord[i]], cys[ord[i]], 0);
        }
        sp = top_sp;
      }
    }
    if (res.w) break;
  }
  __syncthreads();
  if (tid == 0) out[blockIdx.x] = res;
}

// ShrinkToFit bounds (correlative_scan_matcher_2d.cc:73-91) of one (pair,
// rotation) per workgroup, from the scan discretized exactly as the search
// discretizes it: (min_x, max_x, min_y, max_y) after the linear window clamp.
__global__ void __launch_bounds__(256)
fast2d_rotation_bounds(const SubmapDesc* __restrict__ submaps, const PairDesc* __restrict__ pairs,
                       const float* __restrict__ points, const float2* __restrict__ rot_table,
                       const int2* __restrict__ jobs, int4* __restrict__ bounds) {
  __shared__ int mm[4];
  const int2 job = jobs[blockIdx.x];
  const PairDesc pd = pairs[job.x];
  const SubmapDesc& sm = submaps[pd.submap];
  const float2 q = rot_table[pd.rot_offset + job.y];
  if (threadIdx.x == 0) {
    mm[0] = 0x7fffffff; mm[1] = -0x7fffffff; mm[2] = 0x7fffffff; mm[3] = -0x7fffffff;
  }
  __syncthreads();
  int mnx = 0x7fffffff, mxx = -0x7fffffff, mny = 0x7fffffff, mxy = -0x7fffffff;
  const double inv_res = 1.0 / sm.resolution;  // CellCoordFast
  for (int i = threadIdx.x; i < pd.num_points; i += blockDim.x) {
    const float* p = points + 3 * (pd.point_offset + i);
    float x, y;
    RotateZDev(pd.pre_w, pd.pre_s, p[0], p[1], &x, &y);
    RotateZDev(q.x, q.y, x, y, &x, &y);
    const float px = __fadd_rn(pd.tx, x);
    const float py = __fadd_rn(pd.ty, y);
    const double cx = CellCoordFast(sm.max_y, py, sm.resolution, inv_res);
    const double cy = CellCoordFast(sm.max_x, px, sm.resolution, inv_res);
    const int ix = fabs(cx) > kIndexLimit ? 0 : static_cast<int>(cx);
    const int iy = fabs(cy) > kIndexLimit ? 0 : static_cast<int>(cy);
    mnx = min(mnx, ix); mxx = max(mxx, ix);
    mny = min(mny, iy); mxy = max(mxy, iy);
  }
  mnx = WaveMin(mnx); mxx = WaveMax(mxx); mny = WaveMin(mny); mxy = WaveMax(mxy);
  if ((threadIdx.x & 63) == 0) {
    atomicMin(&mm[0], mnx); atomicMax(&mm[1], mxx);
    atomicMin(&mm[2], mny); atomicMax(&mm[3], mxy);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int lo_x = min(0, -mm[1]), hi_x = max(0, sm.nx - 1 - mm[0]);
    const int lo_y = min(0, -mm[3]), hi_y = max(0, sm.ny - 1 - mm[2]);
    bounds[blockIdx.x] = make_int4(max(-pd.num_linear, lo_x), min(pd.num_linear, hi_x),
                                   max(-pd.num_linear, lo_y), min(pd.num_linear, hi_y));
  }
}

// Grid cells -> float through a 32768-entry table (ValueConversionTables;
// the Ceres refinement's correspondence-cost grid).
__global__ void cells_to_probability(const uint16_t* __restrict__ cells,
                                     const float* __restrict__ ptab,
                                     float* __restrict__ out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = ptab[cells[i] & 0x7fff];
}

}  // namespace csm

// ---------------------------------------------------------------- launchers -
namespace csm {

hipError_t LaunchPyramidLevel0(const uint16_t* cells, const uint8_t* qtab, uint8_t* out, int n,
                               hipStream_t st) {
  hipLaunchKernelGGL(pyramid_level0, dim3((n + 1 + 255) / 256), dim3(256), 0, st, cells, qtab, out, n);
  return hipGetLastError();
}

hipError_t LaunchPyramidDouble(const uint8_t* prev, int pnx, int pny, uint8_t* next, int nnx,
                               int nny, int h, hipStream_t st) {
  hipLaunchKernelGGL(pyramid_double, dim3((nnx + 255) / 256, nny), dim3(256), 0, st, prev, pnx, pny,
                     next, nnx, nny, h);
  return hipGetLastError();
}

hipError_t LaunchFast2dSearch(int grid, size_t dyn_lds, hipStream_t st, const SubmapDesc* submaps,
                              const PairDesc* pairs, const float* points, const float2* rot_table,
                              const WorkQueues& queues, unsigned long long* counters,
                              uint64_t* best, int32_t* status, unsigned long long* stats) {
  hipLaunchKernelGGL(fast2d_search, dim3(grid), dim3(kSearchThreads), dyn_lds, st, submaps, pairs,
                     points, rot_table, queues, counters, best, status, stats);
  return hipGetLastError();
}

hipError_t LaunchPyramidQuad(const uint8_t* level, int wnx, int wny, int log_h, int km1,
                             uint32_t* out, int qw, int qh, int pws, int pph, int total,
                             hipStream_t st) {
  hipLaunchKernelGGL(pyramid_quad, dim3((total + 255) / 256), dim3(256), 0, st, level, wnx, wny,
                     log_h, km1, out, qw, qh, pws, pph, total);
  return hipGetLastError();
}

hipError_t LaunchFast2dSearchV2(int grid, size_t dyn_lds, hipStream_t st, const SubmapDesc* submaps,
                                const PairDesc* pairs, const float* points, const float2* rot_table,
                                const WorkQueues2& queues, unsigned long long* counters,
                                uint64_t* best, int32_t* status, unsigned long long* stats,
                                uint2* spill, int npad, int capc, bool hex, bool fifo,
                                uint64_t* best_hi, uint2* ties, int32_t* tie_count, bool collect) {
#define CSM_LAUNCH_V4(H, F, K)                                                                     \
  hipLaunchKernelGGL((fast2d_search_v4<H, F, K>), dim3(grid), dim3(kSearchThreads), dyn_lds, st,  \
                     submaps, pairs, points, rot_table, queues, counters, best, status, stats,     \
                     spill, npad, capc, best_hi, ties, tie_count)
  if (collect) {
    if (hex && fifo) CSM_LAUNCH_V4(true, true, true);
    else if (hex) CSM_LAUNCH_V4(true, false, true);
    else if (fifo) CSM_LAUNCH_V4(false, true, true);
    else CSM_LAUNCH_V4(false, false, true);
  } else {
    if (hex && fifo) CSM_LAUNCH_V4(true, true, false);
    else if (hex) CSM_LAUNCH_V4(true, false, false);
    else if (fifo) CSM_LAUNCH_V4(false, true, false);
    else CSM_LAUNCH_V4(false, false, false);
  }
#undef CSM_LAUNCH_V4
  return hipGetLastError();
}

hipError_t LaunchFast2dScoreQueries(int num_jobs, int npad, hipStream_t st, const SubmapDesc* submaps,
                                    const PairDesc* pairs, const float* points,
                                    const float2* rot_table, const ScoreJob* jobs,
                                    const int4* queries, int32_t* sums) {
  hipLaunchKernelGGL(fast2d_score_queries, dim3(num_jobs), dim3(256), sizeof(uint32_t) * npad, st,
                     submaps, pairs, points, rot_table, jobs, queries, sums, npad);
  return hipGetLastError();
}

hipError_t LaunchFast2dWalk(int num_jobs, int npad, hipStream_t st, const SubmapDesc* submaps,
                            const PairDesc* pairs, const float* points, const float2* rot_table,
                            const WalkJob2* jobs, const int4* top, const int4* bounds, int4* out) {
  hipLaunchKernelGGL(fast2d_walk, dim3(num_jobs), dim3(256), sizeof(uint32_t) * npad, st, submaps,
                     pairs, points, rot_table, jobs, top, bounds, out, npad);
  return hipGetLastError();
}

hipError_t LaunchFast2dRotationBounds(int num_jobs, hipStream_t st, const SubmapDesc* submaps,
                                      const PairDesc* pairs, const float* points,
                                      const float2* rot_table, const int2* jobs, int4* bounds) {
  hipLaunchKernelGGL(fast2d_rotation_bounds, dim3(num_jobs), dim3(256), 0, st, submaps, pairs, points,
                     rot_table, jobs, bounds);
  return hipGetLastError();
}

int Fast2dSearchV2BlocksPerCu(bool hex, bool fifo, size_t dyn_lds) {
  int blocks = 0;
  hipError_t e;
  if (hex && fifo)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fast2d_search_v4<true, true, false>, kSearchThreads, dyn_lds);
  else if (hex)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fast2d_search_v4<true, false, false>, kSearchThreads, dyn_lds);
  else if (fifo)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fast2d_search_v4<false, true, false>, kSearchThreads, dyn_lds);
  else
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, fast2d_search_v4<false, false, false>, kSearchThreads, dyn_lds);
  return e == hipSuccess ? blocks : 0;
}

hipError_t LaunchPyramidHex(const uint8_t* level, int wnx, int wny, int log_h, int km1,
                            uint8_t* scratch, uint32_t* out, int qw, int qh, int pws, int pph,
                            int total, hipStream_t st) {
  const int mw = wnx + km1, mh = wny + km1;
  hipLaunchKernelGGL(pyramid_widen, dim3((mw + 255) / 256, mh), dim3(256), 0, st, level, wnx, wny, km1,
                     scratch, mw, mh);
  hipLaunchKernelGGL(pyramid_hex, dim3((total + 255) / 256), dim3(256), 0, st, scratch, mw, mh, log_h,
                     static_cast<void*>(out), qw, qh, pws, pph, total);
  return hipGetLastError();
}

hipError_t LaunchCellsToProbability(const uint16_t* cells, const float* ptab, float* out, int n,
                                    hipStream_t st) {
  hipLaunchKernelGGL(cells_to_probability, dim3((n + 255) / 256), dim3(256), 0, st, cells, ptab, out, n);
  return hipGetLastError();
}

}  // namespace csm
