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

// Quad layout of level d (h = 2^d): the dword for quad cell (X', Y'),
// X' < qw = wnx + h, Y' < qh = wny + h, packs the children values of a node
// whose child (0,0) sits at wide cell (X, Y) = (X' - h, Y' - h):
// byte0 G(X, Y), byte1 G(X, Y+h), byte2 G(X+h, Y), byte3 G(X+h, Y+h);
// G = 0 outside the wide grid. Cells are stored polyphase with period
// P = 2h: plane (X' mod P, Y' mod P), entry (X' / P, Y' / P), row stride pws,
// plane size pws * pph dwords. Same-level nodes of one rotation sit on one
// P-lattice, so one point's lookups by sibling nodes are adjacent dwords.
__global__ void pyramid_quad(const uint8_t* __restrict__ level, int wnx, int wny, int log_h,
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
    v = g(X, Y) | (g(X, Y + h) << 8) | (g(X + h, Y) << 16) | (g(X + h, Y + h) << 24);
  }
  out[o] = v;
}

// ---------------------------------------------------------------- K2-K4 v4 -
//
// A workgroup (4 waves) searches a chunk of R rotations of one pair at once.
// The DFS stack mixes the chunk's rotations; a batch pops up to 16 nodes of
// one level (best first) and scores their 2x2 children: a lane takes one node
// and a strided subset of that node's rotated scan, and per point issues ONE
// dword load from the quad layout that returns all four children's values.
// The 4 waves split the points and meet in LDS; wave 0 combines, prunes,
// pushes survivors sorted (best on top) and pops the next batch. Roots are
// virtual nodes one level above the top lattice.

constexpr int kMaxRotChunk = 16;

struct V4Shared {
  uint2 stack[kStack2];  // w0: xo | yo << 16; w1: sum | rot << 22 | level << 27
  int part[kBatchNodes][4];  // children sums, accumulated by the 4 waves (LDS atomics)
  int n_eff;                  // run-list length shared by the chunk's rotations
  int run_len[kMaxRotChunk];  // each rotation's own run-list length
  int node_xo[kBatchNodes], node_yo[kBatchNodes], node_rot[kBatchNodes], node_level[kBatchNodes];
  int nodes, done;
  int item_pair, item_chunk, queue;
  int sp;
  uint64_t best;
  int mm[kMaxRotChunk][4];
  int bounds[kMaxRotChunk][4];
  int vny[kMaxRotChunk];
  int root_prefix[kMaxRotChunk + 1];
  int vnext;
  int range_error, batch_no, high_water;
  unsigned long long lv_cands[kMaxLevels];
  unsigned long long lv_batches[kMaxLevels];
};

// The DFS stack: entries [0, kStack2) in LDS, [kStack2, kStack2 + kSpill2)
// in the workgroup's spill region (global memory; the workgroup's own waves
// write and read it, ordered by the __syncthreads between phases).
__device__ __forceinline__ uint2 StackGet(const V4Shared& sh, const uint2* spill, int i) {
  return i < kStack2 ? sh.stack[i] : spill[i - kStack2];
}
__device__ __forceinline__ void StackPut(V4Shared& sh, uint2* spill, int i, uint2 v) {
  if (i < kStack2) sh.stack[i] = v; else spill[i - kStack2] = v;
}

// Scores the children of the batch's nodes over the chunk's run lists: entry
// k of rotation r is a cell (pts) and the number of consecutive scan points
// that fell into it (cnt, <= 255; 0 for padding). A child's sum is
// sum_k cnt[k] * value, the reference's per-point sum regrouped.
__device__ __forceinline__ void V4Score(V4Shared& sh, const uint32_t* pts, const uint8_t* cnt,
                                        int npad, int n, const SubmapDesc& sm) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nodes = Uniform(sh.nodes);
  const int groups = 64 / nodes;
  const int node = lane & (nodes - 1);
  const int g = lane / nodes;
  // Each node scores its children at its own child level: one descriptor
  // spans the whole pyramid, the level is a per-lane byte offset.
  const int level = sh.node_level[node] - 1;
  const int h = 1 << level;
  const int qw = sm.quad_w[level], qh = sm.quad_h[level];
  const int qoff = sm.quad_off[level];
  const int sft = level + 1, pmask = (2 << level) - 1;
  const int pws4 = sm.quad_pws[level] * 4, ps4 = sm.quad_pws[level] * sm.quad_pph[level] * 4;
  const __amdgpu_buffer_rsrc_t rsrc = LevelRsrc(sm.pyramid_base, Uniform(sm.pyramid_bytes));
  const uint32_t* P = pts + sh.node_rot[node] * npad;
  const uint8_t* Cn = cnt + sh.node_rot[node] * npad;
  const int cx = sh.node_xo[node] + (h - 1) + h;
  const int cy = sh.node_yo[node] + (h - 1) + h;
  const int quarter = (n + kWaves - 1) / kWaves;
  const int s = Uniform(min(n, wave * quarter)), e = Uniform(min(n, wave * quarter + quarter));
  constexpr int kOOB = 0x7ffffff0;
  constexpr int U = 8;
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
  // v_dot4_u32_u8 with the run count in one byte of the weight multiplies
  // that child's byte by the count and accumulates.
  auto accumulate = [&](uint32_t v, uint32_t c) {
    a0 = __builtin_amdgcn_udot4(v, c, a0, false);
    a1 = __builtin_amdgcn_udot4(v, c << 8, a1, false);
    a2 = __builtin_amdgcn_udot4(v, c << 16, a2, false);
    a3 = __builtin_amdgcn_udot4(v, c << 24, a3, false);
  };
  int i = s;
  for (; i + U * groups <= e; i += U * groups) {
    int ad[U];
    uint32_t c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ad[u] = address(P[i + u * groups + g], true);
      c[u] = Cn[i + u * groups + g];
    }
    uint32_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, ad[u], 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) accumulate(v[u], c[u]);
  }
  for (; i < e; i += groups) {
    const int idx = i + g;
    const bool in = idx < e;
    const uint32_t vv = __builtin_amdgcn_raw_buffer_load_b32(rsrc, address(in ? P[idx] : 0u, in),
                                                             0, 0);
    accumulate(vv, in ? Cn[idx] : 0u);
  }
  for (int m = nodes; m < 64; m <<= 1) {
    a0 += __shfl_xor(a0, m, 64);
    a1 += __shfl_xor(a1, m, 64);
    a2 += __shfl_xor(a2, m, 64);
    a3 += __shfl_xor(a3, m, 64);
  }
  if (lane < nodes) {
    atomicAdd(&sh.part[lane][0], static_cast<int>(a0));  // (xo,     yo)
    atomicAdd(&sh.part[lane][1], static_cast<int>(a1));  // (xo,     yo + h)
    atomicAdd(&sh.part[lane][2], static_cast<int>(a2));  // (xo + h, yo)
    atomicAdd(&sh.part[lane][3], static_cast<int>(a3));  // (xo + h, yo + h)
  }
}

// Run lists (per rotation, in place): consecutive scan points that fall in
// the same cell become one entry with their count. Wave w compacts rotations
// w, w + 4, ...; a run longer than 255 points is split so counts fit a byte.
// Writes each rotation's list length to lens[r]; returns this wave's longest
// list (wave-uniform).
__device__ int CompactRuns(uint32_t* pts, uint8_t* cnt, int npad, int n, int nrot, int* lens) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const unsigned long long below = (1ull << lane) - 1;
  int longest = 0;
  for (int r = wave; r < nrot; r += kWaves) {
    uint32_t* P = pts + r * npad;
    uint8_t* C = cnt + r * npad;
    int out = 0;                // entries written so far
    int run_start = 0;          // start of the run open at the block boundary
    uint32_t last = 0;          // last cell of the previous block
    int open_k = -1, open_pos = 0;  // the previous block's last entry, count pending
    for (int base = 0; base < n; base += 64) {
      const int i = base + lane;
      const bool in = i < n;
      const uint32_t v = in ? P[i] : 0u;
      uint32_t prev = __shfl_up(v, 1, 64);
      if (lane == 0) prev = last;
      const bool head0 = in && (i == 0 || v != prev);
      // Start of each lane's run: inclusive max-scan of head positions.
      int rs = head0 ? i : -1;
      for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(rs, d, 64);
        if (lane >= d) rs = max(rs, o);
      }
      rs = max(rs, run_start);
      const bool head = head0 || (in && (i - rs) % 255 == 0);
      const unsigned long long hm = __ballot(head);
      const int k = out + __popcll(hm & below);
      // Close the entry left open by the previous block.
      if (open_k >= 0 && hm) {
        const int first = base + static_cast<int>(__ffsll(static_cast<long long>(hm))) - 1;
        if (lane == 0) C[open_k] = static_cast<uint8_t>(first - open_pos);
        open_k = -1;
      }
      if (head) {
        const unsigned long long above = hm & ~(below | (1ull << lane));
        P[k] = v;
        if (above) C[k] = static_cast<uint8_t>(__ffsll(static_cast<long long>(above)) - 1 - lane);
      }
      if (hm) {
        const int lastl = 63 - __clzll(hm);
        open_k = out + __popcll(hm) - 1;
        open_pos = base + lastl;
      }
      out += __popcll(hm);
      run_start = __shfl(rs, 63, 64);
      last = __shfl(v, 63, 64);
    }
    if (open_k >= 0 && lane == 0) C[open_k] = static_cast<uint8_t>(n - open_pos);
    if (lane == 0) lens[r] = out;
    longest = max(longest, out);
  }
  return longest;
}

__global__ void __launch_bounds__(kSearchThreads) __attribute__((amdgpu_waves_per_eu(5)))
fast2d_search_v4(const SubmapDesc* __restrict__ submaps,
                 const PairDesc* __restrict__ pairs,
                 const float* __restrict__ points,
                 const float2* __restrict__ rot_table,
                 WorkQueues2 queues,
                 unsigned long long* __restrict__ counters,
                 uint64_t* __restrict__ best,
                 int32_t* __restrict__ status,
                 unsigned long long* __restrict__ stats,
                 uint2* __restrict__ spill_base, int npad) {
  extern __shared__ __align__(16) uint32_t pts[];  // rot_chunk * npad cells, then counts
  __shared__ V4Shared sh;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rc = queues.rot_chunk;
  uint8_t* cnt = reinterpret_cast<uint8_t*>(pts + rc * npad);
  uint2* spill = spill_base + static_cast<size_t>(blockIdx.x) * kSpill2;
  for (int k = tid; k < kBatchNodes * 4; k += kSearchThreads) sh.part[k >> 2][k & 3] = 0;
  if (tid == 0) sh.high_water = 0;
  unsigned long long local_cands = 0, local_lookups = 0;
#ifdef CSM_KPROF
  long long kprof[4] = {0, 0, 0, 0};  // thread 0: discretize, control, score cycles; batches
#endif
  if (tid == 0) sh.queue = blockIdx.x % kNumXcd;
  if (tid < kMaxLevels) { sh.lv_cands[tid] = 0; sh.lv_batches[tid] = 0; }
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
    uint64_t* pair_best = best + pair_index;
    const int rot0 = Uniform(sh.item_chunk) * rc;
    const int nrot = min(rc, pd.num_scans - rot0);
    const int top_level = sm.levels - 1;
    const int step = 1 << top_level;

    // ---- K2: discretize the chunk's rotated scans into LDS ----------------
#ifdef CSM_KPROF
    long long t_mark = clock64();
#endif
    if (tid < kMaxRotChunk * 4) sh.mm[tid >> 2][tid & 3] = (tid & 1) ? -0x7fffffff : 0x7fffffff;
    if (tid == 0) sh.range_error = 0;
    __syncthreads();
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
        pts[r * npad + i] = (static_cast<uint32_t>(ix) & 0xffff) | (static_cast<uint32_t>(iy) << 16);
      }
      mnx = WaveMin(mnx); mxx = WaveMax(mxx); mny = WaveMin(mny); mxy = WaveMax(mxy);
      if (lane == 0) {
        atomicMin(&sh.mm[r][0], mnx); atomicMax(&sh.mm[r][1], mxx);
        atomicMin(&sh.mm[r][2], mny); atomicMax(&sh.mm[r][3], mxy);
      }
    }
    if (range_error) sh.range_error = 1;
    if (tid == 0) sh.n_eff = 0;
    __syncthreads();
    // ---- Run lists; pad every rotation to the longest with empty entries ----
    {
      const int longest = CompactRuns(pts, cnt, npad, n, nrot, sh.run_len);
      if (lane == 0) atomicMax(&sh.n_eff, longest);
    }
    __syncthreads();
    const int n_eff = Uniform(sh.n_eff);
    for (int r = 0; r < nrot; ++r)  // past a rotation's own list: out-of-range cell, count 0
      for (int k = sh.run_len[r] + tid; k < n_eff; k += kSearchThreads) {
        pts[r * npad + k] = 0x80008000u;
        cnt[r * npad + k] = 0;
      }
    __syncthreads();
    // ---- ShrinkToFit per rotation; root counts ------------------------------
    if (tid < nrot) {
      const int r = tid;
      const int lo_x = min(0, -sh.mm[r][1]), hi_x = max(0, sm.nx - 1 - sh.mm[r][0]);
      const int lo_y = min(0, -sh.mm[r][3]), hi_y = max(0, sm.ny - 1 - sh.mm[r][2]);
      const int b0 = max(-pd.num_linear, lo_x), b1 = min(pd.num_linear, hi_x);
      const int b2 = max(-pd.num_linear, lo_y), b3 = min(pd.num_linear, hi_y);
      sh.bounds[r][0] = b0; sh.bounds[r][1] = b1; sh.bounds[r][2] = b2; sh.bounds[r][3] = b3;
      const int tnx = (b1 - b0 + step) / step, tny = (b3 - b2 + step) / step;
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
      sh.best = LoadBest(pair_best);
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
        const int pn = sh.nodes;
        for (int pass = wave; pass * 16 < pn; pass += kWaves) {
          const int nd = pass * 16 + (lane >> 2), c = lane & 3;
          int sum = 0, xo = 0, yo = 0, r = 0, clvl = 0;
          bool exists = false;
          if (nd < pn) {
            clvl = sh.node_level[nd] - 1;
            const int h = 1 << clvl;
            sum = sh.part[nd][c];
            sh.part[nd][c] = 0;
            r = sh.node_rot[nd];
            xo = sh.node_xo[nd] + ((c & 2) ? h : 0);
            yo = sh.node_yo[nd] + ((c & 1) ? h : 0);
            exists = xo <= sh.bounds[r][1] && yo <= sh.bounds[r][3];
          }
          const uint64_t cur = sh.best;
          const uint32_t cur_sum = static_cast<uint32_t>(cur >> kSumShift);
          const bool keep = exists && sum > s_min && static_cast<uint32_t>(sum) >= cur_sum;
          // Leaves (child level 0) update the incumbent.
          uint64_t key = 0;
          if (keep && clvl == 0) {
            if (xo < -kOffsetLimit || xo > kOffsetLimit || yo < -kOffsetLimit || yo > kOffsetLimit)
              atomicOr(&status[pair_index], kStatusRange);
            else
              key = PackLeafKey(sum, rot0 + r, xo, yo);
          }
          if (__ballot(key != 0)) {  // wave-uniform: any leaf this pass
            for (int m = 32; m >= 1; m >>= 1) {
              const uint64_t o = __shfl_xor(key, m, 64);
              key = o > key ? o : key;
            }
            if (lane == 0 && key > cur) {
              atomicMax(reinterpret_cast<unsigned long long*>(pair_best), key);
              atomicMax(reinterpret_cast<unsigned long long*>(&sh.best), key);
            }
          }
          // Inner survivors: deepest level first, then best bound, on top.
          // Rank among survivors by counting larger keys (lane ids make keys
          // distinct); each survivor writes its own entry.
          const bool push = keep && clvl > 0;
          const uint32_t skey = push ? ((static_cast<uint32_t>(15 - clvl) << 28) |
                                        (static_cast<uint32_t>(sum) << 6) | static_cast<uint32_t>(lane))
                                     : 0u;
          const unsigned long long pm = __ballot(push);
          const int kept = __popcll(pm);
          int rank = 0;
          for (unsigned long long m = pm; m; m &= m - 1) {
            const int jl = static_cast<int>(__ffsll(static_cast<long long>(m))) - 1;
            rank += static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(skey), jl)) > skey;
          }
          int sp = 0;
          if (lane == 0 && kept > 0) {
            sp = atomicAdd(&sh.sp, kept);
            atomicMax(&sh.high_water, sp + kept);
          }
          sp = __shfl(sp, 0, 64);
          // Entries past the LDS stack go to this workgroup's spill region in
          // global memory (StackPut); past that the pair is flagged (the
          // bound is ~2.8k entries: <= 256 pushed per level).
          if (push && sp + kept <= kStack2 + kSpill2)
            StackPut(sh, spill, sp + kept - 1 - rank, make_uint2(
                (static_cast<uint32_t>(xo) & 0xffff) | (static_cast<uint32_t>(yo) << 16),
                static_cast<uint32_t>(sum) | (static_cast<uint32_t>(r) << 22) |
                    (static_cast<uint32_t>(clvl) << 27)));
          if (lane == 0 && sp + kept > kStack2 + kSpill2) atomicOr(&status[pair_index], kStatusRange);
        }
      }
      __syncthreads();
      if (wave == 0) {
        // (b) Refill roots when the stack is empty. (An overflowed stack has
        // flagged the pair; its result is discarded.)
        int sp = min(sh.sp, kStack2 + kSpill2);
        if (sp == 0 && sh.vnext < vtotal) {
          const int v0 = sh.vnext, vc = min(kRootChunk, vtotal - v0);
          for (int k = lane; k < vc; k += 64) {
            const int v = v0 + vc - 1 - k;  // lowest root index on top
            int r = 0;
            while (sh.root_prefix[r + 1] <= v) ++r;
            const int lv = v - sh.root_prefix[r];
            const int xo = sh.bounds[r][0] + (lv / sh.vny[r]) * 2 * step;
            const int yo = sh.bounds[r][2] + (lv % sh.vny[r]) * 2 * step;
            sh.stack[k] = make_uint2((static_cast<uint32_t>(xo) & 0xffff) | (static_cast<uint32_t>(yo) << 16),
                                     0x3fffffu | (static_cast<uint32_t>(r) << 22) |
                                         (static_cast<uint32_t>(top_level + 1) << 27));
          }
          sp = vc;
          if (lane == 0) sh.vnext = v0 + vc;
        }
        // (c) Pop the next batch: up to 16 same-level nodes, best first.
        if (lane == 0 && (sh.batch_no++ & 7) == 0) {
          const uint64_t fresh = LoadBest(pair_best);
          if (fresh > sh.best) sh.best = fresh;
        }
        const uint32_t cur_sum = static_cast<uint32_t>(sh.best >> kSumShift);
        int nodes = 0;
        if (sp > 0) {
          // Up to 64 entries from the top (any level); expand a power of two
          // of the unpruned ones, discard pruned ones passed over.
          uint2 ent = make_uint2(0, 0);
          const bool in = lane < kBatchNodes && lane < sp;
          if (in) ent = StackGet(sh, spill, sp - 1 - lane);
          const unsigned long long inm = __ballot(in);
          const bool expandable = in && (ent.y & 0x3fffff) >= cur_sum;
          const unsigned long long em = __ballot(expandable);
          const int ne = __popcll(em);
          int take = __popcll(inm);
          if (ne > 0) {
            nodes = 1 << (31 - __clz(ne));
            unsigned long long m = em;
            for (int k = 1; k < nodes; ++k) m &= m - 1;
            take = static_cast<int>(__ffsll(static_cast<long long>(m)));
            const int rank = __popcll(em & ((1ull << lane) - 1));
            if (expandable && lane < take) {
              sh.node_xo[rank] = static_cast<int16_t>(ent.x & 0xffff);
              sh.node_yo[rank] = static_cast<int>(ent.x) >> 16;
              sh.node_rot[rank] = (ent.y >> 22) & 0x1f;
              sh.node_level[rank] = static_cast<int>(ent.y >> 27);
            }
          }
          sp -= take;
        }
        if (lane == 0) {
          sh.sp = sp;
          sh.nodes = nodes;
          sh.done = (nodes == 0 && sp == 0 && sh.vnext >= vtotal) ? 1 : 0;
        }
      }
      __syncthreads();
#ifdef CSM_KPROF
      if (tid == 0) {
        const long long now = clock64();
        kprof[1] += now - t_mark;
        t_mark = now;
        kprof[3] += 1;
      }
#endif
      const int nodes = Uniform(sh.nodes);
      const int done = Uniform(sh.done);
      if (done) break;
      if (nodes > 0) {
        V4Score(sh, pts, cnt, npad, n_eff, sm);
        local_cands += 4 * nodes;
        local_lookups += static_cast<unsigned long long>(4 * nodes) * n;
        if (tid < nodes) {
          const int cl = sh.node_level[tid] - 1;
          atomicAdd(&sh.lv_cands[cl], 4ull);
          if (tid == 0) atomicAdd(&sh.lv_batches[cl], 1ull);
        }
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
  if (stats && tid < kMaxLevels) {
    atomicAdd(&stats[2 + tid], sh.lv_cands[tid]);
    atomicAdd(&stats[2 + kMaxLevels + tid], sh.lv_batches[tid]);
  }
  if (stats && tid == 0) atomicMax(&stats[kStatHighWater], static_cast<unsigned long long>(sh.high_water));
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

hipError_t LaunchPyramidQuad(const uint8_t* level, int wnx, int wny, int log_h, uint32_t* out,
                             int qw, int qh, int pws, int pph, int total, hipStream_t st) {
  hipLaunchKernelGGL(pyramid_quad, dim3((total + 255) / 256), dim3(256), 0, st, level, wnx, wny,
                     log_h, out, qw, qh, pws, pph, total);
  return hipGetLastError();
}

hipError_t LaunchFast2dSearchV2(int grid, size_t dyn_lds, hipStream_t st, const SubmapDesc* submaps,
                                const PairDesc* pairs, const float* points, const float2* rot_table,
                                const WorkQueues2& queues, unsigned long long* counters,
                                uint64_t* best, int32_t* status, unsigned long long* stats,
                                uint2* spill, int npad) {
  hipLaunchKernelGGL(fast2d_search_v4, dim3(grid), dim3(kSearchThreads), dyn_lds, st, submaps, pairs,
                     points, rot_table, queues, counters, best, status, stats, spill, npad);
  return hipGetLastError();
}

hipError_t LaunchCellsToProbability(const uint16_t* cells, const float* ptab, float* out, int n,
                                    hipStream_t st) {
  hipLaunchKernelGGL(cells_to_probability, dim3((n + 255) / 256), dim3(256), 0, st, cells, ptab, out, n);
  return hipGetLastError();
}

}  // namespace csm
