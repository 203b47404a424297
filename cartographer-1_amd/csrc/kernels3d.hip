// HIP kernels of the 3D path (gfx950): HybridGrid bricks, PrecomputationGrid3D
// levels, RealTimeCorrelativeScanMatcher3D scoring and the FastCSM3D
// branch and bound. Built with -ffp-contract=off: every float expression that
// feeds a cell index or a compared sum follows the reference's operation
// order (Eigen _transformVector, float division, lround).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csm_device3d.h"

namespace csm {

// ------------------------------------------------------------- helpers ----

// Eigen QuaternionBase::_transformVector: uv = q.vec x v; uv += uv;
// v + w*uv + q.vec x uv (Quaternion.h), unfused.
__device__ __forceinline__ void Rotate3(float qw, float qx, float qy, float qz, float vx, float vy,
                                        float vz, float* ox, float* oy, float* oz) {
  float ux = __fsub_rn(__fmul_rn(qy, vz), __fmul_rn(qz, vy));
  float uy = __fsub_rn(__fmul_rn(qz, vx), __fmul_rn(qx, vz));
  float uz = __fsub_rn(__fmul_rn(qx, vy), __fmul_rn(qy, vx));
  ux = __fadd_rn(ux, ux);
  uy = __fadd_rn(uy, uy);
  uz = __fadd_rn(uz, uz);
  const float cx = __fsub_rn(__fmul_rn(qy, uz), __fmul_rn(qz, uy));
  const float cy = __fsub_rn(__fmul_rn(qz, ux), __fmul_rn(qx, uz));
  const float cz = __fsub_rn(__fmul_rn(qx, uy), __fmul_rn(qy, ux));
  *ox = __fadd_rn(__fadd_rn(vx, __fmul_rn(qw, ux)), cx);
  *oy = __fadd_rn(__fadd_rn(vy, __fmul_rn(qw, uy)), cy);
  *oz = __fadd_rn(__fadd_rn(vz, __fmul_rn(qw, uz)), cz);
}

// std::lround(v / res) with the float quotient correctly rounded
// (HybridGridBase::GetCellIndex, hybrid_grid.h:428-433). The product with the
// rounded reciprocal is within 2 ulps of the quotient; only when it lies
// within a few ulps of a half-integer does the rounding decision need the
// exact IEEE quotient.
__device__ __forceinline__ int RoundDiv(float v, float res, float inv) {
  const float y = __fmul_rn(v, inv);
  const float r = rintf(y);
  const float d = fabsf(__fsub_rn(y, r));
  const float tol = fmaxf(fabsf(y), 1.f) * 1.9073486e-6f;  // 2^-19 relative
  if (fabsf(__fsub_rn(d, 0.5f)) <= tol) return static_cast<int>(roundf(__fdiv_rn(v, res)));
  return static_cast<int>(r);
}

__device__ __forceinline__ bool InBrick(const Brick3& b, int x, int y, int z, int64_t* idx) {
  const int lx = x - b.ox, ly = y - b.oy, lz = z - b.oz;
  if (static_cast<unsigned>(lx) >= static_cast<unsigned>(b.nx) ||
      static_cast<unsigned>(ly) >= static_cast<unsigned>(b.ny) ||
      static_cast<unsigned>(lz) >= static_cast<unsigned>(b.nz))
    return false;
  *idx = (static_cast<int64_t>(lz) * b.ny + ly) * b.nx + lx;
  return true;
}

// ------------------------------------------------------- grid building ----

// HybridGrid values -> float probabilities (ValueToProbability,
// probability_values.h:100-102) and -> level-0 precomputation values
// (ConvertToPrecomputationGrid, precomputation_grid_3d.cc:49-61).
__global__ void brick_from_values(const uint16_t* __restrict__ values, int64_t n,
                                  const float* __restrict__ ptab, const uint8_t* __restrict__ qtab,
                                  float* __restrict__ prob, uint8_t* __restrict__ level0) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint16_t v = values[i] & 0x7fff;
  if (prob) prob[i] = ptab[v];
  if (level0) level0[i] = qtab[v];
}

// PrecomputeGrid (precomputation_grid_3d.cc:63-81) in gather form:
// out[j] = max over octants o of prev[j + shift*o], or, at half resolution,
// max over o and e in {0,1}^3 of prev[2j + e + shift*o].
__global__ void level_gather(const uint8_t* __restrict__ prev, Brick3 pb, uint8_t* __restrict__ out,
                             Brick3 ob, int shift, int half) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t total = static_cast<int64_t>(ob.nx) * ob.ny * ob.nz;
  if (i >= total) return;
  const int lx = static_cast<int>(i % ob.nx);
  const int ly = static_cast<int>((i / ob.nx) % ob.ny);
  const int lz = static_cast<int>(i / (static_cast<int64_t>(ob.nx) * ob.ny));
  const int x = lx + ob.ox, y = ly + ob.oy, z = lz + ob.oz;
  unsigned v = 0;
  const int reps = half ? 8 : 1;
  for (int e = 0; e < reps; ++e) {
    const int bx = half ? 2 * x + (e & 1) : x;
    const int by = half ? 2 * y + ((e >> 1) & 1) : y;
    const int bz = half ? 2 * z + ((e >> 2) & 1) : z;
    for (int o = 0; o < 8; ++o) {
      int64_t k;
      if (InBrick(pb, bx + shift * (o & 1), by + shift * ((o >> 1) & 1),
                  bz + shift * ((o >> 2) & 1), &k))
        v = max(v, static_cast<unsigned>(prev[k]));
    }
  }
  out[i] = static_cast<uint8_t>(v);
}

// ------------------------------------------------------------- RTCSM3D ----
//
// One workgroup per search rotation r; thread t scores translation t. The
// rotated cloud R_r p is computed once per tile into LDS (shared by all
// translations); each thread then adds its translation, rounds to a cell and
// accumulates probabilities in the reference's point order, so the float sum
// is bit-identical to ScoreCandidate (real_time_correlative_scan_matcher_3d.cc
// :97-113). Key = score bits << 32 | ~(t * num_rot + r): the first strict
// maximum in (z, y, x, rz, ry, rx) order wins, as in Match (:34-54).
constexpr int kRt3Threads = 384;
constexpr int kRt3Tile = 512;

__global__ void __launch_bounds__(kRt3Threads)
rt3d_score(const float* __restrict__ prob, Brick3 gb, float res, float inv,
           const float* __restrict__ points, int n, const float4* __restrict__ rot,
           const float* __restrict__ rot_angle, const float4* __restrict__ trans, int num_trans,
           int t_base, int num_rot, double wt, double wr, unsigned long long* __restrict__ best) {
  __shared__ float4 rp[kRt3Tile];
  __shared__ unsigned long long red[kRt3Threads / 64];
  const int r = blockIdx.x;
  const int t = threadIdx.x;
  const float4 q = rot[r];
  const float4 tr = t < num_trans ? trans[t] : make_float4(0.f, 0.f, 0.f, 0.f);
  float sum = 0.f;
  for (int base = 0; base < n; base += kRt3Tile) {
    const int cnt = min(kRt3Tile, n - base);
    __syncthreads();
    for (int i = t; i < cnt; i += kRt3Threads) {
      const float* p = points + 3 * static_cast<int64_t>(base + i);
      float ox, oy, oz;
      Rotate3(q.w, q.x, q.y, q.z, p[0], p[1], p[2], &ox, &oy, &oz);
      rp[i] = make_float4(ox, oy, oz, 0.f);
    }
    __syncthreads();
    if (t < num_trans) {
      for (int i = 0; i < cnt; ++i) {
        const float4 a = rp[i];
        const int ix = RoundDiv(__fadd_rn(a.x, tr.x), res, inv);
        const int iy = RoundDiv(__fadd_rn(a.y, tr.y), res, inv);
        const int iz = RoundDiv(__fadd_rn(a.z, tr.z), res, inv);
        int64_t k;
        const float p = InBrick(gb, ix, iy, iz, &k) ? prob[k] : 0.1f;
        sum = __fadd_rn(sum, p);
      }
    }
  }
  unsigned long long key = 0;
  if (t < num_trans) {
    float score = __fdiv_rn(sum, static_cast<float>(n));
    const double e = static_cast<double>(tr.w) * wt + static_cast<double>(rot_angle[r]) * wr;
    score = static_cast<float>(static_cast<double>(score) * exp(-(e * e)));
    const unsigned idx = static_cast<unsigned>(t_base + t) * static_cast<unsigned>(num_rot) + r;
    key = (static_cast<unsigned long long>(__float_as_uint(score)) << 32) | (0xffffffffu - idx);
  }
  for (int m = 32; m > 0; m >>= 1) {
    const unsigned long long o = __shfl_xor(key, m, 64);
    key = o > key ? o : key;
  }
  if ((t & 63) == 0) red[t >> 6] = key;
  __syncthreads();
  if (t == 0) {
    unsigned long long k = red[0];
    for (int w = 1; w < kRt3Threads / 64; ++w) k = red[w] > k ? red[w] : k;
    atomicMax(best, k);
  }
}

// ------------------------------------------------------------ FastCSM3D ----
//
// Persistent workgroups pull (pair, yaw) items from a global counter. Per
// item: discretize the cloud with the yaw's pose into LDS (int16 cells),
// score the lowest-resolution candidates, then a best-first DFS over the
// 8-ary tree of BranchAndBound (fast_correlative_scan_matcher_3d.cc:377-440):
// a node's children are scored together (lanes = points, 8 accumulators),
// nodes whose bound is below the pair's best sum are pruned, and leaves are
// accepted in descending (sum, -id) order once their low-resolution score
// passes min_low_resolution_score (:384-401). Each pair keeps one 64-bit key
// sum << 42 | ~leaf_id, updated with atomicMax.

struct F3Shared {
  int16_t cx[kMax3dPoints], cy[kMax3dPoints], cz[kMax3dPoints];
  int16_t sx[kStack3d], sy[kStack3d], sz[kStack3d];
  int8_t sd[kStack3d];
  int ssum[kStack3d];
  int part[kSearch3dThreads / 64][8];
  int sums[8];
  int co_x[8], co_y[8], co_z[8];
  unsigned long long leaf_key[8];
  int order[8];
  float lr[kSearch3dThreads];
  int nchild, child_depth, sp, item, error, accepted;
  unsigned long long best;
};

__device__ __forceinline__ unsigned long long LeafId(const Pair3Desc& pd, int yaw, int ox, int oy,
                                                     int oz) {
  unsigned long long id = static_cast<unsigned long long>(yaw);
  id = (id << pd.bits_xy) | static_cast<unsigned long long>(ox + pd.wxy);
  id = (id << pd.bits_xy) | static_cast<unsigned long long>(oy + pd.wxy);
  id = (id << pd.bits_z) | static_cast<unsigned long long>(oz + pd.wz);
  return id;
}

// Sums of `count` (<= 8) candidates at `depth` (ScoreCandidates :332-355):
// reduction exponent e = max(0, depth - full_resolution_depth + 1); the
// discrete scan at depth >= full_resolution_depth is ((c + ws) >> e) - (ws >> e).
__device__ void ScoreOffsets(F3Shared& sh, const Submap3Desc& sm, const Pair3Desc& pd, int depth,
                             int count, const int* ox, const int* oy, const int* oz, int n) {
  const int tid = threadIdx.x;
  const int e = max(0, depth - sm.full_resolution_depth + 1);
  const Brick3 b = sm.level[depth];
  const uint8_t* g = sm.levels + b.offset;
  const int wsx = -pd.wxy, wsy = -pd.wxy, wsz = -pd.wz;
  const int lwx = wsx >> e, lwy = wsy >> e, lwz = wsz >> e;
  int sx[8], sy[8], sz[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sx[k] = k < count ? (ox[k] >> e) : 0;
    sy[k] = k < count ? (oy[k] >> e) : 0;
    sz[k] = k < count ? (oz[k] >> e) : 0;
  }
  int acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const bool reduced = depth >= sm.full_resolution_depth;
  for (int i = tid; i < n; i += kSearch3dThreads) {
    int x = sh.cx[i], y = sh.cy[i], z = sh.cz[i];
    if (reduced) {
      x = ((x + wsx) >> e) - lwx;
      y = ((y + wsy) >> e) - lwy;
      z = ((z + wsz) >> e) - lwz;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < count) {
        int64_t idx;
        if (InBrick(b, x + sx[k], y + sy[k], z + sz[k], &idx)) acc[k] += g[idx];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    int v = acc[k];
    for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
    acc[k] = v;
  }
  if ((tid & 63) == 0) {
#pragma unroll
    for (int k = 0; k < 8; ++k) sh.part[tid >> 6][k] = acc[k];
  }
  __syncthreads();
  if (tid < 8) {
    int s = 0;
    for (int w = 0; w < kSearch3dThreads / 64; ++w) s += sh.part[w][tid];
    sh.sums[tid] = s;
  }
  __syncthreads();
}

// Low-resolution matcher score of a leaf pose (low_resolution_matcher.cc:23-35):
// float sum in point order. Probabilities are computed in parallel, summed
// sequentially by thread 0. Result valid in thread 0.
__device__ float LowResScore(F3Shared& sh, const Submap3Desc& sm, const float* __restrict__ low_pts,
                             int m, float qw, float qx, float qy, float qz, float tx, float ty,
                             float tz) {
  const int tid = threadIdx.x;
  const float res = sm.low_resolution, inv = 1.f / sm.low_resolution;
  float sum = 0.f;
  for (int base = 0; base < m; base += kSearch3dThreads) {
    const int i = base + tid;
    if (i < m) {
      const float* p = low_pts + 3 * static_cast<int64_t>(i);
      float ox, oy, oz;
      Rotate3(qw, qx, qy, qz, p[0], p[1], p[2], &ox, &oy, &oz);
      const int ix = RoundDiv(__fadd_rn(ox, tx), res, inv);
      const int iy = RoundDiv(__fadd_rn(oy, ty), res, inv);
      const int iz = RoundDiv(__fadd_rn(oz, tz), res, inv);
      int64_t k;
      sh.lr[tid] = InBrick(sm.low, ix, iy, iz, &k) ? sm.low_prob[k] : 0.1f;
    }
    __syncthreads();
    if (tid == 0) {
      const int cnt = min(kSearch3dThreads, m - base);
      for (int j = 0; j < cnt; ++j) sum = __fadd_rn(sum, sh.lr[j]);
    }
    __syncthreads();
  }
  return __fdiv_rn(sum, static_cast<float>(m));
}

__global__ void __launch_bounds__(kSearch3dThreads)
fast3d_search(const Submap3Desc* __restrict__ submaps, const Pair3Desc* __restrict__ pairs,
              const Yaw3Desc* __restrict__ yaws, int num_items, const float* __restrict__ points,
              const float* __restrict__ low_points, unsigned* __restrict__ counter,
              unsigned long long* __restrict__ best, int32_t* __restrict__ status,
              unsigned long long* __restrict__ stats) {
  __shared__ F3Shared sh;
  const int tid = threadIdx.x;
  unsigned long long lookups = 0;
  for (;;) {
    if (tid == 0) sh.item = static_cast<int>(atomicAdd(counter, 1u));
    __syncthreads();
    const int item = sh.item;
    if (item >= num_items) break;
    const Yaw3Desc yw = yaws[item];
    const Pair3Desc pd = pairs[yw.pair];
    const Submap3Desc& sm = submaps[pd.submap];
    const int n = pd.num_points;
    const float res = sm.resolution, inv = 1.f / sm.resolution;
    if (tid == 0) sh.error = 0;
    __syncthreads();
    // DiscretizeScan (:201-244): cell of pose * p at full resolution.
    for (int i = tid; i < n; i += kSearch3dThreads) {
      const float* p = points + 3 * (pd.point_offset + i);
      float ox, oy, oz;
      Rotate3(yw.qw, yw.qx, yw.qy, yw.qz, p[0], p[1], p[2], &ox, &oy, &oz);
      const int ix = RoundDiv(__fadd_rn(ox, yw.tx), res, inv);
      const int iy = RoundDiv(__fadd_rn(oy, yw.ty), res, inv);
      const int iz = RoundDiv(__fadd_rn(oz, yw.tz), res, inv);
      if (abs(ix) > kCellLimit3d || abs(iy) > kCellLimit3d || abs(iz) > kCellLimit3d) sh.error = 1;
      sh.cx[i] = static_cast<int16_t>(ix);
      sh.cy[i] = static_cast<int16_t>(iy);
      sh.cz[i] = static_cast<int16_t>(iz);
    }
    __syncthreads();
    if (sh.error) {
      if (tid == 0) atomicExch(reinterpret_cast<int*>(status + yw.pair), -4);
      __syncthreads();
      continue;
    }
    const int top = sm.num_levels - 1;
    const int step = 1 << top;
    const int T = pd.top_nx * pd.top_ny * pd.top_nz;
    if (tid == 0) {
      sh.sp = 0;
      sh.best = best[yw.pair];
    }
    __syncthreads();
    // Lowest-resolution candidates (GenerateLowestResolutionCandidates
    // :297-330), in chunks of kRootChunk3d: each chunk is scored, ordered best
    // last and searched to exhaustion before the next one.
    for (int r0 = 0; r0 < T; r0 += kRootChunk3d) {
    const int r1 = min(T, r0 + kRootChunk3d);
    for (int c0 = r0; c0 < r1; c0 += 8) {
      const int cnt = min(8, r1 - c0);
      if (tid < 8) {
        const int j = c0 + min(tid, cnt - 1);
        const int ixx = j % pd.top_nx, iyy = (j / pd.top_nx) % pd.top_ny,
                  izz = j / (pd.top_nx * pd.top_ny);
        sh.co_x[tid] = -pd.wxy + ixx * step;
        sh.co_y[tid] = -pd.wxy + iyy * step;
        sh.co_z[tid] = -pd.wz + izz * step;
      }
      __syncthreads();
      int ox[8], oy[8], oz[8];
      for (int k = 0; k < 8; ++k) {
        ox[k] = sh.co_x[k];
        oy[k] = sh.co_y[k];
        oz[k] = sh.co_z[k];
      }
      ScoreOffsets(sh, sm, pd, top, cnt, ox, oy, oz, n);
      lookups += static_cast<unsigned long long>(cnt) * n;
      if (tid == 0) {
        const int best_sum = static_cast<int>(sh.best >> pd.key_shift);
        for (int k = 0; k < cnt; ++k) {
          const int s = sh.sums[k];
          if (s >= pd.min_sum && s >= best_sum) {
            const int at = sh.sp++;
            sh.sx[at] = static_cast<int16_t>(ox[k]);
            sh.sy[at] = static_cast<int16_t>(oy[k]);
            sh.sz[at] = static_cast<int16_t>(oz[k]);
            sh.sd[at] = static_cast<int8_t>(top);
            sh.ssum[at] = s;
          }
        }
      }
      __syncthreads();
    }
    // Order the roots so that the best bound is popped first (insertion sort
    // by thread 0; at most kRootChunk3d entries).
    if (tid == 0) {
      for (int a = 1; a < sh.sp; ++a) {
        const int16_t x = sh.sx[a], y = sh.sy[a], z = sh.sz[a];
        const int8_t d = sh.sd[a];
        const int s = sh.ssum[a];
        int b = a - 1;
        while (b >= 0 && sh.ssum[b] > s) {
          sh.sx[b + 1] = sh.sx[b];
          sh.sy[b + 1] = sh.sy[b];
          sh.sz[b + 1] = sh.sz[b];
          sh.sd[b + 1] = sh.sd[b];
          sh.ssum[b + 1] = sh.ssum[b];
          --b;
        }
        sh.sx[b + 1] = x;
        sh.sy[b + 1] = y;
        sh.sz[b + 1] = z;
        sh.sd[b + 1] = d;
        sh.ssum[b + 1] = s;
      }
    }
    __syncthreads();
    // Best-first DFS.
    for (;;) {
      if (tid == 0) {
        sh.nchild = 0;
        sh.best = max(sh.best, *reinterpret_cast<volatile unsigned long long*>(best + yw.pair));
        const int best_sum = static_cast<int>(sh.best >> pd.key_shift);
        while (sh.sp > 0 && sh.nchild == 0) {
          const int at = --sh.sp;
          const int s = sh.ssum[at];
          if (s < best_sum || s < pd.min_sum) continue;
          const int d = sh.sd[at];
          const int ox = sh.sx[at], oy = sh.sy[at], oz = sh.sz[at];
          const int hw = 1 << (d - 1);
          int c = 0;
          for (int z = 0; z <= hw; z += hw) {
            if (oz + z > pd.wz) break;
            for (int y = 0; y <= hw; y += hw) {
              if (oy + y > pd.wxy) break;
              for (int x = 0; x <= hw; x += hw) {
                if (ox + x > pd.wxy) break;
                sh.co_x[c] = ox + x;
                sh.co_y[c] = oy + y;
                sh.co_z[c] = oz + z;
                ++c;
              }
            }
          }
          sh.nchild = c;
          sh.child_depth = d - 1;
        }
        if (sh.nchild == 0) sh.nchild = -1;  // stack exhausted
      }
      __syncthreads();
      const int nc = sh.nchild;
      if (nc < 0) break;
      const int cd = sh.child_depth;
      int ox[8], oy[8], oz[8];
      for (int k = 0; k < 8; ++k) {
        ox[k] = sh.co_x[k];
        oy[k] = sh.co_y[k];
        oz[k] = sh.co_z[k];
      }
      ScoreOffsets(sh, sm, pd, cd, nc, ox, oy, oz, n);
      lookups += static_cast<unsigned long long>(nc) * n;
      if (cd > 0) {
        if (tid == 0) {
          const int best_sum = static_cast<int>(sh.best >> pd.key_shift);
          // Push ascending so that the best child is on top.
          int idx[8];
          int m = 0;
          for (int k = 0; k < nc; ++k)
            if (sh.sums[k] >= pd.min_sum && sh.sums[k] >= best_sum) idx[m++] = k;
          for (int a = 1; a < m; ++a) {
            const int v = idx[a];
            int b = a - 1;
            while (b >= 0 && sh.sums[idx[b]] > sh.sums[v]) {
              idx[b + 1] = idx[b];
              --b;
            }
            idx[b + 1] = v;
          }
          for (int a = 0; a < m; ++a) {
            const int k = idx[a];
            const int at = sh.sp++;
            sh.sx[at] = static_cast<int16_t>(ox[k]);
            sh.sy[at] = static_cast<int16_t>(oy[k]);
            sh.sz[at] = static_cast<int16_t>(oz[k]);
            sh.sd[at] = static_cast<int8_t>(cd);
            sh.ssum[at] = sh.sums[k];
          }
        }
        __syncthreads();
        continue;
      }
      // Leaves: descending key order; the first one that passes the
      // low-resolution check is this group's answer (:384-401).
      if (tid == 0) {
        for (int k = 0; k < nc; ++k) {
          const unsigned long long id = LeafId(pd, yw.yaw_id, ox[k], oy[k], oz[k]);
          sh.leaf_key[k] = (static_cast<unsigned long long>(sh.sums[k]) << pd.key_shift) |
                           (~id & ((1ull << pd.key_shift) - 1));
          sh.order[k] = k;
        }
        for (int a = 1; a < nc; ++a) {
          const int v = sh.order[a];
          int b = a - 1;
          while (b >= 0 && sh.leaf_key[sh.order[b]] < sh.leaf_key[v]) {
            sh.order[b + 1] = sh.order[b];
            --b;
          }
          sh.order[b + 1] = v;
        }
        sh.accepted = 0;
      }
      __syncthreads();
      for (int a = 0; a < nc; ++a) {
        const int k = sh.order[a];
        if (sh.sums[k] < pd.min_sum) break;
        if (sh.leaf_key[k] <= sh.best) break;  // uniform: sh.best is shared
        const float rf = res;
        const float tx = __fadd_rn(yw.tx, __fmul_rn(rf, static_cast<float>(ox[k])));
        const float ty = __fadd_rn(yw.ty, __fmul_rn(rf, static_cast<float>(oy[k])));
        const float tz = __fadd_rn(yw.tz, __fmul_rn(rf, static_cast<float>(oz[k])));
        const float lrs = LowResScore(sh, sm, low_points + 3 * pd.low_offset, pd.num_low, yw.nw,
                                      yw.nx, yw.ny, yw.nz, tx, ty, tz);
        if (tid == 0) {
          if (static_cast<double>(lrs) >= static_cast<double>(pd.min_low_resolution_score)) {
            atomicMax(best + yw.pair, sh.leaf_key[k]);
            sh.best = max(sh.best, sh.leaf_key[k]);
            sh.accepted = 1;
          }
        }
        __syncthreads();
        if (sh.accepted) break;
      }
      __syncthreads();
    }
    }  // root chunks
  }
  if (tid == 0 && stats) atomicAdd(stats, lookups);
}

// Low-resolution score of each pair's winning leaf (the Result field), with
// the same arithmetic as the search: one workgroup per pair.
__global__ void __launch_bounds__(kSearch3dThreads)
fast3d_finalize(const Submap3Desc* __restrict__ submaps, const Pair3Desc* __restrict__ pairs,
                const Yaw3Desc* __restrict__ yaws, const float* __restrict__ low_points,
                const unsigned long long* __restrict__ best, float* __restrict__ low_score) {
  __shared__ F3Shared sh;
  const int p = blockIdx.x;
  const unsigned long long key = best[p];
  const Pair3Desc pd = pairs[p];
  if (key == 0 || pd.num_yaws == 0) {
    if (threadIdx.x == 0) low_score[p] = 0.f;
    return;
  }
  const unsigned long long id = ~key & ((1ull << pd.key_shift) - 1);
  const int oz = static_cast<int>(id & ((1ull << pd.bits_z) - 1)) - pd.wz;
  const int oy = static_cast<int>((id >> pd.bits_z) & ((1ull << pd.bits_xy) - 1)) - pd.wxy;
  const int ox = static_cast<int>((id >> (pd.bits_z + pd.bits_xy)) & ((1ull << pd.bits_xy) - 1)) - pd.wxy;
  const int yaw = static_cast<int>(id >> (pd.bits_z + 2 * pd.bits_xy));
  const Yaw3Desc yw = yaws[pd.yaw_begin + yaw];
  const Submap3Desc& sm = submaps[pd.submap];
  const float rf = sm.resolution;
  const float tx = __fadd_rn(yw.tx, __fmul_rn(rf, static_cast<float>(ox)));
  const float ty = __fadd_rn(yw.ty, __fmul_rn(rf, static_cast<float>(oy)));
  const float tz = __fadd_rn(yw.tz, __fmul_rn(rf, static_cast<float>(oz)));
  const float s = LowResScore(sh, sm, low_points + 3 * pd.low_offset, pd.num_low, yw.nw, yw.nx,
                              yw.ny, yw.nz, tx, ty, tz);
  if (threadIdx.x == 0) low_score[p] = s;
}

// ------------------------------------------------------------ launchers ----

hipError_t LaunchBrickFromValues(const uint16_t* values, int64_t n, const float* ptab,
                                 const uint8_t* qtab, float* prob, uint8_t* level0,
                                 hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(brick_from_values, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st,
                     values, n, ptab, qtab, prob, level0);
  return hipGetLastError();
}

hipError_t LaunchLevelGather(const uint8_t* prev, const Brick3& pb, uint8_t* out, const Brick3& ob,
                             int shift, int half, hipStream_t st) {
  const int64_t total = static_cast<int64_t>(ob.nx) * ob.ny * ob.nz;
  if (total <= 0) return hipSuccess;
  hipLaunchKernelGGL(level_gather, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0,
                     st, prev, pb, out, ob, shift, half);
  return hipGetLastError();
}

hipError_t LaunchRt3dScore(int num_rot, hipStream_t st, const float* prob, const Brick3& gb,
                           float res, const float* points, int n, const float4* rot,
                           const float* rot_angle, const float4* trans, int num_trans, int t_base,
                           double wt, double wr, unsigned long long* best) {
  hipLaunchKernelGGL(rt3d_score, dim3(num_rot), dim3(kRt3Threads), 0, st, prob, gb, res,
                     1.f / res, points, n, rot, rot_angle, trans + t_base, num_trans, t_base,
                     num_rot, wt, wr, best);
  return hipGetLastError();
}

hipError_t LaunchFast3dSearch(int grid, hipStream_t st, const Submap3Desc* submaps,
                              const Pair3Desc* pairs, const Yaw3Desc* yaws, int num_items,
                              const float* points, const float* low_points, unsigned* counter,
                              unsigned long long* best, int32_t* status,
                              unsigned long long* stats) {
  hipLaunchKernelGGL(fast3d_search, dim3(grid), dim3(kSearch3dThreads), 0, st, submaps, pairs,
                     yaws, num_items, points, low_points, counter, best, status, stats);
  return hipGetLastError();
}

hipError_t LaunchFast3dFinalize(int num_pairs, hipStream_t st, const Submap3Desc* submaps,
                                const Pair3Desc* pairs, const Yaw3Desc* yaws,
                                const float* low_points, const unsigned long long* best,
                                float* low_score) {
  if (num_pairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(fast3d_finalize, dim3(num_pairs), dim3(kSearch3dThreads), 0, st, submaps,
                     pairs, yaws, low_points, best, low_score);
  return hipGetLastError();
}

}  // namespace csm
