// HIP kernels of the 3D path (gfx950): HybridGrid bricks, PrecomputationGrid3D
// levels, RealTimeCorrelativeScanMatcher3D scoring and the FastCSM3D
// branch and bound. Built with -ffp-contract=off: every float expression that
// feeds a cell index or a compared sum follows the reference's operation
// order (Eigen _transformVector, float division, lround).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "csm_device3d.h"
#include "csm_launch3d.h"

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

// A HybridGrid's known cells (the list its iterator yields) into the zeroed
// dense brick: cell i at its offset in the brick (the list holds each cell
// once, as HybridGrid's iteration / ToProto does).
__global__ void brick_scatter(const int32_t* __restrict__ ijk, const uint16_t* __restrict__ values,
                              int64_t count, Brick3 b, uint16_t* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const int64_t k = (static_cast<int64_t>(ijk[3 * i + 2] - b.oz) * b.ny + (ijk[3 * i + 1] - b.oy)) * b.nx +
                    (ijk[3 * i] - b.ox);
  out[k] = values[i];
}

// Batched grid builds (csm_hybrid_grid_create_batch), blockIdx.y = job:
// zero the value bricks (16 bytes per thread and step), scatter the cell
// lists into them, then the probabilities, as brick_scatter and
// brick_from_values do for one grid.
__global__ void __launch_bounds__(256) grid_zero_batch(const GridJob3* __restrict__ jobs) {
  const GridJob3 j = jobs[blockIdx.y];
  const int64_t n8 = j.n / 8;  // whole 16-byte pieces (value bricks are 256-byte aligned)
  uint4* v = reinterpret_cast<uint4*>(j.values);
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  for (int64_t i = t; i < n8; i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    v[i] = make_uint4(0u, 0u, 0u, 0u);
  if (t < j.n - 8 * n8) j.values[8 * n8 + t] = 0;  // the last < 8 values
}
__global__ void __launch_bounds__(256) grid_scatter_batch(const GridJob3* __restrict__ jobs) {
  const GridJob3 j = jobs[blockIdx.y];
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < j.count;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int64_t k = (static_cast<int64_t>(j.ijk[3 * i + 2] - j.b.oz) * j.b.ny + (j.ijk[3 * i + 1] - j.b.oy)) *
                          j.b.nx + (j.ijk[3 * i] - j.b.ox);
    j.values[k] = j.vals[i];
  }
}
__global__ void __launch_bounds__(256) grid_prob_batch(const GridJob3* __restrict__ jobs,
                                                       const float* __restrict__ ptab) {
  const GridJob3 j = jobs[blockIdx.y];
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < j.n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    j.prob[i] = ptab[j.values[i] & 0x7fff];
}

// Cell (x, y, z) of brick b as a 32-bit offset (bricks are < 2^31 cells), or
// -1 outside.
__device__ __forceinline__ int BrickIndex32(const Brick3& b, int x, int y, int z) {
  const int lx = x - b.ox, ly = y - b.oy, lz = z - b.oz;
  if (static_cast<unsigned>(lx) >= static_cast<unsigned>(b.nx) ||
      static_cast<unsigned>(ly) >= static_cast<unsigned>(b.ny) ||
      static_cast<unsigned>(lz) >= static_cast<unsigned>(b.nz))
    return -1;
  return (lz * b.ny + ly) * b.nx + lx;
}

// PrecomputeGrid (precomputation_grid_3d.cc:63-81) in gather form:
// out[j] = max over octants o of prev[j + shift*o], or, at half resolution,
// max over o and e in {0,1}^3 of prev[2j + e + shift*o]. Grid: (x blocks of
// 256, y, z; strided past 65535), so a thread's cell needs no division.
__global__ void __launch_bounds__(256)
level_gather(const uint8_t* __restrict__ prev, Brick3 pb, uint8_t* __restrict__ out, Brick3 ob,
             int shift, int half) {
  const int lx = blockIdx.x * 256 + threadIdx.x;
  if (lx >= ob.nx) return;
  const int x = lx + ob.ox;
  const int reps = half ? 8 : 1;
  for (int lz = blockIdx.z; lz < ob.nz; lz += gridDim.z) {
    for (int ly = blockIdx.y; ly < ob.ny; ly += gridDim.y) {
      const int y = ly + ob.oy, z = lz + ob.oz;
      unsigned v = 0;
      for (int e = 0; e < reps; ++e) {
        const int bx = half ? 2 * x + (e & 1) : x;
        const int by = half ? 2 * y + ((e >> 1) & 1) : y;
        const int bz = half ? 2 * z + ((e >> 2) & 1) : z;
#pragma unroll
        for (int o = 0; o < 8; ++o) {
          const int k = BrickIndex32(pb, bx + shift * (o & 1), by + shift * ((o >> 1) & 1),
                                     bz + shift * ((o >> 2) & 1));
          if (k >= 0) v = max(v, static_cast<unsigned>(prev[k]));
        }
      }
      out[(lz * ob.ny + ly) * ob.nx + lx] = static_cast<uint8_t>(v);
    }
  }
}

// Octet layout (Submap3Desc::octs): out[c] packs level[c + H*(x, y, z)].
// Grid as level_gather's.
__global__ void __launch_bounds__(256)
octet_build(const uint8_t* __restrict__ level, Brick3 lb, int h, uint64_t* __restrict__ out,
            Brick3 ob) {
  const int lx = blockIdx.x * 256 + threadIdx.x;
  if (lx >= ob.nx) return;
  const int x = lx + ob.ox;
  for (int lz = blockIdx.z; lz < ob.nz; lz += gridDim.z) {
    for (int ly = blockIdx.y; ly < ob.ny; ly += gridDim.y) {
      const int y = ly + ob.oy, z = lz + ob.oz;
      uint64_t v = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int idx =
            BrickIndex32(lb, x + h * (k & 1), y + h * ((k >> 1) & 1), z + h * ((k >> 2) & 1));
        if (idx >= 0) v |= static_cast<uint64_t>(level[idx]) << (8 * k);
      }
      out[(lz * ob.ny + ly) * ob.nx + lx] = v;
    }
  }
}

// Row form of octet_build and level_gather: a workgroup makes whole output
// rows (y, z) from the source rows they read, staged in LDS with dword loads
// (the per-cell kernels issue 8 or 64 byte loads per cell, which binds them
// on the texture path). Cells outside the source brick read 0, as InBrick
// does.
//   kOctet: out[c] packs byte k = level[c + h (k&1, k>>1&1, k>>2)] (octet_build;
//     4 source rows (y + h ky, z + h kz)).
//   else, full resolution: out[c] = the max of those 8 bytes (level_gather
//     with shift h, half = 0; 4 source rows).
//   kHalf: out[c] = max over e, o in {0,1}^3 of prev[2c + e + h o]
//     (level_gather with half = 1): 16 source rows (2y + {0, 1, h, h + 1}) x
//     (2z + {0, 1, h, h + 1}), 4 x positions each.
// One wave per output row: a row's loads and stores are a few instructions,
// so the kernel is bound by how many rows are in flight (latency), and
// single-wave workgroups keep 4x as many rows resident as 256-thread ones.
constexpr int kRowThreads = 64;
template <bool kOctet, bool kHalf>
__device__ __forceinline__ void BrickRows(const uint8_t* __restrict__ src, Brick3 sb, int h,
                                          void* __restrict__ out, Brick3 ob, int block, int blocks,
                                          uint8_t* rows) {
  static_assert(!(kOctet && kHalf), "octets are built at the level's own resolution");
  constexpr int kRows = kHalf ? 16 : 4;
  const int W = kHalf ? 2 * ob.nx + h : ob.nx + h, pitch = BrickRowsPitch(W);
  uint32_t* roww = reinterpret_cast<uint32_t*>(rows);
  const int src_bytes = sb.nx * sb.ny * sb.nz;
  // Up to 3 bytes past the brick are read (levels are 256-byte aligned in
  // their buffer) and masked below.
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(src), 0, (src_bytes + 3) & ~3, 0x00020000);
  const int xs = (kHalf ? 2 * ob.ox : ob.ox) - sb.ox;  // source x (brick-relative) of position 0
  const int nrows = ob.ny * ob.nz;
  for (int row = block; row < nrows; row += blocks) {
    {
      const int ly = row % ob.ny, lz = row / ob.ny;
      const int y = ly + ob.oy, z = lz + ob.oz;
      __syncthreads();  // the previous row's reads are done
      // Source rows staged as the dwords that hold them (a dword store per
      // loaded dword; bytes outside the source row zeroed): position pos of
      // row r is byte roff[r] + pos. Every row's loads of a 128-dword span are
      // issued before any is stored, so a row costs one memory round trip
      // per span, not one per source row.
      int roff[kRows], a0s[kRows], rs0s[kRows], nws[kRows];
      bool oks[kRows];
      int span = 0;
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        int yy, zz;
        if constexpr (kHalf) {
          yy = 2 * y + (r & 1) + h * ((r >> 1) & 1);
          zz = 2 * z + ((r >> 2) & 1) + h * (r >> 3);
        } else {
          yy = y + h * (r & 1);
          zz = z + h * (r >> 1);
        }
        yy -= sb.oy;
        zz -= sb.oz;
        oks[r] = static_cast<unsigned>(yy) < static_cast<unsigned>(sb.ny) &&
                 static_cast<unsigned>(zz) < static_cast<unsigned>(sb.nz);
        rs0s[r] = oks[r] ? (zz * sb.ny + yy) * sb.nx : 0;  // byte of source x = 0
        const int b0 = rs0s[r] + xs;                        // byte of position 0
        a0s[r] = b0 & ~3;
        roff[r] = r * pitch + (b0 - a0s[r]);
        nws[r] = (W + (b0 - a0s[r]) + 3) >> 2;
        span = max(span, nws[r]);
      }
      for (int i0 = 0; i0 < span; i0 += 2 * kRowThreads) {
        uint32_t w[kRows][2];
#pragma unroll
        for (int r = 0; r < kRows; ++r)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int i = i0 + q * kRowThreads + static_cast<int>(threadIdx.x);
            w[r][q] = oks[r] && i < nws[r] ? __builtin_amdgcn_raw_buffer_load_b32(rs, a0s[r] + 4 * i, 0, 0) : 0u;
          }
#pragma unroll
        for (int r = 0; r < kRows; ++r)
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int i = i0 + q * kRowThreads + static_cast<int>(threadIdx.x);
            if (i >= nws[r]) continue;
            const int a = a0s[r] + 4 * i;
            uint32_t v = w[r][q];
            if (a < rs0s[r] || a + 4 > rs0s[r] + sb.nx) {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (static_cast<unsigned>(a + j - rs0s[r]) >= static_cast<unsigned>(sb.nx)) v &= ~(0xffu << (8 * j));
            }
            roww[r * (pitch >> 2) + i] = v;
          }
      }
      __syncthreads();
      const int base = (lz * ob.ny + ly) * ob.nx;
      for (int lx = threadIdx.x; lx < ob.nx; lx += kRowThreads) {
        if constexpr (kOctet) {
          uint64_t v = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k)
            v |= static_cast<uint64_t>(rows[roff[k >> 1] + lx + h * (k & 1)]) << (8 * k);
          static_cast<uint64_t*>(out)[base + lx] = v;
        } else if constexpr (kHalf) {
          unsigned v = 0;
          const int p = 2 * lx;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const uint8_t* row = rows + roff[r] + p;
            v = max(v, max(max(static_cast<unsigned>(row[0]), static_cast<unsigned>(row[1])),
                           max(static_cast<unsigned>(row[h]), static_cast<unsigned>(row[h + 1]))));
          }
          static_cast<uint8_t*>(out)[base + lx] = static_cast<uint8_t>(v);
        } else {
          unsigned v = 0;
#pragma unroll
          for (int k = 0; k < 8; ++k)
            v = max(v, static_cast<unsigned>(rows[roff[k >> 1] + lx + h * (k & 1)]));
          static_cast<uint8_t*>(out)[base + lx] = static_cast<uint8_t>(v);
        }
      }
    }
  }
}

template <bool kOctet, bool kHalf>
__global__ void __launch_bounds__(kRowThreads)
brick_rows(const uint8_t* __restrict__ src, Brick3 sb, int h, void* __restrict__ out, Brick3 ob) {
  extern __shared__ uint8_t rows[];  // kRows rows x pitch
  BrickRows<kOctet, kHalf>(src, sb, h, out, ob, blockIdx.x, gridDim.x, rows);
}

// Batched form (csm_fast3d_create_batch): blockIdx.y picks the job, so one
// launch builds a level (or its octets) for every submap of the batch.
template <bool kOctet, bool kHalf>
__global__ void __launch_bounds__(kRowThreads)
brick_rows_batch(const RowJob3* __restrict__ jobs) {
  extern __shared__ uint8_t rows[];
  const RowJob3 jb = jobs[blockIdx.y];
  if (jb.ob.nx <= 0 || jb.ob.ny <= 0 || jb.ob.nz <= 0) return;
  BrickRows<kOctet, kHalf>(jb.src, jb.sb, jb.h, jb.out, jb.ob, blockIdx.x, gridDim.x, rows);
}

// Batched level-0 conversion (ConvertToPrecomputationGrid, the qtab path of
// brick_from_values): blockIdx.y picks the submap.
__global__ void __launch_bounds__(256)
values_to_level0_batch(const ValueJob3* __restrict__ jobs, const uint8_t* __restrict__ qtab) {
  const ValueJob3 jb = jobs[blockIdx.y];
  // 4 cells per lane and step: an 8-byte load, a dword store (both bricks
  // 256-byte aligned); the last < 4 cells one each.
  const int64_t n4 = jb.n / 4;
  const uint2* v4 = reinterpret_cast<const uint2*>(jb.values);
  uint32_t* o4 = reinterpret_cast<uint32_t*>(jb.level0);
  const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  for (int64_t i = t; i < n4; i += static_cast<int64_t>(gridDim.x) * 256) {
    const uint2 v = v4[i];
    o4[i] = static_cast<uint32_t>(qtab[v.x & 0x7fff]) | (static_cast<uint32_t>(qtab[(v.x >> 16) & 0x7fff]) << 8) |
            (static_cast<uint32_t>(qtab[v.y & 0x7fff]) << 16) |
            (static_cast<uint32_t>(qtab[(v.y >> 16) & 0x7fff]) << 24);
  }
  if (t < jb.n - 4 * n4) jb.level0[4 * n4 + t] = qtab[jb.values[4 * n4 + t] & 0x7fff];
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

// RTCSM3D, v2. Same candidates, sums and key as rt3d_score, cheaper per lookup:
//  * the probability brick is padded by one cell of 0.1 (the unknown / outside
//    probability) on every side, so a lookup clamps each cell coordinate into
//    [-1, n] (v_med3) instead of testing bounds and selecting the default;
//  * the cell coordinate is rint(v * (1 / res)), and the exact IEEE quotient
//    (RoundDiv) is taken only for points whose product lies within 2^-21 |y|
//    of a half-integer, where the product's error could change the rounding
//    decision (RoundFast);
//  * two rotations per workgroup (2 x 343 = 686 of 704 lanes busy at C4's
//    7^3 translations, against 343 of 384).
constexpr int kRt3Rpb = 2;

__global__ void pad_prob_brick(const float* __restrict__ prob, Brick3 gb, int P, float* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int px = gb.nx + 2 * P, py = gb.ny + 2 * P, pz = gb.nz + 2 * P;
  if (i >= static_cast<int64_t>(px) * py * pz) return;
  const int x = static_cast<int>(i % px) - P;
  const int y = static_cast<int>((i / px) % py) - P;
  const int z = static_cast<int>(i / (static_cast<int64_t>(px) * py)) - P;
  float v = 0.1f;
  if (x >= 0 && x < gb.nx && y >= 0 && y < gb.ny && z >= 0 && z < gb.nz)
    v = prob[(static_cast<int64_t>(z) * gb.ny + y) * gb.nx + x];
  out[i] = v;
}

// rint(v * inv) as a float; flags products too close to a half-integer.
// y = fl(v * fl(1 / res)) is within 2^-23 |x| of x = v / res, and fl(x) within
// half an ulp (<= 2^-24 |x|) of x, so when y lies more than 2^-21 |y| from a
// half-integer h, fl(x) lies strictly on y's side of h and lround(fl(x)) =
// rint(y).
__device__ __forceinline__ float RoundFast(float v, float inv, bool* risky) {
  const float y = __fmul_rn(v, inv);
  const float r = rintf(y);
  const float d = fabsf(__fsub_rn(y, r));
  *risky |= fmaf(fabsf(y), 4.7683716e-7f, d) >= 0.5f;
  return r;
}

__global__ void __launch_bounds__(768)
rt3d_score2(const float* __restrict__ pad, int pnx, int pny, int pnz, int ox, int oy, int oz,
            float res, float inv, const float* __restrict__ points, int n,
            const float4* __restrict__ rot, const float* __restrict__ rot_angle,
            const float4* __restrict__ trans, int num_trans, int t_base, int num_rot, double wt,
            double wr, unsigned long long* __restrict__ best, float* __restrict__ scores,
            int scores_pitch) {
  __shared__ float4 rp[kRt3Rpb][kRt3Tile];
  __shared__ unsigned long long red[768 / 64];
  const int tid = threadIdx.x;
  const int sub = tid / num_trans;
  const int t = tid - sub * num_trans;
  const int r = blockIdx.x * kRt3Rpb + sub;
  const bool active = sub < kRt3Rpb && r < num_rot;
  const float4 tr = active ? trans[t] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* my = rp[active ? sub : 0];
  // Cell (ix, iy, iz) lives at padded index ((iz + 1 - oz) * pny + iy + 1 - oy) * pnx + ix + 1 - ox,
  // each coordinate clamped to the padded box (exact in float: |coordinates| < 2^24).
  const float bx = static_cast<float>(1 - ox), by = static_cast<float>(1 - oy),
              bz = static_cast<float>(1 - oz);
  const float mx = static_cast<float>(pnx - 1), my_ = static_cast<float>(pny - 1),
              mz = static_cast<float>(pnz - 1);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(pad), 0, static_cast<int>(4u * pnx * pny * pnz), 0x00020000);
  float sum = 0.f;
  for (int base = 0; base < n; base += kRt3Tile) {
    const int cnt = min(kRt3Tile, n - base);
    __syncthreads();
    for (int i = tid; i < kRt3Rpb * cnt; i += blockDim.x) {
      const int s = i / cnt, j = i - s * cnt;
      const int rr = min(blockIdx.x * kRt3Rpb + s, num_rot - 1);
      const float4 q = rot[rr];
      const float* p = points + 3 * static_cast<int64_t>(base + j);
      float ox_, oy_, oz_;
      Rotate3(q.w, q.x, q.y, q.z, p[0], p[1], p[2], &ox_, &oy_, &oz_);
      rp[s][j] = make_float4(ox_, oy_, oz_, 0.f);
    }
    __syncthreads();
    if (active) {
      auto cell = [&](const float4& a, bool* risky, float* f) {
        f[0] = RoundFast(__fadd_rn(a.x, tr.x), inv, risky);
        f[1] = RoundFast(__fadd_rn(a.y, tr.y), inv, risky);
        f[2] = RoundFast(__fadd_rn(a.z, tr.z), inv, risky);
      };
      auto exact = [&](const float4& a, float* f) {  // rare: the IEEE quotient decides
        f[0] = static_cast<float>(RoundDiv(__fadd_rn(a.x, tr.x), res, inv));
        f[1] = static_cast<float>(RoundDiv(__fadd_rn(a.y, tr.y), res, inv));
        f[2] = static_cast<float>(RoundDiv(__fadd_rn(a.z, tr.z), res, inv));
      };
      auto load = [&](const float* f) {
        const unsigned cx = static_cast<unsigned>(__builtin_amdgcn_fmed3f(__fadd_rn(f[0], bx), 0.f, mx));
        const unsigned cy = static_cast<unsigned>(__builtin_amdgcn_fmed3f(__fadd_rn(f[1], by), 0.f, my_));
        const unsigned cz = static_cast<unsigned>(__builtin_amdgcn_fmed3f(__fadd_rn(f[2], bz), 0.f, mz));
        const unsigned k = __umul24(__umul24(cz, pny) + cy, pnx) + cx;
        return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, k << 2, 0, 0));
      };
      // One point per step: batching 2 or 4 points' loads, software-pipelining
      // the loads one point ahead, or a 4 x 4 x 2 tiled brick were all slower
      // on C4 (8.9, 7.4 and 8.3 s against 6.6-6.9 s). The exact
      // path re-reads the point from LDS inside its own loop: this shape
      // compiled to the fastest schedule measured (6.9 s; 7.6 s reusing `a`).
      for (int i = 0; i + 1 <= cnt; i += 1) {
        float4 a[1];
        a[0] = my[i];
        bool risky = false;
        float f[1][3];
        cell(a[0], &risky, f[0]);
        if (risky) {
#pragma unroll 1
          for (int u = 0; u < 1; ++u) {
            float g[3];
            exact(my[i + u], g);
            f[0][0] = g[0];
            f[0][1] = g[1];
            f[0][2] = g[2];
          }
        }
        sum = __fadd_rn(sum, load(f[0]));
      }
    }
  }
  unsigned long long key = 0;
  if (active) {
    float score = __fdiv_rn(sum, static_cast<float>(n));
    const double e = static_cast<double>(tr.w) * wt + static_cast<double>(rot_angle[r]) * wr;
    score = static_cast<float>(static_cast<double>(score) * exp(-(e * e)));
    const unsigned idx = static_cast<unsigned>(t_base + t) * static_cast<unsigned>(num_rot) + r;
    key = (static_cast<unsigned long long>(__float_as_uint(score)) << 32) | (0xffffffffu - idx);
    // Test-visible scoring of a rotation subset (csm_rt3d_score_rotations):
    // every candidate's score, no reduction.
    if (scores) scores[static_cast<int64_t>(r) * scores_pitch + t_base + t] = score;
  }
  if (scores) return;  // uniform: no reduction in the scoring mode
  for (int m = 32; m > 0; m >>= 1) {
    const unsigned long long o = __shfl_xor(key, m, 64);
    key = o > key ? o : key;
  }
  if ((tid & 63) == 0) red[tid >> 6] = key;
  __syncthreads();
  if (tid == 0) {
    unsigned long long k = red[0];
    for (int w = 1; w < static_cast<int>(blockDim.x / 64); ++w) k = red[w] > k ? red[w] : k;
    atomicMax(best, k);
  }
}

// RTCSM3D, v3 (bricks under 2^22 cells): same candidates, sums and key as
// v2, about half the VALU per lookup (the v2 kernel is VALU-bound at ~33
// instructions per lookup):
//  * the rotated points are stored pre-scaled, a' = a * (1 / res), and each
//    thread holds its translation pre-scaled, tr' = tr * (1 / res): a cell
//    coordinate is rint(a' + tr') (one add, not an add and a multiply);
//  * one rounding-safety test per lookup: the largest |y - rint(y)| of the
//    three axes against 0.5 - eps, eps an absolute bound on |(a' + tr') -
//    fl(fl(a + tr) / res)| from the magnitudes of a' and tr' (host, per
//    launch); lookups within eps of a half-integer take the exact IEEE path
//    (the point is re-rotated from the cloud, RoundDiv per axis);
//  * the clamp into the padded brick runs on the rounded coordinates with
//    per-thread bounds, and the byte offset is three exact float FMAs.
template <int U>
__global__ void __launch_bounds__(768)
rt3d_score3(const float* __restrict__ pad, int pnx, int pny, int pnz, int ox, int oy, int oz,
            float res, float inv, float eps, const float* __restrict__ points, int n,
            const float4* __restrict__ rot, const float* __restrict__ rot_angle,
            const float4* __restrict__ trans, int num_trans, int t_base, int num_rot, double wt,
            double wr, unsigned long long* __restrict__ best, float* __restrict__ scores,
            int scores_pitch) {
  __shared__ float4 rp[kRt3Rpb][kRt3Tile];
  __shared__ unsigned long long red[768 / 64];
  const int tid = threadIdx.x;
  const int sub = tid / num_trans;
  const int t = tid - sub * num_trans;
  const int r = blockIdx.x * kRt3Rpb + sub;
  const bool active = sub < kRt3Rpb && r < num_rot;
  const float4 tr = active ? trans[t] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* my = rp[active ? sub : 0];
  const float4 q = rot[min(r, num_rot - 1)];
  const float tsx = __fmul_rn(tr.x, inv), tsy = __fmul_rn(tr.y, inv), tsz = __fmul_rn(tr.z, inv);
  // Padded cell (ix + bx, iy + by, iz + bz), each coordinate clamped into
  // [0, pn - 1]: the rounded coordinate clamps into [-b, pn - 1 - b].
  const float bx = static_cast<float>(1 - ox), by = static_cast<float>(1 - oy),
              bz = static_cast<float>(1 - oz);
  const float lx = -bx, ly = -by, lz = -bz;
  const float hx = static_cast<float>(pnx - 1) - bx, hy = static_cast<float>(pny - 1) - by,
              hz = static_cast<float>(pnz - 1) - bz;
  const float sx = 4.f, sy = 4.f * static_cast<float>(pnx),
              sz = 4.f * static_cast<float>(pnx) * static_cast<float>(pny);
  const float base = 4.f * ((bz * static_cast<float>(pny) + by) * static_cast<float>(pnx) + bx);
  const float half = 0.5f - eps;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(pad), 0, static_cast<int>(4u * pnx * pny * pnz), 0x00020000);
  float sum = 0.f;
  for (int tb = 0; tb < n; tb += kRt3Tile) {
    const int cnt = min(kRt3Tile, n - tb);
    __syncthreads();
    for (int i = tid; i < kRt3Rpb * cnt; i += blockDim.x) {
      const int s2 = i / cnt, j = i - s2 * cnt;
      const int rr = min(blockIdx.x * kRt3Rpb + s2, num_rot - 1);
      const float4 qq = rot[rr];
      const float* p = points + 3 * static_cast<int64_t>(tb + j);
      float ox_, oy_, oz_;
      Rotate3(qq.w, qq.x, qq.y, qq.z, p[0], p[1], p[2], &ox_, &oy_, &oz_);
      rp[s2][j] = make_float4(__fmul_rn(ox_, inv), __fmul_rn(oy_, inv), __fmul_rn(oz_, inv), 0.f);
    }
    __syncthreads();
    if (active) {
      // Cell coordinates of point i for this thread's translation, with the
      // rounding-safety test; the rare lookups within eps of a half-integer
      // take the reference's IEEE quotient (the point re-rotated from the
      // cloud, RoundDiv per axis).
      auto cell = [&](int i, float* rx, float* ry, float* rz) {
        const float4 a = my[i];
        const float yx = __fadd_rn(a.x, tsx), yy = __fadd_rn(a.y, tsy), yz = __fadd_rn(a.z, tsz);
        *rx = rintf(yx);
        *ry = rintf(yy);
        *rz = rintf(yz);
        const float dm = fmaxf(fmaxf(fabsf(__fsub_rn(yx, *rx)), fabsf(__fsub_rn(yy, *ry))),
                               fabsf(__fsub_rn(yz, *rz)));
        return dm;
      };
      auto exact = [&](int i, float* rx, float* ry, float* rz) {
        const float* p = points + 3 * static_cast<int64_t>(tb + i);
        float ax, ay, az;
        Rotate3(q.w, q.x, q.y, q.z, p[0], p[1], p[2], &ax, &ay, &az);
        *rx = static_cast<float>(RoundDiv(__fadd_rn(ax, tr.x), res, inv));
        *ry = static_cast<float>(RoundDiv(__fadd_rn(ay, tr.y), res, inv));
        *rz = static_cast<float>(RoundDiv(__fadd_rn(az, tr.z), res, inv));
      };
      auto offset = [&](float rx, float ry, float rz) {
        rx = __builtin_amdgcn_fmed3f(rx, lx, hx);
        ry = __builtin_amdgcn_fmed3f(ry, ly, hy);
        rz = __builtin_amdgcn_fmed3f(rz, lz, hz);
        // Exact: every term is an integer below 2^24.
        return static_cast<int>(fmaf(rz, sz, fmaf(ry, sy, fmaf(rx, sx, base))));
      };
      // U points per step: their U gathers are issued together and added in
      // point order afterwards (the same float sum, U loads in flight).
      int i = 0;
      for (; i + U <= cnt; i += U) {
        float rx[U], ry[U], rz[U], dm[U];
#pragma unroll
        for (int u = 0; u < U; ++u) dm[u] = cell(i + u, &rx[u], &ry[u], &rz[u]);
        float dmax = dm[0];
#pragma unroll
        for (int u = 1; u < U; ++u) dmax = fmaxf(dmax, dm[u]);
        if (dmax >= half) {
#pragma unroll
          for (int u = 0; u < U; ++u)
            if (dm[u] >= half) exact(i + u, &rx[u], &ry[u], &rz[u]);
        }
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
          v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
              rsrc, offset(rx[u], ry[u], rz[u]), 0, 0));
#pragma unroll
        for (int u = 0; u < U; ++u) sum = __fadd_rn(sum, v[u]);
      }
      for (; i < cnt; ++i) {
        float rx, ry, rz;
        if (cell(i, &rx, &ry, &rz) >= half) exact(i, &rx, &ry, &rz);
        sum = __fadd_rn(sum, __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                                 rsrc, offset(rx, ry, rz), 0, 0)));
      }
    }
  }
  unsigned long long key = 0;
  if (active) {
    float score = __fdiv_rn(sum, static_cast<float>(n));
    const double e = static_cast<double>(tr.w) * wt + static_cast<double>(rot_angle[r]) * wr;
    score = static_cast<float>(static_cast<double>(score) * exp(-(e * e)));
    const unsigned idx = static_cast<unsigned>(t_base + t) * static_cast<unsigned>(num_rot) + r;
    key = (static_cast<unsigned long long>(__float_as_uint(score)) << 32) | (0xffffffffu - idx);
    if (scores) scores[static_cast<int64_t>(r) * scores_pitch + t_base + t] = score;
  }
  if (scores) return;  // uniform: no reduction in the scoring mode
  for (int m = 32; m > 0; m >>= 1) {
    const unsigned long long o = __shfl_xor(key, m, 64);
    key = o > key ? o : key;
  }
  if ((tid & 63) == 0) red[tid >> 6] = key;
  __syncthreads();
  if (tid == 0) {
    unsigned long long k = red[0];
    for (int w = 1; w < static_cast<int>(blockDim.x / 64); ++w) k = red[w] > k ? red[w] : k;
    atomicMax(best, k);
  }
}

// RTCSM3D, v4: the same candidates, cell rule, sums and key as v3, with the
// lanes of a wave on 64 ROTATIONS (a 4 x 4 x 4 block of the angular lattice)
// and the waves on translations (kRt4Tw each). For one point and one
// translation, neighbouring rotations move the point by about a cell at the
// scan's maximum range and by a fraction of one nearer in, so a gather
// touches ~4 cache lines instead of the ~15 of 64 translations of one
// rotation (tools/rt3d_lines_sim.py). Each lane rotates the points of a tile
// by its own rotation into LDS (shared by the workgroup's translations). The
// brick is padded by P cells of 0.1 per side; a point whose scaled rotation
// lies inside [safe_lo, safe_hi] (host: the padded box shrunk by every
// translation's reach) needs no clamp for any translation, the others and
// the rounding band take the clamped, exact path.
__global__ void __launch_bounds__(64 * kRt4Waves)
rt3d_score4(const float* __restrict__ pad, int pnx, int pny, int pnz, float bx, float by, float bz,
            float res, float inv, float eps, float4 safe_lo, float4 safe_hi,
            const float* __restrict__ points, int n, const float4* __restrict__ rot,
            const int* __restrict__ rot_index, const float* __restrict__ rot_angle,
            const float4* __restrict__ trans, int num_trans, int num_rot, double wt, double wr,
            unsigned long long* __restrict__ best, float* __restrict__ scores, int scores_pitch) {
  __shared__ float4 rp[kRt4Tile][64];
  __shared__ unsigned long long red[kRt4Waves];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slot = blockIdx.x * 64 + lane;
  const int ri = rot_index[slot];
  const float4 q = rot[slot];  // (x, y, z, w); identity in holes
  const int t0 = (blockIdx.y * kRt4Waves + wave) * kRt4Tw;
  float tsx[kRt4Tw], tsy[kRt4Tw], tsz[kRt4Tw];
  float4 tr[kRt4Tw];
#pragma unroll
  for (int u = 0; u < kRt4Tw; ++u) {
    tr[u] = trans[min(t0 + u, num_trans - 1)];
    tsx[u] = __fmul_rn(tr[u].x, inv);
    tsy[u] = __fmul_rn(tr[u].y, inv);
    tsz[u] = __fmul_rn(tr[u].z, inv);
  }
  const float lx = -bx, ly = -by, lz = -bz;
  const float hx = static_cast<float>(pnx - 1) - bx, hy = static_cast<float>(pny - 1) - by,
              hz = static_cast<float>(pnz - 1) - bz;
  const float sx = 4.f, sy = 4.f * static_cast<float>(pnx),
              sz = 4.f * static_cast<float>(pnx) * static_cast<float>(pny);
  const float base = 4.f * ((bz * static_cast<float>(pny) + by) * static_cast<float>(pnx) + bx);
  const float half = 0.5f - eps;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(pad), 0, static_cast<int>(4u * pnx * pny * pnz), 0x00020000);
  float sum[kRt4Tw];
#pragma unroll
  for (int u = 0; u < kRt4Tw; ++u) sum[u] = 0.f;
  for (int tb = 0; tb < n; tb += kRt4Tile) {
    const int cnt = min(kRt4Tile, n - tb);
    __syncthreads();
    for (int j = wave; j < cnt; j += kRt4Waves) {
      const float* p = points + 3 * static_cast<int64_t>(tb + j);
      float ax, ay, az;
      Rotate3(q.w, q.x, q.y, q.z, p[0], p[1], p[2], &ax, &ay, &az);
      const float sxv = __fmul_rn(ax, inv), syv = __fmul_rn(ay, inv), szv = __fmul_rn(az, inv);
      const bool inside = sxv >= safe_lo.x && sxv <= safe_hi.x && syv >= safe_lo.y &&
                          syv <= safe_hi.y && szv >= safe_lo.z && szv <= safe_hi.z;
      rp[j][lane] = make_float4(sxv, syv, szv, inside ? 0.f : 1.f);
    }
    __syncthreads();
    for (int i = 0; i < cnt; ++i) {
      const float4 a = rp[i][lane];
      float rx[kRt4Tw], ry[kRt4Tw], rz[kRt4Tw], dm[kRt4Tw];
      float dmax = a.w;  // 1 outside the safe box: the clamped path
#pragma unroll
      for (int u = 0; u < kRt4Tw; ++u) {
        const float yx = __fadd_rn(a.x, tsx[u]), yy = __fadd_rn(a.y, tsy[u]),
                    yz = __fadd_rn(a.z, tsz[u]);
        rx[u] = rintf(yx);
        ry[u] = rintf(yy);
        rz[u] = rintf(yz);
        dm[u] = fmaxf(fmaxf(fabsf(__fsub_rn(yx, rx[u])), fabsf(__fsub_rn(yy, ry[u]))),
                      fabsf(__fsub_rn(yz, rz[u])));
        dmax = fmaxf(dmax, dm[u]);
      }
      if (dmax >= half) {  // rare: exact quotient and / or clamp
        const float* p = points + 3 * static_cast<int64_t>(tb + i);
        float ax, ay, az;
        Rotate3(q.w, q.x, q.y, q.z, p[0], p[1], p[2], &ax, &ay, &az);
#pragma unroll
        for (int u = 0; u < kRt4Tw; ++u) {
          if (dm[u] >= half) {
            rx[u] = static_cast<float>(RoundDiv(__fadd_rn(ax, tr[u].x), res, inv));
            ry[u] = static_cast<float>(RoundDiv(__fadd_rn(ay, tr[u].y), res, inv));
            rz[u] = static_cast<float>(RoundDiv(__fadd_rn(az, tr[u].z), res, inv));
          }
          rx[u] = __builtin_amdgcn_fmed3f(rx[u], lx, hx);
          ry[u] = __builtin_amdgcn_fmed3f(ry[u], ly, hy);
          rz[u] = __builtin_amdgcn_fmed3f(rz[u], lz, hz);
        }
      }
      float v[kRt4Tw];
#pragma unroll
      for (int u = 0; u < kRt4Tw; ++u) {
        // Exact: every term is an integer below 2^24.
        const float off = fmaf(rz[u], sz, fmaf(ry[u], sy, fmaf(rx[u], sx, base)));
        v[u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, static_cast<int>(off), 0, 0));
      }
#pragma unroll
      for (int u = 0; u < kRt4Tw; ++u) sum[u] = __fadd_rn(sum[u], v[u]);
    }
  }
  unsigned long long key = 0;
#pragma unroll
  for (int u = 0; u < kRt4Tw; ++u) {
    const int t = t0 + u;
    if (ri < 0 || t >= num_trans) continue;
    float score = __fdiv_rn(sum[u], static_cast<float>(n));
    const double e = static_cast<double>(tr[u].w) * wt + static_cast<double>(rot_angle[ri]) * wr;
    score = static_cast<float>(static_cast<double>(score) * exp(-(e * e)));
    const unsigned idx = static_cast<unsigned>(t) * static_cast<unsigned>(num_rot) + ri;
    const unsigned long long k =
        (static_cast<unsigned long long>(__float_as_uint(score)) << 32) | (0xffffffffu - idx);
    key = k > key ? k : key;
    if (scores) scores[static_cast<int64_t>(ri) * scores_pitch + t] = score;
  }
  if (scores) return;  // uniform: no reduction in the scoring mode
  for (int m = 32; m > 0; m >>= 1) {
    const unsigned long long o = __shfl_xor(key, m, 64);
    key = o > key ? o : key;
  }
  if (lane == 0) red[wave] = key;
  __syncthreads();
  if (tid == 0) {
    unsigned long long k = red[0];
    for (int w = 1; w < kRt4Waves; ++w) k = red[w] > k ? red[w] : k;
    atomicMax(best, k);
  }
}

// RTCSM3D, v5 (column gathers): as v4 — lanes on a 4 x 4 x 4 block of
// rotations — but each wave takes one (x, y) column of the translation
// lattice with all NL of its z steps, over a padded brick stored z-fastest.
// The kernels above are bound by the texture address path (TA/TD 91-99%
// busy at ~23-26 cycles per 64-lane dword gather, profiles/r2d/pmc_rt3d):
// the per-instruction cost, not bytes or lines. Along a z column the cell of
// step k is the cell of step 0 plus k in z whenever the rounding of step 0
// clears the column's drift (host: per column and axis, the largest
// |t'(k) - t'(0) - k e_z| plus a rounding allowance), so one lane fetches its
// NL cells with one or two 16-byte loads and adds them to NL sums in point
// order. A lookup that fails the column test (or a point outside the safe
// box) takes v3's per-step path: fast rounding or the IEEE quotient, clamp.
template <int NL>
__global__ void __launch_bounds__(64 * NL)
rt3d_score5(const float* __restrict__ col, int pnx, int pny, int pnz, float bx, float by, float bz,
            float res, float inv, float eps, float4 safe_lo, float4 safe_hi,
            const float* __restrict__ points, int n, const float4* __restrict__ rot,
            const int* __restrict__ rot_index, const float* __restrict__ rot_angle,
            const float4* __restrict__ trans, const float4* __restrict__ col_t0,
            const float4* __restrict__ col_thr, int num_rot, double wt, double wr,
            unsigned long long* __restrict__ best, float* __restrict__ scores, int scores_pitch) {
  __shared__ float4 rp[kRt4Tile][64];
  __shared__ unsigned long long red[NL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int slot = blockIdx.x * 64 + lane;
  const int ri = rot_index[slot];
  const float4 q = rot[slot];
  const int c = blockIdx.y * NL + wave;  // column (y, x) of the lattice
  constexpr int kCols = NL * NL;
  const float4 t0 = col_t0[c], th = col_thr[c];
  const float lx = -bx, ly = -by, lz = -bz;
  const float hx = static_cast<float>(pnx - 1) - bx, hy = static_cast<float>(pny - 1) - by,
              hz = static_cast<float>(pnz - 1) - bz;
  // z-fastest: byte offset 4 * (((x + bx) * pny + (y + by)) * pnz + (z + bz)).
  const float sx = 4.f * static_cast<float>(pny) * static_cast<float>(pnz),
              sy = 4.f * static_cast<float>(pnz), sz = 4.f;
  const float base = 4.f * ((bx * static_cast<float>(pny) + by) * static_cast<float>(pnz) + bz);
  const float half = 0.5f - eps;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(col), 0, static_cast<int>(4u * pnx * pny * pnz), 0x00020000);
  float sum[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) sum[k] = 0.f;
  for (int tb = 0; tb < n; tb += kRt4Tile) {
    const int cnt = min(kRt4Tile, n - tb);
    __syncthreads();
    for (int j = wave; j < cnt; j += NL) {
      const float* p = points + 3 * static_cast<int64_t>(tb + j);
      float ax, ay, az;
      Rotate3(q.w, q.x, q.y, q.z, p[0], p[1], p[2], &ax, &ay, &az);
      const float sxv = __fmul_rn(ax, inv), syv = __fmul_rn(ay, inv), szv = __fmul_rn(az, inv);
      const bool inside = sxv >= safe_lo.x && sxv <= safe_hi.x && syv >= safe_lo.y &&
                          syv <= safe_hi.y && szv >= safe_lo.z && szv <= safe_hi.z;
      rp[j][lane] = make_float4(sxv, syv, szv, inside ? 0.f : 1.f);
    }
    __syncthreads();
    for (int i = 0; i < cnt; ++i) {
      const float4 a = rp[i][lane];
      const float yx = __fadd_rn(a.x, t0.x), yy = __fadd_rn(a.y, t0.y), yz = __fadd_rn(a.z, t0.z);
      const float rx = rintf(yx), ry = rintf(yy), rz = rintf(yz);
      // Column test: every step's rounding is step 0's (+k in z), clear of the band.
      const float m = fmaxf(fmaxf(__fsub_rn(fabsf(__fsub_rn(yx, rx)), th.x),
                                  __fsub_rn(fabsf(__fsub_rn(yy, ry)), th.y)),
                            fmaxf(__fsub_rn(fabsf(__fsub_rn(yz, rz)), th.z), __fsub_rn(a.w, 0.5f)));
      float v[NL];
      if (m < 0.f) {
        // The column's NL cells: ceil(NL / 4) 16-byte loads (one or two up to
        // 7 steps, three for 9 and 11, four for 13 and 15); the cells read
        // past the column's last step are discarded.
        const float off = fmaf(rz, sz, fmaf(ry, sy, fmaf(rx, sx, base)));  // exact (< 2^24)
        const int o = static_cast<int>(off);
        constexpr int kLoads = (NL + 3) / 4;
        decltype(__builtin_amdgcn_raw_buffer_load_b128(rsrc, 0, 0, 0)) q4[kLoads];
#pragma unroll
        for (int j = 0; j < kLoads; ++j) q4[j] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o + 16 * j, 0, 0);
#pragma unroll
        for (int k = 0; k < NL; ++k) v[k] = __uint_as_float(q4[k >> 2][k & 3]);
      } else {  // rare: v3's per-step path
        const float* p = points + 3 * static_cast<int64_t>(tb + i);
        float ax, ay, az;
        Rotate3(q.w, q.x, q.y, q.z, p[0], p[1], p[2], &ax, &ay, &az);
#pragma unroll
        for (int k = 0; k < NL; ++k) {
          const float4 tr = trans[k * kCols + c];
          const float tx = __fmul_rn(tr.x, inv), ty = __fmul_rn(tr.y, inv), tz = __fmul_rn(tr.z, inv);
          const float ux = __fadd_rn(a.x, tx), uy = __fadd_rn(a.y, ty), uz = __fadd_rn(a.z, tz);
          float ox = rintf(ux), oy = rintf(uy), oz = rintf(uz);
          const float dm = fmaxf(fmaxf(fabsf(__fsub_rn(ux, ox)), fabsf(__fsub_rn(uy, oy))),
                                 fabsf(__fsub_rn(uz, oz)));
          if (dm >= half) {
            ox = static_cast<float>(RoundDiv(__fadd_rn(ax, tr.x), res, inv));
            oy = static_cast<float>(RoundDiv(__fadd_rn(ay, tr.y), res, inv));
            oz = static_cast<float>(RoundDiv(__fadd_rn(az, tr.z), res, inv));
          }
          ox = __builtin_amdgcn_fmed3f(ox, lx, hx);
          oy = __builtin_amdgcn_fmed3f(oy, ly, hy);
          oz = __builtin_amdgcn_fmed3f(oz, lz, hz);
          const float off = fmaf(oz, sz, fmaf(oy, sy, fmaf(ox, sx, base)));
          v[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, static_cast<int>(off), 0, 0));
        }
      }
#pragma unroll
      for (int k = 0; k < NL; ++k) sum[k] = __fadd_rn(sum[k], v[k]);
    }
  }
  unsigned long long key = 0;
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int t = k * kCols + c;
    if (ri < 0) continue;
    float score = __fdiv_rn(sum[k], static_cast<float>(n));
    const double e = static_cast<double>(trans[t].w) * wt + static_cast<double>(rot_angle[ri]) * wr;
    score = static_cast<float>(static_cast<double>(score) * exp(-(e * e)));
    const unsigned idx = static_cast<unsigned>(t) * static_cast<unsigned>(num_rot) + ri;
    const unsigned long long kk =
        (static_cast<unsigned long long>(__float_as_uint(score)) << 32) | (0xffffffffu - idx);
    key = kk > key ? kk : key;
    if (scores) scores[static_cast<int64_t>(ri) * scores_pitch + t] = score;
  }
  if (scores) return;  // uniform: no reduction in the scoring mode
  for (int mm = 32; mm > 0; mm >>= 1) {
    const unsigned long long o = __shfl_xor(key, mm, 64);
    key = o > key ? o : key;
  }
  if (lane == 0) red[wave] = key;
  __syncthreads();
  if (tid == 0) {
    unsigned long long k = red[0];
    for (int w = 1; w < NL; ++w) k = red[w] > k ? red[w] : k;
    atomicMax(best, k);
  }
}

// The brick padded by P cells of 0.1 per side, z fastest (rt3d_score5).
__global__ void pad_prob_brick_zfast(const float* __restrict__ prob, Brick3 gb, int P,
                                     float* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int px = gb.nx + 2 * P, py = gb.ny + 2 * P, pz = gb.nz + 2 * P;
  if (i >= static_cast<int64_t>(px) * py * pz) return;
  const int z = static_cast<int>(i % pz) - P;
  const int y = static_cast<int>((i / pz) % py) - P;
  const int x = static_cast<int>(i / (static_cast<int64_t>(pz) * py)) - P;
  float v = 0.1f;
  if (x >= 0 && x < gb.nx && y >= 0 && y < gb.ny && z >= 0 && z < gb.nz)
    v = prob[(static_cast<int64_t>(z) * gb.ny + y) * gb.nx + x];
  out[i] = v;
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

static_assert(kMax3dWindow < 32768, "leaf offsets are kept as int16 in LDS");
template <int kPts, int kStack, int kBatch>
struct F3SharedT {
  // The discretized cloud: full-resolution cells (int16 x, y, z), or — once
  // roots are scored from the cell list — packed words relative to an origin
  // aligned to 2^E (PackedCloud below).
  union {
    struct {
      int16_t x[kPts], y[kPts], z[kPts];
    } c;
    uint32_t pk[kPts];
  } cloud;
  int org[3];              // packed origin (full-resolution cells)
  int rel_min[3], rel_max[3];
  int fmin[3], fmax[3];    // full-resolution cloud bounds
  int packed;
  int16_t sx[kStack], sy[kStack], sz[kStack];
  int8_t sd[kStack];
  int ssum[kStack];
  float lr[kSearch3dThreads];
  alignas(16) uint8_t top[kTopLds3d];
  int bn_x[kBatch], bn_y[kBatch], bn_z[kBatch], bn_d[kBatch];
  unsigned long long leaf_keys[8 * kBatch];
  int16_t leaf_x[8 * kBatch], leaf_y[8 * kBatch], leaf_z[8 * kBatch];  // |offset| <= kMax3dWindow
  int rmin[3], rmax[3];  // bounds of the cloud's cells at the top level
  int16_t rbx[kRootScore3d], rby[kRootScore3d], rbz[kRootScore3d];
  int rbs[kRootScore3d];
  int nroot;
  // The cloud at top-level resolution as distinct cells with counts (root
  // sums = sum over cells of count x top[cell + offset]).
  int tcell[kTopCells3d];
  uint16_t tcount[kTopCells3d];
  int ntcell;
  int nbatch, nleaf, sp, item, error, skip, cached_submap, high_water;
  int tie_sum;   // a sum the witness keys already show two passing leaves at (-1: none)
  int abandon;   // collect pass: the pair's tied leaves overflowed the record
  unsigned long long best;
  unsigned long long best_seen;  // last read of the pair's global best
};

__device__ __forceinline__ unsigned long long LeafId(const Pair3Desc& pd, int yaw, int ox, int oy,
                                                     int oz) {
  unsigned long long id = static_cast<unsigned long long>(yaw);
  id = (id << pd.bits_xy) | static_cast<unsigned long long>(ox + pd.wxy);
  id = (id << pd.bits_xy) | static_cast<unsigned long long>(oy + pd.wxy);
  id = (id << pd.bits_z) | static_cast<unsigned long long>(oz + pd.wz);
  return id;
}

// Low-resolution matcher score of a leaf pose (low_resolution_matcher.cc:23-35):
// float sum in point order. Probabilities are computed in parallel, summed
// sequentially by thread 0. Result valid in thread 0.
template <class Shared>
__device__ float LowResScore(Shared& sh, const Submap3Desc& sm, const float* __restrict__ low_pts,
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

// Phase timers of thread 0 (s_memtime), compiled in with -DCSM_KPROF only:
// they cost ~24 VGPRs. stats[1 + slot]: 0 item+discretize, 7 top copy,
// 8 cloud box, 9 cell list, 1 roots, 2 sort, 3 DFS + leaves (cycles);
// 5 batches, 6 leaves, 11 roots kept (counts).
#ifdef CSM_KPROF
#define F3_PROF_DECL long long prof[12] = {}, t_mark = 0
#define F3_RESET() (t_mark = clock64())
#define F3_MARK(slot)                    \
  do {                                   \
    if (tid == 0) {                      \
      const long long now_ = clock64();  \
      prof[slot] += now_ - t_mark;       \
      t_mark = now_;                     \
    }                                    \
  } while (0)
#define F3_COUNT(slot, v) \
  do {                    \
    if (tid == 0) prof[slot] += (v); \
  } while (0)
#define F3_FLUSH(stats)                                                                   \
  do {                                                                                    \
    if (tid == 0 && (stats))                                                              \
      for (int k_ = 0; k_ < 12; ++k_)                                                     \
        atomicAdd((stats) + 1 + k_, static_cast<unsigned long long>(prof[k_]));          \
  } while (0)
#else
#define F3_PROF_DECL (void)0
#define F3_RESET() (void)0
#define F3_MARK(slot) (void)0
#define F3_COUNT(slot, v) (void)0
#define F3_FLUSH(stats) (void)0
#endif

// kPts: cloud capacity in LDS; kWaves: waves per SIMD the kernel is built
// for (= workgroups per CU with 256 threads); kStack: DFS stack entries in
// LDS (the rest of kDfsCap3d spills to global memory); kInflight: octet
// loads a lane keeps in flight (16, 12, 8 or 4); kBatch: DFS nodes scored
// per step (16 or 32: 16 or 8 lanes each).
template <int kPts, int kWaves, int kStack, int kInflight, int kBatch>
__global__ void __launch_bounds__(kSearch3dThreads) __attribute__((amdgpu_waves_per_eu(kWaves, kWaves)))
fast3d_search(const Submap3Desc* __restrict__ submaps, const Pair3Desc* __restrict__ pairs,
              const Yaw3Desc* __restrict__ yaws, int item_begin, int num_items,
              const float* __restrict__ points,
              const float* __restrict__ low_points, unsigned* __restrict__ counter,
              unsigned long long* __restrict__ best, int32_t* __restrict__ status,
              unsigned long long* __restrict__ stats, int4* __restrict__ spill_base,
              unsigned long long* __restrict__ best_hi, uint4* __restrict__ ties,
              int32_t* __restrict__ tie_count) {
  static_assert(kInflight == 16 || kInflight == 12 || kInflight == 8 || kInflight == 4, "");
  __shared__ F3SharedT<kPts, kStack, kBatch> sh;
  const int tid = threadIdx.x;
  unsigned long long lookups = 0, root_lookups = 0;
  F3_PROF_DECL;
  // DFS stack entries past kStack live in this workgroup's spill region
  // (global memory, written and read only by this workgroup's waves).
  int4* spill = spill_base + static_cast<size_t>(blockIdx.x) * (kDfsCap3d - kStack);
  if (tid == 0) {
    sh.cached_submap = -1;
    sh.high_water = 0;
  }
  for (;;) {
    if (tid == 0) sh.item = static_cast<int>(atomicAdd(counter, 1u));
    __syncthreads();
    if (sh.item >= num_items) break;
    const int item = item_begin + sh.item;
    F3_RESET();
    const Yaw3Desc yw = yaws[item];
    const Pair3Desc pd = pairs[yw.pair];
    const Submap3Desc& sm = submaps[pd.submap];
    const int n = pd.num_points;
    const float res = sm.resolution, inv = 1.f / sm.resolution;
    const int top = pd.root_level;
    const int te = max(0, top - sm.full_resolution_depth + 1);
    const bool treduced = top >= sm.full_resolution_depth;
    const int lwx = (-pd.wxy) >> te, lwy = (-pd.wxy) >> te, lwz = (-pd.wz) >> te;
    if (tid == 0) {
      sh.error = 0;
      sh.sp = 0;
      sh.best = best[yw.pair];
      sh.best_seen = 0;
      sh.tie_sum = -1;
      sh.abandon = 0;
    }
    if (tid < 3) {
      sh.rmin[tid] = 1 << 30;
      sh.rmax[tid] = -(1 << 30);
      sh.fmin[tid] = 1 << 30;
      sh.fmax[tid] = -(1 << 30);
    }
    __syncthreads();
    // DiscretizeScan (:201-244): cell of pose * p at full resolution, with
    // the cloud's box at full resolution and at the root level (in the
    // reduced coordinates the roots are scored in).
    {
      int mn[3] = {1 << 30, 1 << 30, 1 << 30}, mx[3] = {-(1 << 30), -(1 << 30), -(1 << 30)};
      int fmn[3] = {1 << 30, 1 << 30, 1 << 30}, fmx[3] = {-(1 << 30), -(1 << 30), -(1 << 30)};
      for (int i = tid; i < n; i += kSearch3dThreads) {
        const float* p = points + 3 * (pd.point_offset + i);
        float ox, oy, oz;
        Rotate3(yw.qw, yw.qx, yw.qy, yw.qz, p[0], p[1], p[2], &ox, &oy, &oz);
        const int ix = RoundDiv(__fadd_rn(ox, yw.tx), res, inv);
        const int iy = RoundDiv(__fadd_rn(oy, yw.ty), res, inv);
        const int iz = RoundDiv(__fadd_rn(oz, yw.tz), res, inv);
        if (abs(ix) > kCellLimit3d || abs(iy) > kCellLimit3d || abs(iz) > kCellLimit3d) sh.error = 1;
        sh.cloud.c.x[i] = static_cast<int16_t>(ix);
        sh.cloud.c.y[i] = static_cast<int16_t>(iy);
        sh.cloud.c.z[i] = static_cast<int16_t>(iz);
        int c[3] = {ix, iy, iz};
        for (int a = 0; a < 3; ++a) {
          fmn[a] = min(fmn[a], c[a]);
          fmx[a] = max(fmx[a], c[a]);
        }
        if (treduced) {
          c[0] = ((c[0] - pd.wxy) >> te) - lwx;
          c[1] = ((c[1] - pd.wxy) >> te) - lwy;
          c[2] = ((c[2] - pd.wz) >> te) - lwz;
        }
        for (int a = 0; a < 3; ++a) {
          mn[a] = min(mn[a], c[a]);
          mx[a] = max(mx[a], c[a]);
        }
      }
      for (int a = 0; a < 3; ++a) {
        for (int m = 32; m > 0; m >>= 1) {
          mn[a] = min(mn[a], __shfl_xor(mn[a], m, 64));
          mx[a] = max(mx[a], __shfl_xor(mx[a], m, 64));
          fmn[a] = min(fmn[a], __shfl_xor(fmn[a], m, 64));
          fmx[a] = max(fmx[a], __shfl_xor(fmx[a], m, 64));
        }
      }
      if ((tid & 63) == 0) {
        for (int a = 0; a < 3; ++a) {
          atomicMin(&sh.rmin[a], mn[a]);
          atomicMax(&sh.rmax[a], mx[a]);
          atomicMin(&sh.fmin[a], fmn[a]);
          atomicMax(&sh.fmax[a], fmx[a]);
        }
      }
    }
    __syncthreads();
    if (sh.error) {
      if (tid == 0) atomicExch(reinterpret_cast<int*>(status + yw.pair), -4);
      __syncthreads();
      continue;
    }
    F3_MARK(0);
    const int step = 1 << top;
    const int T = pd.top_nx * pd.top_ny * pd.top_nz;
    // Lowest-resolution candidates (GenerateLowestResolutionCandidates
    // :297-330), in chunks of kRootChunk3d: each chunk is scored (one root
    // per lane, the top level from LDS when it fits), ordered best last and
    // searched to exhaustion before the next one.
    const Brick3 tb = sm.level[top];
    const int64_t tbytes = static_cast<int64_t>(tb.nx) * tb.ny * tb.nz;
    const int tvec = static_cast<int>((tbytes + 15) / 16);  // level offsets are 256-aligned
    const bool lds_top = tvec * 16 <= kTopLds3d;
    if (lds_top && sh.cached_submap != pd.submap * 16 + top) {
      const uint4* src = reinterpret_cast<const uint4*>(sm.levels + tb.offset);
      uint4* dst = reinterpret_cast<uint4*>(sh.top);
      static_assert(kTopLds3d <= 2 * 16 * kSearch3dThreads, "two 16-byte pieces per thread");
      const int k0 = tid, k1 = tid + kSearch3dThreads;
      uint4 v0 = make_uint4(0, 0, 0, 0), v1 = make_uint4(0, 0, 0, 0);
      if (k0 < tvec) v0 = src[k0];
      if (k1 < tvec) v1 = src[k1];
      if (k0 < tvec) dst[k0] = v0;
      if (k1 < tvec) dst[k1] = v1;
      __syncthreads();
      if (tid == 0) sh.cached_submap = pd.submap * 16 + top;
    }
    __syncthreads();
    F3_MARK(7);
    const uint8_t* tglobal = sm.levels + tb.offset;
    F3_MARK(8);
    // Histogram of the cloud's top-level cells over its box (count grid in
    // the empty stack sums), compacted to a list when box and list fit.
    const int gbx = sh.rmax[0] - sh.rmin[0] + 1, gby = sh.rmax[1] - sh.rmin[1] + 1,
              gbz = sh.rmax[2] - sh.rmin[2] + 1;
    const bool use_cells = n > 0 && static_cast<int64_t>(gbx) * gby * gbz <= kStack &&
                           sh.rmin[0] >= -1024 && sh.rmax[0] < 1024 && sh.rmin[1] >= -1024 &&
                           sh.rmax[1] < 1024 && sh.rmin[2] >= -512 && sh.rmax[2] < 512;
    if (use_cells) {
      for (int k = tid; k < gbx * gby * gbz; k += kSearch3dThreads) sh.ssum[k] = 0;
      if (tid == 0) sh.ntcell = 0;
      __syncthreads();
      for (int i = tid; i < n; i += kSearch3dThreads) {
        int c[3] = {sh.cloud.c.x[i], sh.cloud.c.y[i], sh.cloud.c.z[i]};
        if (treduced) {
          c[0] = ((c[0] - pd.wxy) >> te) - lwx;
          c[1] = ((c[1] - pd.wxy) >> te) - lwy;
          c[2] = ((c[2] - pd.wz) >> te) - lwz;
        }
        atomicAdd(&sh.ssum[((c[2] - sh.rmin[2]) * gby + (c[1] - sh.rmin[1])) * gbx + (c[0] - sh.rmin[0])], 1);
      }
      __syncthreads();
      for (int k = tid; k < gbx * gby * gbz; k += kSearch3dThreads) {
        const int cnt = sh.ssum[k];
        if (cnt > 0) {
          const int at = atomicAdd(&sh.ntcell, 1);
          if (at < kTopCells3d) {
            const int x = k % gbx + sh.rmin[0], y = (k / gbx) % gby + sh.rmin[1],
                      z = k / (gbx * gby) + sh.rmin[2];
            sh.tcell[at] = (x + 1024) | ((y + 1024) << 11) | ((z + 512) << 22);
            sh.tcount[at] = static_cast<uint16_t>(cnt);
          }
        }
      }
      __syncthreads();
    }
    const bool cells_ok = use_cells && sh.ntcell <= kTopCells3d;
    const int ntc = cells_ok ? sh.ntcell : 0;
    // Packed cloud for the DFS (only when roots are scored from the cell list:
    // nothing reads the int16 cells after this). Origin o = w + 2^E * floor((min
    // - w) / 2^E), E the largest reduction exponent of the DFS child levels, so
    // that ((c - w) >> e) = ((o - w) >> e) + ((c - o) >> e) for every e <= E.
    // Fields: x bits 0-10, y 11-21, z 22-31 of c - o; the words are recomputed
    // from the points with the discretization's arithmetic.
    if (tid == 0) {
      const int E = max(0, (top - 1) - sm.full_resolution_depth + 1);
      const int w3[3] = {pd.wxy, pd.wxy, pd.wz};
      const int lim[3] = {2048, 2048, 1024};
      bool ok = cells_ok && n > 0 && top >= 1 && E <= 9;
      for (int l = 0; ok && l < top; ++l)  // slab strides fit __umul24
        ok = static_cast<int64_t>(sm.oct[l].nx) * sm.oct[l].ny * 8 < (1 << 24);
      for (int a = 0; a < 3; ++a) {
        const int o = w3[a] + (((sh.fmin[a] - w3[a]) >> E) << E);
        sh.org[a] = o;
        sh.rel_min[a] = sh.fmin[a] - o;
        sh.rel_max[a] = sh.fmax[a] - o;
        ok = ok && sh.rel_max[a] < lim[a];
      }
      sh.packed = ok;
    }
    __syncthreads();
    const bool packed = sh.packed;
    if (packed) {
      for (int i = tid; i < n; i += kSearch3dThreads) {
        const float* p = points + 3 * (pd.point_offset + i);
        float ox, oy, oz;
        Rotate3(yw.qw, yw.qx, yw.qy, yw.qz, p[0], p[1], p[2], &ox, &oy, &oz);
        const int ix = RoundDiv(__fadd_rn(ox, yw.tx), res, inv) - sh.org[0];
        const int iy = RoundDiv(__fadd_rn(oy, yw.ty), res, inv) - sh.org[1];
        const int iz = RoundDiv(__fadd_rn(oz, yw.tz), res, inv) - sh.org[2];
        sh.cloud.pk[i] = static_cast<uint32_t>(ix) | (static_cast<uint32_t>(iy) << 11) |
                         (static_cast<uint32_t>(iz) << 22);
      }
    }
    __syncthreads();
    F3_MARK(9);
    // A root whose shifted cloud box misses the top-level brick sums to 0: it
    // cannot exceed min_score when min_sum > 0 and is not scored.
    const bool skip_empty = pd.min_sum > 0;
    for (int r0 = 0; r0 < T; r0 += kRootScore3d) {
    if (sh.abandon) break;  // uniform: written before the last batch's barrier
    const int r1 = min(T, r0 + kRootScore3d);
    if (tid == 0) sh.nroot = 0;
    __syncthreads();
    {
      const int best_sum = static_cast<int>(sh.best >> pd.key_shift);
      const int lane = tid & 63;
      for (int j0 = r0; j0 < r1; j0 += kSearch3dThreads) {
        const int j = j0 + tid;
        const int ixx = j % pd.top_nx, iyy = (j / pd.top_nx) % pd.top_ny,
                  izz = j / (pd.top_nx * pd.top_ny);
        const int ox = -pd.wxy + ixx * step, oy = -pd.wxy + iyy * step, oz = -pd.wz + izz * step;
        const int sx = ox >> te, sy = oy >> te, sz = oz >> te;
        const bool valid =
            j < r1 && !(skip_empty &&
                        (sh.rmax[0] + sx < tb.ox || sh.rmin[0] + sx >= tb.ox + tb.nx ||
                         sh.rmax[1] + sy < tb.oy || sh.rmin[1] + sy >= tb.oy + tb.ny ||
                         sh.rmax[2] + sz < tb.oz || sh.rmin[2] + sz >= tb.oz + tb.nz));
        if (__ballot(valid) == 0) continue;  // wave-uniform
        int sum = 0;
        if (cells_ok) {
          // Each group of 64 cells sits in the wave's registers (one per
          // lane) and is broadcast with readlane: only the level value is
          // read per (root, cell).
          if (valid) root_lookups += ntc;
          const int qx = (valid ? sx : -(1 << 20)) - tb.ox - 1024, qy = sy - tb.oy - 1024,
                    qz = sz - tb.oz - 512;
          for (int cb = 0; cb < ntc; cb += 64) {
            const int myc = cb + lane < ntc ? sh.tcell[cb + lane] : 0;
            const int mycnt = cb + lane < ntc ? sh.tcount[cb + lane] : 0;
            const int cn = min(64, ntc - cb);
            if (lds_top) {
              for (int c = 0; c < cn; ++c) {
                const int pc = __builtin_amdgcn_readlane(myc, c);
                const int cnt = __builtin_amdgcn_readlane(mycnt, c);
                const int x = (pc & 2047) + qx, y = ((pc >> 11) & 2047) + qy,
                          z = static_cast<int>(static_cast<unsigned>(pc) >> 22) + qz;
                const bool in = static_cast<unsigned>(x) < static_cast<unsigned>(tb.nx) &&
                                static_cast<unsigned>(y) < static_cast<unsigned>(tb.ny) &&
                                static_cast<unsigned>(z) < static_cast<unsigned>(tb.nz);
                const int v = sh.top[in ? (z * tb.ny + y) * tb.nx + x : 0];
                sum += in ? cnt * v : 0;
              }
            } else {
              for (int c = 0; c < cn; ++c) {
                const int pc = __builtin_amdgcn_readlane(myc, c);
                const int cnt = __builtin_amdgcn_readlane(mycnt, c);
                const int x = (pc & 2047) + qx, y = ((pc >> 11) & 2047) + qy,
                          z = static_cast<int>(static_cast<unsigned>(pc) >> 22) + qz;
                if (static_cast<unsigned>(x) < static_cast<unsigned>(tb.nx) &&
                    static_cast<unsigned>(y) < static_cast<unsigned>(tb.ny) &&
                    static_cast<unsigned>(z) < static_cast<unsigned>(tb.nz))
                  sum += cnt * tglobal[(z * tb.ny + y) * tb.nx + x];
              }
            }
          }
        } else if (valid) {
          root_lookups += n;
          for (int i = 0; i < n; ++i) {
            int x = sh.cloud.c.x[i], y = sh.cloud.c.y[i], z = sh.cloud.c.z[i];
            if (treduced) {
              x = ((x - pd.wxy) >> te) - lwx;
              y = ((y - pd.wxy) >> te) - lwy;
              z = ((z - pd.wz) >> te) - lwz;
            }
            int64_t idx;
            if (InBrick(tb, x + sx, y + sy, z + sz, &idx)) sum += lds_top ? sh.top[idx] : tglobal[idx];
          }
        }
        if (valid && sum >= pd.min_sum && sum >= best_sum) {
          const int at = atomicAdd(&sh.nroot, 1);
          sh.rbx[at] = static_cast<int16_t>(ox);
          sh.rby[at] = static_cast<int16_t>(oy);
          sh.rbz[at] = static_cast<int16_t>(oz);
          sh.rbs[at] = sum;
        }
      }

    }
    __syncthreads();
    F3_MARK(1);
    F3_COUNT(11, sh.nroot);
    // Order the roots ascending by bound (the best is fed last, popped
    // first): parallel rank sort into the (empty) stack arrays.
    {
      const int m = sh.nroot;
      for (int a = tid; a < m; a += kSearch3dThreads) {
        const int s0 = sh.rbs[a];
        int rank = 0;
        for (int b2 = 0; b2 < m; ++b2) {
          const int s1 = sh.rbs[b2];
          rank += (s1 < s0) || (s1 == s0 && b2 < a);
        }
        sh.sx[rank] = sh.rbx[a];
        sh.sy[rank] = sh.rby[a];
        sh.sz[rank] = sh.rbz[a];
        sh.ssum[rank] = s0;
      }
      __syncthreads();
      for (int a = tid; a < m; a += kSearch3dThreads) {
        sh.rbx[a] = sh.sx[a];
        sh.rby[a] = sh.sy[a];
        sh.rbz[a] = sh.sz[a];
        sh.rbs[a] = sh.ssum[a];
      }
    }
    __syncthreads();
    F3_MARK(2);
    for (int rb_end = sh.nroot; rb_end > 0;) {
      const int k0 = max(0, rb_end - kRootChunk3d);
      for (int a = tid; a < rb_end - k0; a += kSearch3dThreads) {
        sh.sx[a] = sh.rbx[k0 + a];
        sh.sy[a] = sh.rby[k0 + a];
        sh.sz[a] = sh.rbz[k0 + a];
        sh.sd[a] = static_cast<int8_t>(top);
        sh.ssum[a] = sh.rbs[k0 + a];
      }
      if (tid == 0) sh.sp = rb_end - k0;
      __syncthreads();
    // Best-first DFS in batches of up to kBatch nodes, kLanes lanes each:
    // the lanes of a node split the points and score its (up to) 8 children,
    // reduced with shuffles only.
    for (;;) {
      // Pop up to kBatch nodes, skipping pruned ones, 64 entries per step
      // across wave 0 (the same nodes, in the same order, as popping one by
      // one from the top).
      if (tid < 64) {
        const unsigned long long bk = max(sh.best, sh.best_seen);
        const int best_sum = static_cast<int>(bk >> pd.key_shift);
        // Once this workgroup has seen two passing leaves at a sum (the leaf
        // loop below sets sh.tie_sum), only a larger sum can change the
        // maximum: nodes bounded by it are pruned (tie resolution searches
        // those leaves again, ResolveTies3d). The collect pass instead
        // abandons a pair whose record overflowed (the host then walks it,
        // fast3d_walk).
        const int tie_sum = sh.tie_sum;
        const bool abandon =
            pd.collect && *reinterpret_cast<volatile int32_t*>(tie_count + pd.collect - 1) > kTieCap3d;
        int sp = abandon ? 0 : sh.sp, m = 0;
        while (sp > 0 && m < kBatch) {
          const int at = sp - 1 - tid;
          int s = 0;
          bool keep = false;
          int4 e = make_int4(0, 0, 0, 0);
          if (at >= 0) {
            e = at < kStack ? make_int4(sh.sx[at], sh.sy[at], (sh.sz[at] & 0xffff) | (sh.sd[at] << 16), sh.ssum[at])
                            : spill[at - kStack];
            s = e.w;
            keep = s >= best_sum && s >= pd.min_sum && s > tie_sum;
          }
          const unsigned long long mask = __ballot(keep);
          const int rank = m + __popcll(mask & ((1ull << tid) - 1ull));
          if (keep && rank < kBatch) {
            sh.bn_x[rank] = e.x;
            sh.bn_y[rank] = e.y;
            sh.bn_z[rank] = static_cast<int16_t>(e.z & 0xffff);
            sh.bn_d[rank] = e.z >> 16;
          }
          const unsigned long long last = __ballot(keep && rank == kBatch - 1);
          const int consumed = last ? __ffsll(static_cast<long long>(last)) : min(64, sp);
          m = min(kBatch, m + __popcll(mask));
          sp -= consumed;
        }
        if (tid == 0) {
          sh.best = bk;
          sh.sp = sp;
          sh.nbatch = m;
          sh.nleaf = 0;
          if (abandon) sh.abandon = 1;
        }
      }
      __syncthreads();
      const int nb = sh.nbatch;
      if (nb == 0) break;
      constexpr int kLanes = kSearch3dThreads / kBatch;  // lanes per node
      const int half = tid / kLanes, hl = tid % kLanes;
      int nc = 0, cd = 0, ox = 0, oy = 0, oz = 0, hw = 0;
      int acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      // Other yaws' progress on this pair, read while the batch scores and
      // folded in at the next pop.
      unsigned long long gbest = 0;
      if (tid == 0) gbest = *reinterpret_cast<volatile unsigned long long*>(best + yw.pair);
      if (half < nb) {
        const int d = sh.bn_d[half];
        ox = sh.bn_x[half];
        oy = sh.bn_y[half];
        oz = sh.bn_z[half];
        hw = 1 << (d - 1);
        // Children by octant k = z << 2 | y << 1 | x. Octant 0 sits at the
        // node's own offset (inside the window); the others are present unless
        // past it (the reference's breaks, :412-430).
        nc = (ox + hw <= pd.wxy ? 0xFF : 0x55) & (oy + hw <= pd.wxy ? 0xFF : 0x33) &
             (oz + hw <= pd.wz ? 0xFF : 0x0F);
        cd = d - 1;
        const int e = max(0, cd - sm.full_resolution_depth + 1);
        const bool reduced = cd >= sm.full_resolution_depth;
        const int lx = (-pd.wxy) >> e, ly = (-pd.wxy) >> e, lz = (-pd.wz) >> e;
        const Brick3 ob = sm.oct[cd];
        // Base child (octant 0) offset relative to the octet box origin.
        const int bx = (ox >> e) - ob.ox, by = (oy >> e) - ob.oy, bz = (oz >> e) - ob.oz;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(sm.octs), 0, sm.octs_bytes, 0x00020000);
        const int onx = ob.nx, ony = ob.ny, onz = ob.nz, ooff = static_cast<int>(ob.offset);
        constexpr int kOOB3 = 0x7ffffff0;
        auto load = [&](int i) -> uint64_t {
          const bool live = i < n;
          i = live ? i : 0;
          int a = sh.cloud.c.x[i], bb = sh.cloud.c.y[i], c = sh.cloud.c.z[i];
          if (reduced) {
            a = ((a - pd.wxy) >> e) - lx;
            bb = ((bb - pd.wxy) >> e) - ly;
            c = ((c - pd.wz) >> e) - lz;
          }
          a += bx;
          bb += by;
          c += bz;
          const bool in = live && static_cast<unsigned>(a) < static_cast<unsigned>(onx) &&
                          static_cast<unsigned>(bb) < static_cast<unsigned>(ony) &&
                          static_cast<unsigned>(c) < static_cast<unsigned>(onz);
          const int off = in ? ooff + ((c * ony + bb) * onx + a) * 8 : kOOB3;
          const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
          const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4, 0, 0);
          return (static_cast<uint64_t>(hi) << 32) | lo;
        };
        uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
        auto accumulate = [&](uint64_t v) {
          const uint32_t lo = static_cast<uint32_t>(v), hi = static_cast<uint32_t>(v >> 32);
          a0 = __builtin_amdgcn_udot4(lo, 0x00000001u, a0, false);
          a1 = __builtin_amdgcn_udot4(lo, 0x00000100u, a1, false);
          a2 = __builtin_amdgcn_udot4(lo, 0x00010000u, a2, false);
          a3 = __builtin_amdgcn_udot4(lo, 0x01000000u, a3, false);
          a4 = __builtin_amdgcn_udot4(hi, 0x00000001u, a4, false);
          a5 = __builtin_amdgcn_udot4(hi, 0x00000100u, a5, false);
          a6 = __builtin_amdgcn_udot4(hi, 0x00010000u, a6, false);
          a7 = __builtin_amdgcn_udot4(hi, 0x01000000u, a7, false);
        };
        // A lane's points in flight at once, kInflight per round. A load past
        // the cloud still costs texture-path cycles (it reads the out-of-range
        // offset and adds 0), so the last round is cut to the 4, 8, 12 or 16
        // loads that cover the cloud's nu = ceil(n / 16) points per lane
        // (wave-uniform: every node of the item has the same cloud): a
        // 186-point cloud issues 12 loads per lane, not 16.
        const int nu = (n + kLanes - 1) / kLanes;
        auto rounds = [&](auto&& ld) {
          int u0 = 0;
          auto issue = [&](auto kk) {
            constexpr int K = decltype(kk)::value;
            uint64_t v[K];
#pragma unroll
            for (int u = 0; u < K; ++u) v[u] = ld(hl + (u0 + u) * kLanes);
#pragma unroll
            for (int u = 0; u < K; ++u) accumulate(v[u]);
            u0 += K;
          };
          while (nu - u0 >= kInflight) issue(std::integral_constant<int, kInflight>{});
          const int left = nu - u0;  // < kInflight
          if (kInflight > 12 && left > 12)
            issue(std::integral_constant<int, (kInflight > 12 ? 16 : 4)>{});
          else if (kInflight > 8 && left > 8)
            issue(std::integral_constant<int, (kInflight > 8 ? 12 : 4)>{});
          else if (kInflight > 4 && left > 4)
            issue(std::integral_constant<int, (kInflight > 4 ? 8 : 4)>{});
          else if (left > 0)
            issue(std::integral_constant<int, 4>{});
        };
        if (packed) {
          // c - o of a point as bitfields; at this level, with e <= E,
          // a = ((c - o) >> e) + Kx etc. (the window and box origin folded in).
          const int kx = (reduced ? ((sh.org[0] - pd.wxy) >> e) - lx : sh.org[0]) + bx;
          const int ky = (reduced ? ((sh.org[1] - pd.wxy) >> e) - ly : sh.org[1]) + by;
          const int kz = (reduced ? ((sh.org[2] - pd.wz) >> e) - lz : sh.org[2]) + bz;
          const unsigned wxy = 11 - e, wzz = 10 - e;  // e <= E <= 9
          // Wave-uniform: every node of the wave has the whole cloud box inside
          // its octet brick, so no point needs a bounds check.
          const bool inside = (sh.rel_min[0] >> e) + kx >= 0 && (sh.rel_max[0] >> e) + kx < onx &&
                              (sh.rel_min[1] >> e) + ky >= 0 && (sh.rel_max[1] >> e) + ky < ony &&
                              (sh.rel_min[2] >> e) + kz >= 0 && (sh.rel_max[2] >> e) + kz < onz;
          if (__ballot(!inside) == 0) {
            const unsigned sy = static_cast<unsigned>(onx) * 8u, sz = static_cast<unsigned>(ony) * sy;
            const int kall = static_cast<int>(
                static_cast<unsigned>(ooff) +
                ((static_cast<unsigned>(kz) * ony + static_cast<unsigned>(ky)) * onx +
                 static_cast<unsigned>(kx)) * 8u);
            auto load_in = [&](int i) -> uint64_t {
              const bool live = i < n;
              const uint32_t w = sh.cloud.pk[live ? i : 0];
              const unsigned rx = __builtin_amdgcn_ubfe(w, e, wxy);
              const unsigned ry = __builtin_amdgcn_ubfe(w, 11 + e, wxy);
              const unsigned rz = __builtin_amdgcn_ubfe(w, 22 + e, wzz);
              const int off = live ? static_cast<int>(__umul24(rz, sz) + __umul24(ry, sy) + (rx << 3) +
                                                      static_cast<unsigned>(kall))
                                   : kOOB3;
              const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
              const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4, 0, 0);
              return (static_cast<uint64_t>(hi) << 32) | lo;
            };
            rounds(load_in);
          } else {
            auto load_chk = [&](int i) -> uint64_t {
              const bool live = i < n;
              const uint32_t w = sh.cloud.pk[live ? i : 0];
              const int a = static_cast<int>(__builtin_amdgcn_ubfe(w, e, wxy)) + kx;
              const int bb = static_cast<int>(__builtin_amdgcn_ubfe(w, 11 + e, wxy)) + ky;
              const int c = static_cast<int>(__builtin_amdgcn_ubfe(w, 22 + e, wzz)) + kz;
              const bool in = live && static_cast<unsigned>(a) < static_cast<unsigned>(onx) &&
                              static_cast<unsigned>(bb) < static_cast<unsigned>(ony) &&
                              static_cast<unsigned>(c) < static_cast<unsigned>(onz);
              const int off = in ? ooff + ((c * ony + bb) * onx + a) * 8 : kOOB3;
              const uint32_t lo = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
              const uint32_t hi = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4, 0, 0);
              return (static_cast<uint64_t>(hi) << 32) | lo;
            };
            rounds(load_chk);
          }
        } else {
          rounds(load);
        }
        acc[0] = a0;
        acc[1] = a1;
        acc[2] = a2;
        acc[3] = a3;
        acc[4] = a4;
        acc[5] = a5;
        acc[6] = a6;
        acc[7] = a7;
      }
      // Node (8- or 16-lane) sums with DPP: xor 1, xor 2 (quad_perm), then the
      // half-row mirror (8 lanes) and the row mirror (16); every lane of the
      // node ends with the sum.
      // Lane k < 8 of a node ranks and pushes child k below: 8 lanes at least.
      static_assert(kLanes == 16 || kLanes == 8, "DPP reduction over 8 or 16 lanes per node");
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        int v = acc[k];
        v += __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
        v += __builtin_amdgcn_update_dpp(0, v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
        v += __builtin_amdgcn_update_dpp(0, v, 0x141, 0xF, 0xF, false);  // row_half_mirror
        if (kLanes == 16) v += __builtin_amdgcn_update_dpp(0, v, 0x140, 0xF, 0xF, false);  // row_mirror
        acc[k] = v;
      }
      // Lane k < 8 of a node handles child k: its sum, then its rank among
      // the kept children (ascending bound, stable; the best is popped first).
      if (half < nb && hl < 8) {
        const int k = hl;
        if (k == 0) lookups += static_cast<unsigned long long>(__popc(nc)) * n;
        const int best_sum = static_cast<int>(sh.best >> pd.key_shift);
        const int tie_sum = sh.tie_sum;
        int my = acc[0];
#pragma unroll
        for (int j = 1; j < 8; ++j) my = k == j ? acc[j] : my;
        const int cxk = ox + ((k & 1) ? hw : 0), cyk = oy + ((k & 2) ? hw : 0),
                  czk = oz + ((k & 4) ? hw : 0);
        const bool pres = (nc >> k) & 1;
        if (cd > 0) {
          int m = 0, rank = 0;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const bool kj = ((nc >> j) & 1) && acc[j] >= pd.min_sum && acc[j] >= best_sum && acc[j] > tie_sum;
            m += kj;
            rank += kj && (acc[j] < my || (acc[j] == my && j < k));
          }
          int base = 0;
          if (k == 0 && m > 0) {
            base = atomicAdd(&sh.sp, m);
            atomicMax(&sh.high_water, base + m);
            if (base + m > kDfsCap3d) sh.error = 1;  // flagged after the batch
          }
          base = __shfl(base, (tid & 63) & ~(kLanes - 1), 64);
          const int at = base + rank;
          if (pres && my >= pd.min_sum && my >= best_sum && my > tie_sum && at < kDfsCap3d) {
            if (at < kStack) {
              sh.sx[at] = static_cast<int16_t>(cxk);
              sh.sy[at] = static_cast<int16_t>(cyk);
              sh.sz[at] = static_cast<int16_t>(czk);
              sh.sd[at] = static_cast<int8_t>(cd);
              sh.ssum[at] = my;
            } else {
              spill[at - kStack] = make_int4(cxk, cyk, (czk & 0xffff) | (cd << 16), my);
            }
          }
        } else if (pres && my >= pd.min_sum) {
          const unsigned long long id = LeafId(pd, yw.yaw_id, cxk, cyk, czk);
          const unsigned long long key = (static_cast<unsigned long long>(my) << pd.key_shift) |
                                         (~id & ((1ull << pd.key_shift) - 1));
          // Leaves at the best sum too (not only above the best key): a
          // second leaf at the maximum is the tie witness.
          if (my >= best_sum && my > tie_sum) {
            const int at = atomicAdd(&sh.nleaf, 1);
            sh.leaf_keys[at] = key;
            sh.leaf_x[at] = cxk;
            sh.leaf_y[at] = cyk;
            sh.leaf_z[at] = czk;
          }
        }
      }
      if (tid == 0) sh.best_seen = gbest;
      F3_COUNT(5, 1);
      __syncthreads();
      if (sh.error) {  // stack beyond LDS + spill: the pair's result is void
        if (tid == 0) atomicExch(reinterpret_cast<int*>(status + yw.pair), -4);
        break;
      }
      const int nl = sh.nleaf;
      if (nl == 0) continue;
      // Leaves: descending key order; the first that passes the
      // low-resolution check (:384-401) beats every later one. Leaves at the
      // best sum that do not beat its key are still checked (witness path):
      // one that passes is a second leaf at the maximum, recorded in best_hi
      // (sum << shift | leaf id, the largest id) so the host can tell an
      // exact tie (host3d.cc ResolveTies3d); once best_hi shows a tie at the
      // current best sum, further witnesses are skipped unless collecting.
      if (tid == 0) {
        for (int a = 1; a < nl; ++a) {
          const unsigned long long kk = sh.leaf_keys[a];
          const int x = sh.leaf_x[a], y = sh.leaf_y[a], z = sh.leaf_z[a];
          int b2 = a - 1;
          while (b2 >= 0 && sh.leaf_keys[b2] < kk) {
            sh.leaf_keys[b2 + 1] = sh.leaf_keys[b2];
            sh.leaf_x[b2 + 1] = sh.leaf_x[b2];
            sh.leaf_y[b2 + 1] = sh.leaf_y[b2];
            sh.leaf_z[b2 + 1] = sh.leaf_z[b2];
            --b2;
          }
          sh.leaf_keys[b2 + 1] = kk;
          sh.leaf_x[b2 + 1] = x;
          sh.leaf_y[b2 + 1] = y;
          sh.leaf_z[b2 + 1] = z;
        }
        sh.best = max(sh.best, *reinterpret_cast<volatile unsigned long long*>(best + yw.pair));
      }
      __syncthreads();
      const unsigned long long id_mask = (1ull << pd.key_shift) - 1;
      for (int a = 0; a < nl; ++a) {
        const unsigned long long lkey = sh.leaf_keys[a], cur = sh.best;  // uniform: shared
        const int lsum = static_cast<int>(lkey >> pd.key_shift);
        if (lsum < static_cast<int>(cur >> pd.key_shift)) break;
        const bool witness = lkey <= cur;
        if (witness && !pd.collect) {
          if (tid == 0) {
            const unsigned long long hi =
                *reinterpret_cast<volatile unsigned long long*>(best_hi + yw.pair);
            sh.skip = static_cast<int>(hi >> pd.key_shift) == lsum &&
                      (hi & id_mask) != (~cur & id_mask);
            if (sh.skip) sh.tie_sum = max(sh.tie_sum, lsum);  // the witness shows the tie
          }
          __syncthreads();
          // Every wave takes its copy before thread 0 may rewrite the flag
          // for the next leaf.
          const int skip = sh.skip;
          __syncthreads();
          if (skip) continue;
        }
        const float rf = res;
        const float tx = __fadd_rn(yw.tx, __fmul_rn(rf, static_cast<float>(sh.leaf_x[a])));
        const float ty = __fadd_rn(yw.ty, __fmul_rn(rf, static_cast<float>(sh.leaf_y[a])));
        const float tz = __fadd_rn(yw.tz, __fmul_rn(rf, static_cast<float>(sh.leaf_z[a])));
        const float lrs = LowResScore(sh, sm, low_points + 3 * pd.low_offset, pd.num_low, yw.nw,
                                      yw.nx, yw.ny, yw.nz, tx, ty, tz);
        if (tid == 0 && static_cast<double>(lrs) >= static_cast<double>(pd.min_low_resolution_score)) {
          const unsigned long long lid = ~lkey & id_mask;
          if (!witness) {
            atomicMax(best + yw.pair, lkey);
            sh.best = max(sh.best, lkey);
          } else if (!pd.collect && lkey != cur) {
            sh.tie_sum = max(sh.tie_sum, lsum);  // a second passing leaf at the best sum
          }
          atomicMax(best_hi + yw.pair, (static_cast<unsigned long long>(lsum) << pd.key_shift) | lid);
          if (pd.collect && lsum == pd.collect_sum) {  // collect = tie slot + 1
            const int slot = pd.collect - 1;
            const int at = atomicAdd(tie_count + slot, 1);
            if (at < kTieCap3d)
              ties[static_cast<int64_t>(slot) * kTieCap3d + at] =
                  make_uint4(static_cast<unsigned>(yw.yaw_id), static_cast<unsigned>(sh.leaf_x[a]),
                             static_cast<unsigned>(sh.leaf_y[a]), static_cast<unsigned>(sh.leaf_z[a]));
          }
        }
        __syncthreads();
      }
      __syncthreads();
      F3_COUNT(6, nl);
    }
      rb_end = sh.abandon ? 0 : k0;
    }
    F3_MARK(3);
    }  // root chunks
  }
  lookups += root_lookups;
  for (int m = 32; m > 0; m >>= 1) lookups += __shfl_xor(lookups, m, 64);
  if ((tid & 63) == 0 && stats && lookups) atomicAdd(stats, lookups);
  if (tid == 0 && stats) atomicMax(stats + kStat3dHighWater, static_cast<unsigned long long>(sh.high_water));
  F3_FLUSH(stats);
}

// The reference's ScoreCandidates sum (:332-352) for tie resolution
// (host3d.cc ResolveTies3d): per job, one yaw item's cloud discretized as the
// search does (DiscretizeScan :201-244), then for each (depth, x, y, z) query
// the sum over points of level `depth` at the point's cell at that depth plus
// the offset >> the depth's reduction exponent; cells outside the level's
// brick read 0 (PrecomputationGrid3D::value of an unknown cell).
__global__ void __launch_bounds__(kSearch3dThreads)
fast3d_score_queries(const Submap3Desc* __restrict__ submaps, const Pair3Desc* __restrict__ pairs,
                     const Yaw3Desc* __restrict__ yaws, const float* __restrict__ points,
                     const Score3Job* __restrict__ jobs, const int4* __restrict__ queries,
                     int32_t* __restrict__ sums) {
  __shared__ int16_t cx[kMax3dPoints], cy[kMax3dPoints], cz[kMax3dPoints];
  __shared__ int part[kSearch3dThreads / 64];
  const int tid = threadIdx.x;
  const Score3Job job = jobs[blockIdx.x];
  const Yaw3Desc yw = yaws[job.item];
  const Pair3Desc pd = pairs[yw.pair];
  const Submap3Desc& sm = submaps[pd.submap];
  const int n = min(pd.num_points, kMax3dPoints);
  const float res = sm.resolution, inv = 1.f / sm.resolution;
  for (int i = tid; i < n; i += kSearch3dThreads) {
    const float* p = points + 3 * (pd.point_offset + i);
    float ox, oy, oz;
    Rotate3(yw.qw, yw.qx, yw.qy, yw.qz, p[0], p[1], p[2], &ox, &oy, &oz);
    cx[i] = static_cast<int16_t>(RoundDiv(__fadd_rn(ox, yw.tx), res, inv));
    cy[i] = static_cast<int16_t>(RoundDiv(__fadd_rn(oy, yw.ty), res, inv));
    cz[i] = static_cast<int16_t>(RoundDiv(__fadd_rn(oz, yw.tz), res, inv));
  }
  __syncthreads();
  for (int q = 0; q < job.count; ++q) {
    const int4 qq = queries[job.first + q];
    const int d = qq.x;
    const int e = max(0, d - sm.full_resolution_depth + 1);
    const bool reduced = d >= sm.full_resolution_depth;
    const int lx = (-pd.wxy) >> e, ly = (-pd.wxy) >> e, lz = (-pd.wz) >> e;
    const Brick3 b = sm.level[d];
    const uint8_t* lv = sm.levels + b.offset;
    int sum = 0;
    for (int i = tid; i < n; i += kSearch3dThreads) {
      int x = cx[i], y = cy[i], z = cz[i];
      if (reduced) {
        x = ((x - pd.wxy) >> e) - lx;
        y = ((y - pd.wxy) >> e) - ly;
        z = ((z - pd.wz) >> e) - lz;
      }
      int64_t idx;
      if (InBrick(b, x + (qq.y >> e), y + (qq.z >> e), z + (qq.w >> e), &idx)) sum += lv[idx];
    }
    for (int m = 32; m > 0; m >>= 1) sum += __shfl_xor(sum, m, 64);
    if ((tid & 63) == 0) part[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int w = 0; w < kSearch3dThreads / 64; ++w) t += part[w];
      sums[job.first + q] = t;
    }
    __syncthreads();
  }
}

// PrecomputationGrid3D::ToProbability(sum / n) (precomputation_grid_3d.h:32-35)
// with the host's float operations (host3d.cc SumToProbability).
__device__ __forceinline__ float SumToProbabilityDev(int sum, int n) {
  const float kMinP = 0.1f, kMaxP = 1.f - kMinP;
  return __fadd_rn(kMinP, __fmul_rn(__fdiv_rn(static_cast<float>(sum), static_cast<float>(n)),
                                    __fdiv_rn(__fsub_rn(kMaxP, kMinP), 255.f)));
}

struct Walk3Shared {
  int16_t cx[kMax3dPoints], cy[kMax3dPoints], cz[kMax3dPoints];
  int4 stk[kWalkStack3d];  // (depth, x, y, z)
  int sp;
  int csum[8];
  int4 res;                // (yaw, x, y, z) of the pick
  int found, pass;
  float lr[kSearch3dThreads];  // LowResScore's staging
};

// Ordered walk to the reference's pick among exactly tied maxima, for pairs
// whose passing tied leaves overflow the collect pass (host3d.cc
// ResolveTies3d). BranchAndBound (fast_correlative_scan_matcher_3d.cc:377-440)
// visits the sorted lowest-resolution list in order, each node's <= 8
// children (z, then y, then x, x fastest; a child past the window ends its
// loop, :412-430) by descending score with equal scores in generation order
// (insertion sort), and at depth 0 returns the first child that passes the
// low-resolution check (:384-401). Until the first passing leaf at the
// maximum is reached the incumbent is below the maximum, so every node whose
// sum reaches it is visited; a passing leaf above the maximum does not exist.
// One workgroup per job walks that order depth-first over nodes whose exact
// sum is >= target (wave w scores children w and w + 4) and stops at the
// first child, in order, that reaches the target and passes.
__global__ void __launch_bounds__(kSearch3dThreads)
fast3d_walk(const Submap3Desc* __restrict__ submaps, const Pair3Desc* __restrict__ pairs,
            const Yaw3Desc* __restrict__ yaws, const float* __restrict__ points,
            const float* __restrict__ low_points, const Walk3Job* __restrict__ jobs,
            const int4* __restrict__ top, int4* __restrict__ out) {
  // out[2 j] = (yaw, x, y, z) of job j's pick, out[2 j + 1].x = found.
  __shared__ Walk3Shared sh;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const Walk3Job job = jobs[blockIdx.x];
  const Pair3Desc pd = pairs[job.pair];
  const Submap3Desc& sm = submaps[pd.submap];
  const int n = min(pd.num_points, kMax3dPoints);
  const int target = job.target_sum;
  const float res = sm.resolution, inv = 1.f / sm.resolution;
  if (tid == 0) {
    sh.res = make_int4(0, 0, 0, 0);
    sh.found = 0;
    sh.pass = 0;
  }
  int cur_yaw = -1;
  Yaw3Desc yw{};
  // Low-resolution check of leaf (x, y, z) of the current yaw (uniform).
  auto passes = [&](int x, int y, int z) {
    const float tx = __fadd_rn(yw.tx, __fmul_rn(res, static_cast<float>(x)));
    const float ty = __fadd_rn(yw.ty, __fmul_rn(res, static_cast<float>(y)));
    const float tz = __fadd_rn(yw.tz, __fmul_rn(res, static_cast<float>(z)));
    const float lrs = LowResScore(sh, sm, low_points + 3 * pd.low_offset, pd.num_low, yw.nw, yw.nx,
                                  yw.ny, yw.nz, tx, ty, tz);
    if (tid == 0)
      sh.pass = static_cast<double>(lrs) >= static_cast<double>(pd.min_low_resolution_score);
    __syncthreads();
    const int p = sh.pass;
    __syncthreads();
    return p != 0;
  };
  __syncthreads();
  for (int ti = 0; ti < job.top_count && !sh.found; ++ti) {
    const int4 te = top[job.top_first + ti];  // (yaw, x | y << 16, z, sum), uniform
    const int tx0 = static_cast<int16_t>(te.y & 0xffff), ty0 = te.y >> 16;
    if (te.x != cur_yaw) {
      __syncthreads();  // the previous yaw's readers are done
      cur_yaw = te.x;
      yw = yaws[pd.yaw_begin + cur_yaw];
      for (int i = tid; i < n; i += kSearch3dThreads) {  // DiscretizeScan (:201-244)
        const float* p = points + 3 * (pd.point_offset + i);
        float ox, oy, oz;
        Rotate3(yw.qw, yw.qx, yw.qy, yw.qz, p[0], p[1], p[2], &ox, &oy, &oz);
        sh.cx[i] = static_cast<int16_t>(RoundDiv(__fadd_rn(ox, yw.tx), res, inv));
        sh.cy[i] = static_cast<int16_t>(RoundDiv(__fadd_rn(oy, yw.ty), res, inv));
        sh.cz[i] = static_cast<int16_t>(RoundDiv(__fadd_rn(oz, yw.tz), res, inv));
      }
      __syncthreads();
    }
    if (job.top_level == 0) {  // the list holds the leaves (depth-0 loop, :384-401)
      const bool hit = te.w >= target && passes(tx0, ty0, te.z);
      if (hit && tid == 0) {
        sh.res = make_int4(te.x, tx0, ty0, te.z);
        sh.found = 1;
      }
      __syncthreads();
      continue;
    }
    __syncthreads();  // every wave has read the previous walk's empty stack
    if (tid == 0) {
      sh.stk[0] = make_int4(job.top_level, tx0, ty0, te.z);
      sh.sp = 1;
    }
    for (;;) {
      __syncthreads();
      const int s = sh.sp;
      if (s == 0 || sh.found) break;
      const int4 nd = sh.stk[s - 1];
      const int d = nd.x, hw = 1 << (d - 1);
      // Children in generation order (:412-430).
      int cxs[8], cys[8], czs[8], nc = 0;
      for (int a = 0; a < 2; ++a) {
        const int zo = nd.w + a * hw;
        if (zo > pd.wz) break;
        for (int b = 0; b < 2; ++b) {
          const int yo = nd.z + b * hw;
          if (yo > pd.wxy) break;
          for (int c = 0; c < 2; ++c) {
            const int xo = nd.y + c * hw;
            if (xo > pd.wxy) break;
            cxs[nc] = xo;
            cys[nc] = yo;
            czs[nc] = zo;
            ++nc;
          }
        }
      }
      // ScoreCandidates at depth d - 1 (:332-352), as fast3d_score_queries.
      const int cd = d - 1;
      const int e = max(0, cd - sm.full_resolution_depth + 1);
      const bool reduced = cd >= sm.full_resolution_depth;
      const int lx = (-pd.wxy) >> e, ly = (-pd.wxy) >> e, lz = (-pd.wz) >> e;
      const Brick3 bk = sm.level[cd];
      const uint8_t* lv = sm.levels + bk.offset;
      for (int c = wave; c < nc; c += kSearch3dThreads / 64) {
        int qx = 0, qy = 0, qz = 0;
        for (int k = 0; k < 8; ++k)
          if (k == c) { qx = cxs[k]; qy = cys[k]; qz = czs[k]; }
        int sum = 0;
        for (int i = lane; i < n; i += 64) {
          int x = sh.cx[i], y = sh.cy[i], z = sh.cz[i];
          if (reduced) {
            x = ((x - pd.wxy) >> e) - lx;
            y = ((y - pd.wxy) >> e) - ly;
            z = ((z - pd.wz) >> e) - lz;
          }
          int64_t idx;
          if (InBrick(bk, x + (qx >> e), y + (qy >> e), z + (qz >> e), &idx)) sum += lv[idx];
        }
        for (int m = 32; m > 0; m >>= 1) sum += __shfl_xor(sum, m, 64);
        if (lane == 0) sh.csum[c] = sum;
      }
      __syncthreads();
      // Stable descending order by score (insertion sort, every thread alike).
      int ord[8];
      float sc[8];
      for (int c = 0; c < nc; ++c) {
        ord[c] = c;
        sc[c] = SumToProbabilityDev(sh.csum[c], pd.num_points);
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
      if (cd == 0) {
        // Depth 0: the first child, in order, at or above the target that
        // passes (none above it passes: the target is the passing maximum).
        int hit = -1;
        for (int i = 0; i < nc && hit < 0; ++i) {
          const int c = ord[i];
          if (sh.csum[c] < target) break;
          int x = 0, y = 0, z = 0;
          for (int k = 0; k < 8; ++k)
            if (k == c) { x = cxs[k]; y = cys[k]; z = czs[k]; }
          if (passes(x, y, z)) hit = c;
        }
        if (tid == 0) {
          if (hit >= 0) {
            int x = 0, y = 0, z = 0;
            for (int k = 0; k < 8; ++k)
              if (k == hit) { x = cxs[k]; y = cys[k]; z = czs[k]; }
            sh.res = make_int4(cur_yaw, x, y, z);
            sh.found = 1;
          }
          sh.sp = s - 1;
        }
      } else if (tid == 0) {
        int top_sp = s - 1;
        for (int i = nc - 1; i >= 0; --i) {
          const int c = ord[i];
          if (sh.csum[c] >= target && top_sp < kWalkStack3d)
            sh.stk[top_sp++] = make_int4(cd, cxs[c], cys[c], czs[c]);
        }
        sh.sp = top_sp;
      }
    }
    __syncthreads();
  }
  __syncthreads();
  if (tid == 0) {
    out[2 * blockIdx.x] = sh.res;
    out[2 * blockIdx.x + 1] = make_int4(sh.found, 0, 0, 0);
  }
}

// Low-resolution score of each pair's winning leaf (the Result field), with
// the same arithmetic as the search: one workgroup per pair.
__global__ void __launch_bounds__(kSearch3dThreads)
fast3d_finalize(const Submap3Desc* __restrict__ submaps, const Pair3Desc* __restrict__ pairs,
                const Yaw3Desc* __restrict__ yaws, const float* __restrict__ low_points,
                const unsigned long long* __restrict__ best, float* __restrict__ low_score) {
  __shared__ F3SharedT<kSmall3dPoints, kStack3d, kBatch3d> sh;
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

// --------------------------------------------------- rotational scores ----
//
// RotationalScanMatcher::Match (rotational_scan_matcher.cc:173-185) for every
// (pair, yaw): RotateHistogram (:138-158) then MatchHistograms (:119-131), one
// thread per yaw, with the float operations of the reference's x86-64 build:
// Eigen's 4-wide packet order for dot() / norm() (Redux.h), correctly rounded
// sqrt and division. Note: sqrtf, not __fsqrt_rn — on this toolchain the latter
// is not correctly rounded for gfx950 (tools/check_fp.hip: 15% of inputs differ
// from IEEE), while sqrtf and '/' are.
struct RotPair3 {
  int32_t node_hist;    // float offset of the node histogram
  int32_t submap_hist;  // float offset of the submap histogram
  int32_t size;         // buckets
  int32_t window;       // angular window A: yaws k = 0..2A
  float step, yaw0;
  int64_t out;          // score offset
  double min_score;     // the submap's min_rotational_score
};

template <typename F>
__device__ __forceinline__ float PacketSum(F v, int n) {
  // Redux.h LinearVectorizedTraversal, aligned, 4-wide packets.
  const int a2 = (n / 8) * 8, a1 = (n / 4) * 4;
  if (a1 == 0) {
    if (n == 0) return 0.f;
    float r = v(0);
    for (int i = 1; i < n; ++i) r = __fadd_rn(r, v(i));
    return r;
  }
  float p0 = v(0), p1 = v(1), p2 = v(2), p3 = v(3);
  if (a1 > 4) {
    float q0 = v(4), q1 = v(5), q2 = v(6), q3 = v(7);
    for (int i = 8; i < a2; i += 8) {
      p0 = __fadd_rn(p0, v(i));
      p1 = __fadd_rn(p1, v(i + 1));
      p2 = __fadd_rn(p2, v(i + 2));
      p3 = __fadd_rn(p3, v(i + 3));
      q0 = __fadd_rn(q0, v(i + 4));
      q1 = __fadd_rn(q1, v(i + 5));
      q2 = __fadd_rn(q2, v(i + 6));
      q3 = __fadd_rn(q3, v(i + 7));
    }
    p0 = __fadd_rn(p0, q0);
    p1 = __fadd_rn(p1, q1);
    p2 = __fadd_rn(p2, q2);
    p3 = __fadd_rn(p3, q3);
    if (a1 > a2) {
      p0 = __fadd_rn(p0, v(a2));
      p1 = __fadd_rn(p1, v(a2 + 1));
      p2 = __fadd_rn(p2, v(a2 + 2));
      p3 = __fadd_rn(p3, v(a2 + 3));
    }
  }
  float r = __fadd_rn(__fadd_rn(p0, p2), __fadd_rn(p1, p3));
  for (int i = a1; i < n; ++i) r = __fadd_rn(r, v(i));
  return r;
}

// Two sums over the same terms in one pass, each in PacketSum's order.
template <typename F>
__device__ __forceinline__ float2 PacketSum2(F v, int n) {
  const int a2 = (n / 8) * 8, a1 = (n / 4) * 4;
  auto add = [](float2 a, float2 b) { return make_float2(__fadd_rn(a.x, b.x), __fadd_rn(a.y, b.y)); };
  if (a1 == 0) {
    if (n == 0) return make_float2(0.f, 0.f);
    float2 r = v(0);
    for (int i = 1; i < n; ++i) r = add(r, v(i));
    return r;
  }
  float2 p0 = v(0), p1 = v(1), p2 = v(2), p3 = v(3);
  if (a1 > 4) {
    float2 q0 = v(4), q1 = v(5), q2 = v(6), q3 = v(7);
    for (int i = 8; i < a2; i += 8) {
      p0 = add(p0, v(i));
      p1 = add(p1, v(i + 1));
      p2 = add(p2, v(i + 2));
      p3 = add(p3, v(i + 3));
      q0 = add(q0, v(i + 4));
      q1 = add(q1, v(i + 5));
      q2 = add(q2, v(i + 6));
      q3 = add(q3, v(i + 7));
    }
    p0 = add(p0, q0);
    p1 = add(p1, q1);
    p2 = add(p2, q2);
    p3 = add(p3, q3);
    if (a1 > a2) {
      p0 = add(p0, v(a2));
      p1 = add(p1, v(a2 + 1));
      p2 = add(p2, v(a2 + 2));
      p3 = add(p3, v(a2 + 3));
    }
  }
  float2 r = add(add(p0, p2), add(p1, p3));
  for (int i = a1; i < n; ++i) r = add(r, v(i));
  return r;
}

// One block per (pair, 64 yaws): both histograms staged in LDS, the submap
// norm computed once per block, the rotated bucket index wrapped by a
// compare instead of '%', and the scan norm and the dot product summed in
// one pass (each still in the packet order of its own Eigen reduction).
constexpr int kRotThreads = 64;

__global__ void __launch_bounds__(kRotThreads)
rot_scores(const RotPair3* __restrict__ pairs, int num_pairs, const float* __restrict__ hists,
           float* __restrict__ out) {
  __shared__ float hs[kMaxHistogram + 1], ss[kMaxHistogram];
  __shared__ float submap_norm_sh;
  const int p = blockIdx.y;
  if (p >= num_pairs) return;
  const RotPair3 rp = pairs[p];
  if (static_cast<int>(blockIdx.x) * kRotThreads > 2 * rp.window) return;
  const int n = rp.size;
  const int tid = threadIdx.x;
  for (int i = tid; i < n; i += kRotThreads) {
    hs[i] = hists[rp.node_hist + i];
    ss[i] = hists[rp.submap_hist + i];
  }
  if (tid == 0 && n > 0) hs[n] = hists[rp.node_hist];  // h[(n - 1 + 1 + full) mod n] at full = 0
  __syncthreads();
  if (tid == 0)
    submap_norm_sh = sqrtf(PacketSum([&](int i) { return __fmul_rn(ss[i], ss[i]); }, n));
  __syncthreads();
  const int k = blockIdx.x * kRotThreads + tid;
  if (k > 2 * rp.window) return;
  const float angle = __fadd_rn(rp.yaw0, __fmul_rn(static_cast<float>(k - rp.window), rp.step));
  int full = 0;
  float fraction = 0.f;
  if (n > 0) {
    const float rb = static_cast<float>(
        static_cast<double>(__fmul_rn(-angle, static_cast<float>(n))) / 3.14159265358979323846);
    full = static_cast<int>(roundf(__fsub_rn(rb, 0.5f)));
    fraction = __fsub_rn(rb, static_cast<float>(full));
    while (full < 0) full += n;
    full %= n;  // (i + full) mod n below is i + full, less n past the end
  }
  const float one_minus = __fsub_rn(1.f, fraction);
  // hs[n] repeats hs[0], so j + 1 needs no second wrap when j = n - 1.
  const float2 sums = PacketSum2([&](int i) {
    int j = i + full;
    j -= j >= n ? n : 0;
    const float r = __fadd_rn(__fmul_rn(fraction, hs[j + 1]), __fmul_rn(one_minus, hs[j]));
    return make_float2(__fmul_rn(r, r), __fmul_rn(ss[i], r));
  }, n);
  const float scan_norm = sqrtf(sums.x);
  const float normalization = __fmul_rn(scan_norm, submap_norm_sh);
  float score = 1.f;
  if (!(normalization < 1e-3f)) score = __fdiv_rn(sums.y, normalization);
  out[rp.out + k] = score;
}

// GenerateDiscreteScans :277-294 on the device for the passing yaws, with
// the float arithmetic of the host restatement (host3d.cc BuildYaws):
// angle = (k - A) * step, AngleAxisToQuat through double sin / cos of
// norm / 2 rounded to float, Eigen's SSE quaternion products, the normalized
// rotation of GetPoseFromCandidate. The device's double sin / cos may differ
// from libm's in the last ulps; a float rounding of them is kept only when
// the double value lies farther than 2^-40 relative from a float rounding
// boundary (both results are then on the same side), otherwise the yaw is
// flagged and the host rebuilds it.
__device__ __forceinline__ bool NearFloatBoundary(double v) {
  v = fabs(v);  // round-to-nearest-even is symmetric (cos < 0 past |angle| = pi)
  const float f = static_cast<float>(v);
  if (!(f >= 1.2e-38f) || !(f < 3.0e38f)) return true;  // zero, subnormal, huge: the host decides
  const double fd = static_cast<double>(f);
  const double up = static_cast<double>(__int_as_float(__float_as_int(f) + 1));
  const double dn = static_cast<double>(__int_as_float(__float_as_int(f) - 1));
  const double d = fmin(fabs(v - 0.5 * (fd + up)), fabs(v - 0.5 * (fd + dn)));
  return d <= fabs(v) * 0x1p-40;
}

__device__ __forceinline__ float4 QMulDev(float4 a, float4 b) {  // (w, x, y, z) in (x, y, z, w)
  // a.w*b.w - a.x*b.x - (a.z*b.z + a.y*b.y), ... : host3d.cc QMul term order.
  const float w = __fsub_rn(__fsub_rn(__fmul_rn(a.x, b.x), __fmul_rn(a.y, b.y)),
                            __fadd_rn(__fmul_rn(a.w, b.w), __fmul_rn(a.z, b.z)));
  const float x = __fadd_rn(__fsub_rn(__fmul_rn(a.y, b.x), __fmul_rn(a.w, b.z)),
                            __fadd_rn(__fmul_rn(a.z, b.w), __fmul_rn(a.x, b.y)));
  const float y = __fadd_rn(__fsub_rn(__fmul_rn(a.z, b.x), __fmul_rn(a.y, b.w)),
                            __fadd_rn(__fmul_rn(a.w, b.y), __fmul_rn(a.x, b.z)));
  const float z = __fadd_rn(__fsub_rn(__fmul_rn(a.w, b.x), __fmul_rn(a.z, b.y)),
                            __fadd_rn(__fmul_rn(a.y, b.z), __fmul_rn(a.x, b.w)));
  return make_float4(w, x, y, z);
}

__global__ void __launch_bounds__(64)
yaw_build(const YawBuild3* __restrict__ items, const int32_t* __restrict__ ks,
          const float* __restrict__ ss, Yaw3Desc* __restrict__ out, unsigned* __restrict__ flag_count,
          YawFlag3* __restrict__ flags) {
  const int dp = blockIdx.x;
  const YawBuild3 it = items[dp];
  // Quaternions held as float4 (x = w, y = x, z = y, w = z).
  const float4 si = make_float4(it.siw, it.six, it.siy, it.siz);
  const float4 nq = make_float4(it.nqw, it.nqx, it.nqy, it.nqz);
  for (int j = threadIdx.x; j < it.num; j += 64) {
    const int k = ks[it.src + j];
    const float score = ss[it.src + j];
    const float angle = __fmul_rn(static_cast<float>(k - it.window), it.astep);
    // AngleAxisToQuat(V3{0, 0, angle}).
    float scale = 0.5f, w = 1.f;
    const float sq = __fadd_rn(__fmul_rn(0.f, 0.f), __fadd_rn(__fmul_rn(0.f, 0.f), __fmul_rn(angle, angle)));
    bool flag = false;
    if (static_cast<double>(sq) > 1e-8) {
      const float norm = sqrtf(sq);
      const double h = static_cast<double>(norm) / 2.;
      const double sv = sin(h) / static_cast<double>(norm), cv = cos(h);
      flag = NearFloatBoundary(sv) || NearFloatBoundary(cv);
      scale = static_cast<float>(sv);
      w = static_cast<float>(cv);
    }
    const float4 yaw = make_float4(w, __fmul_rn(scale, 0.f), __fmul_rn(scale, 0.f), __fmul_rn(scale, angle));
    const float4 q = QMulDev(QMulDev(si, yaw), nq);
    float4 qn = QMulDev(make_float4(1.f, 0.f, 0.f, 0.f), q);
    const float n2 = __fadd_rn(__fadd_rn(__fmul_rn(qn.y, qn.y), __fmul_rn(qn.w, qn.w)),
                               __fadd_rn(__fmul_rn(qn.z, qn.z), __fmul_rn(qn.x, qn.x)));
    if (n2 > 0.f) {
      const float n = sqrtf(n2);
      qn = make_float4(__fdiv_rn(qn.x, n), __fdiv_rn(qn.y, n), __fdiv_rn(qn.z, n), __fdiv_rn(qn.w, n));
    }
    Yaw3Desc y;
    y.qw = q.x;
    y.qx = q.y;
    y.qy = q.z;
    y.qz = q.w;
    y.nw = qn.x;
    y.nx = qn.y;
    y.ny = qn.z;
    y.nz = qn.w;
    y.tx = it.tx;
    y.ty = it.ty;
    y.tz = it.tz;
    y.rotational_score = score;
    y.pair = dp;
    y.yaw_id = j;
    out[it.yaw_begin + j] = y;
    if (flag) {
      const unsigned f = atomicAdd(flag_count, 1u);
      if (f < static_cast<unsigned>(kYawFlagCap)) {
        YawFlag3 r;
        r.dp = dp;
        r.j = j;
        r.k = k;
        r.score = score;
        flags[f] = r;
      }
    }
  }
}

// The yaws of each pair whose rotational score passes (the filter of
// GetDiscreteScans, fast_correlative_scan_matcher_3d.cc:258-270: kept unless
// score < min_rotational_score, compared in double), in increasing k,
// appended at a global cursor: range[p] = {offset, count}. Only these travel
// back to the host.
__global__ void __launch_bounds__(256)
yaw_compact(const RotPair3* __restrict__ pairs, const float* __restrict__ scores,
            unsigned* __restrict__ cursor, int2* __restrict__ range, int32_t* __restrict__ out_k,
            float* __restrict__ out_s) {
  __shared__ int wcount[4];
  __shared__ int base_sh;
  const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const RotPair3 rp = pairs[p];
  const int nk = 2 * rp.window + 1;
  const float* sc = scores + rp.out;
  auto pass = [&](int k) { return k < nk && !(static_cast<double>(sc[k]) < rp.min_score); };
  int cnt = 0;
  for (int k = tid; k < nk; k += 256) cnt += pass(k);
  for (int m = 32; m > 0; m >>= 1) cnt += __shfl_xor(cnt, m, 64);
  if (lane == 0) wcount[w] = cnt;
  __syncthreads();
  if (tid == 0) {
    const int total = wcount[0] + wcount[1] + wcount[2] + wcount[3];
    const int base = static_cast<int>(atomicAdd(cursor, static_cast<unsigned>(total)));
    range[p] = make_int2(base, total);
    base_sh = base;
  }
  __syncthreads();
  int at = base_sh;
  for (int c0 = 0; c0 < nk; c0 += 256) {
    const int k = c0 + tid;
    const bool f = pass(k);
    const unsigned long long b = __ballot(f);
    __syncthreads();
    if (lane == 0) wcount[w] = __popcll(b);
    __syncthreads();
    int before = 0;
    for (int v = 0; v < w; ++v) before += wcount[v];
    if (f) {
      const int pos = at + before + __popcll(b & ((1ull << lane) - 1ull));
      out_k[pos] = k;
      out_s[pos] = sc[k];
    }
    at += wcount[0] + wcount[1] + wcount[2] + wcount[3];
  }
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
  if (ob.nx <= 0 || ob.ny <= 0 || ob.nz <= 0) return hipSuccess;
  const size_t row_lds = BrickRowsLds(ob.nx, shift, half != 0);
  if (row_lds <= 65536) {
    const dim3 grid(static_cast<unsigned>(std::min<int64_t>(static_cast<int64_t>(ob.ny) * ob.nz, 1 << 20)));
    if (half)
      hipLaunchKernelGGL((brick_rows<false, true>), grid, dim3(kRowThreads), row_lds, st, prev, pb, shift,
                         static_cast<void*>(out), ob);
    else
      hipLaunchKernelGGL((brick_rows<false, false>), grid, dim3(kRowThreads), row_lds, st, prev, pb, shift,
                         static_cast<void*>(out), ob);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(level_gather,
                     dim3(static_cast<unsigned>((ob.nx + 255) / 256), std::min(ob.ny, 65535),
                          std::min(ob.nz, 65535)),
                     dim3(256), 0, st, prev, pb, out, ob, shift, half);
  return hipGetLastError();
}

hipError_t LaunchOctetBuild(const uint8_t* level, const Brick3& lb, int h, uint64_t* out,
                            const Brick3& ob, hipStream_t st) {
  if (ob.nx <= 0 || ob.ny <= 0 || ob.nz <= 0) return hipSuccess;
  const size_t row_lds = BrickRowsLds(ob.nx, h, false);
  if (row_lds <= 65536) {
    hipLaunchKernelGGL((brick_rows<true, false>),
                       dim3(static_cast<unsigned>(std::min<int64_t>(static_cast<int64_t>(ob.ny) * ob.nz, 1 << 20))),
                       dim3(kRowThreads), row_lds, st, level, lb, h, static_cast<void*>(out), ob);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(octet_build,
                     dim3(static_cast<unsigned>((ob.nx + 255) / 256), std::min(ob.ny, 65535),
                          std::min(ob.nz, 65535)),
                     dim3(256), 0, st, level, lb, h, out, ob);
  return hipGetLastError();
}

hipError_t LaunchBrickRowsBatch(const RowJob3* jobs, int num_jobs, int max_rows, int max_lds,
                                bool octet, bool half, hipStream_t st) {
  if (num_jobs <= 0 || max_rows <= 0) return hipSuccess;
  if (num_jobs > 65535 || max_lds > 65536 || (octet && half)) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(std::min(max_rows, 1 << 16)), static_cast<unsigned>(num_jobs));
  if (octet)
    hipLaunchKernelGGL((brick_rows_batch<true, false>), grid, dim3(kRowThreads), max_lds, st, jobs);
  else if (half)
    hipLaunchKernelGGL((brick_rows_batch<false, true>), grid, dim3(kRowThreads), max_lds, st, jobs);
  else
    hipLaunchKernelGGL((brick_rows_batch<false, false>), grid, dim3(kRowThreads), max_lds, st, jobs);
  return hipGetLastError();
}

hipError_t LaunchValuesToLevel0Batch(const ValueJob3* jobs, int num_jobs, int64_t max_n,
                                     const uint8_t* qtab, hipStream_t st) {
  if (num_jobs <= 0 || max_n <= 0) return hipSuccess;
  if (num_jobs > 65535) return hipErrorInvalidValue;
  const dim3 grid(static_cast<unsigned>(std::min<int64_t>((max_n / 4 + 256) / 256, 1 << 14)),
                  static_cast<unsigned>(num_jobs));
  hipLaunchKernelGGL(values_to_level0_batch, grid, dim3(256), 0, st, jobs, qtab);
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

hipError_t LaunchPadProbBrick(const float* prob, const Brick3& gb, float* out, hipStream_t st) {
  return LaunchPadProbBrickP(prob, gb, 1, out, st);
}

hipError_t LaunchPadProbBrickP(const float* prob, const Brick3& gb, int P, float* out,
                               hipStream_t st) {
  const int64_t total =
      static_cast<int64_t>(gb.nx + 2 * P) * (gb.ny + 2 * P) * (gb.nz + 2 * P);
  hipLaunchKernelGGL(pad_prob_brick, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256), 0,
                     st, prob, gb, P, out);
  return hipGetLastError();
}

hipError_t LaunchPadProbBrickZ(const float* prob, const Brick3& gb, int P, float* out,
                               hipStream_t st) {
  const int64_t total =
      static_cast<int64_t>(gb.nx + 2 * P) * (gb.ny + 2 * P) * (gb.nz + 2 * P);
  hipLaunchKernelGGL(pad_prob_brick_zfast, dim3(static_cast<unsigned>((total + 255) / 256)), dim3(256),
                     0, st, prob, gb, P, out);
  return hipGetLastError();
}

hipError_t LaunchRt3dScore5(int nl, int num_blocks, hipStream_t st, const float* col,
                            const Brick3& gb, int P, float res, float eps, float4 safe_lo,
                            float4 safe_hi, const float* points, int n, const float4* rot,
                            const int* rot_index, const float* rot_angle, const float4* trans,
                            const float4* col_t0, const float4* col_thr, int num_rot, double wt,
                            double wr, unsigned long long* best, float* scores, int scores_pitch) {
  const float fbx = static_cast<float>(P - gb.ox), fby = static_cast<float>(P - gb.oy),
              fbz = static_cast<float>(P - gb.oz);
  const int px = gb.nx + 2 * P, py = gb.ny + 2 * P, pz = gb.nz + 2 * P;
#define CSM_RT5(NLV)                                                                              \
  hipLaunchKernelGGL(rt3d_score5<NLV>, dim3(num_blocks, NLV), dim3(64 * NLV), 0, st, col, px, py, \
                     pz, fbx, fby, fbz, res, 1.f / res, eps, safe_lo, safe_hi, points, n, rot,    \
                     rot_index, rot_angle, trans, col_t0, col_thr, num_rot, wt, wr, best, scores, \
                     scores_pitch)
  switch (nl) {
    case 3: CSM_RT5(3); break;
    case 5: CSM_RT5(5); break;
    case 7: CSM_RT5(7); break;
    case 9: CSM_RT5(9); break;
    case 11: CSM_RT5(11); break;
    case 13: CSM_RT5(13); break;
    case 15: CSM_RT5(15); break;
    default: return hipErrorInvalidValue;
  }
#undef CSM_RT5
  return hipGetLastError();
}

hipError_t LaunchRt3dScore4(int num_blocks, hipStream_t st, const float* pad, const Brick3& gb,
                            int P, float res, float eps, float4 safe_lo, float4 safe_hi,
                            const float* points, int n, const float4* rot, const int* rot_index,
                            const float* rot_angle, const float4* trans, int num_trans,
                            int num_rot, double wt, double wr, unsigned long long* best,
                            float* scores, int scores_pitch) {
  const int per = kRt4Waves * kRt4Tw;
  hipLaunchKernelGGL(rt3d_score4, dim3(num_blocks, (num_trans + per - 1) / per), dim3(64 * kRt4Waves),
                     0, st, pad, gb.nx + 2 * P, gb.ny + 2 * P, gb.nz + 2 * P,
                     static_cast<float>(P - gb.ox), static_cast<float>(P - gb.oy),
                     static_cast<float>(P - gb.oz), res, 1.f / res, eps, safe_lo, safe_hi, points, n,
                     rot, rot_index, rot_angle, trans, num_trans, num_rot, wt, wr, best, scores,
                     scores_pitch);
  return hipGetLastError();
}

hipError_t LaunchRt3dScore2(int num_rot, hipStream_t st, const float* pad,
                            const Brick3& gb, float res, const float* points, int n,
                            const float4* rot, const float* rot_angle, const float4* trans,
                            int num_trans, int t_base, double wt, double wr,
                            unsigned long long* best, float* scores, int scores_pitch) {
  const int threads = (kRt3Rpb * num_trans + 63) / 64 * 64;
  const int blocks = (num_rot + kRt3Rpb - 1) / kRt3Rpb;
  hipLaunchKernelGGL(rt3d_score2, dim3(blocks), dim3(threads), 0, st, pad, gb.nx + 2, gb.ny + 2,
                     gb.nz + 2, gb.ox, gb.oy, gb.oz, res, 1.f / res, points, n, rot, rot_angle,
                     trans + t_base, num_trans, t_base, num_rot, wt, wr, best, scores,
                     scores_pitch);
  return hipGetLastError();
}

hipError_t LaunchRt3dScore3(int num_rot, hipStream_t st, const float* pad, const Brick3& gb,
                            float res, float eps, const float* points, int n, const float4* rot,
                            const float* rot_angle, const float4* trans, int num_trans, int t_base,
                            double wt, double wr, unsigned long long* best, float* scores,
                            int scores_pitch) {
  const int threads = (kRt3Rpb * num_trans + 63) / 64 * 64;
  const int blocks = (num_rot + kRt3Rpb - 1) / kRt3Rpb;
  hipLaunchKernelGGL(rt3d_score3<4>, dim3(blocks), dim3(threads), 0, st, pad, gb.nx + 2, gb.ny + 2,
                     gb.nz + 2, gb.ox, gb.oy, gb.oz, res, 1.f / res, eps, points, n, rot, rot_angle,
                     trans + t_base, num_trans, t_base, num_rot, wt, wr, best, scores,
                     scores_pitch);
  return hipGetLastError();
}

hipError_t LaunchFast3dSearch(int tier, int grid, hipStream_t st, const Submap3Desc* submaps,
                              const Pair3Desc* pairs, const Yaw3Desc* yaws, int item_begin,
                              int num_items, const float* points, const float* low_points,
                              unsigned* counter, unsigned long long* best, int32_t* status,
                              unsigned long long* stats, int4* spill, unsigned long long* best_hi,
                              uint4* ties, int32_t* tie_count) {
  if (tier == 0)
    hipLaunchKernelGGL((fast3d_search<kTiny3dPoints, kSearch3dBlocksPerCuTiny, kTinyStack3d,
                                      kTinyInflight3d, kTinyBatch3d>),
                       dim3(grid), dim3(kSearch3dThreads), 0, st, submaps, pairs, yaws, item_begin,
                       num_items, points, low_points, counter, best, status, stats, spill, best_hi,
                       ties, tie_count);
  else if (tier == 1)
    hipLaunchKernelGGL((fast3d_search<kSmall3dPoints, kSearch3dBlocksPerCu, kStack3d, 16, kBatch3d>),
                       dim3(grid), dim3(kSearch3dThreads), 0, st, submaps, pairs, yaws, item_begin,
                       num_items, points, low_points, counter, best, status, stats, spill, best_hi,
                       ties, tie_count);
  else
    hipLaunchKernelGGL((fast3d_search<kMax3dPoints, kSearch3dBlocksPerCuLarge, kStack3d, 16, kBatch3d>),
                       dim3(grid), dim3(kSearch3dThreads), 0, st, submaps, pairs, yaws, item_begin,
                       num_items, points, low_points, counter, best, status, stats, spill, best_hi,
                       ties, tie_count);
  return hipGetLastError();
}

hipError_t LaunchGridBuildBatch(const GridJob3* jobs, int num_jobs, int64_t max_n, int64_t max_count,
                                const float* ptab, hipStream_t st) {
  if (num_jobs <= 0 || max_n <= 0) return hipSuccess;
  // Grid-stride over each job: at most 2048 blocks per job in x.
  auto blocks = [](int64_t work) {
    const int64_t b = (work + 255) / 256;
    return static_cast<unsigned>(b < 1 ? 1 : b > 2048 ? 2048 : b);
  };
  hipLaunchKernelGGL(grid_zero_batch, dim3(blocks(max_n / 8 + 8), num_jobs), dim3(256), 0, st, jobs);
  if (max_count > 0)
    hipLaunchKernelGGL(grid_scatter_batch, dim3(blocks(max_count), num_jobs), dim3(256), 0, st, jobs);
  hipLaunchKernelGGL(grid_prob_batch, dim3(blocks(max_n), num_jobs), dim3(256), 0, st, jobs, ptab);
  return hipGetLastError();
}

hipError_t LaunchBrickScatter(const int32_t* ijk, const uint16_t* values, int64_t count,
                              const Brick3& b, uint16_t* out, hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(brick_scatter, dim3(static_cast<unsigned>((count + 255) / 256)), dim3(256), 0, st,
                     ijk, values, count, b, out);
  return hipGetLastError();
}

hipError_t LaunchFast3dScoreQueries(int num_jobs, hipStream_t st, const Submap3Desc* submaps,
                                    const Pair3Desc* pairs, const Yaw3Desc* yaws,
                                    const float* points, const Score3Job* jobs,
                                    const int4* queries, int32_t* sums) {
  if (num_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(fast3d_score_queries, dim3(num_jobs), dim3(kSearch3dThreads), 0, st, submaps,
                     pairs, yaws, points, jobs, queries, sums);
  return hipGetLastError();
}

// blockIdx.y = segment, 64 workgroups each: out == nullptr zeroes the
// segments, else segment k is copied to out + (the bytes of segments 0..k-1).
__global__ void __launch_bounds__(256) segments_kernel(Segs3 segs, uint32_t* __restrict__ out) {
  const int k = blockIdx.y;
  int64_t at = 0;
  for (int j = 0; j < k; ++j) at += segs.bytes[j];
  uint32_t* p = static_cast<uint32_t*>(segs.ptr[k]);
  const int64_t words = segs.bytes[k] / 4;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < words; i += 256 * gridDim.x) {
    if (out)
      out[at / 4 + i] = p[i];
    else
      p[i] = 0u;
  }
}

hipError_t LaunchSegments(const Segs3& segs, void* out, hipStream_t st) {
  if (segs.n <= 0) return hipSuccess;
  for (int k = 0; k < segs.n; ++k)
    if (segs.bytes[k] % 4 != 0 || (segs.bytes[k] > 0 && !segs.ptr[k])) return hipErrorInvalidValue;
  hipLaunchKernelGGL(segments_kernel, dim3(64, segs.n), dim3(256), 0, st, segs,
                     static_cast<uint32_t*>(out));
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

hipError_t LaunchFast3dWalk(int num_jobs, hipStream_t st, const Submap3Desc* submaps,
                            const Pair3Desc* pairs, const Yaw3Desc* yaws, const float* points,
                            const float* low_points, const Walk3Job* jobs, const int4* top,
                            int4* out) {
  if (num_jobs <= 0) return hipSuccess;
  hipLaunchKernelGGL(fast3d_walk, dim3(num_jobs), dim3(kSearch3dThreads), 0, st, submaps, pairs,
                     yaws, points, low_points, jobs, top, out);
  return hipGetLastError();
}

hipError_t LaunchRotScores(const void* pairs, int num_pairs, int max_yaws, const float* hists,
                           float* out, hipStream_t st) {
  if (num_pairs <= 0 || max_yaws <= 0) return hipSuccess;
  const int threads = kRotThreads;
  hipLaunchKernelGGL(rot_scores, dim3((max_yaws + threads - 1) / threads, num_pairs), dim3(threads),
                     0, st, static_cast<const RotPair3*>(pairs), num_pairs, hists, out);
  return hipGetLastError();
}

hipError_t LaunchYawBuild(const YawBuild3* items, int num_pairs, const int32_t* k, const float* s,
                          Yaw3Desc* out, unsigned* flag_count, YawFlag3* flags, hipStream_t st) {
  if (num_pairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(yaw_build, dim3(num_pairs), dim3(64), 0, st, items, k, s, out, flag_count,
                     flags);
  return hipGetLastError();
}

hipError_t LaunchYawCompact(const void* pairs, int num_pairs, const float* scores,
                            unsigned* cursor, int2* range, int32_t* out_k, float* out_s,
                            hipStream_t st) {
  if (num_pairs <= 0) return hipSuccess;
  hipLaunchKernelGGL(yaw_compact, dim3(num_pairs), dim3(256), 0, st,
                     static_cast<const RotPair3*>(pairs), scores, cursor, range, out_k, out_s);
  return hipGetLastError();
}

}  // namespace csm
