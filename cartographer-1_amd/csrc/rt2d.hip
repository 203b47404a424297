// RealTimeCorrelativeScanMatcher2D on gfx950 (real_time_correlative_scan_
// matcher_2d.cc): Match (:117-149) and the test-visible ScoreCandidates
// (:151-176) over a ProbabilityGrid or a TSDF2D.
//
// Layout. The grid crosses the boundary as uint16 cells; the device keeps it
// converted and PADDED: a (nx + 2P) x (ny + 2P) float grid (ProbabilityGrid:
// GetProbability, kMinProbability outside the limits, :61-75) or float2 grid
// (TSDF2D: the per-cell term normalized_tsd * weight and the weight, (0, 0)
// outside, :38-59), with P = 2L + 1 for a linear window of L cells. A point's
// cell is clamped to [-(L+1), n + L] per axis, so with any offset |o| <= L
// every lookup stays inside the padded grid and a point outside the limits
// still reads the outside value: no bounds test in the inner loop. The
// converted grid is cached on the device and re-made only when the cells
// (compared with the host copy of the last call) or the padding change — in
// local SLAM the same submap is matched by consecutive scans.
//
// Kernels.
//   rt2d_convert     cells -> padded float / float2 grid (32768-entry tables,
//                    value_conversion_tables.cc:28-52).
//   rt2d_discretize  one thread per (rotation, point): GenerateRotatedScans +
//                    DiscretizeScans (correlative_scan_matcher_2d.cc:93-127)
//                    in the reference's float/double order, stored as padded
//                    flat cell indices, rotation-major.
//   rt2d_score       one 64-lane workgroup per (rotation, y offset): a lane
//                    is one x offset, so a wave's gathers read one grid row
//                    (one or two cache lines per instruction); the rotation's
//                    point indices are wave-uniform (scalar loads), the float
//                    sum runs in point order (bit-identical to the reference),
//                    and the gathers are software-pipelined two batches of
//                    kDepth points ahead, so the chain is bound by issue, not
//                    load latency. (2L+1) x num_scans single-wave workgroups
//                    spread the work over the CUs' texture units. The exp penalty is applied in double, and
//                    the first maximum in (scan, x, y) order wins
//                    (std::max_element, :142-143) through a 64-bit atomicMax.
//   rt2d_score_list  ScoreCandidates for an arbitrary candidate list and
//                    caller-given discrete scans (bounds-checked lookups).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <mutex>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "csm_internal.h"
#include "geom2d_dev.h"

namespace csm {
namespace {

constexpr int kDepthMax = 32;  // largest pipeline batch (index padding)

struct Rt2dGridDev {
  const float* prob;   // padded ProbabilityGrid (nullptr for TSDF)
  const float2* tsdf;  // padded TSDF2D (term, weight) (nullptr for probability)
  int W;               // padded row pitch
};

__device__ __forceinline__ float ConvFloat(const float* tab, uint16_t v) { return tab[v & 0x7fff]; }

// Padded grid: cell (x, y) of the limits at ((y + P) * W + x + P).
__global__ void rt2d_convert(const uint16_t* __restrict__ cells, const uint16_t* __restrict__ wcells,
                             const float* __restrict__ tab0, const float* __restrict__ tab1,
                             float max_tsd, int nx, int ny, int P, float* __restrict__ prob,
                             float2* __restrict__ tsdf) {
  const int W = nx + 2 * P, H = ny + 2 * P;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * H) return;
  const int x = i % W - P, y = i / W - P;
  const bool in = x >= 0 && y >= 0 && x < nx && y < ny;
  if (!tsdf) {
    // ProbabilityGrid::GetProbability; kMinProbability outside the limits.
    prob[i] = in ? ConvFloat(tab0, cells[y * nx + x]) : 0.1f;
    return;
  }
  if (!in) {
    tsdf[i] = make_float2(0.f, 0.f);  // (-max_tsd, 0): its term and weight are 0
    return;
  }
  const float tsd = ConvFloat(tab0, cells[y * nx + x]);
  const float w = ConvFloat(tab1, wcells[y * nx + x]);
  // (max - |tsd|) / max, times the weight (ComputeCandidateScore, :48-53).
  const float norm = __fdiv_rn(__fsub_rn(max_tsd, fabsf(tsd)), max_tsd);
  tsdf[i] = make_float2(__fmul_rn(norm, w), w);
}

__global__ void rt2d_discretize(const float* __restrict__ points, int n, int npad,
                                const float2* __restrict__ rot, int num_scans, float pre_w,
                                float pre_s, float tx, float ty, double max_x, double max_y,
                                double res, int nx, int ny, int L, int P,
                                int* __restrict__ bases, unsigned long long* __restrict__ best,
                                const uint32_t* __restrict__ warm, int warm_words,
                                uint32_t* __restrict__ sink) {
  const int64_t g = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g == 0 && best) *best = 0ull;
  {
    // Warm every XCD's L2 with the padded grid before rt2d_score gathers from
    // it: workgroups are dispatched round-robin over the 8 XCDs, so the
    // workgroups of one XCD (blockIdx % 8) together read the whole grid once.
    const int xcd_blocks = (gridDim.x + kNumXcd - 1 - blockIdx.x % kNumXcd) / kNumXcd;
    const int slot = blockIdx.x / kNumXcd;
    uint32_t acc = 0;
    for (int i = (slot * blockDim.x + threadIdx.x) * 32; i < warm_words;
         i += xcd_blocks * blockDim.x * 32)
      acc ^= warm[i];  // one word per 128-byte line
    if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads
  }
  if (g >= static_cast<int64_t>(num_scans) * npad) return;
  const int r = static_cast<int>(g / npad), i = static_cast<int>(g % npad);
  const int W = nx + 2 * P;
  if (i >= n) {  // padding up to a whole batch: any cell inside the padded grid
    bases[g] = P * W + P;
    return;
  }
  float x, y;
  // The cloud rotated by the initial angle (Match, :123-126), then by the
  // scan's angle (GenerateRotatedScans), then the translation add.
  RotateZDev(pre_w, pre_s, points[3 * i], points[3 * i + 1], &x, &y);
  const float2 q = rot[r];
  RotateZDev(q.x, q.y, x, y, &x, &y);
  const float px = __fadd_rn(tx, x), py = __fadd_rn(ty, y);
  const double cx = fmin(fmax(CellCoord(max_y, py, res), -(L + 1.)), nx + static_cast<double>(L));
  const double cy = fmin(fmax(CellCoord(max_x, px, res), -(L + 1.)), ny + static_cast<double>(L));
  bases[g] = (static_cast<int>(cy) + P) * W + static_cast<int>(cx) + P;
}

__device__ __forceinline__ unsigned long long PenalizedKey(float sum, double res, int xo, int yo,
                                                          int r, int num_angular, double step,
                                                          double wt, double wr, uint32_t idx) {
  const double cand_x = -yo * res, cand_y = -xo * res;
  const double theta = (r - num_angular) * step;
  const double pen = __dadd_rn(__dmul_rn(hypot(cand_x, cand_y), wt), __dmul_rn(fabs(theta), wr));
  const float score = static_cast<float>(__dmul_rn(static_cast<double>(sum), exp(-__dmul_rn(pen, pen))));
  return (static_cast<unsigned long long>(__float_as_uint(score)) << 32) |
         static_cast<unsigned long long>(0xffffffffu - idx);
}

template <bool kTsdf, int kDepth>
__global__ void __launch_bounds__(64)
rt2d_score(Rt2dGridDev grid, int grid_bytes, const int* __restrict__ bases, int n, int npad,
           int side, int parts_x, int L, int num_angular, double step, double res,
           double wt, double wr, unsigned long long* __restrict__ best,
           unsigned long long* __restrict__ wg_keys) {
  // Workgroup = (rotation, y offset, chunk of x offsets); lane = x offset.
  // wg_keys (mapped host memory): each workgroup stores its best key there
  // instead of the device atomicMax, and the host takes the max.
  // Lanes then read one grid row (x is the fastest index), so a gather
  // touches one or two cache lines.
  const int blk = blockIdx.x;
  const int r = blk / (side * parts_x);
  const int rem = blk - r * side * parts_x;
  const int yi = rem / parts_x, xi = (rem - yi * parts_x) * 64 + static_cast<int>(threadIdx.x);
  const int lane = threadIdx.x;
  const bool valid = xi < side;
  const int xo = -L + (valid ? xi : 0), yo = -L + yi;
  // Candidate order of GenerateExhaustiveSearchCandidates: (scan, x, y).
  const int t = (valid ? xi : 0) * side + yi;
  const int off = yo * grid.W + xo;
  // The rotation's point indices: wave-uniform, 16-byte aligned (npad is a
  // multiple of kDepth), read with scalar loads.
  const int4* __restrict__ B = reinterpret_cast<const int4*>(bases + static_cast<int64_t>(r) * npad);
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      kTsdf ? static_cast<void*>(const_cast<float2*>(grid.tsdf))
            : static_cast<void*>(const_cast<float*>(grid.prob)),
      0, grid_bytes, 0x00020000);
  constexpr int kShift = kTsdf ? 3 : 2;
  float s = 0.f, sw = 0.f;
  // Two batches of kDepth gathers in flight (A and B alternate): one batch is
  // summed while the next two are loading. The point indices (scalar loads)
  // run one more step ahead, so no gather waits on its index. Sums stay in
  // point order.
  float va[kDepth], vb[kDepth], wa[kDepth], wb[kDepth];
  int ia[kDepth], ib[kDepth];
  auto fetch = [&](int batch, int* idx) {
#pragma unroll
    for (int q = 0; q < kDepth / 4; ++q) {
      const int4 v = B[batch * (kDepth / 4) + q];
      idx[4 * q] = v.x;
      idx[4 * q + 1] = v.y;
      idx[4 * q + 2] = v.z;
      idx[4 * q + 3] = v.w;
    }
  };
  auto load = [&](const int* idx, float* v, float* w) {
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
      const int byte = (idx[k] + off) << kShift;
      if constexpr (kTsdf) {
        const auto p = __builtin_amdgcn_raw_buffer_load_b64(rsrc, byte, 0, 0);
        v[k] = __uint_as_float(p[0]);
        w[k] = __uint_as_float(p[1]);
      } else {
        v[k] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, byte, 0, 0));
      }
    }
  };
  auto add_full = [&](const float* v, const float* w) {
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
      s = __fadd_rn(s, v[k]);
      if constexpr (kTsdf) sw = __fadd_rn(sw, w[k]);
    }
  };
  auto add_part = [&](const float* v, const float* w, int count) {
#pragma unroll
    for (int k = 0; k < kDepth; ++k) {
      if (k < count) {  // uniform
        s = __fadd_rn(s, v[k]);
        if constexpr (kTsdf) sw = __fadd_rn(sw, w[k]);
      }
    }
  };
  // No branches in the steady state: loads of batches up to b + 5 are
  // unconditional (the index list is padded by four batches past the last
  // full one), so the compiler keeps the pipeline full.
  const int nfull = n / kDepth;
  fetch(0, ia);
  fetch(1, ib);
  load(ia, va, wa);
  load(ib, vb, wb);
  fetch(2, ia);
  fetch(3, ib);
  int b = 0;
  for (; b + 2 <= nfull; b += 2) {
    // sched_barrier keeps the phases in this order: without it the
    // scheduler hoists both batches' sums above the loads and drains the
    // pipeline every iteration.
    add_full(va, wa);
    __builtin_amdgcn_sched_barrier(0);
    load(ia, va, wa);
    fetch(b + 4, ia);
    __builtin_amdgcn_sched_barrier(0);
    add_full(vb, wb);
    __builtin_amdgcn_sched_barrier(0);
    load(ib, vb, wb);
    fetch(b + 5, ib);
    __builtin_amdgcn_sched_barrier(0);
  }
  add_part(va, wa, n - b * kDepth);
  add_part(vb, wb, n - (b + 1) * kDepth);
  float score;
  if constexpr (kTsdf) score = sw == 0.f ? 0.f : __fdiv_rn(s, sw);
  else score = __fdiv_rn(s, static_cast<float>(n));
  unsigned long long key = 0;
  if (valid)
    key = PenalizedKey(score, res, xo, yo, r, num_angular, step, wt, wr,
                       static_cast<uint32_t>(r * side * side + t));
  for (int m = 32; m >= 1; m >>= 1) {
    const unsigned long long o = __shfl_xor(key, m, 64);
    key = o > key ? o : key;
  }
  if (wg_keys) {
    if (lane == 0) wg_keys[blk] = key;
  } else if (lane == 0 && key != 0) {
    atomicMax(best, key);
  }
}

struct CandDev {
  int scan, xo, yo;
};

// ScoreCandidates over caller-given discrete scans (cells of the limits, not
// padded) for any candidate list; lookups outside the padded grid read the
// outside value.
template <bool kTsdf>
__global__ void rt2d_score_list(Rt2dGridDev grid, int nx, int ny, int P,
                                const int2* __restrict__ scans, int n,
                                const CandDev* __restrict__ cands, int64_t count, int num_angular,
                                double step, double res, double wt, double wr,
                                float* __restrict__ out) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (c >= count) return;
  const CandDev cd = cands[c];
  const int2* S = scans + static_cast<int64_t>(cd.scan) * n;
  float s = 0.f, sw = 0.f;
  for (int i = 0; i < n; ++i) {
    const int gx = S[i].x + cd.xo, gy = S[i].y + cd.yo;
    const bool in = gx >= 0 && gy >= 0 && gx < nx && gy < ny;
    const int64_t idx = in ? static_cast<int64_t>(gy + P) * grid.W + gx + P : 0;
    if constexpr (kTsdf) {
      const float2 v = in ? grid.tsdf[idx] : make_float2(0.f, 0.f);
      s = __fadd_rn(s, v.x);
      sw = __fadd_rn(sw, v.y);
    } else {
      s = __fadd_rn(s, in ? grid.prob[idx] : 0.1f);
    }
  }
  float score;
  if constexpr (kTsdf) score = sw == 0.f ? 0.f : __fdiv_rn(s, sw);
  else score = __fdiv_rn(s, static_cast<float>(n));
  const unsigned long long key =
      PenalizedKey(score, res, cd.xo, cd.yo, cd.scan, num_angular, step, wt, wr, 0u);
  out[c] = __uint_as_float(static_cast<uint32_t>(key >> 32));
}

// ---------------------------------------------------------------- host -----

struct GridArgs {
  const csm_map_limits* limits;
  const uint16_t* cells;
  const uint16_t* wcells;  // TSDF weights (nullptr: ProbabilityGrid)
  float truncation, max_weight;
};

bool ValidGrid(const GridArgs& g) {
  const csm_map_limits* l = g.limits;
  if (!l || !g.cells || l->num_x_cells < 1 || l->num_y_cells < 1 || !(l->resolution > 0.))
    return false;
  if (g.wcells && !(g.truncation > 0.f && g.max_weight > 0.f)) return false;
  return static_cast<int64_t>(l->num_x_cells) * l->num_y_cells <= (1ll << 28);
}

// Makes the converted, padded grid current on the device (caller holds
// ctx->mu). Re-converts only when the cells, the padding or the TSDF
// parameters differ from the previous call's.
int EnsureGrid(csm_context* ctx, const GridArgs& g, int P, Rt2dGridDev* out) {
  csm::Rt2dCache& c = ctx->rt2d;
  const int nx = g.limits->num_x_cells, ny = g.limits->num_y_cells;
  const size_t ncell = static_cast<size_t>(nx) * ny;
  const bool tsdf = g.wcells != nullptr;
  const int W = nx + 2 * P, H = ny + 2 * P;
  const bool same = c.valid && c.nx == nx && c.ny == ny && c.P == P && c.tsdf == tsdf &&
                    (!tsdf || (c.truncation == g.truncation && c.max_weight == g.max_weight)) &&
                    std::memcmp(c.cells.data(), g.cells, ncell * sizeof(uint16_t)) == 0 &&
                    (!tsdf || std::memcmp(c.wcells.data(), g.wcells, ncell * sizeof(uint16_t)) == 0);
  out->W = W;
  out->prob = tsdf ? nullptr : c.grid.as<float>();
  out->tsdf = tsdf ? c.grid.as<float2>() : nullptr;
  if (same) return CSM_OK;
  c.valid = false;
  hipStream_t st = ctx->stream;
  int rc;
  if (!c.tables) {
    // Tables: ProbabilityGrid probabilities; the TSDF ones are made per
    // (truncation, max_weight) below.
    std::vector<float> tab(32768);
    ProbabilityTable(tab.data());
    if ((rc = c.ptab.Reserve(sizeof(float) * 32768))) return rc;
    CSM_HIP(hipMemcpy(c.ptab.ptr, tab.data(), sizeof(float) * 32768, hipMemcpyHostToDevice));
    c.tables = true;
  }
  if (tsdf && (!c.ttab_ok || c.ttab_key[0] != g.truncation || c.ttab_key[1] != g.max_weight)) {
    // tsd_value_converter.cc:22-33: TSD table (min_tsd, min_tsd, max_tsd),
    // weight table (0, 0, max_weight).
    std::vector<float> tab(2 * 32768);
    ConversionTable(-g.truncation, -g.truncation, g.truncation, tab.data());
    ConversionTable(0.f, 0.f, g.max_weight, tab.data() + 32768);
    if ((rc = c.ttab.Reserve(sizeof(float) * 2 * 32768))) return rc;
    CSM_HIP(hipMemcpy(c.ttab.ptr, tab.data(), sizeof(float) * 2 * 32768, hipMemcpyHostToDevice));
    c.ttab_key[0] = g.truncation;
    c.ttab_key[1] = g.max_weight;
    c.ttab_ok = true;
  }
  const size_t cell_bytes = ncell * sizeof(uint16_t) * (tsdf ? 2 : 1);
  if ((rc = c.stage_cells.Reserve(cell_bytes))) return rc;
  if ((rc = c.dcells.Reserve(cell_bytes))) return rc;
  if ((rc = c.grid.Reserve(static_cast<size_t>(W) * H * (tsdf ? sizeof(float2) : sizeof(float)))))
    return rc;
  out->prob = tsdf ? nullptr : c.grid.as<float>();
  out->tsdf = tsdf ? c.grid.as<float2>() : nullptr;
  uint16_t* stage = c.stage_cells.as<uint16_t>();
  std::memcpy(stage, g.cells, ncell * sizeof(uint16_t));
  if (tsdf) std::memcpy(stage + ncell, g.wcells, ncell * sizeof(uint16_t));
  CSM_HIP(hipMemcpyAsync(c.dcells.ptr, stage, cell_bytes, hipMemcpyHostToDevice, st));
  const uint16_t* dc = c.dcells.as<uint16_t>();
  const int total = W * H;
  hipLaunchKernelGGL(rt2d_convert, dim3((total + 255) / 256), dim3(256), 0, st, dc,
                     tsdf ? dc + ncell : nullptr, tsdf ? c.ttab.as<float>() : c.ptab.as<float>(),
                     tsdf ? c.ttab.as<float>() + 32768 : nullptr, g.truncation, nx, ny, P,
                     tsdf ? nullptr : c.grid.as<float>(), tsdf ? c.grid.as<float2>() : nullptr);
  CSM_HIP(hipGetLastError());
  c.cells.assign(g.cells, g.cells + ncell);
  if (tsdf) c.wcells.assign(g.wcells, g.wcells + ncell);
  else c.wcells.clear();
  c.nx = nx;
  c.ny = ny;
  c.P = P;
  c.tsdf = tsdf;
  c.truncation = g.truncation;
  c.max_weight = g.max_weight;
  c.valid = true;
  return CSM_OK;
}

using Rt2dClock = std::chrono::steady_clock;

// CSM_PROFILE_RT2D=1: mean host time per Match phase (window + rotation
// table, grid check, staging + uploads, launches, wait), printed to stderr
// every 200 calls.
void Rt2dProfile(Rt2dClock::time_point a, Rt2dClock::time_point b, Rt2dClock::time_point c,
                 Rt2dClock::time_point d, Rt2dClock::time_point e, Rt2dClock::time_point f) {
  static const bool on = std::getenv("CSM_PROFILE_RT2D") != nullptr;
  if (!on) return;
  static std::mutex mu;
  static double acc[5] = {0, 0, 0, 0, 0};
  static int calls = 0;
  const Rt2dClock::time_point t[6] = {a, b, c, d, e, f};
  std::lock_guard<std::mutex> lock(mu);
  for (int k = 0; k < 5; ++k) acc[k] += std::chrono::duration<double, std::micro>(t[k + 1] - t[k]).count();
  if (++calls == 200) {
    std::fprintf(stderr,
                 "rt2d host (us/call): window %.2f, grid check %.2f, staging %.2f, launches %.2f, "
                 "wait %.2f\n",
                 acc[0] / calls, acc[1] / calls, acc[2] / calls, acc[3] / calls, acc[4] / calls);
    for (double& v : acc) v = 0;
    calls = 0;
  }
}

// RealTimeCorrelativeScanMatcher2D::Match (:117-149).
int Rt2dMatch(csm_context* ctx, const csm_rt_options* o, const GridArgs& g,
              const csm_pose2d* initial, const float* xyz, int32_t n, double* score,
              csm_pose2d* pose) {
  if (!ctx || !o || !initial || !score || !pose || n <= 0 || !xyz || !ValidGrid(g))
    return CSM_EINVAL;
  const auto t_entry = Rt2dClock::now();
  const csm_map_limits* l = g.limits;
  // :123-130: the window is built on the cloud rotated by the initial angle.
  const ZRot pre = MakeZRot(static_cast<float>(initial->theta));
  const SearchWindow2D w = MakeSearchWindow2D(o->linear_search_window, o->angular_search_window,
                                              xyz, n, l->resolution, &pre);
  const int L = w.num_linear_perturbations;
  const int side = 2 * L + 1;
  const int64_t per_rot = static_cast<int64_t>(side) * side;
  if (L > 4096 || per_rot * w.num_scans > 0xfffffffell ||
      static_cast<int64_t>(w.num_scans) * (n + 4 * kDepthMax) > (1ll << 31) - 1)
    return CSM_ERANGE;
  const int P = 2 * L + 1;
  if ((static_cast<int64_t>(l->num_x_cells) + 2 * P) * (l->num_y_cells + 2 * P) > (1ll << 27))
    return CSM_ERANGE;
  std::vector<ZRot> table;
  RotationTable(w, &table);
  const auto t_window = Rt2dClock::now();
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CSM_EHIP;
  int rc;
  Rt2dGridDev grid;
  if ((rc = EnsureGrid(ctx, g, P, &grid))) return rc;
  const auto t_grid = Rt2dClock::now();
  csm::Rt2dCache& c = ctx->rt2d;
  hipStream_t st = ctx->stream;
  // One pinned staging block: points, then the rotation table.
  const size_t pts_bytes = sizeof(float) * 3 * n;
  const size_t rot_off = (pts_bytes + 15) & ~size_t(15);
  const size_t stage_bytes = rot_off + sizeof(float2) * table.size();
  if ((rc = c.stage.Reserve(stage_bytes))) return rc;
  if ((rc = c.dstage.Reserve(stage_bytes))) return rc;
  // Whole batches plus four more of padding (see rt2d_score).
  const int npad = (n / kDepthMax + 4) * kDepthMax;
  if ((rc = c.bases.Reserve(sizeof(int) * static_cast<size_t>(w.num_scans) * npad))) return rc;
  if ((rc = c.best.Reserve(sizeof(unsigned long long)))) return rc;
  if ((rc = c.host_key.Reserve(sizeof(unsigned long long)))) return rc;
  const int parts_x = (side + 63) / 64;
  const int64_t num_blocks = static_cast<int64_t>(w.num_scans) * side * parts_x;
  // Keys to host memory (default; CSM_RT2D_HOSTKEYS=0 for the copy path):
  // each scoring workgroup writes its best key to mapped pinned memory,
  // reduced here after the synchronize, so no device-to-host copy is queued
  // and the workgroups do not contend on one atomic.
  static const bool hostkeys = [] {
    const char* e = std::getenv("CSM_RT2D_HOSTKEYS");
    return !(e && std::atoi(e) == 0);
  }();
  if ((rc = c.wg_keys.Reserve(sizeof(unsigned long long) * (hostkeys ? num_blocks : 1)))) return rc;
  unsigned long long* dkeys = nullptr;
  if (hostkeys) {
    void* dk = nullptr;
    CSM_HIP(hipHostGetDevicePointer(&dk, c.wg_keys.ptr, 0));
    dkeys = static_cast<unsigned long long*>(dk);
  }
  char* h = c.stage.as<char>();
  std::memcpy(h, xyz, pts_bytes);
  float2* hr = reinterpret_cast<float2*>(h + rot_off);
  for (size_t i = 0; i < table.size(); ++i) hr[i] = make_float2(table[i].w, table[i].s);
  CSM_HIP(hipMemcpyAsync(c.dstage.ptr, h, stage_bytes, hipMemcpyHostToDevice, st));
  const float* dpts = c.dstage.as<float>();
  const float2* drot = reinterpret_cast<const float2*>(c.dstage.as<char>() + rot_off);
  const int grid_bytes = static_cast<int>(
      (static_cast<int64_t>(l->num_x_cells) + 2 * P) * (l->num_y_cells + 2 * P) *
      (g.wcells ? sizeof(float2) : sizeof(float)));
  if ((rc = c.sink.Reserve(sizeof(uint32_t)))) return rc;
  unsigned long long* hk = c.host_key.as<unsigned long long>();
  const auto t_prep = Rt2dClock::now();
  if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev0, st));
  const int64_t nthreads = static_cast<int64_t>(w.num_scans) * npad;
  hipLaunchKernelGGL(rt2d_discretize, dim3(static_cast<unsigned>((nthreads + 255) / 256)), dim3(256),
                     0, st, dpts, n, npad, drot, w.num_scans, pre.w, pre.s,
                     static_cast<float>(initial->x), static_cast<float>(initial->y), l->max_x,
                     l->max_y, l->resolution, l->num_x_cells, l->num_y_cells, L, P,
                     c.bases.as<int>(), hostkeys ? nullptr : c.best.as<unsigned long long>(),
                     c.grid.as<uint32_t>(), grid_bytes / 4, c.sink.as<uint32_t>());
  CSM_HIP(hipGetLastError());
  const dim3 blocks(static_cast<unsigned>(num_blocks));
  // Pipeline batch: 32 gathers (x2 in flight) by default, measured fastest
  // (C1: 20.5 us against 22.8 at 16 and 29.4 at 8, profiles/r2/rt2d_depth);
  // CSM_RT2D_DEPTH selects 8 or 16 for experiments.
  static const int depth = [] {
    const char* e = std::getenv("CSM_RT2D_DEPTH");
    const int d = e ? std::atoi(e) : 32;
    return (d == 8 || d == 16) ? d : 32;
  }();
#define CSM_RT2D_LAUNCH(TSDF, D)                                                                \
  hipLaunchKernelGGL((rt2d_score<TSDF, D>), blocks, dim3(64), 0, st, grid, grid_bytes,          \
                     c.bases.as<int>(), n, npad, side, parts_x, L, w.num_angular_perturbations, \
                     w.angular_perturbation_step_size, l->resolution,                           \
                     o->translation_delta_cost_weight, o->rotation_delta_cost_weight,           \
                     c.best.as<unsigned long long>(), dkeys)
#define CSM_RT2D_DEPTHS(TSDF)                 \
  do {                                        \
    if (depth == 8) CSM_RT2D_LAUNCH(TSDF, 8); \
    else if (depth == 32) CSM_RT2D_LAUNCH(TSDF, 32); \
    else CSM_RT2D_LAUNCH(TSDF, 16);           \
  } while (0)
  if (g.wcells) CSM_RT2D_DEPTHS(true);
  else CSM_RT2D_DEPTHS(false);
#undef CSM_RT2D_DEPTHS
#undef CSM_RT2D_LAUNCH
  CSM_HIP(hipGetLastError());
  if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev1, st));
  if (!hostkeys)
    CSM_HIP(hipMemcpyAsync(hk, c.best.ptr, sizeof(unsigned long long), hipMemcpyDeviceToHost, st));
  const auto t_launch = Rt2dClock::now();
  CSM_HIP(hipStreamSynchronize(st));
  if (hostkeys) {  // the workgroups' keys: the first maximum in (scan, x, y) order wins
    const volatile unsigned long long* keys = c.wg_keys.as<unsigned long long>();
    unsigned long long k = 0;
    for (int64_t b = 0; b < num_blocks; ++b) {
      const unsigned long long v = keys[b];
      k = v > k ? v : k;
    }
    *hk = k;
  }
  if (ctx->timing) {
    float ms = 0.f;
    CSM_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->t.other_kernel_ms += ms;
  }
  Rt2dProfile(t_entry, t_window, t_grid, t_prep, t_launch, Rt2dClock::now());
  const unsigned long long key = *hk;
  if (key == 0) return CSM_EINVAL;
  const uint32_t bits = static_cast<uint32_t>(key >> 32);
  float s;
  std::memcpy(&s, &bits, sizeof(s));
  const uint32_t idx = 0xffffffffu - static_cast<uint32_t>(key & 0xffffffffu);
  const int r = static_cast<int>(idx / per_rot);
  const int t = static_cast<int>(idx % per_rot);
  const int xo = -L + t / side, yo = -L + t % side;
  // Candidate2D (correlative_scan_matcher_2d.h:73-83) and the pose update (:144-147).
  const double cx = -yo * l->resolution, cy = -xo * l->resolution;
  const double co = (r - w.num_angular_perturbations) * w.angular_perturbation_step_size;
  pose->x = initial->x + cx;
  pose->y = initial->y + cy;
  pose->theta = initial->theta + co;
  *score = s;
  return CSM_OK;
}

// RealTimeCorrelativeScanMatcher2D::ScoreCandidates (:151-176).
int Rt2dScoreCandidates(csm_context* ctx, const csm_rt_options* o, const GridArgs& g,
                        const int32_t* discrete_xy, int32_t num_scans, int32_t points_per_scan,
                        const csm_search_parameters* sp, csm_candidate2d* cands, int64_t count) {
  if (!ctx || !o || !sp || !ValidGrid(g) || count < 0 || (count > 0 && !cands) ||
      num_scans < 1 || points_per_scan < 1 || !discrete_xy)
    return CSM_EINVAL;
  if (count == 0) return CSM_OK;
  if (count > (1ll << 31) || static_cast<int64_t>(num_scans) * points_per_scan > (1ll << 28))
    return CSM_ERANGE;
  std::vector<CandDev> cd(static_cast<size_t>(count));
  for (int64_t i = 0; i < count; ++i) {
    if (cands[i].scan_index < 0 || cands[i].scan_index >= num_scans) return CSM_EINVAL;
    cd[i] = CandDev{cands[i].scan_index, cands[i].x_index_offset, cands[i].y_index_offset};
  }
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CSM_EHIP;
  int rc;
  Rt2dGridDev grid;
  // Any padding works for bounds-checked lookups: keep the cached one.
  const int P = ctx->rt2d.valid ? ctx->rt2d.P : 1;
  if ((rc = EnsureGrid(ctx, g, P, &grid))) return rc;
  hipStream_t st = ctx->stream;
  csm::DevBuf dscan, dcand, dout;
  const size_t scan_bytes = sizeof(int32_t) * 2 * static_cast<size_t>(num_scans) * points_per_scan;
  if ((rc = dscan.Reserve(scan_bytes)) || (rc = dcand.Reserve(sizeof(CandDev) * count)) ||
      (rc = dout.Reserve(sizeof(float) * count)))
    return rc;
  CSM_HIP(hipMemcpyAsync(dscan.ptr, discrete_xy, scan_bytes, hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(dcand.ptr, cd.data(), sizeof(CandDev) * count, hipMemcpyHostToDevice, st));
  const dim3 blocks(static_cast<unsigned>((count + 63) / 64));
  const csm_map_limits* l = g.limits;
  if (g.wcells)
    hipLaunchKernelGGL(rt2d_score_list<true>, blocks, dim3(64), 0, st, grid, l->num_x_cells,
                       l->num_y_cells, P, dscan.as<int2>(), points_per_scan, dcand.as<CandDev>(),
                       count, sp->num_angular_perturbations, sp->angular_perturbation_step_size,
                       sp->resolution, o->translation_delta_cost_weight,
                       o->rotation_delta_cost_weight, dout.as<float>());
  else
    hipLaunchKernelGGL(rt2d_score_list<false>, blocks, dim3(64), 0, st, grid, l->num_x_cells,
                       l->num_y_cells, P, dscan.as<int2>(), points_per_scan, dcand.as<CandDev>(),
                       count, sp->num_angular_perturbations, sp->angular_perturbation_step_size,
                       sp->resolution, o->translation_delta_cost_weight,
                       o->rotation_delta_cost_weight, dout.as<float>());
  CSM_HIP(hipGetLastError());
  std::vector<float> scores(static_cast<size_t>(count));
  CSM_HIP(hipMemcpyAsync(scores.data(), dout.ptr, sizeof(float) * count, hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  for (int64_t i = 0; i < count; ++i) cands[i].score = scores[i];
  return CSM_OK;
}

}  // namespace
}  // namespace csm

extern "C" {

int csm_rt2d_match(csm_context* ctx, const csm_rt_options* o, const csm_map_limits* l,
                   const uint16_t* cells, float min_cc, float max_cc, const csm_pose2d* initial,
                   const float* xyz, int32_t n, double* score, csm_pose2d* pose) {
  (void)min_cc;  // ProbabilityGrid's bounds are the library constants
  (void)max_cc;
  return csm::Rt2dMatch(ctx, o, csm::GridArgs{l, cells, nullptr, 0.f, 0.f}, initial, xyz, n,
                        score, pose);
}

int csm_rt2d_match_tsdf(csm_context* ctx, const csm_rt_options* o, const csm_map_limits* l,
                        const uint16_t* tsd_cells, const uint16_t* weight_cells,
                        float truncation_distance, float max_weight, const csm_pose2d* initial,
                        const float* xyz, int32_t n, double* score, csm_pose2d* pose) {
  if (!weight_cells) return CSM_EINVAL;
  return csm::Rt2dMatch(ctx, o,
                        csm::GridArgs{l, tsd_cells, weight_cells, truncation_distance, max_weight},
                        initial, xyz, n, score, pose);
}

int csm_rt2d_score_candidates(csm_context* ctx, const csm_rt_options* o, const csm_map_limits* l,
                              const uint16_t* cells, float min_cc, float max_cc,
                              const int32_t* discrete_xy, int32_t num_scans,
                              int32_t points_per_scan, const csm_search_parameters* sp,
                              csm_candidate2d* candidates, int64_t num_candidates) {
  (void)min_cc;
  (void)max_cc;
  return csm::Rt2dScoreCandidates(ctx, o, csm::GridArgs{l, cells, nullptr, 0.f, 0.f},
                                  discrete_xy, num_scans, points_per_scan, sp, candidates,
                                  num_candidates);
}

int csm_rt2d_score_candidates_tsdf(csm_context* ctx, const csm_rt_options* o,
                                   const csm_map_limits* l, const uint16_t* tsd_cells,
                                   const uint16_t* weight_cells, float truncation_distance,
                                   float max_weight, const int32_t* discrete_xy,
                                   int32_t num_scans, int32_t points_per_scan,
                                   const csm_search_parameters* sp, csm_candidate2d* candidates,
                                   int64_t num_candidates) {
  if (!weight_cells) return CSM_EINVAL;
  return csm::Rt2dScoreCandidates(
      ctx, o, csm::GridArgs{l, tsd_cells, weight_cells, truncation_distance, max_weight},
      discrete_xy, num_scans, points_per_scan, sp, candidates, num_candidates);
}

}  // extern "C"
