// Host runtime of the 3D path: implements the HybridGrid, RTCSM3D and
// FastCSM3D entry points of include/csm_amd.h on top of kernels3d.hip.
//
// Per pair the host does what is O(#yaws x histogram) and below — search
// window, rotational histogram scores (RotationalScanMatcher::Match), the
// discrete-scan poses (GenerateDiscreteScans) — with the reference's float
// arithmetic; the device does everything O(points x candidates). Float
// quaternion products follow Eigen's SSE path (Geometry_SSE.h), VectorXf
// reductions Eigen's packet order (Redux.h); see DESIGN.md "3D".

#include <hip/hip_runtime.h>

#include <smmintrin.h>

#include <algorithm>
#include <array>
#include <limits>
#include <map>
#include <tuple>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/csm_amd.h"
#include "csm_device3d.h"
#include "csm_internal.h"
#include "csm_launch3d.h"
#include "parallel_sort.h"

using namespace csm;

namespace {

// ------------------------------------------------------------ float math --
struct V3 {
  float x, y, z;
};
struct Q4 {
  float w, x, y, z;
};
struct R3 {
  V3 t;
  Q4 q;
};

inline int Lround(double v) { return static_cast<int>(std::lround(v)); }
inline int LroundF(float v) { return static_cast<int>(std::lround(v)); }

V3 Rotate(const Q4& q, const V3& v) {  // Eigen _transformVector
  V3 u{q.y * v.z - q.z * v.y, q.z * v.x - q.x * v.z, q.x * v.y - q.y * v.x};
  u.x += u.x;
  u.y += u.y;
  u.z += u.z;
  const V3 c{q.y * u.z - q.z * u.y, q.z * u.x - q.x * u.z, q.x * u.y - q.y * u.x};
  return V3{(v.x + q.w * u.x) + c.x, (v.y + q.w * u.y) + c.y, (v.z + q.w * u.z) + c.z};
}
V3 Apply(const R3& r, const V3& p) {
  const V3 v = Rotate(r.q, p);
  return V3{v.x + r.t.x, v.y + r.t.y, v.z + r.t.z};
}
Q4 QMul(const Q4& a, const Q4& b) {  // Geometry_SSE.h quat_product<float>
  return Q4{(a.w * b.w - a.x * b.x) - (a.z * b.z + a.y * b.y),
            (a.x * b.w - a.z * b.y) + (a.y * b.z + a.w * b.x),
            (a.y * b.w - a.x * b.z) + (a.z * b.x + a.w * b.y),
            (a.z * b.w - a.y * b.x) + (a.x * b.y + a.w * b.z)};
}
float SqNorm4(const Q4& q) { return (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w); }
Q4 QNormalized(const Q4& q) {
  const float n2 = SqNorm4(q);
  if (n2 > 0.f) {
    const float n = std::sqrt(n2);
    return Q4{q.w / n, q.x / n, q.y / n, q.z / n};
  }
  return q;
}
Q4 QInverse(const Q4& q) {  // Quaternion::inverse
  const float n2 = SqNorm4(q);
  if (n2 > 0.f) return Q4{q.w / n2, -q.x / n2, -q.y / n2, -q.z / n2};
  return Q4{0.f, 0.f, 0.f, 0.f};
}
R3 Mul(const R3& a, const R3& b) { return R3{Apply(a, b.t), QNormalized(QMul(a.q, b.q))}; }
R3 Inverse(const R3& a) {
  const Q4 c{a.q.w, -a.q.x, -a.q.y, -a.q.z};
  const V3 t = Rotate(c, a.t);
  return R3{V3{-t.x, -t.y, -t.z}, c};
}
// Vector3f::norm(): Eigen unrolls a 3-element sum as x0 + (x1 + x2)
// (Redux.h redux_novec_unroller splits at Length / 2).
float NormV(const V3& v) { return std::sqrt(v.x * v.x + (v.y * v.y + v.z * v.z)); }
// transform.h:86-100 for float: sin/cos of norm/2. in double.
Q4 AngleAxisToQuat(const V3& aa) {
  float scale = 0.5f, w = 1.f;
  const float sq = aa.x * aa.x + (aa.y * aa.y + aa.z * aa.z);
  if (sq > 1e-8) {
    const float norm = std::sqrt(sq);
    scale = static_cast<float>(std::sin(norm / 2.) / norm);
    w = static_cast<float>(std::cos(norm / 2.));
  }
  return Q4{w, scale * aa.x, scale * aa.y, scale * aa.z};
}
float GetAngle(const Q4& q) {  // transform.h:34-37
  return 2.f * std::atan2(std::sqrt(q.x * q.x + (q.y * q.y + q.z * q.z)), std::abs(q.w));
}
float GetYaw(const Q4& q) {  // transform.h:43-47 (C ::atan2 on promoted floats)
  const V3 d = Rotate(q, V3{1.f, 0.f, 0.f});
  return static_cast<float>(::atan2(static_cast<double>(d.y), static_cast<double>(d.x)));
}
R3 CastF(const csm_pose3d& p) {
  return R3{V3{static_cast<float>(p.t[0]), static_cast<float>(p.t[1]), static_cast<float>(p.t[2])},
            Q4{static_cast<float>(p.q[0]), static_cast<float>(p.q[1]), static_cast<float>(p.q[2]),
               static_cast<float>(p.q[3])}};
}
csm_pose3d ToPose(const V3& t, const Q4& q) {
  csm_pose3d p;
  p.t[0] = t.x;
  p.t[1] = t.y;
  p.t[2] = t.z;
  p.q[0] = q.w;
  p.q[1] = q.x;
  p.q[2] = q.y;
  p.q[3] = q.z;
  return p;
}

// kValueToProbability (probability_values.cc:26-66) and the level-0
// precomputation value (precomputation_grid_3d.cc:53-56) for every value.
void ValueTables(std::vector<float>* ptab, std::vector<uint8_t>* qtab) {
  const float kMinP = 0.1f, kMaxP = 1.f - kMinP;
  const float scale = (kMaxP - kMinP) / (32768 - 2.f);
  ptab->resize(32768);
  qtab->resize(32768);
  for (int v = 0; v < 32768; ++v) {
    const float p = v == 0 ? kMinP : v * scale + (kMinP - scale);
    (*ptab)[v] = p;
    const int c = LroundF((p - kMinP) * (255.f / (kMaxP - kMinP)));
    (*qtab)[v] = static_cast<uint8_t>(std::min(255, std::max(0, c)));
  }
}

// PrecomputationGrid3D::ToProbability(sum / float(n)) (precomputation_grid_3d.h:32-35).
float SumToProbability(int64_t sum, int n) {
  const float kMinP = 0.1f, kMaxP = 1.f - kMinP;
  return kMinP + (static_cast<float>(sum) / static_cast<float>(n)) * ((kMaxP - kMinP) / 255.f);
}
// Smallest sum whose score is > min_score (n * 255 + 1 if none).
int MinAcceptedSum(float min_score, int n) {
  int lo = -1, hi = n * 255 + 1;  // score(lo) <= min (virtual), score(hi) > min (virtual)
  while (hi - lo > 1) {
    const int mid = lo + (hi - lo) / 2;
    if (SumToProbability(mid, n) > min_score)
      hi = mid;
    else
      lo = mid;
  }
  return hi;
}

int EnsureDevice3(csm_context* ctx) {
  return hipSetDevice(ctx->device) == hipSuccess ? CSM_OK : CSM_EHIP;
}

// The value tables on the device, made once per context (caller holds ctx->mu).
int EnsureValueTables(csm_context* ctx) {
  if (ctx->f3_tables) return CSM_OK;
  std::vector<float> ptab;
  std::vector<uint8_t> qtab;
  ValueTables(&ptab, &qtab);
  int rc;
  if ((rc = ctx->f3_ptab.Reserve(sizeof(float) * 32768)) || (rc = ctx->f3_qtab.Reserve(32768)))
    return rc;
  CSM_HIP(hipMemcpy(ctx->f3_ptab.ptr, ptab.data(), sizeof(float) * 32768, hipMemcpyHostToDevice));
  CSM_HIP(hipMemcpy(ctx->f3_qtab.ptr, qtab.data(), 32768, hipMemcpyHostToDevice));
  ctx->f3_tables = true;
  return CSM_OK;
}

}  // namespace

// ----------------------------------------------------------- HybridGrid --
// Copies a HybridGrid cell list (count x (x, y, z)) into the pinned staging
// and returns its bounds in one pass: 4 cells (12 ints) per step in three
// 4-lane vectors whose lanes hold the components (x y z x), (y z x y),
// (z x y z), folded per component after the loop. count > 0.
static __attribute__((target("sse4.1"))) void StageCells(const int32_t* ijk, int64_t count, int32_t* hs,
                                                          int lo[3], int hi[3]) {
  int lx = ijk[0], ly = ijk[1], lz = ijk[2], ux = lx, uy = ly, uz = lz;
  int64_t i = 0;
  {
    const __m128i* src = reinterpret_cast<const __m128i*>(ijk);
    __m128i* dst = reinterpret_cast<__m128i*>(hs);
    __m128i lo0 = _mm_set1_epi32(INT32_MAX), lo1 = lo0, lo2 = lo0;
    __m128i hi0 = _mm_set1_epi32(INT32_MIN), hi1 = hi0, hi2 = hi0;
    for (; i + 4 <= count; i += 4, src += 3, dst += 3) {
      const __m128i a = _mm_loadu_si128(src), b = _mm_loadu_si128(src + 1),
                    c = _mm_loadu_si128(src + 2);
      _mm_storeu_si128(dst, a);
      _mm_storeu_si128(dst + 1, b);
      _mm_storeu_si128(dst + 2, c);
      lo0 = _mm_min_epi32(lo0, a); hi0 = _mm_max_epi32(hi0, a);
      lo1 = _mm_min_epi32(lo1, b); hi1 = _mm_max_epi32(hi1, b);
      lo2 = _mm_min_epi32(lo2, c); hi2 = _mm_max_epi32(hi2, c);
    }
    alignas(16) int32_t l[12], h[12];
    _mm_store_si128(reinterpret_cast<__m128i*>(l), lo0);
    _mm_store_si128(reinterpret_cast<__m128i*>(l + 4), lo1);
    _mm_store_si128(reinterpret_cast<__m128i*>(l + 8), lo2);
    _mm_store_si128(reinterpret_cast<__m128i*>(h), hi0);
    _mm_store_si128(reinterpret_cast<__m128i*>(h + 4), hi1);
    _mm_store_si128(reinterpret_cast<__m128i*>(h + 8), hi2);
    for (int k = 0; k < 12; ++k) {  // lane k holds component k % 3
      int* lo_c = k % 3 == 0 ? &lx : (k % 3 == 1 ? &ly : &lz);
      int* hi_c = k % 3 == 0 ? &ux : (k % 3 == 1 ? &uy : &uz);
      if (i > 0) {
        *lo_c = std::min(*lo_c, l[k]);
        *hi_c = std::max(*hi_c, h[k]);
      }
    }
  }
  for (; i < count; ++i) {
    const int x = ijk[3 * i], y = ijk[3 * i + 1], z = ijk[3 * i + 2];
    hs[3 * i] = x;
    hs[3 * i + 1] = y;
    hs[3 * i + 2] = z;
    lx = std::min(lx, x); ux = std::max(ux, x);
    ly = std::min(ly, y); uy = std::max(uy, y);
    lz = std::min(lz, z); uz = std::max(uz, z);
  }
  lo[0] = lx; lo[1] = ly; lo[2] = lz;
  hi[0] = ux; hi[1] = uy; hi[2] = uz;
}

int csm_hybrid_grid_create(csm_context* ctx, float resolution, const int32_t* ijk,
                           const uint16_t* values, int64_t count, int32_t grid_size,
                           csm_hybrid_grid** out) {
  if (!ctx || !out || !(resolution > 0.f) || count < 0 || (count > 0 && (!ijk || !values)))
    return CSM_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  int rc;
  if ((rc = EnsureDevice3(ctx))) return rc;
  auto g = std::make_unique<csm_hybrid_grid>();
  g->ctx = ctx;
  g->resolution = resolution;
  // The cell list goes up through pinned staging and is scattered into the
  // zeroed brick on the device (no dense host copy); bricks come from the
  // context's pool (BufPool). One pass copies the indices into the staging
  // and takes their bounds (the brick box). Each create stages into its own
  // slot (StageRing), so creates queue up without waiting for the device,
  // e.g. behind a running search.
  const size_t list_bytes = static_cast<size_t>(count) * (3 * sizeof(int32_t) + sizeof(uint16_t));
  int lo[3] = {0, 0, 0}, hi[3] = {-1, -1, -1};
  csm::StageRing::Slot* slot = nullptr;
  if (count > 0) {
    if ((rc = ctx->f3_grid_stage.Take(list_bytes, &slot))) return rc;
    int32_t* hs = slot->buf.as<int32_t>();
    StageCells(ijk, count, hs, lo, hi);
    std::memcpy(hs + 3 * count, values, sizeof(uint16_t) * count);
  }
  if (grid_size <= 0) {  // DynamicGrid growth (hybrid_grid.h:283-296, :384-399)
    int gs = 128;
    for (int a = 0; a < 3 && count > 0; ++a)
      while (lo[a] < -(gs / 2) || hi[a] >= gs / 2) gs *= 2;
    grid_size = gs;
  }
  g->grid_size = grid_size;
  Brick3& b = g->brick;
  b.ox = lo[0];
  b.oy = lo[1];
  b.oz = lo[2];
  b.nx = count > 0 ? hi[0] - lo[0] + 1 : 0;
  b.ny = count > 0 ? hi[1] - lo[1] + 1 : 0;
  b.nz = count > 0 ? hi[2] - lo[2] + 1 : 0;
  b.offset = 0;
  const int64_t n = static_cast<int64_t>(b.nx) * b.ny * b.nz;
  if (n > (int64_t{1} << 31)) return CSM_ERANGE;
  if (n > 0) {
    if ((rc = EnsureValueTables(ctx))) return rc;
    if ((rc = ctx->f3_grid_cells.Reserve(list_bytes))) return rc;
    if ((rc = ctx->pool.Take(sizeof(uint16_t) * n, &g->values))) return rc;
    if ((rc = ctx->pool.Take(sizeof(float) * n, &g->prob))) return rc;
    hipStream_t st = ctx->stream;
    CSM_HIP(hipMemcpyAsync(ctx->f3_grid_cells.ptr, slot->buf.ptr, list_bytes, hipMemcpyHostToDevice, st));
    CSM_HIP(hipEventRecord(slot->copied, st));
    CSM_HIP(hipMemsetAsync(g->values.ptr, 0, sizeof(uint16_t) * n, st));
    const int32_t* dijk = ctx->f3_grid_cells.as<int32_t>();
    const uint16_t* dval = reinterpret_cast<const uint16_t*>(dijk + 3 * count);
    CSM_HIP(LaunchBrickScatter(dijk, dval, count, b, g->values.as<uint16_t>(), st));
    CSM_HIP(LaunchBrickFromValues(g->values.as<uint16_t>(), n, ctx->f3_ptab.as<float>(), nullptr,
                                  g->prob.as<float>(), nullptr, st));
    CSM_HIP(hipEventCreateWithFlags(&g->ready, hipEventDisableTiming));
    CSM_HIP(hipEventRecord(g->ready, st));
  }
  *out = g.release();
  return CSM_OK;
}

// csm_hybrid_grid_create for many grids: one staging upload (every cell
// list and the job list), one zero / scatter / probability launch each for
// all of them (LaunchGridBuildBatch) instead of four operations per grid.
int csm_hybrid_grid_create_batch(csm_context* ctx, int32_t num, const float* resolutions,
                                 const int32_t* const* ijk, const uint16_t* const* values,
                                 const int64_t* counts, const int32_t* grid_sizes,
                                 csm_hybrid_grid** out) {
  if (!ctx || num < 0 || (num > 0 && (!resolutions || !ijk || !values || !counts || !out)))
    return CSM_EINVAL;
  if (num > 65535) return CSM_ERANGE;  // one launch's grid.y
  for (int i = 0; i < num; ++i)
    if (!(resolutions[i] > 0.f) || counts[i] < 0 || (counts[i] > 0 && (!ijk[i] || !values[i])))
      return CSM_EINVAL;
  if (num == 0) return CSM_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  int rc;
  if ((rc = EnsureDevice3(ctx))) return rc;
  // Staging layout: each grid's cells (3 int32 per cell) then values (uint16),
  // 16-byte aligned, then the job array.
  std::vector<size_t> at(num);
  size_t bytes = 0;
  for (int i = 0; i < num; ++i) {
    at[i] = bytes;
    bytes += (static_cast<size_t>(counts[i]) * (3 * sizeof(int32_t) + sizeof(uint16_t)) + 15) & ~size_t{15};
  }
  const size_t jobs_at = bytes;
  bytes += sizeof(GridJob3) * num;
  csm::StageRing::Slot* slot = nullptr;
  if ((rc = ctx->f3_grid_batch_stage.Take(bytes, &slot))) return rc;
  if ((rc = ctx->f3_grid_batch.Reserve(bytes))) return rc;
  char* hs = slot->buf.as<char>();
  char* dev = ctx->f3_grid_batch.as<char>();
  GridJob3* jobs = reinterpret_cast<GridJob3*>(hs + jobs_at);
  std::vector<std::unique_ptr<csm_hybrid_grid>> made(num);
  int njobs = 0;
  int64_t max_n = 0, max_count = 0;
  for (int i = 0; i < num; ++i) {
    auto g = std::make_unique<csm_hybrid_grid>();
    g->ctx = ctx;
    g->resolution = resolutions[i];
    const int64_t count = counts[i];
    int lo[3] = {0, 0, 0}, hi[3] = {-1, -1, -1};
    int32_t* hc = reinterpret_cast<int32_t*>(hs + at[i]);
    if (count > 0) {
      StageCells(ijk[i], count, hc, lo, hi);
      std::memcpy(hc + 3 * count, values[i], sizeof(uint16_t) * count);
    }
    int grid_size = grid_sizes ? grid_sizes[i] : 0;
    if (grid_size <= 0) {  // DynamicGrid growth, as csm_hybrid_grid_create
      int gs = 128;
      for (int a = 0; a < 3 && count > 0; ++a)
        while (lo[a] < -(gs / 2) || hi[a] >= gs / 2) gs *= 2;
      grid_size = gs;
    }
    g->grid_size = grid_size;
    Brick3& b = g->brick;
    b.ox = lo[0];
    b.oy = lo[1];
    b.oz = lo[2];
    b.nx = count > 0 ? hi[0] - lo[0] + 1 : 0;
    b.ny = count > 0 ? hi[1] - lo[1] + 1 : 0;
    b.nz = count > 0 ? hi[2] - lo[2] + 1 : 0;
    b.offset = 0;
    const int64_t n = static_cast<int64_t>(b.nx) * b.ny * b.nz;
    if (n > (int64_t{1} << 31)) return CSM_ERANGE;  // made[] returns its buffers to the pool
    if (n > 0) {
      if ((rc = ctx->pool.Take(sizeof(uint16_t) * n, &g->values))) return rc;
      if ((rc = ctx->pool.Take(sizeof(float) * n, &g->prob))) return rc;
      const int32_t* dijk = reinterpret_cast<const int32_t*>(dev + at[i]);
      jobs[njobs++] = GridJob3{dijk, reinterpret_cast<const uint16_t*>(dijk + 3 * count), count, b,
                               g->values.as<uint16_t>(), g->prob.as<float>(), n};
      max_n = std::max(max_n, n);
      max_count = std::max(max_count, count);
    }
    made[i] = std::move(g);
  }
  if (njobs > 0) {
    if ((rc = EnsureValueTables(ctx))) return rc;
    hipStream_t st = ctx->stream;
    // The job array sits at jobs_at whatever njobs is: copy through it.
    const size_t copy = jobs_at + sizeof(GridJob3) * njobs;
    CSM_HIP(hipMemcpyAsync(dev, hs, copy, hipMemcpyHostToDevice, st));
    CSM_HIP(hipEventRecord(slot->copied, st));
    CSM_HIP(LaunchGridBuildBatch(reinterpret_cast<const GridJob3*>(dev + jobs_at), njobs, max_n, max_count,
                                 ctx->f3_ptab.as<float>(), st));
    for (int i = 0; i < num; ++i) {
      if (made[i]->values.ptr == nullptr) continue;
      CSM_HIP(hipEventCreateWithFlags(&made[i]->ready, hipEventDisableTiming));
      CSM_HIP(hipEventRecord(made[i]->ready, st));
    }
  }
  for (int i = 0; i < num; ++i) out[i] = made[i].release();
  return CSM_OK;
}

void csm_hybrid_grid_destroy(csm_hybrid_grid* g) {
  if (!g) return;
  (void)hipSetDevice(g->ctx->device);
  g->ctx->pool.Give(&g->values);  // reused by the next create
  g->ctx->pool.Give(&g->prob);
  if (g->ready) (void)hipEventDestroy(g->ready);
  delete g;
}

int csm_hybrid_grid_info(const csm_hybrid_grid* g, int32_t* origin3, int32_t* dims3,
                         int32_t* grid_size) {
  if (!g) return CSM_EINVAL;
  if (origin3) {
    origin3[0] = g->brick.ox;
    origin3[1] = g->brick.oy;
    origin3[2] = g->brick.oz;
  }
  if (dims3) {
    dims3[0] = g->brick.nx;
    dims3[1] = g->brick.ny;
    dims3[2] = g->brick.nz;
  }
  if (grid_size) *grid_size = g->grid_size;
  return CSM_OK;
}

// ------------------------------------------------------------- RTCSM3D --
namespace {

// GenerateExhaustiveSearchTransforms (real_time_correlative_scan_matcher_3d.cc:
// 55-95) composed with the initial pose (:41-42): rotation r = ((rz + A) *
// na + ry + A) * na + rx + A and translation t = ((z + L) * nl + y + L) * nl +
// x + L, candidate index t * num_rot + r (the reference's loop order).
struct Rt3dWindow {
  int L = 0, A = 0;
  int64_t nl = 0, na = 0, num_trans = 0, num_rot = 0;
  std::vector<float4> rot, trans;
  std::vector<float> angle;
};

int MakeRt3dWindow(const csm_rt_options* o, float res, const csm_pose3d* initial, const float* xyz,
                   int32_t n, Rt3dWindow* w) {
  w->L = Lround(o->linear_search_window / res);
  float max_range = 3.f * res;
  for (int i = 0; i < n; ++i)
    max_range = std::max(NormV(V3{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]}), max_range);
  const float step = (1.f - 1e-3f) * std::acos(1.f - (res * res) / (2.f * (max_range * max_range)));
  w->A = Lround(o->angular_search_window / step);
  const int L = w->L, A = w->A;
  if (L < 0 || A < 0 || L > 1000 || A > 1000) return CSM_ERANGE;
  w->nl = 2 * L + 1;
  w->na = 2 * A + 1;
  w->num_trans = w->nl * w->nl * w->nl;
  w->num_rot = w->na * w->na * w->na;
  if (w->num_trans * w->num_rot >= (int64_t{1} << 32) || w->num_rot > (int64_t{1} << 31))
    return CSM_ERANGE;
  const R3 init = CastF(*initial);
  w->rot.resize(w->num_rot);
  w->angle.resize(w->num_rot);
  const int64_t na = w->na, nl = w->nl;
  for (int rz = -A; rz <= A; ++rz)
    for (int ry = -A; ry <= A; ++ry)
      for (int rx = -A; rx <= A; ++rx) {
        const int64_t r = ((rz + A) * na + (ry + A)) * na + (rx + A);
        const Q4 qs = AngleAxisToQuat(V3{static_cast<float>(rx) * step,
                                         static_cast<float>(ry) * step,
                                         static_cast<float>(rz) * step});
        const Q4 q = QNormalized(QMul(init.q, qs));  // initial.cast<float>() * transform
        w->rot[r] = make_float4(q.x, q.y, q.z, q.w);
        w->angle[r] = GetAngle(qs);
      }
  w->trans.resize(w->num_trans);
  for (int z = -L; z <= L; ++z)
    for (int y = -L; y <= L; ++y)
      for (int x = -L; x <= L; ++x) {
        const int64_t t = ((z + L) * nl + (y + L)) * nl + (x + L);
        const V3 tv{static_cast<float>(x) * res, static_cast<float>(y) * res,
                    static_cast<float>(z) * res};
        const V3 T = Apply(init, tv);
        w->trans[t] = make_float4(T.x, T.y, T.z, NormV(tv));
      }
  return CSM_OK;
}

// Scores the window's candidates over `rot` (num_rot of the window's
// rotations, angles alongside): the best key (scores == nullptr) or every
// candidate's score into the device array scores[r * num_trans + t].
int RunRt3d(csm_context* ctx, const csm_rt_options* o, const csm_hybrid_grid* grid, const float* xyz,
            int32_t n, const Rt3dWindow& w, const float4* rot, const float* angle,
            int64_t num_rot, unsigned long long* key, float* dscores, bool lattice) {
  hipStream_t st = ctx->stream;
  int rc;
  const float res = grid->resolution;
  const int64_t num_trans = w.num_trans;
  if ((rc = ctx->rt3_rot.Reserve(sizeof(float4) * num_rot + sizeof(float) * num_rot))) return rc;
  if ((rc = ctx->rt3_trans.Reserve(sizeof(float4) * num_trans))) return rc;
  if ((rc = ctx->rt3_points.Reserve(sizeof(float) * 3 * n))) return rc;
  if ((rc = ctx->rt3_best.Reserve(sizeof(unsigned long long)))) return rc;
  float4* drot = ctx->rt3_rot.as<float4>();
  float* dangle = reinterpret_cast<float*>(drot + num_rot);
  CSM_HIP(hipMemcpyAsync(drot, rot, sizeof(float4) * num_rot, hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(dangle, angle, sizeof(float) * num_rot, hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(ctx->rt3_trans.ptr, w.trans.data(), sizeof(float4) * num_trans,
                         hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(ctx->rt3_points.ptr, xyz, sizeof(float) * 3 * n, hipMemcpyHostToDevice,
                         st));
  CSM_HIP(hipMemsetAsync(ctx->rt3_best.ptr, 0, sizeof(unsigned long long), st));
  const Brick3& gb = grid->brick;
  // v2 addresses the padded brick with 24-bit row products and a 32-bit byte
  // offset; larger bricks take the v1 kernel (no scoring mode).
  const bool v2 = !std::getenv("CSM_RT3D_V1") &&
                  static_cast<int64_t>(gb.nx + 2) * (gb.ny + 2) * (gb.nz + 2) < (int64_t{1} << 29) &&
                  static_cast<int64_t>(gb.ny + 2) * (gb.nz + 2) < (int64_t{1} << 24);
  if (dscores && !v2) return CSM_ERANGE;
  if (v2 && !grid->prob_pad_ready) {
    csm_hybrid_grid* g = const_cast<csm_hybrid_grid*>(grid);
    if ((rc = g->prob_pad.Reserve(sizeof(float) * (gb.nx + 2) * (gb.ny + 2) * (gb.nz + 2))))
      return rc;
    CSM_HIP(LaunchPadProbBrick(grid->prob.as<float>(), gb, g->prob_pad.as<float>(), st));
    g->prob_pad_ready = true;
  }
  // v4 (rotation lanes) over a brick padded by P cells, P = the translation
  // lattice's reach in cells + 2, when its byte offsets are exact in float.
  int P = 0;
  {
    float reach = 0.f;
    const float4 c = w.trans[w.num_trans / 2];  // the centre: initial translation
    for (const float4& t : w.trans)
      reach = std::max({reach, std::fabs(t.x - c.x), std::fabs(t.y - c.y), std::fabs(t.z - c.z)});
    P = static_cast<int>(std::ceil(reach / res)) + 2;
  }
  const bool v4 = v2 && !std::getenv("CSM_RT3D_V3") && !std::getenv("CSM_RT3D_V2") &&
                  4 * static_cast<int64_t>(gb.nx + 2 * P) * (gb.ny + 2 * P) * (gb.nz + 2 * P) <
                      (int64_t{1} << 24);
  // v3 when the padded brick's byte offsets are exact in float (< 2^24).
  const bool v3 = v2 && !v4 && !std::getenv("CSM_RT3D_V2") &&
                  4 * static_cast<int64_t>(gb.nx + 2) * (gb.ny + 2) * (gb.nz + 2) < (int64_t{1} << 24);
  // |(a' + tr') - fl(fl(a + tr) / res)| <= 2.5 * 2^-23 * (|a| + |tr|) / res
  // (rt3d_score3); the threshold takes 4 * 2^-23 * (A + T + 1).
  float eps = 0.f;
  if (v3 || v4) {
    float amax = 0.f, tmax = 0.f;
    for (int i = 0; i < n; ++i)
      amax = std::max(amax, NormV(V3{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]}));
    for (const float4& t : w.trans)
      tmax = std::max({tmax, std::fabs(t.x), std::fabs(t.y), std::fabs(t.z)});
    eps = static_cast<float>(4.0 * std::ldexp(1.0, -23) *
                             (static_cast<double>(amax) * 1.001 / res + tmax / res + 1.0));
  }
  if (v4) {
    csm_hybrid_grid* g = const_cast<csm_hybrid_grid*>(grid);
    if (g->prob_wide_pad != P) {
      if ((rc = g->prob_wide.Reserve(sizeof(float) * (gb.nx + 2 * P) * (gb.ny + 2 * P) *
                                     (gb.nz + 2 * P))))
        return rc;
      CSM_HIP(LaunchPadProbBrickP(grid->prob.as<float>(), gb, P, g->prob_wide.as<float>(), st));
      g->prob_wide_pad = P;
    }
    // Rotations in 4 x 4 x 4 blocks of the (rx, ry, rz) lattice (one block
    // per 64 lanes; holes past the lattice edge carry index -1), or in the
    // given order for a subset.
    std::vector<float4> brot;
    std::vector<int32_t> bidx;
    if (lattice) {
      const int64_t na = w.na, nb = (na + 3) / 4;
      brot.assign(static_cast<size_t>(nb * nb * nb * 64), make_float4(0.f, 0.f, 0.f, 1.f));
      bidx.assign(brot.size(), -1);
      int64_t slot = 0;
      for (int64_t bz = 0; bz < nb; ++bz)
        for (int64_t by = 0; by < nb; ++by)
          for (int64_t bx = 0; bx < nb; ++bx)
            for (int lane = 0; lane < 64; ++lane, ++slot) {
              const int64_t rx = 4 * bx + (lane & 3), ry = 4 * by + ((lane >> 2) & 3),
                            rz = 4 * bz + (lane >> 4);
              if (rx >= na || ry >= na || rz >= na) continue;
              const int64_t r = (rz * na + ry) * na + rx;
              brot[slot] = rot[r];
              bidx[slot] = static_cast<int32_t>(r);
            }
    } else {
      brot.assign(static_cast<size_t>((num_rot + 63) / 64 * 64), make_float4(0.f, 0.f, 0.f, 1.f));
      bidx.assign(brot.size(), -1);
      for (int64_t r = 0; r < num_rot; ++r) {
        brot[r] = rot[r];
        bidx[r] = static_cast<int32_t>(r);
      }
    }
    // The scaled rotated point a' keeps rint(a' + t') inside the padded box
    // for every translation t' when a' + min t' >= lo and a' + max t' <= hi
    // per axis (a margin covers the add's rounding).
    float tmin[3] = {0.f, 0.f, 0.f}, tmax3[3] = {0.f, 0.f, 0.f};
    const float inv = 1.f / res;
    for (int64_t t = 0; t < num_trans; ++t) {
      const float v[3] = {w.trans[t].x * inv, w.trans[t].y * inv, w.trans[t].z * inv};
      for (int a = 0; a < 3; ++a) {
        tmin[a] = t == 0 ? v[a] : std::min(tmin[a], v[a]);
        tmax3[a] = t == 0 ? v[a] : std::max(tmax3[a], v[a]);
      }
    }
    const int org[3] = {gb.ox, gb.oy, gb.oz}, dim[3] = {gb.nx, gb.ny, gb.nz};
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
      lo[a] = static_cast<float>(org[a] - P) - tmin[a] + 0.01f;
      hi[a] = static_cast<float>(org[a] - P + dim[a] + 2 * P - 1) - tmax3[a] - 0.01f;
    }
    const size_t rot_bytes = sizeof(float4) * brot.size() + sizeof(int32_t) * bidx.size();
    if ((rc = ctx->rt3_rot4.Reserve(rot_bytes))) return rc;
    float4* drot4 = ctx->rt3_rot4.as<float4>();
    int32_t* didx = reinterpret_cast<int32_t*>(drot4 + brot.size());
    CSM_HIP(hipMemcpyAsync(drot4, brot.data(), sizeof(float4) * brot.size(), hipMemcpyHostToDevice,
                           st));
    CSM_HIP(hipMemcpyAsync(didx, bidx.data(), sizeof(int32_t) * bidx.size(), hipMemcpyHostToDevice,
                           st));
    // v5 (column gathers) for z columns of 3 to 15 steps (one wave per
    // column, nl waves per workgroup; wider windows run v4).
    const int nl = static_cast<int>(w.nl);
    const bool v5 = !std::getenv("CSM_RT3D_V4") && nl >= 3 && nl <= 15 && (nl & 1);
    if (v5) {
      csm_hybrid_grid* g = const_cast<csm_hybrid_grid*>(grid);
      if (g->prob_col_pad != P) {
        if ((rc = g->prob_col.Reserve(sizeof(float) * (gb.nx + 2 * P) * (gb.ny + 2 * P) *
                                      (gb.nz + 2 * P))))
          return rc;
        CSM_HIP(LaunchPadProbBrickZ(grid->prob.as<float>(), gb, P, g->prob_col.as<float>(), st));
        g->prob_col_pad = P;
      }
      // Per column: step 0's scaled translation and the per-axis thresholds
      // half - drift - allowance (drift: the largest |t'(k) - t'(0) - k e_z|;
      // allowance: the two float adds' rounding, 2^-22 (|a'| + |t'| + 1)).
      float amax = 0.f, tmaxs = 0.f;
      for (int i = 0; i < n; ++i)
        amax = std::max(amax, NormV(V3{xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]}));
      for (int64_t t = 0; t < num_trans; ++t)
        tmaxs = std::max({tmaxs, std::fabs(w.trans[t].x * inv), std::fabs(w.trans[t].y * inv),
                          std::fabs(w.trans[t].z * inv)});
      const float allow = static_cast<float>(
          std::ldexp(1.0, -22) * (static_cast<double>(amax) * 1.001 / res + tmaxs + 1.0));
      const float half = 0.5f - eps;
      const int cols = nl * nl;
      std::vector<float4> ct0(static_cast<size_t>(cols)), cth(static_cast<size_t>(cols));
      for (int c = 0; c < cols; ++c) {
        const float4 T0 = w.trans[c];
        const float b0[3] = {T0.x * inv, T0.y * inv, T0.z * inv};
        float dev[3] = {0.f, 0.f, 0.f};
        for (int k = 1; k < nl; ++k) {
          const float4 T = w.trans[static_cast<int64_t>(k) * cols + c];
          const float bk[3] = {T.x * inv, T.y * inv, T.z * inv};
          dev[0] = std::max(dev[0], std::fabs(bk[0] - b0[0]));
          dev[1] = std::max(dev[1], std::fabs(bk[1] - b0[1]));
          dev[2] = std::max(dev[2], std::fabs(static_cast<float>(
                                        static_cast<double>(bk[2]) - b0[2] - k)));
        }
        ct0[c] = make_float4(b0[0], b0[1], b0[2], 0.f);
        cth[c] = make_float4(half - dev[0] - allow, half - dev[1] - allow, half - dev[2] - allow,
                             0.f);
      }
      if ((rc = ctx->rt3_cols.Reserve(sizeof(float4) * 2 * cols))) return rc;
      float4* dct0 = ctx->rt3_cols.as<float4>();
      CSM_HIP(hipMemcpyAsync(dct0, ct0.data(), sizeof(float4) * cols, hipMemcpyHostToDevice, st));
      CSM_HIP(hipMemcpyAsync(dct0 + cols, cth.data(), sizeof(float4) * cols, hipMemcpyHostToDevice,
                             st));
      if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev0, st));
      CSM_HIP(LaunchRt3dScore5(nl, static_cast<int>(brot.size() / 64), st, grid->prob_col.as<float>(),
                               gb, P, res, eps, make_float4(lo[0], lo[1], lo[2], 0.f),
                               make_float4(hi[0], hi[1], hi[2], 0.f), ctx->rt3_points.as<float>(),
                               n, drot4, didx, dangle, ctx->rt3_trans.as<float4>(), dct0,
                               dct0 + cols, static_cast<int>(num_rot),
                               o->translation_delta_cost_weight, o->rotation_delta_cost_weight,
                               ctx->rt3_best.as<unsigned long long>(), dscores,
                               static_cast<int>(num_trans)));
    } else {
    if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev0, st));
    CSM_HIP(LaunchRt3dScore4(static_cast<int>(brot.size() / 64), st, grid->prob_wide.as<float>(), gb,
                             P, res, eps, make_float4(lo[0], lo[1], lo[2], 0.f),
                             make_float4(hi[0], hi[1], hi[2], 0.f), ctx->rt3_points.as<float>(), n,
                             drot4, didx, dangle, ctx->rt3_trans.as<float4>(),
                             static_cast<int>(num_trans), static_cast<int>(num_rot),
                             o->translation_delta_cost_weight, o->rotation_delta_cost_weight,
                             ctx->rt3_best.as<unsigned long long>(), dscores,
                             static_cast<int>(num_trans)));
    }
  } else if (ctx->timing) {
    CSM_HIP(hipEventRecord(ctx->ev0, st));
  }
  for (int64_t t0 = 0; t0 < num_trans && !v4; t0 += kRt3dThreads) {
    const int cnt = static_cast<int>(std::min<int64_t>(kRt3dThreads, num_trans - t0));
    if (v3)
      CSM_HIP(LaunchRt3dScore3(static_cast<int>(num_rot), st, grid->prob_pad.as<float>(), gb, res,
                               eps, ctx->rt3_points.as<float>(), n, drot, dangle,
                               ctx->rt3_trans.as<float4>(), cnt, static_cast<int>(t0),
                               o->translation_delta_cost_weight, o->rotation_delta_cost_weight,
                               ctx->rt3_best.as<unsigned long long>(), dscores,
                               static_cast<int>(num_trans)));
    else if (v2)
      CSM_HIP(LaunchRt3dScore2(static_cast<int>(num_rot), st, grid->prob_pad.as<float>(), gb, res,
                               ctx->rt3_points.as<float>(), n, drot, dangle,
                               ctx->rt3_trans.as<float4>(), cnt, static_cast<int>(t0),
                               o->translation_delta_cost_weight, o->rotation_delta_cost_weight,
                               ctx->rt3_best.as<unsigned long long>(), dscores,
                               static_cast<int>(num_trans)));
    else
      CSM_HIP(LaunchRt3dScore(static_cast<int>(num_rot), st, grid->prob.as<float>(), gb, res,
                              ctx->rt3_points.as<float>(), n, drot, dangle,
                              ctx->rt3_trans.as<float4>(), cnt, static_cast<int>(t0),
                              o->translation_delta_cost_weight, o->rotation_delta_cost_weight,
                              ctx->rt3_best.as<unsigned long long>()));
  }
  if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev1, st));
  if (key) CSM_HIP(hipMemcpyAsync(key, ctx->rt3_best.ptr, sizeof(*key), hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  if (ctx->timing) {
    float ms = 0.f;
    CSM_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->t.other_kernel_ms += ms;
    ctx->t.rt3d_kernel_ms += ms;
    ctx->t.rt3d_lookups += static_cast<double>(num_trans) * num_rot * n;
  }
  return CSM_OK;
}

}  // namespace

int csm_rt3d_match(csm_context* ctx, const csm_rt_options* o, const csm_hybrid_grid* grid,
                   const csm_pose3d* initial, const float* xyz, int32_t n, float* score,
                   csm_pose3d* pose) {
  if (!ctx || !o || !grid || !initial || !score || !pose || n <= 0 || !xyz) return CSM_EINVAL;
  if (grid->ctx != ctx) return CSM_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  int rc;
  if ((rc = EnsureDevice3(ctx))) return rc;
  Rt3dWindow w;
  if ((rc = MakeRt3dWindow(o, grid->resolution, initial, xyz, n, &w))) return rc;
  unsigned long long key = 0;
  if ((rc = RunRt3d(ctx, o, grid, xyz, n, w, w.rot.data(), w.angle.data(), w.num_rot, &key,
                    nullptr, true)))
    return rc;
  if (key == 0) return CSM_EHIP;
  const uint32_t low = static_cast<uint32_t>(key & 0xffffffffu);
  const uint32_t idx = 0xffffffffu - low;
  const int64_t t = idx / w.num_rot, r = idx % w.num_rot;
  const uint32_t bits = static_cast<uint32_t>(key >> 32);
  float s;
  std::memcpy(&s, &bits, sizeof(s));
  *score = s;
  const float4 q = w.rot[r];
  const float4 T = w.trans[t];
  *pose = ToPose(V3{T.x, T.y, T.z}, Q4{q.w, q.x, q.y, q.z});
  return CSM_OK;
}

int csm_rt3d_window(const csm_rt_options* o, float resolution, const float* xyz, int32_t n,
                    int32_t* num_translations, int32_t* num_rotations) {
  if (!o || !(resolution > 0.f) || n <= 0 || !xyz) return CSM_EINVAL;
  const csm_pose3d id{{0., 0., 0.}, {1., 0., 0., 0.}};
  Rt3dWindow w;
  int rc;
  if ((rc = MakeRt3dWindow(o, resolution, &id, xyz, n, &w))) return rc;
  if (num_translations) *num_translations = static_cast<int32_t>(w.num_trans);
  if (num_rotations) *num_rotations = static_cast<int32_t>(w.num_rot);
  return CSM_OK;
}

int csm_rt3d_score_rotations(csm_context* ctx, const csm_rt_options* o,
                             const csm_hybrid_grid* grid, const csm_pose3d* initial,
                             const float* xyz, int32_t n, const int32_t* rotations,
                             int32_t num_rotations, float* scores) {
  if (!ctx || !o || !grid || !initial || n <= 0 || !xyz || num_rotations < 0 ||
      (num_rotations > 0 && (!rotations || !scores)))
    return CSM_EINVAL;
  if (grid->ctx != ctx) return CSM_EINVAL;
  if (num_rotations == 0) return CSM_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  int rc;
  if ((rc = EnsureDevice3(ctx))) return rc;
  Rt3dWindow w;
  if ((rc = MakeRt3dWindow(o, grid->resolution, initial, xyz, n, &w))) return rc;
  std::vector<float4> rot(static_cast<size_t>(num_rotations));
  std::vector<float> angle(static_cast<size_t>(num_rotations));
  for (int32_t k = 0; k < num_rotations; ++k) {
    if (rotations[k] < 0 || rotations[k] >= w.num_rot) return CSM_EINVAL;
    rot[k] = w.rot[rotations[k]];
    angle[k] = w.angle[rotations[k]];
  }
  DevBuf dscores;
  const size_t count = static_cast<size_t>(num_rotations) * w.num_trans;
  if ((rc = dscores.Reserve(sizeof(float) * count))) return rc;
  if ((rc = RunRt3d(ctx, o, grid, xyz, n, w, rot.data(), angle.data(), num_rotations, nullptr,
                    dscores.as<float>(), false)))
    return rc;
  CSM_HIP(hipMemcpy(scores, dscores.ptr, sizeof(float) * count, hipMemcpyDeviceToHost));
  return CSM_OK;
}

// ----------------------------------------------------------- FastCSM3D --
struct csm_fast3d {
  csm_context* ctx = nullptr;
  csm_fast3d_options options{};
  float resolution = 0.f;
  int32_t width_in_voxels = 0;
  const csm_hybrid_grid* low = nullptr;
  std::vector<float> histogram;
  DevBuf levels, octs;
  Submap3Desc desc{};
  hipEvent_t ready = nullptr;  // after the build's kernels on ctx->stream (WaitBuilt)
};

namespace {

// A matcher's level boxes and buffers (PrecomputationGridStack3D,
// fast_correlative_scan_matcher_3d.cc:57-77); the build kernels are queued by
// BuildFast3d. Caller holds ctx->mu.
struct Fast3dPlan {
  int depth = 0;
  bool empty = true;
  int shifts[kMaxLevels3d] = {0};
  int halves[kMaxLevels3d] = {0};
  const csm_hybrid_grid* high = nullptr;
};

int PlanFast3d(csm_context* ctx, const csm_hybrid_grid* high, const csm_hybrid_grid* low,
               const float* histogram, int32_t histogram_size, const csm_fast3d_options* options,
               std::unique_ptr<csm_fast3d>* out, Fast3dPlan* plan) {
  if (!high || !low || histogram_size < 0 || (histogram_size > 0 && !histogram)) return CSM_EINVAL;
  if (high->ctx != ctx || low->ctx != ctx) return CSM_EINVAL;
  int rc;
  auto m = std::make_unique<csm_fast3d>();
  m->ctx = ctx;
  m->options = *options;
  m->resolution = high->resolution;
  m->width_in_voxels = high->grid_size;
  m->low = low;
  m->histogram.assign(histogram, histogram + histogram_size);
  // Level boxes: level d covers the cells its scatter-max can reach from
  // level d-1.
  const int depth = std::min(options->branch_and_bound_depth + kExtraLevels3d, kMaxLevels3d);
  plan->depth = depth;
  plan->high = high;
  Submap3Desc& d = m->desc;
  d.num_levels = options->branch_and_bound_depth;
  d.search_levels = depth;
  d.full_resolution_depth = options->full_resolution_depth;
  d.resolution = high->resolution;
  int64_t total = 0;
  const bool empty = high->brick.nx == 0;
  plan->empty = empty;
  d.level[0] = high->brick;
  int last_width = 1;
  for (int l = 0; l < depth; ++l) {
    if (l > 0) {
      const bool half = l >= options->full_resolution_depth;
      const int next_width = 1 << l;
      const int f = 1 << std::max(0, l - options->full_resolution_depth);
      const int s = (next_width - last_width + (f - 1)) / f;
      plan->shifts[l] = s;
      plan->halves[l] = half ? 1 : 0;
      const Brick3& p = d.level[l - 1];
      Brick3 b{};
      if (!empty) {
        const int lo[3] = {p.ox - s, p.oy - s, p.oz - s};
        const int hi[3] = {p.ox + p.nx - 1, p.oy + p.ny - 1, p.oz + p.nz - 1};
        int nlo[3], nhi[3];
        for (int a = 0; a < 3; ++a) {
          nlo[a] = half ? (lo[a] >> 1) : lo[a];
          nhi[a] = half ? (hi[a] >> 1) : hi[a];
        }
        b.ox = nlo[0];
        b.oy = nlo[1];
        b.oz = nlo[2];
        b.nx = nhi[0] - nlo[0] + 1;
        b.ny = nhi[1] - nlo[1] + 1;
        b.nz = nhi[2] - nlo[2] + 1;
      }
      d.level[l] = b;
      last_width = next_width;
    }
    d.level[l].offset = total;
    const int64_t bytes = static_cast<int64_t>(d.level[l].nx) * d.level[l].ny * d.level[l].nz;
    if (bytes > (int64_t{1} << 31)) return CSM_ERANGE;
    total += (bytes + 255) & ~int64_t{255};
  }
  if (total > 0x7fffff00) return CSM_ERANGE;
  if ((rc = ctx->pool.Take(std::max<int64_t>(total, 256), &m->levels))) return rc;
  d.levels = m->levels.as<uint8_t>();
  d.levels_bytes = static_cast<int32_t>(std::max<int64_t>(total, 256));
  // Octet bricks of the DFS child levels 0..search_levels-2.
  int64_t otot = 0;
  for (int l = 0; l + 1 < depth; ++l) {
    const int h = l < options->full_resolution_depth ? (1 << l)
                                                     : (1 << (options->full_resolution_depth - 1));
    d.oct_h[l] = h;
    Brick3 ob = d.level[l];
    if (ob.nx > 0) {
      ob.ox -= h;
      ob.oy -= h;
      ob.oz -= h;
      ob.nx += h;
      ob.ny += h;
      ob.nz += h;
    }
    ob.offset = otot;
    d.oct[l] = ob;
    otot += static_cast<int64_t>(ob.nx) * ob.ny * ob.nz * 8;
  }
  if (otot > 0x7fffff00) return CSM_ERANGE;
  if ((rc = ctx->pool.Take(std::max<int64_t>(otot, 256), &m->octs))) return rc;
  d.octs = m->octs.as<uint8_t>();
  d.octs_bytes = static_cast<int32_t>(std::max<int64_t>(otot, 256));
  d.low_prob = low->prob.as<float>();
  d.low = low->brick;
  d.low_resolution = low->resolution;
  *out = std::move(m);
  return CSM_OK;
}

// Queues the pyramid builds of `count` planned matchers on ctx->stream: the
// level-0 conversion, then level by level the gathers, then the octets, each
// one launch for every matcher of the batch (blockIdx.y = matcher; a single
// matcher takes its own launches), and records each matcher's ready event. The job lists go up through pinned
// staging, rewritten only after the previous batch's copy has finished.
int BuildFast3d(csm_context* ctx, csm_fast3d* const* ms, const Fast3dPlan* plans, int count) {
  int rc;
  if ((rc = EnsureValueTables(ctx))) return rc;
  hipStream_t st = ctx->stream;
  if (count == 1) {  // one matcher: its own launches, no job list to stage
    csm_fast3d* m = ms[0];
    const Fast3dPlan& pl = plans[0];
    if (pl.empty) return CSM_OK;
    const Submap3Desc& d = m->desc;
    uint8_t* lv = m->levels.as<uint8_t>();
    const int64_t n0 = static_cast<int64_t>(d.level[0].nx) * d.level[0].ny * d.level[0].nz;
    CSM_HIP(LaunchBrickFromValues(pl.high->values.as<uint16_t>(), n0, nullptr,
                                  ctx->f3_qtab.as<uint8_t>(), nullptr, lv + d.level[0].offset, st));
    for (int l = 1; l < pl.depth; ++l)
      CSM_HIP(LaunchLevelGather(lv + d.level[l - 1].offset, d.level[l - 1], lv + d.level[l].offset,
                                d.level[l], pl.shifts[l], pl.halves[l], st));
    for (int l = 0; l + 1 < pl.depth; ++l)
      CSM_HIP(LaunchOctetBuild(lv + d.level[l].offset, d.level[l], d.oct_h[l],
                               reinterpret_cast<uint64_t*>(m->octs.as<uint8_t>() + d.oct[l].offset),
                               d.oct[l], st));
    CSM_HIP(hipEventCreateWithFlags(&m->ready, hipEventDisableTiming));
    CSM_HIP(hipEventRecord(m->ready, st));
    return CSM_OK;
  }
  std::vector<ValueJob3> vjobs;
  int depth = 0;
  for (int i = 0; i < count; ++i) depth = std::max(depth, plans[i].depth);
  std::vector<std::vector<RowJob3>> level_jobs(depth), oct_jobs(depth);
  auto row_lds = [](const Brick3& ob, int h, bool half) { return BrickRowsLds(ob.nx, h, half); };
  for (int i = 0; i < count; ++i) {
    const Fast3dPlan& pl = plans[i];
    if (pl.empty) continue;
    const Submap3Desc& d = ms[i]->desc;
    uint8_t* lv = ms[i]->levels.as<uint8_t>();
    const int64_t n0 = static_cast<int64_t>(d.level[0].nx) * d.level[0].ny * d.level[0].nz;
    vjobs.push_back(ValueJob3{pl.high->values.as<uint16_t>(), lv + d.level[0].offset, n0});
    for (int l = 1; l < pl.depth; ++l)
      level_jobs[l].push_back(RowJob3{lv + d.level[l - 1].offset, lv + d.level[l].offset,
                                      d.level[l - 1], d.level[l], pl.shifts[l],
                                      row_lds(d.level[l], pl.shifts[l], pl.halves[l] != 0)});
    for (int l = 0; l + 1 < pl.depth; ++l)
      oct_jobs[l].push_back(RowJob3{lv + d.level[l].offset, ms[i]->octs.as<uint8_t>() + d.oct[l].offset,
                                    d.level[l], d.oct[l], d.oct_h[l], row_lds(d.oct[l], d.oct_h[l], false)});
  }
  // One job array: values jobs, then each level's, then each octet level's.
  size_t nrow = 0;
  for (int l = 0; l < depth; ++l) nrow += level_jobs[l].size() + oct_jobs[l].size();
  const size_t vbytes = (sizeof(ValueJob3) * vjobs.size() + 255) & ~size_t{255};
  const size_t bytes = vbytes + sizeof(RowJob3) * nrow;
  if (bytes > 0) {
    csm::StageRing::Slot* slot = nullptr;
    if ((rc = ctx->f3_job_stage.Take(bytes, &slot))) return rc;
    if ((rc = ctx->f3_jobs.Reserve(bytes))) return rc;
    char* h = slot->buf.as<char>();
    std::memcpy(h, vjobs.data(), sizeof(ValueJob3) * vjobs.size());
    RowJob3* rj = reinterpret_cast<RowJob3*>(h + vbytes);
    for (int l = 0; l < depth; ++l) {
      for (const RowJob3& j : level_jobs[l]) *rj++ = j;
      for (const RowJob3& j : oct_jobs[l]) *rj++ = j;
    }
    CSM_HIP(hipMemcpyAsync(ctx->f3_jobs.ptr, h, bytes, hipMemcpyHostToDevice, st));
    CSM_HIP(hipEventRecord(slot->copied, st));
    const char* dev = ctx->f3_jobs.as<char>();
    int64_t max_n = 0;
    for (const ValueJob3& v : vjobs) max_n = std::max(max_n, v.n);
    CSM_HIP(LaunchValuesToLevel0Batch(reinterpret_cast<const ValueJob3*>(dev), static_cast<int>(vjobs.size()),
                                      max_n, ctx->f3_qtab.as<uint8_t>(), st));
    const RowJob3* drow = reinterpret_cast<const RowJob3*>(dev + vbytes);
    auto launch = [&](const std::vector<RowJob3>& jobs, bool octet, bool half) -> int {
      if (jobs.empty()) return CSM_OK;
      int max_rows = 0, max_lds = 0;
      for (const RowJob3& j : jobs) {
        max_rows = std::max(max_rows, j.ob.ny * j.ob.nz);
        max_lds = std::max(max_lds, j.lds);
      }
      if (max_lds > 65536) {  // rows past 16k cells: the per-cell kernels, one job at a time
        for (const RowJob3& j : jobs)
          CSM_HIP(octet ? LaunchOctetBuild(j.src, j.sb, j.h, static_cast<uint64_t*>(j.out), j.ob, st)
                        : LaunchLevelGather(j.src, j.sb, static_cast<uint8_t*>(j.out), j.ob, j.h,
                                            half ? 1 : 0, st));
      } else {
        CSM_HIP(LaunchBrickRowsBatch(drow, static_cast<int>(jobs.size()), max_rows, max_lds, octet,
                                     half, st));
      }
      drow += jobs.size();
      return CSM_OK;
    };
    const int frd = ms[0]->options.full_resolution_depth;
    for (int l = 0; l < depth; ++l) {
      if ((rc = launch(level_jobs[l], false, l >= frd && l > 0))) return rc;
      if ((rc = launch(oct_jobs[l], true, false))) return rc;
    }
  }
  for (int i = 0; i < count; ++i) {
    if (plans[i].empty) continue;
    CSM_HIP(hipEventCreateWithFlags(&ms[i]->ready, hipEventDisableTiming));
    CSM_HIP(hipEventRecord(ms[i]->ready, st));
  }
  return CSM_OK;
}

}  // namespace

int csm_fast3d_create(csm_context* ctx, const csm_hybrid_grid* high, const csm_hybrid_grid* low,
                      const float* histogram, int32_t histogram_size,
                      const csm_fast3d_options* options, csm_fast3d** out) {
  return csm_fast3d_create_batch(ctx, 1, &high, &low, &histogram, &histogram_size, options, out);
}

int csm_fast3d_create_batch(csm_context* ctx, int32_t count, const csm_hybrid_grid* const* high,
                            const csm_hybrid_grid* const* low, const float* const* histograms,
                            const int32_t* histogram_sizes, const csm_fast3d_options* options,
                            csm_fast3d** out) {
  if (!ctx || !options || count < 0 || (count > 0 && (!high || !low || !histograms ||
                                                      !histogram_sizes || !out)))
    return CSM_EINVAL;
  // fast_correlative_scan_matcher_3d.cc:60-61
  if (options->branch_and_bound_depth < 1 || options->full_resolution_depth < 1) return CSM_EINVAL;
  if (options->branch_and_bound_depth > kMaxLevels3d) return CSM_ERANGE;
  if (count > 65535) return CSM_ERANGE;  // one launch's grid.y
  if (count == 0) return CSM_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  int rc;
  if ((rc = EnsureDevice3(ctx))) return rc;
  std::vector<std::unique_ptr<csm_fast3d>> made(count);
  std::vector<Fast3dPlan> plans(count);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < count; ++i)
    if ((rc = PlanFast3d(ctx, high[i], low[i], histograms[i], histogram_sizes[i], options, &made[i],
                         &plans[i])))
      return rc;  // made[] frees what was planned
  std::vector<csm_fast3d*> ms(count);
  for (int i = 0; i < count; ++i) ms[i] = made[i].get();
  const auto t1 = std::chrono::steady_clock::now();
  if ((rc = BuildFast3d(ctx, ms.data(), plans.data(), count))) return rc;
  if (std::getenv("CSM_PROFILE3D_BUILD")) {
    const auto t2 = std::chrono::steady_clock::now();
    std::fprintf(stderr, "fast3d create_batch: %d matchers, plan %.2f ms, build issue %.2f ms\n", count,
                 std::chrono::duration<double, std::milli>(t1 - t0).count(),
                 std::chrono::duration<double, std::milli>(t2 - t1).count());
  }
  for (int i = 0; i < count; ++i) out[i] = made[i].release();
  return CSM_OK;
}

int64_t csm_fast3d_device_bytes(const csm_fast3d* m) {
  return m ? static_cast<int64_t>(m->levels.bytes + m->octs.bytes) : 0;
}

int64_t csm_hybrid_grid_device_bytes(const csm_hybrid_grid* g) {
  return g ? static_cast<int64_t>(g->values.bytes + g->prob.bytes + g->prob_pad.bytes +
                                  g->prob_wide.bytes + g->prob_col.bytes)
           : 0;
}

void csm_fast3d_destroy(csm_fast3d* m) {
  if (!m) return;
  (void)hipSetDevice(m->ctx->device);
  m->ctx->pool.Give(&m->levels);  // reused by the next create
  m->ctx->pool.Give(&m->octs);
  if (m->ready) (void)hipEventDestroy(m->ready);
  delete m;
}

int csm_fast3d_read_level(const csm_fast3d* m, int32_t level, uint8_t* out, int64_t capacity,
                          int32_t* origin3, int32_t* dims3) {
  if (!m || level < 0 || level >= m->desc.num_levels) return CSM_EINVAL;
  const Brick3& b = m->desc.level[level];
  if (origin3) {
    origin3[0] = b.ox;
    origin3[1] = b.oy;
    origin3[2] = b.oz;
  }
  if (dims3) {
    dims3[0] = b.nx;
    dims3[1] = b.ny;
    dims3[2] = b.nz;
  }
  const int64_t n = static_cast<int64_t>(b.nx) * b.ny * b.nz;
  if (!out) return CSM_OK;
  if (capacity < n) return CSM_EINVAL;
  std::lock_guard<std::mutex> lock(m->ctx->mu);
  int rc;
  if ((rc = EnsureDevice3(m->ctx))) return rc;
  if (n > 0) {
    if (m->ready) CSM_HIP(hipEventSynchronize(m->ready));
    CSM_HIP(hipMemcpy(out, m->levels.as<uint8_t>() + b.offset, n, hipMemcpyDeviceToHost));
  }
  return CSM_OK;
}

namespace {

struct PairPrep {
  Pair3Desc desc{};
  int num_yaws = 0;
  int status = CSM_OK;
  // Phase 1 results: the discrete-scan yaws and their rotational inputs.
  int angular_window = 0;
  float astep = 0.f, yaw0 = 0.f;
  R3 node_to_submap{};
  Q4 submap_inv{}, node_q{};
};

// MatchWithSearchParameters' host half up to the rotational scores
// (fast_correlative_scan_matcher_3d.cc:127-199, GenerateDiscreteScans :246-276).
// Largest point norm of a node's high-resolution cloud (float, point order):
// both the full-submap window (:215-222) and the angular step (:258-270)
// take it; computed once per node per batch.
float MaxNorm(const csm_node3d& node) {
  float m = 0.f;
  for (int i = 0; i < node.num_high_resolution; ++i)
    m = std::max(m, NormV(V3{node.high_resolution_xyz[3 * i], node.high_resolution_xyz[3 * i + 1],
                             node.high_resolution_xyz[3 * i + 2]}));
  return m;
}

void PreparePair(const csm_fast3d* m, const csm_node3d& node, const csm_pair3d& p, float max_norm,
                 PairPrep* out) {
  const csm_fast3d_options& o = m->options;
  const float res = m->resolution;
  const int n = node.num_high_resolution;
  Pair3Desc& d = out->desc;
  d.num_points = n;
  d.num_low = node.num_low_resolution;
  int wxy, wz;
  double ang;
  R3 node_pose, submap_pose;
  if (p.full_submap) {
    const float maxd = max_norm;
    wxy = wz = (m->width_in_voxels + 1) / 2 + LroundF(maxd / res + 0.5f);
    ang = M_PI;
    csm_pose3d a = p.node_pose, b = p.submap_pose;
    a.t[0] = a.t[1] = a.t[2] = 0.;
    b.t[0] = b.t[1] = b.t[2] = 0.;
    node_pose = CastF(a);
    submap_pose = CastF(b);
  } else {
    wxy = Lround(o.linear_xy_search_window / res);
    wz = Lround(o.linear_z_search_window / res);
    ang = o.angular_search_window;
    node_pose = CastF(p.node_pose);
    submap_pose = CastF(p.submap_pose);
  }
  if (wxy > kMax3dWindow || wz > kMax3dWindow || wxy < 0 || wz < 0) {
    out->status = CSM_ERANGE;
    return;
  }
  d.wxy = wxy;
  d.wz = wz;
  // Roots: the reference's lowest-resolution candidates (:301-326) at level
  // max_depth, or a coarser level of the same grid of offsets when that
  // level has more than kRootTarget3d of them or does not fit the LDS cache.
  int level = m->desc.num_levels - 1;
  for (;;) {
    const int step = 1 << level;
    d.root_level = level;
    d.top_nx = d.top_ny = (2 * wxy + step) / step;
    d.top_nz = (2 * wz + step) / step;
    const Brick3& b = m->desc.level[level];
    const int64_t bytes = static_cast<int64_t>(b.nx) * b.ny * b.nz;
    if (level + 1 >= m->desc.search_levels ||
        (static_cast<int64_t>(d.top_nx) * d.top_ny * d.top_nz <= kRootTarget3d &&
         bytes <= kTopLds3d))
      break;
    ++level;
  }
  if (static_cast<int64_t>(d.top_nx) * d.top_ny * d.top_nz > kMax3dTop) {
    out->status = CSM_ERANGE;
    return;
  }
  d.min_low_resolution_score = static_cast<float>(o.min_low_resolution_score);
  d.min_sum = MinAcceptedSum(p.min_score, std::max(n, 1));
  // Angular steps (:258-270).
  const float max_range = n > 0 ? std::max(3.f * res, max_norm) : 3.f * res;
  out->astep = (1.f - 1e-2f) * std::acos(1.f - (res * res) / (2.f * (max_range * max_range)));
  out->angular_window = Lround(ang / out->astep);
  if (out->angular_window > kMax3dYaws / 2) {
    out->status = CSM_ERANGE;
    return;
  }
  out->node_to_submap = Mul(Inverse(submap_pose), node_pose);
  // gravity_alignment.inverse().cast<float>() (double Quaternion::inverse).
  const double* g = node.gravity_alignment;
  const double gn2 = (g[1] * g[1] + g[3] * g[3]) + (g[2] * g[2] + g[0] * g[0]);
  Q4 gi{0.f, 0.f, 0.f, 0.f};
  if (gn2 > 0.)
    gi = Q4{static_cast<float>(g[0] / gn2), static_cast<float>(-g[1] / gn2),
            static_cast<float>(-g[2] / gn2), static_cast<float>(-g[3] / gn2)};
  out->yaw0 = GetYaw(QMul(out->node_to_submap.q, gi));
  out->submap_inv = QInverse(submap_pose.q);
  out->node_q = node_pose.q;
}

// Leaf key layout (kernels3d.hip LeafId): sum bits + yaw + 2 x xy + z bits;
// CSM_ERANGE when a pair with `count` discrete scans does not fit 63 bits.
void KeyBits(int count, PairPrep* out) {
  Pair3Desc& d = out->desc;
  auto bits = [](int64_t v) {
    int b = 0;
    while ((int64_t{1} << b) <= v) ++b;
    return std::max(b, 1);
  };
  d.bits_xy = bits(2 * d.wxy);
  d.bits_z = bits(2 * d.wz);
  const int yaw_bits = bits(static_cast<int64_t>(count));
  d.key_shift = yaw_bits + 2 * d.bits_xy + d.bits_z;
  const int sum_bits = bits(static_cast<int64_t>(d.num_points) * 255);
  if (d.key_shift + sum_bits > 63) out->status = CSM_ERANGE;
}

// GenerateDiscreteScans :277-294 given the rotational scores of the pair:
// the discrete scans of the yaws that passed the rotational filter (k in
// increasing order, with their scores; yaw_compact on the device), written
// straight into the batch's pinned staging at `dst`.
void BuildYaws(const int32_t* ks, const float* scores, int count, int32_t pair,
               const PairPrep& prep, Yaw3Desc* dst) {
  const int A = prep.angular_window;
  for (int j = 0; j < count; ++j) {
    const int k = ks[j];
    const float angle = static_cast<float>(k - A) * prep.astep;
    const Q4 yaw = AngleAxisToQuat(V3{0.f, 0.f, angle});
    const Q4 q = QMul(QMul(prep.submap_inv, yaw), prep.node_q);
    const Q4 qn = QNormalized(QMul(Q4{1.f, 0.f, 0.f, 0.f}, q));  // GetPoseFromCandidate
    Yaw3Desc& y = dst[j];
    y.qw = q.w;
    y.qx = q.x;
    y.qy = q.y;
    y.qz = q.z;
    y.nw = qn.w;
    y.nx = qn.x;
    y.ny = qn.y;
    y.nz = qn.z;
    y.tx = prep.node_to_submap.t.x;
    y.ty = prep.node_to_submap.t.y;
    y.tz = prep.node_to_submap.t.z;
    y.rotational_score = scores[j];
    y.pair = pair;
    y.yaw_id = j;  // increasing angle order
  }
}

// A persistent pool of host workers for the batch's per-pair host phases
// (spawning threads per phase cost ~1 ms per phase on the GPU box).
class HostPool {
 public:
  static HostPool& Get() {
    static HostPool pool;
    return pool;
  }
  // Runs f(i) for i in [0, num) on the workers and the calling thread.
  void Run(int64_t num, const std::function<void(int64_t)>& f) {
    if (num <= 0) return;
    std::unique_lock<std::mutex> lock(mu_);  // one batch phase at a time
    {
      std::lock_guard<std::mutex> g(state_);
      f_ = &f;
      num_ = num;
      next_.store(0);
      active_ = static_cast<int>(workers_.size());
      ++epoch_;
    }
    cv_.notify_all();
    Work(f, num);
    std::unique_lock<std::mutex> g(state_);
    done_.wait(g, [&] { return active_ == 0; });
    f_ = nullptr;
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(state_);
      stop_ = true;
      ++epoch_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  HostPool() {
    const int nt = static_cast<int>(
        std::max<unsigned>(1, std::min<unsigned>(16, std::thread::hardware_concurrency())));
    for (int t = 1; t < nt; ++t) workers_.emplace_back([this] { Loop(); });
  }
  void Work(const std::function<void(int64_t)>& f, int64_t num) {
    for (int64_t i = next_.fetch_add(1); i < num; i = next_.fetch_add(1)) f(i);
  }
  void Loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int64_t)>* f;
      int64_t num;
      {
        std::unique_lock<std::mutex> g(state_);
        cv_.wait(g, [&] { return stop_ || epoch_ != seen; });
        if (stop_) return;
        seen = epoch_;
        f = f_;
        num = num_;
      }
      Work(*f, num);
      std::lock_guard<std::mutex> g(state_);
      if (--active_ == 0) done_.notify_one();
    }
  }
  std::mutex mu_, state_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> workers_;
  const std::function<void(int64_t)>* f_ = nullptr;
  int64_t num_ = 0;
  std::atomic<int64_t> next_{0};
  int active_ = 0;
  uint64_t epoch_ = 0;
  bool stop_ = false;
};

template <typename F>
void ParallelPairs(int64_t num, F&& f) {
  if (num < 64) {  // not worth waking the pool
    for (int64_t i = 0; i < num; ++i) f(i);
    return;
  }
  const std::function<void(int64_t)> fn = f;
  HostPool::Get().Run(num, fn);
}

uint64_t LeafId3(const Pair3Desc& d, int yaw, int x, int y, int z) {  // kernels3d.hip LeafId
  uint64_t id = static_cast<uint64_t>(yaw);
  id = (id << d.bits_xy) | static_cast<uint64_t>(x + d.wxy);
  id = (id << d.bits_xy) | static_cast<uint64_t>(y + d.wxy);
  id = (id << d.bits_z) | static_cast<uint64_t>(z + d.wz);
  return id;
}

// fast3d_search workgroups for `items` items of a build tier: the tier's
// resident workgroups on every CU at most.
int SearchGrid3(const csm_context* ctx, int tier, int items) {
  static constexpr int kPerCu[kSearch3dTiers] = {kSearch3dBlocksPerCuTiny, kSearch3dBlocksPerCu,
                                                  kSearch3dBlocksPerCuLarge};
  return std::max(1, std::min(items, ctx->num_cus * kPerCu[tier]));
}

// DFS stack spill of every tier's grid: kDfsCap3d entries less the build's
// LDS stack per workgroup (the tiers run one after another on one stream).
size_t SpillBytes3(const csm_context* ctx) {
  return sizeof(int4) * static_cast<size_t>(kDfsCap3d - std::min(kTinyStack3d, kStack3d)) *
         static_cast<size_t>(ctx->num_cus) * kSearch3dBlocksPerCuMax;
}

// Exactly tied maxima in 3D. The search keeps, among the
// leaves that pass the low-resolution check at the best sum, the smallest
// (yaw, x, y, z) key and, next to it, the largest (best_hi). The reference
// returns the first such leaf its depth-first search reaches
// (fast_correlative_scan_matcher_3d.cc:377-440): the lowest-resolution
// candidates in the order std::sort(greater<Candidate3D>) leaves their
// generation order (scan_index, z, y, x; :297-330, :353-354) in, each node's
// children (<= 8, generated z, y, x with x fastest, :412-430) by descending
// score with ties in generation order (insertion sort: stable), and at depth 0
// the first child that passes the low-resolution check (:384-401), the
// incumbent kept on equal scores (:433-437). For a tied pair: (1) a collect
// search with the maximum as its starting best records every passing leaf at
// it; (2) their ancestors' exact scores at every reference depth are computed
// on the device (fast3d_score_queries); (3) when two distinct
// lowest-resolution ancestors share the highest score, the pair's whole
// lowest-resolution list is scored and ordered with the same introsort
// (parallel_sort.h). No oracle and no CPU scoring is involved. `code` gets
// CSM_TIE_* per device pair.
int ResolveTies3d(csm_context* ctx, csm_fast3d* const* submaps, const std::vector<Pair3Desc>& pdesc,
                  std::vector<int32_t>* stat_io, const std::vector<unsigned long long>& keys_hi,
                  std::vector<unsigned long long>* keys, std::vector<int8_t>* code) {
  const int np = static_cast<int>(pdesc.size());
  const std::vector<int32_t>& stat = *stat_io;
  std::vector<int> tied;
  for (int dp = 0; dp < np; ++dp) {
    const unsigned long long key = (*keys)[dp];
    if (stat[dp] < 0 || key == 0) continue;
    const Pair3Desc& d = pdesc[dp];
    const unsigned long long mask = (1ull << d.key_shift) - 1;
    const unsigned long long hi = keys_hi[dp];
    if ((hi >> d.key_shift) == (key >> d.key_shift) && (hi & mask) != (~key & mask))
      tied.push_back(dp);
  }
  if (tied.empty()) return CSM_OK;
  ctx->t.tied_pairs_3d += static_cast<int64_t>(tied.size());
  hipStream_t st = ctx->stream;
  Pair3Desc* dpairs = ctx->f3_pairs.as<Pair3Desc>();
  const Submap3Desc* dsub = reinterpret_cast<const Submap3Desc*>(dpairs + np);
  const Yaw3Desc* dyaws = ctx->f3_yaws.as<Yaw3Desc>();
  const int nt = static_cast<int>(tied.size());
  int rc;
  // (1) Collect search over the tied pairs' yaws (by search build tier).
  std::vector<Pair3Desc> mod(nt);
  std::vector<unsigned long long> init(nt);
  int items = 0, tier_end[kSearch3dTiers] = {};
  for (int pass = 0; pass < kSearch3dTiers; ++pass) {
    for (int t = 0; t < nt; ++t) {
      const Pair3Desc& d = pdesc[tied[t]];
      if (Search3dTier(d.num_points) != pass) continue;
      items += d.num_yaws;
    }
    tier_end[pass] = items;
  }
  if ((rc = ctx->f3_tie_yaws.Reserve(sizeof(Yaw3Desc) * std::max(items, 1)))) return rc;
  if ((rc = ctx->f3_tie_count.Reserve(sizeof(int32_t) * nt))) return rc;
  if ((rc = ctx->f3_ties.Reserve(sizeof(uint4) * kTieCap3d * static_cast<size_t>(nt)))) return rc;
  Yaw3Desc* tyaws = ctx->f3_tie_yaws.as<Yaw3Desc>();
  int at = 0;
  for (int pass = 0; pass < kSearch3dTiers; ++pass)
    for (int t = 0; t < nt; ++t) {
      const int dp = tied[t];
      const Pair3Desc& d = pdesc[dp];
      if (Search3dTier(d.num_points) != pass) continue;
      CSM_HIP(hipMemcpyAsync(tyaws + at, dyaws + d.yaw_begin, sizeof(Yaw3Desc) * d.num_yaws,
                             hipMemcpyDeviceToDevice, st));
      at += d.num_yaws;
    }
  for (int t = 0; t < nt; ++t) {
    const int dp = tied[t];
    mod[t] = pdesc[dp];
    mod[t].collect = t + 1;
    mod[t].collect_sum = static_cast<int32_t>((*keys)[dp] >> pdesc[dp].key_shift);
    init[t] = static_cast<unsigned long long>(mod[t].collect_sum) << pdesc[dp].key_shift;
    CSM_HIP(hipMemcpyAsync(dpairs + dp, &mod[t], sizeof(Pair3Desc), hipMemcpyHostToDevice, st));
    CSM_HIP(hipMemcpyAsync(ctx->f3_best.as<unsigned long long>() + dp, &init[t],
                           sizeof(unsigned long long), hipMemcpyHostToDevice, st));
  }
  CSM_HIP(hipMemsetAsync(ctx->f3_tie_count.ptr, 0, sizeof(int32_t) * nt, st));
  CSM_HIP(hipMemsetAsync(ctx->f3_counter.ptr, 0, 4 * kSearch3dTiers, st));
  unsigned* dcounter = ctx->f3_counter.as<unsigned>();
  for (int tier = 0, b = 0; tier < kSearch3dTiers; b = tier_end[tier++])
    if (tier_end[tier] > b)
      CSM_HIP(LaunchFast3dSearch(tier, SearchGrid3(ctx, tier, tier_end[tier] - b), st, dsub, dpairs,
                                 tyaws, b, tier_end[tier] - b, ctx->f3_points.as<float>(),
                                 ctx->f3_low_points.as<float>(), dcounter + tier,
                                 ctx->f3_best.as<unsigned long long>(), ctx->f3_status.as<int32_t>(),
                                 nullptr, ctx->f3_spill.as<int4>(),
                                 ctx->f3_best_hi.as<unsigned long long>(), ctx->f3_ties.as<uint4>(),
                                 ctx->f3_tie_count.as<int32_t>()));
  std::vector<int32_t> counts(nt), stat2(np);
  std::vector<uint4> leaves_all(static_cast<size_t>(kTieCap3d) * nt);
  CSM_HIP(hipMemcpyAsync(counts.data(), ctx->f3_tie_count.ptr, sizeof(int32_t) * nt,
                         hipMemcpyDeviceToHost, st));
  CSM_HIP(hipMemcpyAsync(leaves_all.data(), ctx->f3_ties.ptr, sizeof(uint4) * leaves_all.size(),
                         hipMemcpyDeviceToHost, st));
  CSM_HIP(hipMemcpyAsync(stat2.data(), ctx->f3_status.ptr, sizeof(int32_t) * np,
                         hipMemcpyDeviceToHost, st));
  // The pair descriptors back as the finalize kernel reads them.
  for (int t = 0; t < nt; ++t)
    CSM_HIP(hipMemcpyAsync(dpairs + tied[t], &pdesc[tied[t]], sizeof(Pair3Desc),
                           hipMemcpyHostToDevice, st));
  CSM_HIP(hipStreamSynchronize(st));

  // (2) Ancestor scores at every reference depth 1..D (D = max_depth).
  struct Work {
    int dp, t, D, first, count;
  };
  std::vector<Work> work;
  std::vector<int4> lv;  // per leaf: (yaw, x, y, z)
  std::vector<Score3Job> jobs;
  std::vector<int4> queries;
  std::vector<int> leaf_query;  // per leaf: index of its depth-1 ancestor query
  std::vector<int> walk;        // tied pairs (device index) whose leaves overflow the record
  for (int t = 0; t < nt; ++t) {
    const int dp = tied[t];
    const Pair3Desc& d = pdesc[dp];
    const int cnt = counts[t];
    if (stat2[dp] < 0 || cnt < 2 || cnt > kTieCap3d) {
      // More passing tied leaves than the collect pass records (or its
      // stack overflowed): the device walks the reference's order (5).
      ctx->t.ties_walked_3d += 1;
      (*code)[dp] = CSM_TIE_WALK;
      walk.push_back(dp);
      continue;
    }
    const int D = submaps[d.submap]->desc.num_levels - 1;
    Work w{dp, t, D, static_cast<int>(lv.size()), cnt};
    std::vector<std::vector<int>> by_yaw(d.num_yaws);
    for (int i = 0; i < cnt; ++i) {
      const uint4 e = leaves_all[static_cast<size_t>(t) * kTieCap3d + i];
      lv.push_back(make_int4(static_cast<int>(e.x), static_cast<int>(e.y), static_cast<int>(e.z),
                             static_cast<int>(e.w)));
      if (static_cast<int>(e.x) < d.num_yaws) by_yaw[e.x].push_back(w.first + i);
    }
    leaf_query.resize(lv.size(), -1);
    for (int j = 0; j < d.num_yaws; ++j) {
      if (by_yaw[j].empty() || D < 1) continue;
      Score3Job job{d.yaw_begin + j, static_cast<int32_t>(queries.size()), 0, 0};
      for (int li : by_yaw[j]) {
        leaf_query[li] = static_cast<int>(queries.size());
        for (int l = 1; l <= D; ++l)
          queries.push_back(make_int4(l, -d.wxy + (((lv[li].y + d.wxy) >> l) << l),
                                      -d.wxy + (((lv[li].z + d.wxy) >> l) << l),
                                      -d.wz + (((lv[li].w + d.wz) >> l) << l)));
      }
      job.count = static_cast<int32_t>(queries.size()) - job.first;
      jobs.push_back(job);
    }
    work.push_back(w);
  }
  auto score = [&](const std::vector<Score3Job>& js, const std::vector<int4>& qs,
                   std::vector<int32_t>* sums) -> int {
    sums->assign(qs.size(), 0);
    if (js.empty()) return CSM_OK;
    int r2;
    if ((r2 = ctx->f3_sq_jobs.Reserve(sizeof(Score3Job) * js.size()))) return r2;
    if ((r2 = ctx->f3_sq_queries.Reserve(sizeof(int4) * qs.size()))) return r2;
    if ((r2 = ctx->f3_sq_sums.Reserve(sizeof(int32_t) * qs.size()))) return r2;
    CSM_HIP(hipMemcpyAsync(ctx->f3_sq_jobs.ptr, js.data(), sizeof(Score3Job) * js.size(),
                           hipMemcpyHostToDevice, st));
    CSM_HIP(hipMemcpyAsync(ctx->f3_sq_queries.ptr, qs.data(), sizeof(int4) * qs.size(),
                           hipMemcpyHostToDevice, st));
    CSM_HIP(LaunchFast3dScoreQueries(static_cast<int>(js.size()), st, dsub, dpairs, dyaws,
                                     ctx->f3_points.as<float>(), ctx->f3_sq_jobs.as<Score3Job>(),
                                     ctx->f3_sq_queries.as<int4>(), ctx->f3_sq_sums.as<int32_t>()));
    CSM_HIP(hipMemcpyAsync(sums->data(), ctx->f3_sq_sums.ptr, sizeof(int32_t) * qs.size(),
                           hipMemcpyDeviceToHost, st));
    CSM_HIP(hipStreamSynchronize(st));
    return CSM_OK;
  };
  std::vector<int32_t> sums;
  if ((rc = score(jobs, queries, &sums))) return rc;
  // Ancestor of leaf li at depth l: (yaw, x, y, z, score).
  struct Anc {
    int yaw, x, y, z;
    float score;
  };
  auto anc = [&](const Work& w, int li, int l) {
    const Pair3Desc& d = pdesc[w.dp];
    if (l == 0) return Anc{lv[li].x, lv[li].y, lv[li].z, lv[li].w, 0.f};
    const int4 q = queries[leaf_query[li] + l - 1];
    return Anc{lv[li].x, q.y, q.z, q.w, SumToProbability(sums[leaf_query[li] + l - 1], d.num_points)};
  };
  // (3) Leaves under a highest-scoring lowest-resolution ancestor; the whole
  // top list of pairs where two distinct such ancestors tie.
  struct Cand {
    std::vector<int> live;
    bool need_perm = false;
    int nx = 0, ny = 0, nz = 0;
    std::vector<int64_t> pos;  // generation index -> sorted position
  };
  std::vector<Cand> cand(work.size());
  std::vector<int> perm;
  for (size_t wi = 0; wi < work.size(); ++wi) {
    const Work& w = work[wi];
    Cand& c = cand[wi];
    float top = -std::numeric_limits<float>::infinity();
    for (int i = 0; i < w.count; ++i) top = std::max(top, anc(w, w.first + i, w.D).score);
    std::vector<std::array<int, 4>> nodes;
    for (int i = 0; i < w.count; ++i) {
      const Anc a = anc(w, w.first + i, w.D);
      if (w.D > 0 && a.score != top) continue;
      c.live.push_back(w.first + i);
      const std::array<int, 4> key{a.yaw, a.x, a.y, a.z};
      if (std::find(nodes.begin(), nodes.end(), key) == nodes.end()) nodes.push_back(key);
    }
    c.need_perm = nodes.size() > 1;
    (*code)[w.dp] = c.need_perm ? CSM_TIE_TOPLIST : CSM_TIE_ANCESTORS;
    if (c.need_perm) perm.push_back(static_cast<int>(wi));
  }
  ctx->t.ties_toplist += static_cast<int64_t>(perm.size());
  if (!perm.empty()) {
    std::vector<Score3Job> tj;
    std::vector<int4> tq;
    std::vector<int64_t> base(perm.size());
    for (size_t k = 0; k < perm.size(); ++k) {
      const Work& w = work[perm[k]];
      Cand& c = cand[perm[k]];
      const Pair3Desc& d = pdesc[w.dp];
      const int step = 1 << w.D;
      c.nx = c.ny = (2 * d.wxy + step) / step;  // GenerateLowestResolutionCandidates (:301-310)
      c.nz = (2 * d.wz + step) / step;
      base[k] = static_cast<int64_t>(tq.size());
      for (int j = 0; j < d.num_yaws; ++j) {
        Score3Job job{d.yaw_begin + j, static_cast<int32_t>(tq.size()), 0, 0};
        for (int z = -d.wz; z <= d.wz; z += step)
          for (int y = -d.wxy; y <= d.wxy; y += step)
            for (int x = -d.wxy; x <= d.wxy; x += step) tq.push_back(make_int4(w.D, x, y, z));
        job.count = static_cast<int32_t>(tq.size()) - job.first;
        tj.push_back(job);
      }
    }
    std::vector<int32_t> ts;
    if ((rc = score(tj, tq, &ts))) return rc;
    for (size_t k = 0; k < perm.size(); ++k) {
      const Work& w = work[perm[k]];
      Cand& c = cand[perm[k]];
      const int64_t n = static_cast<int64_t>(pdesc[w.dp].num_yaws) * c.nx * c.ny * c.nz;
      // ScoreCandidates' std::sort(greater<Candidate3D>) on the generation
      // order: the same comparisons give the same permutation for any element.
      std::vector<std::pair<float, int32_t>> lst(n);
      for (int64_t i = 0; i < n; ++i)
        lst[i] = {SumToProbability(ts[base[k] + i], pdesc[w.dp].num_points), static_cast<int32_t>(i)};
      IntroSort(lst.data(), lst.data() + n,
                [](const std::pair<float, int32_t>& a, const std::pair<float, int32_t>& b) {
                  return a.first > b.first;
                },
                8);
      c.pos.resize(n);
      for (int64_t i = 0; i < n; ++i) c.pos[lst[i].second] = i;
    }
  }
  // (4) The reference's first leaf among the live ones.
  for (size_t wi = 0; wi < work.size(); ++wi) {
    const Work& w = work[wi];
    const Cand& c = cand[wi];
    const Pair3Desc& d = pdesc[w.dp];
    const int step = 1 << w.D;
    auto top_pos = [&](const Anc& a) {
      const int ix = (a.x + d.wxy) / step, iy = (a.y + d.wxy) / step, iz = (a.z + d.wz) / step;
      return c.pos[((static_cast<int64_t>(a.yaw) * c.nz + iz) * c.ny + iy) * c.nx + ix];
    };
    auto first = [&](int a, int b) {
      for (int l = w.D; l >= 0; --l) {
        const Anc x = anc(w, a, l), y = anc(w, b, l);
        if (x.yaw == y.yaw && x.x == y.x && x.y == y.y && x.z == y.z) continue;
        if (l == w.D) {  // lowest-resolution candidates: score, then the sorted order
          if (l > 0 && x.score != y.score) return x.score > y.score;
          return top_pos(x) < top_pos(y);
        }
        if (l > 0 && x.score != y.score) return x.score > y.score;
        // Siblings of one parent: generation order (z, then y, then x).
        return std::make_tuple(x.z, x.y, x.x) < std::make_tuple(y.z, y.y, y.x);
      }
      return false;
    };
    int best = c.live[0];
    for (size_t i = 1; i < c.live.size(); ++i)
      if (first(c.live[i], best)) best = c.live[i];
    const unsigned long long mask = (1ull << d.key_shift) - 1;
    const unsigned long long sum = (*keys)[w.dp] >> d.key_shift;
    (*keys)[w.dp] = (sum << d.key_shift) |
                    (~LeafId3(d, lv[best].x, lv[best].y, lv[best].z, lv[best].w) & mask);
  }
  // (5) Pairs whose passing tied leaves overflow the record: the whole
  // lowest-resolution list scored and sorted as in (3), and the device walks
  // the reference's visiting order from it (fast3d_walk); only entries whose
  // sum reaches the maximum can lead to the pick.
  if (!walk.empty()) {
    std::vector<Score3Job> tj;
    std::vector<int4> tq;
    std::vector<int64_t> base(walk.size());
    std::vector<int> wD(walk.size());
    for (size_t k = 0; k < walk.size(); ++k) {
      const Pair3Desc& d = pdesc[walk[k]];
      const int D = submaps[d.submap]->desc.num_levels - 1, step = 1 << D;
      wD[k] = D;
      base[k] = static_cast<int64_t>(tq.size());
      for (int j = 0; j < d.num_yaws; ++j) {
        Score3Job job{d.yaw_begin + j, static_cast<int32_t>(tq.size()), 0, 0};
        for (int z = -d.wz; z <= d.wz; z += step)  // GenerateLowestResolutionCandidates (:297-330)
          for (int y = -d.wxy; y <= d.wxy; y += step)
            for (int x = -d.wxy; x <= d.wxy; x += step) tq.push_back(make_int4(D, x, y, z));
        job.count = static_cast<int32_t>(tq.size()) - job.first;
        tj.push_back(job);
      }
    }
    std::vector<int32_t> ts;
    if ((rc = score(tj, tq, &ts))) return rc;
    std::vector<Walk3Job> wj;
    std::vector<int4> wtop;
    for (size_t k = 0; k < walk.size(); ++k) {
      const Pair3Desc& d = pdesc[walk[k]];
      const int64_t n = (k + 1 < walk.size() ? base[k + 1] : static_cast<int64_t>(tq.size())) - base[k];
      std::vector<std::pair<float, int32_t>> lst(n);
      for (int64_t i = 0; i < n; ++i)
        lst[i] = {SumToProbability(ts[base[k] + i], d.num_points), static_cast<int32_t>(i)};
      IntroSort(lst.data(), lst.data() + n,
                [](const std::pair<float, int32_t>& a, const std::pair<float, int32_t>& b) {
                  return a.first > b.first;
                },
                8);
      const int32_t target = static_cast<int32_t>((*keys)[walk[k]] >> d.key_shift);
      Walk3Job j{walk[k], target, wD[k], static_cast<int32_t>(wtop.size()), 0, {0, 0, 0}};
      const int per_yaw = static_cast<int>(n / std::max(1, d.num_yaws));
      for (const auto& e : lst) {
        const int32_t sum = ts[base[k] + e.second];
        if (sum < target) continue;
        const int4 q = tq[base[k] + e.second];
        const int yaw = e.second / per_yaw;
        wtop.push_back(make_int4(yaw, (q.y & 0xffff) | (q.z << 16), q.w, sum));
      }
      j.top_count = static_cast<int32_t>(wtop.size()) - j.top_first;
      wj.push_back(j);
    }
    const size_t o_top = sizeof(Walk3Job) * wj.size();
    const size_t o_out = o_top + sizeof(int4) * std::max<size_t>(wtop.size(), 1);
    const size_t bytes = o_out + 2 * sizeof(int4) * wj.size();
    if ((rc = ctx->f3_walk_buf.Reserve(bytes))) return rc;
    char* dw = ctx->f3_walk_buf.as<char>();
    std::vector<char> hw(o_out);
    std::memcpy(hw.data(), wj.data(), o_top);
    if (!wtop.empty()) std::memcpy(hw.data() + o_top, wtop.data(), sizeof(int4) * wtop.size());
    CSM_HIP(hipMemcpyAsync(dw, hw.data(), o_out, hipMemcpyHostToDevice, st));
    CSM_HIP(LaunchFast3dWalk(static_cast<int>(wj.size()), st, dsub, dpairs, dyaws,
                             ctx->f3_points.as<float>(), ctx->f3_low_points.as<float>(),
                             reinterpret_cast<const Walk3Job*>(dw),
                             reinterpret_cast<const int4*>(dw + o_top),
                             reinterpret_cast<int4*>(dw + o_out)));
    std::vector<int4> found(2 * wj.size());
    CSM_HIP(hipMemcpyAsync(found.data(), dw + o_out, 2 * sizeof(int4) * wj.size(),
                           hipMemcpyDeviceToHost, st));
    CSM_HIP(hipStreamSynchronize(st));
    for (size_t k = 0; k < walk.size(); ++k) {
      const int dp = walk[k];
      const Pair3Desc& d = pdesc[dp];
      if (!found[2 * k + 1].x) {
        // Unreachable (the maximum is a passing leaf's sum and the walk visits
        // every node whose sum reaches it): never return a leaf that is not
        // the reference's, the pair's result is void.
        (*stat_io)[dp] = CSM_ERANGE;
        continue;
      }
      const int4 f = found[2 * k];
      const unsigned long long mask = (1ull << d.key_shift) - 1;
      const unsigned long long sum = (*keys)[dp] >> d.key_shift;
      (*keys)[dp] = (sum << d.key_shift) | (~LeafId3(d, f.x, f.y, f.z, f.w) & mask);
    }
  }
  return CSM_OK;
}

}  // namespace

namespace {
// MatchBatch3's answer when the device flagged a yaw whose float rounding it
// could not decide after the flag check was deferred: the batch runs again
// with the check before the search.
constexpr int kRetryWithYawFlags = 0x7fff0001;

// defer_flags: the yaw build's flag count is read back with the results
// instead of synchronizing after the build (one synchronization less per
// batch; a flag, ~2^-16 per yaw, makes the caller rerun with the check).
int MatchBatch3(csm_context* ctx, csm_fast3d* const* submaps, int32_t num_submaps,
                const csm_node3d* nodes, int32_t num_nodes, const csm_pair3d* pairs,
                int64_t num_pairs, csm_result3d* results, bool defer_flags) {
  if (!ctx || num_pairs < 0 || (num_pairs > 0 && (!pairs || !results || !submaps || !nodes)))
    return CSM_EINVAL;
  // Matchers from any context on ctx's device (e.g. a single call's call
  // context searching its creator's matcher): their pyramids are read-only.
  for (int i = 0; i < num_submaps; ++i)
    if (!submaps[i] || submaps[i]->ctx->device != ctx->device) return CSM_EINVAL;
  using Clock = std::chrono::steady_clock;
  const bool prof3 = std::getenv("CSM_PROFILE3D") != nullptr;
  auto ht = Clock::now();
  double hms[6] = {0, 0, 0, 0, 0, 0};
  auto lap = [&](int k) {
    const auto now = Clock::now();
    hms[k] += std::chrono::duration<double, std::milli>(now - ht).count();
    ht = now;
  };
  // Nodes: offsets of the clouds some pair references (packed below).
  std::vector<int64_t> hoff(num_nodes, -1), loff(num_nodes, -1);
  std::vector<int32_t> used_nodes;
  int64_t nh = 0, nl = 0;
  for (int64_t i = 0; i < num_pairs; ++i) {
    results[i] = csm_result3d{};
    results[i].status = CSM_NO_MATCH;
    const csm_pair3d& p = pairs[i];
    if (p.submap < 0 || p.submap >= num_submaps || p.node < 0 || p.node >= num_nodes) {
      results[i].status = CSM_EINVAL;
      continue;
    }
    const csm_node3d& nd = nodes[p.node];
    if (nd.num_high_resolution < 0 || nd.num_low_resolution < 0 ||
        nd.num_high_resolution > kMax3dPoints || nd.histogram_size < 0) {
      results[i].status = nd.num_high_resolution > kMax3dPoints ? CSM_ERANGE : CSM_EINVAL;
      continue;
    }
    if (hoff[p.node] < 0) {
      hoff[p.node] = nh;
      loff[p.node] = nl;
      nh += nd.num_high_resolution;
      nl += nd.num_low_resolution;
      used_nodes.push_back(p.node);
    }
  }
  // One lock for the whole device section: the clouds uploaded here are read
  // by the search below.
  std::unique_lock<std::mutex> ctx_lock(ctx->mu);
  {
    int rc;
    if ((rc = EnsureDevice3(ctx))) return rc;
    // Matchers built on another stream: their builds finish first.
    for (int i = 0; i < num_submaps; ++i)
      if ((rc = WaitBuilt(submaps[i]->ready, submaps[i]->ctx->stream, ctx->stream))) return rc;
    if (!ctx->f3_copy_stream) {
      CSM_HIP(hipStreamCreateWithFlags(&ctx->f3_copy_stream, hipStreamNonBlocking));
      CSM_HIP(hipEventCreateWithFlags(&ctx->f3_points_ready, hipEventDisableTiming));
    }
    if ((rc = ctx->f3_host_points.Reserve(sizeof(float) * 3 * std::max<int64_t>(nh + nl, 1))))
      return rc;
    if ((rc = ctx->f3_points.Reserve(sizeof(float) * 3 * std::max<int64_t>(nh, 1)))) return rc;
    if ((rc = ctx->f3_low_points.Reserve(sizeof(float) * 3 * std::max<int64_t>(nl, 1)))) return rc;
  }
  float* const hstage = ctx->f3_host_points.as<float>();
  float* const lstage = hstage + 3 * nh;
  // Per node, in one pass: its clouds into the pinned staging and its
  // high-resolution cloud's largest norm (phase 1 below).
  std::vector<float> max_norm(num_nodes, 0.f);
  ParallelPairs(static_cast<int64_t>(used_nodes.size()), [&](int64_t j) {
    const csm_node3d& nd = nodes[used_nodes[j]];
    std::memcpy(hstage + 3 * hoff[used_nodes[j]], nd.high_resolution_xyz,
                sizeof(float) * 3 * nd.num_high_resolution);
    std::memcpy(lstage + 3 * loff[used_nodes[j]], nd.low_resolution_xyz,
                sizeof(float) * 3 * nd.num_low_resolution);
    max_norm[used_nodes[j]] = MaxNorm(nd);
  });
  if (nh > 0)
    CSM_HIP(hipMemcpyAsync(ctx->f3_points.ptr, hstage, sizeof(float) * 3 * nh, hipMemcpyHostToDevice,
                           ctx->f3_copy_stream));
  if (nl > 0)
    CSM_HIP(hipMemcpyAsync(ctx->f3_low_points.ptr, lstage, sizeof(float) * 3 * nl,
                           hipMemcpyHostToDevice, ctx->f3_copy_stream));
  CSM_HIP(hipEventRecord(ctx->f3_points_ready, ctx->f3_copy_stream));
  lap(0);
  // Phase 1 (host, parallel): per-node cloud extents, then search windows,
  // angular steps, initial yaws per pair.
  std::vector<PairPrep> prep(static_cast<size_t>(num_pairs));
  ParallelPairs(num_pairs, [&](int64_t i) {
    if (results[i].status != CSM_NO_MATCH) return;
    const csm_pair3d& p = pairs[i];
    const csm_node3d& nd = nodes[p.node];
    if (nd.histogram_size != static_cast<int32_t>(submaps[p.submap]->histogram.size()) ||
        nd.histogram_size > kMaxHistogram || (nd.histogram_size > 0 && !nd.histogram)) {
      prep[i].status = CSM_EINVAL;
      return;
    }
    PreparePair(submaps[p.submap], nd, p, max_norm[p.node], &prep[i]);
  });
  lap(1);
  if (prof3 && num_pairs > 0) {
    long hist[kMaxLevels3d] = {};
    for (int64_t i = 0; i < num_pairs; ++i)
      if (prep[i].status == CSM_OK) ++hist[prep[i].desc.root_level];
    const Submap3Desc& sd0 = submaps[pairs[0].submap]->desc;
    std::fprintf(stderr, "fast3d root levels:");
    for (int l = 0; l < kMaxLevels3d; ++l)
      if (hist[l]) std::fprintf(stderr, " L%d:%ld", l, hist[l]);
    std::fprintf(stderr, " | submap0 levels %d/%d bytes:", sd0.num_levels, sd0.search_levels);
    for (int l = 0; l < sd0.search_levels; ++l)
      std::fprintf(stderr, " %lld", static_cast<long long>(sd0.level[l].nx) * sd0.level[l].ny * sd0.level[l].nz);
    std::fprintf(stderr, " | pair0 w %d/%d T %d\n", prep[0].desc.wxy, prep[0].desc.wz,
                 prep[0].desc.top_nx * prep[0].desc.top_ny * prep[0].desc.top_nz);
  }
  // Phase 2 (device): rotational scores of every (pair, yaw); the passing
  // yaws (k, score) per pair come back compacted (yk, ys from yaw_src[i]).
  std::vector<int32_t> yk;
  std::vector<float> ys;
  unsigned kept = 0;
  const int32_t* dev_k = nullptr;
  const float* dev_s = nullptr;
  std::vector<int64_t> yaw_src(static_cast<size_t>(num_pairs), 0);
  {
    std::vector<float> hists;
    std::vector<int64_t> node_hist(num_nodes, -1), sub_hist(num_submaps, -1);
    std::vector<RotPair3Host> rp;
    std::vector<int64_t> rp_pair;
    int64_t total = 0;
    int max_yaws = 0;
    for (int64_t i = 0; i < num_pairs; ++i) {
      if (results[i].status != CSM_NO_MATCH || prep[i].status != CSM_OK) continue;
      const csm_pair3d& p = pairs[i];
      if (node_hist[p.node] < 0) {
        node_hist[p.node] = static_cast<int64_t>(hists.size());
        const csm_node3d& nd = nodes[p.node];
        hists.insert(hists.end(), nd.histogram, nd.histogram + nd.histogram_size);
      }
      if (sub_hist[p.submap] < 0) {
        sub_hist[p.submap] = static_cast<int64_t>(hists.size());
        const auto& h = submaps[p.submap]->histogram;
        hists.insert(hists.end(), h.begin(), h.end());
      }
      RotPair3Host r{};
      r.node_hist = static_cast<int32_t>(node_hist[p.node]);
      r.submap_hist = static_cast<int32_t>(sub_hist[p.submap]);
      r.size = nodes[p.node].histogram_size;
      r.window = prep[i].angular_window;
      r.step = prep[i].astep;
      r.yaw0 = prep[i].yaw0;
      r.out = total;
      r.min_score = submaps[p.submap]->options.min_rotational_score;
      total += 2 * r.window + 1;
      max_yaws = std::max(max_yaws, 2 * r.window + 1);
      rp.push_back(r);
      rp_pair.push_back(i);
    }
    std::vector<int2> range(rp.size());
    if (!rp.empty()) {
      int rc;
      hipStream_t st = ctx->stream;
      if ((rc = ctx->f3_items.Reserve(sizeof(RotPair3Host) * rp.size() +
                                      sizeof(float) * std::max<size_t>(hists.size(), 1))))
        return rc;
      // [scores | passing k | passing scores | ranges | cursor]
      if ((rc = ctx->f3_scores.Reserve(12 * total + sizeof(int2) * rp.size() + 16))) return rc;
      float* dscores = ctx->f3_scores.as<float>();
      int32_t* dk = reinterpret_cast<int32_t*>(dscores + total);
      float* ds = reinterpret_cast<float*>(dk + total);
      int2* drange = reinterpret_cast<int2*>(ds + total + (total & 1));
      unsigned* dcursor = reinterpret_cast<unsigned*>(drange + rp.size());
      RotPair3Host* drp = ctx->f3_items.as<RotPair3Host>();
      float* dh = reinterpret_cast<float*>(drp + rp.size());
      // Pinned staging both ways, one copy each: the pair records and
      // histograms up (contiguous on the device), the ranges and the cursor
      // (adjacent) back. Pageable copies cost ~25 us each, which dominated
      // a single call's latency (profiles/r6h/).
      const size_t up_bytes = sizeof(RotPair3Host) * rp.size() + sizeof(float) * hists.size();
      const size_t rb_bytes = sizeof(int2) * rp.size() + sizeof(unsigned);
      if ((rc = ctx->f3_up.Reserve(up_bytes)) || (rc = ctx->f3_rb.Reserve(rb_bytes))) return rc;
      std::memcpy(ctx->f3_up.ptr, rp.data(), sizeof(RotPair3Host) * rp.size());
      if (!hists.empty())
        std::memcpy(ctx->f3_up.as<char>() + sizeof(RotPair3Host) * rp.size(), hists.data(),
                    sizeof(float) * hists.size());
      CSM_HIP(hipMemcpyAsync(drp, ctx->f3_up.ptr, up_bytes, hipMemcpyHostToDevice, st));
      CSM_HIP(hipMemsetAsync(dcursor, 0, sizeof(unsigned), st));
      CSM_HIP(LaunchRotScores(drp, static_cast<int>(rp.size()), max_yaws, dh, dscores, st));
      CSM_HIP(LaunchYawCompact(drp, static_cast<int>(rp.size()), dscores, dcursor, drange, dk, ds,
                               st));
      CSM_HIP(hipMemcpyAsync(ctx->f3_rb.ptr, drange, rb_bytes, hipMemcpyDeviceToHost, st));
      CSM_HIP(hipStreamSynchronize(st));
      std::memcpy(range.data(), ctx->f3_rb.ptr, sizeof(int2) * rp.size());
      std::memcpy(&kept, ctx->f3_rb.as<char>() + sizeof(int2) * rp.size(), sizeof(unsigned));
      // The passing (k, score) lists stay on the device (f3_scores) for the
      // yaw_build kernel; the host reads them back with the results.
      dev_k = dk;
      dev_s = ds;
    }
    lap(2);
    for (size_t j = 0; j < rp_pair.size(); ++j) {
      const int64_t i = rp_pair[j];
      prep[i].num_yaws = range[j].y;
      yaw_src[i] = range[j].x;
      KeyBits(range[j].y, &prep[i]);
    }
  }
  lap(3);
  std::vector<Submap3Desc> sdesc(num_submaps);
  for (int i = 0; i < num_submaps; ++i) sdesc[i] = submaps[i]->desc;
  std::vector<Pair3Desc> pdesc;
  std::vector<int64_t> pair_of;  // device pair index -> input pair
  int ny = 0;
  // Pairs whose cloud fits the small-cloud build first, then the rest: two
  // launches over the two item ranges.
  int tier_end[kSearch3dTiers] = {};
  for (int pass = 0; pass < kSearch3dTiers; ++pass) {
  for (int64_t i = 0; i < num_pairs; ++i) {
    if (results[i].status != CSM_NO_MATCH) continue;
    if (prep[i].status != CSM_OK) {
      if (pass == 0) results[i].status = prep[i].status;
      continue;
    }
    if (pairs[i].min_score >= 1.f || nodes[pairs[i].node].num_high_resolution == 0) continue;
    if (Search3dTier(nodes[pairs[i].node].num_high_resolution) != pass) continue;
    Pair3Desc d = prep[i].desc;
    d.submap = pairs[i].submap;
    d.point_offset = hoff[pairs[i].node];
    d.low_offset = loff[pairs[i].node];
    d.yaw_begin = ny;
    d.num_yaws = prep[i].num_yaws;
    ny += d.num_yaws;
    pdesc.push_back(d);
    pair_of.push_back(i);
  }
  tier_end[pass] = ny;
  }
  const int np = static_cast<int>(pdesc.size());
  hipStream_t st = ctx->stream;
  if (np == 0) {
    CSM_HIP(hipStreamSynchronize(ctx->f3_copy_stream));  // staging is reused by the next batch
    return CSM_OK;
  }
  int rc;
  if ((rc = ctx->f3_pairs.Reserve(sizeof(Pair3Desc) * np + sizeof(Submap3Desc) * num_submaps)))
    return rc;
  if ((rc = ctx->f3_yaws.Reserve(sizeof(Yaw3Desc) * std::max(ny, 1)))) return rc;
  if ((rc = ctx->f3_best.Reserve(sizeof(unsigned long long) * np + sizeof(float) * np))) return rc;
  if ((rc = ctx->f3_best_hi.Reserve(sizeof(unsigned long long) * np))) return rc;
  if ((rc = ctx->f3_tie_count.Reserve(sizeof(int32_t)))) return rc;
  if ((rc = ctx->f3_ties.Reserve(sizeof(uint4)))) return rc;
  if ((rc = ctx->f3_status.Reserve(sizeof(int32_t) * np))) return rc;
  if ((rc = ctx->f3_counter.Reserve(16 + 16 * sizeof(unsigned long long)))) return rc;
  Pair3Desc* dpairs = ctx->f3_pairs.as<Pair3Desc>();
  Submap3Desc* dsub = reinterpret_cast<Submap3Desc*>(dpairs + np);
  unsigned long long* dbest = ctx->f3_best.as<unsigned long long>();
  float* dlow = reinterpret_cast<float*>(dbest + np);
  unsigned* dcounter = ctx->f3_counter.as<unsigned>();
  unsigned long long* dstats = reinterpret_cast<unsigned long long*>(
      reinterpret_cast<char*>(ctx->f3_counter.ptr) + 16);
  // Pair and submap descriptors (adjacent on the device) in one pinned
  // upload; the yaw-build records follow in the same staging buffer.
  const size_t desc_bytes = sizeof(Pair3Desc) * np + sizeof(Submap3Desc) * num_submaps;
  const size_t yb_at = (desc_bytes + 15) & ~size_t{15};
  if ((rc = ctx->f3_up.Reserve(yb_at + sizeof(YawBuild3) * np))) return rc;
  unsigned* dflag_count = nullptr;  // the yaw build's flag count (device)
  if (std::getenv("CSM_YAW_HOST_BUILD")) defer_flags = false;
  std::memcpy(ctx->f3_up.ptr, pdesc.data(), sizeof(Pair3Desc) * np);
  std::memcpy(ctx->f3_up.as<char>() + sizeof(Pair3Desc) * np, sdesc.data(),
              sizeof(Submap3Desc) * num_submaps);
  CSM_HIP(hipMemcpyAsync(dpairs, ctx->f3_up.ptr, desc_bytes, hipMemcpyHostToDevice, st));
  if (ny > 0) {
    // Discrete-scan poses of the yaws that pass, built on the device from the
    // compacted (k, score) lists; the few yaws whose float sin / cos rounding
    // the device cannot decide are rebuilt here with libm and patched in.
    std::vector<YawBuild3> yb(static_cast<size_t>(np));
    for (int dp = 0; dp < np; ++dp) {
      const PairPrep& pr = prep[pair_of[dp]];
      YawBuild3& b = yb[dp];
      b.siw = pr.submap_inv.w;
      b.six = pr.submap_inv.x;
      b.siy = pr.submap_inv.y;
      b.siz = pr.submap_inv.z;
      b.nqw = pr.node_q.w;
      b.nqx = pr.node_q.x;
      b.nqy = pr.node_q.y;
      b.nqz = pr.node_q.z;
      b.tx = pr.node_to_submap.t.x;
      b.ty = pr.node_to_submap.t.y;
      b.tz = pr.node_to_submap.t.z;
      b.astep = pr.astep;
      b.window = pr.angular_window;
      b.src = static_cast<int32_t>(yaw_src[pair_of[dp]]);
      b.yaw_begin = pdesc[dp].yaw_begin;
      b.num = pdesc[dp].num_yaws;
    }
    // f3_items held the rotational-score inputs, which are consumed (synced).
    // Layout [flag count (16 B) | flags | build records]: the count and the
    // first 64 flags come back in one pinned copy.
    if ((rc = ctx->f3_items.Reserve(16 + sizeof(YawFlag3) * kYawFlagCap + sizeof(YawBuild3) * np)))
      return rc;
    dflag_count = ctx->f3_items.as<unsigned>();
    YawFlag3* dflags = reinterpret_cast<YawFlag3*>(ctx->f3_items.as<char>() + 16);
    YawBuild3* dyb = reinterpret_cast<YawBuild3*>(dflags + kYawFlagCap);
    std::memcpy(ctx->f3_up.as<char>() + yb_at, yb.data(), sizeof(YawBuild3) * np);
    CSM_HIP(hipMemcpyAsync(dyb, ctx->f3_up.as<char>() + yb_at, sizeof(YawBuild3) * np,
                           hipMemcpyHostToDevice, st));
    CSM_HIP(hipMemsetAsync(dflag_count, 0, sizeof(unsigned), st));
    CSM_HIP(LaunchYawBuild(dyb, np, dev_k, dev_s, ctx->f3_yaws.as<Yaw3Desc>(), dflag_count, dflags,
                           st));
    unsigned nflag = 0;
    YawFlag3 flags[64];
    const size_t flag_rb = 16 + sizeof(flags);
    if (!defer_flags) {
      if ((rc = ctx->f3_rb.Reserve(flag_rb))) return rc;
      CSM_HIP(hipMemcpyAsync(ctx->f3_rb.ptr, dflag_count, flag_rb, hipMemcpyDeviceToHost, st));
      CSM_HIP(hipStreamSynchronize(st));
      std::memcpy(&nflag, ctx->f3_rb.ptr, sizeof(unsigned));
      std::memcpy(flags, ctx->f3_rb.as<char>() + 16, sizeof(flags));
      // CSM_YAW_HOST_BUILD (tests): the host path for every yaw.
      if (nflag > static_cast<unsigned>(kYawFlagCap) || std::getenv("CSM_YAW_HOST_BUILD")) {
        // More undecided roundings than the flag list holds (~2^-15 per value,
        // so only in batches of ~10^8 yaws): rebuild every yaw on the host.
        std::vector<int32_t> hk(std::max(kept, 1u));
        std::vector<float> hs(std::max(kept, 1u));
        CSM_HIP(hipMemcpyAsync(hk.data(), dev_k, sizeof(int32_t) * kept, hipMemcpyDeviceToHost, st));
        CSM_HIP(hipMemcpyAsync(hs.data(), dev_s, sizeof(float) * kept, hipMemcpyDeviceToHost, st));
        CSM_HIP(hipStreamSynchronize(st));
        if ((rc = ctx->f3_host_yaws.Reserve(sizeof(Yaw3Desc) * ny))) return rc;
        Yaw3Desc* hy = ctx->f3_host_yaws.as<Yaw3Desc>();
        ParallelPairs(np, [&](int64_t dp) {
          const int64_t i = pair_of[dp];
          BuildYaws(hk.data() + yaw_src[i], hs.data() + yaw_src[i], prep[i].num_yaws,
                    static_cast<int32_t>(dp), prep[i], hy + pdesc[dp].yaw_begin);
        });
        CSM_HIP(hipMemcpyAsync(ctx->f3_yaws.ptr, hy, sizeof(Yaw3Desc) * ny, hipMemcpyHostToDevice, st));
        nflag = 0;
      }
      if (nflag > 0) {
        std::vector<YawFlag3> all(flags, flags + std::min<unsigned>(nflag, 64));
        if (nflag > 64) {
          all.resize(nflag);
          CSM_HIP(hipMemcpy(all.data(), dflags, sizeof(YawFlag3) * nflag, hipMemcpyDeviceToHost));
        }
        if ((rc = ctx->f3_host_yaws.Reserve(sizeof(Yaw3Desc) * all.size()))) return rc;
        Yaw3Desc* hy = ctx->f3_host_yaws.as<Yaw3Desc>();
        for (size_t f = 0; f < all.size(); ++f) {
          const YawFlag3& fl = all[f];
          BuildYaws(&fl.k, &fl.score, 1, fl.dp, prep[pair_of[fl.dp]], &hy[f]);
          hy[f].yaw_id = fl.j;
          CSM_HIP(hipMemcpyAsync(ctx->f3_yaws.as<Yaw3Desc>() + pdesc[fl.dp].yaw_begin + fl.j, &hy[f],
                                 sizeof(Yaw3Desc), hipMemcpyHostToDevice, st));
        }
      }
    }  // !defer_flags
  }
  CSM_HIP(hipStreamWaitEvent(st, ctx->f3_points_ready, 0));
  {  // best keys, witnesses, statuses, claim counters and stats: one launch
    Segs3 z{};
    z.ptr[0] = dbest;
    z.bytes[0] = sizeof(unsigned long long) * np;
    z.ptr[1] = ctx->f3_best_hi.ptr;
    z.bytes[1] = sizeof(unsigned long long) * np;
    z.ptr[2] = ctx->f3_status.ptr;
    z.bytes[2] = sizeof(int32_t) * np;
    z.ptr[3] = ctx->f3_counter.ptr;
    z.bytes[3] = 16 + 16 * sizeof(unsigned long long);
    z.n = 4;
    CSM_HIP(LaunchSegments(z, nullptr, st));
  }
  lap(4);
  if ((rc = ctx->f3_spill.Reserve(SpillBytes3(ctx)))) return rc;
  if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev0, st));
  for (int tier = 0, b = 0; tier < kSearch3dTiers; b = tier_end[tier++])
    if (tier_end[tier] > b)
      CSM_HIP(LaunchFast3dSearch(tier, SearchGrid3(ctx, tier, tier_end[tier] - b), st, dsub, dpairs,
                                 ctx->f3_yaws.as<Yaw3Desc>(), b, tier_end[tier] - b,
                                 ctx->f3_points.as<float>(), ctx->f3_low_points.as<float>(),
                                 dcounter + tier, dbest, ctx->f3_status.as<int32_t>(), dstats,
                                 ctx->f3_spill.as<int4>(), ctx->f3_best_hi.as<unsigned long long>(),
                                 ctx->f3_ties.as<uint4>(), ctx->f3_tie_count.as<int32_t>()));
  if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev1, st));
  std::vector<unsigned long long> keys(np), keys_hi(np);
  std::vector<float> lows(np);
  std::vector<int32_t> stat(np);
  unsigned long long lookups = 0, prof[16] = {0};
  yk.resize(std::max(kept, 1u));
  ys.resize(std::max(kept, 1u));
  // The winners' low-resolution scores (the Result field) for the keys as
  // the search left them; redone below only if tie resolution moves a key.
  CSM_HIP(LaunchFast3dFinalize(np, st, dsub, dpairs, ctx->f3_yaws.as<Yaw3Desc>(),
                               ctx->f3_low_points.as<float>(), dbest, dlow));
  unsigned nflag = 0;
  {  // keys, witnesses, statuses, stats, the passing yaws, the low-resolution
     // scores and (deferred) the yaw flag count: packed on the device, one
     // pinned readback
    Segs3 g{};
    const bool rb_flags = defer_flags && dflag_count;
    void* src[8] = {dbest, ctx->f3_best_hi.ptr, ctx->f3_status.ptr, dstats,
                    const_cast<int32_t*>(dev_k), const_cast<float*>(dev_s), dlow,
                    rb_flags ? dflag_count : nullptr};
    const int64_t by[8] = {static_cast<int64_t>(sizeof(unsigned long long)) * np,
                           static_cast<int64_t>(sizeof(unsigned long long)) * np,
                           static_cast<int64_t>(sizeof(int32_t)) * np, static_cast<int64_t>(sizeof(prof)),
                           static_cast<int64_t>(sizeof(int32_t)) * kept,
                           static_cast<int64_t>(sizeof(float)) * kept,
                           static_cast<int64_t>(sizeof(float)) * np,
                           static_cast<int64_t>(sizeof(unsigned))};
    int64_t total = 0;
    for (int k = 0; k < 8; ++k) {
      g.ptr[k] = src[k];
      g.bytes[k] = src[k] ? by[k] : 0;
      total += g.bytes[k];
    }
    g.n = 8;
    if ((rc = ctx->f3_pack.Reserve(total)) || (rc = ctx->f3_rb.Reserve(total))) return rc;
    CSM_HIP(LaunchSegments(g, ctx->f3_pack.ptr, st));
    CSM_HIP(hipMemcpyAsync(ctx->f3_rb.ptr, ctx->f3_pack.ptr, total, hipMemcpyDeviceToHost, st));
    CSM_HIP(hipStreamSynchronize(st));
    const char* h = ctx->f3_rb.as<char>();
    void* dst[8] = {keys.data(), keys_hi.data(), stat.data(), prof, yk.data(), ys.data(),
                    lows.data(), &nflag};
    for (int k = 0; k < 8; ++k) {
      if (g.bytes[k]) std::memcpy(dst[k], h, g.bytes[k]);
      h += g.bytes[k];
    }
  }
  // Only with deferred flags; CSM_YAW_FORCE_RETRY (tests) takes the retry
  // path on every batch.
  if (nflag != 0 || (defer_flags && std::getenv("CSM_YAW_FORCE_RETRY"))) return kRetryWithYawFlags;
  // Exactly tied maxima: the reference's pick (ResolveTies3d), then the
  // winning leaves' low-resolution scores (the Result field).
  std::vector<int8_t> tie_code(np, CSM_TIE_NONE);
  {
    const std::vector<unsigned long long> before = keys;
    if ((rc = ResolveTies3d(ctx, submaps, pdesc, &stat, keys_hi, &keys, &tie_code))) return rc;
    if (keys != before) {
      CSM_HIP(hipMemcpyAsync(dbest, keys.data(), sizeof(unsigned long long) * np,
                             hipMemcpyHostToDevice, st));
      CSM_HIP(LaunchFast3dFinalize(np, st, dsub, dpairs, ctx->f3_yaws.as<Yaw3Desc>(),
                                   ctx->f3_low_points.as<float>(), dbest, dlow));
      if ((rc = ctx->f3_rb.Reserve(sizeof(float) * np))) return rc;
      CSM_HIP(hipMemcpyAsync(ctx->f3_rb.ptr, dlow, sizeof(float) * np, hipMemcpyDeviceToHost, st));
      CSM_HIP(hipStreamSynchronize(st));
      std::memcpy(lows.data(), ctx->f3_rb.ptr, sizeof(float) * np);
    }
  }
  if (ctx->timing) {
    float ms = 0.f;
    CSM_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->t.fast3d_kernel_ms += ms;
    ctx->t.fast3d_launches += 1;
    lookups = prof[0];
    ctx->t.fast3d_lookups += static_cast<double>(lookups);
    ctx->t.stack_high_water =
        std::max<int64_t>(ctx->t.stack_high_water, static_cast<int64_t>(prof[kStat3dHighWater]));
    for (int dp = 0; dp < np; ++dp) ctx->t.search_errors += stat[dp] < 0 ? 1 : 0;
    if (std::getenv("CSM_PROFILE3D"))
      std::fprintf(stderr,
                   "fast3d phases (Mcycles, thread 0 sums): item+discretize %.1f top-copy %.1f "
                   "box %.1f cells %.1f roots %.1f sort %.1f dfs %.1f leaf %.1f | batches %llu "
                   "leaves %llu items %d roots-scored %llu roots-kept %llu\n",
                   prof[1] / 1e6, prof[8] / 1e6, prof[9] / 1e6, prof[10] / 1e6, prof[2] / 1e6,
                   prof[3] / 1e6, prof[4] / 1e6, prof[5] / 1e6, prof[6], prof[7], ny, prof[11],
                   prof[12]);
  }
  lap(5);
  if (prof3)
    std::fprintf(stderr,
                 "fast3d host (ms): pack %.1f phase1 %.1f rotscores %.1f yaws %.1f descs+upload %.1f "
                 "search+download %.1f\n",
                 hms[0], hms[1], hms[2], hms[3], hms[4], hms[5]);
  // Decode (GetPoseFromCandidate :369-375, Result :193-198).
  for (int dp = 0; dp < np; ++dp) {
    const int64_t i = pair_of[dp];
    const Pair3Desc& d = pdesc[dp];
    if (stat[dp] < 0) {
      results[i].status = stat[dp];
      continue;
    }
    const unsigned long long key = keys[dp];
    if (key == 0) continue;
    const unsigned long long id = ~key & ((1ull << d.key_shift) - 1);
    const int sum = static_cast<int>(key >> d.key_shift);
    const int oz = static_cast<int>(id & ((1ull << d.bits_z) - 1)) - d.wz;
    const int oy = static_cast<int>((id >> d.bits_z) & ((1ull << d.bits_xy) - 1)) - d.wxy;
    const int ox =
        static_cast<int>((id >> (d.bits_z + d.bits_xy)) & ((1ull << d.bits_xy) - 1)) - d.wxy;
    const int yaw = static_cast<int>(id >> (d.bits_z + 2 * d.bits_xy));
    // The winning discrete scan, rebuilt exactly as the device built it.
    Yaw3Desc y;
    BuildYaws(yk.data() + yaw_src[i] + yaw, ys.data() + yaw_src[i] + yaw, 1, dp, prep[i], &y);
    const float res = submaps[d.submap]->resolution;
    const V3 t0 = Rotate(Q4{1.f, 0.f, 0.f, 0.f}, V3{y.tx, y.ty, y.tz});
    const V3 t{t0.x + res * static_cast<float>(ox), t0.y + res * static_cast<float>(oy),
               t0.z + res * static_cast<float>(oz)};
    results[i].status = CSM_OK;
    results[i].score = SumToProbability(sum, d.num_points);
    results[i].pose = ToPose(t, Q4{y.nw, y.nx, y.ny, y.nz});
    results[i].rotational_score = y.rotational_score;
    results[i].low_resolution_score = lows[dp];
    results[i].tie = tie_code[dp];
  }
  return CSM_OK;
}

}  // namespace

int csm_fast3d_match_batch(csm_context* ctx, csm_fast3d* const* submaps, int32_t num_submaps,
                           const csm_node3d* nodes, int32_t num_nodes, const csm_pair3d* pairs,
                           int64_t num_pairs, csm_result3d* results) {
  const int rc = MatchBatch3(ctx, submaps, num_submaps, nodes, num_nodes, pairs, num_pairs, results,
                             /*defer_flags=*/true);
  if (rc != kRetryWithYawFlags) return rc;
  return MatchBatch3(ctx, submaps, num_submaps, nodes, num_nodes, pairs, num_pairs, results, false);
}

namespace {

// One single Match / MatchFullSubmap call waiting in its owner's queue.
struct SingleReq3 {
  const csm_fast3d* m;
  csm_pair3d pair;
  const csm_node3d* node;
  csm_result3d res;
  int rc;
  bool done;
};

constexpr int kCoalesceCap3 = 512;  // pairs per coalesced batch

// Searches queued single calls as one batch on a call context of `owner`:
// the distinct matchers as the batch's submaps, one node per request.
int RunSingleBatch3(csm_context* owner, const std::vector<SingleReq3*>& reqs) {
  csm::CallContext cc(owner);
  csm_context* ctx = cc.get();
  if (!ctx) return CSM_EHIP;
  std::vector<csm_fast3d*> subs;
  std::map<const csm_fast3d*, int> slot;
  std::vector<csm_node3d> nodes(reqs.size());
  std::vector<csm_pair3d> pairs(reqs.size());
  for (size_t k = 0; k < reqs.size(); ++k) {
    auto it = slot.find(reqs[k]->m);
    if (it == slot.end()) {
      it = slot.emplace(reqs[k]->m, static_cast<int>(subs.size())).first;
      subs.push_back(const_cast<csm_fast3d*>(reqs[k]->m));
    }
    nodes[k] = *reqs[k]->node;
    pairs[k] = reqs[k]->pair;
    pairs[k].submap = it->second;
    pairs[k].node = static_cast<int32_t>(k);
  }
  std::vector<csm_result3d> res(reqs.size());
  const int rc = csm_fast3d_match_batch(ctx, subs.data(), static_cast<int32_t>(subs.size()), nodes.data(),
                                        static_cast<int32_t>(nodes.size()), pairs.data(),
                                        static_cast<int64_t>(pairs.size()), res.data());
  if (rc < 0) return rc;
  for (size_t k = 0; k < reqs.size(); ++k) reqs[k]->res = res[k];
  return CSM_OK;
}

// Concurrent single 3D calls on one owner context are coalesced (as in 2D,
// csm_host.cc SingleMatch): each queues its pair; a caller that finds fewer
// than CSM_COALESCE_LEADERS3 (2) batches running becomes a leader, waits up
// to CSM_COALESCE_WINDOW_US3 (300 us) until the queue holds its share of the
// callers, ceil(callers / leaders), searches the queue as one batch and
// wakes the callers it served. `callers` is the owner's recent high-water
// mark of calls in flight (decaying by one per batch), so with T threads
// calling back to back two batches of about T / 2 alternate, one searching
// while the other's callers return and queue again. A 3D pair costs a few
// microseconds of device time against ~0.3 ms of fixed latency per batch
// (the pipeline's launches, copies and synchronizations), so batch size,
// not device time, sets the single-call rate: the previous rule (wait for
// as many callers as the previous batch had, 3 leaders) settled at ~2
// pairs per batch (profiles/r6h/). A pair's result does not depend on its
// batch. CSM_SINGLE_COALESCE=0: each call alone on its own call context.
int SingleMatch3(const csm_fast3d* m, const csm_pair3d& pair, const csm_node3d* node,
                 csm_result3d* result) {
  csm_context* owner = m->ctx;
  SingleReq3 r{m, pair, node, csm_result3d{}, CSM_OK, false};
  static const bool coalesce = [] {
    const char* e = std::getenv("CSM_SINGLE_COALESCE");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  static const int leaders = [] {
    const char* e = std::getenv("CSM_COALESCE_LEADERS3");
    return e ? std::max(1, std::atoi(e)) : 2;
  }();
  static const int window_us = [] {
    const char* e = std::getenv("CSM_COALESCE_WINDOW_US3");
    return e ? std::max(0, std::atoi(e)) : 300;
  }();
  if (!coalesce) {
    std::vector<SingleReq3*> one{&r};
    try {
      r.rc = RunSingleBatch3(owner, one);
    } catch (...) {  // no exception crosses the C-ABI
      r.rc = CSM_ENOMEM;
    }
  } else {
    std::unique_lock<std::mutex> lk(owner->co_mu);
    owner->co3_queue.push_back(&r);
    owner->co3_callers = std::max(owner->co3_callers, ++owner->co3_in_flight);
    owner->co_cv.notify_all();
    while (!r.done) {
      const bool queued = std::find(owner->co3_queue.begin(), owner->co3_queue.end(), &r) !=
                          owner->co3_queue.end();
      if (queued && owner->co3_leaders < leaders) {
        ++owner->co3_leaders;
        owner->co3_callers = std::max(owner->co3_in_flight, owner->co3_callers - 1);
        const size_t want = static_cast<size_t>((owner->co3_callers + leaders - 1) / leaders);
        const auto deadline = std::chrono::steady_clock::now() + std::chrono::microseconds(window_us);
        while (owner->co3_queue.size() < want &&
               owner->co_cv.wait_until(lk, deadline) != std::cv_status::timeout) {
        }
        const size_t take_n = std::min<size_t>(owner->co3_queue.size(), kCoalesceCap3);
        std::vector<SingleReq3*> take;
        for (size_t i = 0; i < take_n; ++i) take.push_back(static_cast<SingleReq3*>(owner->co3_queue[i]));
        owner->co3_queue.erase(owner->co3_queue.begin(), owner->co3_queue.begin() + take_n);
        owner->co3_last_batch = static_cast<int>(take_n);
        lk.unlock();
        int rc;  // as in 2D: every request taken is answered, whatever the batch throws
        try {
          rc = RunSingleBatch3(owner, take);
        } catch (...) {
          rc = CSM_ENOMEM;
        }
        lk.lock();
        for (SingleReq3* q : take) {
          q->rc = rc;
          q->done = true;
        }
        --owner->co3_leaders;
        owner->co_cv.notify_all();
      } else {
        owner->co_cv.wait(lk);
      }
    }
    --owner->co3_in_flight;
  }
  *result = r.res;
  if (r.rc < 0) return r.rc;
  return result->status;
}

}  // namespace

int csm_fast3d_match(const csm_fast3d* m, const csm_pose3d* node_pose,
                     const csm_pose3d* submap_pose, const csm_node3d* node, float min_score,
                     csm_result3d* result) {
  if (!m || !node_pose || !submap_pose || !node || !result) return CSM_EINVAL;
  csm_pair3d p{};
  p.submap = 0;
  p.node = 0;
  p.full_submap = 0;
  p.min_score = min_score;
  p.node_pose = *node_pose;
  p.submap_pose = *submap_pose;
  return SingleMatch3(m, p, node, result);
}

int csm_fast3d_match_full_submap(const csm_fast3d* m, const double* node_rotation,
                                 const double* submap_rotation, const csm_node3d* node,
                                 float min_score, csm_result3d* result) {
  if (!m || !node_rotation || !submap_rotation || !node || !result) return CSM_EINVAL;
  csm_pair3d p{};
  p.full_submap = 1;
  p.min_score = min_score;
  for (int k = 0; k < 4; ++k) {
    p.node_pose.q[k] = node_rotation[k];
    p.submap_pose.q[k] = submap_rotation[k];
  }
  return SingleMatch3(m, p, node, result);
}
