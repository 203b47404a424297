// CeresScanMatcher2D::Match (mapping/internal/2d/scan_matching/
// ceres_scan_matcher_2d.cc:64-105), batched on gfx950: the refinement
// ConstraintBuilder2D::ComputeConstraint runs on every accepted branch-and-bound
// match (constraint_builder_2d.cc:245-249).
//
// One workgroup per pair. The residuals are the reference's three blocks:
// OccupiedSpaceCostFunction2D (occupied_space_cost_function_2d.cc:30-91: a
// ceres::BiCubicInterpolator over the submap's correspondence costs, padded by
// kPadding = INT_MAX / 4 cells of max cost, scaled by w / sqrt(N)), the
// translation delta to the match and the rotation delta to its angle. Each
// iteration the workgroup evaluates the N residual rows and their analytic
// Jacobian (what AutoDiff computes) in double, reduces J^T J and J^T r, and
// every lane takes the same Levenberg-Marquardt trust-region step with Ceres
// 1.13's defaults (Jacobi scaling from the initial Jacobian, radius 1e4,
// diagonal clamp [1e-6, 1e32], min relative decrease 1e-3, tolerances 1e-6 /
// 1e-10 / 1e-8, non-monotonic steps as pose_graph.lua:35 sets them). Ceres is
// absent from this image: the solver follows oracle/ceres2d.cc's restatement,
// which the reference's ceres_scan_matcher_2d_test.cc pins.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cmath>
#include <vector>

#include "ceres_lm.h"
#include "csm_internal.h"

namespace csm {
namespace {

constexpr int kRefineThreads = 256;
constexpr int kPadding = INT_MAX / 4;

struct RefineDesc {
  const float* cost;  // num_y_cells x num_x_cells correspondence costs
  double max_x, max_y, resolution;
  int32_t nx, ny;
  double max_cost;
  int64_t point_offset;
  int32_t n;
  double initial[3], target[2];
};

struct RefineOpts {
  double occupied, wt, wr;
  int max_iterations;
  int nonmonotonic;  // ceres_solver_options.use_nonmonotonic_steps
};

__device__ __forceinline__ double CostAt(const RefineDesc& d, int row, int col) {
  if (row < kPadding || col < kPadding || row >= d.ny + kPadding || col >= d.nx + kPadding)
    return d.max_cost;
  return static_cast<double>(d.cost[static_cast<int64_t>(row - kPadding) * d.nx + (col - kPadding)]);
}

// ceres::CubicHermiteSpline.
__device__ __forceinline__ void Hermite(double p0, double p1, double p2, double p3, double x,
                                        double* f, double* dfdx) {
  const double a = 0.5 * (-p0 + 3.0 * p1 - 3.0 * p2 + p3);
  const double b = 0.5 * (2.0 * p0 - 5.0 * p1 + 4.0 * p2 - p3);
  const double c = 0.5 * (-p0 + p2);
  const double d = p1;
  *f = d + x * (c + x * (b + x * a));
  if (dfdx) *dfdx = c + x * (2.0 * b + 3.0 * a * x);
}

// Residual row i (and its Jacobian row when J != nullptr) at pose x.
__device__ void Row(const RefineDesc& d, const float* pts, double scale, const double* x, double s,
                    double c, int i, double* r, double* J) {
  const double px = static_cast<double>(pts[3 * i]), py = static_cast<double>(pts[3 * i + 1]);
  const double wx = c * px + (-s * py + x[0] * 1.);
  const double wy = s * px + (c * py + x[1] * 1.);
  const double rr = (d.max_x - wx) / d.resolution - 0.5 + static_cast<double>(kPadding);
  const double cc = (d.max_y - wy) / d.resolution - 0.5 + static_cast<double>(kPadding);
  const int row = static_cast<int>(floor(rr)), col = static_cast<int>(floor(cc));
  double fr[4], dfr[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int q = row - 1 + k;
    Hermite(CostAt(d, q, col - 1), CostAt(d, q, col), CostAt(d, q, col + 1), CostAt(d, q, col + 2),
            cc - col, &fr[k], &dfr[k]);
  }
  double f, dfdr, dfdc;
  Hermite(fr[0], fr[1], fr[2], fr[3], rr - row, &f, &dfdr);
  Hermite(dfr[0], dfr[1], dfr[2], dfr[3], rr - row, &dfdc, nullptr);
  *r = scale * f;
  if (J) {
    const double dwx_dt = -s * px - c * py, dwy_dt = c * px - s * py;
    J[0] = scale * (dfdr * (-1. / d.resolution));
    J[1] = scale * (dfdc * (-1. / d.resolution));
    J[2] = scale * (dfdr * (-dwx_dt / d.resolution) + dfdc * (-dwy_dt / d.resolution));
  }
}

__device__ __forceinline__ double WaveSumD(double v) {
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

// Sums k doubles per thread over the workgroup; every thread gets the totals.
template <int K>
__device__ void BlockSum(double* v, double (*red)[K]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double t = WaveSumD(v[k]);
    if (lane == 0) red[w][k] = t;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double t = 0.;
    for (int q = 0; q < kRefineThreads / 64; ++q) t += red[q][k];
    v[k] = t;
  }
  __syncthreads();
}

__device__ bool Solve3(double M[3][4], double out[3]) {
  for (int c = 0; c < 3; ++c) {
    int piv = c;
    for (int i = c + 1; i < 3; ++i)
      if (fabs(M[i][c]) > fabs(M[piv][c])) piv = i;
    if (M[piv][c] == 0.) return false;
    for (int j = 0; j < 4; ++j) {
      const double t = M[c][j];
      M[c][j] = M[piv][j];
      M[piv][j] = t;
    }
    for (int i = c + 1; i < 3; ++i) {
      const double f = M[i][c] / M[c][c];
      for (int j = c; j < 4; ++j) M[i][j] -= f * M[c][j];
    }
  }
  for (int i = 2; i >= 0; --i) {
    double v = M[i][3];
    for (int j = i + 1; j < 3; ++j) v -= M[i][j] * out[j];
    out[i] = v / M[i][i];
  }
  return true;
}

// Pass over the N occupied-space rows plus the 3 delta rows at pose x:
// out[0] = sum r^2, and with jac, out[1..6] = Ju^T Ju (upper), out[7..9] = Ju^T r.
template <bool kJac>
__device__ void Pass(const RefineDesc& d, const float* pts, double scale, const RefineOpts& o,
                     const double* x, double* out, double (*red)[10]) {
  const double s = sin(x[2]), c = cos(x[2]);
  double acc[10] = {0., 0., 0., 0., 0., 0., 0., 0., 0., 0.};
  for (int i = threadIdx.x; i < d.n + 3; i += kRefineThreads) {
    double r, J[3] = {0., 0., 0.};
    if (i < d.n) {
      Row(d, pts, scale, x, s, c, i, &r, kJac ? J : nullptr);
    } else if (i == d.n) {
      r = o.wt * (x[0] - d.target[0]);
      J[0] = o.wt;
    } else if (i == d.n + 1) {
      r = o.wt * (x[1] - d.target[1]);
      J[1] = o.wt;
    } else {
      r = o.wr * (x[2] - d.initial[2]);
      J[2] = o.wr;
    }
    acc[0] += r * r;
    if (kJac) {
      acc[1] += J[0] * J[0];
      acc[2] += J[0] * J[1];
      acc[3] += J[0] * J[2];
      acc[4] += J[1] * J[1];
      acc[5] += J[1] * J[2];
      acc[6] += J[2] * J[2];
      acc[7] += J[0] * r;
      acc[8] += J[1] * r;
      acc[9] += J[2] * r;
    }
  }
  BlockSum<10>(acc, red);
  for (int k = 0; k < 10; ++k) out[k] = acc[k];
}

// The minimizer loop is Ceres' TrustRegionMinimizer::Minimize: LM step
// (invalid when the model decrease is not positive), candidate cost,
// parameter then function tolerance (both end the solve without taking the
// candidate), acceptance by step quality > 1e-3; the lowest-cost accepted
// point is returned. Every thread runs the (scalar) step logic on the same
// block-reduced sums, so all of them hold the same state.
__global__ void __launch_bounds__(kRefineThreads)
ceres2d_refine(const RefineDesc* __restrict__ items, const float* __restrict__ points,
               RefineOpts o, double* __restrict__ out_pose, int32_t* __restrict__ out_iters) {
  __shared__ double red[kRefineThreads / 64][10];
  const RefineDesc d = items[blockIdx.x];
  const float* pts = points + 3 * d.point_offset;
  const double scale = o.occupied / sqrt(static_cast<double>(d.n));
  double x[3] = {d.initial[0], d.initial[1], d.initial[2]};
  double S[10];
  Pass<true>(d, pts, scale, o, x, S, red);
  double cost = 0.5 * S[0];
  // Jacobi scaling from the initial Jacobian.
  const double js[3] = {1. / (1. + sqrt(S[1])), 1. / (1. + sqrt(S[4])), 1. / (1. + sqrt(S[6]))};
  StepEvaluator ev(cost, o.nonmonotonic != 0);
  double best[3] = {x[0], x[1], x[2]}, best_cost = cost;
  LmRadius lm;
  int iter = 0, invalid = 0;
  auto gradient_small = [&]() {
    return fmax(fabs(S[7]), fmax(fabs(S[8]), fabs(S[9]))) <= 1e-10;
  };
  bool go = o.max_iterations > 0 && !gradient_small();
  while (go) {
    ++iter;
    const double Au[3][3] = {{S[1], S[2], S[3]}, {S[2], S[4], S[5]}, {S[3], S[5], S[6]}};
    double A[3][3], g[3], M[3][4], ds[3] = {0., 0., 0.};
    for (int a = 0; a < 3; ++a) {
      g[a] = S[7 + a] * js[a];
      for (int b = 0; b < 3; ++b) A[a][b] = Au[a][b] * js[a] * js[b];
    }
    for (int a = 0; a < 3; ++a) {
      for (int b = 0; b < 3; ++b) M[a][b] = A[a][b];
      M[a][a] += fmin(fmax(A[a][a], 1e-6), 1e32) / lm.radius;
      M[a][3] = -g[a];
    }
    const bool solved = Solve3(M, ds);
    double gd = 0., dad = 0.;
    for (int a = 0; a < 3; ++a) {
      gd += g[a] * ds[a];
      for (int b = 0; b < 3; ++b) dad += ds[a] * A[a][b] * ds[b];
    }
    const double model = -(gd + 0.5 * dad);
    if (!solved || !(model > 0.)) {
      if (++invalid > 5) break;  // HandleInvalidStep: LM rejects the step
      lm.Rejected();
    } else {
      invalid = 0;
      double xn[3], step_norm = 0., x_norm = 0.;
      for (int a = 0; a < 3; ++a) {
        const double step = ds[a] * js[a];
        xn[a] = x[a] + step;
        step_norm += step * step;
        x_norm += x[a] * x[a];
      }
      double T[10];
      Pass<false>(d, pts, scale, o, xn, T, red);
      const double new_cost = 0.5 * T[0];
      if (sqrt(step_norm) <= (sqrt(x_norm) + 1e-8) * 1e-8) break;  // parameter tolerance
      if (fabs(cost - new_cost) <= 1e-6 * cost) break;             // function tolerance
      const double quality = ev.Quality(new_cost, model);
      if (quality > 1e-3) {
        for (int a = 0; a < 3; ++a) x[a] = xn[a];
        Pass<true>(d, pts, scale, o, x, S, red);
        cost = 0.5 * S[0];
        lm.Accepted(quality);
        ev.Accepted(new_cost, model);
        if (cost < best_cost) {
          best_cost = cost;
          for (int a = 0; a < 3; ++a) best[a] = x[a];
        }
      } else {
        lm.Rejected();
      }
    }
    go = iter < o.max_iterations && lm.radius >= 1e-32 && !gradient_small();
  }
  if (threadIdx.x == 0) {
    out_pose[3 * blockIdx.x + 0] = best[0];
    out_pose[3 * blockIdx.x + 1] = best[1];
    out_pose[3 * blockIdx.x + 2] = best[2];
    if (out_iters) out_iters[blockIdx.x] = iter;
  }
}

}  // namespace
}  // namespace csm

extern "C" {

int csm_ceres2d_refine_batch(csm_context* ctx, csm_fast2d* const* submaps, int32_t num_submaps,
                             const csm_scan_set* scans, const csm_refine2d* items, int64_t n,
                             const csm_ceres2d_options* options, csm_pose2d* out,
                             int32_t* iterations) {
  using namespace csm;
  if (!ctx || !scans || !options || (n > 0 && (!items || !out || !submaps))) return CSM_EINVAL;
  if (n == 0) return CSM_OK;
  if (!(options->occupied_space_weight > 0.) || !(options->translation_weight > 0.) ||
      !(options->rotation_weight > 0.) || options->max_num_iterations < 0)
    return CSM_EINVAL;  // the reference CHECKs the weights (ceres_scan_matcher_2d.cc:74-97)
  if (n > 0x7fffffff) return CSM_ERANGE;
  const int64_t num_scans = static_cast<int64_t>(scans->offsets.size()) - 1;
  std::vector<RefineDesc> desc(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    const csm_refine2d& it = items[i];
    if (it.submap < 0 || it.submap >= num_submaps || !submaps[it.submap] || it.scan < 0 ||
        it.scan >= num_scans)
      return CSM_EINVAL;
    const csm_fast2d* m = submaps[it.submap];
    if (m->ctx != ctx || !m->cost.ptr) return CSM_EINVAL;
    RefineDesc& d = desc[i];
    d.cost = m->cost.as<float>();
    d.max_x = m->limits.max_x;
    d.max_y = m->limits.max_y;
    d.resolution = m->limits.resolution;
    d.nx = m->limits.num_x_cells;
    d.ny = m->limits.num_y_cells;
    d.max_cost = static_cast<double>(m->max_cc);
    d.point_offset = scans->offsets[it.scan];
    d.n = static_cast<int32_t>(scans->offsets[it.scan + 1] - scans->offsets[it.scan]);
    if (d.n <= 0) return CSM_EINVAL;
    d.initial[0] = it.initial.x;
    d.initial[1] = it.initial.y;
    d.initial[2] = it.initial.theta;
    d.target[0] = it.target_x;
    d.target[1] = it.target_y;
  }
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CSM_EHIP;
  int rc;
  if ((rc = ctx->cr_items.Reserve(sizeof(RefineDesc) * n))) return rc;
  if ((rc = ctx->cr_out.Reserve(sizeof(double) * 3 * n + sizeof(int32_t) * n))) return rc;
  hipStream_t st = ctx->stream;
  CSM_HIP(hipMemcpyAsync(ctx->cr_items.ptr, desc.data(), sizeof(RefineDesc) * n,
                         hipMemcpyHostToDevice, st));
  const RefineOpts o{options->occupied_space_weight, options->translation_weight,
                     options->rotation_weight, options->max_num_iterations,
                     options->use_nonmonotonic_steps ? 1 : 0};
  double* dpose = ctx->cr_out.as<double>();
  int32_t* diters = reinterpret_cast<int32_t*>(dpose + 3 * n);
  hipLaunchKernelGGL(ceres2d_refine, dim3(static_cast<unsigned>(n)), dim3(kRefineThreads), 0, st,
                     ctx->cr_items.as<RefineDesc>(), scans->points.as<float>(), o, dpose, diters);
  CSM_HIP(hipGetLastError());
  std::vector<double> pose(3 * static_cast<size_t>(n));
  CSM_HIP(hipMemcpyAsync(pose.data(), dpose, sizeof(double) * 3 * n, hipMemcpyDeviceToHost, st));
  if (iterations)
    CSM_HIP(hipMemcpyAsync(iterations, diters, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  for (int64_t i = 0; i < n; ++i) out[i] = csm_pose2d{pose[3 * i], pose[3 * i + 1], pose[3 * i + 2]};
  return CSM_OK;
}

}  // extern "C"
