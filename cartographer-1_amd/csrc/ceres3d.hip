// CeresScanMatcher3D::Match (mapping/internal/3d/scan_matching/
// ceres_scan_matcher_3d.cc:84-160), batched on gfx950: the refinement
// ConstraintBuilder3D::ComputeConstraint runs on every accepted match
// (constraint_builder_3d.cc:264-275).
//
// One workgroup per match. Residuals: OccupiedSpaceCostFunction3D for the
// high-resolution cloud in the high-resolution HybridGrid and the
// low-resolution cloud in the low-resolution grid (InterpolatedGrid's
// smooth-step tricubic interpolation, interpolated_grid.h:50-150), the
// translation delta to the match and the rotation delta vec(target^-1 q).
// The pose is (t, q) with ceres::QuaternionParameterization: Jacobians are
// taken in the 6-dimensional tangent space and a step updates
// q <- (cos|d|, sin|d|/|d| d) * q. Each iteration the workgroup reduces
// J^T J (6 x 6) and J^T r in double and one lane takes a Levenberg-Marquardt
// trust-region step with Ceres' defaults, as oracle/ceres3d.cc restates
// (parity with Ceres unpinned).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "ceres_lm.h"
#include "csm_internal.h"

namespace csm {
namespace {

constexpr int kR3Threads = 256;
constexpr int kSums = 1 + 21 + 6;  // cost, upper J^T J, J^T r

struct GridView3 {
  const float* prob;
  Brick3 b;
  float res;
};

struct Refine3Desc {
  GridView3 grid[2];
  int64_t offset[2];  // into the points buffer (points)
  int32_t n[2];
  double t[3], q[4], target[3];
};

struct Refine3Opts {
  double w0, w1, wt, wr;
  int max_iterations;
  int nonmonotonic;  // ceres_solver_options.use_nonmonotonic_steps
};

__device__ __forceinline__ double Prob(const GridView3& g, int x, int y, int z) {
  const int lx = x - g.b.ox, ly = y - g.b.oy, lz = z - g.b.oz;
  if (static_cast<unsigned>(lx) >= static_cast<unsigned>(g.b.nx) ||
      static_cast<unsigned>(ly) >= static_cast<unsigned>(g.b.ny) ||
      static_cast<unsigned>(lz) >= static_cast<unsigned>(g.b.nz))
    return static_cast<double>(0.1f);  // unknown: kMinProbability
  return static_cast<double>(g.prob[(static_cast<int64_t>(lz) * g.b.ny + ly) * g.b.nx + lx]);
}

// HybridGridBase::GetCellIndex: lround(p / res) in float.
__device__ __forceinline__ int CellF(float v, float res) {
  return static_cast<int>(roundf(__fdiv_rn(v, res)));
}

struct StepF {
  double t, tt, ttt;
  __device__ double f(double a, double b) const { return (a - b) * ttt * 2. + (b - a) * tt * 3. + a; }
  __device__ double dt(double a, double b) const { return (a - b) * 6. * tt + (b - a) * 6. * t; }
  __device__ double da() const { return 2. * ttt - 3. * tt + 1.; }
  __device__ double db() const { return -2. * ttt + 3. * tt; }
};

// InterpolatedGrid::GetInterpolatedValue and its gradient.
__device__ double Interpolate(const GridView3& g, double x, double y, double z, double* grad) {
  const float res = g.res;
  const float fx = static_cast<float>(x), fy = static_cast<float>(y), fz = static_cast<float>(z);
  float cx = __fmul_rn(static_cast<float>(CellF(fx, res)), res);
  float cy = __fmul_rn(static_cast<float>(CellF(fy, res)), res);
  float cz = __fmul_rn(static_cast<float>(CellF(fz, res)), res);
  if (cx > x) cx = __fsub_rn(cx, res);
  if (cy > y) cy = __fsub_rn(cy, res);
  if (cz > z) cz = __fsub_rn(cz, res);
  const double x1 = cx, y1 = cy, z1 = cz;
  const double x2 = __fadd_rn(cx, res), y2 = __fadd_rn(cy, res), z2 = __fadd_rn(cz, res);
  const int ix = CellF(cx, res), iy = CellF(cy, res), iz = CellF(cz, res);
  const double q111 = Prob(g, ix, iy, iz), q112 = Prob(g, ix, iy, iz + 1);
  const double q121 = Prob(g, ix, iy + 1, iz), q122 = Prob(g, ix, iy + 1, iz + 1);
  const double q211 = Prob(g, ix + 1, iy, iz), q212 = Prob(g, ix + 1, iy, iz + 1);
  const double q221 = Prob(g, ix + 1, iy + 1, iz), q222 = Prob(g, ix + 1, iy + 1, iz + 1);
  const double nx = (x - x1) / (x2 - x1), ny = (y - y1) / (y2 - y1), nz = (z - z1) / (z2 - z1);
  const StepF sx{nx, nx * nx, nx * (nx * nx)}, sy{ny, ny * ny, ny * (ny * ny)},
      sz{nz, nz * nz, nz * (nz * nz)};
  const double q11 = sz.f(q111, q112), q12 = sz.f(q121, q122);
  const double q21 = sz.f(q211, q212), q22 = sz.f(q221, q222);
  const double q1 = sy.f(q11, q12), q2 = sy.f(q21, q22);
  if (grad) {
    grad[0] = sx.dt(q1, q2) / (x2 - x1);
    grad[1] = (sx.da() * sy.dt(q11, q12) + sx.db() * sy.dt(q21, q22)) / (y2 - y1);
    grad[2] = (sx.da() * (sy.da() * sz.dt(q111, q112) + sy.db() * sz.dt(q121, q122)) +
               sx.db() * (sy.da() * sz.dt(q211, q212) + sy.db() * sz.dt(q221, q222))) /
              (z2 - z1);
  }
  return sx.f(q1, q2);
}

// Eigen _transformVector and its derivative in (w, x, y, z) (3 x 4).
__device__ void Rotate(const double* q, const double v[3], double out[3], double* J) {
  const double w = q[0], qx = q[1], qy = q[2], qz = q[3];
  const double ax = qy * v[2] - qz * v[1], ay = qz * v[0] - qx * v[2], az = qx * v[1] - qy * v[0];
  const double ux = 2. * ax, uy = 2. * ay, uz = 2. * az;
  out[0] = v[0] + w * ux + (qy * uz - qz * uy);
  out[1] = v[1] + w * uy + (qz * ux - qx * uz);
  out[2] = v[2] + w * uz + (qx * uy - qy * ux);
  if (!J) return;
  const double V[9] = {0., -v[2], v[1], v[2], 0., -v[0], -v[1], v[0], 0.};
  const double A[9] = {0., -az, ay, az, 0., -ax, -ay, ax, 0.};
  const double Q[9] = {0., -qz, qy, qz, 0., -qx, -qy, qx, 0.};
  const double u[3] = {ux, uy, uz};
  for (int r = 0; r < 3; ++r) {
    J[4 * r] = u[r];
    for (int c = 0; c < 3; ++c) {
      double qv_v = 0.;
      for (int k = 0; k < 3; ++k) qv_v += Q[3 * r + k] * V[3 * k + c];
      J[4 * r + 1 + c] = -2. * w * V[3 * r + c] - 2. * A[3 * r + c] - 2. * qv_v;
    }
  }
}

__device__ void QuatProduct(const double* a, const double* b, double* z) {
  z[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  z[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  z[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  z[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}

__device__ __forceinline__ double WaveSumD(double v) {
  for (int m = 32; m > 0; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}

__device__ void BlockSum(double* v, double (*red)[kSums]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int k = 0; k < kSums; ++k) {
    const double t = WaveSumD(v[k]);
    if (lane == 0) red[w][k] = t;
  }
  __syncthreads();
  for (int k = 0; k < kSums; ++k) {
    double t = 0.;
    for (int q = 0; q < kR3Threads / 64; ++q) t += red[q][k];
    v[k] = t;
  }
  __syncthreads();
}

// Adds residual r with tangent Jacobian row j[6] to the sums.
__device__ __forceinline__ void Accumulate(double* acc, double r, const double* j, bool jac) {
  acc[0] += r * r;
  if (!jac) return;
  int k = 1;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b) acc[k++] += j[a] * j[b];
  for (int a = 0; a < 6; ++a) acc[22 + a] += j[a] * r;
}

template <bool kJac>
__device__ void Pass3(const Refine3Desc& d, const float* pts, const double* scale,
                      const Refine3Opts& o, const double* t, const double* q,
                      const double* target_inv, double* out, double (*red)[kSums]) {
  double acc[kSums];
  for (int k = 0; k < kSums; ++k) acc[k] = 0.;
  // QuaternionParameterization::ComputeJacobian (4 x 3).
  const double L[12] = {-q[1], -q[2], -q[3], q[0], q[3], -q[2], -q[3], q[0], q[1], q[2], -q[1], q[0]};
  const int n0 = d.n[0], total = d.n[0] + d.n[1] + 6;
  for (int i = threadIdx.x; i < total; i += kR3Threads) {
    double r, j[6] = {0., 0., 0., 0., 0., 0.};
    if (i < n0 + d.n[1]) {
      const int k = i < n0 ? 0 : 1;
      const float* p = pts + 3 * (d.offset[k] + (i < n0 ? i : i - n0));
      const double v[3] = {static_cast<double>(p[0]), static_cast<double>(p[1]),
                           static_cast<double>(p[2])};
      double w[3], Jq[12], grad[3];
      Rotate(q, v, w, kJac ? Jq : nullptr);
      for (int a = 0; a < 3; ++a) w[a] += t[a];
      const double val = Interpolate(d.grid[k], w[0], w[1], w[2], kJac ? grad : nullptr);
      r = scale[k] * (1. - val);
      if (kJac) {
        double dq[4] = {0., 0., 0., 0.};
        for (int c = 0; c < 4; ++c)
          for (int a = 0; a < 3; ++a) dq[c] += -scale[k] * grad[a] * Jq[4 * a + c];
        for (int a = 0; a < 3; ++a) j[a] = -scale[k] * grad[a];
        for (int c = 0; c < 3; ++c) {
          double s = 0.;
          for (int m = 0; m < 4; ++m) s += dq[m] * L[3 * m + c];
          j[3 + c] = s;
        }
      }
    } else if (i < n0 + d.n[1] + 3) {
      const int a = i - n0 - d.n[1];
      r = o.wt * (t[a] - d.target[a]);
      j[a] = o.wt;
    } else {
      const int a = i - n0 - d.n[1] - 3;
      double delta[4];
      QuatProduct(target_inv, q, delta);
      r = o.wr * delta[a + 1];
      const double* ti = target_inv;
      const double M[3][4] = {{ti[1], ti[0], -ti[3], ti[2]},
                              {ti[2], ti[3], ti[0], -ti[1]},
                              {ti[3], -ti[2], ti[1], ti[0]}};
      for (int c = 0; c < 3; ++c) {
        double s = 0.;
        for (int m = 0; m < 4; ++m) s += o.wr * M[a][m] * L[3 * m + c];
        j[3 + c] = s;
      }
    }
    Accumulate(acc, r, j, kJac);
  }
  BlockSum(acc, red);
  for (int k = 0; k < kSums; ++k) out[k] = acc[k];
}

__device__ bool Solve6(double* M, double* b, double* out) {
  for (int c = 0; c < 6; ++c) {
    int piv = c;
    for (int i = c + 1; i < 6; ++i)
      if (fabs(M[i * 6 + c]) > fabs(M[piv * 6 + c])) piv = i;
    if (M[piv * 6 + c] == 0.) return false;
    for (int j = 0; j < 6; ++j) {
      const double s = M[c * 6 + j];
      M[c * 6 + j] = M[piv * 6 + j];
      M[piv * 6 + j] = s;
    }
    const double sb = b[c];
    b[c] = b[piv];
    b[piv] = sb;
    for (int i = c + 1; i < 6; ++i) {
      const double f = M[i * 6 + c] / M[c * 6 + c];
      for (int j = c; j < 6; ++j) M[i * 6 + j] -= f * M[c * 6 + j];
      b[i] -= f * b[c];
    }
  }
  for (int i = 5; i >= 0; --i) {
    double v = b[i];
    for (int j = i + 1; j < 6; ++j) v -= M[i * 6 + j] * out[j];
    out[i] = v / M[i * 6 + i];
  }
  return true;
}

__device__ void Unpack(const double* S, double* Au, double* gu) {
  int k = 1;
  for (int a = 0; a < 6; ++a)
    for (int b = a; b < 6; ++b) {
      Au[6 * a + b] = S[k];
      Au[6 * b + a] = S[k];
      ++k;
    }
  for (int a = 0; a < 6; ++a) gu[a] = S[22 + a];
}

// Ceres 1.13 TrustRegionMinimizer::Minimize as in ceres2d.hip: every thread
// runs the 6-dimensional step logic on the same block-reduced sums.
__global__ void __launch_bounds__(kR3Threads)
ceres3d_refine(const Refine3Desc* __restrict__ items, const float* __restrict__ points,
               Refine3Opts o, double* __restrict__ out, int32_t* __restrict__ out_iters) {
  __shared__ double red[kR3Threads / 64][kSums];
  const Refine3Desc d = items[blockIdx.x];
  const double scale[2] = {o.w0 / sqrt(static_cast<double>(d.n[0])),
                           o.w1 / sqrt(static_cast<double>(d.n[1]))};
  const double target_inv[4] = {d.q[0], -d.q[1], -d.q[2], -d.q[3]};
  double t[3] = {d.t[0], d.t[1], d.t[2]}, q[4] = {d.q[0], d.q[1], d.q[2], d.q[3]};
  double S[kSums], T[kSums];
  Pass3<true>(d, points, scale, o, t, q, target_inv, S, red);
  double cost = 0.5 * S[0];
  double Au[36], gu[6], js[6];
  Unpack(S, Au, gu);
  for (int a = 0; a < 6; ++a) js[a] = 1. / (1. + sqrt(Au[7 * a]));
  StepEvaluator ev(cost, o.nonmonotonic != 0);
  LmRadius lm;
  double best_t[3] = {t[0], t[1], t[2]}, best_q[4] = {q[0], q[1], q[2], q[3]}, best_cost = cost;
  int iter = 0, invalid = 0;
  auto gradient_small = [&]() {
    double gmax = 0.;
    for (int a = 0; a < 6; ++a) gmax = fmax(gmax, fabs(gu[a]));
    return gmax <= 1e-10;
  };
  bool go = o.max_iterations > 0 && !gradient_small();
  while (go) {
    ++iter;
    double A[36], g[6], M[36], rhs[6], ds[6] = {0., 0., 0., 0., 0., 0.};
    for (int a = 0; a < 6; ++a) {
      g[a] = gu[a] * js[a];
      for (int b = 0; b < 6; ++b) A[6 * a + b] = Au[6 * a + b] * js[a] * js[b];
    }
    for (int a = 0; a < 6; ++a) {
      for (int b = 0; b < 6; ++b) M[6 * a + b] = A[6 * a + b];
      M[7 * a] += fmin(fmax(A[7 * a], 1e-6), 1e32) / lm.radius;
      rhs[a] = -g[a];
    }
    const bool solved = Solve6(M, rhs, ds);
    double gd = 0., dad = 0.;
    for (int a = 0; a < 6; ++a) {
      gd += g[a] * ds[a];
      for (int b = 0; b < 6; ++b) dad += ds[a] * A[6 * a + b] * ds[b];
    }
    const double model = -(gd + 0.5 * dad);
    if (!solved || !(model > 0.)) {
      if (++invalid > 5) break;  // HandleInvalidStep: LM rejects the step
      lm.Rejected();
    } else {
      invalid = 0;
      double step[6], step_norm = 0., x_norm = 0.;
      for (int a = 0; a < 6; ++a) {
        step[a] = ds[a] * js[a];
        step_norm += step[a] * step[a];
      }
      for (int a = 0; a < 3; ++a) x_norm += t[a] * t[a];
      for (int a = 0; a < 4; ++a) x_norm += q[a] * q[a];
      // Plus: t + dt; QuaternionParameterization::Plus on the rotation.
      double tn[3] = {t[0] + step[0], t[1] + step[1], t[2] + step[2]}, qn[4];
      const double nrm = sqrt(step[3] * step[3] + step[4] * step[4] + step[5] * step[5]);
      if (nrm > 0.) {
        const double sn = sin(nrm) / nrm;
        const double qd[4] = {cos(nrm), sn * step[3], sn * step[4], sn * step[5]};
        QuatProduct(qd, q, qn);
      } else {
        for (int a = 0; a < 4; ++a) qn[a] = q[a];
      }
      Pass3<false>(d, points, scale, o, tn, qn, target_inv, T, red);
      const double new_cost = 0.5 * T[0];
      if (sqrt(step_norm) <= (sqrt(x_norm) + 1e-8) * 1e-8) break;  // parameter tolerance
      if (fabs(cost - new_cost) <= 1e-6 * cost) break;             // function tolerance
      const double quality = ev.Quality(new_cost, model);
      if (quality > 1e-3) {
        for (int a = 0; a < 3; ++a) t[a] = tn[a];
        for (int a = 0; a < 4; ++a) q[a] = qn[a];
        Pass3<true>(d, points, scale, o, t, q, target_inv, S, red);
        cost = 0.5 * S[0];
        Unpack(S, Au, gu);
        lm.Accepted(quality);
        ev.Accepted(new_cost, model);
        if (cost < best_cost) {
          best_cost = cost;
          for (int a = 0; a < 3; ++a) best_t[a] = t[a];
          for (int a = 0; a < 4; ++a) best_q[a] = q[a];
        }
      } else {
        lm.Rejected();
      }
    }
    go = iter < o.max_iterations && lm.radius >= 1e-32 && !gradient_small();
  }
  if (threadIdx.x == 0) {
    for (int a = 0; a < 3; ++a) out[7 * blockIdx.x + a] = best_t[a];
    for (int a = 0; a < 4; ++a) out[7 * blockIdx.x + 3 + a] = best_q[a];
    if (out_iters) out_iters[blockIdx.x] = iter;
  }
}

// Test-visible lookups on a device grid (csm_hybrid_grid_get_probability /
// _interpolate): the same Prob / Interpolate the refinement kernel uses.
__global__ void grid_probability(GridView3 g, const int32_t* __restrict__ ijk, int64_t n,
                                 float* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = static_cast<float>(Prob(g, ijk[3 * i], ijk[3 * i + 1], ijk[3 * i + 2]));
}
__global__ void grid_interpolate(GridView3 g, const double* __restrict__ xyz, int64_t n,
                                 double* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = Interpolate(g, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], nullptr);
}

template <typename In, typename Out, typename K>
int GridLookup(const csm_hybrid_grid* g, const In* in, int64_t n, Out* out, K kernel) {
  if (!g || n < 0 || (n > 0 && (!in || !out))) return CSM_EINVAL;
  if (n == 0) return CSM_OK;
  csm_context* ctx = g->ctx;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CSM_EHIP;
  DevBuf din, dout;
  int rc;
  if ((rc = din.Reserve(sizeof(In) * 3 * n)) || (rc = dout.Reserve(sizeof(Out) * n))) return rc;
  hipStream_t st = ctx->stream;
  CSM_HIP(hipMemcpyAsync(din.ptr, in, sizeof(In) * 3 * n, hipMemcpyHostToDevice, st));
  const GridView3 view{g->prob.as<float>(), g->brick, g->resolution};
  hipLaunchKernelGGL(kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, st, view,
                     din.as<In>(), n, dout.as<Out>());
  CSM_HIP(hipGetLastError());
  CSM_HIP(hipMemcpyAsync(out, dout.ptr, sizeof(Out) * n, hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  return CSM_OK;
}

}  // namespace
}  // namespace csm

extern "C" {

int csm_ceres3d_refine_batch(csm_context* ctx, const csm_hybrid_grid* const* grids,
                             int32_t num_grids, const csm_node3d* nodes, int32_t num_nodes,
                             const csm_refine3d* items, int64_t n,
                             const csm_ceres3d_options* options, csm_pose3d* out,
                             int32_t* iterations) {
  using namespace csm;
  if (!ctx || !options || (n > 0 && (!items || !out || !grids || !nodes))) return CSM_EINVAL;
  if (n == 0) return CSM_OK;
  if (!(options->occupied_space_weight_0 > 0.) || !(options->occupied_space_weight_1 > 0.) ||
      !(options->translation_weight > 0.) || !(options->rotation_weight > 0.) ||
      options->max_num_iterations < 0)
    return CSM_EINVAL;  // CHECK_GTs of ceres_scan_matcher_3d.cc:106-156
  if (n > 0x7fffffff) return CSM_ERANGE;
  // Node clouds once each, high then low resolution.
  std::vector<int64_t> off(2 * static_cast<size_t>(num_nodes), -1);
  std::vector<float> pts;
  std::vector<Refine3Desc> desc(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    const csm_refine3d& it = items[i];
    if (it.high_grid < 0 || it.high_grid >= num_grids || it.low_grid < 0 ||
        it.low_grid >= num_grids || !grids[it.high_grid] || !grids[it.low_grid] || it.node < 0 ||
        it.node >= num_nodes)
      return CSM_EINVAL;
    const csm_node3d& nd = nodes[it.node];
    if (nd.num_high_resolution <= 0 || nd.num_low_resolution <= 0 || !nd.high_resolution_xyz ||
        !nd.low_resolution_xyz)
      return CSM_EINVAL;
    if (off[2 * it.node] < 0) {
      off[2 * it.node] = static_cast<int64_t>(pts.size() / 3);
      pts.insert(pts.end(), nd.high_resolution_xyz, nd.high_resolution_xyz + 3 * nd.num_high_resolution);
      off[2 * it.node + 1] = static_cast<int64_t>(pts.size() / 3);
      pts.insert(pts.end(), nd.low_resolution_xyz, nd.low_resolution_xyz + 3 * nd.num_low_resolution);
    }
    Refine3Desc& d = desc[i];
    const csm_hybrid_grid* g[2] = {grids[it.high_grid], grids[it.low_grid]};
    for (int k = 0; k < 2; ++k) {
      // Grids from any context on ctx's device (e.g. one whose stream built
      // them while ctx searched); their builds are waited for below.
      if (!g[k]->ctx || g[k]->ctx->device != ctx->device) return CSM_EINVAL;
      d.grid[k] = GridView3{g[k]->prob.as<float>(), g[k]->brick, g[k]->resolution};
      d.offset[k] = off[2 * it.node + k];
    }
    d.n[0] = nd.num_high_resolution;
    d.n[1] = nd.num_low_resolution;
    for (int a = 0; a < 3; ++a) {
      d.t[a] = it.initial.t[a];
      d.target[a] = it.target[a];
    }
    for (int a = 0; a < 4; ++a) d.q[a] = it.initial.q[a];
  }
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return CSM_EHIP;
  int rc;
  if ((rc = ctx->cr3_items.Reserve(sizeof(Refine3Desc) * n))) return rc;
  if ((rc = ctx->cr3_points.Reserve(sizeof(float) * std::max<size_t>(pts.size(), 3)))) return rc;
  if ((rc = ctx->cr3_out.Reserve(sizeof(double) * 7 * n + sizeof(int32_t) * n))) return rc;
  hipStream_t st = ctx->stream;
  for (int32_t k = 0; k < num_grids; ++k)  // grids another context's stream built
    if (grids[k] && (rc = WaitBuilt(grids[k]->ready, grids[k]->ctx->stream, st))) return rc;
  CSM_HIP(hipMemcpyAsync(ctx->cr3_items.ptr, desc.data(), sizeof(Refine3Desc) * n,
                         hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(ctx->cr3_points.ptr, pts.data(), sizeof(float) * pts.size(),
                         hipMemcpyHostToDevice, st));
  const Refine3Opts o{options->occupied_space_weight_0, options->occupied_space_weight_1,
                      options->translation_weight, options->rotation_weight,
                      options->max_num_iterations, options->use_nonmonotonic_steps ? 1 : 0};
  double* dout = ctx->cr3_out.as<double>();
  int32_t* diters = reinterpret_cast<int32_t*>(dout + 7 * n);
  hipLaunchKernelGGL(ceres3d_refine, dim3(static_cast<unsigned>(n)), dim3(kR3Threads), 0, st,
                     ctx->cr3_items.as<Refine3Desc>(), ctx->cr3_points.as<float>(), o, dout, diters);
  CSM_HIP(hipGetLastError());
  std::vector<double> host(7 * static_cast<size_t>(n));
  CSM_HIP(hipMemcpyAsync(host.data(), dout, sizeof(double) * 7 * n, hipMemcpyDeviceToHost, st));
  if (iterations)
    CSM_HIP(hipMemcpyAsync(iterations, diters, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  for (int64_t i = 0; i < n; ++i) {
    for (int a = 0; a < 3; ++a) out[i].t[a] = host[7 * i + a];
    for (int a = 0; a < 4; ++a) out[i].q[a] = host[7 * i + 3 + a];
  }
  return CSM_OK;
}

int csm_hybrid_grid_get_probability(const csm_hybrid_grid* g, const int32_t* xyz_indices, int64_t n,
                                    float* out) {
  return csm::GridLookup(g, xyz_indices, n, out, csm::grid_probability);
}

int csm_hybrid_grid_interpolate(const csm_hybrid_grid* g, const double* xyz, int64_t n,
                                double* out) {
  return csm::GridLookup(g, xyz, n, out, csm::grid_interpolate);
}

}  // extern "C"
