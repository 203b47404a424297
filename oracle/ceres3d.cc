// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h). The checker for
// csm_ceres3d_refine_batch; never linked into libcsm_amd.so.
//
// CeresScanMatcher3D::Match (mapping/internal/3d/scan_matching/
// ceres_scan_matcher_3d.cc:84-160) as ConstraintBuilder3D calls it after the
// branch and bound (constraint_builder_3d.cc:264-275): pose = translation (3)
// + rotation quaternion (w, x, y, z) with ceres::QuaternionParameterization;
// residual blocks
//   * OccupiedSpaceCostFunction3D (occupied_space_cost_function_3d.h) for the
//     high-resolution cloud in the high-resolution HybridGrid (weight
//     occupied_space_weight_0) and the low-resolution cloud in the
//     low-resolution grid (occupied_space_weight_1), each scaled by
//     1 / sqrt(N): r_i = w * (1 - InterpolatedGrid(world_i)), with the
//     smooth-step tricubic interpolation of interpolated_grid.h:50-150;
//   * TranslationDeltaCostFunctor3D: w_t * (t - target);
//   * RotationDeltaCostFunctor3D: w_r * vec(target^-1 * q).
// The solver restates Ceres 1.13's trust-region Levenberg-Marquardt (as
// oracle/ceres2d.cc) on the 6-dimensional tangent space, with
// max_num_iterations = 10 and monotonic steps (pose_graph.lua:49-60) by
// default. Pinned by the reference's ceres_scan_matcher_3d_test.cc (restated
// without its intensity block, which ConstraintBuilder3D never passes,
// constraint_builder_3d.cc:267-274) and rotation_delta_cost_functor_3d_test.cc
// to their tolerances; Ceres itself is absent from this image.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "ceres_minimizer.h"
#include "oracle3d.h"

namespace oracle {
namespace {

// f(t; A, B) = (A - B) 2t^3 + (B - A) 3t^2 + A and its derivatives.
struct Step {
  double t, tt, ttt;
  double f(double a, double b) const { return (a - b) * ttt * 2. + (b - a) * tt * 3. + a; }
  double dt(double a, double b) const { return (a - b) * 6. * tt + (b - a) * 6. * t; }
  double da() const { return 2. * ttt - 3. * tt + 1.; }
  double db() const { return -2. * ttt + 3. * tt; }
};

}  // namespace

// InterpolatedGrid::GetInterpolatedValue and its gradient in (x, y, z)
// (interpolated_grid.h:48-105; tests pin it with interpolated_grid_test.cc
// and the fork's hybrid_test.txt).
double Interpolate(const HybridGrid& g, double x, double y, double z, double grad[3]) {
  const float res = g.resolution();
  // CenterOfLowerVoxel (:118-134): the point is cast to float first.
  const Idx3 c = g.GetCellIndex(Vec3f{static_cast<float>(x), static_cast<float>(y),
                                      static_cast<float>(z)});
  float cx = static_cast<float>(c.x) * res, cy = static_cast<float>(c.y) * res,
        cz = static_cast<float>(c.z) * res;
  if (cx > x) cx -= res;
  if (cy > y) cy -= res;
  if (cz > z) cz -= res;
  const double x1 = cx, y1 = cy, z1 = cz;
  const double x2 = static_cast<float>(cx + res), y2 = static_cast<float>(cy + res),
               z2 = static_cast<float>(cz + res);
  const Idx3 i1 = g.GetCellIndex(Vec3f{cx, cy, cz});
  auto q = [&](int dx, int dy, int dz) {
    return static_cast<double>(g.GetProbability(Idx3{i1.x + dx, i1.y + dy, i1.z + dz}));
  };
  const double q111 = q(0, 0, 0), q112 = q(0, 0, 1), q121 = q(0, 1, 0), q122 = q(0, 1, 1);
  const double q211 = q(1, 0, 0), q212 = q(1, 0, 1), q221 = q(1, 1, 0), q222 = q(1, 1, 1);
  const double nx = (x - x1) / (x2 - x1), ny = (y - y1) / (y2 - y1), nz = (z - z1) / (z2 - z1);
  const Step sx{nx, nx * nx, nx * (nx * nx)}, sy{ny, ny * ny, ny * (ny * ny)},
      sz{nz, nz * nz, nz * (nz * nz)};
  const double q11 = sz.f(q111, q112), q12 = sz.f(q121, q122);
  const double q21 = sz.f(q211, q212), q22 = sz.f(q221, q222);
  const double q1 = sy.f(q11, q12), q2 = sy.f(q21, q22);
  const double v = sx.f(q1, q2);
  if (grad) {
    const double dnx = sx.dt(q1, q2);
    const double dny = sx.da() * sy.dt(q11, q12) + sx.db() * sy.dt(q21, q22);
    const double dnz = sx.da() * (sy.da() * sz.dt(q111, q112) + sy.db() * sz.dt(q121, q122)) +
                       sx.db() * (sy.da() * sz.dt(q211, q212) + sy.db() * sz.dt(q221, q222));
    grad[0] = dnx / (x2 - x1);
    grad[1] = dny / (y2 - y1);
    grad[2] = dnz / (z2 - z1);
  }
  return v;
}

namespace {

// Eigen _transformVector: v + w * uv + q.vec x uv, uv = 2 q.vec x v; and its
// derivative in (w, x, y, z) (3 x 4, row-major).
void Rotate(const double q[4], const double v[3], double out[3], double J[12]) {
  const double w = q[0], qx = q[1], qy = q[2], qz = q[3];
  const double ax = qy * v[2] - qz * v[1], ay = qz * v[0] - qx * v[2], az = qx * v[1] - qy * v[0];
  const double ux = 2. * ax, uy = 2. * ay, uz = 2. * az;
  out[0] = v[0] + w * ux + (qy * uz - qz * uy);
  out[1] = v[1] + w * uy + (qz * ux - qx * uz);
  out[2] = v[2] + w * uz + (qx * uy - qy * ux);
  if (!J) return;
  // d/dw = uv; d/dqv = -2w [v]x - 2 [a]x - 2 [qv]x [v]x.
  auto cross = [](const double a[3]) {
    return std::vector<double>{0., -a[2], a[1], a[2], 0., -a[0], -a[1], a[0], 0.};
  };
  const double a[3] = {ax, ay, az}, qv[3] = {qx, qy, qz};
  const std::vector<double> V = cross(v), A = cross(a), Q = cross(qv);
  for (int r = 0; r < 3; ++r) {
    J[4 * r] = (r == 0 ? ux : r == 1 ? uy : uz);
    for (int c = 0; c < 3; ++c) {
      double qv_v = 0.;
      for (int k = 0; k < 3; ++k) qv_v += Q[3 * r + k] * V[3 * k + c];
      J[4 * r + 1 + c] = -2. * w * V[3 * r + c] - 2. * A[3 * r + c] - 2. * qv_v;
    }
  }
}

// ceres::QuaternionProduct (z = a * b), (w, x, y, z).
void QuatProduct(const double a[4], const double b[4], double z[4]) {
  z[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  z[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  z[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  z[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
}

struct Problem3 {
  const HybridGrid* grid[2];
  const std::vector<Vec3f>* cloud[2];
  double scale[2];
  double wt, wr, target[3], target_inv[4];
};

// Residuals and the Jacobian in the tangent space (t, delta), 6 columns.
double Evaluate3(const Problem3& p, const double t[3], const double q[4], std::vector<double>* r,
                 std::vector<double>* J) {
  r->clear();
  if (J) J->clear();
  double cost = 0.;
  // QuaternionParameterization::ComputeJacobian (4 x 3, row-major).
  const double L[12] = {-q[1], -q[2], -q[3], q[0], q[3], -q[2],
                        -q[3], q[0],  q[1],  q[2], -q[1], q[0]};
  for (int k = 0; k < 2; ++k)
    for (const Vec3f& pt : *p.cloud[k]) {
      const double v[3] = {pt.x, pt.y, pt.z};
      double w[3], Jq[12];
      Rotate(q, v, w, J ? Jq : nullptr);
      for (int a = 0; a < 3; ++a) w[a] += t[a];
      double grad[3];
      const double val = Interpolate(*p.grid[k], w[0], w[1], w[2], J ? grad : nullptr);
      const double res = p.scale[k] * (1. - val);
      r->push_back(res);
      cost += res * res;
      if (J) {
        double dq[4] = {0., 0., 0., 0.};
        for (int c = 0; c < 4; ++c)
          for (int a = 0; a < 3; ++a) dq[c] += -p.scale[k] * grad[a] * Jq[4 * a + c];
        for (int a = 0; a < 3; ++a) J->push_back(-p.scale[k] * grad[a]);
        for (int c = 0; c < 3; ++c) {
          double s = 0.;
          for (int m = 0; m < 4; ++m) s += dq[m] * L[3 * m + c];
          J->push_back(s);
        }
      }
    }
  for (int a = 0; a < 3; ++a) {
    const double res = p.wt * (t[a] - p.target[a]);
    r->push_back(res);
    cost += res * res;
    if (J)
      for (int c = 0; c < 6; ++c) J->push_back(c == a ? p.wt : 0.);
  }
  double delta[4];
  QuatProduct(p.target_inv, q, delta);
  // d delta / d q: left multiplication by target_inv (rows 1..3).
  const double* ti = p.target_inv;
  const double M[3][4] = {{ti[1], ti[0], -ti[3], ti[2]},
                          {ti[2], ti[3], ti[0], -ti[1]},
                          {ti[3], -ti[2], ti[1], ti[0]}};
  for (int a = 0; a < 3; ++a) {
    const double res = p.wr * delta[a + 1];
    r->push_back(res);
    cost += res * res;
    if (J) {
      for (int c = 0; c < 3; ++c) J->push_back(0.);
      for (int c = 0; c < 3; ++c) {
        double s = 0.;
        for (int m = 0; m < 4; ++m) s += p.wr * M[a][m] * L[3 * m + c];
        J->push_back(s);
      }
    }
  }
  return 0.5 * cost;
}

bool SolveN(std::vector<double> M, std::vector<double> b, int n, double* out) {
  for (int c = 0; c < n; ++c) {
    int piv = c;
    for (int i = c + 1; i < n; ++i)
      if (std::fabs(M[i * n + c]) > std::fabs(M[piv * n + c])) piv = i;
    if (M[piv * n + c] == 0.) return false;
    for (int j = 0; j < n; ++j) std::swap(M[c * n + j], M[piv * n + j]);
    std::swap(b[c], b[piv]);
    for (int i = c + 1; i < n; ++i) {
      const double f = M[i * n + c] / M[c * n + c];
      for (int j = c; j < n; ++j) M[i * n + j] -= f * M[c * n + j];
      b[i] -= f * b[c];
    }
  }
  for (int i = n - 1; i >= 0; --i) {
    double v = b[i];
    for (int j = i + 1; j < n; ++j) v -= M[i * n + j] * out[j];
    out[i] = v / M[i * n + i];
  }
  return true;
}

}  // namespace

void RotationDeltaResiduals3D(double scale, const double target_q[4], const double q[4],
                              double out[3]) {
  const double inv[4] = {target_q[0], -target_q[1], -target_q[2], -target_q[3]};
  double delta[4];
  QuatProduct(inv, q, delta);
  for (int a = 0; a < 3; ++a) out[a] = scale * delta[a + 1];
}

int CeresMatch3D(const HybridGrid& high, const HybridGrid& low, const std::vector<Vec3f>& high_cloud,
                 const std::vector<Vec3f>& low_cloud, const CeresOptions3D& o,
                 const double target[3], const double initial_t[3], const double initial_q[4],
                 double out_t[3], double out_q[4], double* final_cost) {
  Problem3 p;
  p.grid[0] = &high;
  p.grid[1] = &low;
  p.cloud[0] = &high_cloud;
  p.cloud[1] = &low_cloud;
  p.scale[0] = o.w0 / std::sqrt(static_cast<double>(high_cloud.size()));
  p.scale[1] = o.w1 / std::sqrt(static_cast<double>(low_cloud.size()));
  p.wt = o.wt;
  p.wr = o.wr;
  for (int a = 0; a < 3; ++a) p.target[a] = target[a];
  p.target_inv[0] = initial_q[0];
  p.target_inv[1] = -initial_q[1];
  p.target_inv[2] = -initial_q[2];
  p.target_inv[3] = -initial_q[3];
  double t[3] = {initial_t[0], initial_t[1], initial_t[2]};
  double q[4] = {initial_q[0], initial_q[1], initial_q[2], initial_q[3]};
  std::vector<double> r, J, rn;
  double cost = Evaluate3(p, t, q, &r, &J);
  const size_t m = r.size();
  auto normal = [&](double* Au, double* gu) {
    for (int a = 0; a < 36; ++a) Au[a] = 0.;
    for (int a = 0; a < 6; ++a) gu[a] = 0.;
    for (size_t i = 0; i < m; ++i)
      for (int a = 0; a < 6; ++a) {
        gu[a] += J[6 * i + a] * r[i];
        for (int b = 0; b < 6; ++b) Au[6 * a + b] += J[6 * i + a] * J[6 * i + b];
      }
  };
  double Au[36], gu[6], scale[6];
  normal(Au, gu);
  for (int a = 0; a < 6; ++a) scale[a] = 1. / (1. + std::sqrt(Au[7 * a]));
  StepEvaluator ev(cost, o.use_nonmonotonic_steps ? 5 : 0);
  double best_t[3] = {t[0], t[1], t[2]}, best_q[4] = {q[0], q[1], q[2], q[3]}, best_cost = cost;
  double radius = 1e4, decrease = 2.;
  int iter = 0, invalid = 0;
  auto gradient_small = [&]() {
    double gmax = 0.;
    for (int a = 0; a < 6; ++a) gmax = std::max(gmax, std::fabs(gu[a]));
    return gmax <= 1e-10;
  };
  // Ceres 1.13 TrustRegionMinimizer::Minimize, as in ceres2d.cc.
  bool go = o.max_num_iterations > 0 && !gradient_small();
  while (go) {
    ++iter;
    std::vector<double> A(36), g(6), M(36), rhs(6);
    for (int a = 0; a < 6; ++a) {
      g[a] = gu[a] * scale[a];
      for (int b = 0; b < 6; ++b) A[6 * a + b] = Au[6 * a + b] * scale[a] * scale[b];
    }
    for (int a = 0; a < 6; ++a) {
      for (int b = 0; b < 6; ++b) M[6 * a + b] = A[6 * a + b];
      M[7 * a] += std::min(std::max(A[7 * a], 1e-6), 1e32) / radius;
      rhs[a] = -g[a];
    }
    double ds[6] = {0., 0., 0., 0., 0., 0.};
    const bool solved = SolveN(M, rhs, 6, ds);
    double gd = 0., dad = 0.;
    for (int a = 0; a < 6; ++a) {
      gd += g[a] * ds[a];
      for (int b = 0; b < 6; ++b) dad += ds[a] * A[6 * a + b] * ds[b];
    }
    const double model = -(gd + 0.5 * dad);
    if (!solved || !(model > 0.)) {
      if (++invalid > 5) break;
      radius /= decrease;
      decrease *= 2.;
    } else {
      invalid = 0;
      double step[6], step_norm = 0., x_norm = 0.;
      for (int a = 0; a < 6; ++a) {
        step[a] = ds[a] * scale[a];
        step_norm += step[a] * step[a];
      }
      for (int a = 0; a < 3; ++a) x_norm += t[a] * t[a];
      for (int a = 0; a < 4; ++a) x_norm += q[a] * q[a];
      // Plus: t + dt; QuaternionParameterization::Plus on the rotation.
      double tn[3] = {t[0] + step[0], t[1] + step[1], t[2] + step[2]}, qn[4];
      const double nrm = std::sqrt(step[3] * step[3] + step[4] * step[4] + step[5] * step[5]);
      if (nrm > 0.) {
        const double sn = std::sin(nrm) / nrm;
        const double qd[4] = {std::cos(nrm), sn * step[3], sn * step[4], sn * step[5]};
        QuatProduct(qd, q, qn);
      } else {
        for (int a = 0; a < 4; ++a) qn[a] = q[a];
      }
      const double new_cost = Evaluate3(p, tn, qn, &rn, nullptr);
      if (std::sqrt(step_norm) <= (std::sqrt(x_norm) + 1e-8) * 1e-8) break;  // parameter tol.
      if (std::fabs(cost - new_cost) <= 1e-6 * cost) break;                 // function tol.
      const double quality = ev.Quality(new_cost, model);
      if (quality > 1e-3) {
        for (int a = 0; a < 3; ++a) t[a] = tn[a];
        for (int a = 0; a < 4; ++a) q[a] = qn[a];
        cost = Evaluate3(p, t, q, &r, &J);
        normal(Au, gu);
        const double tf = 2. * quality - 1.;
        radius = std::min(1e16, radius / std::max(1. / 3., 1. - tf * tf * tf));
        decrease = 2.;
        ev.Accepted(new_cost, model);
        if (cost < best_cost) {
          best_cost = cost;
          for (int a = 0; a < 3; ++a) best_t[a] = t[a];
          for (int a = 0; a < 4; ++a) best_q[a] = q[a];
        }
      } else {
        radius /= decrease;
        decrease *= 2.;
      }
    }
    go = iter < o.max_num_iterations && radius >= 1e-32 && !gradient_small();
  }
  for (int a = 0; a < 3; ++a) t[a] = best_t[a];
  for (int a = 0; a < 4; ++a) q[a] = best_q[a];
  if (final_cost) *final_cost = best_cost;
  for (int a = 0; a < 3; ++a) out_t[a] = t[a];
  for (int a = 0; a < 4; ++a) out_q[a] = q[a];
  return iter;
}

}  // namespace oracle

using namespace oracle;

extern "C" {

// opts: w0, w1, wt, wr, max_num_iterations, use_nonmonotonic_steps. target: xyz. initial/out: t[3], q[4] (w, x, y, z).
int32_t oracle_ceres3d_match(void* high, void* low, const float* high_xyz, int32_t nh,
                             const float* low_xyz, int32_t nl, const double* opts,
                             const double* target, const double* initial, double* out) {
  std::vector<Vec3f> hc(static_cast<size_t>(nh)), lc(static_cast<size_t>(nl));
  for (int32_t i = 0; i < nh; ++i) hc[i] = Vec3f{high_xyz[3 * i], high_xyz[3 * i + 1], high_xyz[3 * i + 2]};
  for (int32_t i = 0; i < nl; ++i) lc[i] = Vec3f{low_xyz[3 * i], low_xyz[3 * i + 1], low_xyz[3 * i + 2]};
  CeresOptions3D o;
  o.w0 = opts[0];
  o.w1 = opts[1];
  o.wt = opts[2];
  o.wr = opts[3];
  o.max_num_iterations = static_cast<int>(opts[4]);
  o.use_nonmonotonic_steps = opts[5] != 0.;
  return CeresMatch3D(*static_cast<HybridGrid*>(high), *static_cast<HybridGrid*>(low), hc, lc, o,
                      target, initial, initial + 3, out, out + 3, nullptr);
}

}  // extern "C"
