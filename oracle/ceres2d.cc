// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h). The checker for
// csm_ceres2d_refine_batch; never linked into libcsm_amd.so.
//
// CeresScanMatcher2D::Match (mapping/internal/2d/scan_matching/
// ceres_scan_matcher_2d.cc:64-105) as ConstraintBuilder2D calls it after the
// branch and bound (constraint_builder_2d.cc:245-249): three residual blocks
// on the pose (x, y, theta):
//   * OccupiedSpaceCostFunction2D (occupied_space_cost_function_2d.cc:30-91):
//     r_i = w / sqrt(N) * BiCubic(grid costs at the transformed point), with
//     ceres::BiCubicInterpolator over the grid padded by kPadding = INT_MAX / 4
//     cells of kMaxCorrespondenceCost;
//   * TranslationDeltaCostFunctor2D: w_t * (x - target), w_t * (y - target);
//   * RotationDeltaCostFunctor2D: w_r * (theta - theta_initial).
// Ceres is not in this image, so the solver below restates
// Ceres' documented trust-region Levenberg-Marquardt with its defaults
// (DENSE_QR on a 3x3 system, Jacobi column scaling from the initial
// Jacobian, initial radius 1e4, min/max diagonal 1e-6 / 1e32, min relative
// decrease 1e-3, function / gradient / parameter tolerances 1e-6 / 1e-10 /
// 1e-8) and the reference's max_num_iterations = 10 and use_nonmonotonic_steps
// = true (pose_graph.lua:30-39), following Ceres 2.x's TrustRegionMinimizer
// and TrustRegionStepEvaluator. Pinned by the reference's own
// ceres_scan_matcher_2d_test.cc and occupied_space_cost_function_2d_test.cc
// (restated in ref_tests.cc) to their tolerances; Ceres itself is absent, so
// agreement beyond those tolerances is unpinned.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <vector>

#include "ceres_minimizer.h"
#include "csm_oracle.h"

namespace oracle {
namespace {

constexpr int kPadding = INT_MAX / 4;

struct CostGrid {
  MapLimits limits;
  const std::vector<float>* table;  // value -> correspondence cost
  const std::vector<uint16_t>* cells;
  double max_cost;
  // GridArrayAdapter::GetValue (occupied_space_cost_function_2d.cc:66-75).
  double Get(int row, int col) const {
    const int nx = limits.cells.num_x_cells, ny = limits.cells.num_y_cells;
    if (row < kPadding || col < kPadding || row >= ny + kPadding || col >= nx + kPadding)
      return max_cost;
    const int x = col - kPadding, y = row - kPadding;
    return static_cast<double>((*table)[(*cells)[static_cast<size_t>(y) * nx + x] & 0x7fff]);
  }
};

// ceres::CubicHermiteSpline (ceres/cubic_interpolation.h).
void Hermite(double p0, double p1, double p2, double p3, double x, double* f, double* dfdx) {
  const double a = 0.5 * (-p0 + 3.0 * p1 - 3.0 * p2 + p3);
  const double b = 0.5 * (2.0 * p0 - 5.0 * p1 + 4.0 * p2 - p3);
  const double c = 0.5 * (-p0 + p2);
  const double d = p1;
  *f = d + x * (c + x * (b + x * a));
  if (dfdx) *dfdx = c + x * (2.0 * b + 3.0 * a * x);
}

// ceres::BiCubicInterpolator::Evaluate(r, c, f, dfdr, dfdc).
void BiCubic(const CostGrid& g, double r, double c, double* f, double* dfdr, double* dfdc) {
  const int row = static_cast<int>(std::floor(r));
  const int col = static_cast<int>(std::floor(c));
  double fr[4], dfr[4];
  for (int k = 0; k < 4; ++k) {
    const int rr = row - 1 + k;
    Hermite(g.Get(rr, col - 1), g.Get(rr, col), g.Get(rr, col + 1), g.Get(rr, col + 2), c - col,
            &fr[k], &dfr[k]);
  }
  Hermite(fr[0], fr[1], fr[2], fr[3], r - row, f, dfdr);
  Hermite(dfr[0], dfr[1], dfr[2], dfr[3], r - row, dfdc, nullptr);
}

struct Problem {
  const CostGrid* grid;
  const std::vector<Vec2d>* points;
  double scale;  // occupied_space_weight / sqrt(N)
  double wt, wr, tx, ty, t0;
};

// Residuals and (optionally) the N + 3 by 3 Jacobian, as AutoDiff evaluates
// them: world = [R t] * (p, 1) with Eigen's 3-term sum x0 + (x1 + x2).
double Evaluate(const Problem& p, const double* x, std::vector<double>* r,
                std::vector<double>* J) {
  const double s = std::sin(x[2]), c = std::cos(x[2]);
  const MapLimits& L = p.grid->limits;
  const size_t n = p.points->size();
  r->resize(n + 3);
  if (J) J->resize(3 * (n + 3));
  double cost = 0.;
  for (size_t i = 0; i < n; ++i) {
    const double px = (*p.points)[i].x, py = (*p.points)[i].y;
    const double wx = c * px + (-s * py + x[0] * 1.);
    const double wy = s * px + (c * py + x[1] * 1.);
    const double rr = (L.max_x - wx) / L.resolution - 0.5 + static_cast<double>(kPadding);
    const double cc = (L.max_y - wy) / L.resolution - 0.5 + static_cast<double>(kPadding);
    double f, dfdr, dfdc;
    BiCubic(*p.grid, rr, cc, &f, &dfdr, &dfdc);
    (*r)[i] = p.scale * f;
    cost += (*r)[i] * (*r)[i];
    if (J) {
      // d(rr)/d(pose) = -d(wx)/d(pose) / res; d(cc)/d(pose) = -d(wy)/d(pose) / res.
      const double dwx_dt = -s * px - c * py, dwy_dt = c * px - s * py;
      (*J)[3 * i + 0] = p.scale * (dfdr * (-1. / L.resolution));
      (*J)[3 * i + 1] = p.scale * (dfdc * (-1. / L.resolution));
      (*J)[3 * i + 2] =
          p.scale * (dfdr * (-dwx_dt / L.resolution) + dfdc * (-dwy_dt / L.resolution));
    }
  }
  (*r)[n] = p.wt * (x[0] - p.tx);
  (*r)[n + 1] = p.wt * (x[1] - p.ty);
  (*r)[n + 2] = p.wr * (x[2] - p.t0);
  for (int k = 0; k < 3; ++k) cost += (*r)[n + k] * (*r)[n + k];
  if (J) {
    for (int k = 0; k < 9; ++k) (*J)[3 * n + k] = 0.;
    (*J)[3 * n + 0] = p.wt;
    (*J)[3 * (n + 1) + 1] = p.wt;
    (*J)[3 * (n + 2) + 2] = p.wr;
  }
  return 0.5 * cost;
}

bool Solve3(double A[3][3], const double b[3], double out[3]) {
  // Gaussian elimination with partial pivoting (the system is SPD here).
  double M[3][4];
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) M[i][j] = A[i][j];
    M[i][3] = b[i];
  }
  for (int c = 0; c < 3; ++c) {
    int piv = c;
    for (int i = c + 1; i < 3; ++i)
      if (std::fabs(M[i][c]) > std::fabs(M[piv][c])) piv = i;
    if (M[piv][c] == 0.) return false;
    for (int j = 0; j < 4; ++j) std::swap(M[c][j], M[piv][j]);
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

}  // namespace

// Returns the number of iterations run; *pose receives the solution and
// *final_cost (if given) Ceres' summary.final_cost, 1/2 |r|^2 at *pose.
// The loop follows Ceres' TrustRegionMinimizer::Minimize: per iteration the
// LM step (invalid if the model decrease is not positive), the candidate's
// cost, the parameter and function tolerance tests (which end the solve
// WITHOUT taking the candidate), then acceptance by step quality > 1e-3. The
// returned parameters are the lowest-cost accepted point
// (FinalizeIterationAndCheckIfMinimizerCanContinue), which differs from the
// last accepted one only with non-monotonic steps.
int CeresMatch2D(const MapLimits& limits, const std::vector<uint16_t>& cells, float min_cc,
                 float max_cc, const CeresOptions2D& o, const double target[2],
                 const double initial[3], const std::vector<Vec2d>& points, double pose[3],
                 double* final_cost) {
  const std::vector<float> table = MakeConversionTable(max_cc, min_cc, max_cc);
  const CostGrid grid{limits, &table, &cells, static_cast<double>(max_cc)};
  Problem p{&grid, &points,
            o.occupied_space_weight / std::sqrt(static_cast<double>(points.size())),
            o.translation_weight, o.rotation_weight, target[0], target[1], initial[2]};
  double x[3] = {initial[0], initial[1], initial[2]};
  std::vector<double> r, J, r_new;
  double cost = Evaluate(p, x, &r, &J);
  const size_t m = r.size();
  double scale[3];
  for (int j = 0; j < 3; ++j) {
    double s = 0.;
    for (size_t i = 0; i < m; ++i) s += J[3 * i + j] * J[3 * i + j];
    scale[j] = 1. / (1. + std::sqrt(s));
  }
  StepEvaluator ev(cost, o.use_nonmonotonic_steps ? 5 : 0);
  double best[3] = {x[0], x[1], x[2]}, best_cost = cost;
  double radius = 1e4, decrease_factor = 2.;
  int iter = 0, invalid = 0;
  // Gradient of the current point: Ju^T r (unscaled), Au = Ju^T Ju.
  double Au[3][3], gu[3];
  auto normal_equations = [&]() {
    for (int a = 0; a < 3; ++a) {
      gu[a] = 0.;
      for (int b = 0; b < 3; ++b) Au[a][b] = 0.;
    }
    for (size_t i = 0; i < m; ++i)
      for (int a = 0; a < 3; ++a) {
        gu[a] += J[3 * i + a] * r[i];
        for (int b = 0; b < 3; ++b) Au[a][b] += J[3 * i + a] * J[3 * i + b];
      }
  };
  normal_equations();
  auto gradient_small = [&]() {
    return std::max({std::fabs(gu[0]), std::fabs(gu[1]), std::fabs(gu[2])}) <= 1e-10;
  };
  bool go = o.max_num_iterations > 0 && !gradient_small();
  while (go) {
    ++iter;
    double A[3][3], g[3];
    for (int a = 0; a < 3; ++a) {
      g[a] = gu[a] * scale[a];
      for (int b = 0; b < 3; ++b) A[a][b] = Au[a][b] * scale[a] * scale[b];
    }
    double M[3][3], rhs[3], ds[3] = {0., 0., 0.};
    for (int a = 0; a < 3; ++a) {
      for (int b = 0; b < 3; ++b) M[a][b] = A[a][b];
      M[a][a] += std::min(std::max(A[a][a], 1e-6), 1e32) / radius;
      rhs[a] = -g[a];
    }
    const bool solved = Solve3(M, rhs, ds);
    // Model cost change -(J ds) . (r + J ds / 2) = -(g . ds + ds^T A ds / 2).
    double gd = 0., dad = 0.;
    for (int a = 0; a < 3; ++a) {
      gd += g[a] * ds[a];
      for (int b = 0; b < 3; ++b) dad += ds[a] * A[a][b] * ds[b];
    }
    const double model = -(gd + 0.5 * dad);
    if (!solved || !(model > 0.)) {
      // HandleInvalidStep: LM treats it as a rejected step.
      if (++invalid > 5) break;
      radius /= decrease_factor;
      decrease_factor *= 2.;
    } else {
      invalid = 0;
      double step[3], step_norm = 0., x_norm = 0.;
      for (int a = 0; a < 3; ++a) {
        step[a] = ds[a] * scale[a];
        step_norm += step[a] * step[a];
        x_norm += x[a] * x[a];
      }
      const double xn[3] = {x[0] + step[0], x[1] + step[1], x[2] + step[2]};
      const double new_cost = Evaluate(p, xn, &r_new, nullptr);
      if (std::sqrt(step_norm) <= (std::sqrt(x_norm) + 1e-8) * 1e-8) break;  // parameter tol.
      if (std::fabs(cost - new_cost) <= 1e-6 * cost) break;                 // function tol.
      const double quality = ev.Quality(new_cost, model);
      if (quality > 1e-3) {
        for (int a = 0; a < 3; ++a) x[a] = xn[a];
        cost = Evaluate(p, x, &r, &J);
        normal_equations();
        const double tf = 2. * quality - 1.;
        radius = std::min(1e16, radius / std::max(1. / 3., 1. - tf * tf * tf));
        decrease_factor = 2.;
        ev.Accepted(new_cost, model);
        if (cost < best_cost) {
          best_cost = cost;
          for (int a = 0; a < 3; ++a) best[a] = x[a];
        }
      } else {
        radius /= decrease_factor;
        decrease_factor *= 2.;
      }
    }
    go = iter < o.max_num_iterations && radius >= 1e-32 && !gradient_small();
  }
  pose[0] = best[0];
  pose[1] = best[1];
  pose[2] = best[2];
  if (final_cost) *final_cost = best_cost;
  return iter;
}

// OccupiedSpaceCostFunction2D::Evaluate residuals only
// (occupied_space_cost_function_2d.cc:40-62) at `pose` (x, y, theta).
std::vector<double> OccupiedSpaceResiduals2D(const MapLimits& limits,
                                             const std::vector<uint16_t>& cells, float min_cc,
                                             float max_cc, double weight,
                                             const std::vector<Vec2d>& points,
                                             const double pose[3]) {
  const std::vector<float> table = MakeConversionTable(max_cc, min_cc, max_cc);
  const CostGrid grid{limits, &table, &cells, static_cast<double>(max_cc)};
  Problem p{&grid, &points, weight / std::sqrt(static_cast<double>(points.size())),
            0., 0., 0., 0., 0.};
  std::vector<double> r;
  Evaluate(p, pose, &r, nullptr);
  r.resize(points.size());
  return r;
}

}  // namespace oracle

using namespace oracle;

extern "C" {

// opts: occupied_space_weight, translation_weight, rotation_weight,
// max_num_iterations, use_nonmonotonic_steps (0/1). target: (x, y). initial / out: (x, y, theta).
int32_t oracle_ceres2d_match(double res, double max_x, double max_y, int32_t nx, int32_t ny,
                             const uint16_t* cells, float min_cc, float max_cc, const double* opts,
                             const double* target, const double* initial, const float* xyz,
                             int32_t n, double* out) {
  MapLimits l;
  l.resolution = res;
  l.max_x = max_x;
  l.max_y = max_y;
  l.cells = CellLimits{nx, ny};
  std::vector<uint16_t> c(cells, cells + static_cast<size_t>(nx) * ny);
  std::vector<Vec2d> pts(static_cast<size_t>(n));
  for (int32_t i = 0; i < n; ++i)
    pts[i] = Vec2d{static_cast<double>(xyz[3 * i]), static_cast<double>(xyz[3 * i + 1])};
  CeresOptions2D o;
  o.occupied_space_weight = opts[0];
  o.translation_weight = opts[1];
  o.rotation_weight = opts[2];
  o.max_num_iterations = static_cast<int>(opts[3]);
  o.use_nonmonotonic_steps = opts[4] != 0.;
  return CeresMatch2D(l, c, min_cc, max_cc, o, target, initial, pts, out, nullptr);
}

}  // extern "C"
