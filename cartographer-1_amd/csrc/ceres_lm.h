// Ceres 1.13's TrustRegionStepEvaluator (trust_region_step_evaluator.cc;
// Conn, Gould & Toint, Trust Region Methods, Algorithm 10.1.2) for the
// CeresScanMatcher2D/3D refinement kernels (ceres2d.hip, ceres3d.hip): the
// quality of a step is judged against the current cost and a reference cost,
// so that with ceres_solver_options.use_nonmonotonic_steps up to
// max_consecutive_nonmonotonic_steps (5) accepted steps may raise the cost.
#ifndef CSM_CERES_LM_H_
#define CSM_CERES_LM_H_

#include <hip/hip_runtime.h>

namespace csm {

struct StepEvaluator {
  double reference_cost, minimum_cost, current_cost, candidate_cost;
  double acc_reference_model, acc_candidate_model;
  int num_nonmonotonic, max_nonmonotonic;
  __device__ StepEvaluator(double cost, bool nonmonotonic)
      : reference_cost(cost), minimum_cost(cost), current_cost(cost), candidate_cost(cost),
        acc_reference_model(0.), acc_candidate_model(0.), num_nonmonotonic(0),
        max_nonmonotonic(nonmonotonic ? 5 : 0) {}
  __device__ double Quality(double cost, double model) const {
    const double relative = (current_cost - cost) / model;
    const double historical = (reference_cost - cost) / (acc_reference_model + model);
    return fmax(relative, historical);
  }
  __device__ void Accepted(double cost, double model) {
    current_cost = cost;
    acc_candidate_model += model;
    acc_reference_model += model;
    if (current_cost < minimum_cost) {
      minimum_cost = current_cost;
      num_nonmonotonic = 0;
      candidate_cost = current_cost;
      acc_candidate_model = 0.;
    } else {
      ++num_nonmonotonic;
      if (current_cost > candidate_cost) {
        candidate_cost = current_cost;
        acc_candidate_model = 0.;
      }
    }
    if (num_nonmonotonic == max_nonmonotonic) {
      reference_cost = candidate_cost;
      acc_reference_model = acc_candidate_model;
    }
  }
};

// LevenbergMarquardtStrategy radius updates (levenberg_marquardt_strategy.cc).
struct LmRadius {
  double radius = 1e4, decrease = 2.;
  __device__ void Accepted(double quality) {
    const double tf = 2. * quality - 1.;
    radius = fmin(1e16, radius / fmax(1. / 3., 1. - tf * tf * tf));
    decrease = 2.;
  }
  __device__ void Rejected() {
    radius /= decrease;
    decrease *= 2.;
  }
};

}  // namespace csm

#endif  // CSM_CERES_LM_H_
