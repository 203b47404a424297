// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// Pieces of Ceres 1.13's TrustRegionMinimizer (the version the reference
// installs, scripts/install_ceres.sh:20) shared by the CeresScanMatcher2D/3D
// restatements (ceres2d.cc, ceres3d.cc). Ceres is not in this image.
#ifndef ORACLE_CERES_MINIMIZER_H_
#define ORACLE_CERES_MINIMIZER_H_

#include <algorithm>

namespace oracle {

// Ceres' TrustRegionStepEvaluator (trust_region_step_evaluator.cc, Conn,
// Gould & Toint Algorithm 10.1.2): step quality against the current and a
// reference cost, so that up to max_consecutive_nonmonotonic_steps (5) steps
// may raise the cost when use_nonmonotonic_steps is set (0 otherwise).
struct StepEvaluator {
  double reference_cost, minimum_cost, current_cost, candidate_cost;
  double acc_reference_model = 0., acc_candidate_model = 0.;
  int num_nonmonotonic = 0, max_nonmonotonic;
  StepEvaluator(double cost, int max_steps)
      : reference_cost(cost), minimum_cost(cost), current_cost(cost), candidate_cost(cost),
        max_nonmonotonic(max_steps) {}
  double Quality(double cost, double model) const {
    const double relative = (current_cost - cost) / model;
    const double historical = (reference_cost - cost) / (acc_reference_model + model);
    return std::max(relative, historical);
  }
  void Accepted(double cost, double model) {
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

}  // namespace oracle

#endif  // ORACLE_CERES_MINIMIZER_H_
