// Host-side search-window arithmetic; see search_window.h. Built without
// FP contraction (-ffp-contract=off) so float expressions round per op like
// the x86-64 reference build.

#include "search_window.h"

#include <algorithm>
#include <cmath>

namespace csm {

ZRot MakeZRot(float angle) {
  const float ha = 0.5f * angle;
  return ZRot{std::cos(ha), std::sin(ha)};
}

// uv = q.vec x v; uv += uv; v + q.w*uv + q.vec x uv with q.vec = (0, 0, s).
void RotateZ(const ZRot& q, float x, float y, float* ox, float* oy) {
  const float zero = 0.f;
  const float uvx = zero * 0.f - q.s * y;  // qy*vz - qz*vy (vz = 0 path)
  const float uvy = q.s * x - zero * 0.f;  // qz*vx - qx*vz
  const float ux = uvx + uvx, uy = uvy + uvy;
  const float cx = zero * 0.f - q.s * uy;  // qy*uvz - qz*uvy (uvz = 0)
  const float cy = q.s * ux - zero * 0.f;  // qz*uvx - qx*uvz
  *ox = (x + q.w * ux) + cx;
  *oy = (y + q.w * uy) + cy;
}

SearchWindow2D MakeSearchWindow2D(double linear_window, double angular_window,
                                  const float* xyz, int32_t n, double res,
                                  const ZRot* pre) {
  SearchWindow2D w;
  float max_scan_range = 3.f * res;  // double product narrowed to float
  for (int32_t i = 0; i < n; ++i) {
    float x = xyz[3 * i], y = xyz[3 * i + 1];
    if (pre) RotateZ(*pre, x, y, &x, &y);
    const float range = std::sqrt(x * x + y * y);
    max_scan_range = std::max(range, max_scan_range);
  }
  const double kSafetyMargin = 1. - 1e-3;
  const float range_sq = max_scan_range * max_scan_range;  // common::Pow2(float)
  w.angular_perturbation_step_size =
      kSafetyMargin * std::acos(1. - (res * res) / (2. * range_sq));
  w.num_angular_perturbations =
      static_cast<int>(std::ceil(angular_window / w.angular_perturbation_step_size));
  w.num_scans = 2 * w.num_angular_perturbations + 1;
  const double lin = std::ceil(linear_window / res);
  w.num_linear_perturbations = lin > 2e9 ? 2000000000 : static_cast<int>(lin);
  return w;
}

void RotationTable(const SearchWindow2D& w, std::vector<ZRot>* out) {
  out->resize(w.num_scans);
  double theta = -w.num_angular_perturbations * w.angular_perturbation_step_size;
  for (int s = 0; s < w.num_scans; ++s, theta += w.angular_perturbation_step_size)
    (*out)[s] = MakeZRot(static_cast<float>(theta));
}

bool QuantizationTable(float min_cc, float max_cc, uint8_t* out) {
  const float scale = (max_cc - min_cc) / 32766.f;
  const float min_s = 1.f - max_cc, max_s = 1.f - min_cc;
  for (int v = 0; v < 32768; ++v) {
    const float cc = v == 0 ? max_cc : v * scale + (min_cc - scale);
    const float p = 1.f - std::abs(cc);
    const long q = std::lround((p - min_s) * (255.f / (max_s - min_s)));
    if (q < 0 || q > 255) return false;
    out[v] = static_cast<uint8_t>(q);
  }
  return true;
}

void ProbabilityTable(float* out) {
  const float kMinP = 0.1f;
  const float kMaxP = 1.f - kMinP;
  const float lo = 1.f - kMaxP, hi = 1.f - kMinP;  // min/max correspondence cost
  const float scale = (hi - lo) / 32766.f;
  for (int v = 0; v < 32768; ++v) {
    const float cc = v == 0 ? hi : v * scale + (lo - scale);
    out[v] = 1.f - cc;
  }
}

void ConversionTable(float unknown_result, float lower, float upper, float* out) {
  const float scale = (upper - lower) / 32766.f;
  for (int v = 0; v < 32768; ++v) out[v] = v == 0 ? unknown_result : v * scale + (lower - scale);
}

float SumToScore(int64_t sum, int32_t n, float min_s, float max_s) {
  const float mean = static_cast<int>(sum) / static_cast<float>(n);
  return min_s + mean * ((max_s - min_s) / 255.f);
}

int64_t MaxRejectedSum(float min_score, int32_t n, float min_s, float max_s) {
  // Score is non-decreasing in sum: binary search the last sum <= min_score.
  int64_t lo = -1, hi = static_cast<int64_t>(n) * 255;  // invariant: lo rejected
  if (SumToScore(hi, n, min_s, max_s) <= min_score) return hi;
  while (hi - lo > 1) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (SumToScore(mid, n, min_s, max_s) <= min_score)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

}  // namespace csm
