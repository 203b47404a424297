// Device restatements of the 2D discretization arithmetic shared by the
// FastCSM2D search kernels (csm_kernels.hip) and the RTCSM2D kernels
// (rt2d.hip), bit-exact with the reference's x86-64 float/double semantics
// (DESIGN.md "Bitwise discretization"; build with -ffp-contract=off).
#ifndef CSM_GEOM2D_DEV_H_
#define CSM_GEOM2D_DEV_H_

#include <hip/hip_runtime.h>

namespace csm {

// Eigen QuaternionBase::_transformVector with q.vec = (0, 0, s)
// (GenerateRotatedScans' AngleAxisf rotation, correlative_scan_matcher_2d.cc:99-106).
__device__ __forceinline__ void RotateZDev(float w, float s, float x, float y, float* ox,
                                           float* oy) {
  const float uvx = __fsub_rn(0.f, __fmul_rn(s, y));
  const float uvy = __fsub_rn(__fmul_rn(s, x), 0.f);
  const float ux = __fadd_rn(uvx, uvx);
  const float uy = __fadd_rn(uvy, uvy);
  const float cx = __fsub_rn(0.f, __fmul_rn(s, uy));
  const float cy = __fsub_rn(__fmul_rn(s, ux), 0.f);
  *ox = __fadd_rn(__fadd_rn(x, __fmul_rn(w, ux)), cx);
  *oy = __fadd_rn(__fadd_rn(y, __fmul_rn(w, uy)), cy);
}

// MapLimits::GetCellIndex (map_limits.h:69-75): lround((max - p) / resolution
// - 0.5) in double.
__device__ __forceinline__ double CellCoord(double max_v, float p, double res) {
  return __builtin_round(
      __dsub_rn(__ddiv_rn(__dsub_rn(max_v, static_cast<double>(p)), res), 0.5));
}

// CellCoord from the double reciprocal of the resolution: q' = (max - p) *
// fl(1/res) is within 2^-52 relative (< 2.2e-10 absolute for |q'| < 2^20) of
// the IEEE quotient q. Away from an integer by more than that, q and q' have
// the same floor, fl(q) - 0.5 is exact and not a half-integer, and lround
// gives floor(q); within 1e-9 of an integer, or for |q'| >= 2^20, the exact
// CellCoord decides. Same result as CellCoord for every input.
__device__ __forceinline__ double CellCoordFast(double max_v, float p, double res, double inv_res) {
  const double d = __dsub_rn(max_v, static_cast<double>(p));
  const double q = __dmul_rn(d, inv_res);
  const double k = floor(q);
  if (fabs(q) < 1048576.0 && q - k > 1e-9 && (k + 1.0) - q > 1e-9) return k;
  return __builtin_round(__dsub_rn(__ddiv_rn(d, res), 0.5));
}

}  // namespace csm

#endif  // CSM_GEOM2D_DEV_H_
