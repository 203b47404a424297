// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// Geometry restated from the reference's transform/ headers and the Eigen 3.3
// formulas they expand to. Every function names the line it follows.

#include <algorithm>
#include <cmath>

#include "csm_oracle.h"

namespace oracle {

// common/port.h:40-42
int RoundToInt(double x) { return static_cast<int>(std::lround(x)); }
int RoundToIntF(float x) { return static_cast<int>(std::lround(x)); }

// Eigen AngleAxis -> Quaternion (Eigen/src/Geometry/Quaternion.h,
// QuaternionBase::operator=(const AngleAxisType&)): ha = 0.5*angle.
Quatf QuatFromAngleAxisF(float angle, float ax, float ay, float az) {
  const float ha = 0.5f * angle;
  const float s = std::sin(ha);
  return Quatf{std::cos(ha), s * ax, s * ay, s * az};
}

Quatd QuatFromAngleAxisD(double angle, double ax, double ay, double az) {
  const double ha = 0.5 * angle;
  const double s = std::sin(ha);
  return Quatd{std::cos(ha), s * ax, s * ay, s * az};
}

namespace {
// Eigen OrthoMethods.h MatrixBase::cross — coefficient order kept.
template <typename T, typename V>
inline V Cross(T ax, T ay, T az, const V& b) {
  return V{ay * b.z - az * b.y, az * b.x - ax * b.z, ax * b.y - ay * b.x};
}

template <typename Q, typename V>
inline V RotateImpl(const Q& q, const V& v) {
  V uv = Cross(q.x, q.y, q.z, v);
  uv.x += uv.x;
  uv.y += uv.y;
  uv.z += uv.z;
  const V c = Cross(q.x, q.y, q.z, uv);
  return V{(v.x + q.w * uv.x) + c.x, (v.y + q.w * uv.y) + c.y,
           (v.z + q.w * uv.z) + c.z};
}

// Eigen Quaternion product (Quaternion.h quat_product generic path).
template <typename Q>
inline Q QuatMulImpl(const Q& a, const Q& b) {
  return Q{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z,
           a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
           a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
           a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}
}  // namespace

// Eigen QuaternionBase::_transformVector.
Vec3f Rotate(const Quatf& q, const Vec3f& v) { return RotateImpl(q, v); }
Vec3d Rotate(const Quatd& q, const Vec3d& v) { return RotateImpl(q, v); }

Quatf QuatMul(const Quatf& a, const Quatf& b) { return QuatMulImpl(a, b); }
Quatd QuatMul(const Quatd& a, const Quatd& b) { return QuatMulImpl(a, b); }

// Eigen QuaternionBase::normalized -> coeffs / coeffs.norm() (x,y,z,w storage).
Quatf QuatNormalized(const Quatf& q) {
  const float n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);  // SSE predux
  const float n = std::sqrt(n2);
  if (n > 0.f) return Quatf{q.w / n, q.x / n, q.y / n, q.z / n};
  return q;
}
Quatd QuatNormalized(const Quatd& q) {
  const double n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);  // SSE2 packets
  const double n = std::sqrt(n2);
  if (n > 0.) return Quatd{q.w / n, q.x / n, q.y / n, q.z / n};
  return q;
}
Quatd QuatConjugate(const Quatd& q) { return Quatd{q.w, -q.x, -q.y, -q.z}; }

// rigid_transform.h:90-96 with Eigen Rotation2D (toRotationMatrix() * v).
template <typename R, typename T>
static R Mul2(const R& a, const R& b) {
  const T s = std::sin(a.angle), c = std::cos(a.angle);
  R r;
  r.tx = (c * b.tx + (-s) * b.ty) + a.tx;
  r.ty = (s * b.tx + c * b.ty) + a.ty;
  r.angle = a.angle + b.angle;
  return r;
}
Rigid2d Mul(const Rigid2d& a, const Rigid2d& b) {
  return Mul2<Rigid2d, double>(a, b);
}
Rigid2f Mul(const Rigid2f& a, const Rigid2f& b) {
  return Mul2<Rigid2f, float>(a, b);
}

// rigid_transform.h:64-68
template <typename R, typename T>
static R Inverse2(const R& a) {
  const T ang = -a.angle;
  const T s = std::sin(ang), c = std::cos(ang);
  R r;
  r.tx = -(c * a.tx + (-s) * a.ty);
  r.ty = -(s * a.tx + c * a.ty);
  r.angle = ang;
  return r;
}
Rigid2f Inverse(const Rigid2f& a) { return Inverse2<Rigid2f, float>(a); }
Rigid2d Inverse(const Rigid2d& a) { return Inverse2<Rigid2d, double>(a); }

// rigid_transform.h:190-196
Vec3f Apply(const Rigid3f& r, const Vec3f& p) {
  const Vec3f v = Rotate(r.q, p);
  return Vec3f{v.x + r.t.x, v.y + r.t.y, v.z + r.t.z};
}
Vec3d Apply(const Rigid3d& r, const Vec3d& p) {
  const Vec3d v = Rotate(r.q, p);
  return Vec3d{v.x + r.t.x, v.y + r.t.y, v.z + r.t.z};
}

// rigid_transform.h:181-188
Rigid3f Mul(const Rigid3f& a, const Rigid3f& b) {
  return Rigid3f{Apply(a, b.t), QuatNormalized(QuatMul(a.q, b.q))};
}
Rigid3d Mul(const Rigid3d& a, const Rigid3d& b) {
  return Rigid3d{Apply(a, b.t), QuatNormalized(QuatMul(a.q, b.q))};
}

// rigid_transform.h:150-154
Rigid3d Inverse(const Rigid3d& a) {
  const Quatd c = QuatConjugate(a.q);
  const Vec3d t = Rotate(c, a.t);
  return Rigid3d{Vec3d{-t.x, -t.y, -t.z}, c};
}

Rigid3f CastF(const Rigid3d& a) {
  return Rigid3f{Vec3f{static_cast<float>(a.t.x), static_cast<float>(a.t.y),
                       static_cast<float>(a.t.z)},
                 Quatf{static_cast<float>(a.q.w), static_cast<float>(a.q.x),
                       static_cast<float>(a.q.y), static_cast<float>(a.q.z)}};
}

// transform.h:109-115
Rigid3f Embed3D(const Rigid2f& r) {
  return Rigid3f{Vec3f{r.tx, r.ty, 0.f},
                 QuatFromAngleAxisF(r.angle, 0.f, 0.f, 1.f)};
}
Rigid3d Embed3D(const Rigid2d& r) {
  return Rigid3d{Vec3d{r.tx, r.ty, 0.},
                 QuatFromAngleAxisD(r.angle, 0., 0., 1.)};
}

// sensor/point_cloud.cc:56-64
PointCloud TransformPointCloud(const PointCloud& cloud, const Rigid3f& r) {
  PointCloud out;
  out.reserve(cloud.size());
  for (const Vec3f& p : cloud) out.push_back(Apply(r, p));
  return out;
}

// rigid_transform_test_helpers.h:42-46 (Eigen isApprox on affine matrices).
bool IsNearly2D(const Rigid2f& a, const Rigid2f& b, float eps) {
  const float ca = std::cos(a.angle), sa = std::sin(a.angle);
  const float cb = std::cos(b.angle), sb = std::sin(b.angle);
  const float ma[9] = {ca, -sa, a.tx, sa, ca, a.ty, 0.f, 0.f, 1.f};
  const float mb[9] = {cb, -sb, b.tx, sb, cb, b.ty, 0.f, 0.f, 1.f};
  float d2 = 0.f, na = 0.f, nb = 0.f;
  for (int i = 0; i < 9; ++i) {
    d2 += (ma[i] - mb[i]) * (ma[i] - mb[i]);
    na += ma[i] * ma[i];
    nb += mb[i] * mb[i];
  }
  return d2 <= eps * eps * std::min(na, nb);
}

}  // namespace oracle
