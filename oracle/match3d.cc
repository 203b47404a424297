// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
// RotationalScanMatcher, low-resolution matcher, FastCorrelativeScanMatcher3D
// and RealTimeCorrelativeScanMatcher3D, restated from the reference.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <map>

#include "oracle3d.h"

namespace oracle {

// ------------------------------------------------------------ Eigen float --
// Geometry_SSE.h quat_product<SSE, float>: coefficients in (x, y, z, w)
// order, res = a*b.w - swz(a)*swz(b) + (+,+,+,-)(s1 + s2).
Quatf QuatMulSse(const Quatf& a, const Quatf& b) {
  Quatf r;
  r.x = (a.x * b.w - a.z * b.y) + (a.y * b.z + a.w * b.x);
  r.y = (a.y * b.w - a.x * b.z) + (a.z * b.x + a.w * b.y);
  r.z = (a.z * b.w - a.y * b.x) + (a.x * b.y + a.w * b.z);
  r.w = (a.w * b.w - a.x * b.x) - (a.z * b.z + a.y * b.y);
  return r;
}

// MatrixBase::normalized on the (x, y, z, w) coefficient packet: squaredNorm
// via predux = (x²+z²)+(y²+w²), then each coefficient / sqrt.
Quatf QuatNormalizedSse(const Quatf& q) {
  const float n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
  if (n2 > 0.f) {
    const float n = std::sqrt(n2);
    return Quatf{q.w / n, q.x / n, q.y / n, q.z / n};
  }
  return q;
}

Quatf QuatConjugateF(const Quatf& q) { return Quatf{q.w, -q.x, -q.y, -q.z}; }

// Quaternion::inverse: conjugate().coeffs() / squaredNorm.
Quatf QuatInverseSse(const Quatf& q) {
  const float n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
  if (n2 > 0.f) return Quatf{q.w / n2, -q.x / n2, -q.y / n2, -q.z / n2};
  return Quatf{0.f, 0.f, 0.f, 0.f};
}

static Quatd QuatInverseD(const Quatd& q) {
  const double n2 = (q.x * q.x + q.z * q.z) + (q.y * q.y + q.w * q.w);
  if (n2 > 0.) return Quatd{q.w / n2, -q.x / n2, -q.y / n2, -q.z / n2};
  return Quatd{0., 0., 0., 0.};
}

// Redux.h LinearVectorizedTraversal with 4-float packets (aligned storage).
float ReduxSumSse(const float* v, int n) {
  const int aligned2 = (n / 8) * 8, aligned = (n / 4) * 4;
  if (aligned == 0) {
    if (n == 0) return 0.f;
    float r = v[0];
    for (int i = 1; i < n; ++i) r += v[i];
    return r;
  }
  float p0[4] = {v[0], v[1], v[2], v[3]};
  if (aligned > 4) {
    float p1[4] = {v[4], v[5], v[6], v[7]};
    for (int i = 8; i < aligned2; i += 8)
      for (int k = 0; k < 4; ++k) {
        p0[k] += v[i + k];
        p1[k] += v[i + 4 + k];
      }
    for (int k = 0; k < 4; ++k) p0[k] += p1[k];
    if (aligned > aligned2)
      for (int k = 0; k < 4; ++k) p0[k] += v[aligned2 + k];
  }
  float r = (p0[0] + p0[2]) + (p0[1] + p0[3]);
  for (int i = aligned; i < n; ++i) r += v[i];
  return r;
}

float DotSse(const std::vector<float>& a, const std::vector<float>& b) {
  std::vector<float> p(a.size());
  for (size_t i = 0; i < a.size(); ++i) p[i] = a[i] * b[i];
  return ReduxSumSse(p.data(), static_cast<int>(p.size()));
}

float NormSse(const std::vector<float>& a) { return std::sqrt(DotSse(a, a)); }

Vec3f Rotate3(const Quatf& q, const Vec3f& v) { return Rotate(q, v); }

Vec3f Apply3(const Rigid3f& r, const Vec3f& p) {
  const Vec3f v = Rotate(r.q, p);
  return Vec3f{v.x + r.t.x, v.y + r.t.y, v.z + r.t.z};
}

Rigid3f Mul3(const Rigid3f& a, const Rigid3f& b) {
  return Rigid3f{Apply3(a, b.t), QuatNormalizedSse(QuatMulSse(a.q, b.q))};
}

Rigid3f Inverse3(const Rigid3f& a) {
  const Quatf c = QuatConjugateF(a.q);
  const Vec3f t = Rotate(c, a.t);
  return Rigid3f{Vec3f{-t.x, -t.y, -t.z}, c};
}

// Vector3f::norm(): Eigen unrolls a 3-element sum as x0 + (x1 + x2)
// (Redux.h redux_novec_unroller splits at Length / 2).
float NormF(const Vec3f& v) { return std::sqrt(v.x * v.x + (v.y * v.y + v.z * v.z)); }

Quatf AngleAxisVectorToRotationQuaternionF(const Vec3f& aa) {
  float scale = 0.5f, w = 1.f;
  const float sq = aa.x * aa.x + (aa.y * aa.y + aa.z * aa.z);
  if (sq > 1e-8) {
    const float norm = std::sqrt(sq);
    scale = static_cast<float>(std::sin(norm / 2.) / norm);
    w = static_cast<float>(std::cos(norm / 2.));
  }
  return Quatf{w, scale * aa.x, scale * aa.y, scale * aa.z};
}

float GetAngleF(const Quatf& q) {
  const float vn = std::sqrt(q.x * q.x + (q.y * q.y + q.z * q.z));
  return 2.f * std::atan2(vn, std::abs(q.w));
}

// transform.h:43-47: unqualified atan2 on floats resolves to the C double
// ::atan2 (libstdc++ <cmath> puts the float overloads only in std).
float GetYawF(const Quatf& q) {
  const Vec3f d = Rotate(q, Vec3f{1.f, 0.f, 0.f});
  return static_cast<float>(::atan2(static_cast<double>(d.y), static_cast<double>(d.x)));
}

static Rigid3f CastRigidF(const Rigid3d& a) {
  return Rigid3f{Vec3f{static_cast<float>(a.t.x), static_cast<float>(a.t.y),
                       static_cast<float>(a.t.z)},
                 Quatf{static_cast<float>(a.q.w), static_cast<float>(a.q.x),
                       static_cast<float>(a.q.y), static_cast<float>(a.q.z)}};
}
static Rigid3d CastRigidD(const Rigid3f& a) {
  return Rigid3d{Vec3d{a.t.x, a.t.y, a.t.z}, Quatd{a.q.w, a.q.x, a.q.y, a.q.z}};
}

// -------------------------------------------------- rotational_scan_matcher --
namespace {
constexpr float kMinDistance = 0.2f, kMaxDistance = 0.9f, kSliceHeight = 0.2f;
const float kPiF = static_cast<float>(M_PI);

void AddValueToHistogram(float angle, float value, std::vector<float>* h) {  // :34-49
  while (angle > kPiF) angle -= kPiF;
  while (angle < 0.f) angle += kPiF;
  const float zero_to_one = angle / kPiF;
  const int size = static_cast<int>(h->size());
  const int bucket =
      std::min(std::max(RoundToIntF(static_cast<float>(size) * zero_to_one - 0.5f), 0), size - 1);
  (*h)[bucket] += value;
}

Vec3f Centroid(const PointCloud& slice) {  // :51-58
  Vec3f s{0.f, 0.f, 0.f};
  for (const Vec3f& p : slice) {
    s.x += p.x;
    s.y += p.y;
    s.z += p.z;
  }
  const float n = static_cast<float>(slice.size());
  return Vec3f{s.x / n, s.y / n, s.z / n};
}

float Norm2(float x, float y) { return std::sqrt(x * x + y * y); }

void AddSlice(const PointCloud& slice, std::vector<float>* h) {  // :60-88
  if (slice.empty()) return;
  const Vec3f c = Centroid(slice);
  Vec3f last = slice.front();
  for (const Vec3f& p : slice) {
    const float dx = p.x - last.x, dy = p.y - last.y;
    const float rx = p.x - c.x, ry = p.y - c.y;
    const float distance = Norm2(dx, dy);
    if (distance < kMinDistance || Norm2(rx, ry) < kMinDistance) continue;
    if (distance > kMaxDistance) {
      last = p;
      continue;
    }
    const float angle = std::atan2(dy, dx);
    const float dn = Norm2(dx, dy), rn = Norm2(rx, ry);
    const float dot = (dx / dn) * (rx / rn) + (dy / dn) * (ry / rn);
    const float value = std::max(0.f, 1.f - std::abs(dot));
    AddValueToHistogram(angle, value, h);
  }
}

PointCloud SortSlice(const PointCloud& slice) {  // :92-117
  struct Pair {
    bool operator<(const Pair& o) const { return angle < o.angle; }
    float angle;
    Vec3f point;
  };
  const Vec3f c = Centroid(slice);
  std::vector<Pair> by_angle;
  by_angle.reserve(slice.size());
  for (const Vec3f& p : slice) {
    const float dx = p.x - c.x, dy = p.y - c.y;
    if (Norm2(dx, dy) < kMinDistance) continue;
    by_angle.push_back(Pair{std::atan2(dy, dx), p});
  }
  std::sort(by_angle.begin(), by_angle.end());
  PointCloud out;
  for (const Pair& q : by_angle) out.push_back(q.point);
  return out;
}
}  // namespace

float MatchHistograms(const std::vector<float>& submap, const std::vector<float>& scan) {
  const float scan_norm = NormSse(scan);  // :119-131
  const float submap_norm = NormSse(submap);
  const float normalization = scan_norm * submap_norm;
  if (normalization < 1e-3f) return 1.f;
  return DotSse(submap, scan) / normalization;
}

std::vector<float> RotateHistogram(const std::vector<float>& h, float angle) {  // :138-158
  if (h.empty()) return h;
  const int size = static_cast<int>(h.size());
  const float rotate_by_buckets =
      static_cast<float>(static_cast<double>(-angle * static_cast<float>(size)) / M_PI);
  int full_buckets = RoundToIntF(rotate_by_buckets - 0.5f);
  const float fraction = rotate_by_buckets - static_cast<float>(full_buckets);
  while (full_buckets < 0) full_buckets += size;
  std::vector<float> out(size);
  for (int i = 0; i != size; ++i) {
    const float r0 = h[(i + full_buckets) % size];
    const float r1 = h[(i + 1 + full_buckets) % size];
    out[i] = fraction * r1 + (1.f - fraction) * r0;
  }
  return out;
}

std::vector<float> ComputeHistogram(const PointCloud& cloud, int histogram_size) {  // :160-171
  std::vector<float> h(histogram_size, 0.f);
  std::map<int, PointCloud> slices;
  for (const Vec3f& p : cloud) slices[RoundToIntF(p.z / kSliceHeight)].push_back(p);
  for (const auto& s : slices) AddSlice(SortSlice(s.second), &h);
  return h;
}

std::vector<float> RotationalMatch(const std::vector<float>& submap_histogram,
                                   const std::vector<float>& histogram, float initial_angle,
                                   const std::vector<float>& angles) {  // :173-185
  std::vector<float> result;
  result.reserve(angles.size());
  for (const float a : angles)
    result.push_back(MatchHistograms(submap_histogram, RotateHistogram(histogram, initial_angle + a)));
  return result;
}

// low_resolution_matcher.cc:23-35
float LowResolutionScore(const HybridGrid& grid, const PointCloud& points, const Rigid3f& pose) {
  float score = 0.f;
  for (const Vec3f& p : points) score += grid.GetProbability(grid.GetCellIndex(Apply3(pose, p)));
  return score / static_cast<float>(points.size());
}

// ------------------------------------------------ FastCorrelativeScanMatcher3D --
// fast_correlative_scan_matcher_3d.cc:57-77, :112-123
FastCorrelativeScanMatcher3D::FastCorrelativeScanMatcher3D(const HybridGrid& hybrid_grid,
                                                           const HybridGrid* low_resolution_grid,
                                                           const std::vector<float>* histogram,
                                                           const FastCsm3dOptions& options)
    : options_(options),
      resolution_(hybrid_grid.resolution()),
      width_in_voxels_(hybrid_grid.grid_size()),
      low_resolution_grid_(low_resolution_grid),
      histogram_(histogram) {
  levels_.push_back(ConvertToPrecomputationGrid(hybrid_grid));
  int last_width = 1;
  for (int depth = 1; depth != options.branch_and_bound_depth; ++depth) {
    const bool half = depth >= options.full_resolution_depth;
    const int next_width = 1 << depth;
    const int f = 1 << std::max(0, depth - options.full_resolution_depth);
    const int s = (next_width - last_width + (f - 1)) / f;
    levels_.push_back(PrecomputeGrid(*levels_.back(), half, Idx3{s, s, s}));
    last_width = next_width;
  }
}

// Search parameters and poses of Match (:127-143) / MatchFullSubmap (:145-170).
void FastCorrelativeScanMatcher3D::Setup(bool full_submap, const Rigid3d& node_pose,
                                         const Rigid3d& submap_pose, const NodeData3D& node,
                                         SearchParameters* sp, Rigid3f* np, Rigid3f* spf) const {
  if (!full_submap) {
    *sp = SearchParameters{RoundToInt(options_.linear_xy_search_window / resolution_),
                           RoundToInt(options_.linear_z_search_window / resolution_),
                           options_.angular_search_window};
    *np = CastRigidF(node_pose);
    *spf = CastRigidF(submap_pose);
    return;
  }
  float max_point_distance = 0.f;
  for (const Vec3f& p : node.high_resolution_point_cloud)
    max_point_distance = std::max(max_point_distance, NormF(p));
  const int lws = (width_in_voxels_ + 1) / 2 + RoundToIntF(max_point_distance / resolution_ + 0.5f);
  *sp = SearchParameters{lws, lws, M_PI};
  *np = CastRigidF(Rigid3d{Vec3d{0., 0., 0.}, node_pose.q});
  *spf = CastRigidF(Rigid3d{Vec3d{0., 0., 0.}, submap_pose.q});
}

bool FastCorrelativeScanMatcher3D::EvaluateLeaf(bool full_submap, const Rigid3d& node_pose,
                                                const Rigid3d& submap_pose, const NodeData3D& node,
                                                const Rigid3d& pose, Fast3dResult* out) const {
  SearchParameters sp;
  Rigid3f np, spf;
  Setup(full_submap, node_pose, submap_pose, node, &sp, &np, &spf);
  const std::vector<DiscreteScan3D> scans =
      GenerateDiscreteScans(sp, node.high_resolution_point_cloud,
                            node.rotational_scan_matcher_histogram, node.gravity_alignment, np, spf);
  const Rigid3f want = CastRigidF(pose);
  for (int k = 0; k < static_cast<int>(scans.size()); ++k) {
    Candidate3D c;
    c.scan_index = k;
    const Rigid3f base = GetPoseFromCandidate(scans, c);
    if (base.q.w != want.q.w || base.q.x != want.q.x || base.q.y != want.q.y ||
        base.q.z != want.q.z)
      continue;
    c.offset = Idx3{RoundToIntF((want.t.x - base.t.x) / resolution_),
                    RoundToIntF((want.t.y - base.t.y) / resolution_),
                    RoundToIntF((want.t.z - base.t.z) / resolution_)};
    const Rigid3f got = GetPoseFromCandidate(scans, c);
    if (got.t.x != want.t.x || got.t.y != want.t.y || got.t.z != want.t.z) continue;
    if (std::abs(c.offset.x) > sp.linear_xy_window_size ||
        std::abs(c.offset.y) > sp.linear_xy_window_size ||
        std::abs(c.offset.z) > sp.linear_z_window_size)
      continue;
    std::vector<Candidate3D> one{c};
    ScoreCandidates(0, scans, &one, &out->lookups);
    out->matched = true;
    out->score = one[0].score;
    out->pose = CastRigidD(got);
    out->rotational_score = scans[k].rotational_score;
    out->low_resolution_score =
        LowResolutionScore(*low_resolution_grid_, node.low_resolution_point_cloud, got);
    return true;
  }
  return false;
}

// :127-143
Fast3dResult FastCorrelativeScanMatcher3D::Match(const Rigid3d& global_node_pose,
                                                 const Rigid3d& global_submap_pose,
                                                 const NodeData3D& node, float min_score) const {
  const SearchParameters sp{RoundToInt(options_.linear_xy_search_window / resolution_),
                            RoundToInt(options_.linear_z_search_window / resolution_),
                            options_.angular_search_window};
  return MatchWithSearchParameters(sp, CastRigidF(global_node_pose),
                                   CastRigidF(global_submap_pose), node, min_score);
}

// :145-170
Fast3dResult FastCorrelativeScanMatcher3D::MatchFullSubmap(const Quatd& node_rotation,
                                                           const Quatd& submap_rotation,
                                                           const NodeData3D& node,
                                                           float min_score) const {
  float max_point_distance = 0.f;
  for (const Vec3f& p : node.high_resolution_point_cloud)
    max_point_distance = std::max(max_point_distance, NormF(p));
  const int lws = (width_in_voxels_ + 1) / 2 + RoundToIntF(max_point_distance / resolution_ + 0.5f);
  const SearchParameters sp{lws, lws, M_PI};
  const Rigid3d node_pose{Vec3d{0., 0., 0.}, node_rotation};
  const Rigid3d submap_pose{Vec3d{0., 0., 0.}, submap_rotation};
  return MatchWithSearchParameters(sp, CastRigidF(node_pose), CastRigidF(submap_pose), node,
                                   min_score);
}

// :172-199
Fast3dResult FastCorrelativeScanMatcher3D::MatchWithSearchParameters(
    const SearchParameters& sp, const Rigid3f& global_node_pose,
    const Rigid3f& global_submap_pose, const NodeData3D& node, float min_score) const {
  Fast3dResult out;
  const std::vector<DiscreteScan3D> scans =
      GenerateDiscreteScans(sp, node.high_resolution_point_cloud,
                            node.rotational_scan_matcher_histogram, node.gravity_alignment,
                            global_node_pose, global_submap_pose);
  out.num_discrete_scans = static_cast<int>(scans.size());
  // GenerateLowestResolutionCandidates :297-330
  const int max_depth = num_levels() - 1;
  const int step = 1 << max_depth;
  std::vector<Candidate3D> candidates;
  for (int k = 0; k != static_cast<int>(scans.size()); ++k)
    for (int z = -sp.linear_z_window_size; z <= sp.linear_z_window_size; z += step)
      for (int y = -sp.linear_xy_window_size; y <= sp.linear_xy_window_size; y += step)
        for (int x = -sp.linear_xy_window_size; x <= sp.linear_xy_window_size; x += step) {
          Candidate3D c;
          c.scan_index = k;
          c.offset = Idx3{x, y, z};
          candidates.push_back(c);
        }
  ScoreCandidates(max_depth, scans, &candidates, &out.lookups);
  const Candidate3D best =
      BranchAndBound(sp, scans, candidates, max_depth, min_score, node, &out);
  if (best.score > min_score) {
    out.matched = true;
    out.score = best.score;
    out.pose = CastRigidD(GetPoseFromCandidate(scans, best));
    out.rotational_score = scans[best.scan_index].rotational_score;
    out.low_resolution_score = best.low_resolution_score;
  }
  return out;
}

// :201-244
FastCorrelativeScanMatcher3D::DiscreteScan3D FastCorrelativeScanMatcher3D::DiscretizeScan(
    const SearchParameters& sp, const PointCloud& cloud, const Rigid3f& pose,
    float rotational_score) const {
  std::vector<std::vector<Idx3>> per_depth;
  const PrecomputationGrid3D& g0 = *levels_[0];
  std::vector<Idx3> full;
  for (const Vec3f& p : cloud) full.push_back(g0.GetCellIndex(Apply3(pose, p)));
  const int frd = std::min(options_.full_resolution_depth, options_.branch_and_bound_depth);
  for (int i = 0; i != frd; ++i) per_depth.push_back(full);
  const int lrd = options_.branch_and_bound_depth - frd;
  const Idx3 ws{-sp.linear_xy_window_size, -sp.linear_xy_window_size, -sp.linear_z_window_size};
  for (int i = 0; i != lrd; ++i) {
    const int e = i + 1;
    const Idx3 lws{ws.x >> e, ws.y >> e, ws.z >> e};
    per_depth.emplace_back();
    for (const Idx3& c : full)
      per_depth.back().push_back(Idx3{((c.x + ws.x) >> e) - lws.x, ((c.y + ws.y) >> e) - lws.y,
                                      ((c.z + ws.z) >> e) - lws.z});
  }
  return DiscreteScan3D{pose, per_depth, rotational_score};
}

// :246-295
std::vector<FastCorrelativeScanMatcher3D::DiscreteScan3D>
FastCorrelativeScanMatcher3D::GenerateDiscreteScans(const SearchParameters& sp,
                                                    const PointCloud& cloud,
                                                    const std::vector<float>& histogram,
                                                    const Quatd& gravity_alignment,
                                                    const Rigid3f& global_node_pose,
                                                    const Rigid3f& global_submap_pose) const {
  std::vector<DiscreteScan3D> result;
  float max_scan_range = 3.f * resolution_;
  for (const Vec3f& p : cloud) max_scan_range = std::max(NormF(p), max_scan_range);
  const float kSafetyMargin = 1.f - 1e-2f;
  const float step = kSafetyMargin * std::acos(1.f - (resolution_ * resolution_) /
                                                         (2.f * (max_scan_range * max_scan_range)));
  const int window = RoundToInt(sp.angular_search_window / step);
  std::vector<float> angles;
  for (int rz = -window; rz <= window; ++rz) angles.push_back(static_cast<float>(rz) * step);
  const Rigid3f node_to_submap = Mul3(Inverse3(global_submap_pose), global_node_pose);
  const Quatd gi = QuatInverseD(gravity_alignment);
  const Quatf gif{static_cast<float>(gi.w), static_cast<float>(gi.x), static_cast<float>(gi.y),
                  static_cast<float>(gi.z)};
  const std::vector<float> scores = RotationalMatch(
      *histogram_, histogram, GetYawF(QuatMulSse(node_to_submap.q, gif)), angles);
  for (size_t i = 0; i != angles.size(); ++i) {
    if (scores[i] < options_.min_rotational_score) continue;
    const Quatf yaw = AngleAxisVectorToRotationQuaternionF(Vec3f{0.f, 0.f, angles[i]});
    const Rigid3f pose{node_to_submap.t,
                       QuatMulSse(QuatMulSse(QuatInverseSse(global_submap_pose.q), yaw),
                                  global_node_pose.q)};
    result.push_back(DiscretizeScan(sp, cloud, pose, scores[i]));
  }
  return result;
}

// :332-355
void FastCorrelativeScanMatcher3D::ScoreCandidates(int depth,
                                                   const std::vector<DiscreteScan3D>& scans,
                                                   std::vector<Candidate3D>* candidates,
                                                   int64_t* lookups) const {
  const int e = std::max(0, depth - options_.full_resolution_depth + 1);
  const PrecomputationGrid3D& g = *levels_[depth];
  for (Candidate3D& c : *candidates) {
    int sum = 0;
    const DiscreteScan3D& s = scans[c.scan_index];
    const Idx3 off{c.offset.x >> e, c.offset.y >> e, c.offset.z >> e};
    const std::vector<Idx3>& cells = s.cell_indices_per_depth[depth];
    for (const Idx3& ci : cells) sum += g.value(Idx3{ci.x + off.x, ci.y + off.y, ci.z + off.z});
    *lookups += static_cast<int64_t>(cells.size());
    c.score = ToProbability3D(static_cast<float>(sum) / static_cast<float>(cells.size()));
  }
  std::sort(candidates->begin(), candidates->end(),
            [](const Candidate3D& a, const Candidate3D& b) { return a.score > b.score; });
}

// :369-375
Rigid3f FastCorrelativeScanMatcher3D::GetPoseFromCandidate(const std::vector<DiscreteScan3D>& scans,
                                                           const Candidate3D& c) const {
  const Rigid3f t{Vec3f{resolution_ * static_cast<float>(c.offset.x),
                        resolution_ * static_cast<float>(c.offset.y),
                        resolution_ * static_cast<float>(c.offset.z)},
                  Quatf{1.f, 0.f, 0.f, 0.f}};
  return Mul3(t, scans[c.scan_index].pose);
}

// :377-440
FastCorrelativeScanMatcher3D::Candidate3D FastCorrelativeScanMatcher3D::BranchAndBound(
    const SearchParameters& sp, const std::vector<DiscreteScan3D>& scans,
    const std::vector<Candidate3D>& candidates, int depth, float min_score,
    const NodeData3D& node, Fast3dResult* stats) const {
  if (depth == 0) {
    for (const Candidate3D& c : candidates) {
      if (c.score <= min_score) return Candidate3D();
      ++stats->low_resolution_checks;
      const float lrs = LowResolutionScore(*low_resolution_grid_, node.low_resolution_point_cloud,
                                           GetPoseFromCandidate(scans, c));
      if (lrs >= options_.min_low_resolution_score) {
        Candidate3D best = c;
        best.low_resolution_score = lrs;
        return best;
      }
    }
    return Candidate3D();
  }
  Candidate3D best;
  best.score = min_score;
  for (const Candidate3D& c : candidates) {
    if (c.score <= min_score) break;
    std::vector<Candidate3D> children;
    const int hw = 1 << (depth - 1);
    for (int z : {0, hw}) {
      if (c.offset.z + z > sp.linear_z_window_size) break;
      for (int y : {0, hw}) {
        if (c.offset.y + y > sp.linear_xy_window_size) break;
        for (int x : {0, hw}) {
          if (c.offset.x + x > sp.linear_xy_window_size) break;
          Candidate3D ch;
          ch.scan_index = c.scan_index;
          ch.offset = Idx3{c.offset.x + x, c.offset.y + y, c.offset.z + z};
          children.push_back(ch);
        }
      }
    }
    ScoreCandidates(depth - 1, scans, &children, &stats->lookups);
    const Candidate3D r = BranchAndBound(sp, scans, children, depth - 1, best.score, node, stats);
    if (best.score < r.score) best = r;  // std::max keeps the first on ties
  }
  return best;
}

// ------------------------------------------- RealTimeCorrelativeScanMatcher3D --
// real_time_correlative_scan_matcher_3d.cc:55-95 (window geometry)
void RealTime3DWindow(const RtOptions3D& o, float resolution, const PointCloud& cloud,
                      int* linear_window, float* angular_step, int* angular_window) {
  *linear_window = RoundToInt(o.linear_search_window / resolution);
  float max_scan_range = 3.f * resolution;
  for (const Vec3f& p : cloud) max_scan_range = std::max(NormF(p), max_scan_range);
  const float kSafetyMargin = 1.f - 1e-3f;
  *angular_step = kSafetyMargin * std::acos(1.f - (resolution * resolution) /
                                                      (2.f * (max_scan_range * max_scan_range)));
  *angular_window = RoundToInt(o.angular_search_window / *angular_step);
}

namespace {
struct Rt3dGeometry {
  int L, A;
  float step, res;
};

Rigid3f RtTransform(const Rt3dGeometry& g, int64_t index) {
  const int64_t na = 2 * g.A + 1, nl = 2 * g.L + 1;
  int64_t r = index;
  const int rx = static_cast<int>(r % na) - g.A;
  r /= na;
  const int ry = static_cast<int>(r % na) - g.A;
  r /= na;
  const int rz = static_cast<int>(r % na) - g.A;
  r /= na;
  const int x = static_cast<int>(r % nl) - g.L;
  r /= nl;
  const int y = static_cast<int>(r % nl) - g.L;
  r /= nl;
  const int z = static_cast<int>(r) - g.L;
  const Vec3f aa{static_cast<float>(rx) * g.step, static_cast<float>(ry) * g.step,
                 static_cast<float>(rz) * g.step};
  return Rigid3f{Vec3f{static_cast<float>(x) * g.res, static_cast<float>(y) * g.res,
                       static_cast<float>(z) * g.res},
                 AngleAxisVectorToRotationQuaternionF(aa)};
}

// :97-113
float RtScore(const RtOptions3D& o, const HybridGrid& grid, const PointCloud& cloud,
              const Rigid3f& candidate, const Rigid3f& transform) {
  float score = 0.f;
  for (const Vec3f& p : cloud) score += grid.GetProbability(grid.GetCellIndex(Apply3(candidate, p)));
  score /= static_cast<float>(cloud.size());
  const float angle = GetAngleF(transform.q);
  const double e = static_cast<double>(NormF(transform.t)) * o.translation_delta_cost_weight +
                   static_cast<double>(angle) * o.rotation_delta_cost_weight;
  score = static_cast<float>(static_cast<double>(score) * std::exp(-(e * e)));
  return score;
}
}  // namespace

float RealTimeScore3D(const RtOptions3D& o, const Rigid3d& initial, const PointCloud& cloud,
                      const HybridGrid& grid, int64_t index, Rigid3f* candidate_out) {
  Rt3dGeometry g;
  g.res = grid.resolution();
  RealTime3DWindow(o, g.res, cloud, &g.L, &g.step, &g.A);
  const Rigid3f t = RtTransform(g, index);
  const Rigid3f candidate = Mul3(CastRigidF(initial), t);
  if (candidate_out) *candidate_out = candidate;
  return RtScore(o, grid, cloud, candidate, t);
}

double RealTimeTime3D(const RtOptions3D& o, const Rigid3d& initial, const PointCloud& cloud,
                      const HybridGrid& grid, int64_t count, int64_t stride, float* sink) {
  Rt3dGeometry g;
  g.res = grid.resolution();
  RealTime3DWindow(o, g.res, cloud, &g.L, &g.step, &g.A);
  const Rigid3f init = CastRigidF(initial);
  const auto t0 = std::chrono::steady_clock::now();
  float acc = 0.f;
  for (int64_t i = 0; i < count; ++i) {
    const Rigid3f t = RtTransform(g, i * stride);
    const Rigid3f candidate = Mul3(init, t);
    // ScoreCandidate on TransformPointCloud(point_cloud, candidate) (:41-44).
    const PointCloud transformed = TransformPointCloud(cloud, candidate);
    float score = 0.f;
    for (const Vec3f& p : transformed) score += grid.GetProbability(grid.GetCellIndex(p));
    acc += score;
  }
  *sink = acc;
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// :34-54 — loops z, y, x, rz, ry, rx; first strict maximum wins.
Rt3dResult RealTimeMatch3D(const RtOptions3D& o, const Rigid3d& initial, const PointCloud& cloud,
                           const HybridGrid& grid) {
  Rt3dGeometry g;
  g.res = grid.resolution();
  RealTime3DWindow(o, g.res, cloud, &g.L, &g.step, &g.A);
  const int64_t na = 2 * g.A + 1, nl = 2 * g.L + 1;
  const int64_t total = nl * nl * nl * na * na * na;
  const Rigid3f init = CastRigidF(initial);
  Rt3dResult r;
  r.candidates = total;
  for (int64_t i = 0; i < total; ++i) {
    const Rigid3f t = RtTransform(g, i);
    const Rigid3f candidate = Mul3(init, t);
    const float s = RtScore(o, grid, cloud, candidate, t);
    if (s > r.score) {
      r.score = s;
      r.pose = CastRigidD(candidate);
      r.best_index = i;
    }
  }
  return r;
}

}  // namespace oracle
