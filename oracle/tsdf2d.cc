// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// TSDF2D, its value converter, 2D normal estimation, the TSDF range data
// inserter and RealTimeCorrelativeScanMatcher2D scoring over a TSDF, restated
// from the reference files cited per function. Float/double promotion follows
// the reference expressions term by term (x86-64, no FMA contraction).

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>

#include "oracle_tsdf.h"

#define ORACLE_CHECK(cond)                                              \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "oracle CHECK failed %s:%d: %s\n", __FILE__, \
                   __LINE__, #cond);                                    \
      std::abort();                                                     \
    }                                                                   \
  } while (0)

namespace oracle {
namespace {

constexpr uint16_t kTsdUpdateMarker = 1u << 15;

// common/math.h:32-40
float ClampF(float v, float lo, float hi) {
  if (v > hi) return hi;
  if (v < lo) return lo;
  return v;
}

// common/math.h:62-67
float NormalizeAngleDifferenceF(float d) {
  const float kPi = static_cast<float>(M_PI);
  while (d > kPi) d -= 2. * kPi;
  while (d < -kPi) d += 2. * kPi;
  return d;
}

float Norm2(float x, float y) { return std::sqrt(x * x + y * y); }
// Vector3f::norm(): Eigen's unrolled 3-element sum is x0 + (x1 + x2).
float Norm3(float x, float y, float z) { return std::sqrt(x * x + (y * y + z * z)); }

}  // namespace

// ---------------------------------------------------------------------------
// tsd_value_converter.cc:22-33; tables from value_conversion_tables.cc with
// (unknown, lower, upper) = (min_tsd, min_tsd, max_tsd) and (0, 0, max_weight).
TSDValueConverter::TSDValueConverter(float max_tsd, float max_weight)
    : max_tsd_(max_tsd),
      min_tsd_(-max_tsd),
      max_weight_(max_weight),
      tsd_resolution_(32766.f / (max_tsd_ - min_tsd_)),
      weight_resolution_(32766.f / (max_weight_ - 0.f)),
      value_to_tsd_(MakeConversionTable(min_tsd_, min_tsd_, max_tsd_)),
      value_to_weight_(MakeConversionTable(0.f, 0.f, max_weight)) {}

// tsd_value_converter.h:33-40
uint16_t TSDValueConverter::TSDToValue(float tsd) const {
  const int value = RoundToIntF((ClampF(tsd, min_tsd_, max_tsd_) - min_tsd_) * tsd_resolution_) + 1;
  return static_cast<uint16_t>(value);
}

// tsd_value_converter.h:43-50
uint16_t TSDValueConverter::WeightToValue(float weight) const {
  const int value =
      RoundToIntF((ClampF(weight, 0.f, max_weight_) - 0.f) * weight_resolution_) + 1;
  return static_cast<uint16_t>(value);
}

// ---------------------------------------------------------------------------
// tsdf_2d.cc:23-34 (weight cells start at the unknown weight value 0).
TSDF2D::TSDF2D(const MapLimits& limits, float truncation_distance, float max_weight)
    : limits_(limits),
      conv_(truncation_distance, max_weight),
      tsd_cells_(static_cast<size_t>(limits.cells.num_x_cells) * limits.cells.num_y_cells, 0),
      weight_cells_(tsd_cells_.size(), 0) {}

TSDF2D::TSDF2D(const MapLimits& limits, float truncation_distance, float max_weight,
               std::vector<uint16_t> tsd_cells, std::vector<uint16_t> weight_cells)
    : limits_(limits),
      conv_(truncation_distance, max_weight),
      tsd_cells_(std::move(tsd_cells)),
      weight_cells_(std::move(weight_cells)) {
  ORACLE_CHECK(tsd_cells_.size() ==
               static_cast<size_t>(limits.cells.num_x_cells) * limits.cells.num_y_cells);
  ORACLE_CHECK(weight_cells_.size() == tsd_cells_.size());
}

// grid_2d.h:113-116 (ToFlatIndex CHECKs containment).
int TSDF2D::FlatIndex(const Idx2& i) const {
  ORACLE_CHECK(limits_.Contains(i));
  return limits_.cells.num_x_cells * i.y + i.x;
}

// tsdf_2d.cc:50-54
bool TSDF2D::CellIsUpdated(const Idx2& i) const {
  return tsd_cells_[FlatIndex(i)] >= kTsdUpdateMarker;
}

// tsdf_2d.cc:56-69
void TSDF2D::SetCell(const Idx2& i, float tsd, float weight) {
  const int flat = FlatIndex(i);
  uint16_t* cell = &tsd_cells_[flat];
  if (*cell >= kTsdUpdateMarker) return;
  update_indices_.push_back(flat);
  if (box_empty_) {
    box_min_x_ = box_max_x_ = i.x;
    box_min_y_ = box_max_y_ = i.y;
    box_empty_ = false;
  } else {
    box_min_x_ = std::min(box_min_x_, i.x);
    box_max_x_ = std::max(box_max_x_, i.x);
    box_min_y_ = std::min(box_min_y_, i.y);
    box_max_y_ = std::max(box_max_y_, i.y);
  }
  *cell = static_cast<uint16_t>(conv_.TSDToValue(tsd) + kTsdUpdateMarker);
  weight_cells_[flat] = conv_.WeightToValue(weight);
}

// tsdf_2d.cc:73-79
float TSDF2D::GetTSD(const Idx2& i) const {
  if (limits_.Contains(i)) return conv_.ValueToTSD(tsd_cells_[FlatIndex(i)]);
  return conv_.min_tsd();
}

// tsdf_2d.cc:81-87
float TSDF2D::GetWeight(const Idx2& i) const {
  if (limits_.Contains(i)) return conv_.ValueToWeight(weight_cells_[FlatIndex(i)]);
  return conv_.min_weight();
}

// tsdf_2d.cc:89-99
std::pair<float, float> TSDF2D::GetTSDAndWeight(const Idx2& i) const {
  if (limits_.Contains(i)) {
    const int flat = FlatIndex(i);
    return {conv_.ValueToTSD(tsd_cells_[flat]), conv_.ValueToWeight(weight_cells_[flat])};
  }
  return {conv_.min_tsd(), conv_.min_weight()};
}

// grid_2d.cc:97-101 (IsKnown on the correspondence-cost cells).
bool TSDF2D::IsKnown(const Idx2& i) const {
  return limits_.Contains(i) && tsd_cells_[FlatIndex(i)] != 0;
}

// grid_2d.cc:88-95
void TSDF2D::FinishUpdate() {
  while (!update_indices_.empty()) {
    tsd_cells_[update_indices_.back()] -= kTsdUpdateMarker;
    update_indices_.pop_back();
  }
}

// grid_2d.cc:121-132
void TSDF2D::ComputeCroppedLimits(Idx2* offset, CellLimits* limits) const {
  if (box_empty_) {
    *offset = Idx2{0, 0};
    *limits = CellLimits{1, 1};
    return;
  }
  *offset = Idx2{box_min_x_, box_min_y_};
  *limits = CellLimits{box_max_x_ - box_min_x_ + 1, box_max_y_ - box_min_y_ + 1};
}

// tsdf_2d.cc:101-106 -> grid_2d.cc:142-175 over both cell arrays (unknown 0).
void TSDF2D::GrowLimits(float px, float py) {
  ORACLE_CHECK(update_indices_.empty());
  while (!limits_.Contains(limits_.GetCellIndex(px, py))) {
    const int xo = limits_.cells.num_x_cells / 2;
    const int yo = limits_.cells.num_y_cells / 2;
    MapLimits grown;
    grown.resolution = limits_.resolution;
    grown.max_x = limits_.max_x + limits_.resolution * yo;
    grown.max_y = limits_.max_y + limits_.resolution * xo;
    grown.cells = CellLimits{2 * limits_.cells.num_x_cells, 2 * limits_.cells.num_y_cells};
    const int stride = grown.cells.num_x_cells;
    for (std::vector<uint16_t>* g : {&tsd_cells_, &weight_cells_}) {
      std::vector<uint16_t> next(static_cast<size_t>(stride) * grown.cells.num_y_cells, 0);
      for (int y = 0; y < limits_.cells.num_y_cells; ++y)
        for (int x = 0; x < limits_.cells.num_x_cells; ++x)
          next[(xo + stride * yo) + x + y * stride] = (*g)[x + y * limits_.cells.num_x_cells];
      g->swap(next);
    }
    limits_ = grown;
    if (!box_empty_) {
      box_min_x_ += xo;
      box_max_x_ += xo;
      box_min_y_ += yo;
      box_max_y_ += yo;
    }
  }
}

// ---------------------------------------------------------------------------
// normal_estimation_2d.cc:23-58
namespace {

float EstimateNormal(const PointCloud& returns, size_t est, size_t begin, size_t end,
                     const Vec3f& origin) {
  const Vec3f& p = returns[est];
  if (end - begin < 2) return std::atan2(origin.y - p.y, origin.x - p.x);
  float mx = 0.f, my = 0.f;
  const float ox = origin.x - p.x, oy = origin.y - p.y, oz = origin.z - p.z;
  for (size_t s = begin; s < end; ++s) {
    if (s == est) continue;
    const Vec3f& q = returns[s];
    const float tx = p.x - q.x, ty = p.y - q.y;
    float nx = -ty, ny = tx;
    const float nz = 0.f;
    constexpr float kMinNormalLength = 1e-6f;
    if (Norm3(nx, ny, nz) < kMinNormalLength) continue;
    if (nx * ox + ny * oy + nz * oz < 0) {
      nx = -nx;
      ny = -ny;
    }
    // Eigen normalize(): divide by sqrt(squaredNorm) when it is positive.
    const float sq = nx * nx + ny * ny + nz * nz;
    if (sq > 0.f) {
      const float n = std::sqrt(sq);
      nx /= n;
      ny /= n;
    }
    mx += nx;
    my += ny;
  }
  return std::atan2(my, mx);
}

}  // namespace

// normal_estimation_2d.cc:74-109
std::vector<float> EstimateNormals(const RangeData& rd, const NormalEstimationOptions2D& o) {
  std::vector<float> normals;
  normals.reserve(rd.returns.size());
  const size_t max_num_samples = static_cast<size_t>(o.num_normal_samples);
  const float radius = o.sample_radius;
  auto dist = [&](const Vec3f& a, const Vec3f& b) {
    return Norm3(a.x - b.x, a.y - b.y, a.z - b.z);
  };
  for (size_t cur = 0; cur < rd.returns.size(); ++cur) {
    const Vec3f& hit = rd.returns[cur];
    size_t wb = cur;
    for (; wb > 0 && cur - wb < max_num_samples / 2 && dist(hit, rd.returns[wb - 1]) < radius;
         --wb) {
    }
    size_t we = cur;
    for (; we < rd.returns.size() && we - cur < std::ceil(max_num_samples / 2.0) + 1 &&
           dist(hit, rd.returns[we]) < radius;
         ++we) {
    }
    normals.push_back(EstimateNormal(rd.returns, cur, wb, we, rd.origin));
  }
  return normals;
}

// ---------------------------------------------------------------------------
// tsdf_range_data_inserter_2d.cc
namespace {

constexpr int kTsdfSubpixelScale = 1000;
constexpr float kMinRangeMeters = 1e-6f;
const float kSqrtTwoPi = std::sqrt(2.0 * M_PI);

// :49-51 (double arithmetic, float result)
float GaussianKernel(float x, float sigma) {
  return 1.0 / (kSqrtTwoPi * sigma) * std::exp(-0.5 * x * x / (sigma * sigma));
}

// :81-87 (std::pow(float, int) is evaluated in double)
float ComputeRangeWeightFactor(float range, int exponent) {
  float weight = 0.f;
  if (std::abs(range) > kMinRangeMeters) weight = 1.f / std::pow(range, exponent);
  return weight;
}

// Eigen Vector2f::normalized()
Vec2f Normalized2(float x, float y) {
  const float sq = x * x + y * y;
  if (sq > 0.f) {
    const float n = std::sqrt(sq);
    return Vec2f{x / n, y / n};
  }
  return Vec2f{x, y};
}

}  // namespace

// :142-179
void TSDFRangeDataInserter2D::Insert(const RangeData& rd, TSDF2D* tsdf) const {
  const float trunc = static_cast<float>(options_.truncation_distance);
  // GrowAsNeeded (:33-47): box over origin and each hit pushed `trunc` further
  // along its (3D, normalized) ray.
  float bmin_x = rd.origin.x, bmax_x = rd.origin.x;
  float bmin_y = rd.origin.y, bmax_y = rd.origin.y;
  for (const Vec3f& h : rd.returns) {
    float dx = h.x - rd.origin.x, dy = h.y - rd.origin.y, dz = h.z - rd.origin.z;
    const float sq = dx * dx + dy * dy + dz * dz;
    if (sq > 0.f) {
      const float n = std::sqrt(sq);
      dx /= n;
      dy /= n;
    }
    const float ex = h.x + trunc * dx, ey = h.y + trunc * dy;
    bmin_x = std::min(bmin_x, ex);
    bmax_x = std::max(bmax_x, ex);
    bmin_y = std::min(bmin_y, ey);
    bmax_y = std::max(bmax_y, ey);
  }
  constexpr float kPadding = 1e-6f;
  tsdf->GrowLimits(bmin_x - kPadding, bmin_y - kPadding);
  tsdf->GrowLimits(bmax_x + kPadding, bmax_y + kPadding);

  const bool angle_weight = options_.update_weight_angle_scan_normal_to_ray_kernel_bandwidth != 0.f;
  RangeData sorted = rd;
  std::vector<float> normals;
  if (options_.project_sdf_distance_to_scan_normal || angle_weight) {
    // RangeDataSorter (:63-79)
    const float ox = rd.origin.x, oy = rd.origin.y;
    std::sort(sorted.returns.begin(), sorted.returns.end(), [&](const Vec3f& l, const Vec3f& r) {
      const Vec2f dl = Normalized2(l.x - ox, l.y - oy);
      const Vec2f dr = Normalized2(r.x - ox, r.y - oy);
      if ((dl.y < 0.f) != (dr.y < 0.f)) return dl.y < 0.f;
      if (dl.y < 0.f) return dl.x < dr.x;
      return dl.x > dr.x;
    });
    normals = EstimateNormals(sorted, options_.normal_estimation);
  }
  const Vec2f origin{sorted.origin.x, sorted.origin.y};
  for (size_t k = 0; k < sorted.returns.size(); ++k) {
    const Vec2f hit{sorted.returns[k].x, sorted.returns[k].y};
    const float normal = normals.empty() ? std::numeric_limits<float>::quiet_NaN() : normals[k];
    InsertHit(hit, origin, normal, tsdf);
  }
  tsdf->FinishUpdate();
}

// :181-227
void TSDFRangeDataInserter2D::InsertHit(const Vec2f& hit, const Vec2f& origin, float normal,
                                        TSDF2D* tsdf) const {
  const float rx = hit.x - origin.x, ry = hit.y - origin.y;
  const float range = Norm2(rx, ry);
  const float trunc = static_cast<float>(options_.truncation_distance);
  if (range < trunc) return;
  const float ratio = trunc / range;
  Vec2f begin = origin;
  if (!options_.update_free_space) {
    const float f = 1.0f - ratio;
    begin = Vec2f{origin.x + f * rx, origin.y + f * ry};
  }
  const float fe = 1.0f + ratio;
  const Vec2f end{origin.x + fe * rx, origin.y + fe * ry};
  // SuperscaleRay (:53-67)
  const MapLimits& limits = tsdf->limits();
  MapLimits fine;
  fine.resolution = limits.resolution / kTsdfSubpixelScale;
  fine.max_x = limits.max_x;
  fine.max_y = limits.max_y;
  fine.cells = CellLimits{limits.cells.num_x_cells * kTsdfSubpixelScale,
                          limits.cells.num_y_cells * kTsdfSubpixelScale};
  const std::vector<Idx2> mask = RayToPixelMask(fine.GetCellIndex(begin.x, begin.y),
                                                fine.GetCellIndex(end.x, end.y), kTsdfSubpixelScale);

  float wf_angle = 1.f;
  if (options_.update_weight_angle_scan_normal_to_ray_kernel_bandwidth != 0.f) {
    const float angle = NormalizeAngleDifferenceF(normal - std::atan2(-ry, -rx));
    wf_angle = GaussianKernel(
        angle, static_cast<float>(options_.update_weight_angle_scan_normal_to_ray_kernel_bandwidth));
  }
  float wf_range = 1.f;
  if (options_.update_weight_range_exponent != 0)
    wf_range = ComputeRangeWeightFactor(range, options_.update_weight_range_exponent);

  for (const Idx2& c : mask) {
    if (tsdf->CellIsUpdated(c)) continue;
    // map_limits.h:79-82 (double, cast to float)
    const float cx = static_cast<float>(limits.max_x - limits.resolution * (c.y + 0.5));
    const float cy = static_cast<float>(limits.max_y - limits.resolution * (c.x + 0.5));
    const float d_origin = Norm2(cx - origin.x, cy - origin.y);
    float tsd = range - d_origin;
    if (options_.project_sdf_distance_to_scan_normal)
      tsd = (cx - hit.x) * std::cos(normal) + (cy - hit.y) * std::sin(normal);
    tsd = ClampF(tsd, -trunc, trunc);
    float w = wf_range * wf_angle;
    if (options_.update_weight_distance_cell_to_hit_kernel_bandwidth != 0.f)
      w *= GaussianKernel(tsd, static_cast<float>(options_.update_weight_distance_cell_to_hit_kernel_bandwidth));
    UpdateCell(c, tsd, w, tsdf);
  }
}

// :229-240
void TSDFRangeDataInserter2D::UpdateCell(const Idx2& cell, float update_sdf, float update_weight,
                                         TSDF2D* tsdf) const {
  if (update_weight == 0.f) return;
  const std::pair<float, float> tw = tsdf->GetTSDAndWeight(cell);
  float updated_weight = tw.second + update_weight;
  const float updated_sdf = (tw.first * tw.second + update_sdf * update_weight) / updated_weight;
  updated_weight = std::min(updated_weight, static_cast<float>(options_.maximum_weight));
  tsdf->SetCell(cell, updated_sdf, updated_weight);
}

// ---------------------------------------------------------------------------
// real_time_correlative_scan_matcher_2d.cc:38-59
static float ComputeCandidateScoreTSDF(const TSDF2D& tsdf, const DiscreteScan2D& scan, int xo,
                                       int yo) {
  float score = 0.f, summed_weight = 0.f;
  const float max_cc = tsdf.GetMaxCorrespondenceCost();
  for (const Idx2& xy : scan) {
    const std::pair<float, float> tw = tsdf.GetTSDAndWeight(Idx2{xy.x + xo, xy.y + yo});
    const float normalized = (max_cc - std::abs(tw.first)) / max_cc;
    const float weight = tw.second;
    score += normalized * weight;
    summed_weight += weight;
  }
  if (summed_weight == 0.f) return 0.f;
  score /= summed_weight;
  ORACLE_CHECK(score >= 0.f);
  return score;
}

// :151-176 (TSDF branch)
void RealTimeScoreCandidatesTSDF(const RealTimeOptions& o, const TSDF2D& tsdf,
                                 const std::vector<DiscreteScan2D>& scans,
                                 std::vector<Candidate2D>* candidates) {
  for (Candidate2D& c : *candidates) {
    c.score = ComputeCandidateScoreTSDF(tsdf, scans[c.scan_index], c.x_index_offset,
                                        c.y_index_offset);
    const double pen = std::hypot(c.x, c.y) * o.translation_delta_cost_weight +
                       std::abs(c.orientation) * o.rotation_delta_cost_weight;
    c.score *= std::exp(-(pen * pen));
  }
}

// :117-149 over a TSDF2D.
double RealTimeMatchTSDF(const RealTimeOptions& o, const Rigid2d& initial, const PointCloud& cloud,
                         const TSDF2D& tsdf, Rigid2d* pose, int64_t* num_candidates) {
  ORACLE_CHECK(pose != nullptr);
  Rigid3f pre;
  pre.q = QuatFromAngleAxisF(static_cast<float>(initial.angle), 0.f, 0.f, 1.f);
  const PointCloud rotated = TransformPointCloud(cloud, pre);
  const SearchParameters sp(o.linear_search_window, o.angular_search_window, rotated,
                            tsdf.limits().resolution);
  const std::vector<PointCloud> rotated_scans = GenerateRotatedScans(rotated, sp);
  const std::vector<DiscreteScan2D> discrete =
      DiscretizeScans(tsdf.limits(), rotated_scans, static_cast<float>(initial.tx),
                      static_cast<float>(initial.ty));
  std::vector<Candidate2D> candidates =
      RealTimeCorrelativeScanMatcher2D(o).GenerateExhaustiveSearchCandidates(sp);
  if (num_candidates) *num_candidates = static_cast<int64_t>(candidates.size());
  RealTimeScoreCandidatesTSDF(o, tsdf, discrete, &candidates);
  const Candidate2D& best = *std::max_element(candidates.begin(), candidates.end());
  pose->tx = initial.tx + best.x;
  pose->ty = initial.ty + best.y;
  pose->angle = initial.angle + best.orientation;
  return best.score;
}

}  // namespace oracle
