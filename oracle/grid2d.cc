// ORACLE — TEST INFRASTRUCTURE ONLY (see csm_oracle.h).
//
// Value encoding, 2D map limits, probability grid, ray casting and the range
// data inserter, restated from the reference files cited per function. The
// inserter exists only to rebuild the grids the reference's own tests use.

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "csm_oracle.h"

#define ORACLE_CHECK(cond)                                              \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "oracle CHECK failed %s:%d: %s\n", __FILE__, \
                   __LINE__, #cond);                                    \
      std::abort();                                                     \
    }                                                                   \
  } while (0)

namespace oracle {

// ---------------------------------------------------------------------------
// common/math.h Clamp
static float ClampF(float v, float lo, float hi) {
  if (v > hi) return hi;
  if (v < lo) return lo;
  return v;
}

// probability_values.h:37-39, 41-43
float Odds(float p) { return p / (1.f - p); }
float ProbabilityFromOdds(float odds) { return odds / (odds + 1.f); }

// probability_values.h:32-45
uint16_t BoundedFloatToValue(float v, float lo, float hi) {
  const int value =
      RoundToIntF((ClampF(v, lo, hi) - lo) * (32766.f / (hi - lo))) + 1;
  return static_cast<uint16_t>(value);
}

// probability_values.h:84-92
uint16_t CorrespondenceCostToValue(float cc) {
  return BoundedFloatToValue(cc, kMinCorrespondenceCost, kMaxCorrespondenceCost);
}
uint16_t ProbabilityToValue(float p) {
  return BoundedFloatToValue(p, kMinProbability, kMaxProbability);
}

// value_conversion_tables.cc:28-52 (bit 15 masked; 0 -> unknown_result).
std::vector<float> MakeConversionTable(float unknown_result, float lo, float hi) {
  std::vector<float> t(65536);
  const float scale = (hi - lo) / 32766.f;
  for (int v = 0; v < 65536; ++v) {
    const uint16_t value = static_cast<uint16_t>(v) & 0x7fff;
    t[v] = value == 0 ? unknown_result : value * scale + (lo - scale);
  }
  return t;
}

// probability_values.cc:26-66 (the table repeated twice == masked).
const std::vector<float>& ValueToCorrespondenceCostTable() {
  static const std::vector<float> t = MakeConversionTable(
      kMaxCorrespondenceCost, kMinCorrespondenceCost, kMaxCorrespondenceCost);
  return t;
}
const std::vector<float>& ValueToProbabilityTable() {
  static const std::vector<float> t =
      MakeConversionTable(kMinProbability, kMinProbability, kMaxProbability);
  return t;
}

// probability_values.cc:89-106
std::vector<uint16_t> LookupTableToApplyCorrespondenceCostOdds(float odds) {
  const std::vector<float>& cc = ValueToCorrespondenceCostTable();
  std::vector<uint16_t> out;
  out.reserve(32768);
  out.push_back(CorrespondenceCostToValue(1.f - ProbabilityFromOdds(odds)) +
                kUpdateMarker);
  for (int cell = 1; cell < 32768; ++cell) {
    const float p = ProbabilityFromOdds(odds * Odds(1.f - cc[cell]));
    out.push_back(CorrespondenceCostToValue(1.f - p) + kUpdateMarker);
  }
  return out;
}

// probability_values.cc:76-87
std::vector<uint16_t> LookupTableToApplyOdds(float odds) {
  const std::vector<float>& pt = ValueToProbabilityTable();
  std::vector<uint16_t> out;
  out.reserve(32768);
  out.push_back(ProbabilityToValue(ProbabilityFromOdds(odds)) + kUpdateMarker);
  for (int cell = 1; cell < 32768; ++cell) {
    out.push_back(ProbabilityToValue(ProbabilityFromOdds(odds * Odds(pt[cell]))) +
                  kUpdateMarker);
  }
  return out;
}

// ---------------------------------------------------------------------------
// map_limits.h:69-75 — double subtract/divide, then lround.
Idx2 MapLimits::GetCellIndex(float px, float py) const {
  return Idx2{RoundToInt((max_y - py) / resolution - 0.5),
              RoundToInt((max_x - px) / resolution - 0.5)};
}

// map_limits.h:84-89
bool MapLimits::Contains(const Idx2& i) const {
  return i.x >= 0 && i.y >= 0 && i.x < cells.num_x_cells &&
         i.y < cells.num_y_cells;
}

// ---------------------------------------------------------------------------
// grid_2d.cc:72-85, probability_grid.cc:26-30
ProbabilityGrid::ProbabilityGrid(const MapLimits& limits)
    : limits_(limits),
      cells_(static_cast<size_t>(limits.cells.num_x_cells) *
                 limits.cells.num_y_cells,
             kUnknownValue) {}

ProbabilityGrid::ProbabilityGrid(const MapLimits& limits,
                                 std::vector<uint16_t> cells)
    : limits_(limits), cells_(std::move(cells)) {
  ORACLE_CHECK(cells_.size() == static_cast<size_t>(limits.cells.num_x_cells) *
                                    limits.cells.num_y_cells);
}

// grid_2d.h:113-116
int ProbabilityGrid::FlatIndex(const Idx2& i) const {
  ORACLE_CHECK(limits_.Contains(i));
  return limits_.cells.num_x_cells * i.y + i.x;
}

// grid_2d.h:53-57 (table from value_conversion_tables with unknown = max cc)
float ProbabilityGrid::GetCorrespondenceCost(const Idx2& i) const {
  if (!limits_.Contains(i)) return kMaxCorrespondenceCost;
  return ValueToCorrespondenceCostTable()[cells_[FlatIndex(i)]];
}

// probability_grid.cc:78-82
float ProbabilityGrid::GetProbability(const Idx2& i) const {
  if (!limits_.Contains(i)) return kMinProbability;
  return 1.f - ValueToCorrespondenceCostTable()[cells_[FlatIndex(i)]];
}

// grid_2d.h:69-73
bool ProbabilityGrid::IsKnown(const Idx2& i) const {
  return limits_.Contains(i) && cells_[FlatIndex(i)] != kUnknownValue;
}

void ProbabilityGrid::ExtendBox(const Idx2& i) {
  if (box_empty_) {
    box_min_x_ = box_max_x_ = i.x;
    box_min_y_ = box_max_y_ = i.y;
    box_empty_ = false;
    return;
  }
  box_min_x_ = std::min(box_min_x_, i.x);
  box_max_x_ = std::max(box_max_x_, i.x);
  box_min_y_ = std::min(box_min_y_, i.y);
  box_max_y_ = std::max(box_max_y_, i.y);
}

// probability_grid.cc:34-43
void ProbabilityGrid::SetProbability(const Idx2& i, float p) {
  uint16_t& cell = cells_[FlatIndex(i)];
  ORACLE_CHECK(cell == kUnknownValue);
  cell = CorrespondenceCostToValue(1.f - p);
  ExtendBox(i);
}

// probability_grid.cc:51-63
bool ProbabilityGrid::ApplyLookupTable(const Idx2& i,
                                       const std::vector<uint16_t>& table) {
  const int flat = FlatIndex(i);
  uint16_t* cell = &cells_[flat];
  if (*cell >= kUpdateMarker) return false;
  update_indices_.push_back(flat);
  *cell = table[*cell];
  ExtendBox(i);
  return true;
}

// grid_2d.cc:110-117
void ProbabilityGrid::FinishUpdate() {
  while (!update_indices_.empty()) {
    cells_[update_indices_.back()] -= kUpdateMarker;
    update_indices_.pop_back();
  }
}

// grid_2d.cc:121-132
void ProbabilityGrid::ComputeCroppedLimits(Idx2* offset,
                                           CellLimits* limits) const {
  if (box_empty_) {
    *offset = Idx2{0, 0};
    *limits = CellLimits{1, 1};
    return;
  }
  *offset = Idx2{box_min_x_, box_min_y_};
  *limits = CellLimits{box_max_x_ - box_min_x_ + 1, box_max_y_ - box_min_y_ + 1};
}

// grid_2d.cc:142-175 — doubles the grid about its centre until 'point' fits.
void ProbabilityGrid::GrowLimits(float px, float py) {
  ORACLE_CHECK(update_indices_.empty());
  while (!limits_.Contains(limits_.GetCellIndex(px, py))) {
    const int xo = limits_.cells.num_x_cells / 2;
    const int yo = limits_.cells.num_y_cells / 2;
    MapLimits grown;
    grown.resolution = limits_.resolution;
    grown.max_x = limits_.max_x + limits_.resolution * yo;
    grown.max_y = limits_.max_y + limits_.resolution * xo;
    grown.cells = CellLimits{2 * limits_.cells.num_x_cells,
                             2 * limits_.cells.num_y_cells};
    const int stride = grown.cells.num_x_cells;
    std::vector<uint16_t> next(static_cast<size_t>(stride) *
                                   grown.cells.num_y_cells,
                               kUnknownValue);
    for (int y = 0; y < limits_.cells.num_y_cells; ++y)
      for (int x = 0; x < limits_.cells.num_x_cells; ++x)
        next[(xo + stride * yo) + x + y * stride] =
            cells_[x + y * limits_.cells.num_x_cells];
    cells_.swap(next);
    limits_ = grown;
    if (!box_empty_) {
      box_min_x_ += xo;
      box_max_x_ += xo;
      box_min_y_ += yo;
      box_max_y_ += yo;
    }
  }
}

// probability_grid.cc:91-106
ProbabilityGrid ProbabilityGrid::ComputeCroppedGrid() const {
  Idx2 offset;
  CellLimits cl;
  ComputeCroppedLimits(&offset, &cl);
  MapLimits ml;
  ml.resolution = limits_.resolution;
  ml.max_x = limits_.max_x - limits_.resolution * offset.y;
  ml.max_y = limits_.max_y - limits_.resolution * offset.x;
  ml.cells = cl;
  ProbabilityGrid out(ml);
  for (int y = 0; y < cl.num_y_cells; ++y)
    for (int x = 0; x < cl.num_x_cells; ++x) {
      const Idx2 src{x + offset.x, y + offset.y};
      if (!IsKnown(src)) continue;
      out.SetProbability(Idx2{x, y}, GetProbability(src));
    }
  return out;
}

// ---------------------------------------------------------------------------
// ray_to_pixel_mask.cc:29-159. Begin/end are sub-pixel scaled, non-negative.
// The walk advances one full pixel column at a time and emits every pixel row
// the segment crosses inside that column; sub_y tracks the segment's height at
// the column border in units of 1 / (2 * scale * dx).
std::vector<Idx2> RayToPixelMask(Idx2 b, Idx2 e, int scale) {
  if (b.x > e.x) std::swap(b, e);
  ORACLE_CHECK(b.x >= 0 && b.y >= 0 && e.y >= 0);
  std::vector<Idx2> mask;
  auto emit = [&mask](const Idx2& c) {
    if (mask.empty() || mask.back().x != c.x || mask.back().y != c.y)
      mask.push_back(c);
  };
  if (b.x / scale == e.x / scale) {
    // Same pixel column: vertical run of full pixels.
    const int col = b.x / scale;
    const int y0 = std::min(b.y, e.y) / scale;
    const int y1 = std::max(b.y, e.y) / scale;
    for (int y = y0; y <= y1; ++y) emit(Idx2{col, y});
    return mask;
  }
  const int64_t dx = e.x - b.x;
  const int64_t dy = e.y - b.y;
  const int64_t denom = 2 * static_cast<int64_t>(scale) * dx;
  Idx2 cur{b.x / scale, b.y / scale};
  mask.push_back(cur);
  int64_t sub_y = (2 * (b.y % scale) + 1) * dx;
  const int first_pixel = 2 * scale - 2 * (b.x % scale) - 1;
  const int last_pixel = 2 * (e.x % scale) + 1;
  const int end_x = std::max(b.x, e.x) / scale;
  sub_y += dy * first_pixel;
  if (dy > 0) {
    for (;;) {
      emit(cur);
      while (sub_y > denom) {
        sub_y -= denom;
        ++cur.y;
        emit(cur);
      }
      ++cur.x;
      if (sub_y == denom) {
        sub_y -= denom;
        ++cur.y;
      }
      if (cur.x == end_x) break;
      sub_y += dy * 2 * scale;
    }
    sub_y += dy * last_pixel;
    emit(cur);
    while (sub_y > denom) {
      sub_y -= denom;
      ++cur.y;
      emit(cur);
    }
    ORACLE_CHECK(sub_y != denom);
    ORACLE_CHECK(cur.y == e.y / scale);
    return mask;
  }
  for (;;) {
    emit(cur);
    while (sub_y < 0) {
      sub_y += denom;
      --cur.y;
      emit(cur);
    }
    ++cur.x;
    if (sub_y == 0) {
      sub_y += denom;
      --cur.y;
    }
    if (cur.x == end_x) break;
    sub_y += dy * 2 * scale;
  }
  sub_y += dy * last_pixel;
  emit(cur);
  while (sub_y < 0) {
    sub_y += denom;
    --cur.y;
    emit(cur);
  }
  ORACLE_CHECK(sub_y != 0);
  ORACLE_CHECK(cur.y == e.y / scale);
  return mask;
}

// ---------------------------------------------------------------------------
// probability_grid_range_data_inserter_2d.cc:115-135
ProbabilityGridInserter2D::ProbabilityGridInserter2D(float hit_probability,
                                                     float miss_probability,
                                                     bool insert_free_space)
    : insert_free_space_(insert_free_space),
      hit_table_(LookupTableToApplyCorrespondenceCostOdds(Odds(hit_probability))),
      miss_table_(
          LookupTableToApplyCorrespondenceCostOdds(Odds(miss_probability))) {}

// probability_grid_range_data_inserter_2d.cc:35-98, 124-136
void ProbabilityGridInserter2D::Insert(const RangeData& rd,
                                       ProbabilityGrid* grid) const {
  constexpr int kSubpixelScale = 1000;
  // GrowAsNeeded: bounding box of origin, hits and misses, padded by 1e-6.
  float bmin_x = rd.origin.x, bmax_x = rd.origin.x;
  float bmin_y = rd.origin.y, bmax_y = rd.origin.y;
  auto extend = [&](const Vec3f& p) {
    bmin_x = std::min(bmin_x, p.x);
    bmax_x = std::max(bmax_x, p.x);
    bmin_y = std::min(bmin_y, p.y);
    bmax_y = std::max(bmax_y, p.y);
  };
  for (const Vec3f& p : rd.returns) extend(p);
  for (const Vec3f& p : rd.misses) extend(p);
  constexpr float kPadding = 1e-6f;
  grid->GrowLimits(bmin_x - kPadding, bmin_y - kPadding);
  grid->GrowLimits(bmax_x + kPadding, bmax_y + kPadding);

  const MapLimits& limits = grid->limits();
  MapLimits fine;
  fine.resolution = limits.resolution / kSubpixelScale;
  fine.max_x = limits.max_x;
  fine.max_y = limits.max_y;
  fine.cells = CellLimits{limits.cells.num_x_cells * kSubpixelScale,
                          limits.cells.num_y_cells * kSubpixelScale};
  const Idx2 begin = fine.GetCellIndex(rd.origin.x, rd.origin.y);
  std::vector<Idx2> ends;
  ends.reserve(rd.returns.size());
  for (const Vec3f& hit : rd.returns) {
    ends.push_back(fine.GetCellIndex(hit.x, hit.y));
    grid->ApplyLookupTable(
        Idx2{ends.back().x / kSubpixelScale, ends.back().y / kSubpixelScale},
        hit_table_);
  }
  if (insert_free_space_) {
    for (const Idx2& end : ends)
      for (const Idx2& c : RayToPixelMask(begin, end, kSubpixelScale))
        grid->ApplyLookupTable(c, miss_table_);
    for (const Vec3f& miss : rd.misses)
      for (const Idx2& c : RayToPixelMask(
               begin, fine.GetCellIndex(miss.x, miss.y), kSubpixelScale))
        grid->ApplyLookupTable(c, miss_table_);
  }
  grid->FinishUpdate();
}

}  // namespace oracle
