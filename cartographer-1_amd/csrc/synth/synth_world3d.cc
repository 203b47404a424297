// Synthetic 3D world (bench / test inputs only; not the match path).
//
// A seeded warehouse: floor, ceiling, outer walls, pillars and crates (axis
// aligned boxes). A 64-ring lidar is ray-cast from node
// poses; each submap inserts the scans of its nearest nodes into a high- and a
// low-resolution HybridGrid-like sparse grid with the range-data inserter's
// update rule (hits, then the last `num_free_space_voxels` misses per ray,
// range_data_inserter_3d.cc:44-136). Node clouds are voxel-decimated (first
// point per voxel) in place of AdaptiveVoxelFilter (not reproducible without
// abseil, SURVEY.md §8a hazard 12). Histograms follow
// rotational_scan_matcher.cc:160-171 (node) and submap_3d.cc:341-346 (submap).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <map>
#include <random>
#include <thread>
#include <unordered_map>
#include <vector>

#include "csm_synth.h"

namespace {

struct Box {
  float lo[3], hi[3];
};

struct V3 {
  float x, y, z;
};

// ------------------------------------------------------------ values --
const float kMinP = 0.1f, kMaxP = 0.9f;
float Odds(float p) { return p / (1.f - p); }
float FromOdds(float o) { return o / (o + 1.f); }
uint16_t ProbToValue(float p) {
  p = std::min(std::max(p, kMinP), kMaxP);
  return static_cast<uint16_t>(std::lround((p - kMinP) * (32766.f / (kMaxP - kMinP))) + 1);
}
float ValueToProb(uint16_t v) {
  v &= 0x7fff;
  if (v == 0) return kMinP;
  const float s = (kMaxP - kMinP) / 32766.f;
  return v * s + (kMinP - s);
}
std::vector<uint16_t> OddsTable(float odds) {  // probability_values.cc:77-88
  std::vector<uint16_t> t(32768);
  t[0] = ProbToValue(FromOdds(odds)) + 32768;
  for (int v = 1; v < 32768; ++v) t[v] = ProbToValue(FromOdds(odds * Odds(ValueToProb(v)))) + 32768;
  return t;
}

struct SparseGrid {
  float resolution;
  std::unordered_map<uint64_t, uint16_t> cells;
  std::vector<uint16_t*> updated;
  static uint64_t Key(int x, int y, int z) {
    return (static_cast<uint64_t>(x + (1 << 20)) << 42) | (static_cast<uint64_t>(y + (1 << 20)) << 21) |
           static_cast<uint64_t>(z + (1 << 20));
  }
  void Cell(const V3& p, int* c) const {
    c[0] = static_cast<int>(std::lround(p.x / resolution));
    c[1] = static_cast<int>(std::lround(p.y / resolution));
    c[2] = static_cast<int>(std::lround(p.z / resolution));
  }
  void Apply(const int* c, const std::vector<uint16_t>& table) {
    uint16_t& v = cells[Key(c[0], c[1], c[2])];
    if (v >= 32768) return;
    v = table[v];
    updated.push_back(&v);
  }
  void Finish() {
    for (uint16_t* v : updated) *v -= 32768;
    updated.clear();
  }
  // range_data_inserter_3d.cc:110-136
  void Insert(const V3& origin, const std::vector<V3>& returns, const std::vector<uint16_t>& hit,
              const std::vector<uint16_t>& miss, int nfree) {
    for (const V3& h : returns) {
      int c[3];
      Cell(h, c);
      Apply(c, hit);
    }
    int o[3];
    Cell(origin, o);
    for (const V3& h : returns) {
      int c[3];
      Cell(h, c);
      const int d[3] = {c[0] - o[0], c[1] - o[1], c[2] - o[2]};
      const int n = std::max(std::abs(d[0]), std::max(std::abs(d[1]), std::abs(d[2])));
      for (int s = std::max(0, n - nfree); s < n; ++s) {
        const int m[3] = {o[0] + d[0] * s / n, o[1] + d[1] * s / n, o[2] + d[2] * s / n};
        Apply(m, miss);
      }
    }
    Finish();
  }
};

// Ray vs. axis-aligned boxes (slab test); returns the nearest hit distance.
float CastRay(const std::vector<Box>& boxes, const V3& o, const V3& d, float max_range) {
  float best = max_range;
  for (const Box& b : boxes) {
    float t0 = 0.f, t1 = best;
    const float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    bool hit = true;
    for (int a = 0; a < 3 && hit; ++a) {
      if (std::abs(dd[a]) < 1e-12f) {
        if (oo[a] < b.lo[a] || oo[a] > b.hi[a]) hit = false;
        continue;
      }
      float ta = (b.lo[a] - oo[a]) / dd[a], tb = (b.hi[a] - oo[a]) / dd[a];
      if (ta > tb) std::swap(ta, tb);
      t0 = std::max(t0, ta);
      t1 = std::min(t1, tb);
      if (t0 > t1) hit = false;
    }
    if (hit && t0 > 1e-3f && t0 < best) best = t0;
  }
  return best;
}

std::vector<V3> VoxelDecimate(const std::vector<V3>& in, float voxel, float max_range) {
  std::unordered_map<uint64_t, bool> seen;
  std::vector<V3> out;
  for (const V3& p : in) {
    if (std::sqrt(p.x * p.x + p.y * p.y + p.z * p.z) > max_range) continue;
    const uint64_t k = SparseGrid::Key(static_cast<int>(std::floor(p.x / voxel)),
                                       static_cast<int>(std::floor(p.y / voxel)),
                                       static_cast<int>(std::floor(p.z / voxel)));
    if (seen.emplace(k, true).second) out.push_back(p);
  }
  return out;
}

// AdaptiveVoxelFilter's search (sensor/internal/voxel_filter.cc): largest
// voxel <= max_length keeping >= min_points, with VoxelDecimate in place of
// the randomized voxel filter.
std::vector<V3> AdaptiveDecimate(const std::vector<V3>& in, float max_length, int min_points,
                                 float max_range) {
  std::vector<V3> cloud;
  for (const V3& p : in)
    if (std::sqrt(p.x * p.x + p.y * p.y + p.z * p.z) <= max_range) cloud.push_back(p);
  if (static_cast<int>(cloud.size()) <= min_points) return cloud;
  std::vector<V3> result = VoxelDecimate(cloud, max_length, 1e9f);
  if (static_cast<int>(result.size()) >= min_points) return result;
  for (float high = max_length; high > 1e-2f * max_length; high /= 2.f) {
    float low = high / 2.f;
    result = VoxelDecimate(cloud, low, 1e9f);
    if (static_cast<int>(result.size()) >= min_points) {
      while (high / low > 1.1f) {
        const float mid = (low + high) / 2.f;
        std::vector<V3> cand = VoxelDecimate(cloud, mid, 1e9f);
        if (static_cast<int>(cand.size()) >= min_points) {
          low = mid;
          result.swap(cand);
        } else {
          high = mid;
        }
      }
      return result;
    }
  }
  return result;
}

// rotational_scan_matcher.cc:34-117, :160-171 (float arithmetic).
void AddValue(float angle, float value, std::vector<float>* h) {
  const float pi = static_cast<float>(M_PI);
  while (angle > pi) angle -= pi;
  while (angle < 0.f) angle += pi;
  const int n = static_cast<int>(h->size());
  const int b = std::min(std::max(static_cast<int>(std::lround(n * (angle / pi) - 0.5f)), 0), n - 1);
  (*h)[b] += value;
}
V3 Centroid(const std::vector<V3>& s) {
  V3 c{0.f, 0.f, 0.f};
  for (const V3& p : s) {
    c.x += p.x;
    c.y += p.y;
    c.z += p.z;
  }
  const float n = static_cast<float>(s.size());
  return V3{c.x / n, c.y / n, c.z / n};
}
std::vector<float> Histogram(const std::vector<V3>& cloud, int size) {
  std::vector<float> h(size, 0.f);
  std::map<int, std::vector<V3>> slices;
  for (const V3& p : cloud) slices[static_cast<int>(std::lround(p.z / 0.2f))].push_back(p);
  for (auto& kv : slices) {
    const V3 c = Centroid(kv.second);
    std::vector<std::pair<float, V3>> by;
    for (const V3& p : kv.second) {
      const float dx = p.x - c.x, dy = p.y - c.y;
      if (std::sqrt(dx * dx + dy * dy) < 0.2f) continue;
      by.push_back({std::atan2(dy, dx), p});
    }
    std::sort(by.begin(), by.end(),
              [](const std::pair<float, V3>& a, const std::pair<float, V3>& b) { return a.first < b.first; });
    if (by.empty()) continue;
    std::vector<V3> sorted;
    for (auto& q : by) sorted.push_back(q.second);
    const V3 cc = Centroid(sorted);
    V3 last = sorted.front();
    for (const V3& p : sorted) {
      const float dx = p.x - last.x, dy = p.y - last.y, rx = p.x - cc.x, ry = p.y - cc.y;
      const float dist = std::sqrt(dx * dx + dy * dy), rn = std::sqrt(rx * rx + ry * ry);
      if (dist < 0.2f || rn < 0.2f) continue;
      if (dist > 0.9f) {
        last = p;
        continue;
      }
      const float dot = (dx / dist) * (rx / rn) + (dy / dist) * (ry / rn);
      AddValue(std::atan2(dy, dx), std::max(0.f, 1.f - std::abs(dot)), &h);
    }
  }
  return h;
}
std::vector<float> RotateHist(const std::vector<float>& h, float angle) {
  const int n = static_cast<int>(h.size());
  const float rb = static_cast<float>(static_cast<double>(-angle * static_cast<float>(n)) / M_PI);
  int full = static_cast<int>(std::lround(rb - 0.5f));
  const float f = rb - full;
  while (full < 0) full += n;
  std::vector<float> out(n);
  for (int i = 0; i < n; ++i) out[i] = f * h[(i + 1 + full) % n] + (1.f - f) * h[(i + full) % n];
  return out;
}

template <typename F>
void ParallelFor(int n, int threads, F&& f) {
  std::atomic<int> next{0};
  auto work = [&]() {
    for (int i = next++; i < n; i = next++) f(i);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < std::min(threads, n); ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
}

}  // namespace

struct csm_synth3d {
  csm_synth3d_config cfg;
  std::vector<double> node_pose;  // x, y, z, yaw
  std::vector<std::vector<V3>> raw, high, low;
  std::vector<std::vector<float>> node_hist;
  std::vector<int32_t> submap_node;
  struct Grid {
    std::vector<int32_t> ijk;
    std::vector<uint16_t> values;
  };
  std::vector<Grid> high_grid, low_grid;
  std::vector<std::vector<float>> submap_hist;
  // flattened exports
  std::vector<float> flat;
  std::vector<int64_t> offsets;
};

extern "C" {

void csm_synth3d_default_config(csm_synth3d_config* c) {
  c->seed = 20250127;
  c->world_x = 60.;
  c->world_y = 60.;
  c->world_z = 6.;
  c->num_boxes = 60;
  c->num_nodes = 16;
  c->num_submaps = 4;
  c->scans_per_submap = 20;
  c->rings = 64;
  c->azimuths = 940;
  c->min_elevation = -25. * M_PI / 180.;
  c->max_elevation = 15. * M_PI / 180.;
  c->max_range = 30.;
  c->range_noise = 0.01;
  c->high_resolution = 0.10;
  c->low_resolution = 0.45;
  c->high_resolution_max_range = 20.;
  // trajectory_builder_3d.lua:24-34 (adaptive voxel filters).
  c->high_voxel = 2.;
  c->high_min_points = 150;
  c->high_max_range = 15.;
  c->low_voxel = 4.;
  c->low_min_points = 200;
  c->low_max_range = 60.;
  c->histogram_size = 120;
  c->insert_voxel = 0.15;  // voxel_filter_size (trajectory_builder_3d.lua)
  c->threads = 0;
  c->submap_begin = 0;
  c->submap_count = 0;
}

int csm_synth3d_create(const csm_synth3d_config* cfg, csm_synth3d** out) {
  if (!cfg || !out || cfg->num_nodes <= 0 || cfg->num_submaps < 0 ||
      cfg->num_submaps > cfg->num_nodes || cfg->rings <= 0 || cfg->azimuths <= 0 ||
      cfg->submap_begin < 0 || cfg->submap_count < 0 ||
      (cfg->submap_count > 0 && cfg->submap_begin + cfg->submap_count > cfg->num_submaps))
    return -1;
  auto* w = new csm_synth3d;
  w->cfg = *cfg;
  const int threads = cfg->threads > 0 ? cfg->threads
                                       : static_cast<int>(std::min(16u, std::max(1u, std::thread::hardware_concurrency())));
  std::mt19937_64 rng(cfg->seed);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  const float X = static_cast<float>(cfg->world_x), Y = static_cast<float>(cfg->world_y),
              Z = static_cast<float>(cfg->world_z);
  std::vector<Box> boxes;
  boxes.push_back(Box{{-0.2f, -0.2f, -0.2f}, {X + 0.2f, Y + 0.2f, 0.f}});  // floor
  boxes.push_back(Box{{-0.2f, -0.2f, Z}, {X + 0.2f, Y + 0.2f, Z + 0.2f}});   // ceiling
  boxes.push_back(Box{{-0.2f, -0.2f, 0.f}, {0.f, Y + 0.2f, Z}});
  boxes.push_back(Box{{X, -0.2f, 0.f}, {X + 0.2f, Y + 0.2f, Z}});
  boxes.push_back(Box{{-0.2f, -0.2f, 0.f}, {X + 0.2f, 0.f, Z}});
  boxes.push_back(Box{{-0.2f, Y, 0.f}, {X + 0.2f, Y + 0.2f, Z}});
  for (int i = 0; i < cfg->num_boxes; ++i) {
    const bool pillar = (i % 3) == 0;
    const float sx = pillar ? 0.4f : 0.8f + 2.5f * U(rng), sy = pillar ? 0.4f : 0.8f + 2.5f * U(rng);
    const float sz = pillar ? Z : 0.5f + 2.5f * U(rng);
    const float x = 2.f + (X - 4.f - sx) * U(rng), y = 2.f + (Y - 4.f - sy) * U(rng);
    boxes.push_back(Box{{x, y, 0.f}, {x + sx, y + sy, sz}});
  }
  auto inside_box = [&](float x, float y) {
    for (size_t b = 6; b < boxes.size(); ++b)
      if (x > boxes[b].lo[0] - 0.5f && x < boxes[b].hi[0] + 0.5f && y > boxes[b].lo[1] - 0.5f &&
          y < boxes[b].hi[1] + 0.5f)
        return true;
    return false;
  };
  const int N = cfg->num_nodes;
  w->node_pose.resize(4 * N);
  for (int i = 0; i < N; ++i) {
    float x, y;
    do {
      x = 3.f + (X - 6.f) * U(rng);
      y = 3.f + (Y - 6.f) * U(rng);
    } while (inside_box(x, y));
    w->node_pose[4 * i] = x;
    w->node_pose[4 * i + 1] = y;
    w->node_pose[4 * i + 2] = 1.5;
    w->node_pose[4 * i + 3] = (2.0 * U(rng) - 1.0) * M_PI;
  }
  auto cast_scan = [&](float px, float py, float pz, float yaw, uint64_t seed, int az_step) {
    std::mt19937_64 r(seed);
    std::normal_distribution<float> noise(0.f, static_cast<float>(cfg->range_noise));
    const float cy = std::cos(yaw), sy = std::sin(yaw);
    std::vector<V3> raw;
    for (int ring = 0; ring < cfg->rings; ++ring) {
      const float el = static_cast<float>(cfg->min_elevation +
                                          (cfg->max_elevation - cfg->min_elevation) * ring /
                                              std::max(1, cfg->rings - 1));
      for (int a = 0; a < cfg->azimuths; a += az_step) {
        const float az = static_cast<float>(2.0 * M_PI * a / cfg->azimuths);
        const V3 ds{std::cos(el) * std::cos(az), std::cos(el) * std::sin(az), std::sin(el)};
        const V3 dw{cy * ds.x - sy * ds.y, sy * ds.x + cy * ds.y, ds.z};
        const float rng_m = CastRay(boxes, V3{px, py, pz}, dw, static_cast<float>(cfg->max_range));
        if (rng_m >= cfg->max_range) continue;
        const float rr = rng_m + noise(r);
        raw.push_back(V3{ds.x * rr, ds.y * rr, ds.z * rr});
      }
    }
    return raw;
  };
  std::vector<uint64_t> seeds(N);
  for (int i = 0; i < N; ++i) seeds[i] = rng();
  w->raw.resize(N);
  w->high.resize(N);
  w->low.resize(N);
  w->node_hist.resize(N);
  ParallelFor(N, threads, [&](int i) {
    w->raw[i] = cast_scan(static_cast<float>(w->node_pose[4 * i]),
                          static_cast<float>(w->node_pose[4 * i + 1]),
                          static_cast<float>(w->node_pose[4 * i + 2]),
                          static_cast<float>(w->node_pose[4 * i + 3]), seeds[i], 1);
    const std::vector<V3>& raw = w->raw[i];
    w->high[i] = AdaptiveDecimate(raw, static_cast<float>(cfg->high_voxel), cfg->high_min_points,
                                  static_cast<float>(cfg->high_max_range));
    w->low[i] = AdaptiveDecimate(raw, static_cast<float>(cfg->low_voxel), cfg->low_min_points,
                                 static_cast<float>(cfg->low_max_range));
    // Histogram of the voxel-filtered returns (local_trajectory_builder_3d.cc
    // :898-903; voxel_filter_size 0.15, trajectory_builder_3d.lua).
    w->node_hist[i] = Histogram(VoxelDecimate(raw, static_cast<float>(cfg->insert_voxel), 1e9f),
                                cfg->histogram_size);
  });
  // Submaps: centred on node c = submap_nodes[s], built like a stretch of
  // trajectory around it: the scan of node c itself plus scans_per_submap - 1
  // scans from viewpoints within +-1 m and any yaw (half the azimuths), all
  // in the submap frame (origin = centre position, axes = world axes).
  const int S_all = cfg->num_submaps;
  const int s0 = cfg->submap_count > 0 ? cfg->submap_begin : 0;
  const int S = cfg->submap_count > 0 ? cfg->submap_count : S_all;
  w->submap_node.resize(S);
  w->high_grid.resize(S);
  w->low_grid.resize(S);
  w->submap_hist.resize(S);
  for (int s = 0; s < S; ++s)
    w->submap_node[s] = static_cast<int32_t>((static_cast<int64_t>(s0 + s) * N) / std::max(S_all, 1));
  std::vector<uint64_t> all_seeds(S_all), submap_seeds(S);
  for (int s = 0; s < S_all; ++s) all_seeds[s] = rng();
  for (int s = 0; s < S; ++s) submap_seeds[s] = all_seeds[s0 + s];
  const std::vector<uint16_t> hit = OddsTable(Odds(0.55f)), miss = OddsTable(Odds(0.49f));
  ParallelFor(S, threads, [&](int s) {
    const int c = w->submap_node[s];
    std::mt19937_64 r(submap_seeds[s]);
    std::uniform_real_distribution<float> J(-1.f, 1.f);
    SparseGrid hg{static_cast<float>(cfg->high_resolution), {}, {}};
    SparseGrid lg{static_cast<float>(cfg->low_resolution), {}, {}};
    std::vector<float> hist(cfg->histogram_size, 0.f);
    for (int k = 0; k < std::max(1, cfg->scans_per_submap); ++k) {
      float dx = 0.f, dy = 0.f, yaw = static_cast<float>(w->node_pose[4 * c + 3]);
      std::vector<V3> scan;
      if (k == 0) {
        scan = w->raw[c];
      } else {
        dx = J(r);
        dy = J(r);
        yaw = static_cast<float>(M_PI) * J(r);
        const float vx = static_cast<float>(w->node_pose[4 * c]) + dx,
                    vy = static_cast<float>(w->node_pose[4 * c + 1]) + dy;
        if (inside_box(vx, vy)) continue;
        scan = cast_scan(vx, vy, 1.5f, yaw, r(), 2);
      }
      const float cy = std::cos(yaw), sy = std::sin(yaw);
      const V3 t{dx, dy, 0.f};
      std::vector<V3> pts = VoxelDecimate(scan, static_cast<float>(cfg->insert_voxel), 1e9f);
      std::vector<V3> all, close;
      for (const V3& p : pts) {
        const V3 q{cy * p.x - sy * p.y + t.x, sy * p.x + cy * p.y + t.y, p.z + t.z};
        all.push_back(q);
        if (std::sqrt(p.x * p.x + p.y * p.y + p.z * p.z) <= cfg->high_resolution_max_range) close.push_back(q);
      }
      hg.Insert(t, close, hit, miss, 2);
      lg.Insert(t, all, hit, miss, 2);
      const std::vector<float> rh = RotateHist(Histogram(pts, cfg->histogram_size), yaw);
      for (int b = 0; b < cfg->histogram_size; ++b) hist[b] += rh[b];
    }
    for (int g = 0; g < 2; ++g) {
      SparseGrid& src = g == 0 ? hg : lg;
      csm_synth3d::Grid& dst = g == 0 ? w->high_grid[s] : w->low_grid[s];
      std::vector<std::pair<uint64_t, uint16_t>> cells(src.cells.begin(), src.cells.end());
      std::sort(cells.begin(), cells.end());
      for (auto& kv : cells) {
        if (kv.second == 0) continue;
        dst.ijk.push_back(static_cast<int32_t>((kv.first >> 42) & ((1u << 21) - 1)) - (1 << 20));
        dst.ijk.push_back(static_cast<int32_t>((kv.first >> 21) & ((1u << 21) - 1)) - (1 << 20));
        dst.ijk.push_back(static_cast<int32_t>(kv.first & ((1u << 21) - 1)) - (1 << 20));
        dst.values.push_back(kv.second);
      }
    }
    w->submap_hist[s] = hist;
  });
  *out = w;
  return 0;
}

void csm_synth3d_destroy(csm_synth3d* w) { delete w; }

const double* csm_synth3d_node_poses(const csm_synth3d* w) { return w->node_pose.data(); }
const int32_t* csm_synth3d_submap_nodes(const csm_synth3d* w) { return w->submap_node.data(); }

// kind: 0 raw, 1 high resolution, 2 low resolution. Returns the point count.
int64_t csm_synth3d_cloud(const csm_synth3d* w, int32_t node, int32_t kind, float* out,
                          int64_t capacity) {
  const std::vector<V3>& c = kind == 0 ? w->raw[node] : kind == 1 ? w->high[node] : w->low[node];
  const int64_t n = static_cast<int64_t>(c.size());
  if (out && capacity >= n)
    for (int64_t i = 0; i < n; ++i) {
      out[3 * i] = c[i].x;
      out[3 * i + 1] = c[i].y;
      out[3 * i + 2] = c[i].z;
    }
  return n;
}

void csm_synth3d_node_histogram(const csm_synth3d* w, int32_t node, float* out) {
  std::copy(w->node_hist[node].begin(), w->node_hist[node].end(), out);
}
void csm_synth3d_submap_histogram(const csm_synth3d* w, int32_t submap, float* out) {
  std::copy(w->submap_hist[submap].begin(), w->submap_hist[submap].end(), out);
}

// grid: 0 high resolution, 1 low resolution. Returns the cell count.
int64_t csm_synth3d_grid(const csm_synth3d* w, int32_t submap, int32_t grid, int32_t* ijk,
                         uint16_t* values, int64_t capacity) {
  const csm_synth3d::Grid& g = grid == 0 ? w->high_grid[submap] : w->low_grid[submap];
  const int64_t n = static_cast<int64_t>(g.values.size());
  if (ijk && values && capacity >= n) {
    std::copy(g.ijk.begin(), g.ijk.end(), ijk);
    std::copy(g.values.begin(), g.values.end(), values);
  }
  return n;
}

}  // extern "C"
