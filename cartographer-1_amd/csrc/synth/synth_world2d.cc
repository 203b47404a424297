// Synthetic 2D world for benchmarks and parity tests.
//
// Not part of the matching path: it only produces inputs of the reference's
// shapes — node point clouds (RangefinderPoint xyz, sensor frame, z = 0) and
// submap ProbabilityGrid cells (uint16 correspondence-cost values, x fastest,
// mapping/2d/grid_2d.h:113-116) — deterministically from a seed.
//
// World: a building of rooms on a lattice (walls with doorways, some walls
// removed) plus random boxes, rasterised at the grid resolution. Nodes are
// random collision-free poses; each casts `beams` rays over `fov` (range noise
// sigma). A global map is accumulated from every node's rays with the
// reference's hit/miss odds (trajectory_builder_2d.lua:97-98) and the value
// encoding of mapping/probability_values.h; submaps are fixed-size windows
// of that map centred on node positions, unobserved cells unknown (0).

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "csm_synth.h"

namespace {

struct Raster {
  int nx = 0, ny = 0;  // columns along world x, rows along world y
  double res = 0.05;
  std::vector<uint8_t> occ;
  bool Occupied(int cx, int cy) const {
    if (cx < 0 || cy < 0 || cx >= nx || cy >= ny) return true;
    return occ[static_cast<size_t>(cy) * nx + cx] != 0;
  }
  void FillRect(double x0, double y0, double x1, double y1) {
    const int cx0 = std::max(0, static_cast<int>(std::floor(x0 / res)));
    const int cy0 = std::max(0, static_cast<int>(std::floor(y0 / res)));
    const int cx1 = std::min(nx - 1, static_cast<int>(std::floor(x1 / res)));
    const int cy1 = std::min(ny - 1, static_cast<int>(std::floor(y1 / res)));
    for (int y = cy0; y <= cy1; ++y)
      for (int x = cx0; x <= cx1; ++x) occ[static_cast<size_t>(y) * nx + x] = 1;
  }
};

// Amanatides-Woo traversal; calls visit(cx, cy) for every free cell before the
// hit and returns the hit distance (or -1 if nothing within max_range).
template <typename F>
double CastRay(const Raster& r, double ox, double oy, double dx, double dy,
               double max_range, F&& visit) {
  int cx = static_cast<int>(std::floor(ox / r.res));
  int cy = static_cast<int>(std::floor(oy / r.res));
  const int sx = dx > 0 ? 1 : -1, sy = dy > 0 ? 1 : -1;
  const double inv_dx = dx != 0 ? std::abs(1.0 / dx) : 1e300;
  const double inv_dy = dy != 0 ? std::abs(1.0 / dy) : 1e300;
  double tmx = dx > 0 ? ((cx + 1) * r.res - ox) * inv_dx
                      : dx < 0 ? (ox - cx * r.res) * inv_dx : 1e300;
  double tmy = dy > 0 ? ((cy + 1) * r.res - oy) * inv_dy
                      : dy < 0 ? (oy - cy * r.res) * inv_dy : 1e300;
  const double tdx = r.res * inv_dx, tdy = r.res * inv_dy;
  double t = 0.0;
  while (t <= max_range) {
    if (r.Occupied(cx, cy)) return t;
    visit(cx, cy);
    if (tmx < tmy) {
      t = tmx;
      tmx += tdx;
      cx += sx;
    } else {
      t = tmy;
      tmy += tdy;
      cy += sy;
    }
  }
  return -1.0;
}

// mapping/probability_values.h:32-45, 84-87
uint16_t CostToValue(float cc) {
  const float lo = 1.f - (1.f - 0.1f), hi = 1.f - 0.1f;
  const float c = std::min(std::max(cc, lo), hi);
  return static_cast<uint16_t>(std::lround((c - lo) * (32766.f / (hi - lo))) + 1);
}

template <typename F>
void ParallelFor(int n, int threads, F&& f) {
  std::atomic<int> next{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&] {
      for (int i = next++; i < n; i = next++) f(i);
    });
  for (auto& th : pool) th.join();
}

}  // namespace

struct csm_synth2d {
  csm_synth2d_config cfg;
  std::vector<double> node_pose;          // x, y, theta per node
  std::vector<int64_t> point_offsets;     // num_nodes + 1
  std::vector<float> points;              // xyz
  std::vector<double> submap_max;         // max_x, max_y per submap
  std::vector<int32_t> submap_node;       // centre node per submap
  std::vector<uint16_t> submap_cells;     // num_submaps * cells^2
};

extern "C" {

void csm_synth2d_default_config(csm_synth2d_config* c) {
  std::memset(c, 0, sizeof(*c));
  c->seed = 20250127ull;
  c->world_x = 200.0;
  c->world_y = 100.0;
  c->resolution = 0.05;
  c->num_nodes = 500;
  c->num_submaps = 50;
  c->submap_cells = 400;
  c->beams = 1080;
  c->fov = 270.0 * M_PI / 180.0;
  c->max_range = 30.0;
  c->range_noise = 0.01;
  c->decimate_to = 0;
  c->room_size = 8.0;
  c->boxes_per_room = 3;
  c->threads = 0;
}

int csm_synth2d_create(const csm_synth2d_config* cfg, csm_synth2d** out) {
  if (!cfg || !out || cfg->num_nodes <= 0 || cfg->num_submaps < 0 ||
      cfg->submap_cells <= 0 || cfg->beams <= 0 || cfg->resolution <= 0)
    return -1;
  auto* w = new csm_synth2d;
  w->cfg = *cfg;
  const int threads = cfg->threads > 0
                          ? cfg->threads
                          : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::mt19937_64 rng(cfg->seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);

  // --- world raster --------------------------------------------------------
  Raster r;
  r.res = cfg->resolution;
  r.nx = static_cast<int>(std::ceil(cfg->world_x / r.res));
  r.ny = static_cast<int>(std::ceil(cfg->world_y / r.res));
  r.occ.assign(static_cast<size_t>(r.nx) * r.ny, 0);
  const double wall = 0.1, W = cfg->world_x, H = cfg->world_y;
  r.FillRect(0, 0, W, wall);
  r.FillRect(0, H - wall, W, H);
  r.FillRect(0, 0, wall, H);
  r.FillRect(W - wall, 0, W, H);
  const double room = cfg->room_size > 0 ? cfg->room_size : 8.0;
  const int rx = std::max(1, static_cast<int>(W / room));
  const int ry = std::max(1, static_cast<int>(H / room));
  const double sxr = W / rx, syr = H / ry;
  for (int i = 1; i < rx; ++i)  // vertical walls, one segment per room row
    for (int j = 0; j < ry; ++j) {
      if (U(rng) < 0.2) continue;  // open plan
      const double x = i * sxr, y0 = j * syr, y1 = (j + 1) * syr;
      const double door = 1.0 + 1.0 * U(rng);
      const double dpos = y0 + 0.5 + (syr - door - 1.0) * U(rng);
      r.FillRect(x - wall / 2, y0, x + wall / 2, dpos);
      r.FillRect(x - wall / 2, dpos + door, x + wall / 2, y1);
    }
  for (int j = 1; j < ry; ++j)  // horizontal walls
    for (int i = 0; i < rx; ++i) {
      if (U(rng) < 0.2) continue;
      const double y = j * syr, x0 = i * sxr, x1 = (i + 1) * sxr;
      const double door = 1.0 + 1.0 * U(rng);
      const double dpos = x0 + 0.5 + (sxr - door - 1.0) * U(rng);
      r.FillRect(x0, y - wall / 2, dpos, y + wall / 2);
      r.FillRect(dpos + door, y - wall / 2, x1, y + wall / 2);
    }
  for (int i = 0; i < rx; ++i)  // furniture
    for (int j = 0; j < ry; ++j)
      for (int b = 0; b < cfg->boxes_per_room; ++b) {
        const double bw = 0.3 + 1.2 * U(rng), bh = 0.3 + 1.2 * U(rng);
        const double bx = i * sxr + 0.8 + (sxr - 1.6 - bw) * U(rng);
        const double by = j * syr + 0.8 + (syr - 1.6 - bh) * U(rng);
        r.FillRect(bx, by, bx + bw, by + bh);
      }

  // --- node poses: collision-free with 0.4 m clearance ---------------------
  const int N = cfg->num_nodes;
  w->node_pose.resize(3 * static_cast<size_t>(N));
  const int clr = static_cast<int>(std::ceil(0.4 / r.res));
  for (int n = 0; n < N; ++n) {
    for (;;) {
      const double x = 1.0 + (W - 2.0) * U(rng), y = 1.0 + (H - 2.0) * U(rng);
      const int cx = static_cast<int>(x / r.res), cy = static_cast<int>(y / r.res);
      bool ok = true;
      for (int dy = -clr; dy <= clr && ok; ++dy)
        for (int dx = -clr; dx <= clr && ok; ++dx) ok = !r.Occupied(cx + dx, cy + dy);
      if (!ok) continue;
      w->node_pose[3 * n] = x;
      w->node_pose[3 * n + 1] = y;
      w->node_pose[3 * n + 2] = (2.0 * U(rng) - 1.0) * M_PI;
      break;
    }
  }
  std::vector<uint64_t> node_seed(N);
  for (int n = 0; n < N; ++n) node_seed[n] = rng();

  // --- scans + global hit/miss counts --------------------------------------
  std::vector<std::vector<float>> pts(N);
  std::vector<std::atomic<uint32_t>> hits(static_cast<size_t>(r.nx) * r.ny);
  std::vector<std::atomic<uint32_t>> misses(static_cast<size_t>(r.nx) * r.ny);
  for (auto& h : hits) h.store(0, std::memory_order_relaxed);
  for (auto& m : misses) m.store(0, std::memory_order_relaxed);
  ParallelFor(N, threads, [&](int n) {
    std::mt19937_64 nrng(node_seed[n]);
    std::normal_distribution<double> noise(0.0, cfg->range_noise);
    const double ox = w->node_pose[3 * n], oy = w->node_pose[3 * n + 1];
    const double th = w->node_pose[3 * n + 2];
    std::vector<float>& out = pts[n];
    for (int b = 0; b < cfg->beams; ++b) {
      const double a = -0.5 * cfg->fov +
                       (cfg->beams > 1 ? cfg->fov * b / (cfg->beams - 1) : 0.0);
      const double dx = std::cos(th + a), dy = std::sin(th + a);
      const double d = CastRay(r, ox, oy, dx, dy, cfg->max_range, [&](int cx, int cy) {
        misses[static_cast<size_t>(cy) * r.nx + cx].fetch_add(1, std::memory_order_relaxed);
      });
      if (d < 0) continue;
      const double rr = d + 0.5 * r.res * 0.2 + noise(nrng);
      const double hx = ox + rr * dx, hy = oy + rr * dy;
      const int hcx = static_cast<int>(std::floor(hx / r.res));
      const int hcy = static_cast<int>(std::floor(hy / r.res));
      if (hcx >= 0 && hcy >= 0 && hcx < r.nx && hcy < r.ny)
        hits[static_cast<size_t>(hcy) * r.nx + hcx].fetch_add(1, std::memory_order_relaxed);
      out.push_back(static_cast<float>(rr * std::cos(a)));
      out.push_back(static_cast<float>(rr * std::sin(a)));
      out.push_back(0.f);
    }
    if (cfg->decimate_to > 0) {
      const int np = static_cast<int>(out.size() / 3);
      if (np > cfg->decimate_to) {
        std::vector<float> dec;
        dec.reserve(3 * static_cast<size_t>(cfg->decimate_to));
        for (int k = 0; k < cfg->decimate_to; ++k) {
          const int src = static_cast<int>(static_cast<int64_t>(k) * np / cfg->decimate_to);
          dec.insert(dec.end(), out.begin() + 3 * src, out.begin() + 3 * src + 3);
        }
        out.swap(dec);
      }
    }
  });
  w->point_offsets.resize(N + 1);
  w->point_offsets[0] = 0;
  for (int n = 0; n < N; ++n)
    w->point_offsets[n + 1] = w->point_offsets[n] + static_cast<int64_t>(pts[n].size() / 3);
  w->points.resize(3 * static_cast<size_t>(w->point_offsets[N]));
  for (int n = 0; n < N; ++n)
    std::copy(pts[n].begin(), pts[n].end(), w->points.begin() + 3 * w->point_offsets[n]);

  // Global map values from the odds model (hit 0.55, miss 0.49).
  const double lo_hit = std::log(0.55 / 0.45), lo_miss = std::log(0.49 / 0.51);
  std::vector<uint16_t> global(static_cast<size_t>(r.nx) * r.ny, 0);
  ParallelFor(r.ny, threads, [&](int y) {
    for (int x = 0; x < r.nx; ++x) {
      const size_t i = static_cast<size_t>(y) * r.nx + x;
      const uint32_t h = hits[i].load(), m = misses[i].load();
      if (h == 0 && m == 0) continue;
      const double lo = h * lo_hit + m * lo_miss;
      const double p = 1.0 / (1.0 + std::exp(-std::max(-50.0, std::min(50.0, lo))));
      global[i] = CostToValue(static_cast<float>(1.0 - p));
    }
  });

  // --- submaps: windows centred on evenly spaced nodes ---------------------
  const int S = cfg->num_submaps, C = cfg->submap_cells;
  w->submap_max.resize(2 * static_cast<size_t>(S));
  w->submap_node.resize(S);
  w->submap_cells.assign(static_cast<size_t>(S) * C * C, 0);
  ParallelFor(S, threads, [&](int s) {
    const int node = static_cast<int>(static_cast<int64_t>(s) * N / std::max(1, S));
    w->submap_node[s] = node;
    // Snap the window corner to the raster so cells align with world cells.
    const int ccx = static_cast<int>(std::floor(w->node_pose[3 * node] / r.res));
    const int ccy = static_cast<int>(std::floor(w->node_pose[3 * node + 1] / r.res));
    const int max_cx = ccx + C / 2, max_cy = ccy + C / 2;  // exclusive corner
    const double max_x = max_cx * r.res, max_y = max_cy * r.res;
    w->submap_max[2 * s] = max_x;
    w->submap_max[2 * s + 1] = max_y;
    uint16_t* cells = &w->submap_cells[static_cast<size_t>(s) * C * C];
    // Cell (i, j): i along -y from max_y, j along -x from max_x
    // (map_limits.h:69-75); flat index i + j * C (grid_2d.h:113-116).
    for (int j = 0; j < C; ++j)
      for (int i = 0; i < C; ++i) {
        const int wx = max_cx - 1 - j, wy = max_cy - 1 - i;
        if (wx < 0 || wy < 0 || wx >= r.nx || wy >= r.ny) continue;
        cells[i + static_cast<size_t>(j) * C] = global[static_cast<size_t>(wy) * r.nx + wx];
      }
  });
  *out = w;
  return 0;
}

void csm_synth2d_destroy(csm_synth2d* w) { delete w; }

int32_t csm_synth2d_num_nodes(const csm_synth2d* w) { return w->cfg.num_nodes; }
int32_t csm_synth2d_num_submaps(const csm_synth2d* w) { return w->cfg.num_submaps; }
const int64_t* csm_synth2d_point_offsets(const csm_synth2d* w) { return w->point_offsets.data(); }
const float* csm_synth2d_points(const csm_synth2d* w) { return w->points.data(); }
const double* csm_synth2d_node_poses(const csm_synth2d* w) { return w->node_pose.data(); }
const double* csm_synth2d_submap_max(const csm_synth2d* w) { return w->submap_max.data(); }
const int32_t* csm_synth2d_submap_nodes(const csm_synth2d* w) { return w->submap_node.data(); }
const uint16_t* csm_synth2d_submap_cells(const csm_synth2d* w) { return w->submap_cells.data(); }

}  // extern "C"
