// Host runtime of the MI355X correlative scan matcher: implements the C-ABI
// of include/csm_amd.h on top of the kernels in csm_kernels.hip.
//
// Ownership follows the reference (fast_correlative_scan_matcher_2d.cc:188-194
// copies what it needs from the grid): csm_fast2d_create copies the cells to
// the device and builds the pyramid there; handles own device memory until
// destroyed. Results are decoded on the host with the reference's double
// arithmetic (Candidate2D, correlative_scan_matcher_2d.h:75-85, and the pose
// composition of fast_correlative_scan_matcher_2d.cc:253-259).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <tuple>
#include <vector>

#include "../../include/csm_amd.h"
#include "csm_device.h"
#include "csm_internal.h"
#include "csm_launch.h"
#include "search_window.h"

namespace csm {



namespace {


int AutoSearchDepth(int configured, int nx, int ny) {
  // Extra coarse levels until the top lattice step reaches ~1/2 of the grid:
  // measured on the synthetic world this cuts lookups 2-4x.
  int d = configured;
  const int span = std::max(nx, ny);
  while (d < kMaxLevels && (1 << (d - 1)) < span / 2) ++d;
  return std::max(d, configured);
}

// Scan cluster size per child level (SubmapDesc::cshift): k = 1, 2, 2, 4, 4,
// 8, ... cells per side (log2), chosen by tools/frontier_sim.py (cluster) on
// the C2 world: 0.39x the lookups of exact per-level bounds. Level 0 is
// always exact (k = 1) and k <= 2^level. CSM_CLUSTER="s0,s1,..." overrides.
void ClusterShifts(int32_t* out) {
  static const int kDefault[kMaxLevels] = {0, 1, 1, 2, 2, 3, 3, 3, 3, 3, 3, 3};
  for (int l = 0; l < kMaxLevels; ++l) out[l] = kDefault[l];
  if (const char* env = std::getenv("CSM_CLUSTER")) {
    int l = 0;
    for (const char* c = env; *c && l < kMaxLevels; ++l) {
      out[l] = std::atoi(c);
      while (*c && *c != ',') ++c;
      if (*c == ',') ++c;
    }
    for (; l < kMaxLevels; ++l) out[l] = out[l - 1];
  }
  for (int l = 0; l < kMaxLevels; ++l)
    out[l] = std::max(0, std::min({out[l], l, kMaxClusterShift}));
}

}  // namespace
}  // namespace csm

using namespace csm;


namespace {

int EnsureDevice(csm_context* ctx) {
  return hipSetDevice(ctx->device) == hipSuccess ? CSM_OK : CSM_EHIP;
}

const std::pair<SearchWindow2D, std::vector<ZRot>>& WindowFor(
    csm_scan_set* s, int scan, double lin, double ang, double res) {
  const auto key = std::make_tuple(scan, ang, lin, res);
  auto it = s->windows.find(key);
  if (it != s->windows.end()) return it->second;
  const int64_t b = s->offsets[scan], e = s->offsets[scan + 1];
  // FastCSM builds SearchParameters from the input cloud (:202-204, :215-218).
  SearchWindow2D w = MakeSearchWindow2D(lin, ang, s->host_points.data() + 3 * b,
                                        static_cast<int32_t>(e - b), res, nullptr);
  std::vector<ZRot> table;
  RotationTable(w, &table);
  return s->windows.emplace(key, std::make_pair(w, std::move(table))).first->second;
}

int RunBatch(csm_context* ctx, csm_fast2d* const* submaps, int32_t num_submaps,
             csm_scan_set* scans, const csm_pair2d* pairs, int64_t num_pairs,
             csm_result2d* results) {
  // ---- host preparation ---------------------------------------------------
  std::vector<SubmapDesc> sdesc(num_submaps);
  for (int i = 0; i < num_submaps; ++i) {
    if (!submaps[i] || submaps[i]->ctx != ctx) return CSM_EINVAL;
    sdesc[i] = submaps[i]->desc;
    // One launch serves one kernel: v4 (no hex levels) or v5 (fixed at create).
    if ((sdesc[i].hex_mask != 0) != (sdesc[0].hex_mask != 0)) return CSM_EINVAL;
  }
  const bool hex = num_submaps > 0 && sdesc[0].hex_mask != 0;
  std::vector<PairDesc> pdesc;
  std::vector<int64_t> pair_src;  // pdesc index -> pair index
  std::vector<float2> rot_host;
  std::map<const void*, int32_t> rot_offsets;  // table ptr -> offset
  int max_npad = 64;
  for (int64_t i = 0; i < num_pairs; ++i) {
    const csm_pair2d& p = pairs[i];
    results[i].status = CSM_NO_MATCH;
    results[i].score = 0.f;
    results[i].pose = csm_pose2d{0., 0., 0.};
    if (p.submap < 0 || p.submap >= num_submaps || p.scan < 0 ||
        p.scan >= static_cast<int32_t>(scans->offsets.size()) - 1) {
      results[i].status = CSM_EINVAL;
      continue;
    }
    const csm_fast2d* m = submaps[p.submap];
    const int32_t n = static_cast<int32_t>(scans->offsets[p.scan + 1] - scans->offsets[p.scan]);
    if (n <= 0) continue;  // empty cloud: the reference cannot exceed min_score
    if (n > kMaxPoints) { results[i].status = CSM_ERANGE; continue; }
    const double res = m->limits.resolution;
    double lin, ang;
    csm_pose2d init;
    if (p.full_submap) {
      // fast_correlative_scan_matcher_2d.cc:215-222
      lin = 1e6 * res;
      ang = M_PI;
      const double half = 0.5 * res;
      init.x = m->limits.max_x - half * m->limits.num_y_cells;
      init.y = m->limits.max_y - half * m->limits.num_x_cells;
      init.theta = 0.;
    } else {
      lin = m->options.linear_search_window;
      ang = m->options.angular_search_window;
      init = p.initial;
    }
    const auto& win = WindowFor(scans, p.scan, lin, ang, res);
    if (win.first.num_scans > kMaxRotations) { results[i].status = CSM_ERANGE; continue; }
    auto ro = rot_offsets.find(&win);
    int32_t off;
    if (ro == rot_offsets.end()) {
      off = static_cast<int32_t>(rot_host.size());
      for (const ZRot& z : win.second) rot_host.push_back(make_float2(z.w, z.s));
      rot_offsets.emplace(&win, off);
    } else {
      off = ro->second;
    }
    PairDesc d{};
    d.submap = p.submap;
    d.num_points = n;
    d.point_offset = scans->offsets[p.scan];
    d.rot_offset = off;
    d.num_scans = win.first.num_scans;
    d.num_linear = std::min(win.first.num_linear_perturbations, 1 << 20);
    d.max_rejected_sum = static_cast<int32_t>(MaxRejectedSum(p.min_score, n, m->min_s, m->max_s));
    d.tx = static_cast<float>(init.x);
    d.ty = static_cast<float>(init.y);
    const ZRot pre = MakeZRot(static_cast<float>(init.theta));
    d.pre_w = pre.w;
    d.pre_s = pre.s;
    pdesc.push_back(d);
    pair_src.push_back(i);
    max_npad = std::max(max_npad, (n + 63) & ~63);
  }
  const int np = static_cast<int>(pdesc.size());
  if (np == 0) return CSM_OK;

  const char* forced_env = std::getenv("CSM_SEARCH_KERNEL");
  const int forced = forced_env ? std::atoi(forced_env) : 0;
  // The v4 kernel keeps rot_chunk discretized scans (4 B/point) in LDS;
  // above ~8k points per scan the v1 kernel (lanes = points) is used.
  const bool use_v2 = forced == 2 || (forced != 1 && max_npad <= 8192);
  const char* rc_env = std::getenv("CSM_ROT_CHUNK");
  const int v4_budget = 9 * 1024;  // C2 (1088 padded points): 2 rotations per chunk, the measured best
  const int v4_rc = rc_env ? std::max(1, std::min(16, std::atoi(rc_env)))
                           : std::max(1, std::min(8, v4_budget / (max_npad * 4)));
  const int lds_budget = 40 * 1024;
  const int rc = use_v2 ? v4_rc : std::max(1, std::min(16, lds_budget / (max_npad * 4)));

  // Per-XCD queues: submap s -> queue s % 8 so a submap's pyramid stays in
  // one XCD's L2; pairs within a queue in submap order.
  std::vector<std::vector<int32_t>> q(kNumXcd);
  for (int i = 0; i < np; ++i) q[pdesc[i].submap % kNumXcd].push_back(i);
  // Rebalance: if a queue is much larger than the mean, spill whole submaps.
  std::vector<int32_t> order;
  std::vector<int64_t> prefix;
  WorkQueues wq{};
  wq.rot_chunk = rc;
  int64_t running = 0;
  for (int x = 0; x < kNumXcd; ++x) {
    std::stable_sort(q[x].begin(), q[x].end(),
                     [&](int a, int b) { return pdesc[a].submap < pdesc[b].submap; });
    wq.queue_begin[x] = static_cast<int32_t>(order.size());
    const int64_t qstart = running;
    for (int pi : q[x]) {
      order.push_back(pi);
      prefix.push_back(running);
      running += (pdesc[pi].num_scans + rc - 1) / rc;
    }
    wq.queue_chunks[x] = running - qstart;
  }
  wq.queue_begin[kNumXcd] = static_cast<int32_t>(order.size());
  prefix.push_back(running);

  // ---- uploads ---------------------------------------------------------------
  int rcode;
  if ((rcode = ctx->submap_desc.Reserve(sizeof(SubmapDesc) * num_submaps))) return rcode;
  if ((rcode = ctx->pair_desc.Reserve(sizeof(PairDesc) * np))) return rcode;
  if ((rcode = ctx->rot_table.Reserve(sizeof(float2) * rot_host.size()))) return rcode;
  if ((rcode = ctx->best.Reserve(sizeof(uint64_t) * np))) return rcode;
  if ((rcode = ctx->status.Reserve(sizeof(int32_t) * np))) return rcode;
  if ((rcode = ctx->counters.Reserve(sizeof(unsigned long long) * kNumXcd))) return rcode;
  if ((rcode = ctx->pair_order.Reserve(sizeof(int32_t) * order.size()))) return rcode;
  if ((rcode = ctx->chunk_prefix.Reserve(sizeof(int64_t) * prefix.size()))) return rcode;
  if ((rcode = ctx->stats.Reserve(sizeof(unsigned long long) * kStatsWords))) return rcode;
  hipStream_t st = ctx->stream;
  CSM_HIP(hipMemcpyAsync(ctx->submap_desc.ptr, sdesc.data(), sizeof(SubmapDesc) * num_submaps,
                         hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(ctx->pair_desc.ptr, pdesc.data(), sizeof(PairDesc) * np,
                         hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(ctx->rot_table.ptr, rot_host.data(), sizeof(float2) * rot_host.size(),
                         hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(ctx->pair_order.ptr, order.data(), sizeof(int32_t) * order.size(),
                         hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(ctx->chunk_prefix.ptr, prefix.data(), sizeof(int64_t) * prefix.size(),
                         hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemsetAsync(ctx->best.ptr, 0, sizeof(uint64_t) * np, st));
  CSM_HIP(hipMemsetAsync(ctx->status.ptr, 0, sizeof(int32_t) * np, st));
  CSM_HIP(hipMemsetAsync(ctx->counters.ptr, 0, sizeof(unsigned long long) * kNumXcd, st));
  CSM_HIP(hipMemsetAsync(ctx->stats.ptr, 0, sizeof(unsigned long long) * kStatsWords, st));
  wq.pair_order = ctx->pair_order.as<int32_t>();
  wq.chunk_prefix = ctx->chunk_prefix.as<int64_t>();

  // ---- launch: persistent workgroups ----------------------------------------
  const int64_t total_chunks = running;
  if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev0, st));
  if (use_v2) {
    // Block table: for every 64 chunks of a queue, the first pair_order entry.
    std::vector<int32_t> blocks;
    WorkQueues2 wq2{};
    wq2.rot_chunk = rc;
    for (int x = 0; x < kNumXcd; ++x) {
      wq2.queue_begin[x] = wq.queue_begin[x];
      wq2.queue_chunks[x] = wq.queue_chunks[x];
      wq2.block_offset[x] = static_cast<int32_t>(blocks.size());
      const int64_t qstart = prefix[wq.queue_begin[x]];
      int e = wq.queue_begin[x];
      for (int64_t c = 0; c < wq.queue_chunks[x]; c += 64) {
        while (prefix[e + 1] - qstart <= c) ++e;
        blocks.push_back(e);
      }
    }
    wq2.queue_begin[kNumXcd] = wq.queue_begin[kNumXcd];
    if ((rcode = ctx->blocks.Reserve(sizeof(int32_t) * std::max<size_t>(blocks.size(), 1))))
      return rcode;
    if (!blocks.empty())
      CSM_HIP(hipMemcpyAsync(ctx->blocks.ptr, blocks.data(), sizeof(int32_t) * blocks.size(),
                             hipMemcpyHostToDevice, st));
    wq2.pair_order = wq.pair_order;
    wq2.chunk_prefix = wq.chunk_prefix;
    wq2.block_first = ctx->blocks.as<int32_t>();
    // Per rotation: npad raw cells / k = 1 entries and capc cluster-list
    // entries, 4 B cell + 1 B count each, 16-B aligned. capc = 3/4 npad holds
    // the three cluster lists of a typical scan (0.55 npad on C2); a list
    // that does not fit falls back to a finer one in the kernel.
    int capc = (3 * max_npad / 4 + 63) & ~63;
    if (const char* ce = std::getenv("CSM_CAPC_PCT"))  // A/B: cluster-list room, % of npad
      capc = std::max(64, (std::atoi(ce) * max_npad / 100 + 63) & ~63);
    const int lds_cap = 96 * 1024;
    // Per rotation: npad raw cells (4 B) + capc cluster entries (4 B cell + 1 B count).
    auto dyn_bytes = [&](int cap) { return static_cast<size_t>(rc) * (max_npad * 4 + cap * 5); };
    while (capc > 0 && dyn_bytes(capc) > lds_cap) capc -= 64;
    const size_t dyn_lds = (dyn_bytes(capc) + 15) & ~size_t{15};
    // Node order: FIFO (level by level, the default) or LIFO (depth-first,
    // CSM_SEARCH_ORDER=lifo).
    const char* order_env = std::getenv("CSM_SEARCH_ORDER");
    const bool fifo = !(order_env && std::strcmp(order_env, "lifo") == 0);
    // Workgroups per CU: what registers and LDS allow (the runtime's
    // occupancy query). CSM_WG_PER_CU caps it (A/B runs).
    int per_cu = std::max(1, std::min(8, Fast2dSearchV2BlocksPerCu(hex, fifo, dyn_lds)));
    if (const char* w = std::getenv("CSM_WG_PER_CU")) per_cu = std::max(1, std::min(per_cu, std::atoi(w)));
    if (std::getenv("CSM_PROFILE2D"))
      std::fprintf(stderr, "fast2d launch: %s %s, %d rotations per item, %zu B dynamic LDS (capc %d), %d workgroups per CU\n",
                   hex ? "v5" : "v4", fifo ? "fifo" : "lifo", rc, dyn_lds, capc, per_cu);
    const int grid = static_cast<int>(std::min<int64_t>(static_cast<int64_t>(ctx->num_cus) * per_cu,
                                                        std::max<int64_t>(total_chunks, 1)));
    // DFS stack spill: kSpill2 entries per persistent workgroup.
    if ((rcode = ctx->spill.Reserve(sizeof(uint2) * kSpill2 * static_cast<size_t>(grid))))
      return rcode;
    CSM_HIP(LaunchFast2dSearchV2(grid, dyn_lds, st, ctx->submap_desc.as<SubmapDesc>(),
                                 ctx->pair_desc.as<PairDesc>(), scans->points.as<float>(),
                                 ctx->rot_table.as<float2>(), wq2,
                                 ctx->counters.as<unsigned long long>(), ctx->best.as<uint64_t>(),
                                 ctx->status.as<int32_t>(), ctx->stats.as<unsigned long long>(),
                                 ctx->spill.as<uint2>(), max_npad, capc, hex, fifo));
  } else {
    const size_t dyn_lds = static_cast<size_t>(rc) * max_npad * sizeof(uint32_t);
    const int grid = static_cast<int>(std::min<int64_t>(static_cast<int64_t>(ctx->num_cus) * 4,
                                                        std::max<int64_t>(total_chunks, 1)));
    CSM_HIP(LaunchFast2dSearch(grid, dyn_lds, st, ctx->submap_desc.as<SubmapDesc>(),
                               ctx->pair_desc.as<PairDesc>(), scans->points.as<float>(),
                               ctx->rot_table.as<float2>(), wq,
                               ctx->counters.as<unsigned long long>(), ctx->best.as<uint64_t>(),
                               ctx->status.as<int32_t>(), ctx->stats.as<unsigned long long>()));
  }
  if (ctx->timing) CSM_HIP(hipEventRecord(ctx->ev1, st));

  std::vector<uint64_t> keys(np);
  std::vector<int32_t> stat(np);
  unsigned long long stats_host[kStatsWords] = {0};
  CSM_HIP(hipMemcpyAsync(keys.data(), ctx->best.ptr, sizeof(uint64_t) * np,
                         hipMemcpyDeviceToHost, st));
  CSM_HIP(hipMemcpyAsync(stat.data(), ctx->status.ptr, sizeof(int32_t) * np,
                         hipMemcpyDeviceToHost, st));
  CSM_HIP(hipMemcpyAsync(stats_host, ctx->stats.ptr, sizeof(stats_host),
                         hipMemcpyDeviceToHost, st));
  CSM_HIP(hipStreamSynchronize(st));
  if (ctx->timing) {
    float ms = 0.f;
    CSM_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    ctx->t.search_kernel_ms += ms;
    ctx->t.search_launches += 1;
    ctx->t.search_candidates += static_cast<double>(stats_host[0]);
    ctx->t.search_lookups += static_cast<double>(stats_host[1]);
    for (int l = 0; l < kMaxLevels; ++l) {
      ctx->level_cands[l] += static_cast<double>(stats_host[2 + l]);
      ctx->level_batches[l] += static_cast<double>(stats_host[2 + kMaxLevels + l]);
    }
    ctx->t.stack_high_water = std::max<int64_t>(ctx->t.stack_high_water,
                                                static_cast<int64_t>(stats_host[kStatHighWater]));
    const unsigned long long* kp = stats_host + 2 + 2 * kMaxLevels;
    if (std::getenv("CSM_PROFILE2D") && (kp[0] | kp[1] | kp[2]))
      std::fprintf(stderr,
                   "fast2d phases (Mcycles, thread 0 sums): setup %.1f (entry lists %.1f) control "
                   "%.1f score %.1f\n",
                   kp[0] / 1e6, kp[3] / 1e6, kp[1] / 1e6, kp[2] / 1e6);
  }

  // ---- decode -----------------------------------------------------------------
  for (int k = 0; k < np; ++k) {
    const int64_t i = pair_src[k];
    const PairDesc& d = pdesc[k];
    const csm_pair2d& p = pairs[i];
    const csm_fast2d* m = submaps[p.submap];
    if (stat[k] & kStatusRange) {
      results[i].status = CSM_ERANGE;
      ctx->t.search_errors += 1;
      continue;
    }
    uint32_t sum;
    int rot, xo, yo;
    UnpackLeafKey(keys[k], &sum, &rot, &xo, &yo);
    if (keys[k] == 0 || static_cast<int64_t>(sum) <= d.max_rejected_sum) {
      results[i].status = CSM_NO_MATCH;
      continue;
    }
    const double res = m->limits.resolution;
    csm_pose2d init;
    if (p.full_submap) {
      const double half = 0.5 * res;
      init.x = m->limits.max_x - half * m->limits.num_y_cells;
      init.y = m->limits.max_y - half * m->limits.num_x_cells;
      init.theta = 0.;
    } else {
      init = p.initial;
    }
    const double lin = p.full_submap ? 1e6 * res : m->options.linear_search_window;
    const double ang = p.full_submap ? M_PI : m->options.angular_search_window;
    const SearchWindow2D& w = WindowFor(scans, p.scan, lin, ang, res).first;
    // Candidate2D: x = -y_off * res, y = -x_off * res,
    // orientation = (scan_index - num_angular) * step.
    const double cx = -yo * res, cy = -xo * res;
    const double co = (rot - w.num_angular_perturbations) * w.angular_perturbation_step_size;
    results[i].status = CSM_OK;
    results[i].score = SumToScore(sum, d.num_points, m->min_s, m->max_s);
    results[i].pose.x = init.x + cx;
    results[i].pose.y = init.y + cy;
    results[i].pose.theta = init.theta + co;
  }
  return CSM_OK;
}

}  // namespace

extern "C" {

const char* csm_strerror(int code) {
  switch (code) {
    case CSM_OK: return "ok";
    case CSM_NO_MATCH: return "no match above min_score";
    case CSM_EINVAL: return "invalid argument";
    case CSM_EHIP: return "HIP runtime error";
    case CSM_ENOMEM: return "device out of memory";
    case CSM_ERANGE: return "input exceeds the device path's index limits";
    default: return "unknown error";
  }
}

int csm_context_create(int32_t device, csm_context** out) {
  if (!out) return CSM_EINVAL;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return CSM_EHIP;
  auto ctx = std::make_unique<csm_context>();
  ctx->device = device;
  CSM_HIP(hipSetDevice(device));
  CSM_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  CSM_HIP(hipEventCreate(&ctx->ev0));
  CSM_HIP(hipEventCreate(&ctx->ev1));
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
    ctx->num_cus = prop.multiProcessorCount;
  *out = ctx.release();
  return CSM_OK;
}

void csm_context_destroy(csm_context* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->f3_copy_stream) (void)hipStreamSynchronize(ctx->f3_copy_stream);
  if (ctx->f3_points_ready) (void)hipEventDestroy(ctx->f3_points_ready);
  if (ctx->f3_copy_stream) (void)hipStreamDestroy(ctx->f3_copy_stream);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

void* csm_context_stream(csm_context* ctx) { return ctx ? ctx->stream : nullptr; }

void csm_context_enable_timing(csm_context* ctx, int32_t enable) {
  if (ctx) ctx->timing = enable != 0;
}
void csm_context_get_timing(csm_context* ctx, csm_timing* out) {
  if (ctx && out) *out = ctx->t;
}
void csm_context_reset_timing(csm_context* ctx) {
  if (!ctx) return;
  ctx->t = csm_timing{};
  for (int l = 0; l < kMaxLevels; ++l) ctx->level_cands[l] = ctx->level_batches[l] = 0.;
}

int32_t csm_context_level_stats(csm_context* ctx, double* candidates, double* batches,
                                int32_t max_levels) {
  if (!ctx) return 0;
  const int n = std::min<int>(max_levels, kMaxLevels);
  for (int l = 0; l < n; ++l) {
    if (candidates) candidates[l] = ctx->level_cands[l];
    if (batches) batches[l] = ctx->level_batches[l];
  }
  return n;
}

int csm_fast2d_create(csm_context* ctx, const csm_map_limits* limits,
                      const uint16_t* cells, float min_cc, float max_cc,
                      const csm_fast2d_options* options, csm_fast2d** out) {
  if (!ctx || !limits || !cells || !options || !out) return CSM_EINVAL;
  if (options->branch_and_bound_depth < 1 || limits->num_x_cells < 1 ||
      limits->num_y_cells < 1 || !(limits->resolution > 0.) || !(min_cc < max_cc))
    return CSM_EINVAL;
  if (limits->num_x_cells > 8192 || limits->num_y_cells > 8192 ||
      options->branch_and_bound_depth > kMaxLevels)
    return CSM_ERANGE;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (EnsureDevice(ctx)) return CSM_EHIP;
  auto m = std::make_unique<csm_fast2d>();
  m->ctx = ctx;
  m->limits = *limits;
  m->options = *options;
  m->min_cc = min_cc;
  m->max_cc = max_cc;
  m->min_s = 1.f - max_cc;  // fast_correlative_scan_matcher_2d.cc:97-98
  m->max_s = 1.f - min_cc;
  const int nx = limits->num_x_cells, ny = limits->num_y_cells;
  int depth = options->search_depth > 0 ? options->search_depth
                                        : AutoSearchDepth(options->branch_and_bound_depth, nx, ny);
  depth = std::max(depth, options->branch_and_bound_depth);
  depth = std::min(depth, kMaxLevels);
  // Node levels that expand two levels at once (search kernel v5, hex
  // planes; SubmapDesc::hex_mask): by default the top level and the one two
  // below it (measured best on C2). CSM_SEARCH_KERNEL=4: none
  // (v4, quad planes only); =5: every even level >= 2; CSM_HEX_LEVELS="8,6"
  // lists them (experiments).
  uint32_t hex_mask = 0;
  {
    const char* kenv = std::getenv("CSM_SEARCH_KERNEL");
    const int kf = kenv ? std::atoi(kenv) : 0;
    if (kf == 5) {
      for (int l = 2; l < depth; l += 2) hex_mask |= 1u << l;
    } else if (kf != 4 && kf != 2) {
      for (int l : {depth - 1, depth - 3})
        if (l >= 2) hex_mask |= 1u << l;
    }
    if (const char* lv = std::getenv("CSM_HEX_LEVELS")) {
      hex_mask = 0;
      for (const char* c = lv; *c;) {
        const int l = std::atoi(c);
        if (l >= 2 && l < depth) hex_mask |= 1u << l;
        while (*c && *c != ',') ++c;
        if (*c == ',') ++c;
      }
    }
  }
  m->options.search_depth = depth;
  std::vector<uint8_t> qtab(32768);
  if (!QuantizationTable(min_cc, max_cc, qtab.data())) return CSM_EINVAL;

  SubmapDesc& d = m->desc;
  d.max_x = limits->max_x;
  d.max_y = limits->max_y;
  d.resolution = limits->resolution;
  d.nx = nx;
  d.ny = ny;
  d.levels = depth;
  size_t total = 0;
  std::vector<size_t> offs(depth);
  for (int l = 0; l < depth; ++l) {
    const int w = 1 << l;
    d.wide_nx[l] = nx + w - 1;
    d.wide_ny[l] = ny + w - 1;
    d.zero_index[l] = d.wide_nx[l] * d.wide_ny[l];
    offs[l] = total;
    total += (static_cast<size_t>(d.zero_index[l]) + 1 + 255) & ~size_t(255);
  }
  const size_t rowmajor = total;
  std::vector<size_t> qoffs(depth);
  ClusterShifts(d.cshift);
  size_t widen_bytes = 0;  // scratch for the widened levels the hex planes are made from
  // Plane layout (SubmapDesc::quad_es): the levels the node chain reaches
  // (virtual roots -> quad plane of the top level; a node level L in the
  // mask -> hex plane of L - 2, any other -> quad plane of L - 1). A layout
  // past the 2^31-byte buffer range falls back to quad planes only.
  auto layout = [&](uint32_t mask) {
    int kind[kMaxLevels] = {0};
    kind[depth - 1] = 4;
    for (int L = depth - 1; L >= 1;) {
      if (L >= 2 && ((mask >> L) & 1u)) {
        kind[L - 2] = 16;
        L -= 2;
      } else {
        kind[L - 1] = 4;
        L -= 1;
      }
    }
    total = rowmajor;
    widen_bytes = 0;
    for (int l = 0; l < depth; ++l) {
      const int h = 1 << l;
      const int km1 = (1 << d.cshift[l]) - 1;
      const bool hexl = kind[l] == 16;
      const int reach = hexl ? 3 * h : h, period = hexl ? 4 * h : 2 * h;
      d.quad_es[l] = kind[l];
      d.quad_bias[l] = (h - 1) + km1 + reach;
      d.quad_w[l] = d.wide_nx[l] + km1 + reach;
      d.quad_h[l] = d.wide_ny[l] + km1 + reach;
      d.quad_pws[l] = (d.quad_w[l] + period - 1) / period;
      d.quad_pph[l] = (d.quad_h[l] + period - 1) / period;
      const size_t qb = static_cast<size_t>(period) * period * d.quad_pws[l] * d.quad_pph[l] * kind[l];
      if (qb > 0x7fffff00u) return false;
      d.quad_bytes[l] = static_cast<int32_t>(qb);
      qoffs[l] = total;
      total += (qb + 255) & ~size_t(255);
      if (hexl)
        widen_bytes = std::max(widen_bytes, static_cast<size_t>(d.wide_nx[l] + km1) *
                                                (d.wide_ny[l] + km1));
    }
    return total <= 0x7fffff00u;
  };
  if (!layout(hex_mask)) {
    if (!hex_mask || !layout(0)) return CSM_ERANGE;
    hex_mask = 0;
  }
  d.hex_mask = static_cast<int32_t>(hex_mask);
  int rc;
  if ((rc = m->pyramid.Reserve(total))) return rc;
  d.pyramid_base = m->pyramid.as<uint8_t>();
  d.pyramid_bytes = static_cast<int32_t>(total);
  for (int l = 0; l < depth; ++l) {
    d.level[l] = m->pyramid.as<uint8_t>() + offs[l];
    d.quad[l] = reinterpret_cast<const uint32_t*>(m->pyramid.as<uint8_t>() + qoffs[l]);
    d.quad_off[l] = static_cast<int32_t>(qoffs[l]);
  }

  DevBuf dcells, dq;
  if ((rc = dcells.Reserve(sizeof(uint16_t) * nx * ny))) return rc;
  if ((rc = dq.Reserve(32768))) return rc;
  hipStream_t st = ctx->stream;
  CSM_HIP(hipMemcpyAsync(dcells.ptr, cells, sizeof(uint16_t) * nx * ny, hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemcpyAsync(dq.ptr, qtab.data(), 32768, hipMemcpyHostToDevice, st));
  const int n0 = nx * ny;
  CSM_HIP(LaunchPyramidLevel0(dcells.as<uint16_t>(), dq.as<uint8_t>(),
                              const_cast<uint8_t*>(d.level[0]), n0, st));
  for (int l = 1; l < depth; ++l) {
    CSM_HIP(LaunchPyramidDouble(d.level[l - 1], d.wide_nx[l - 1], d.wide_ny[l - 1],
                                const_cast<uint8_t*>(d.level[l]), d.wide_nx[l], d.wide_ny[l],
                                1 << (l - 1), st));
  }
  DevBuf dwiden;
  if (widen_bytes && (rc = dwiden.Reserve(widen_bytes))) return rc;
  for (int l = 0; l < depth; ++l) {
    const int km1 = (1 << d.cshift[l]) - 1;
    if (d.quad_es[l] == 4)
      CSM_HIP(LaunchPyramidQuad(d.level[l], d.wide_nx[l], d.wide_ny[l], l, km1,
                                const_cast<uint32_t*>(d.quad[l]), d.quad_w[l], d.quad_h[l],
                                d.quad_pws[l], d.quad_pph[l], d.quad_bytes[l] / 4, st));
    else if (d.quad_es[l] == 16)
      CSM_HIP(LaunchPyramidHex(d.level[l], d.wide_nx[l], d.wide_ny[l], l, km1, dwiden.as<uint8_t>(),
                               const_cast<uint32_t*>(d.quad[l]), d.quad_w[l], d.quad_h[l],
                               d.quad_pws[l], d.quad_pph[l], d.quad_bytes[l] / 16, st));
  }
  // Correspondence costs (Grid2D::GetCorrespondenceCost, grid_2d.cc) for the
  // CeresScanMatcher2D refinement: the value table with unknown -> max_cc.
  {
    std::vector<float> ctab(32768);
    ConversionTable(max_cc, min_cc, max_cc, ctab.data());
    DevBuf dtab;
    if ((rc = dtab.Reserve(sizeof(float) * 32768))) return rc;
    if ((rc = m->cost.Reserve(sizeof(float) * n0))) return rc;
    CSM_HIP(hipMemcpyAsync(dtab.ptr, ctab.data(), sizeof(float) * 32768, hipMemcpyHostToDevice, st));
    CSM_HIP(LaunchCellsToProbability(dcells.as<uint16_t>(), dtab.as<float>(), m->cost.as<float>(),
                                     n0, st));
    CSM_HIP(hipStreamSynchronize(st));  // dcells/dq/dtab are freed on return
  }
  *out = m.release();
  return CSM_OK;
}

void csm_fast2d_destroy(csm_fast2d* m) {
  if (!m) return;
  (void)hipSetDevice(m->ctx->device);
  delete m;
}

int csm_fast2d_read_level(const csm_fast2d* m, int32_t level, uint8_t* out,
                          int64_t capacity, int32_t* wide_nx, int32_t* wide_ny) {
  if (!m || level < 0 || level >= m->desc.levels || !wide_nx || !wide_ny) return CSM_EINVAL;
  *wide_nx = m->desc.wide_nx[level];
  *wide_ny = m->desc.wide_ny[level];
  const int64_t n = static_cast<int64_t>(*wide_nx) * *wide_ny;
  if (!out) return CSM_OK;
  if (capacity < n) return CSM_EINVAL;
  std::lock_guard<std::mutex> lock(m->ctx->mu);
  if (EnsureDevice(m->ctx)) return CSM_EHIP;
  CSM_HIP(hipMemcpyAsync(out, m->desc.level[level], n, hipMemcpyDeviceToHost, m->ctx->stream));
  CSM_HIP(hipStreamSynchronize(m->ctx->stream));
  return CSM_OK;
}

int csm_scan_set_create(csm_context* ctx, const float* points_xyz, const int64_t* offsets,
                        int32_t num_scans, csm_scan_set** out) {
  if (!ctx || !offsets || !out || num_scans < 0) return CSM_EINVAL;
  const int64_t total = offsets[num_scans];
  if (total < 0 || (total > 0 && !points_xyz)) return CSM_EINVAL;
  for (int32_t i = 0; i < num_scans; ++i)
    if (offsets[i + 1] < offsets[i]) return CSM_EINVAL;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (EnsureDevice(ctx)) return CSM_EHIP;
  auto s = std::make_unique<csm_scan_set>();
  s->ctx = ctx;
  s->offsets.assign(offsets, offsets + num_scans + 1);
  s->host_points.assign(points_xyz, points_xyz + 3 * total);
  int rc;
  if ((rc = s->points.Reserve(sizeof(float) * 3 * std::max<int64_t>(total, 1)))) return rc;
  if (total > 0)
    CSM_HIP(hipMemcpyAsync(s->points.ptr, points_xyz, sizeof(float) * 3 * total,
                           hipMemcpyHostToDevice, ctx->stream));
  CSM_HIP(hipStreamSynchronize(ctx->stream));
  *out = s.release();
  return CSM_OK;
}

void csm_scan_set_destroy(csm_scan_set* s) {
  if (!s) return;
  (void)hipSetDevice(s->ctx->device);
  delete s;
}

int csm_fast2d_match_batch(csm_context* ctx, csm_fast2d* const* submaps, int32_t num_submaps,
                           const csm_scan_set* scans, const csm_pair2d* pairs,
                           int64_t num_pairs, csm_result2d* results) {
  if (!ctx || !submaps || !scans || (num_pairs > 0 && (!pairs || !results)) || num_pairs < 0 ||
      scans->ctx != ctx)
    return CSM_EINVAL;
  if (num_pairs == 0) return CSM_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (EnsureDevice(ctx)) return CSM_EHIP;
  return RunBatch(ctx, submaps, num_submaps, const_cast<csm_scan_set*>(scans), pairs, num_pairs,
                  results);
}

static int SingleMatch(const csm_fast2d* m, const csm_pose2d* initial, int full,
                       const float* xyz, int32_t n, float min_score, float* score,
                       csm_pose2d* pose) {
  if (!m || !score || !pose || (n > 0 && !xyz) || n < 0 || (!full && !initial)) return CSM_EINVAL;
  csm_context* ctx = m->ctx;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (EnsureDevice(ctx)) return CSM_EHIP;
  csm_scan_set s;
  s.ctx = ctx;
  s.offsets = {0, n};
  s.host_points.assign(xyz, xyz + 3 * static_cast<size_t>(n));
  int rc;
  if ((rc = s.points.Reserve(sizeof(float) * 3 * std::max(n, 1)))) return rc;
  if (n > 0)
    CSM_HIP(hipMemcpyAsync(s.points.ptr, xyz, sizeof(float) * 3 * n, hipMemcpyHostToDevice,
                           ctx->stream));
  csm_pair2d p{};
  p.submap = 0;
  p.scan = 0;
  p.full_submap = full;
  p.min_score = min_score;
  if (!full) p.initial = *initial;
  csm_fast2d* const handles[1] = {const_cast<csm_fast2d*>(m)};
  csm_result2d r{};
  rc = RunBatch(ctx, handles, 1, &s, &p, 1, &r);
  if (rc < 0) return rc;
  if (r.status == CSM_OK) {
    *score = r.score;
    *pose = r.pose;
  }
  return r.status;
}

int csm_fast2d_match(const csm_fast2d* m, const csm_pose2d* initial, const float* points_xyz,
                     int32_t n, float min_score, float* score, csm_pose2d* pose) {
  return SingleMatch(m, initial, 0, points_xyz, n, min_score, score, pose);
}

int csm_fast2d_match_full_submap(const csm_fast2d* m, const float* points_xyz, int32_t n,
                                 float min_score, float* score, csm_pose2d* pose) {
  return SingleMatch(m, nullptr, 1, points_xyz, n, min_score, score, pose);
}

}  // extern "C"


