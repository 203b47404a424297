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
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <thread>
#include <array>
#include <tuple>
#include <vector>

#include "../../include/csm_amd.h"
#include "csm_device.h"
#include "csm_internal.h"
#include "csm_launch.h"
#include "parallel_sort.h"
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

// Scan cluster size per child level (SubmapDesc::cshift): k = 1, 1, 4, 4, 4,
// 8, ... cells per side (log2), first chosen by tools/frontier_sim.py
// (cluster) on the C2 world (0.39x the lookups of exact per-level bounds),
// then by GPU A/B with kernel v5: level 2 at k = 4 (profiles/r3t), level 1 on
// the raw scan so no k = 2 list is built (profiles/r3w). Level 0 is always
// exact (k = 1) and k <= 2^level. CSM_CLUSTER="s0,s1,..." overrides.
void ClusterShifts(int32_t* out) {
  static const int kDefault[kMaxLevels] = {0, 0, 2, 2, 2, 3, 3, 3, 3, 3, 3, 3};
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

}  // namespace

namespace csm {

namespace {
std::mutex& PoolRegistryMutex() {
  static std::mutex m;
  return m;
}
std::vector<BufPool*>& PoolRegistry() {
  static std::vector<BufPool*> r;
  return r;
}
}  // namespace

BufPool::BufPool() {
  std::lock_guard<std::mutex> g(PoolRegistryMutex());
  PoolRegistry().push_back(this);
}

BufPool::~BufPool() {
  {
    std::lock_guard<std::mutex> g(PoolRegistryMutex());
    auto& r = PoolRegistry();
    r.erase(std::remove(r.begin(), r.end(), this), r.end());
  }
  Release();
}

void BufPool::Release() {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& b : bufs_) (void)hipFree(b.first);
  bufs_.clear();
  held_ = 0;
}

int BufPool::Take(size_t n, DevBuf* out) {
  {
    std::lock_guard<std::mutex> g(mu_);
    int best = -1;
    for (int i = 0; i < static_cast<int>(bufs_.size()); ++i) {
      const size_t b = bufs_[i].second;
      if (b >= n && b <= 2 * n + 4096 && (best < 0 || b < bufs_[best].second)) best = i;
    }
    if (best >= 0) {
      out->ptr = bufs_[best].first;
      out->bytes = bufs_[best].second;
      held_ -= bufs_[best].second;
      bufs_.erase(bufs_.begin() + best);
      return CSM_OK;
    }
  }
  return out->Reserve(n);  // releases every pool and retries if the device is full
}

void BufPool::Give(DevBuf* b) {
  constexpr size_t kMaxPooled = 8192;
  if (!b->ptr) return;
  std::lock_guard<std::mutex> g(mu_);
  bufs_.emplace_back(b->ptr, b->bytes);
  held_ += b->bytes;
  b->ptr = nullptr;
  b->bytes = 0;
  size_t drop = 0;
  while (drop < bufs_.size() && (bufs_.size() - drop > kMaxPooled || held_ > cap_bytes_)) {
    held_ -= bufs_[drop].second;
    (void)hipFree(bufs_[drop].first);
    ++drop;
  }
  bufs_.erase(bufs_.begin(), bufs_.begin() + static_cast<std::ptrdiff_t>(drop));
}

void ReleaseIdlePools() {
  std::lock_guard<std::mutex> g(PoolRegistryMutex());
  for (BufPool* p : PoolRegistry()) p->Release();
}

csm_context* AcquireCallContext(csm_context* owner) {
  {
    std::lock_guard<std::mutex> g(owner->call_mu);
    if (!owner->call_free.empty()) {
      csm_context* c = owner->call_free.back();
      owner->call_free.pop_back();
      c->timing = owner->timing.load();
      return c;
    }
  }
  csm_context* c = nullptr;
  if (csm_context_create(owner->device, &c) != CSM_OK) return nullptr;
  c->call_owner = owner;
  c->timing = owner->timing.load();
  std::lock_guard<std::mutex> g(owner->call_mu);
  owner->call_all.push_back(c);
  return c;
}

void ReleaseCallContext(csm_context* owner, csm_context* c) {
  if (!c) return;
  std::lock_guard<std::mutex> g(owner->call_mu);
  AddTiming(&owner->call_t, c->t);
  c->t = csm_timing{};
  owner->call_free.push_back(c);
}

}  // namespace csm

namespace {

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

struct SearchPlan {
  bool use_v2 = true, hex = false, fifo = true;
  int rc = 2, max_npad = 64;
};

// One search launch over `pdesc` (the submap descriptors and the rotation
// table are on the device already). init_best: per-pair starting best keys
// (tie enumeration: the pair's maximum, so only nodes reaching it expand and
// every leaf at it is recorded, PairDesc::collect_sum); null = 0.
int LaunchSearch(csm_context* ctx, csm_scan_set* scans, const std::vector<PairDesc>& pdesc,
                 const std::vector<uint64_t>* init_best, const SearchPlan& plan, bool timed,
                 std::vector<uint64_t>* keys, std::vector<uint64_t>* keys_hi,
                 std::vector<int32_t>* stat, unsigned long long* stats_host,
                 std::vector<uint2>* ties = nullptr, std::vector<int32_t>* tie_counts = nullptr) {
  const int np = static_cast<int>(pdesc.size());
  const int rc = plan.rc;
  // Per-XCD queues: submap s -> queue s % 8 so a submap's pyramid stays in
  // one XCD's L2; pairs within a queue in submap order. A batch of fewer
  // than 8 submaps (the C3 chunks hold 4) spreads each submap's pairs over
  // 8 / S queues, so every XCD starts on a submap of its own instead of the
  // empty queues' workgroups all stealing from the first one: C3 chunk
  // launch 591 -> 570 ms (profiles/r4o/; CSM_QUEUE_SPREAD=0 for the A/B).
  static const bool spread_on = [] {
    const char* e = std::getenv("CSM_QUEUE_SPREAD");
    return !(e && std::atoi(e) == 0);
  }();
  int nsub = 0;
  for (int i = 0; i < np; ++i) nsub = std::max(nsub, pdesc[i].submap + 1);
  const int reps = spread_on && nsub > 0 && nsub < kNumXcd ? kNumXcd / nsub : 1;
  std::vector<int32_t> seen(reps > 1 ? nsub : 0, 0);
  std::vector<std::vector<int32_t>> q(kNumXcd);
  for (int i = 0; i < np; ++i) {
    const int sm = pdesc[i].submap;
    const int qi = reps > 1 ? sm + nsub * (seen[sm]++ % reps) : sm % kNumXcd;
    q[qi].push_back(i);
  }
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

  // Block table (v2 kernel): for every 64 chunks of a queue, the first
  // pair_order entry.
  std::vector<int32_t> blocks;
  WorkQueues2 wq2{};
  if (plan.use_v2) {
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
  }

  // One device arena per launch (csm_context::arena): the inputs, uploaded
  // with one copy from pinned staging, then the outputs, zeroed with one
  // memset and read back with one copy into pinned memory:
  //   pair_desc | pair_order | chunk_prefix | blocks || best | best_hi |
  //   status | tie_count | counters | stats
  // (init_best, when given, is uploaded into `best` with the inputs.)
  auto align = [](size_t v) { return (v + 255) & ~size_t{255}; };
  size_t at = 0;
  auto region = [&](size_t bytes) {
    const size_t o = at;
    at = align(at + std::max<size_t>(bytes, 1));
    return o;
  };
  const size_t o_pd = region(sizeof(PairDesc) * np), o_order = region(sizeof(int32_t) * order.size()),
               o_prefix = region(sizeof(int64_t) * prefix.size()),
               o_blocks = region(sizeof(int32_t) * blocks.size());
  const size_t o_best = region(sizeof(uint64_t) * np), o_hi = region(sizeof(uint64_t) * np),
               o_status = region(sizeof(int32_t) * np), o_tcount = region(sizeof(int32_t) * np),
               o_counters = region(sizeof(unsigned long long) * kNumXcd);
  const size_t o_stats = region(sizeof(unsigned long long) * kStatsWords);
  const size_t arena_bytes = at;
  const size_t in_end = init_best ? o_hi : o_best;  // uploaded bytes
  const size_t zero_begin = in_end;
  int rcode;
  if ((rcode = ctx->arena.Reserve(arena_bytes))) return rcode;
  if ((rcode = ctx->arena_in.Reserve(in_end))) return rcode;
  if ((rcode = ctx->arena_out.Reserve(arena_bytes - o_best))) return rcode;
  if (ties && (rcode = ctx->ties.Reserve(sizeof(uint2) * kTieCap * static_cast<size_t>(np))))
    return rcode;
  char* hin = ctx->arena_in.as<char>();
  std::memcpy(hin + o_pd, pdesc.data(), sizeof(PairDesc) * np);
  std::memcpy(hin + o_order, order.data(), sizeof(int32_t) * order.size());
  std::memcpy(hin + o_prefix, prefix.data(), sizeof(int64_t) * prefix.size());
  if (!blocks.empty()) std::memcpy(hin + o_blocks, blocks.data(), sizeof(int32_t) * blocks.size());
  if (init_best) std::memcpy(hin + o_best, init_best->data(), sizeof(uint64_t) * np);
  char* dev = ctx->arena.as<char>();
  hipStream_t st = ctx->stream;
  CSM_HIP(hipMemcpyAsync(dev, hin, in_end, hipMemcpyHostToDevice, st));
  CSM_HIP(hipMemsetAsync(dev + zero_begin, 0, arena_bytes - zero_begin, st));
  ctx->pair_desc_dev = dev + o_pd;
  PairDesc* d_pairs = reinterpret_cast<PairDesc*>(dev + o_pd);
  uint64_t* d_best = reinterpret_cast<uint64_t*>(dev + o_best);
  uint64_t* d_hi = reinterpret_cast<uint64_t*>(dev + o_hi);
  int32_t* d_status = reinterpret_cast<int32_t*>(dev + o_status);
  int32_t* d_tcount = reinterpret_cast<int32_t*>(dev + o_tcount);
  unsigned long long* d_counters = reinterpret_cast<unsigned long long*>(dev + o_counters);
  unsigned long long* d_stats = reinterpret_cast<unsigned long long*>(dev + o_stats);
  wq.pair_order = reinterpret_cast<int32_t*>(dev + o_order);
  wq.chunk_prefix = reinterpret_cast<int64_t*>(dev + o_prefix);

  // ---- launch: persistent workgroups ----------------------------------------
  const int64_t total_chunks = running;
  const int max_npad = plan.max_npad;
  if (timed) CSM_HIP(hipEventRecord(ctx->ev0, st));
  if (plan.use_v2) {
    wq2.pair_order = wq.pair_order;
    wq2.chunk_prefix = wq.chunk_prefix;
    wq2.block_first = reinterpret_cast<int32_t*>(dev + o_blocks);
    // Per rotation: npad raw cells and capc cluster-list entries. capc =
    // 3/4 npad holds the three cluster lists of a typical scan (0.55 npad on
    // C2); a list that does not fit falls back to a finer one in the kernel.
    int capc = (3 * max_npad / 4 + 63) & ~63;
    if (const char* ce = std::getenv("CSM_CAPC_PCT"))  // A/B: cluster-list room, % of npad
      capc = std::max(64, (std::atoi(ce) * max_npad / 100 + 63) & ~63);
    const int lds_cap = 96 * 1024;
    // Per rotation: npad raw cells (4 B) + capc cluster entries (4 B cell + 1 B count).
    auto dyn_bytes = [&](int cap) { return static_cast<size_t>(rc) * (max_npad * 4 + cap * 5); };
    while (capc > 0 && dyn_bytes(capc) > lds_cap) capc -= 64;
    const size_t dyn_lds = (dyn_bytes(capc) + 15) & ~size_t{15};
    // Workgroups per CU: what registers and LDS allow (the runtime's
    // occupancy query). CSM_WG_PER_CU caps it (A/B runs).
    int per_cu = std::max(1, std::min(8, Fast2dSearchV2BlocksPerCu(plan.hex, plan.fifo, dyn_lds)));
    if (const char* w = std::getenv("CSM_WG_PER_CU")) per_cu = std::max(1, std::min(per_cu, std::atoi(w)));
    if (std::getenv("CSM_PROFILE2D") && !init_best)
      std::fprintf(stderr, "fast2d launch: %s %s, %d rotations per item, %zu B dynamic LDS (capc %d), %d workgroups per CU\n",
                   plan.hex ? "v5" : "v4", plan.fifo ? "fifo" : "lifo", rc, dyn_lds, capc, per_cu);
    // Concurrent single calls (call contexts, csm_internal.h) each take a
    // share of the chip, so their persistent grids tile it instead of
    // queueing behind one another (at least one workgroup per CU each).
    const int64_t full = static_cast<int64_t>(ctx->num_cus) * per_cu;
    const int64_t share = std::max<int64_t>(ctx->num_cus, full / std::max(1, ctx->grid_share));
    const int grid = static_cast<int>(std::min<int64_t>(share, std::max<int64_t>(total_chunks, 1)));
    // DFS stack spill: kSpill2 entries per persistent workgroup.
    if ((rcode = ctx->spill.Reserve(sizeof(uint2) * kSpill2 * static_cast<size_t>(grid))))
      return rcode;
    CSM_HIP(LaunchFast2dSearchV2(grid, dyn_lds, st, ctx->submap_desc.as<SubmapDesc>(), d_pairs,
                                 scans->points.as<float>(), scans->rot_dev.as<float2>(), wq2,
                                 d_counters, d_best, d_status, d_stats, ctx->spill.as<uint2>(),
                                 max_npad, capc, plan.hex, plan.fifo, d_hi,
                                 ties ? ctx->ties.as<uint2>() : nullptr, d_tcount, ties != nullptr));
  } else {
    const size_t dyn_lds = static_cast<size_t>(rc) * max_npad * sizeof(uint32_t);
    const int grid = static_cast<int>(std::min<int64_t>(static_cast<int64_t>(ctx->num_cus) * 4,
                                                        std::max<int64_t>(total_chunks, 1)));
    CSM_HIP(LaunchFast2dSearch(grid, dyn_lds, st, ctx->submap_desc.as<SubmapDesc>(), d_pairs,
                               scans->points.as<float>(), scans->rot_dev.as<float2>(), wq,
                               d_counters, d_best, d_status, d_stats));
  }
  if (timed) CSM_HIP(hipEventRecord(ctx->ev1, st));
  char* hout = ctx->arena_out.as<char>();
  CSM_HIP(hipMemcpyAsync(hout, dev + o_best, arena_bytes - o_best, hipMemcpyDeviceToHost, st));
  if (ties) {
    ties->resize(static_cast<size_t>(kTieCap) * np);
    CSM_HIP(hipMemcpyAsync(ties->data(), ctx->ties.ptr, sizeof(uint2) * ties->size(),
                           hipMemcpyDeviceToHost, st));
  }
  CSM_HIP(hipStreamSynchronize(st));
  auto out = [&](size_t o) { return hout + (o - o_best); };
  keys->assign(reinterpret_cast<uint64_t*>(out(o_best)), reinterpret_cast<uint64_t*>(out(o_best)) + np);
  keys_hi->assign(reinterpret_cast<uint64_t*>(out(o_hi)), reinterpret_cast<uint64_t*>(out(o_hi)) + np);
  stat->assign(reinterpret_cast<int32_t*>(out(o_status)), reinterpret_cast<int32_t*>(out(o_status)) + np);
  std::memcpy(stats_host, out(o_stats), sizeof(unsigned long long) * kStatsWords);
  if (ties)
    tie_counts->assign(reinterpret_cast<int32_t*>(out(o_tcount)),
                       reinterpret_cast<int32_t*>(out(o_tcount)) + np);
  return CSM_OK;
}

// ShrinkToFit bounds (correlative_scan_matcher_2d.cc:73-91) of rotation r of
// a pair, from the scan discretized on the host with the device's arithmetic
// (two z rotations in Eigen's order, the float translation add, GetCellIndex
// in double, map_limits.h:69-75).
void RotationBounds(const csm_scan_set* scans, const PairDesc& d, const SubmapDesc& sm,
                    const ZRot& rot, int b[4]) {
  int mnx = 0x7fffffff, mxx = -0x7fffffff, mny = 0x7fffffff, mxy = -0x7fffffff;
  const ZRot pre{d.pre_w, d.pre_s};
  const float* p = scans->host_points.data() + 3 * d.point_offset;
  for (int i = 0; i < d.num_points; ++i) {
    float x, y;
    RotateZ(pre, p[3 * i], p[3 * i + 1], &x, &y);
    RotateZ(rot, x, y, &x, &y);
    const float px = d.tx + x, py = d.ty + y;
    const int ix = static_cast<int>(std::round((sm.max_y - static_cast<double>(py)) / sm.resolution - 0.5));
    const int iy = static_cast<int>(std::round((sm.max_x - static_cast<double>(px)) / sm.resolution - 0.5));
    mnx = std::min(mnx, ix); mxx = std::max(mxx, ix);
    mny = std::min(mny, iy); mxy = std::max(mxy, iy);
  }
  b[0] = std::max(-d.num_linear, std::min(0, -mxx));
  b[1] = std::min(d.num_linear, std::max(0, sm.nx - 1 - mnx));
  b[2] = std::max(-d.num_linear, std::min(0, -mxy));
  b[3] = std::min(d.num_linear, std::max(0, sm.ny - 1 - mny));
}

// Exactly tied maxima. The device keeps the smallest (rotation, x, y) leaf;
// the reference keeps the FIRST maximal leaf its depth-first search visits
// (std::max keeps the incumbent on equal scores and later subtrees whose
// bound does not exceed it are cut, fast_correlative_scan_matcher_2d.cc:
// 344-376). It visits a node's children (<= 4, std::sort = insertion sort:
// stable) by descending score, equal scores in generation order (x, then y;
// :353-366), and the lowest-resolution candidates in the order std::sort
// (introsort, not stable) leaves their generation order (scan, x, y;
// :276-312) in. So among tied leaves the reference's pick is the one whose
// chain of ancestors, top level first, comes first in those orders. For a
// pair whose two witness keys show a tie: (1) a second search with the
// maximum as its starting best records every leaf at it; (2) the ancestors'
// exact bounds at the reference's depth are scored on the device
// (fast2d_score_queries); (3) when two tied leaves descend from different
// lowest-resolution candidates of equal score, the pair's whole
// lowest-resolution list is scored and sorted with the same std::sort and
// comparison, which reproduces the reference's permutation. No oracle and no
// CPU scoring is involved.
int ResolveTies(csm_context* ctx, csm_fast2d* const* submaps, csm_scan_set* scans,
                const std::vector<PairDesc>& pdesc, const std::vector<float2>& rot_host,
                const SearchPlan& plan, std::vector<int32_t>* stat,
                const std::vector<uint64_t>& keys_hi, std::vector<uint64_t>* keys,
                std::vector<int8_t>* tie_code) {
  std::vector<int> tied;
  for (int k = 0; k < static_cast<int>(pdesc.size()); ++k) {
    const uint64_t key = (*keys)[k];
    if (((*stat)[k] & kStatusRange) || key == 0) continue;
    const int64_t sum = static_cast<int64_t>(key >> kSumShift);
    if (sum <= pdesc[k].max_rejected_sum) continue;
    if ((keys_hi[k] >> kSumShift) == (key >> kSumShift) && keys_hi[k] != HighLeafKey(key))
      tied.push_back(k);
  }
  if (tied.empty()) return CSM_OK;
  ctx->t.tied_pairs += static_cast<int64_t>(tied.size());
  const bool prof = std::getenv("CSM_PROFILE2D") != nullptr;
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  const auto tp0 = now();
  // (1) Every leaf at the maximum.
  std::vector<PairDesc> pd2;
  std::vector<uint64_t> init;
  for (int k : tied) {
    PairDesc d = pdesc[k];
    d.collect = 1;
    d.collect_sum = static_cast<int32_t>((*keys)[k] >> kSumShift);
    pd2.push_back(d);
    init.push_back(static_cast<uint64_t>(d.collect_sum) << kSumShift);
  }
  std::vector<uint64_t> k2, kh2;
  std::vector<int32_t> st2, counts;
  std::vector<uint2> ties;
  unsigned long long stats2[kStatsWords] = {0};
  int rc;
  if ((rc = LaunchSearch(ctx, scans, pd2, &init, plan, false, &k2, &kh2, &st2, stats2, &ties,
                         &counts)))
    return rc;
  auto zrot = [&](const PairDesc& d, int r) {
    const float2 z = rot_host[d.rot_offset + r];
    return ZRot{z.x, z.y};
  };
  // (2) Ancestors at the reference's depth D: level d node of a leaf is
  // (b0 + ((x - b0) >> d << d), b2 + ((y - b2) >> d << d)).
  struct Tie {
    int k, t, depth, leaves_first, leaves_count;
  };
  std::vector<Tie> work;
  std::vector<int3> leaves;          // (rot, x, y)
  std::vector<ScoreJob> jobs;
  std::vector<int4> queries;
  std::vector<int> leaf_query;       // per leaf: first of its D - 1 ancestor queries
  std::vector<int> walk;             // tied pairs (pd2 index) whose leaves overflow the record
  for (size_t t = 0; t < tied.size(); ++t) {
    const int k = tied[t];
    const int cnt = counts[t];
    if ((st2[t] & kStatusRange) || cnt > kTieCap || cnt < 2) {
      // More tied leaves than the collect pass records (or its frontier
      // overflowed): walk the reference's order on the device instead (4).
      ctx->t.ties_walked += 1;
      (*tie_code)[k] = CSM_TIE_WALK;
      walk.push_back(static_cast<int>(t));
      continue;
    }
    const PairDesc& d = pdesc[k];
    const csm_fast2d* m = submaps[d.submap];
    Tie w{k, static_cast<int>(t), m->options.branch_and_bound_depth,
          static_cast<int>(leaves.size()), cnt};
    std::map<int, std::vector<int>> by_rot;
    for (int i = 0; i < cnt; ++i) {
      const uint2 e = ties[static_cast<size_t>(t) * kTieCap + i];
      const int r = static_cast<int>(e.x);
      const int x = static_cast<int16_t>(e.y & 0xffff), y = static_cast<int>(e.y) >> 16;
      leaves.push_back(make_int3(r, x, y));
      by_rot[r].push_back(w.leaves_first + i);
    }
    leaf_query.resize(leaves.size(), -1);
    const int T = w.depth - 1;
    for (auto& [r, idx] : by_rot) {
      int b[4];
      RotationBounds(scans, d, m->desc, zrot(d, r), b);
      if (T < 1) continue;
      ScoreJob job{static_cast<int32_t>(t), r, static_cast<int32_t>(queries.size()), 0};
      for (int li : idx) {
        leaf_query[li] = static_cast<int>(queries.size());
        for (int lv = 1; lv <= T; ++lv) {
          const int ax = b[0] + (((leaves[li].y - b[0]) >> lv) << lv);
          const int ay = b[2] + (((leaves[li].z - b[2]) >> lv) << lv);
          queries.push_back(make_int4(lv, ax, ay, 0));
        }
      }
      job.count = static_cast<int32_t>(queries.size()) - job.first;
      jobs.push_back(job);
    }
    work.push_back(w);
  }
  auto score = [&](const std::vector<ScoreJob>& js, const std::vector<int4>& qs,
                   std::vector<int32_t>* sums) -> int {
    sums->assign(qs.size(), 0);
    if (js.empty()) return CSM_OK;
    int r2;
    if ((r2 = ctx->sq_jobs.Reserve(sizeof(ScoreJob) * js.size()))) return r2;
    if ((r2 = ctx->sq_queries.Reserve(sizeof(int4) * qs.size()))) return r2;
    if ((r2 = ctx->sq_sums.Reserve(sizeof(int32_t) * qs.size()))) return r2;
    hipStream_t st = ctx->stream;
    CSM_HIP(hipMemcpyAsync(ctx->sq_jobs.ptr, js.data(), sizeof(ScoreJob) * js.size(),
                           hipMemcpyHostToDevice, st));
    CSM_HIP(hipMemcpyAsync(ctx->sq_queries.ptr, qs.data(), sizeof(int4) * qs.size(),
                           hipMemcpyHostToDevice, st));
    CSM_HIP(LaunchFast2dScoreQueries(static_cast<int>(js.size()), plan.max_npad, st,
                                     ctx->submap_desc.as<SubmapDesc>(), static_cast<const PairDesc*>(ctx->pair_desc_dev),
                                     scans->points.as<float>(), scans->rot_dev.as<float2>(),
                                     ctx->sq_jobs.as<ScoreJob>(), ctx->sq_queries.as<int4>(),
                                     ctx->sq_sums.as<int32_t>()));
    CSM_HIP(hipMemcpyAsync(sums->data(), ctx->sq_sums.ptr, sizeof(int32_t) * qs.size(),
                           hipMemcpyDeviceToHost, st));
    CSM_HIP(hipStreamSynchronize(st));
    return CSM_OK;
  };
  const auto tp1 = now();
  // The jobs index pd2 (ctx->pair_desc_dev holds it after the second search).
  std::vector<int32_t> sums;
  if ((rc = score(jobs, queries, &sums))) return rc;
  // Per tie: the leaves that can come first. The reference visits the
  // lowest-resolution candidates by descending score, so only leaves under a
  // top-level ancestor of the highest score compete; the top-level order is
  // needed only when two distinct such ancestors share that score.
  struct Cand {
    std::vector<int> live;  // leaf indices under a highest-score top ancestor
    bool need_perm = false;
    std::vector<std::array<int, 4>> rb;  // per rotation bounds (need_perm)
    std::vector<int64_t> rot_first;      // per rotation first lattice index
    std::vector<int64_t> pos;            // lattice index -> sorted position
  };
  std::vector<Cand> cand(work.size());
  auto anc_of = [&](const Tie& w, int li, int lv) {
    const PairDesc& d = pdesc[w.k];
    const csm_fast2d* m = submaps[d.submap];
    const int4 q = queries[leaf_query[li] + lv - 1];
    return std::make_tuple(q.y, q.z,
                           SumToScore(sums[leaf_query[li] + lv - 1], d.num_points, m->min_s, m->max_s));
  };
  for (size_t wi = 0; wi < work.size(); ++wi) {
    const Tie& w = work[wi];
    Cand& c = cand[wi];
    const int T = w.depth - 1;
    if (T == 0) {  // the top-level list is the leaves themselves
      for (int i = 0; i < w.leaves_count; ++i) c.live.push_back(w.leaves_first + i);
      c.need_perm = true;
      continue;
    }
    float top = -std::numeric_limits<float>::infinity();
    for (int i = 0; i < w.leaves_count; ++i) top = std::max(top, std::get<2>(anc_of(w, w.leaves_first + i, T)));
    std::set<std::tuple<int, int, int>> nodes;
    for (int i = 0; i < w.leaves_count; ++i) {
      const int li = w.leaves_first + i;
      const auto [x, y, sc] = anc_of(w, li, T);
      if (sc != top) continue;
      c.live.push_back(li);
      nodes.insert({leaves[li].x, x, y});
    }
    c.need_perm = nodes.size() > 1;
  }
  const auto tp2 = now();
  auto tp3 = tp2, tp4 = tp2;
  // (3) The whole lowest-resolution list of every pair that needs the
  // top-level permutation: bounds of all its rotations on the device, every
  // lattice node scored in one launch, each list sorted on its own thread.
  std::vector<int> perm;
  for (size_t wi = 0; wi < work.size(); ++wi) {
    (*tie_code)[work[wi].k] = cand[wi].need_perm ? CSM_TIE_TOPLIST : CSM_TIE_ANCESTORS;
    if (cand[wi].need_perm) perm.push_back(static_cast<int>(wi));
  }
  ctx->t.ties_toplist += static_cast<int64_t>(perm.size());
  // The whole lowest-resolution list of tied pairs `ts` (pd2 indices) in the
  // reference's order: ShrinkToFit bounds of every rotation on the device,
  // every lattice node of the reference's top level scored in one launch
  // (GenerateLowestResolutionCandidates, :276-312), each list sorted on its
  // own threads.
  struct TopList {
    std::vector<std::array<int, 4>> rb;  // per rotation bounds
    std::vector<int64_t> rot_first;      // per rotation first lattice index
    std::vector<int32_t> sums;           // lattice index -> sum
    std::vector<int32_t> order;          // sorted position -> lattice index
  };
  auto top_lists = [&](const std::vector<int>& ts, std::vector<TopList>* out) -> int {
    out->assign(ts.size(), TopList{});
    if (ts.empty()) return CSM_OK;
    std::vector<int2> bjobs;
    for (int t : ts)
      for (int r = 0; r < pd2[t].num_scans; ++r) bjobs.push_back(make_int2(t, r));
    int r2;
    if ((r2 = ctx->sq_jobs.Reserve(sizeof(int2) * bjobs.size()))) return r2;
    if ((r2 = ctx->sq_sums.Reserve(sizeof(int4) * bjobs.size()))) return r2;
    hipStream_t st = ctx->stream;
    std::vector<int4> bounds(bjobs.size());
    CSM_HIP(hipMemcpyAsync(ctx->sq_jobs.ptr, bjobs.data(), sizeof(int2) * bjobs.size(),
                           hipMemcpyHostToDevice, st));
    CSM_HIP(LaunchFast2dRotationBounds(static_cast<int>(bjobs.size()), st, ctx->submap_desc.as<SubmapDesc>(),
                                       static_cast<const PairDesc*>(ctx->pair_desc_dev), scans->points.as<float>(),
                                       scans->rot_dev.as<float2>(), ctx->sq_jobs.as<int2>(),
                                       ctx->sq_sums.as<int4>()));
    CSM_HIP(hipMemcpyAsync(bounds.data(), ctx->sq_sums.ptr, sizeof(int4) * bjobs.size(),
                           hipMemcpyDeviceToHost, st));
    CSM_HIP(hipStreamSynchronize(st));
    std::vector<ScoreJob> tj;
    std::vector<int4> tq;
    std::vector<int64_t> base(ts.size());
    size_t bi = 0;
    for (size_t pi = 0; pi < ts.size(); ++pi) {
      const PairDesc& d = pd2[ts[pi]];
      TopList& c = (*out)[pi];
      const int n = d.num_scans;
      const int T = submaps[d.submap]->options.branch_and_bound_depth - 1, step = 1 << T;
      base[pi] = static_cast<int64_t>(tq.size());
      c.rb.resize(n);
      c.rot_first.assign(n + 1, 0);
      for (int r = 0; r < n; ++r, ++bi) {
        const int4 b = bounds[bi];
        c.rb[r] = {b.x, b.y, b.z, b.w};
        ScoreJob job{ts[pi], r, static_cast<int32_t>(tq.size()), 0};
        for (int x = b.x; x <= b.y; x += step)
          for (int y = b.z; y <= b.w; y += step) tq.push_back(make_int4(T, x, y, 0));
        job.count = static_cast<int32_t>(tq.size()) - job.first;
        c.rot_first[r + 1] = static_cast<int64_t>(tq.size()) - base[pi];
        if (job.count) tj.push_back(job);
      }
    }
    tp3 = now();
    std::vector<int32_t> sc;
    if ((r2 = score(tj, tq, &sc))) return r2;
    tp4 = now();
    // ScoreCandidates: score = ToScore(sum / n), then
    // std::sort(greater<Candidate2D>) — the same algorithm and the same
    // comparisons give the same permutation for any element type; IntroSort
    // (parallel_sort.h) is that algorithm with independent partitions on
    // threads. Up to 8 lists at once, 8 threads between them.
    const size_t nthreads = std::min<size_t>(ts.size(), 8);
    const int sort_threads = static_cast<int>(8 / std::max<size_t>(nthreads, 1));
    auto sort_one = [&](size_t pi) {
      TopList& c = (*out)[pi];
      const PairDesc& d = pd2[ts[pi]];
      const csm_fast2d* m = submaps[d.submap];
      const int64_t n = c.rot_first.back();
      c.sums.assign(sc.begin() + base[pi], sc.begin() + base[pi] + n);
      // 8-byte elements (the comparisons, and so the permutation, are the
      // same whatever the element carries).
      std::vector<std::pair<float, int32_t>> lst(n);
      ParallelRanges(n, sort_threads, [&](std::ptrdiff_t lo, std::ptrdiff_t hi) {
        for (std::ptrdiff_t i = lo; i < hi; ++i)
          lst[i] = {SumToScore(c.sums[i], d.num_points, m->min_s, m->max_s), static_cast<int32_t>(i)};
      });
      IntroSort(lst.data(), lst.data() + n,
                [](const std::pair<float, int32_t>& a, const std::pair<float, int32_t>& b) {
                  return a.first > b.first;
                },
                sort_threads);
      c.order.resize(n);
      ParallelRanges(n, sort_threads, [&](std::ptrdiff_t lo, std::ptrdiff_t hi) {
        for (std::ptrdiff_t i = lo; i < hi; ++i) c.order[i] = lst[i].second;
      });
    };
    if (nthreads <= 1) {
      for (size_t pi = 0; pi < ts.size(); ++pi) sort_one(pi);
    } else {
      std::vector<std::thread> pool;
      std::atomic<size_t> next{0};
      for (size_t i = 0; i < nthreads; ++i)
        pool.emplace_back([&] {
          for (size_t pi; (pi = next.fetch_add(1)) < ts.size();) sort_one(pi);
        });
      for (auto& th : pool) th.join();
    }
    return CSM_OK;
  };
  if (!perm.empty()) {
    std::vector<int> ts;
    for (int wi : perm) ts.push_back(work[wi].t);
    std::vector<TopList> tl;
    if ((rc = top_lists(ts, &tl))) return rc;
    for (size_t pi = 0; pi < perm.size(); ++pi) {
      Cand& c = cand[perm[pi]];
      c.rb = std::move(tl[pi].rb);
      c.rot_first = std::move(tl[pi].rot_first);
      const std::vector<int32_t>& order = tl[pi].order;
      c.pos.resize(order.size());
      ParallelRanges(static_cast<std::ptrdiff_t>(order.size()), 8,
                     [&](std::ptrdiff_t lo, std::ptrdiff_t hi) {
                       for (std::ptrdiff_t i = lo; i < hi; ++i) c.pos[order[i]] = i;
                     });
    }
  }
  // (4) Pairs whose tied leaves overflow the record: the device walks the
  // reference's visiting order (fast2d_walk) from the sorted top list, of
  // which only the entries whose sum reaches the maximum can lead to it.
  if (!walk.empty()) {
    std::vector<TopList> tl;
    if ((rc = top_lists(walk, &tl))) return rc;
    std::vector<WalkJob2> wj;
    std::vector<int4> wtop, wb;
    for (size_t wi = 0; wi < walk.size(); ++wi) {
      const int t = walk[wi];
      const PairDesc& d = pd2[t];
      const csm_fast2d* m = submaps[d.submap];
      const TopList& c = tl[wi];
      const int T = m->options.branch_and_bound_depth - 1, step = 1 << T;
      WalkJob2 j{t, d.collect_sum, T, static_cast<int32_t>(wtop.size()), 0,
                 static_cast<int32_t>(wb.size()), m->min_s, m->max_s};
      for (const auto& b : c.rb) wb.push_back(make_int4(b[0], b[1], b[2], b[3]));
      for (const int32_t li : c.order) {
        if (c.sums[li] < d.collect_sum) continue;
        const int r = static_cast<int>(std::upper_bound(c.rot_first.begin(), c.rot_first.end(), li) -
                                       c.rot_first.begin()) - 1;
        const int ny = (c.rb[r][3] - c.rb[r][2] + step) / step;
        const int64_t loc = li - c.rot_first[r];
        wtop.push_back(make_int4(r, c.rb[r][0] + static_cast<int>(loc / ny) * step,
                                 c.rb[r][2] + static_cast<int>(loc % ny) * step, c.sums[li]));
      }
      j.top_count = static_cast<int32_t>(wtop.size()) - j.top_first;
      wj.push_back(j);
    }
    // One buffer: jobs | top entries | bounds | results.
    const size_t o_top = (sizeof(WalkJob2) * wj.size() + 15) & ~size_t{15};
    const size_t o_b = o_top + sizeof(int4) * std::max<size_t>(wtop.size(), 1);
    const size_t o_out = o_b + sizeof(int4) * wb.size();
    const size_t bytes = o_out + sizeof(int4) * wj.size();
    if ((rc = ctx->walk_buf.Reserve(bytes))) return rc;
    char* dw = ctx->walk_buf.as<char>();
    std::vector<char> hw(o_out);
    std::memcpy(hw.data(), wj.data(), sizeof(WalkJob2) * wj.size());
    if (!wtop.empty()) std::memcpy(hw.data() + o_top, wtop.data(), sizeof(int4) * wtop.size());
    std::memcpy(hw.data() + o_b, wb.data(), sizeof(int4) * wb.size());
    hipStream_t st = ctx->stream;
    CSM_HIP(hipMemcpyAsync(dw, hw.data(), o_out, hipMemcpyHostToDevice, st));
    CSM_HIP(LaunchFast2dWalk(static_cast<int>(wj.size()), plan.max_npad, st,
                             ctx->submap_desc.as<SubmapDesc>(),
                             static_cast<const PairDesc*>(ctx->pair_desc_dev), scans->points.as<float>(),
                             scans->rot_dev.as<float2>(), reinterpret_cast<const WalkJob2*>(dw),
                             reinterpret_cast<const int4*>(dw + o_top),
                             reinterpret_cast<const int4*>(dw + o_b), reinterpret_cast<int4*>(dw + o_out)));
    std::vector<int4> found(wj.size());
    CSM_HIP(hipMemcpyAsync(found.data(), dw + o_out, sizeof(int4) * wj.size(), hipMemcpyDeviceToHost, st));
    CSM_HIP(hipStreamSynchronize(st));
    for (size_t wi = 0; wi < walk.size(); ++wi) {
      const int k = tied[walk[wi]];
      if (!found[wi].w) {
        // Unreachable: the maximum is some leaf's sum, and the walk visits
        // every node whose sum reaches it. Never return a leaf that is not
        // the reference's: the pair's result is void.
        (*keys)[k] = 0;
        (*stat)[k] |= kStatusRange;
        continue;
      }
      (*keys)[k] = PackLeafKey(static_cast<uint32_t>(pd2[walk[wi]].collect_sum), found[wi].x,
                               found[wi].y, found[wi].z);
    }
  }
  const auto tp5 = now();
  for (size_t wi = 0; wi < work.size(); ++wi) {
    const Tie& w = work[wi];
    const Cand& c = cand[wi];
    const PairDesc& d2 = pd2[w.t];
    const int T = w.depth - 1;
    const int step = 1 << T;
    auto anc = [&](int li, int lv) { return anc_of(w, li, lv); };
    // Sorted position of the top-level node (rot, x, y).
    auto top_pos = [&](int r, int x, int y) {
      const int ny = (c.rb[r][3] - c.rb[r][2] + step) / step;
      return c.pos[c.rot_first[r] + static_cast<int64_t>((x - c.rb[r][0]) / step) * ny +
                   (y - c.rb[r][2]) / step];
    };
    // The reference's visiting order of two tied leaves.
    auto first = [&](int a, int b) {
      for (int lv = T; lv >= 1; --lv) {
        const auto [ax, ay, as] = anc(a, lv);
        const auto [bx, by, bs] = anc(b, lv);
        const int ra = leaves[a].x, rb2 = leaves[b].x;
        if (ra == rb2 && ax == bx && ay == by) continue;
        if (as != bs) return as > bs;
        if (lv == T) return top_pos(ra, ax, ay) < top_pos(rb2, bx, by);
        return std::make_pair(ax, ay) < std::make_pair(bx, by);
      }
      if (T == 0)
        return top_pos(leaves[a].x, leaves[a].y, leaves[a].z) <
               top_pos(leaves[b].x, leaves[b].y, leaves[b].z);
      return std::make_pair(leaves[a].y, leaves[a].z) < std::make_pair(leaves[b].y, leaves[b].z);
    };
    int best = c.live[0];
    for (size_t i = 1; i < c.live.size(); ++i)
      if (first(c.live[i], best)) best = c.live[i];
    (*keys)[w.k] = PackLeafKey(static_cast<uint32_t>(d2.collect_sum), leaves[best].x,
                               leaves[best].y, leaves[best].z);
  }
  if (prof)
    std::fprintf(stderr,
                 "ties (ms): collect search %.2f, ancestors %.2f, bounds + lattice %.2f, "
                 "lattice scores %.2f, sorts %.2f, picks %.2f; %zu tied, %zu need the order\n",
                 ms(tp0, tp1), ms(tp1, tp2), ms(tp2, tp3), ms(tp3, tp4), ms(tp4, tp5),
                 ms(tp5, now()), tied.size(), perm.size());
  return CSM_OK;
}

int RunBatch(csm_context* ctx, csm_fast2d* const* submaps, int32_t num_submaps,
             csm_scan_set* scans, const csm_pair2d* pairs, int64_t num_pairs,
             csm_result2d* results) {
  // ---- host preparation ---------------------------------------------------
  const bool prof = std::getenv("CSM_PROFILE2D") != nullptr;
  const auto t_start = std::chrono::steady_clock::now();
  auto ms_since = [](std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
  };
  std::vector<SubmapDesc> sdesc(num_submaps);
  for (int i = 0; i < num_submaps; ++i) {
    // Any context on this device: a second context may build the next
    // batch's pyramids on its own stream while this one searches.
    if (!submaps[i] || submaps[i]->ctx->device != ctx->device) return CSM_EINVAL;
    sdesc[i] = submaps[i]->desc;
    // One launch serves one kernel: v4 (no hex levels) or v5 (fixed at create).
    if ((sdesc[i].hex_mask != 0) != (sdesc[0].hex_mask != 0)) return CSM_EINVAL;
  }
  const bool hex = num_submaps > 0 && sdesc[0].hex_mask != 0;
  std::vector<PairDesc> pdesc;
  std::vector<int64_t> pair_src;  // pdesc index -> pair index
  // Rotation tables live on the scan set's device table, appended once per
  // (scan, window) and kept across batches (csm_scan_set::rot_all).
  std::vector<float2>& rot_host = scans->rot_all;
  int max_npad = 64;
  for (int64_t i = 0; i < num_pairs; ++i) {
    const csm_pair2d& p = pairs[i];
    results[i].status = CSM_NO_MATCH;
    results[i].score = 0.f;
    results[i].pose = csm_pose2d{0., 0., 0.};
    results[i].tie = CSM_TIE_NONE;
    results[i].reserved = 0;
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
    auto ro = scans->rot_offsets.find(&win);
    int32_t off;
    if (ro == scans->rot_offsets.end()) {
      off = static_cast<int32_t>(rot_host.size());
      for (const ZRot& z : win.second) rot_host.push_back(make_float2(z.w, z.s));
      scans->rot_offsets.emplace(&win, off);
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
  SearchPlan plan;
  // The v4/v5 kernel keeps rot_chunk discretized scans (4 B/point) and their
  // cluster lists in LDS: up to kMaxPoints (16448 points, one rotation per
  // workgroup, ~128 KB) it fits, so it takes every batch; the v1 kernel
  // (lanes = points) runs only when forced (CSM_SEARCH_KERNEL=1).
  plan.use_v2 = forced != 1;
  plan.hex = hex;
  plan.max_npad = max_npad;
  const char* rc_env = std::getenv("CSM_ROT_CHUNK");
  const int v4_budget = 9 * 1024;  // C2 (1088 padded points): 2 rotations per chunk, the measured best
  const int v4_rc = rc_env ? std::max(1, std::min(kV4MaxRotChunk, std::atoi(rc_env)))
                           : std::max(1, std::min(std::min(8, kV4MaxRotChunk), v4_budget / (max_npad * 4)));
  const int lds_budget = 40 * 1024;
  plan.rc = plan.use_v2 ? v4_rc : std::max(1, std::min(16, lds_budget / (max_npad * 4)));
  // Node order: FIFO (level by level, the default) or LIFO (depth-first,
  // CSM_SEARCH_ORDER=lifo).
  const char* order_env = std::getenv("CSM_SEARCH_ORDER");
  plan.fifo = !(order_env && std::strcmp(order_env, "lifo") == 0);

  // ---- uploads shared by the search and the tie resolution ------------------
  int rcode;
  if ((rcode = ctx->submap_desc.Reserve(sizeof(SubmapDesc) * num_submaps))) return rcode;
  if (rot_host.size() > scans->rot_uploaded) {  // new windows since the last batch
    const size_t want = sizeof(float2) * rot_host.size();
    if (want > scans->rot_dev.bytes) {  // a new buffer: upload the whole table below
      if ((rcode = scans->rot_dev.Reserve(want + want / 2))) return rcode;
      scans->rot_uploaded = 0;
    }
  }
  hipStream_t st = ctx->stream;
  // Staged through pinned memory (async copies; the stage is rewritten only
  // by the next batch on this context, after this one's synchronize).
  {
    const size_t sd_bytes = sizeof(SubmapDesc) * num_submaps;
    const size_t rot_new = rot_host.size() - std::min(rot_host.size(), scans->rot_uploaded);
    const size_t rot_at = (sd_bytes + 255) & ~size_t{255};
    if ((rcode = ctx->upload_stage.Reserve(rot_at + sizeof(float2) * rot_new))) return rcode;
    char* h = ctx->upload_stage.as<char>();
    std::memcpy(h, sdesc.data(), sd_bytes);
    CSM_HIP(hipMemcpyAsync(ctx->submap_desc.ptr, h, sd_bytes, hipMemcpyHostToDevice, st));
    if (rot_new > 0) {
      const size_t first = rot_host.size() - rot_new;
      std::memcpy(h + rot_at, rot_host.data() + first, sizeof(float2) * rot_new);
      CSM_HIP(hipMemcpyAsync(scans->rot_dev.as<float2>() + first, h + rot_at, sizeof(float2) * rot_new,
                             hipMemcpyHostToDevice, st));
      scans->rot_uploaded = rot_host.size();
    }
  }
  std::vector<uint64_t> keys, keys_hi;
  std::vector<int32_t> stat;
  unsigned long long stats_host[kStatsWords] = {0};
  const double prep_ms = ms_since(t_start);
  const auto t_search = std::chrono::steady_clock::now();
  if ((rcode = LaunchSearch(ctx, scans, pdesc, nullptr, plan, ctx->timing, &keys, &keys_hi, &stat,
                            stats_host)))
    return rcode;
  float kernel_ms = 0.f;
  if (ctx->timing) {
    float ms = 0.f;
    CSM_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
    kernel_ms = ms;
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
    const unsigned long long* kl = stats_host + kStatLines;
    bool any_lines = false;
    for (int l = 0; l < kMaxLevels; ++l) any_lines |= kl[kMaxLevels + l] != 0;
    if (std::getenv("CSM_PROFILE2D") && any_lines) {
      std::fprintf(stderr, "fast2d lines per gather by child level:");
      for (int l = 0; l < kMaxLevels; ++l)
        if (kl[kMaxLevels + l])
          std::fprintf(stderr, " L%d %.1f (%.3g instr)", l,
                       static_cast<double>(kl[l]) / kl[kMaxLevels + l],
                       static_cast<double>(kl[kMaxLevels + l]));
      std::fprintf(stderr, "\n");
      std::fprintf(stderr, "fast2d quad lines per gather by child level:");
      for (int l = 0; l < kMaxLevels; ++l)
        if (kl[kMaxLevels + l])
          std::fprintf(stderr, " L%d %.1f", l, static_cast<double>(kl[2 * kMaxLevels + l]) / kl[kMaxLevels + l]);
      std::fprintf(stderr, "\n");
      std::fprintf(stderr, "fast2d out-of-range / active lanes per gather by child level:");
      for (int l = 0; l < kMaxLevels; ++l)
        if (kl[kMaxLevels + l])
          std::fprintf(stderr, " L%d %.1f/%.1f", l, static_cast<double>(kl[4 * kMaxLevels + l]) / kl[kMaxLevels + l],
                       static_cast<double>(kl[3 * kMaxLevels + l]) / kl[kMaxLevels + l]);
      std::fprintf(stderr, "\n");
    }
  }

  // ---- exactly tied maxima: the reference's pick (ResolveTies) ---------------
  const double search_ms = ms_since(t_search);
  const auto t_ties = std::chrono::steady_clock::now();
  const int64_t tied_before = ctx->t.tied_pairs;
  std::vector<int8_t> tie_code(np, CSM_TIE_NONE);
  if (plan.use_v2 && (rcode = ResolveTies(ctx, submaps, scans, pdesc, rot_host, plan, &stat, keys_hi,
                                           &keys, &tie_code)))
    return rcode;
  const double ties_ms = ms_since(t_ties);
  const auto t_decode = std::chrono::steady_clock::now();

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
    results[i].tie = tie_code[k];
    results[i].score = SumToScore(sum, d.num_points, m->min_s, m->max_s);
    results[i].pose.x = init.x + cx;
    results[i].pose.y = init.y + cy;
    results[i].pose.theta = init.theta + co;
  }
  if (prof)
    std::fprintf(stderr,
                 "fast2d batch host (ms): prep %.2f, search + readback %.2f (kernel %.2f), ties %.2f "
                 "(%lld pairs), decode %.2f; %d pairs\n",
                 prep_ms, search_ms, kernel_ms, ties_ms,
                 static_cast<long long>(ctx->t.tied_pairs - tied_before), ms_since(t_decode), np);
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
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && total_b > 0)
    ctx->pool.SetCapBytes(total_b / 4);  // idle pooled buffers: at most a quarter of the device
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
  if (!ctx || !out) return;
  *out = ctx->t;
  std::lock_guard<std::mutex> g(ctx->call_mu);  // single calls' share
  AddTiming(out, ctx->call_t);
}
void csm_context_reset_timing(csm_context* ctx) {
  if (!ctx) return;
  ctx->t = csm_timing{};
  {
    std::lock_guard<std::mutex> g(ctx->call_mu);
    ctx->call_t = csm_timing{};
  }
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
  hipStream_t st = ctx->stream;
  int rc;
  // Quantization and correspondence-cost tables, kept on the device for the
  // last (min_cc, max_cc).
  if (ctx->f2_tab_key[0] != min_cc || ctx->f2_tab_key[1] != max_cc) {
    std::vector<uint8_t> qtab(32768);
    if (!QuantizationTable(min_cc, max_cc, qtab.data())) return CSM_EINVAL;
    std::vector<float> ctab(32768);
    ConversionTable(max_cc, min_cc, max_cc, ctab.data());
    if ((rc = ctx->f2_qtab.Reserve(32768)) || (rc = ctx->f2_ctab.Reserve(sizeof(float) * 32768)))
      return rc;
    CSM_HIP(hipMemcpyAsync(ctx->f2_qtab.ptr, qtab.data(), 32768, hipMemcpyHostToDevice, st));
    CSM_HIP(hipMemcpyAsync(ctx->f2_ctab.ptr, ctab.data(), sizeof(float) * 32768,
                           hipMemcpyHostToDevice, st));
    CSM_HIP(hipStreamSynchronize(st));
    ctx->f2_tab_key[0] = min_cc;
    ctx->f2_tab_key[1] = max_cc;
  }

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
        kind[L - 2] = kHexEntryBytes;
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
      const bool hexl = kind[l] == kHexEntryBytes;
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
  if ((rc = ctx->pool.Take(total, &m->pyramid))) return rc;
  d.pyramid_base = m->pyramid.as<uint8_t>();
  d.pyramid_bytes = static_cast<int32_t>(total);
  for (int l = 0; l < depth; ++l) {
    d.level[l] = m->pyramid.as<uint8_t>() + offs[l];
    d.quad[l] = reinterpret_cast<const uint32_t*>(m->pyramid.as<uint8_t>() + qoffs[l]);
    d.quad_off[l] = static_cast<int32_t>(qoffs[l]);
  }

  DevBuf& dcells = ctx->f2_cells;
  const DevBuf& dq = ctx->f2_qtab;
  if ((rc = dcells.Reserve(sizeof(uint16_t) * nx * ny))) return rc;
  CSM_HIP(hipMemcpyAsync(dcells.ptr, cells, sizeof(uint16_t) * nx * ny, hipMemcpyHostToDevice, st));
  const int n0 = nx * ny;
  CSM_HIP(LaunchPyramidLevel0(dcells.as<uint16_t>(), dq.as<uint8_t>(),
                              const_cast<uint8_t*>(d.level[0]), n0, st));
  for (int l = 1; l < depth; ++l) {
    CSM_HIP(LaunchPyramidDouble(d.level[l - 1], d.wide_nx[l - 1], d.wide_ny[l - 1],
                                const_cast<uint8_t*>(d.level[l]), d.wide_nx[l], d.wide_ny[l],
                                1 << (l - 1), st));
  }
  DevBuf& dwiden = ctx->f2_widen;
  if (widen_bytes && (rc = dwiden.Reserve(widen_bytes))) return rc;
  for (int l = 0; l < depth; ++l) {
    const int km1 = (1 << d.cshift[l]) - 1;
    if (d.quad_es[l] == 4)
      CSM_HIP(LaunchPyramidQuad(d.level[l], d.wide_nx[l], d.wide_ny[l], l, km1,
                                const_cast<uint32_t*>(d.quad[l]), d.quad_w[l], d.quad_h[l],
                                d.quad_pws[l], d.quad_pph[l], d.quad_bytes[l] / 4, st));
    else if (d.quad_es[l] == kHexEntryBytes)
      CSM_HIP(LaunchPyramidHex(d.level[l], d.wide_nx[l], d.wide_ny[l], l, km1, dwiden.as<uint8_t>(),
                               const_cast<uint32_t*>(d.quad[l]), d.quad_w[l], d.quad_h[l],
                               d.quad_pws[l], d.quad_pph[l], d.quad_bytes[l] / kHexEntryBytes, st));
  }
  // Correspondence costs (Grid2D::GetCorrespondenceCost, grid_2d.cc) for the
  // CeresScanMatcher2D refinement: the value table with unknown -> max_cc.
  if ((rc = ctx->pool.Take(sizeof(float) * n0, &m->cost))) return rc;
  CSM_HIP(LaunchCellsToProbability(dcells.as<uint16_t>(), ctx->f2_ctab.as<float>(),
                                   m->cost.as<float>(), n0, st));
  // The cells are read from the caller's memory and the context's scratch
  // is reused by the next create: finish before returning.
  CSM_HIP(hipStreamSynchronize(st));
  *out = m.release();
  return CSM_OK;
}

void csm_fast2d_destroy(csm_fast2d* m) {
  if (!m) return;
  (void)hipSetDevice(m->ctx->device);
  m->ctx->pool.Give(&m->pyramid);  // reused by the next create
  m->ctx->pool.Give(&m->cost);
  delete m;
}

int64_t csm_fast2d_device_bytes(const csm_fast2d* m) {
  return m ? static_cast<int64_t>(m->pyramid.bytes + m->cost.bytes) : 0;
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

int csm_scan_set_append(csm_scan_set* s, const float* points_xyz, const int64_t* offsets,
                        int32_t num_scans, int32_t* first_index) {
  if (!s || !offsets || !first_index || num_scans < 0 || offsets[0] != 0) return CSM_EINVAL;
  const int64_t added = offsets[num_scans];
  if (added < 0 || (added > 0 && !points_xyz)) return CSM_EINVAL;
  for (int32_t i = 0; i < num_scans; ++i)
    if (offsets[i + 1] < offsets[i]) return CSM_EINVAL;
  csm_context* ctx = s->ctx;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (EnsureDevice(ctx)) return CSM_EHIP;
  const int64_t old_total = s->offsets.back();
  if (static_cast<int64_t>(s->offsets.size()) - 1 + num_scans > INT32_MAX) return CSM_ERANGE;
  const size_t need = sizeof(float) * 3 * static_cast<size_t>(old_total + added);
  if (need > s->points.bytes) {
    // Grow by half again, keeping the resident clouds (device-to-device).
    csm::DevBuf grown;
    if (grown.Reserve(std::max(need, s->points.bytes + s->points.bytes / 2))) return CSM_ENOMEM;
    if (old_total > 0)
      CSM_HIP(hipMemcpyAsync(grown.ptr, s->points.ptr, sizeof(float) * 3 * old_total,
                             hipMemcpyDeviceToDevice, ctx->stream));
    CSM_HIP(hipStreamSynchronize(ctx->stream));
    std::swap(grown.ptr, s->points.ptr);
    std::swap(grown.bytes, s->points.bytes);
  }
  if (added > 0)
    CSM_HIP(hipMemcpyAsync(s->points.as<float>() + 3 * old_total, points_xyz,
                           sizeof(float) * 3 * added, hipMemcpyHostToDevice, ctx->stream));
  CSM_HIP(hipStreamSynchronize(ctx->stream));
  *first_index = static_cast<int32_t>(s->offsets.size() - 1);
  s->host_points.insert(s->host_points.end(), points_xyz, points_xyz + 3 * added);
  for (int32_t i = 0; i < num_scans; ++i) s->offsets.push_back(old_total + offsets[i + 1]);
  return CSM_OK;
}

int csm_scan_set_size(const csm_scan_set* s, int32_t* num_scans, int64_t* num_points) {
  if (!s || !num_scans || !num_points) return CSM_EINVAL;
  *num_scans = static_cast<int32_t>(s->offsets.size() - 1);
  *num_points = s->offsets.back();
  return CSM_OK;
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

// One single Match / MatchFullSubmap call waiting in its owner's queue.
struct SingleReq2 {
  const csm_fast2d* m;
  int full;
  csm_pose2d initial;
  const float* xyz;
  int32_t n;
  float min_score;
  csm_result2d res;
  int rc;
  bool done;
};

constexpr int kCoalesceCap = 512;  // pairs per coalesced batch
// Batches of queued single calls in flight, and a leader's longest wait for
// more callers (A/B: CSM_COALESCE_LEADERS, CSM_COALESCE_WINDOW_US).
static int CoalesceLeaders() {
  static const int v = [] {
    const char* e = std::getenv("CSM_COALESCE_LEADERS");
    return e ? std::max(1, std::atoi(e)) : 3;
  }();
  return v;
}
static int CoalesceWindowUs() {
  static const int v = [] {
    const char* e = std::getenv("CSM_COALESCE_WINDOW_US");
    return e ? std::max(0, std::atoi(e)) : 150;
  }();
  return v;
}

// Searches queued single calls as batches on one call context of `owner`: all
// clouds in the call context's scan set, one pair per request (one batch per
// plane kind, since a launch serves one kernel).
static int RunSingleBatch(csm_context* owner, const std::vector<SingleReq2*>& reqs, int share) {
  csm::CallContext cc(owner);
  csm_context* ctx = cc.get();
  if (!ctx) return CSM_EHIP;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (EnsureDevice(ctx)) return CSM_EHIP;
  ctx->grid_share = std::max(1, share);
  csm_scan_set& s = ctx->single;
  s.ctx = ctx;
  s.offsets.assign(1, 0);
  s.host_points.clear();
  for (const SingleReq2* r : reqs) {
    s.host_points.insert(s.host_points.end(), r->xyz, r->xyz + 3 * static_cast<size_t>(r->n));
    s.offsets.push_back(s.offsets.back() + r->n);
  }
  // Scan indices name different clouds on every batch: no window is kept.
  s.windows.clear();
  s.rot_all.clear();
  s.rot_offsets.clear();
  s.rot_uploaded = 0;
  const int64_t total = s.offsets.back();
  int rc;
  if ((rc = s.points.Reserve(sizeof(float) * 3 * std::max<int64_t>(total, 1)))) return rc;
  if (total > 0) {
    if ((rc = ctx->single_stage.Reserve(sizeof(float) * 3 * total))) return rc;
    std::memcpy(ctx->single_stage.ptr, s.host_points.data(), sizeof(float) * 3 * total);
    CSM_HIP(hipMemcpyAsync(s.points.ptr, ctx->single_stage.ptr, sizeof(float) * 3 * total,
                           hipMemcpyHostToDevice, ctx->stream));
  }
  for (int kind = 0; kind < 2; ++kind) {  // v4 (no hex planes), then v5
    std::vector<csm_fast2d*> handles;
    std::map<const csm_fast2d*, int> slot;
    std::vector<csm_pair2d> pairs;
    std::vector<size_t> which;
    for (size_t k = 0; k < reqs.size(); ++k) {
      const SingleReq2* r = reqs[k];
      if ((r->m->desc.hex_mask != 0) != (kind == 1)) continue;
      auto it = slot.find(r->m);
      if (it == slot.end()) {
        it = slot.emplace(r->m, static_cast<int>(handles.size())).first;
        handles.push_back(const_cast<csm_fast2d*>(r->m));
      }
      csm_pair2d p{};
      p.submap = it->second;
      p.scan = static_cast<int32_t>(k);
      p.full_submap = r->full;
      p.min_score = r->min_score;
      if (!r->full) p.initial = r->initial;
      pairs.push_back(p);
      which.push_back(k);
    }
    if (pairs.empty()) continue;
    std::vector<csm_result2d> res(pairs.size());
    if ((rc = RunBatch(ctx, handles.data(), static_cast<int32_t>(handles.size()), &s, pairs.data(),
                       static_cast<int64_t>(pairs.size()), res.data())) < 0)
      return rc;
    for (size_t k = 0; k < which.size(); ++k) reqs[which[k]]->res = res[k];
  }
  return CSM_OK;
}

// The reference's tasks call Match / MatchFullSubmap concurrently from
// ThreadPool workers (constraint_builder_2d.cc:100-111, :188-215). One call
// is one pair, far too little to fill the GPU, so concurrent callers of one
// owner context are coalesced: each queues its pair; a caller that finds
// fewer than CoalesceLeaders() (3) batches running becomes a leader, waits up
// to CoalesceWindowUs() (150 us) for as many callers as the previous batch
// had, takes the
// queue and searches it as one batch on a call context, then wakes the
// callers it served. Results are the same as one call at a time (a pair's
// result does not depend on its batch). CSM_SINGLE_COALESCE=0 runs each call
// alone on its own call context.
static int SingleMatch(const csm_fast2d* m, const csm_pose2d* initial, int full,
                       const float* xyz, int32_t n, float min_score, float* score,
                       csm_pose2d* pose) {
  if (!m || !score || !pose || (n > 0 && !xyz) || n < 0 || (!full && !initial)) return CSM_EINVAL;
  csm_context* owner = m->ctx;
  struct InFlight {  // this call counted among the owner's concurrent single calls
    std::atomic<int>& c;
    explicit InFlight(std::atomic<int>& a) : c(a) { ++c; }
    ~InFlight() { --c; }
  } in_flight(owner->calls_in_flight);
  SingleReq2 r{m, full, full ? csm_pose2d{0., 0., 0.} : *initial, xyz, n, min_score, {}, CSM_OK, false};
  static const bool coalesce = [] {
    const char* e = std::getenv("CSM_SINGLE_COALESCE");
    return !(e && std::strcmp(e, "0") == 0);
  }();
  if (!coalesce) {
    std::vector<SingleReq2*> one{&r};
    try {
      r.rc = RunSingleBatch(owner, one, owner->calls_in_flight.load());
    } catch (...) {  // no exception crosses the C-ABI
      r.rc = CSM_ENOMEM;
    }
  } else {
    std::unique_lock<std::mutex> lk(owner->co_mu);
    owner->co_queue.push_back(&r);
    owner->co_cv.notify_all();
    while (!r.done) {
      const bool queued = std::find(owner->co_queue.begin(), owner->co_queue.end(), &r) !=
                          owner->co_queue.end();
      if (queued && owner->co_leaders < CoalesceLeaders()) {
        ++owner->co_leaders;
        const size_t want = static_cast<size_t>(std::max(1, owner->co_last_batch));
        const auto deadline =
            std::chrono::steady_clock::now() + std::chrono::microseconds(CoalesceWindowUs());
        while (owner->co_queue.size() < want &&
               owner->co_cv.wait_until(lk, deadline) != std::cv_status::timeout) {
        }
        const size_t take_n = std::min<size_t>(owner->co_queue.size(), kCoalesceCap);
        std::vector<SingleReq2*> take;
        for (size_t i = 0; i < take_n; ++i) take.push_back(static_cast<SingleReq2*>(owner->co_queue[i]));
        owner->co_queue.erase(owner->co_queue.begin(), owner->co_queue.begin() + take_n);
        owner->co_last_batch = static_cast<int>(take_n);
        // The batch's share of the persistent grid: the whole grid (a
        // second batch's workgroups start as the first one's drain; measured
        // 11.3k -> 12.7k pairs/s at 16 threads against a share per leader,
        // profiles/r5r/). CSM_COALESCE_SHARE=n: 1/n of it; 0: one share per
        // leader running.
        static const int fixed_share = [] {
          const char* e = std::getenv("CSM_COALESCE_SHARE");
          return e ? std::max(0, std::atoi(e)) : 1;
        }();
        const int share = fixed_share ? fixed_share : owner->co_leaders;
        lk.unlock();
        // Whatever happens in the batch (an allocation that throws), every
        // request taken is answered and the leader slot given back below;
        // otherwise their callers would wait on co_cv forever.
        int rc;
        try {
          rc = RunSingleBatch(owner, take, share);
        } catch (...) {
          rc = CSM_ENOMEM;
        }
        lk.lock();
        for (SingleReq2* q : take) {
          q->rc = rc;
          q->done = true;
        }
        --owner->co_leaders;
        owner->co_cv.notify_all();
      } else {
        owner->co_cv.wait(lk);
      }
    }
  }
  if (r.rc < 0) return r.rc;
  if (r.res.status == CSM_OK) {
    *score = r.res.score;
    *pose = r.res.pose;
  }
  return r.res.status;
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


