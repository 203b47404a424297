// Internal host-side types shared by the 2D and 3D halves of the C-ABI
// implementation (csm_host.cc, host3d.cc). Not part of the public boundary.
#ifndef CSM_INTERNAL_H_
#define CSM_INTERNAL_H_

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <condition_variable>
#include <mutex>
#include <tuple>
#include <deque>
#include <vector>

#include "../../include/csm_amd.h"
#include "csm_device.h"
#include "csm_device3d.h"
#include "search_window.h"

namespace csm {

#define CSM_HIP(call)                               \
  do {                                              \
    if ((call) != hipSuccess) return CSM_EHIP;      \
  } while (0)

// Frees every context's idle pooled buffers (BufPool below); a device
// allocation that fails calls it and tries once more.
void ReleaseIdlePools();

// Grow-only device buffer.
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  ~DevBuf() {
    if (ptr) (void)hipFree(ptr);
  }
  int Reserve(size_t n) {
    if (n <= bytes) return CSM_OK;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    bytes = 0;
    const size_t want = std::max<size_t>(n, 256);
    if (hipMalloc(&ptr, want) != hipSuccess) {
      ReleaseIdlePools();
      if (hipMalloc(&ptr, want) != hipSuccess) {
        ptr = nullptr;
        return CSM_ENOMEM;
      }
    }
    bytes = want;
    return CSM_OK;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(ptr); }
};

// Device buffers of destroyed matchers and grids (2D pyramids and cost
// grids, 3D bricks, levels and octets), kept for reuse by the next create: a
// sweep builds and drops thousands of submaps, and hipMalloc / hipFree of
// tens to hundreds of MB dominate a build otherwise (C5: 1.75 ms per submap).
// Take: the smallest idle buffer holding n bytes and at most twice that, else
// a new allocation. Give: keeps the buffer, freeing the oldest ones past the
// caps (bytes: a quarter of the device's memory by default; count). Every
// pool is registered process-wide so that any failed device allocation in the
// library first releases all idle pooled memory (ReleaseIdlePools).
class BufPool {
 public:
  BufPool();
  ~BufPool();
  BufPool(const BufPool&) = delete;
  BufPool& operator=(const BufPool&) = delete;
  int Take(size_t n, DevBuf* out);
  void Give(DevBuf* b);
  void Release();
  void SetCapBytes(size_t cap) { cap_bytes_ = cap; }
  size_t held() const { return held_; }

 private:
  std::mutex mu_;
  std::vector<std::pair<void*, size_t>> bufs_;
  size_t held_ = 0;
  size_t cap_bytes_ = size_t{1} << 30;
};

// Page-locked host staging (H2D copies at full PCIe rate).
struct PinnedBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  ~PinnedBuf() {
    if (ptr) (void)hipHostFree(ptr);
  }
  int Reserve(size_t n) {
    if (n <= bytes) return CSM_OK;
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    bytes = 0;
    const size_t want = std::max<size_t>(n + n / 4, 4096);
    if (hipHostMalloc(&ptr, want, hipHostMallocDefault) != hipSuccess) return CSM_ENOMEM;
    bytes = want;
    return CSM_OK;
  }
  template <typename T>
  T* as() const { return static_cast<T*>(ptr); }
};

// Pinned staging slots, each with the event of its last upload. Take(bytes):
// the smallest slot whose upload has finished and that already holds `bytes`;
// else a new slot sized for this request (while fewer than kMax slots and
// kMaxPinned bytes are held); else a finished slot (or, when none is, the
// next one in turn once its upload is done) regrown to the request. A slot is
// never regrown while a fitting one is free, because freeing pinned memory
// (hipHostFree) waits for the device, which may be busy with a search kernel
// for tens of ms. Each slot is sized to the requests it served, not to the
// largest upload ever staged, so one large batch upload does not inflate
// every later small create's slot. A deque, so slots never move. The caller
// records `copied` after its copy.
struct StageRing {
  struct Slot {
    PinnedBuf buf;
    hipEvent_t copied = nullptr;
  };
  static constexpr size_t kMax = 128;
  static constexpr size_t kMaxPinned = size_t{1} << 30;  // pinned bytes past which slots are reused
  std::deque<Slot> slots;
  size_t next = 0;
  size_t pinned = 0;  // sum of the slots' buffer sizes
  ~StageRing() {
    for (Slot& s : slots)
      if (s.copied) (void)hipEventDestroy(s.copied);
  }
  int Take(size_t bytes, Slot** out) {
    const size_t n = slots.size();
    size_t fit = n, any = n;  // smallest finished slot that fits; some finished slot
    for (size_t k = 0; k < n; ++k) {
      const size_t i = (next + k) % n;
      if (hipEventQuery(slots[i].copied) != hipSuccess) continue;
      if (any == n) any = i;
      if (slots[i].buf.bytes >= bytes && (fit == n || slots[i].buf.bytes < slots[fit].buf.bytes)) fit = i;
    }
    size_t at = fit;
    if (at == n && n < kMax && (n == 0 || pinned + bytes <= kMaxPinned)) {
      slots.emplace_back();
      if (hipEventCreateWithFlags(&slots.back().copied, hipEventDisableTiming) != hipSuccess) return CSM_EHIP;
      at = n;
    } else if (at == n && any != n) {
      at = any;
    } else if (at == n) {
      at = next % n;
      if (hipEventSynchronize(slots[at].copied) != hipSuccess) return CSM_EHIP;
    }
    next = at + 1;
    *out = &slots[at];
    PinnedBuf& b = slots[at].buf;
    pinned -= b.bytes;
    const int rc = b.Reserve(bytes);
    pinned += b.bytes;
    return rc;
  }
};

// RealTimeCorrelativeScanMatcher2D state (rt2d.hip): the converted, padded
// grid of the last call (re-made only when cells / padding / TSDF
// parameters change), its host copy for the comparison, conversion tables
// and per-call scratch.
struct Rt2dCache {
  bool valid = false, tsdf = false, tables = false, ttab_ok = false;
  int nx = 0, ny = 0, P = 0;
  float truncation = 0.f, max_weight = 0.f;
  float ttab_key[2] = {0.f, 0.f};
  std::vector<uint16_t> cells, wcells;
  DevBuf grid, dcells, ptab, ttab, bases, best, dstage, sink;
  PinnedBuf stage, stage_cells, host_key, wg_keys;  // wg_keys: per-workgroup keys (zero-copy path)
};

}  // namespace csm

struct csm_scan_set {
  csm_context* ctx = nullptr;
  std::vector<float> host_points;
  std::vector<int64_t> offsets;
  csm::DevBuf points;
  // Rotation tables per (scan, angular window, linear window, resolution).
  std::map<std::tuple<int, double, double, double>,
           std::pair<csm::SearchWindow2D, std::vector<csm::ZRot>>>
      windows;
  // Their device copy, appended as batches meet new windows: (w, s) per
  // rotation, the offset of each window's table, and how much is uploaded.
  std::vector<float2> rot_all;
  std::map<const void*, int32_t> rot_offsets;
  csm::DevBuf rot_dev;
  size_t rot_uploaded = 0;
};

// Timing records add up field by field (the stack high-water mark: max).
inline void AddTiming(csm_timing* a, const csm_timing& b) {
  a->search_kernel_ms += b.search_kernel_ms;
  a->search_launches += b.search_launches;
  a->search_lookups += b.search_lookups;
  a->search_candidates += b.search_candidates;
  a->other_kernel_ms += b.other_kernel_ms;
  a->rt3d_kernel_ms += b.rt3d_kernel_ms;
  a->rt3d_lookups += b.rt3d_lookups;
  a->fast3d_kernel_ms += b.fast3d_kernel_ms;
  a->fast3d_launches += b.fast3d_launches;
  a->fast3d_lookups += b.fast3d_lookups;
  a->search_errors += b.search_errors;
  a->stack_high_water = std::max(a->stack_high_water, b.stack_high_water);
  a->tied_pairs += b.tied_pairs;
  a->ties_walked += b.ties_walked;
  a->ties_toplist += b.ties_toplist;
  a->tied_pairs_3d += b.tied_pairs_3d;
  a->ties_walked_3d += b.ties_walked_3d;
}

struct csm_context {
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // Single Match / MatchFullSubmap calls (csm_fast2d_match*, csm_fast3d_match*)
  // run on a call context taken from the matcher's context for the duration
  // of the call: its own stream and scratch, the matcher's device pyramid
  // shared read-only. The reference calls these const methods concurrently
  // from ThreadPool workers (constraint_builder_2d.cc:100-111); concurrent
  // callers get distinct call contexts, so their searches overlap on the GPU
  // instead of queuing on the creator's stream. The pool grows to the largest
  // number of concurrent callers and is destroyed with the context.
  std::mutex call_mu;
  std::vector<csm_context*> call_free, call_all;
  csm_context* call_owner = nullptr;  // set on call contexts
  std::atomic<int> calls_in_flight{0};  // single calls running on this owner's call contexts
  int grid_share = 1;  // a call context's search launch takes 1/grid_share of the GPU
  // Coalesced single 2D calls (csm_host.cc SingleMatch): concurrent callers of
  // this owner queue their pairs; a leader takes the queue after a short
  // window and searches it as one batch on a call context, at most
  // kCoalesceLeaders batches at a time.
  std::mutex co_mu;
  std::condition_variable co_cv;
  std::vector<void*> co_queue;
  int co_leaders = 0;
  int co_last_batch = 1;  // the last batch's size: the next leader waits for as many
  // The same for single 3D calls (host3d.cc SingleMatch3), under co_mu.
  std::vector<void*> co3_queue;
  int co3_leaders = 0;
  int co3_last_batch = 1;
  int co3_in_flight = 0;  // single 3D calls between queueing and their return
  int co3_callers = 0;    // recent high-water of co3_in_flight (one less per batch)
  csm_timing call_t{};                // finished single calls' timing (call_mu)
  csm_scan_set single;                // the cloud of the current single 2D call
  csm::PinnedBuf single_stage;
  csm::DevBuf submap_desc, spill, single_points, ties, sq_jobs, sq_queries, sq_sums, walk_buf;
  // One 2D search launch's descriptors and outputs (csm_host.cc LaunchSearch),
  // with pinned staging for its one upload and one readback.
  csm::DevBuf arena;
  csm::PinnedBuf arena_in, arena_out, upload_stage;
  const void* pair_desc_dev = nullptr;  // the last launch's PairDesc array (in arena)
  csm::Rt2dCache rt2d;
  std::atomic<bool> timing{false};
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  csm_timing t{};
  double level_cands[csm::kMaxLevels] = {0};
  double level_batches[csm::kMaxLevels] = {0};
  int num_cus = 256;
  // 3D path scratch (host3d.cc).
  csm::DevBuf rt3_rot, rt3_rot4, rt3_cols, rt3_trans, rt3_points, rt3_best, f3_pairs, f3_yaws, f3_points,
      f3_low_points, f3_best, f3_status, f3_counter, f3_items, f3_scores, f3_spill, f3_best_hi,
      f3_ties, f3_tie_count, f3_tie_yaws, f3_sq_jobs, f3_sq_queries, f3_sq_sums, f3_walk_buf;
  csm::PinnedBuf f3_host_yaws, f3_host_points;
  // Pinned staging of a 3D batch's small uploads and readbacks (one copy
  // each way per phase), and the device buffer the readbacks are packed in.
  csm::PinnedBuf f3_up, f3_rb;
  csm::DevBuf f3_pack;
  // Side stream for the 3D batch's cloud upload (overlaps the rotational
  // scores on `stream`); the search waits on f3_points_ready.
  hipStream_t f3_copy_stream = nullptr;
  hipEvent_t f3_points_ready = nullptr;
  // Pinned staging of csm_hybrid_grid_create's cell lists and
  // csm_fast3d_create_batch's job lists: one slot per upload in flight (a
  // create takes a slot whose copy has finished, or a new one; TakeStageSlot),
  // so a create never waits for an earlier create's upload, which may sit
  // behind a search kernel holding every CU. Batched grid creates
  // (csm_hybrid_grid_create_batch) stage whole groups and have a ring of
  // their own, so single creates never take a slot sized for a batch.
  csm::StageRing f3_grid_stage, f3_grid_batch_stage, f3_job_stage;
  // Batched pyramid builds (csm_fast3d_create_batch): job lists.
  csm::DevBuf f3_jobs;
  // Voxel filter scratch (voxel_filter.hip).
  csm::DevBuf vf_points, vf_offsets, vf_keep, vf_counts;
  // CeresScanMatcher2D refinement scratch (ceres2d.hip).
  csm::DevBuf cr_items, cr_out, cr3_items, cr3_points, cr3_out;
  // Device buffers of destroyed matchers and grids kept for reuse (BufPool),
  // csm_fast2d_create's scratch and the quantization / cost tables of the
  // last (min_cc, max_cc); the 3D value tables and the pinned staging of
  // csm_hybrid_grid_create.
  csm::BufPool pool;
  csm::DevBuf f2_cells, f2_widen, f2_qtab, f2_ctab;
  float f2_tab_key[2] = {-1.f, -1.f};
  csm::DevBuf f3_ptab, f3_qtab, f3_grid_cells, f3_grid_batch;
  bool f3_tables = false;
  ~csm_context() {
    for (csm_context* c : call_all) csm_context_destroy(c);
  }
};

// One submap's device data (csm_host.cc builds it).
struct csm_fast2d {
  csm_context* ctx = nullptr;
  csm_map_limits limits{};
  csm_fast2d_options options{};
  float min_cc = 0.f, max_cc = 0.f, min_s = 0.f, max_s = 0.f;
  csm::SubmapDesc desc{};
  csm::DevBuf pyramid;
  csm::DevBuf cost;  // float correspondence costs, x fastest (CeresScanMatcher2D refinement)
};

namespace csm {
// Call contexts (csm_context::call_free): taken for one single Match call,
// returned with its timing added to the owner's.
csm_context* AcquireCallContext(csm_context* owner);
void ReleaseCallContext(csm_context* owner, csm_context* c);
class CallContext {
 public:
  explicit CallContext(csm_context* owner) : owner_(owner), c_(AcquireCallContext(owner)) {}
  ~CallContext() { ReleaseCallContext(owner_, c_); }
  CallContext(const CallContext&) = delete;
  CallContext& operator=(const CallContext&) = delete;
  csm_context* get() const { return c_; }

 private:
  csm_context* owner_;
  csm_context* c_;
};
}  // namespace csm

// A HybridGrid on the device (host3d.cc builds it).
struct csm_hybrid_grid {
  csm_context* ctx = nullptr;
  // Recorded on ctx->stream after the build's kernels (creates return
  // without waiting): consumers on other streams wait on it (WaitBuilt).
  hipEvent_t ready = nullptr;
  float resolution = 0.f;
  int32_t grid_size = 0;
  csm::Brick3 brick{};
  csm::DevBuf values;    // uint16 brick
  csm::DevBuf prob;      // float probability brick
  csm::DevBuf prob_pad;  // the same padded by one 0.1 cell per side (RTCSM3D), built on first use
  bool prob_pad_ready = false;
  csm::DevBuf prob_wide;  // padded by prob_wide_pad 0.1 cells per side (rt3d_score4)
  int prob_wide_pad = 0;
  csm::DevBuf prob_col;   // padded by prob_col_pad cells, z fastest (rt3d_score5)
  int prob_col_pad = 0;
};

namespace csm {
// Grids and matchers are built asynchronously on their context's stream and
// marked by a `ready` event. Work on the same stream is ordered after the
// build already; another stream (a call context, another context of the
// device) waits for the event on the device, host reads synchronize on it.
inline int WaitBuilt(hipEvent_t ready, hipStream_t producer, hipStream_t consumer) {
  if (!ready || producer == consumer) return CSM_OK;
  return hipStreamWaitEvent(consumer, ready, 0) == hipSuccess ? CSM_OK : CSM_EHIP;
}
}  // namespace csm

#endif  // CSM_INTERNAL_H_
