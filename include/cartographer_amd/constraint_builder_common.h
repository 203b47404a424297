// Types shared by the ConstraintBuilder2D / 3D drop-ins: ids, the
// ConstraintBuilderOptions proto (one proto carries both scan-matcher
// configurations, constraint_builder_options.proto:24-59) and
// common::FixedRatioSampler.
#ifndef CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_COMMON_H_
#define CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_COMMON_H_

#include <cstdint>
#include <list>
#include <map>
#include <memory>

#include "scan_matching.h"
#include "scan_matching_3d.h"

namespace cartographer_amd {

struct SubmapId {
  int trajectory_id = 0, submap_index = 0;
  bool operator<(const SubmapId& o) const {
    return trajectory_id != o.trajectory_id ? trajectory_id < o.trajectory_id
                                            : submap_index < o.submap_index;
  }
};
struct NodeId {
  int trajectory_id = 0, node_index = 0;
  bool operator<(const NodeId& o) const {
    return trajectory_id != o.trajectory_id ? trajectory_id < o.trajectory_id
                                            : node_index < o.node_index;
  }
};

// proto::ConstraintBuilderOptions (constraint_builder_options.proto:24-59),
// defaults from configuration_files/pose_graph.lua:17-29.
struct ConstraintBuilderOptions {
  double sampling_ratio = 0.3;
  double max_constraint_distance = 15.;
  float min_score = 0.55f;
  float global_localization_min_score = 0.6f;
  double loop_closure_translation_weight = 1.1e4;
  double loop_closure_rotation_weight = 1e5;
  FastCorrelativeScanMatcherOptions2D fast_correlative_scan_matcher_options;
  FastCorrelativeScanMatcherOptions3D fast_correlative_scan_matcher_options_3d;
  int flush_pairs = 0;  // 0: search each node's pairs when the node ends
  // ceres_scan_matcher (pose_graph.lua:30-39): accepted 2D matches are refined
  // with CeresScanMatcher2D (constraint_builder_2d.cc:245-249).
  csm_ceres2d_options ceres_scan_matcher_options{20., 10., 1., 10, /*nonmonotonic=*/1};
  // ceres_scan_matcher_3d (pose_graph.lua:49-60), ConstraintBuilder3D (:264-275).
  csm_ceres3d_options ceres_scan_matcher_options_3d{5., 30., 10., 1., 10, /*nonmonotonic=*/0};
  bool refine_with_ceres = true;
  // Node clouds stay on the device across flushes (a node's cloud is uploaded
  // once); past this many resident points the 2D builder starts a new set.
  int64_t scan_cache_points = int64_t{1} << 25;
  // Device memory the per-submap matcher cache may hold (MatcherCache below;
  // 0 = unbounded, the reference's behaviour: it keeps every matcher until
  // DeleteScanMatcher, constraint_builder_2d.cc:165-186, :307-316). A 400x400
  // 2D submap's matcher holds ~25 MB, so the default keeps ~1300 of them.
  int64_t matcher_cache_bytes = int64_t{32} << 30;
  // log_matches (pose_graph.lua:24): one line per accepted match and the score
  // histogram at every WhenDone, to the builder's log sink (metrics.h).
  bool log_matches = true;
};

// The per-submap matcher cache (DispatchScanMatcherConstruction,
// constraint_builder_2d.cc:165-186) under a device-memory budget: least
// recently used matchers are dropped once the cached ones hold more than
// `budget` bytes, and rebuilt from the submap on their next use (a 2D build is
// ~0.1 ms of device time). A matcher some batch still holds (a shared_ptr
// besides the cache's) is never dropped, so a batch's matchers stay valid;
// the builders cut a flush into sub-batches whose matchers fit the budget.
template <typename M>
class MatcherCache {
 public:
  explicit MatcherCache(int64_t budget) : budget_(budget) {}

  bool Contains(const SubmapId& id) const { return map_.count(id) != 0; }
  size_t size() const { return map_.size(); }
  int64_t bytes() const { return bytes_; }
  int64_t budget() const { return budget_; }
  bool bounded() const { return budget_ > 0; }

  // The cached matcher (now the most recent), or make() -> shared_ptr<M>
  // inserted with its device bytes (bytes_of(const M&)).
  template <typename Make, typename Bytes>
  std::shared_ptr<M> Get(const SubmapId& id, Make&& make, Bytes&& bytes_of) {
    auto it = map_.find(id);
    if (it != map_.end()) {
      lru_.splice(lru_.begin(), lru_, it->second.pos);
      return it->second.m;
    }
    std::shared_ptr<M> m = make();
    ++builds;
    const int64_t b = bytes_of(*m);
    lru_.push_front(id);
    map_.emplace(id, Entry{m, b, lru_.begin()});
    bytes_ += b;
    Trim();
    return m;
  }

  void Erase(const SubmapId& id) {
    auto it = map_.find(id);
    if (it == map_.end()) return;
    bytes_ -= it->second.bytes;
    lru_.erase(it->second.pos);
    map_.erase(it);
  }

  int64_t builds = 0, evictions = 0;

  // Drops least recently used matchers no batch holds until the cache is
  // within its budget (Get does this after every build).
  void Trim() {
    if (budget_ <= 0) return;
    for (auto p = lru_.end(); bytes_ > budget_ && p != lru_.begin();) {
      --p;
      auto it = map_.find(*p);
      if (it->second.m.use_count() > 1) continue;  // held by a batch
      bytes_ -= it->second.bytes;
      map_.erase(it);
      p = lru_.erase(p);
      ++evictions;
    }
  }

 private:
  struct Entry {
    std::shared_ptr<M> m;
    int64_t bytes;
    std::list<SubmapId>::iterator pos;
  };
  std::map<SubmapId, Entry> map_;
  std::list<SubmapId> lru_;  // most recent first
  int64_t bytes_ = 0;
  int64_t budget_;
};

// common/fixed_ratio_sampler.cc:32-39
class FixedRatioSampler {
 public:
  explicit FixedRatioSampler(double ratio) : ratio_(ratio) {}
  bool Pulse() {
    ++num_pulses_;
    if (static_cast<double>(num_samples_) / num_pulses_ < ratio_) {
      ++num_samples_;
      return true;
    }
    return false;
  }

 private:
  double ratio_;
  int64_t num_pulses_ = 0, num_samples_ = 0;
};

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_COMMON_H_
