// ConstraintBuilder2D drop-in over the batched C-ABI.
//
// Mirrors mapping/internal/constraints/constraint_builder_2d.{h,cc}: the
// public methods, the distance filter and per-submap FixedRatioSampler of
// MaybeAddConstraint (:77-112), MaybeAddGlobalConstraint (:114-137),
// NotifyEndOfNode (:139-151), WhenDone (:153-163) with results in submission
// order and failures dropped (:279-300), GetNumFinishedNodes (:302-305),
// DeleteScanMatcher (:307-316), the per-submap matcher cache
// (DispatchScanMatcherConstruction :165-186), the metrics (:46-53,
// RegisterMetrics :318-343: constraint counters, queue-length and matcher
// gauges, local and global score histograms), the score histogram and the
// log_matches lines (:239, :260-276, :289-293). Instead of one Task per pair on common::ThreadPool, pending pairs
// are searched as one GPU batch when a node ends (or when `flush_pairs` are
// pending). Accepted matches are then refined as one batch by the
// CeresScanMatcher2D restatement of ComputeConstraint (:245-249;
// csm_ceres2d_refine_batch, parity with Ceres unpinned) unless
// options.refine_with_ceres is off.
//
// Lifetimes: the Submap2DView and PointCloud passed to MaybeAdd* must stay
// valid (and unchanged) until the flush that searches the pair — the next
// NotifyEndOfNode that flushes, or WhenDone — as the reference's tasks read
// them until they run. Matchers are built from the view when the pair is
// enqueued (kStatic) or searched (kClaim, or after the budgeted matcher cache
// dropped the submap's matcher: options.matcher_cache_bytes, MatcherCache).
// DeleteScanMatcher drops the submap's pending pairs.
//
// Multi-GPU (set_communicator): every rank makes the same calls; a rank
// searches only the pairs of the submaps it owns (ShardOwner, Sharding::kStatic)
// or the chunks of each flush it claims (Sharding::kClaim) on its own device,
// and WhenDone gathers the accepted constraints to rank 0 in submission order
// (constraint_gather.h). Rank 0's callback gets the whole
// result, the other ranks' callbacks an empty one; the metric counters are
// summed over the ranks and last_error reduced over them at every WhenDone.
#ifndef CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_2D_H_
#define CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_2D_H_

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "constraint_builder_common.h"
#include "constraint_gather.h"
#include "metrics.h"
#include "scan_matching.h"

namespace cartographer_amd {

// What the builder reads of a Submap2D: its grid and ComputeSubmapPose(),
// i.e. Project2D(submap.local_pose()) (constraint_builder_2d.cc:55-57).
struct Submap2DView {
  Grid2DView grid;
  Rigid2d local_pose;
};

// PoseGraphInterface::Constraint (pose_graph_interface.h:36-53), 2D pose.
struct Constraint {
  SubmapId submap_id;
  NodeId node_id;
  Rigid2d relative_pose;  // submap <- node (Embed3D of this in the reference)
  double translation_weight = 0., rotation_weight = 0.;
  enum Tag { INTRA_SUBMAP, INTER_SUBMAP } tag = INTER_SUBMAP;
  float score = 0.f;
};

inline Rigid2d Compose(const Rigid2d& a, const Rigid2d& b) {
  const double c = std::cos(a.theta), s = std::sin(a.theta);
  return Rigid2d{c * b.x + (-s) * b.y + a.x, s * b.x + c * b.y + a.y, a.theta + b.theta};
}
inline Rigid2d Inverse(const Rigid2d& a) {
  const double c = std::cos(-a.theta), s = std::sin(-a.theta);
  return Rigid2d{-(c * a.x + (-s) * a.y), -(s * a.x + c * a.y), -a.theta};
}

class ConstraintBuilder2D {
 public:
  using Result = std::vector<Constraint>;

  explicit ConstraintBuilder2D(const ConstraintBuilderOptions& options,
                               csm_context* context = nullptr)
      : options_(options),
        context_(context ? context : ThreadContext()),
        matchers_(options.matcher_cache_bytes) {}

  ~ConstraintBuilder2D() {
    if (scans_) csm_scan_set_destroy(scans_);
  }

  // Shards the search over the ranks of `comm` (not owned; outlives the
  // builder). Call before the first MaybeAdd*. kClaim needs
  // csm_comm_claim_open on `comm`; builders that share a communicator in
  // kClaim mode need distinct `claim_namespace`s (their counters' keys).
  void set_communicator(csm_comm* comm, Sharding sharding = Sharding::kStatic,
                        int chunk_submaps = 4, int claim_namespace = 0) {
    comm_ = comm;
    sharding_ = sharding;
    chunk_submaps_ = chunk_submaps;
    claim_key_ = static_cast<int64_t>(claim_namespace) << 40;
  }

  void MaybeAddConstraint(const SubmapId& submap_id, const Submap2DView* submap,
                          const NodeId& node_id, const PointCloud* cloud,
                          const Rigid2d& initial_relative_pose) {
    if (std::hypot(initial_relative_pose.x, initial_relative_pose.y) >
        options_.max_constraint_distance)
      return;
    auto it = samplers_.emplace(submap_id, FixedRatioSampler(options_.sampling_ratio)).first;
    if (!it->second.Pulse()) return;
    Enqueue(submap_id, submap, node_id, cloud, false,
            Compose(submap->local_pose, initial_relative_pose));
  }

  void MaybeAddGlobalConstraint(const SubmapId& submap_id, const Submap2DView* submap,
                                const NodeId& node_id, const PointCloud* cloud) {
    Enqueue(submap_id, submap, node_id, cloud, true, Rigid2d::Identity());
  }

  void NotifyEndOfNode() {
    ++num_started_nodes_;
    if (static_cast<int>(pending_.size()) >= options_.flush_pairs) Flush();
  }

  void WhenDone(const std::function<void(const Result&)>& callback) {
    Flush();
    Result result;
    if (comm_ && csm_comm_size(comm_) > 1) {
      GatherToRoot(&result);
    } else {
      for (auto& c : constraints_)
        if (c) result.push_back(*c);
    }
    if (options_.log_matches) {  // RunWhenDoneCallback (:289-293)
      log_(std::to_string(constraints_.size()) + " computations resulted in " +
           std::to_string(result.size()) + " additional constraints.");
      log_("Score histogram:\n" + score_histogram_.ToString(10));
    }
    constraints_.clear();
    Metrics().queue_length->Set(constraints_.size());
    callback(result);
  }

  int GetNumFinishedNodes() const { return num_finished_nodes_; }

  // Also drops the submap's pairs still pending (they yield no constraint):
  // the reference's tasks would read the deleted matcher, and a pending pair
  // must not make the builder rebuild it from a submap the caller is trimming.
  void DeleteScanMatcher(const SubmapId& submap_id) {
    matchers_.Erase(submap_id);
    samplers_.erase(submap_id);
    Metrics().num_submap_scan_matchers->Set(matchers_.size());
    const size_t before = pending_.size();
    pending_.erase(std::remove_if(pending_.begin(), pending_.end(),
                                  [&](const Pending& p) {
                                    return !(p.submap_id < submap_id) &&
                                           !(submap_id < p.submap_id);
                                  }),
                   pending_.end());
    if (pending_.size() != before)
      std::fprintf(stderr,
                   "ConstraintBuilder2D: DeleteScanMatcher dropped %zu pending pairs of a "
                   "deleted submap\n",
                   before - pending_.size());
  }

  // kNumSubmapScanMatchersMetric, and the cache's device bytes and churn.
  int num_submap_scan_matchers() const { return static_cast<int>(matchers_.size()); }
  int64_t matcher_cache_bytes() const { return matchers_.bytes(); }
  int64_t matcher_builds() const { return matchers_.builds; }
  int64_t matcher_evictions() const { return matchers_.evictions; }

  // The metric families (constraint_builder_2d.cc:318-343): the same names
  // and labels. Until called, the metrics are Null ones (:46-53). Shared by
  // every ConstraintBuilder2D of the process, as the reference's statics.
  static void RegisterMetrics(metrics::FamilyFactory* factory) {
    MetricSet& m = Metrics();
    auto* counts = factory->NewCounterFamily("mapping_constraints_constraint_builder_2d_constraints",
                                             "Constraints computed");
    m.searched = counts->Add({{"search_region", "local"}, {"matcher", "searched"}});
    m.found = counts->Add({{"search_region", "local"}, {"matcher", "found"}});
    m.global_searched = counts->Add({{"search_region", "global"}, {"matcher", "searched"}});
    m.global_found = counts->Add({{"search_region", "global"}, {"matcher", "found"}});
    m.queue_length = factory->NewGaugeFamily("mapping_constraints_constraint_builder_2d_queue_length",
                                             "Queue length")->Add({});
    auto* scores = factory->NewHistogramFamily("mapping_constraints_constraint_builder_2d_scores",
                                               "Constraint scores built",
                                               metrics::Histogram::FixedWidth(0.05, 20));
    m.scores = scores->Add({{"search_region", "local"}});
    m.global_scores = scores->Add({{"search_region", "global"}});
    m.num_submap_scan_matchers =
        factory->NewGaugeFamily("mapping_constraints_constraint_builder_2d_num_submap_scan_matchers",
                                "Current number of constructed submap scan matchers")->Add({});
  }

  // score_histogram_ (:239): every accepted match's score, over the builder's life.
  const ScoreHistogram& score_histogram() const { return score_histogram_; }
  // Where the log_matches lines go (LOG(INFO) in the reference).
  void set_log_sink(LogSink sink) { log_ = std::move(sink); }

  // Counters of this builder (the metric counters above are process-wide).
  int64_t constraints_searched = 0, constraints_found = 0;
  int64_t global_constraints_searched = 0, global_constraints_found = 0;
  // Pairs skipped because the device search returned an error (not counted
  // as searched), and the last such status.
  int64_t constraints_failed = 0;
  // Sharding::kClaim: chunks this rank searched (not summed over ranks).
  int64_t chunks_claimed = 0;
  int last_error = CSM_OK;

 private:
  struct Pending {
    SubmapId submap_id;
    const Submap2DView* submap;
    NodeId node_id;
    const PointCloud* cloud;
    bool full;
    Rigid2d initial;
    size_t slot;
  };

  bool Claiming() const {
    return comm_ && csm_comm_size(comm_) > 1 && sharding_ == Sharding::kClaim;
  }
  bool Owned(const SubmapId& id) const {
    return !comm_ || csm_comm_size(comm_) <= 1 || sharding_ == Sharding::kClaim ||
           ShardOwner(id.trajectory_id, id.submap_index, csm_comm_size(comm_)) ==
               csm_comm_rank(comm_);
  }

  // DispatchScanMatcherConstruction (constraint_builder_2d.cc:165-186), through
  // the budgeted cache (a dropped matcher is rebuilt from the submap's grid).
  std::shared_ptr<FastCorrelativeScanMatcher2D> EnsureMatcher(const SubmapId& submap_id,
                                                              const Submap2DView* submap) {
    auto m = matchers_.Get(
        submap_id,
        [&] {
          return std::make_shared<FastCorrelativeScanMatcher2D>(
              submap->grid, options_.fast_correlative_scan_matcher_options, context_);
        },
        [](const FastCorrelativeScanMatcher2D& m) { return m.device_bytes(); });
    Metrics().num_submap_scan_matchers->Set(matchers_.size());
    return m;
  }

  // Rank 0 receives every rank's accepted constraints in slot order; the
  // metric deltas since the last WhenDone are summed over the ranks.
  void GatherToRoot(Result* result) {
    CheckSameSubmissions(comm_, static_cast<int64_t>(constraints_.size()));
    last_error = ReduceLastError(comm_, last_error);
    std::vector<ConstraintRecord> local;
    for (size_t slot = 0; slot < constraints_.size(); ++slot) {
      const Constraint* c = constraints_[slot].get();
      if (!c) continue;
      ConstraintRecord r{};
      r.slot = static_cast<int64_t>(slot);
      r.submap_trajectory = c->submap_id.trajectory_id;
      r.submap_index = c->submap_id.submap_index;
      r.node_trajectory = c->node_id.trajectory_id;
      r.node_index = c->node_id.node_index;
      r.x = c->relative_pose.x;
      r.y = c->relative_pose.y;
      r.theta = c->relative_pose.theta;
      r.score = c->score;
      r.tag = static_cast<int32_t>(c->tag);
      local.push_back(r);
    }
    const std::vector<ConstraintRecord> all = GatherConstraintRecords(comm_, local);
    int64_t d[5] = {constraints_searched - reduced_[0], constraints_found - reduced_[1],
                    global_constraints_searched - reduced_[2],
                    global_constraints_found - reduced_[3], constraints_failed - reduced_[4]};
    CommCheck(csm_comm_allreduce_i64(comm_, d, 5, CSM_REDUCE_SUM), "csm_comm_allreduce_i64");
    int64_t* counters[5] = {&constraints_searched, &constraints_found, &global_constraints_searched,
                            &global_constraints_found, &constraints_failed};
    for (int k = 0; k < 5; ++k) {
      reduced_[k] += d[k];
      *counters[k] = reduced_[k];
    }
    for (const ConstraintRecord& r : all) {
      Constraint c;
      c.submap_id = SubmapId{r.submap_trajectory, r.submap_index};
      c.node_id = NodeId{r.node_trajectory, r.node_index};
      c.relative_pose = Rigid2d{r.x, r.y, r.theta};
      c.translation_weight = options_.loop_closure_translation_weight;
      c.rotation_weight = options_.loop_closure_rotation_weight;
      c.tag = static_cast<Constraint::Tag>(r.tag);
      c.score = r.score;
      result->push_back(c);
    }
  }

  void Enqueue(const SubmapId& submap_id, const Submap2DView* submap, const NodeId& node_id,
               const PointCloud* cloud, bool full, const Rigid2d& initial) {
    constraints_.emplace_back();
    Metrics().queue_length->Set(constraints_.size());  // (:98, :123)
    if (!Owned(submap_id)) return;  // another rank searches it; the slot keeps submission order
    if (!Claiming()) EnsureMatcher(submap_id, submap);  // claimed chunks build theirs
    pending_.push_back(Pending{submap_id, submap, node_id, cloud, full, initial,
                               constraints_.size() - 1});
  }

  void Flush() {
    if (pending_.empty()) {
      num_finished_nodes_ = num_started_nodes_;
      return;
    }
    if (Claiming()) {
      const std::vector<std::vector<size_t>> chunks = ClaimChunks(pending_, chunk_submaps_);
      ForClaimedChunks(comm_, claim_key_++, chunks.size(), [&](size_t c) {
        ++chunks_claimed;
        Search(chunks[c]);
      });
    } else {
      std::vector<size_t> all(pending_.size());
      for (size_t i = 0; i < all.size(); ++i) all[i] = i;
      Search(all);
    }
    pending_.clear();
    num_finished_nodes_ = num_started_nodes_;
  }

  // Device index of every pending_[which_pending[k]]'s cloud in scans_, which
  // keeps node clouds resident across flushes: clouds not seen before (or a
  // node whose cloud changed) are appended in one upload.
  // A cached cloud is reused only if it is the same PointCloud with the same
  // size and content hash, so a caller refilling one PointCloud object for a
  // node is uploaded again (the Python mirror compares the points).
  static uint64_t CloudHash(const PointCloud& c) {
    uint64_t h = 1469598103934665603ull;  // FNV-1a over the float bytes
    const unsigned char* b = reinterpret_cast<const unsigned char*>(c.xyz.data());
    for (size_t i = 0, n = c.xyz.size() * sizeof(float); i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
  }
  std::vector<int32_t> ResidentScans(const std::vector<size_t>& which_pending) {
    std::map<const PointCloud*, uint64_t> hashes;
    auto hash_of = [&](const PointCloud* c) {
      auto it = hashes.find(c);
      if (it == hashes.end()) it = hashes.emplace(c, CloudHash(*c)).first;
      return it->second;
    };
    auto stale = [&](const CachedScan& c, const PointCloud* cloud) {
      return c.index == kUnset || c.cloud != cloud || c.size != cloud->size() ||
             c.hash != hash_of(cloud);
    };
    int64_t fresh_points = 0;
    for (size_t i : which_pending) {
      auto c = scan_cache_.find(pending_[i].node_id);
      if (c == scan_cache_.end() || stale(c->second, pending_[i].cloud))
        fresh_points += static_cast<int64_t>(pending_[i].cloud->size());
    }
    if (scans_ && cached_points_ + fresh_points > options_.scan_cache_points) {
      csm_scan_set_destroy(scans_);
      scans_ = nullptr;
      scan_cache_.clear();
      cached_points_ = 0;
    }
    if (!scans_) {
      const int64_t zero = 0;
      CheckOk(csm_scan_set_create(context_, nullptr, &zero, 0, &scans_), "csm_scan_set_create");
    }
    std::vector<float> xyz;
    std::vector<int64_t> offsets{0};
    std::vector<int32_t> index;  // >= 0: resident; < 0: -1 - (k-th cloud of this upload)
    std::vector<CachedScan*> fresh;
    for (size_t i : which_pending) {
      const Pending& p = pending_[i];
      CachedScan& c = scan_cache_[p.node_id];
      if (stale(c, p.cloud)) {
        c.cloud = p.cloud;
        c.size = p.cloud->size();
        c.hash = hash_of(p.cloud);
        c.index = -static_cast<int32_t>(offsets.size());
        fresh.push_back(&c);
        xyz.insert(xyz.end(), p.cloud->xyz.begin(), p.cloud->xyz.end());
        offsets.push_back(offsets.back() + static_cast<int64_t>(p.cloud->size()));
      }
      index.push_back(c.index);
    }
    if (offsets.size() > 1) {
      int32_t first = 0;
      CheckOk(csm_scan_set_append(scans_, xyz.data(), offsets.data(),
                                  static_cast<int32_t>(offsets.size() - 1), &first),
              "csm_scan_set_append");
      cached_points_ += offsets.back();
      for (int32_t& k : index)
        if (k < 0) k = first - 1 - k;
      for (CachedScan* c : fresh) c->index = first - 1 - c->index;
    }
    return index;
  }

  // Cuts pending_[which] into sub-batches whose matchers fit the matcher
  // cache's budget together (one batch when unbounded or when they fit),
  // whole submaps per sub-batch, and searches each.
  void Search(const std::vector<size_t>& which_pending) {
    std::vector<size_t> order(which_pending);
    if (matchers_.bounded())
      std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return pending_[a].submap_id < pending_[b].submap_id;
      });
    std::vector<size_t> part;
    Held held;
    int64_t held_bytes = 0;
    for (size_t i : order) {
      const Pending& p = pending_[i];
      if (!held.count(p.submap_id)) {
        auto m = EnsureMatcher(p.submap_id, p.submap);
        const int64_t b = m->device_bytes();
        if (!part.empty() && matchers_.bounded() && held_bytes + b > matchers_.budget()) {
          SearchBatch(part, held);
          part.clear();
          held.clear();
          held_bytes = 0;
          matchers_.Trim();  // the searched part's matchers are no longer held
        }
        held.emplace(p.submap_id, std::move(m));
        held_bytes += b;
      }
      part.push_back(i);
    }
    if (!part.empty()) SearchBatch(part, held);
    held.clear();
    matchers_.Trim();
  }

  using Held = std::map<SubmapId, std::shared_ptr<FastCorrelativeScanMatcher2D>>;

  // Searches (and refines) pending_[which] as one batch over `held`'s matchers.
  void SearchBatch(const std::vector<size_t>& which_pending, const Held& held) {
    const std::vector<int32_t> scan_index = ResidentScans(which_pending);
    std::vector<csm_fast2d*> handles;
    std::map<SubmapId, int> slot_of;
    std::vector<csm_pair2d> pairs;
    for (size_t k = 0; k < which_pending.size(); ++k) {
      const Pending& p = pending_[which_pending[k]];
      auto s = slot_of.find(p.submap_id);
      if (s == slot_of.end()) {
        s = slot_of.emplace(p.submap_id, static_cast<int>(handles.size())).first;
        handles.push_back(held.at(p.submap_id)->handle());
      }
      csm_pair2d q{};
      q.submap = s->second;
      q.scan = scan_index[k];
      q.full_submap = p.full ? 1 : 0;
      q.min_score = p.full ? options_.global_localization_min_score : options_.min_score;
      q.initial = csm_pose2d{p.initial.x, p.initial.y, p.initial.theta};
      pairs.push_back(q);
    }
    std::vector<csm_result2d> results(pairs.size());
    CheckOk(csm_fast2d_match_batch(context_, handles.data(), static_cast<int32_t>(handles.size()),
                                   scans_, pairs.data(), static_cast<int64_t>(pairs.size()),
                                   results.data()),
            "csm_fast2d_match_batch");
    // CeresScanMatcher2D::Match(pose.translation(), pose, cloud, grid) on the accepted ones.
    if (options_.refine_with_ceres) {
      std::vector<csm_refine2d> items;
      std::vector<size_t> which;
      for (size_t i = 0; i < pairs.size(); ++i)
        if (results[i].status == CSM_OK) {
          items.push_back(csm_refine2d{pairs[i].submap, pairs[i].scan, results[i].pose,
                                       results[i].pose.x, results[i].pose.y});
          which.push_back(i);
        }
      std::vector<csm_pose2d> out(items.size());
      if (!items.empty())
        CheckOk(csm_ceres2d_refine_batch(context_, handles.data(),
                                         static_cast<int32_t>(handles.size()), scans_,
                                         items.data(), static_cast<int64_t>(items.size()),
                                         &options_.ceres_scan_matcher_options, out.data(),
                                         nullptr),
                "csm_ceres2d_refine_batch");
      for (size_t k = 0; k < which.size(); ++k) results[which[k]].pose = out[k];
    }
    int64_t failed_this_flush = 0;
    for (size_t i = 0; i < which_pending.size(); ++i) {
      const Pending& p = pending_[which_pending[i]];
      if (results[i].status < 0) {
        // A pair the device path could not search (CSM_ERANGE: a cloud or
        // window past the kernels' limits) yields no
        // constraint; it is counted and reported, never fatal.
        ++constraints_failed;
        ++failed_this_flush;
        last_error = results[i].status;
        continue;
      }
      MetricSet& m = Metrics();
      (p.full ? global_constraints_searched : constraints_searched) += 1;
      (p.full ? m.global_searched : m.searched)->Increment();
      if (results[i].status != CSM_OK) continue;
      (p.full ? global_constraints_found : constraints_found) += 1;
      (p.full ? m.global_found : m.found)->Increment();
      (p.full ? m.global_scores : m.scores)->Observe(results[i].score);
      score_histogram_.Add(results[i].score);
      const Rigid2d pose{results[i].pose.x, results[i].pose.y, results[i].pose.theta};
      Constraint c;
      c.submap_id = p.submap_id;
      c.node_id = p.node_id;
      c.relative_pose = Compose(Inverse(p.submap->local_pose), pose);
      c.translation_weight = options_.loop_closure_translation_weight;
      c.rotation_weight = options_.loop_closure_rotation_weight;
      c.tag = Constraint::INTER_SUBMAP;
      c.score = results[i].score;
      constraints_[p.slot].reset(new Constraint(c));
      if (options_.log_matches) LogMatch(p, pose, results[i].score);
    }
    if (failed_this_flush)
      std::fprintf(stderr, "ConstraintBuilder2D: %lld of %zu pairs skipped (%s)\n",
                   static_cast<long long>(failed_this_flush), which_pending.size(),
                   csm_strerror(last_error));
  }

  // ComputeConstraint's log_matches line (:260-276); `pose` is the refined
  // pose_estimate (map <- node), p.initial the search start.
  void LogMatch(const Pending& p, const Rigid2d& pose, float score) {
    char buf[160];
    std::string info = "Node (" + std::to_string(p.node_id.trajectory_id) + ", " +
                       std::to_string(p.node_id.node_index) + ") with " +
                       std::to_string(p.cloud->size()) + " points on submap (" +
                       std::to_string(p.submap_id.trajectory_id) + ", " +
                       std::to_string(p.submap_id.submap_index) + ")";
    if (p.full) {
      info += " matches";
    } else {
      const Rigid2d d = Compose(Inverse(p.initial), pose);
      double a = d.theta;  // common::NormalizeAngleDifference
      while (a > M_PI) a -= 2. * M_PI;
      while (a < -M_PI) a += 2. * M_PI;
      std::snprintf(buf, sizeof(buf), " differs by translation %.2f rotation %.3f",
                    std::hypot(d.x, d.y), std::abs(a));
      info += buf;
    }
    std::snprintf(buf, sizeof(buf), " with score %.1f%%.", 100. * score);
    log_(info + buf);
  }

  // The process-wide metrics (the reference's static k*Metric pointers).
  struct MetricSet {
    metrics::Counter* searched = metrics::Counter::Null();
    metrics::Counter* found = metrics::Counter::Null();
    metrics::Counter* global_searched = metrics::Counter::Null();
    metrics::Counter* global_found = metrics::Counter::Null();
    metrics::Gauge* queue_length = metrics::Gauge::Null();
    metrics::Histogram* scores = metrics::Histogram::Null();
    metrics::Histogram* global_scores = metrics::Histogram::Null();
    metrics::Gauge* num_submap_scan_matchers = metrics::Gauge::Null();
  };
  static MetricSet& Metrics() {
    static MetricSet m;
    return m;
  }

  ConstraintBuilderOptions options_;
  csm_context* context_;
  ScoreHistogram score_histogram_;
  LogSink log_ = DefaultLogSink("ConstraintBuilder2D");
  MatcherCache<FastCorrelativeScanMatcher2D> matchers_;
  std::map<SubmapId, FixedRatioSampler> samplers_;
  std::vector<std::unique_ptr<Constraint>> constraints_;
  std::vector<Pending> pending_;
  struct CachedScan {
    const PointCloud* cloud = nullptr;
    size_t size = 0;
    uint64_t hash = 0;
    int32_t index = kUnset;
  };
  static constexpr int32_t kUnset = INT32_MIN;
  csm_scan_set* scans_ = nullptr;         // node clouds resident across flushes
  std::map<NodeId, CachedScan> scan_cache_;
  int64_t cached_points_ = 0;
  int num_started_nodes_ = 0, num_finished_nodes_ = 0;
  csm_comm* comm_ = nullptr;
  Sharding sharding_ = Sharding::kStatic;
  int chunk_submaps_ = 4;
  int64_t claim_key_ = 0;                  // kClaim: the next flush's counter
  int64_t reduced_[5] = {0, 0, 0, 0, 0};  // counter totals over ranks at the last WhenDone
};

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_2D_H_
