// ConstraintBuilder3D drop-in over the batched 3D C-ABI.
//
// Mirrors mapping/internal/constraints/constraint_builder_3d.{h,cc}: the
// public methods; MaybeAddConstraint's distance filter on the global
// translations and its per-submap FixedRatioSampler (:79-114);
// MaybeAddGlobalConstraint with the poses reduced to their rotations
// (:116-142); NotifyEndOfNode (:144-156); WhenDone (:158-168) with results in
// submission order and failed searches dropped (RunWhenDoneCallback
// :307-333); GetNumFinishedNodes (:335-338); DeleteScanMatcher (:340-349); the
// per-submap matcher cache (DispatchScanMatcherConstruction :170-198, which
// reads the submap's high/low-resolution grids and rotational histogram); and
// the metrics (:46-59, counters and score lists). Pending pairs are searched
// as one GPU batch when a node ends (or once `flush_pairs` are pending)
// instead of one Task per pair. Accepted matches are then refined as one
// batch by the CeresScanMatcher3D restatement (:264-275;
// csm_ceres3d_refine_batch, parity with Ceres unpinned) unless
// options.refine_with_ceres is off.
//
// Lifetimes as ConstraintBuilder2D: a Submap3DView and a node's data must stay
// valid until the flush that searches the pair (matchers may be built, or
// rebuilt after the budgeted cache dropped them, at that flush).
//
// Multi-GPU (set_communicator), as ConstraintBuilder2D: every rank makes the
// same calls; a rank builds matchers for and searches only the submaps it
// owns (ShardOwner, Sharding::kStatic) or the chunks of each flush it claims
// (Sharding::kClaim) on its own device; WhenDone gathers the accepted
// constraints to rank 0 as ConstraintRecord3D in submission order
// (constraint_gather.h), sums the counters and reduces last_error over the
// ranks. The score lists (constraint_scores, global_constraint_scores,
// rotational_scores, low_resolution_scores) are appended at WhenDone from the
// delivered result, in submission order, so on rank 0 they cover every rank.
#ifndef CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_3D_H_
#define CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_3D_H_

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
#include "scan_matching_3d.h"

namespace cartographer_amd {

// What the builder reads of a Submap3D (submap_3d.h:57-73).
struct Submap3DView {
  HybridGridView high_resolution_hybrid_grid;
  HybridGridView low_resolution_hybrid_grid;
  std::vector<float> rotational_scan_matcher_histogram;
};

// PoseGraphInterface::Constraint (pose_graph_interface.h:36-53).
struct Constraint3D {
  SubmapId submap_id;
  NodeId node_id;
  Rigid3d relative_pose;  // zbar_ij: submap <- node
  double translation_weight = 0., rotation_weight = 0.;
  enum Tag { INTRA_SUBMAP, INTER_SUBMAP } tag = INTER_SUBMAP;
  float score = 0.f, rotational_score = 0.f, low_resolution_score = 0.f;
  bool global = false;  // found by MaybeAddGlobalConstraint (the metrics split)
};

class ConstraintBuilder3D {
 public:
  using Result = std::vector<Constraint3D>;

  explicit ConstraintBuilder3D(const ConstraintBuilderOptions& options,
                               csm_context* context = nullptr)
      : options_(options),
        context_(context ? context : ThreadContext()),
        matchers_(options.matcher_cache_bytes) {}

  // Shards the search over the ranks of `comm` (not owned; outlives the
  // builder). Call before the first MaybeAdd*. kClaim needs
  // csm_comm_claim_open on `comm`; builders that share a communicator in
  // kClaim mode need distinct `claim_namespace`s.
  void set_communicator(csm_comm* comm, Sharding sharding = Sharding::kStatic,
                        int chunk_submaps = 4, int claim_namespace = 1) {
    comm_ = comm;
    sharding_ = sharding;
    chunk_submaps_ = chunk_submaps;
    claim_key_ = static_cast<int64_t>(claim_namespace) << 40;
  }

  void MaybeAddConstraint(const SubmapId& submap_id, const Submap3DView* submap,
                          const NodeId& node_id, const TrajectoryNodeData3D* constant_data,
                          const Rigid3d& global_node_pose, const Rigid3d& global_submap_pose) {
    const double dx = global_node_pose.t[0] - global_submap_pose.t[0],
                 dy = global_node_pose.t[1] - global_submap_pose.t[1],
                 dz = global_node_pose.t[2] - global_submap_pose.t[2];
    if (std::sqrt(dx * dx + dy * dy + dz * dz) > options_.max_constraint_distance) return;
    auto it = samplers_.emplace(submap_id, FixedRatioSampler(options_.sampling_ratio)).first;
    if (!it->second.Pulse()) return;
    Enqueue(submap_id, submap, node_id, constant_data, false, global_node_pose,
            global_submap_pose);
  }

  void MaybeAddGlobalConstraint(const SubmapId& submap_id, const Submap3DView* submap,
                                const NodeId& node_id, const TrajectoryNodeData3D* constant_data,
                                const Quaterniond& global_node_rotation,
                                const Quaterniond& global_submap_rotation) {
    Enqueue(submap_id, submap, node_id, constant_data, true,
            Rigid3d::Rotation(global_node_rotation), Rigid3d::Rotation(global_submap_rotation));
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
    if (options_.log_matches) {  // RunWhenDoneCallback (:317-326)
      log_(std::to_string(constraints_.size()) + " computations resulted in " +
           std::to_string(result.size()) + " additional constraints.\nScore histogram:\n" +
           score_histogram_.ToString(10) + "\nRotational score histogram:\n" +
           rotational_score_histogram_.ToString(10) + "\nLow resolution score histogram:\n" +
           low_resolution_score_histogram_.ToString(10));
    }
    constraints_.clear();
    Metrics().queue_length->Set(constraints_.size());
    // The score lists (constraint_builder_3d.cc:46-59), submission order.
    for (const Constraint3D& c : result) {
      (c.global ? global_constraint_scores : constraint_scores).push_back(c.score);
      rotational_scores.push_back(c.rotational_score);
      low_resolution_scores.push_back(c.low_resolution_score);
    }
    callback(result);
  }

  int GetNumFinishedNodes() const { return num_finished_nodes_; }

  // Also drops the submap's pairs still pending (no constraint; see
  // ConstraintBuilder2D::DeleteScanMatcher).
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
                   "ConstraintBuilder3D: DeleteScanMatcher dropped %zu pending pairs of a "
                   "deleted submap\n",
                   before - pending_.size());
  }

  // The metric families (constraint_builder_3d.cc:351-386), same names and
  // labels; Null metrics until called (:46-59); process-wide like the
  // reference's statics.
  static void RegisterMetrics(metrics::FamilyFactory* factory) {
    MetricSet& m = Metrics();
    auto* counts = factory->NewCounterFamily("mapping_constraints_constraint_builder_3d_constraints",
                                             "Constraints computed");
    m.searched = counts->Add({{"search_region", "local"}, {"matcher", "searched"}});
    m.found = counts->Add({{"search_region", "local"}, {"matcher", "found"}});
    m.global_searched = counts->Add({{"search_region", "global"}, {"matcher", "searched"}});
    m.global_found = counts->Add({{"search_region", "global"}, {"matcher", "found"}});
    m.queue_length = factory->NewGaugeFamily("mapping_constraints_constraint_builder_3d_queue_length",
                                             "Queue length")->Add({});
    auto* scores = factory->NewHistogramFamily("mapping_constraints_constraint_builder_3d_scores",
                                               "Constraint scores built",
                                               metrics::Histogram::FixedWidth(0.05, 20));
    for (int g = 0; g < 2; ++g) {
      const std::string region = g ? "global" : "local";
      m.scores[g][0] = scores->Add({{"search_region", region}, {"kind", "score"}});
      m.scores[g][1] = scores->Add({{"search_region", region}, {"kind", "rotational_score"}});
      m.scores[g][2] = scores->Add({{"search_region", region}, {"kind", "low_resolution_score"}});
    }
    m.num_submap_scan_matchers =
        factory->NewGaugeFamily("mapping_constraints_constraint_builder_3d_num_submap_scan_matchers",
                                "Current number of constructed submap scan matchers")->Add({});
  }

  // score_histogram_, rotational_score_histogram_, low_resolution_score_histogram_ (:257-259).
  const ScoreHistogram& score_histogram() const { return score_histogram_; }
  const ScoreHistogram& rotational_score_histogram() const { return rotational_score_histogram_; }
  const ScoreHistogram& low_resolution_score_histogram() const {
    return low_resolution_score_histogram_;
  }
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
  std::vector<float> constraint_scores, global_constraint_scores;
  std::vector<float> rotational_scores, low_resolution_scores;
  int num_submap_scan_matchers() const { return static_cast<int>(matchers_.size()); }
  int64_t matcher_cache_bytes() const { return matchers_.bytes(); }
  int64_t matcher_builds() const { return matchers_.builds; }
  int64_t matcher_evictions() const { return matchers_.evictions; }

 private:
  // SubmapScanMatcher (constraint_builder_3d.h:117-123): device grids and the
  // matcher built from them.
  struct SubmapScanMatcher {
    std::unique_ptr<HybridGrid3D> high, low;
    std::unique_ptr<FastCorrelativeScanMatcher3D> matcher;
    int64_t device_bytes() const {
      return high->device_bytes() + low->device_bytes() + matcher->device_bytes();
    }
  };

  struct Pending {
    SubmapId submap_id;
    const Submap3DView* submap;
    NodeId node_id;
    const TrajectoryNodeData3D* data;
    bool full;
    Rigid3d node_pose, submap_pose;
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

  // Rank 0 receives every rank's accepted constraints in slot order; the
  // metric counter deltas since the last WhenDone are summed over the ranks.
  void GatherToRoot(Result* result) {
    CheckSameSubmissions(comm_, static_cast<int64_t>(constraints_.size()));
    last_error = ReduceLastError(comm_, last_error);
    std::vector<ConstraintRecord3D> local;
    for (size_t slot = 0; slot < constraints_.size(); ++slot) {
      const Constraint3D* c = constraints_[slot].get();
      if (!c) continue;
      ConstraintRecord3D r{};
      r.slot = static_cast<int64_t>(slot);
      r.submap_trajectory = c->submap_id.trajectory_id;
      r.submap_index = c->submap_id.submap_index;
      r.node_trajectory = c->node_id.trajectory_id;
      r.node_index = c->node_id.node_index;
      for (int a = 0; a < 3; ++a) r.t[a] = c->relative_pose.t[a];
      const Quaterniond& q = c->relative_pose.rotation;
      r.q[0] = q.w;
      r.q[1] = q.x;
      r.q[2] = q.y;
      r.q[3] = q.z;
      r.score = c->score;
      r.rotational_score = c->rotational_score;
      r.low_resolution_score = c->low_resolution_score;
      r.tag = static_cast<int32_t>(c->tag);
      r.global = c->global ? 1 : 0;
      local.push_back(r);
    }
    const std::vector<ConstraintRecord3D> all = GatherRecords(comm_, local);
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
    for (const ConstraintRecord3D& r : all) {
      Constraint3D c;
      c.submap_id = SubmapId{r.submap_trajectory, r.submap_index};
      c.node_id = NodeId{r.node_trajectory, r.node_index};
      for (int a = 0; a < 3; ++a) c.relative_pose.t[a] = r.t[a];
      c.relative_pose.rotation = Quaterniond{r.q[0], r.q[1], r.q[2], r.q[3]};
      c.translation_weight = options_.loop_closure_translation_weight;
      c.rotation_weight = options_.loop_closure_rotation_weight;
      c.tag = static_cast<Constraint3D::Tag>(r.tag);
      c.score = r.score;
      c.rotational_score = r.rotational_score;
      c.low_resolution_score = r.low_resolution_score;
      c.global = r.global != 0;
      result->push_back(c);
    }
  }

  void Enqueue(const SubmapId& submap_id, const Submap3DView* submap, const NodeId& node_id,
               const TrajectoryNodeData3D* data, bool full, const Rigid3d& node_pose,
               const Rigid3d& submap_pose) {
    constraints_.emplace_back();
    Metrics().queue_length->Set(constraints_.size());  // (:101, :127)
    if (!Owned(submap_id)) return;  // another rank searches it; the slot keeps submission order
    if (!Claiming()) EnsureMatcher(submap_id, submap);  // claimed chunks build theirs
    pending_.push_back(Pending{submap_id, submap, node_id, data, full, node_pose, submap_pose,
                               constraints_.size() - 1});
  }

  // DispatchScanMatcherConstruction (constraint_builder_3d.cc:170-198).
  // Through the budgeted cache (MatcherCache): a dropped matcher is rebuilt
  // from the submap's grids and histogram on its next use.
  std::shared_ptr<SubmapScanMatcher> EnsureMatcher(const SubmapId& submap_id,
                                                   const Submap3DView* submap) {
    auto held = matchers_.Get(
        submap_id,
        [&] {
          auto m = std::make_shared<SubmapScanMatcher>();
          m->high.reset(new HybridGrid3D(submap->high_resolution_hybrid_grid, context_));
          m->low.reset(new HybridGrid3D(submap->low_resolution_hybrid_grid, context_));
          m->matcher.reset(new FastCorrelativeScanMatcher3D(
              *m->high, m->low.get(), &submap->rotational_scan_matcher_histogram,
              options_.fast_correlative_scan_matcher_options_3d, context_));
          return m;
        },
        [](const SubmapScanMatcher& m) { return m.device_bytes(); });
    Metrics().num_submap_scan_matchers->Set(matchers_.size());
    return held;
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

  // Sub-batches whose matchers fit the cache budget together (as
  // ConstraintBuilder2D::Search), each searched and refined as one batch.
  void Search(const std::vector<size_t>& which_pending) {
    std::vector<size_t> order(which_pending);
    if (matchers_.bounded())
      std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) {
        return pending_[a].submap_id < pending_[b].submap_id;
      });
    std::vector<size_t> part;
    std::map<SubmapId, std::shared_ptr<SubmapScanMatcher>> held;
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

  // Searches (and refines) pending_[which] as one batch over `held`'s matchers.
  void SearchBatch(const std::vector<size_t>& which_pending,
                   const std::map<SubmapId, std::shared_ptr<SubmapScanMatcher>>& held) {
    std::vector<csm_fast3d*> handles;
    std::vector<const SubmapScanMatcher*> keep;
    std::map<SubmapId, int> slot_of;
    std::map<const TrajectoryNodeData3D*, int32_t> node_of;  // a node's data uploads once
    std::vector<csm_node3d> nodes;
    std::vector<csm_pair3d> pairs;
    for (size_t i : which_pending) {
      const Pending& p = pending_[i];
      auto s = slot_of.find(p.submap_id);
      if (s == slot_of.end()) {
        s = slot_of.emplace(p.submap_id, static_cast<int>(handles.size())).first;
        const SubmapScanMatcher* m = held.at(p.submap_id).get();
        handles.push_back(m->matcher->handle());
        keep.push_back(m);
      }
      auto n = node_of.find(p.data);
      if (n == node_of.end()) {
        n = node_of.emplace(p.data, static_cast<int32_t>(nodes.size())).first;
        nodes.push_back(p.data->ToC());
      }
      csm_pair3d q{};
      q.submap = s->second;
      q.node = n->second;
      q.full_submap = p.full ? 1 : 0;
      q.min_score = p.full ? options_.global_localization_min_score : options_.min_score;
      q.node_pose = p.node_pose.ToC();
      q.submap_pose = p.submap_pose.ToC();
      pairs.push_back(q);
    }
    std::vector<csm_result3d> results(pairs.size());
    CheckOk(csm_fast3d_match_batch(context_, handles.data(), static_cast<int32_t>(handles.size()),
                                   nodes.data(), static_cast<int32_t>(nodes.size()), pairs.data(),
                                   static_cast<int64_t>(pairs.size()), results.data()),
            "csm_fast3d_match_batch");
    if (options_.refine_with_ceres) {
      // ceres_scan_matcher_.Match(pose.translation(), pose, {high, low}) (:264-275).
      std::vector<const csm_hybrid_grid*> grids;
      for (const auto& m : keep) {
        grids.push_back(m->high->handle());
        grids.push_back(m->low->handle());
      }
      std::vector<csm_refine3d> items;
      std::vector<size_t> which;
      for (size_t i = 0; i < pairs.size(); ++i)
        if (results[i].status == CSM_OK) {
          csm_refine3d it{};
          it.high_grid = 2 * pairs[i].submap;
          it.low_grid = 2 * pairs[i].submap + 1;
          it.node = pairs[i].node;
          it.initial = results[i].pose;
          for (int a = 0; a < 3; ++a) it.target[a] = results[i].pose.t[a];
          items.push_back(it);
          which.push_back(i);
        }
      std::vector<csm_pose3d> out(items.size());
      if (!items.empty())
        CheckOk(csm_ceres3d_refine_batch(context_, grids.data(), static_cast<int32_t>(grids.size()),
                                         nodes.data(), static_cast<int32_t>(nodes.size()),
                                         items.data(), static_cast<int64_t>(items.size()),
                                         &options_.ceres_scan_matcher_options_3d, out.data(),
                                         nullptr),
                "csm_ceres3d_refine_batch");
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
      m.scores[p.full][0]->Observe(results[i].score);
      m.scores[p.full][1]->Observe(results[i].rotational_score);
      m.scores[p.full][2]->Observe(results[i].low_resolution_score);
      score_histogram_.Add(results[i].score);
      rotational_score_histogram_.Add(results[i].rotational_score);
      low_resolution_score_histogram_.Add(results[i].low_resolution_score);
      Constraint3D c;
      c.submap_id = p.submap_id;
      c.node_id = p.node_id;
      c.relative_pose = Rigid3d::FromC(results[i].pose);
      c.translation_weight = options_.loop_closure_translation_weight;
      c.rotation_weight = options_.loop_closure_rotation_weight;
      c.tag = Constraint3D::INTER_SUBMAP;
      c.score = results[i].score;
      c.rotational_score = results[i].rotational_score;
      c.low_resolution_score = results[i].low_resolution_score;
      c.global = p.full;
      constraints_[p.slot].reset(new Constraint3D(c));
      if (options_.log_matches) LogMatch(p, c.relative_pose, results[i].score);
    }
    if (failed_this_flush)
      std::fprintf(stderr, "ConstraintBuilder3D: %lld of %zu pairs skipped (%s)\n",
                   static_cast<long long>(failed_this_flush), which_pending.size(),
                   csm_strerror(last_error));
  }

  // ComputeConstraint's log_matches line (:284-303). difference =
  // global_node_pose^-1 * global_submap_pose * constraint_transform; its
  // angle is transform::GetAngle (2 atan2(|vec|, |w|)).
  void LogMatch(const Pending& p, const Rigid3d& constraint, float score) {
    char buf[160];
    std::string info = "Node (" + std::to_string(p.node_id.trajectory_id) + ", " +
                       std::to_string(p.node_id.node_index) + ") with " +
                       std::to_string(p.data->high_resolution_point_cloud.size()) +
                       " points on submap (" + std::to_string(p.submap_id.trajectory_id) + ", " +
                       std::to_string(p.submap_id.submap_index) + ")";
    if (p.full) {
      info += " matches";
    } else {
      const Rigid3d d = Mul(Mul(Inv(p.node_pose), p.submap_pose), constraint);
      const Quaterniond& q = d.rotation;
      const double angle = 2. * std::atan2(std::sqrt(q.x * q.x + q.y * q.y + q.z * q.z),
                                           std::abs(q.w));
      std::snprintf(buf, sizeof(buf), " differs by translation %.2f rotation %.3f",
                    std::sqrt(d.t[0] * d.t[0] + d.t[1] * d.t[1] + d.t[2] * d.t[2]), angle);
      info += buf;
    }
    std::snprintf(buf, sizeof(buf), " with score %.1f%%.", 100. * score);
    log_(info + buf);
  }
  // transform::Rigid3d operator* and inverse (rigid_transform.h:163-200) in double.
  static Quaterniond QMul(const Quaterniond& a, const Quaterniond& b) {
    return Quaterniond{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z,
                       a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
                       a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z,
                       a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
  }
  static void QRot(const Quaterniond& q, const double v[3], double out[3]) {
    const Quaterniond p{0., v[0], v[1], v[2]};
    const Quaterniond r = QMul(QMul(q, p), Quaterniond{q.w, -q.x, -q.y, -q.z});
    const double n = q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z;
    out[0] = r.x / n;
    out[1] = r.y / n;
    out[2] = r.z / n;
  }
  static Rigid3d Mul(const Rigid3d& a, const Rigid3d& b) {
    Rigid3d r;
    QRot(a.rotation, b.t, r.t);
    for (int k = 0; k < 3; ++k) r.t[k] += a.t[k];
    r.rotation = QMul(a.rotation, b.rotation);
    return r;
  }
  static Rigid3d Inv(const Rigid3d& a) {
    const Quaterniond& q = a.rotation;
    const double n = q.w * q.w + q.x * q.x + q.y * q.y + q.z * q.z;
    Rigid3d r;
    r.rotation = Quaterniond{q.w / n, -q.x / n, -q.y / n, -q.z / n};
    QRot(r.rotation, a.t, r.t);
    for (int k = 0; k < 3; ++k) r.t[k] = -r.t[k];
    return r;
  }

  struct MetricSet {  // the reference's static k*Metric pointers (:46-59)
    metrics::Counter* searched = metrics::Counter::Null();
    metrics::Counter* found = metrics::Counter::Null();
    metrics::Counter* global_searched = metrics::Counter::Null();
    metrics::Counter* global_found = metrics::Counter::Null();
    metrics::Gauge* queue_length = metrics::Gauge::Null();
    // [local, global][score, rotational_score, low_resolution_score]
    metrics::Histogram* scores[2][3] = {
        {metrics::Histogram::Null(), metrics::Histogram::Null(), metrics::Histogram::Null()},
        {metrics::Histogram::Null(), metrics::Histogram::Null(), metrics::Histogram::Null()}};
    metrics::Gauge* num_submap_scan_matchers = metrics::Gauge::Null();
  };
  static MetricSet& Metrics() {
    static MetricSet m;
    return m;
  }

  ConstraintBuilderOptions options_;
  csm_context* context_;
  ScoreHistogram score_histogram_, rotational_score_histogram_, low_resolution_score_histogram_;
  LogSink log_ = DefaultLogSink("ConstraintBuilder3D");
  MatcherCache<SubmapScanMatcher> matchers_;
  std::map<SubmapId, FixedRatioSampler> samplers_;
  std::vector<std::unique_ptr<Constraint3D>> constraints_;
  std::vector<Pending> pending_;
  int num_started_nodes_ = 0, num_finished_nodes_ = 0;
  csm_comm* comm_ = nullptr;
  Sharding sharding_ = Sharding::kStatic;
  int chunk_submaps_ = 4;
  int64_t claim_key_ = 0;                  // kClaim: the next flush's counter
  int64_t reduced_[5] = {0, 0, 0, 0, 0};  // counter totals over ranks at the last WhenDone
};

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_CONSTRAINT_BUILDER_3D_H_
