// The constraint-search half of PoseGraph2D: which (node, submap) pairs reach
// the ConstraintBuilder2D, as local (windowed Match) or global
// (MatchFullSubmap) searches, and in which order.
//
// Mirrors mapping/internal/2d/pose_graph_2d.cc:
//   ComputeConstraintsForNode  :304-402  (finished submaps in SubmapId order,
//                                        then, for a newly finished submap, the
//                                        older nodes in NodeId order)
//   ComputeConstraint          :260-302  (local when the trajectories are the
//                                        same or were connected less than
//                                        global_constraint_search_after_n_seconds
//                                        before the node; else global if the
//                                        node trajectory's sampler pulses)
//   GetLatestNodeTime          :404-416
//   UpdateTrajectoryConnectivity :418-425 (called for every found constraint,
//                                        :478-482)
// and mapping/internal/trajectory_connectivity_state.cc /
// connected_components.cc for the connection times.
//
// The optimization problem is not part of this: callers pass the global poses
// the matcher's initial estimates come from (the reference reads them from
// optimization_problem_, :293-297). The builder is a template parameter so a
// recording builder can stand in for ConstraintBuilder2D in tests.
#ifndef CARTOGRAPHER_AMD_POSE_GRAPH_2D_SEARCH_H_
#define CARTOGRAPHER_AMD_POSE_GRAPH_2D_SEARCH_H_

#include <algorithm>
#include <limits>
#include <map>
#include <set>
#include <utility>
#include <vector>

#include "constraint_builder_2d.h"

namespace cartographer_amd {

// proto::PoseGraphOptions fields read here (pose_graph.lua:79-80).
struct PoseGraphSearchOptions {
  double global_sampling_ratio = 0.003;
  double global_constraint_search_after_n_seconds = 10.;
};

// TrajectoryConnectivityState over ConnectedComponents (union-find without the
// reference's mutex: one thread drives the search here).
class TrajectoryConnectivityState {
 public:
  // Times are seconds on the universal time scale (common::Time's epoch is
  // 0). A pair never connected reads the epoch: last_connection_time_map_'s
  // value-initialised common::Time (trajectory_connectivity_state.cc:67-70).
  static constexpr double kEpoch = 0.;

  void Add(int trajectory_id) { forest_.emplace(trajectory_id, trajectory_id); }

  void Connect(int a, int b, double time) {
    if (TransitivelyConnected(a, b)) {
      double& t = last_connection_[std::minmax(a, b)];
      if (t < time) t = time;
    } else {
      for (int ia : GetComponent(a))
        for (int ib : GetComponent(b)) last_connection_[std::minmax(ia, ib)] = time;
    }
    forest_.emplace(a, a);
    forest_.emplace(b, b);
    const int ra = FindSet(a), rb = FindSet(b);
    forest_[ra] = rb;
  }

  bool TransitivelyConnected(int a, int b) {
    if (a == b) return true;
    if (!forest_.count(a) || !forest_.count(b)) return false;
    return FindSet(a) == FindSet(b);
  }

  // The epoch for pairs never connected (the map's default value).
  double LastConnectionTime(int a, int b) {
    const auto it = last_connection_.find(std::minmax(a, b));
    return it == last_connection_.end() ? kEpoch : it->second;
  }

 private:
  int FindSet(int id) {
    auto it = forest_.find(id);
    if (it->first != it->second) it->second = FindSet(it->second);
    return it->second;
  }
  std::vector<int> GetComponent(int id) {
    if (!forest_.count(id)) forest_.emplace(id, id);
    const int set = FindSet(id);
    std::vector<int> out;
    for (auto& e : forest_)
      if (FindSet(e.first) == set) out.push_back(e.first);
    return out;
  }

  std::map<int, int> forest_;
  std::map<std::pair<int, int>, double> last_connection_;
};

template <typename Builder = ConstraintBuilder2D>
class PoseGraph2DConstraintSearch {
 public:
  PoseGraph2DConstraintSearch(const PoseGraphSearchOptions& options, Builder* builder)
      : options_(options), builder_(builder) {}

  // A submap enters the graph (PoseGraph2D::InitializeGlobalSubmapPoses) with
  // its global pose; it is searched only once finished.
  void AddSubmap(const SubmapId& id, const Submap2DView* submap, const Rigid2d& global_pose) {
    AddTrajectoryIfNeeded(id.trajectory_id);
    SubmapData& d = submaps_[id];
    d.submap = submap;
    d.global_pose = global_pose;
  }

  // ComputeConstraintsForNode: the node was inserted into insertion_submaps
  // (front = the matching submap); newly_finished_submap says the front one
  // finished with it.
  void AddNode(const NodeId& node_id, double time, const Rigid2d& global_pose,
               const PointCloud* cloud, const std::vector<SubmapId>& insertion_submaps,
               bool newly_finished_submap) {
    AddTrajectoryIfNeeded(node_id.trajectory_id);
    nodes_[node_id] = NodeData{time, global_pose, cloud};
    for (const SubmapId& s : insertion_submaps) submaps_.at(s).node_ids.insert(node_id);
    std::vector<SubmapId> finished;
    for (auto& e : submaps_)
      if (e.second.finished) finished.push_back(e.first);
    std::set<NodeId> newly_finished_nodes;
    if (newly_finished_submap) {
      SubmapData& d = submaps_.at(insertion_submaps.front());
      d.finished = true;
      newly_finished_nodes = d.node_ids;
    }
    for (const SubmapId& s : finished) ComputeConstraint(node_id, s);
    if (newly_finished_submap) {
      const SubmapId& s = insertion_submaps.front();
      for (auto& e : nodes_)
        if (!newly_finished_nodes.count(e.first)) ComputeConstraint(e.first, s);
    }
    builder_->NotifyEndOfNode();
  }

  // PoseGraph2D::HandleWorkQueue (:478-482): found loop closures connect the
  // trajectories.
  void HandleConstraints(const std::vector<Constraint>& constraints) {
    for (const Constraint& c : constraints)
      connectivity_.Connect(c.node_id.trajectory_id, c.submap_id.trajectory_id,
                            GetLatestNodeTime(c.node_id, c.submap_id));
  }

  TrajectoryConnectivityState& connectivity() { return connectivity_; }
  int64_t local_searches = 0, global_searches = 0;

 private:
  struct SubmapData {
    const Submap2DView* submap = nullptr;
    Rigid2d global_pose;
    std::set<NodeId> node_ids;
    bool finished = false;
  };
  struct NodeData {
    double time = 0.;
    Rigid2d global_pose;
    const PointCloud* cloud = nullptr;
  };

  void AddTrajectoryIfNeeded(int trajectory_id) {
    if (samplers_.count(trajectory_id)) return;
    connectivity_.Add(trajectory_id);
    samplers_.emplace(trajectory_id, FixedRatioSampler(options_.global_sampling_ratio));
  }

  double GetLatestNodeTime(const NodeId& node_id, const SubmapId& submap_id) const {
    double time = nodes_.at(node_id).time;
    const SubmapData& d = submaps_.at(submap_id);
    if (!d.node_ids.empty()) time = std::max(time, nodes_.at(*d.node_ids.rbegin()).time);
    return time;
  }

  void ComputeConstraint(const NodeId& node_id, const SubmapId& submap_id) {
    const double node_time = GetLatestNodeTime(node_id, submap_id);
    const double last =
        connectivity_.LastConnectionTime(node_id.trajectory_id, submap_id.trajectory_id);
    const SubmapData& s = submaps_.at(submap_id);
    const NodeData& n = nodes_.at(node_id);
    if (node_id.trajectory_id == submap_id.trajectory_id ||
        node_time < last + options_.global_constraint_search_after_n_seconds) {
      ++local_searches;
      builder_->MaybeAddConstraint(submap_id, s.submap, node_id, n.cloud,
                                   Compose(Inverse(s.global_pose), n.global_pose));
    } else if (samplers_.at(node_id.trajectory_id).Pulse()) {
      ++global_searches;
      builder_->MaybeAddGlobalConstraint(submap_id, s.submap, node_id, n.cloud);
    }
  }

  PoseGraphSearchOptions options_;
  Builder* builder_;
  std::map<SubmapId, SubmapData> submaps_;
  std::map<NodeId, NodeData> nodes_;
  std::map<int, FixedRatioSampler> samplers_;
  TrajectoryConnectivityState connectivity_;
};

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_POSE_GRAPH_2D_SEARCH_H_
