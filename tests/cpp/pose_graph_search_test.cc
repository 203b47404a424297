// Drives include/cartographer_amd/pose_graph_2d_search.h with a recording
// builder over a scripted scenario read from stdin, and prints the builder
// calls (tests/test_pose_graph_search.py compares them with the Python mirror).
//   S traj idx x y theta                      AddSubmap
//   N traj idx time x y theta fin k (t i)*k   AddNode (insertion submaps)
//   C ntraj nidx straj sidx                   HandleConstraints({constraint})
#include <cstdio>
#include <iostream>
#include <string>
#include <vector>

#include "cartographer_amd/pose_graph_2d_search.h"

using namespace cartographer_amd;

struct RecordingBuilder {
  void MaybeAddConstraint(const SubmapId& s, const Submap2DView*, const NodeId& n,
                          const PointCloud*, const Rigid2d& r) {
    std::printf("L %d %d %d %d %.9f %.9f %.9f\n", n.trajectory_id, n.node_index,
                s.trajectory_id, s.submap_index, r.x, r.y, r.theta);
  }
  void MaybeAddGlobalConstraint(const SubmapId& s, const Submap2DView*, const NodeId& n,
                                const PointCloud*) {
    std::printf("G %d %d %d %d\n", n.trajectory_id, n.node_index, s.trajectory_id,
                s.submap_index);
  }
  void NotifyEndOfNode() { std::printf("E\n"); }
};

int main(int argc, char** argv) {
  PoseGraphSearchOptions o;
  if (argc > 1) o.global_sampling_ratio = std::stod(argv[1]);
  if (argc > 2) o.global_constraint_search_after_n_seconds = std::stod(argv[2]);
  RecordingBuilder b;
  PoseGraph2DConstraintSearch<RecordingBuilder> g(o, &b);
  Submap2DView view;
  PointCloud cloud;
  std::string op;
  while (std::cin >> op) {
    if (op == "S") {
      SubmapId id;
      Rigid2d p;
      std::cin >> id.trajectory_id >> id.submap_index >> p.x >> p.y >> p.theta;
      g.AddSubmap(id, &view, p);
    } else if (op == "N") {
      NodeId id;
      double t;
      Rigid2d p;
      int fin, k;
      std::cin >> id.trajectory_id >> id.node_index >> t >> p.x >> p.y >> p.theta >> fin >> k;
      std::vector<SubmapId> ins(k);
      for (auto& s : ins) std::cin >> s.trajectory_id >> s.submap_index;
      g.AddNode(id, t, p, &cloud, ins, fin != 0);
    } else if (op == "C") {
      Constraint c;
      std::cin >> c.node_id.trajectory_id >> c.node_id.node_index >> c.submap_id.trajectory_id >>
          c.submap_id.submap_index;
      g.HandleConstraints({c});
    }
  }
  return 0;
}
