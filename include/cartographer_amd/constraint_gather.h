// Sharding of the constraint search across ranks (one process per GPU) and
// the hand-off of accepted constraints to rank 0.
//
// Every rank makes the same sequence of builder calls (the SLAM front end is
// replicated, or replays the same node stream), so every rank assigns the same
// submission slot to every pair; a rank searches only the pairs of the
// submaps it owns. At WhenDone the ranks' accepted constraints travel to rank
// 0 as fixed-width records over csm_comm_gather (RCCL over xGMI, or TCP between
// host processes) and rank 0 orders them by slot, which is the order the
// reference's WhenDone delivers (constraint_builder_2d.cc:279-300: results
// are appended in submission order, failures dropped).
#ifndef CARTOGRAPHER_AMD_CONSTRAINT_GATHER_H_
#define CARTOGRAPHER_AMD_CONSTRAINT_GATHER_H_

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "../csm_amd.h"

namespace cartographer_amd {

// One accepted constraint on the wire (64 bytes, no padding).
struct ConstraintRecord {
  int64_t slot;  // submission index of the pair
  int32_t submap_trajectory, submap_index, node_trajectory, node_index;
  double x, y, theta;  // relative pose, submap <- node
  float score;
  int32_t tag;
  int64_t reserved;  // zero
};
static_assert(sizeof(ConstraintRecord) == 64, "ConstraintRecord is a fixed wire format");

// One accepted 3D constraint on the wire (104 bytes, no padding): the 2D
// fields with a Rigid3d pose and FastCorrelativeScanMatcher3D::Result's three
// scores; `global` marks MaybeAddGlobalConstraint pairs (the metrics split).
struct ConstraintRecord3D {
  int64_t slot;
  int32_t submap_trajectory, submap_index, node_trajectory, node_index;
  double t[3], q[4];  // relative pose, submap <- node; q = (w, x, y, z)
  float score, rotational_score, low_resolution_score;
  int32_t tag;
  int32_t global;
  int32_t reserved;  // zero
};
static_assert(sizeof(ConstraintRecord3D) == 104, "ConstraintRecord3D is a fixed wire format");

// The rank that searches a submap's pairs: (trajectory_id * 0x9E3779B1 +
// submap_index) mod world_size, i.e. round robin over the submaps of one
// trajectory with a per-trajectory offset, so every rank gets a share of each
// region of the map. Every rank must make the identical sequence of builder
// calls (MaybeAdd*, NotifyEndOfNode, and with them the samplers' pulses):
// slots are assigned by that sequence, and WhenDone checks that every rank
// holds the same number of slots (CheckSameSubmissions).
inline int ShardOwner(int trajectory_id, int submap_index, int world_size) {
  const uint64_t h = static_cast<uint64_t>(static_cast<uint32_t>(trajectory_id)) * 0x9E3779B1u +
                     static_cast<uint32_t>(submap_index);
  return static_cast<int>(h % static_cast<uint64_t>(world_size));
}

inline void CommCheck(int code, const char* what) {
  if (code != CSM_OK) {
    std::fprintf(stderr, "F %s: %s (%d)\n", what, csm_strerror(code), code);
    std::abort();
  }
}

// How a sharded builder splits its pairs over the ranks.
//   kStatic: by submap (ShardOwner). A rank builds and keeps only the
//            matchers of its own submaps; no exchange until WhenDone.
//   kClaim:  dynamically, the reference's shared task queue
//            (common/thread_pool.cc:80-106) stretched over ranks: every flush's
//            pairs are cut into chunks of `chunk_submaps` submaps (submaps in
//            first-submission order) and idle ranks claim the next chunk with
//            csm_comm_fetch_add (the communicator needs csm_comm_claim_open).
//            A rank builds the matchers of the submaps it claims, on first
//            claim. Balances uneven pair costs; each rank may end up holding
//            any submap's matcher.
enum class Sharding { kStatic, kClaim };

// A flush's pending pairs (anything with a `submap_id`) grouped into claim
// chunks: indices into `pending`, chunk_submaps submaps per chunk.
template <typename Pending>
std::vector<std::vector<size_t>> ClaimChunks(const std::vector<Pending>& pending, int chunk_submaps) {
  std::vector<std::vector<size_t>> by_submap;
  std::map<decltype(pending[0].submap_id), size_t> index;
  for (size_t i = 0; i < pending.size(); ++i) {
    auto it = index.emplace(pending[i].submap_id, by_submap.size()).first;
    if (it->second == by_submap.size()) by_submap.emplace_back();
    by_submap[it->second].push_back(i);
  }
  const size_t per = static_cast<size_t>(chunk_submaps < 1 ? 1 : chunk_submaps);
  std::vector<std::vector<size_t>> chunks;
  for (size_t s = 0; s < by_submap.size(); ++s) {
    if (s % per == 0) chunks.emplace_back();
    chunks.back().insert(chunks.back().end(), by_submap[s].begin(), by_submap[s].end());
  }
  return chunks;
}

// Claims chunks of counter `key` until they run out, calling fn(chunk index)
// for each one this rank wins. Not collective; every rank must call it with
// the same key and count for the queue to drain.
template <typename Fn>
void ForClaimedChunks(csm_comm* comm, int64_t key, size_t num_chunks, Fn fn) {
  for (;;) {
    int64_t c = 0;
    CommCheck(csm_comm_fetch_add(comm, key, 1, &c), "csm_comm_fetch_add");
    if (c < 0 || static_cast<size_t>(c) >= num_chunks) return;
    fn(static_cast<size_t>(c));
  }
}

// Collective over `comm`: rank 0 returns every rank's records sorted by slot
// (slots are unique across ranks); the other ranks return an empty vector.
template <typename Record>
std::vector<Record> GatherRecords(csm_comm* comm, const std::vector<Record>& local) {
  int64_t total = 0;
  CommCheck(csm_comm_gather(comm, local.data(), static_cast<int64_t>(local.size() * sizeof(Record)),
                            &total),
            "csm_comm_gather");
  std::vector<Record> all;
  if (csm_comm_rank(comm) != 0) return all;
  all.resize(static_cast<size_t>(total) / sizeof(Record));
  std::vector<int64_t> sizes(static_cast<size_t>(csm_comm_size(comm)));
  CommCheck(csm_comm_gathered(comm, all.data(), total, sizes.data()), "csm_comm_gathered");
  std::stable_sort(all.begin(), all.end(),
                   [](const Record& a, const Record& b) { return a.slot < b.slot; });
  return all;
}

inline std::vector<ConstraintRecord> GatherConstraintRecords(
    csm_comm* comm, const std::vector<ConstraintRecord>& local) {
  return GatherRecords(comm, local);
}

// Collective: aborts unless every rank assigned the same number of slots
// since the last WhenDone (diverging submission streams would make rank 0
// mix or reorder constraints silently).
inline void CheckSameSubmissions(csm_comm* comm, int64_t slots) {
  int64_t v[2] = {slots, -slots};
  CommCheck(csm_comm_allreduce_i64(comm, v, 2, CSM_REDUCE_MAX), "csm_comm_allreduce_i64");
  if (v[0] != -v[1]) {
    std::fprintf(stderr, "F ranks submitted different pair sequences (%lld to %lld slots)\n",
                 static_cast<long long>(-v[1]), static_cast<long long>(v[0]));
    std::abort();
  }
}

// Collective: the builder's last error over the ranks (error codes are
// negative: the most negative wins; CSM_OK only if no rank saw an error).
inline int ReduceLastError(csm_comm* comm, int last_error) {
  int64_t v = -static_cast<int64_t>(last_error);
  CommCheck(csm_comm_allreduce_i64(comm, &v, 1, CSM_REDUCE_MAX), "csm_comm_allreduce_i64");
  return static_cast<int>(-v);
}

}  // namespace cartographer_amd

#endif  // CARTOGRAPHER_AMD_CONSTRAINT_GATHER_H_
