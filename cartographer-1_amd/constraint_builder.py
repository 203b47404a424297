"""ConstraintBuilder2D — the caller of the scan-matching hot path, over the
batched C-ABI (Python mirror of ``include/cartographer_amd/constraint_builder_2d.h``).

Follows reference ``mapping/internal/constraints/constraint_builder_2d.cc``:

* ``MaybeAddConstraint`` (:77-112): drop pairs farther than
  ``max_constraint_distance``, then one ``FixedRatioSampler`` per submap
  (``common/fixed_ratio_sampler.cc:32-39``) decides; the search starts at
  ``ComputeSubmapPose(submap) * initial_relative_pose`` (:195-197).
* ``MaybeAddGlobalConstraint`` (:114-137): ``MatchFullSubmap`` with
  ``global_localization_min_score`` (:208-222).
* ``NotifyEndOfNode`` (:139-151) / ``GetNumFinishedNodes`` (:302-305): a node
  is finished once its pairs have been searched.
* ``WhenDone`` (:153-163, ``RunWhenDoneCallback`` :279-300): constraints in
  submission order, failed searches dropped.
* ``DeleteScanMatcher`` (:307-316) and the per-submap matcher cache
  (``DispatchScanMatcherConstruction`` :165-186).
* Constraint pose ``ComputeSubmapPose(submap).inverse() * pose_estimate``
  (:251-252), tagged INTER_SUBMAP with the loop-closure weights (:253-257).

Instead of one ``common::Task`` per pair, the pending pairs are searched as one
GPU batch (``match_batch``) when a node ends, or once ``flush_pairs`` pairs are
pending. Accepted matches are then refined as one batch with the
CeresScanMatcher2D restatement (:245-249; ``ceres_refine_batch``, parity with
Ceres unpinned) unless ``refine_with_ceres`` is off.
"""

from __future__ import annotations

import logging
import math
import sys
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np

from . import (CSM_OK, strerror, CeresOptions2D, CeresOptions3D, Context, FastCorrelativeScanMatcher2D,
               FastCorrelativeScanMatcher3D, ceres_refine_batch, ceres_refine_batch_3d,
               FastCorrelativeScanMatcherOptions2D, FastCorrelativeScanMatcherOptions3D,
               HybridGrid, NodeData3D, ProbabilityGrid, ScanSet, _f32_points, default_context,
               make_pairs, make_pairs_3d, match_batch, match_batch_3d)
from . import metrics as _metrics

_LOG = logging.getLogger("cartographer_amd.constraint_builder")


def _normalize_angle_difference(a: float) -> float:
    """common::NormalizeAngleDifference (common/math.h)."""
    while a > math.pi:
        a -= 2.0 * math.pi
    while a < -math.pi:
        a += 2.0 * math.pi
    return a


def _quat_mul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return (aw * bw - ax * bx - ay * by - az * bz, aw * bx + ax * bw + ay * bz - az * by,
            aw * by + ay * bw + az * bx - ax * bz, aw * bz + az * bw + ax * by - ay * bx)


def _quat_rotate(q, v):
    n = sum(c * c for c in q)
    r = _quat_mul(_quat_mul(q, (0.0,) + tuple(v)), (q[0], -q[1], -q[2], -q[3]))
    return tuple(c / n for c in r[1:])


def rigid3d_compose(a, b):
    """transform::Rigid3d operator* on ((t), (w, x, y, z))."""
    t = _quat_rotate(a[1], b[0])
    return (tuple(t[k] + a[0][k] for k in range(3)), _quat_mul(a[1], b[1]))


def rigid3d_inverse(a):
    q = a[1]
    n = sum(c * c for c in q)
    qi = (q[0] / n, -q[1] / n, -q[2] / n, -q[3] / n)
    t = _quat_rotate(qi, a[0])
    return (tuple(-c for c in t), qi)


class _BuilderMetrics:
    """The process-wide metrics of one builder kind (the reference's static
    k*Metric pointers, constraint_builder_2d.cc:46-53 / _3d.cc:46-59): Null
    until RegisterMetrics."""

    def __init__(self, three_d: bool):
        C, G, H = _metrics.Counter.Null(), _metrics.Gauge.Null(), _metrics.Histogram.Null()
        self.searched = self.found = self.global_searched = self.global_found = C
        self.queue_length = self.num_submap_scan_matchers = G
        # [local, global] x [score] (2D) or [score, rotational, low resolution] (3D)
        self.scores = [[H] * (3 if three_d else 1) for _ in range(2)]

    def register(self, factory, dim: str):
        base = f"mapping_constraints_constraint_builder_{dim}"
        counts = factory.NewCounterFamily(f"{base}_constraints", "Constraints computed")
        self.searched = counts.Add({"search_region": "local", "matcher": "searched"})
        self.found = counts.Add({"search_region": "local", "matcher": "found"})
        self.global_searched = counts.Add({"search_region": "global", "matcher": "searched"})
        self.global_found = counts.Add({"search_region": "global", "matcher": "found"})
        self.queue_length = factory.NewGaugeFamily(f"{base}_queue_length", "Queue length").Add({})
        scores = factory.NewHistogramFamily(f"{base}_scores", "Constraint scores built",
                                            _metrics.Histogram.FixedWidth(0.05, 20))
        for g, region in enumerate(("local", "global")):
            if dim == "2d":
                self.scores[g] = [scores.Add({"search_region": region})]
            else:
                self.scores[g] = [scores.Add({"search_region": region, "kind": k})
                                  for k in ("score", "rotational_score", "low_resolution_score")]
        self.num_submap_scan_matchers = factory.NewGaugeFamily(
            f"{base}_num_submap_scan_matchers",
            "Current number of constructed submap scan matchers").Add({})


def rigid2d_compose(a, b):
    """transform::Rigid2d operator* (rigid_transform.h:90-96)."""
    c, s = math.cos(a[2]), math.sin(a[2])
    return (c * b[0] - s * b[1] + a[0], s * b[0] + c * b[1] + a[1], a[2] + b[2])


def rigid2d_inverse(a):
    """transform::Rigid2d::inverse (rigid_transform.h:74-78)."""
    c, s = math.cos(-a[2]), math.sin(-a[2])
    return (-(c * a[0] - s * a[1]), -(s * a[0] + c * a[1]), -a[2])


class FixedRatioSampler:
    """common/fixed_ratio_sampler.cc:32-39."""

    def __init__(self, ratio: float):
        if not (0.0 <= ratio <= 1.0):  # fixed_ratio_sampler.cc:25-28
            raise ValueError("ratio must be within [0, 1]")
        self.ratio = ratio
        self.num_pulses = 0
        self.num_samples = 0

    def Pulse(self) -> bool:
        self.num_pulses += 1
        if self.num_samples / self.num_pulses < self.ratio:
            self.num_samples += 1
            return True
        return False


class _MatcherCache:
    """The per-submap matcher cache (DispatchScanMatcherConstruction,
    constraint_builder_2d.cc:165-186) under a device-memory budget: once the
    cached matchers hold more than ``budget`` bytes the least recently used
    ones that no batch holds (``pinned``) are closed; a dropped matcher is
    rebuilt from its submap on its next use. Mirrors
    include/cartographer_amd/constraint_builder_common.h MatcherCache."""

    def __init__(self, budget: int):
        from collections import OrderedDict
        self.budget = int(budget)
        self._entries = OrderedDict()  # key -> (matcher, bytes), most recent last
        self.bytes = 0
        self.builds = 0
        self.evictions = 0
        self.pinned = set()

    def __len__(self):
        return len(self._entries)

    def __contains__(self, key):
        return key in self._entries

    def get(self, key, make, bytes_of):
        e = self._entries.get(key)
        if e is not None:
            self._entries.move_to_end(key)
            return e[0]
        m = make()
        b = int(bytes_of(m))
        self._entries[key] = (m, b)
        self.bytes += b
        self.builds += 1
        self.pinned.add(key)  # the caller holds it until it unpins
        self.trim()
        return m

    def pop(self, key, close):
        e = self._entries.pop(key, None)
        if e is not None:
            self.bytes -= e[1]
            close(e[0])

    def trim(self, close=None):
        if self.budget <= 0:
            return
        for key in list(self._entries):
            if self.bytes <= self.budget:
                break
            if key in self.pinned:
                continue
            m, b = self._entries.pop(key)
            self.bytes -= b
            self.evictions += 1
            (close or self._close)(m)

    @staticmethod
    def _close(m):
        for obj in (m if isinstance(m, tuple) else (m,))[::-1]:
            obj.close()

    def values(self):
        return [e[0] for e in self._entries.values()]


def _budget_parts(pending, key_of, cache: _MatcherCache, make, bytes_of):
    """Cuts a flush's pending pairs into parts whose matchers fit the cache's
    budget together (whole submaps per part; one part when unbounded or when
    they fit). Yields (part, {key: matcher}); the part's matchers stay pinned
    until the next part starts."""
    order = list(pending)
    if cache.budget > 0:
        order.sort(key=key_of)  # stable: submission order within a submap
    part, held, held_bytes = [], {}, 0
    try:
        for p in order:
            k = key_of(p)
            if k not in held:
                m = cache.get(k, lambda: make(p), bytes_of)
                b = int(bytes_of(m))
                if part and cache.budget > 0 and held_bytes + b > cache.budget:
                    yield part, held
                    cache.pinned = {k}
                    part, held, held_bytes = [], {}, 0
                    cache.trim()
                cache.pinned.add(k)
                held[k] = m
                held_bytes += b
            part.append(p)
        if part:
            yield part, held
    finally:
        # Also when a part's search raises (the generator is then closed):
        # no matcher stays pinned, so the budget keeps working.
        cache.pinned = set()
        cache.trim()


@dataclass
class Submap2D:
    """What the builder reads of a Submap2D: its grid and local pose
    (ComputeSubmapPose = Project2D(local_pose), constraint_builder_2d.cc:55-57)."""
    grid: ProbabilityGrid
    local_pose: Tuple[float, float, float] = (0.0, 0.0, 0.0)


@dataclass
class ConstraintBuilderOptions:
    """proto::ConstraintBuilderOptions (constraint_builder_options.proto:24-59);
    defaults from configuration_files/pose_graph.lua:17-29."""
    sampling_ratio: float = 0.3
    max_constraint_distance: float = 15.0
    min_score: float = 0.55
    global_localization_min_score: float = 0.6
    loop_closure_translation_weight: float = 1.1e4
    loop_closure_rotation_weight: float = 1e5
    fast_correlative_scan_matcher_options: FastCorrelativeScanMatcherOptions2D = field(
        default_factory=FastCorrelativeScanMatcherOptions2D)
    fast_correlative_scan_matcher_options_3d: FastCorrelativeScanMatcherOptions3D = field(
        default_factory=FastCorrelativeScanMatcherOptions3D)
    flush_pairs: int = 0  # 0: search each node's pairs when the node ends
    # Node clouds stay on the device across flushes; past this many resident
    # points the builder starts a new set (as the C++ header's option).
    scan_cache_points: int = 1 << 25
    # Device bytes the per-submap matcher cache may hold (0 = unbounded, the
    # reference's behaviour); least recently used matchers are dropped and
    # rebuilt on their next use (_MatcherCache, as the C++ MatcherCache).
    matcher_cache_bytes: int = 32 << 30
    # ceres_scan_matcher (pose_graph.lua:30-39): every accepted 2D match is
    # refined with CeresScanMatcher2D (constraint_builder_2d.cc:245-249).
    ceres_scan_matcher_options: CeresOptions2D = field(default_factory=CeresOptions2D.make)
    # ceres_scan_matcher_3d (pose_graph.lua:49-60), ConstraintBuilder3D (:264-275).
    ceres_scan_matcher_options_3d: CeresOptions3D = field(default_factory=CeresOptions3D.make)
    refine_with_ceres: bool = True
    # log_matches (pose_graph.lua:24): a line per accepted match and the score
    # histogram at every WhenDone, to the builder's log_sink (default: the
    # logging module at INFO, logger "cartographer_amd.constraint_builder").
    log_matches: bool = True


@dataclass
class Constraint:
    """PoseGraphInterface::Constraint (pose_graph_interface.h:36-53), 2D pose."""
    submap_id: Tuple[int, int]
    node_id: Tuple[int, int]
    relative_pose: Tuple[float, float, float]
    translation_weight: float
    rotation_weight: float
    tag: str = "INTER_SUBMAP"
    score: float = 0.0


@dataclass
class _Pending:
    submap_id: Tuple[int, int]
    submap: Submap2D
    node_id: Tuple[int, int]
    cloud: np.ndarray
    full: bool
    initial: Tuple[float, float, float]
    slot: int


class ConstraintBuilder2D:
    _metrics = _BuilderMetrics(False)

    @classmethod
    def RegisterMetrics(cls, factory):
        """The metric families of constraint_builder_2d.cc:318-343 (same names
        and labels), shared by every ConstraintBuilder2D of the process."""
        cls._metrics.register(factory, "2d")

    def __init__(self, options: ConstraintBuilderOptions, context: Optional[Context] = None):
        self.options = options
        self.score_histogram = _metrics.ScoreHistogram()  # score_histogram_ (:239)
        self.log_sink = _LOG.info  # where the log_matches lines go (LOG(INFO))
        self.context = context or default_context()
        self._matchers = _MatcherCache(options.matcher_cache_bytes)
        self._samplers: Dict[Tuple[int, int], FixedRatioSampler] = {}
        self._constraints: List[Optional[Constraint]] = []
        self._pending: List[_Pending] = []
        self._scans: Optional[ScanSet] = None  # node clouds resident across flushes
        self._scan_cache: Dict[Tuple[int, int], tuple] = {}  # node -> (cloud, index, points)
        self._started_nodes = 0
        self._finished_nodes = 0
        # Metrics (constraint_builder_2d.cc:46-53).
        self.constraints_searched = 0
        self.constraints_found = 0
        self.global_constraints_searched = 0
        self.global_constraints_found = 0
        self.constraints_failed = 0  # pairs skipped on a device error status
        self.last_error = CSM_OK
        self.constraint_scores: List[float] = []
        self.global_constraint_scores: List[float] = []

    # -- public interface (constraint_builder_2d.h:63-110) ------------------
    def MaybeAddConstraint(self, submap_id, submap: Submap2D, node_id, cloud,
                           initial_relative_pose):
        if math.hypot(initial_relative_pose[0], initial_relative_pose[1]) > \
                self.options.max_constraint_distance:
            return
        sampler = self._samplers.setdefault(tuple(submap_id),
                                            FixedRatioSampler(self.options.sampling_ratio))
        if not sampler.Pulse():
            return
        self._enqueue(submap_id, submap, node_id, cloud, False,
                      rigid2d_compose(submap.local_pose, initial_relative_pose))

    def MaybeAddGlobalConstraint(self, submap_id, submap: Submap2D, node_id, cloud):
        self._enqueue(submap_id, submap, node_id, cloud, True, (0.0, 0.0, 0.0))

    def NotifyEndOfNode(self):
        self._started_nodes += 1
        if len(self._pending) >= self.options.flush_pairs:
            self._flush()

    def WhenDone(self, callback: Callable[[List[Constraint]], None]):
        self._flush()
        result = [c for c in self._constraints if c is not None]
        if self.options.log_matches:  # RunWhenDoneCallback (:289-293)
            self.log_sink(f"{len(self._constraints)} computations resulted in {len(result)} "
                          "additional constraints.")
            self.log_sink("Score histogram:\n" + self.score_histogram.ToString(10))
        self._constraints = []
        self._metrics.queue_length.Set(len(self._constraints))
        callback(result)

    def GetNumFinishedNodes(self) -> int:
        return self._finished_nodes

    def DeleteScanMatcher(self, submap_id):
        """Also drops the submap's pending pairs (no constraint), as the C++
        header does."""
        key = tuple(submap_id)
        self._matchers.pop(key, lambda m: m.close())
        self._metrics.num_submap_scan_matchers.Set(len(self._matchers))
        self._samplers.pop(key, None)
        before = len(self._pending)
        self._pending = [p for p in self._pending if p.submap_id != key]
        if len(self._pending) != before:
            print(f"ConstraintBuilder2D: DeleteScanMatcher dropped {before - len(self._pending)} "
                  "pending pairs of a deleted submap", file=sys.stderr)

    @property
    def num_submap_scan_matchers(self) -> int:  # kNumSubmapScanMatchersMetric
        return len(self._matchers)

    @property
    def matcher_cache(self) -> _MatcherCache:
        return self._matchers

    # -- internals ----------------------------------------------------------
    def _make_matcher(self, p):
        return FastCorrelativeScanMatcher2D(p.submap.grid,
                                            self.options.fast_correlative_scan_matcher_options,
                                            self.context)

    def _resident_scans(self) -> ScanSet:
        """The node clouds' device set, kept across flushes (TrajectoryNode
        clouds are immutable, so each node's cloud is uploaded once); a new
        set is started past options.scan_cache_points resident points."""
        if self._scans is not None and \
                int(self._scans.offsets[-1]) > self.options.scan_cache_points:
            self._drop_scans()
        if self._scans is None:
            self._scans = ScanSet([], self.context)
        return self._scans

    def _drop_scans(self):
        if self._scans is not None:
            self._scans.close()
        self._scans, self._scan_cache = None, {}

    def _scan_indices(self, pending, scans: ScanSet) -> List[int]:
        """Scan index of each pending pair's cloud; a node's cloud is reused
        when it is the same points (compared, so callers may pass a fresh
        array each time), appended otherwise."""
        fresh, fresh_keys, index, seen = [], [], [], {}
        for p in pending:
            c = self._scan_cache.get(p.node_id)
            if c is None or (c[0] is not p.cloud and (p.node_id, id(p.cloud)) not in seen):
                pts = _f32_points(p.cloud)
                seen[(p.node_id, id(p.cloud))] = True
                if c is None or not np.array_equal(c[2], pts):
                    c = (p.cloud, -1 - len(fresh), pts)
                    fresh.append(pts)
                    fresh_keys.append(p.node_id)
                else:
                    c = (p.cloud, c[1], c[2])
                self._scan_cache[p.node_id] = c
            index.append(c[1])
        if fresh:
            first = scans.append(fresh)
            index = [first - 1 - k if k < 0 else k for k in index]
            for key in fresh_keys:
                cloud, k, pts = self._scan_cache[key]
                if k < 0:
                    self._scan_cache[key] = (cloud, first - 1 - k, pts)
        return index

    def _enqueue(self, submap_id, submap, node_id, cloud, full, initial):
        key = tuple(submap_id)
        self._constraints.append(None)
        self._metrics.queue_length.Set(len(self._constraints))  # (:98, :123)
        p = _Pending(key, submap, tuple(node_id), cloud, full, tuple(initial),
                     len(self._constraints) - 1)
        # DispatchScanMatcherConstruction at enqueue (:165-186), via the cache.
        self._matchers.get(key, lambda: self._make_matcher(p), lambda m: m.device_bytes())
        self._matchers.pinned.discard(key)
        self._matchers.trim()
        self._metrics.num_submap_scan_matchers.Set(len(self._matchers))
        self._pending.append(p)

    def _flush(self):
        pending, self._pending = self._pending, []
        if pending:
            for part, held in _budget_parts(pending, lambda p: p.submap_id, self._matchers,
                                            self._make_matcher, lambda m: m.device_bytes()):
                self._search(part, held)
        self._finished_nodes = self._started_nodes

    def _search(self, pending, held):
        """One batch (and its Ceres refinement) over the matchers in ``held``."""
        if pending:
            matchers, slot_of = [], {}
            submap_idx = []
            for p in pending:
                if p.submap_id not in slot_of:
                    slot_of[p.submap_id] = len(matchers)
                    matchers.append(held[p.submap_id])
                submap_idx.append(slot_of[p.submap_id])
            scans = self._resident_scans()
            scan_idx = self._scan_indices(pending, scans)
            pairs = make_pairs(submap_idx, scan_idx, 0.0, full_submap=True)
            for i, p in enumerate(pending):
                pairs[i]["full_submap"] = 1 if p.full else 0
                pairs[i]["min_score"] = (self.options.global_localization_min_score if p.full
                                         else self.options.min_score)
                pairs[i]["x"], pairs[i]["y"], pairs[i]["theta"] = p.initial
            try:
                results = match_batch(matchers, scans, pairs, self.context)
                refined = {}
                ok = [i for i, r in enumerate(results) if int(r["status"]) == CSM_OK]
                if self.options.refine_with_ceres and ok:
                    # ceres_scan_matcher_.Match(pose.translation(), pose, cloud, grid)
                    init = [(float(results[i]["x"]), float(results[i]["y"]),
                             float(results[i]["theta"])) for i in ok]
                    poses, _ = ceres_refine_batch(
                        matchers, scans, [submap_idx[i] for i in ok], [scan_idx[i] for i in ok],
                        init, [q[:2] for q in init], self.options.ceres_scan_matcher_options,
                        self.context)
                    refined = {i: tuple(float(v) for v in poses[k]) for k, i in enumerate(ok)}
            except BaseException:
                self._drop_scans()
                raise
            failed = 0
            for i, (p, r) in enumerate(zip(pending, results)):
                if int(r["status"]) < 0:
                    # Not searchable on the device (CSM_ERANGE):
                    # no constraint, counted, never fatal (as the C++ header).
                    self.constraints_failed += 1
                    self.last_error = int(r["status"])
                    failed += 1
                    continue
                m = self._metrics
                if p.full:
                    self.global_constraints_searched += 1
                    m.global_searched.Increment()
                else:
                    self.constraints_searched += 1
                    m.searched.Increment()
                if int(r["status"]) != CSM_OK:
                    continue
                score = float(r["score"])
                if p.full:
                    self.global_constraints_found += 1
                    self.global_constraint_scores.append(score)
                    m.global_found.Increment()
                else:
                    self.constraints_found += 1
                    self.constraint_scores.append(score)
                    m.found.Increment()
                m.scores[p.full][0].Observe(score)
                self.score_histogram.Add(score)
                pose = refined.get(i, (float(r["x"]), float(r["y"]), float(r["theta"])))
                if self.options.log_matches:
                    self._log_match(p, pose, score)
                self._constraints[p.slot] = Constraint(
                    submap_id=p.submap_id, node_id=p.node_id,
                    relative_pose=rigid2d_compose(rigid2d_inverse(p.submap.local_pose), pose),
                    translation_weight=self.options.loop_closure_translation_weight,
                    rotation_weight=self.options.loop_closure_rotation_weight,
                    score=score)
            if failed:
                print(f"ConstraintBuilder2D: {failed} of {len(pending)} pairs skipped "
                      f"({strerror(self.last_error)})", file=sys.stderr)

    def _log_match(self, p, pose, score):
        """ComputeConstraint's log_matches line (:260-276); `pose` is the
        refined pose estimate (map <- node), p.initial the search start."""
        info = (f"Node ({p.node_id[0]}, {p.node_id[1]}) with {len(p.cloud)} points on submap "
                f"({p.submap_id[0]}, {p.submap_id[1]})")
        if p.full:
            info += " matches"
        else:
            d = rigid2d_compose(rigid2d_inverse(p.initial), pose)
            info += " differs by translation %.2f rotation %.3f" % (
                math.hypot(d[0], d[1]), abs(_normalize_angle_difference(d[2])))
        self.log_sink(info + " with score %.1f%%." % (100.0 * score))


# ---------------------------------------------------------------------------
# ConstraintBuilder3D (reference constraint_builder_3d.cc; C++ mirror
# include/cartographer_amd/constraint_builder_3d.h).
#
# * MaybeAddConstraint (:79-114): drop pairs whose global translations are
#   farther apart than max_constraint_distance, then the per-submap
#   FixedRatioSampler; FastCorrelativeScanMatcher3D::Match(global_node_pose,
#   global_submap_pose, data, min_score) (:239-241).
# * MaybeAddGlobalConstraint (:116-142): MatchFullSubmap(node rotation,
#   submap rotation, data, global_localization_min_score) (:221-223).
# * NotifyEndOfNode / WhenDone / GetNumFinishedNodes / DeleteScanMatcher
#   (:144-168, :307-349); metrics (:46-59) as counters and score lists.
# * Constraint pose: the CSM estimate (submap <- node), refined by the
#   CeresScanMatcher3D restatement (:264-275; ceres_refine_batch_3d, parity
#   with Ceres unpinned) unless refine_with_ceres is off.
# ---------------------------------------------------------------------------

@dataclass
class Submap3D:
    """What the builder reads of a Submap3D (submap_3d.h:57-73): the high and
    low resolution HybridGrids (as (indices, values) cell lists) and the
    rotational scan-matcher histogram."""
    high_resolution: float
    high_cells: Tuple[np.ndarray, np.ndarray]
    low_resolution: float
    low_cells: Tuple[np.ndarray, np.ndarray]
    rotational_scan_matcher_histogram: np.ndarray
    high_grid_size: int = 0
    low_grid_size: int = 0


@dataclass
class Constraint3D:
    """PoseGraphInterface::Constraint (pose_graph_interface.h:36-53), 3D pose
    ((tx, ty, tz), (qw, qx, qy, qz)), submap <- node."""
    submap_id: Tuple[int, int]
    node_id: Tuple[int, int]
    relative_pose: Tuple[Tuple[float, float, float], Tuple[float, float, float, float]]
    translation_weight: float
    rotation_weight: float
    tag: str = "INTER_SUBMAP"
    score: float = 0.0
    rotational_score: float = 0.0
    low_resolution_score: float = 0.0


@dataclass
class _Pending3D:
    submap_id: Tuple[int, int]
    node_id: Tuple[int, int]
    data: NodeData3D
    full: bool
    node_pose: tuple
    submap_pose: tuple
    slot: int


class ConstraintBuilder3D:
    _metrics = _BuilderMetrics(True)

    @classmethod
    def RegisterMetrics(cls, factory):
        """The metric families of constraint_builder_3d.cc:351-386."""
        cls._metrics.register(factory, "3d")

    def __init__(self, options: ConstraintBuilderOptions, context: Optional[Context] = None):
        self.options = options
        # score_histogram_, rotational_score_histogram_, low_resolution_score_histogram_ (:257-259)
        self.score_histogram = _metrics.ScoreHistogram()
        self.rotational_score_histogram = _metrics.ScoreHistogram()
        self.low_resolution_score_histogram = _metrics.ScoreHistogram()
        self.log_sink = _LOG.info
        self.context = context or default_context()
        self._matchers = _MatcherCache(options.matcher_cache_bytes)  # key -> (high, low, m)
        self._submaps: Dict[Tuple[int, int], Submap3D] = {}  # for rebuilds of dropped matchers
        self._samplers: Dict[Tuple[int, int], FixedRatioSampler] = {}
        self._constraints: List[Optional[Constraint3D]] = []
        self._pending: List[_Pending3D] = []
        self._started_nodes = 0
        self._finished_nodes = 0
        self.constraints_searched = 0
        self.constraints_found = 0
        self.global_constraints_searched = 0
        self.global_constraints_found = 0
        self.constraints_failed = 0  # pairs skipped on a device error status
        self.last_error = CSM_OK
        self.constraint_scores: List[float] = []
        self.global_constraint_scores: List[float] = []
        self.rotational_scores: List[float] = []
        self.low_resolution_scores: List[float] = []

    # -- public interface (constraint_builder_3d.h:55-108) ------------------
    def MaybeAddConstraint(self, submap_id, submap: Submap3D, node_id, constant_data: NodeData3D,
                           global_node_pose, global_submap_pose):
        d = np.asarray(global_node_pose[0], np.float64) - np.asarray(global_submap_pose[0],
                                                                      np.float64)
        if float(np.linalg.norm(d)) > self.options.max_constraint_distance:
            return
        sampler = self._samplers.setdefault(tuple(submap_id),
                                            FixedRatioSampler(self.options.sampling_ratio))
        if not sampler.Pulse():
            return
        self._enqueue(submap_id, submap, node_id, constant_data, False,
                      global_node_pose, global_submap_pose)

    def MaybeAddGlobalConstraint(self, submap_id, submap: Submap3D, node_id,
                                 constant_data: NodeData3D, global_node_rotation,
                                 global_submap_rotation):
        self._enqueue(submap_id, submap, node_id, constant_data, True,
                      ((0.0, 0.0, 0.0), tuple(global_node_rotation)),
                      ((0.0, 0.0, 0.0), tuple(global_submap_rotation)))

    def NotifyEndOfNode(self):
        self._started_nodes += 1
        if len(self._pending) >= self.options.flush_pairs:
            self._flush()

    def WhenDone(self, callback: Callable[[List[Constraint3D]], None]):
        self._flush()
        result = [c for c in self._constraints if c is not None]
        if self.options.log_matches:  # RunWhenDoneCallback (:317-326)
            self.log_sink(f"{len(self._constraints)} computations resulted in {len(result)} "
                          "additional constraints.\nScore histogram:\n"
                          + self.score_histogram.ToString(10)
                          + "\nRotational score histogram:\n"
                          + self.rotational_score_histogram.ToString(10)
                          + "\nLow resolution score histogram:\n"
                          + self.low_resolution_score_histogram.ToString(10))
        self._constraints = []
        self._metrics.queue_length.Set(len(self._constraints))
        callback(result)

    def GetNumFinishedNodes(self) -> int:
        return self._finished_nodes

    def DeleteScanMatcher(self, submap_id):
        """Also drops the submap's pending pairs (no constraint)."""
        key = tuple(submap_id)
        self._matchers.pop(key, _MatcherCache._close)  # matcher, then its grids
        self._metrics.num_submap_scan_matchers.Set(len(self._matchers))
        self._samplers.pop(key, None)
        self._submaps.pop(key, None)
        before = len(self._pending)
        self._pending = [p for p in self._pending if p.submap_id != key]
        if len(self._pending) != before:
            print(f"ConstraintBuilder3D: DeleteScanMatcher dropped {before - len(self._pending)} "
                  "pending pairs of a deleted submap", file=sys.stderr)

    @property
    def num_submap_scan_matchers(self) -> int:  # kNumSubmapScanMatchersMetric
        return len(self._matchers)

    # -- internals ----------------------------------------------------------
    def _make_matcher(self, p):
        """DispatchScanMatcherConstruction (:170-198): grids and matcher."""
        submap = self._submaps[p.submap_id]
        high = HybridGrid(submap.high_resolution, *submap.high_cells,
                          grid_size=submap.high_grid_size, context=self.context)
        low = HybridGrid(submap.low_resolution, *submap.low_cells,
                         grid_size=submap.low_grid_size, context=self.context)
        m = FastCorrelativeScanMatcher3D(high, low, submap.rotational_scan_matcher_histogram,
                                         self.options.fast_correlative_scan_matcher_options_3d,
                                         self.context)
        return (high, low, m)

    @staticmethod
    def _bytes_of(entry):
        return sum(obj.device_bytes() for obj in entry)

    def _enqueue(self, submap_id, submap, node_id, data, full, node_pose, submap_pose):
        key = tuple(submap_id)
        self._submaps[key] = submap
        self._constraints.append(None)
        self._metrics.queue_length.Set(len(self._constraints))  # (:101, :127)
        p = _Pending3D(key, tuple(node_id), data, full, node_pose, submap_pose,
                       len(self._constraints) - 1)
        self._matchers.get(key, lambda: self._make_matcher(p), self._bytes_of)
        self._matchers.pinned.discard(key)
        self._matchers.trim()
        self._metrics.num_submap_scan_matchers.Set(len(self._matchers))
        self._pending.append(p)

    def _flush(self):
        pending, self._pending = self._pending, []
        if pending:
            for part, held in _budget_parts(pending, lambda p: p.submap_id, self._matchers,
                                            self._make_matcher, self._bytes_of):
                self._search(part, held)
        self._finished_nodes = self._started_nodes

    def _search(self, pending, held):
        """One batch (and its Ceres refinement) over the matchers in ``held``."""
        if pending:
            matchers, slot_of, nodes, node_of = [], {}, [], {}
            for p in pending:
                if p.submap_id not in slot_of:
                    slot_of[p.submap_id] = len(matchers)
                    matchers.append(held[p.submap_id][2])
                if id(p.data) not in node_of:  # a node's data uploads once
                    node_of[id(p.data)] = len(nodes)
                    nodes.append(p.data)
            pairs = make_pairs_3d(
                [slot_of[p.submap_id] for p in pending], [node_of[id(p.data)] for p in pending],
                [self.options.global_localization_min_score if p.full else self.options.min_score
                 for p in pending],
                [p.full for p in pending],
                node_q=[p.node_pose[1] for p in pending], node_t=[p.node_pose[0] for p in pending],
                submap_q=[p.submap_pose[1] for p in pending],
                submap_t=[p.submap_pose[0] for p in pending])
            results = match_batch_3d(matchers, nodes, pairs, self.context)
            refined = {}
            ok = [i for i, r in enumerate(results) if int(r["status"]) == CSM_OK]
            if self.options.refine_with_ceres and ok:
                # ceres_scan_matcher_.Match(pose.translation(), pose, {high, low clouds and grids})
                grids = []
                for key in slot_of:
                    grids.extend(held[key][:2])
                items = []
                for i in ok:
                    p, r = pending[i], results[i]
                    t = tuple(float(v) for v in r["t"])
                    q = tuple(float(v) for v in r["q"])
                    slot = slot_of[p.submap_id]
                    items.append((2 * slot, 2 * slot + 1, node_of[id(p.data)], (t, q), t))
                poses, _ = ceres_refine_batch_3d(grids, nodes, items,
                                                 self.options.ceres_scan_matcher_options_3d,
                                                 self.context)
                refined = dict(zip(ok, poses))
            failed = 0
            for i, (p, r) in enumerate(zip(pending, results)):
                if int(r["status"]) < 0:
                    # Not searchable on the device (CSM_ERANGE):
                    # no constraint, counted, never fatal (as the C++ header).
                    self.constraints_failed += 1
                    self.last_error = int(r["status"])
                    failed += 1
                    continue
                m = self._metrics
                if p.full:
                    self.global_constraints_searched += 1
                    m.global_searched.Increment()
                else:
                    self.constraints_searched += 1
                    m.searched.Increment()
                if int(r["status"]) != CSM_OK:
                    continue
                score = float(r["score"])
                rot, low = float(r["rotational_score"]), float(r["low_resolution_score"])
                if p.full:
                    self.global_constraints_found += 1
                    self.global_constraint_scores.append(score)
                    m.global_found.Increment()
                else:
                    self.constraints_found += 1
                    self.constraint_scores.append(score)
                    m.found.Increment()
                for h, v in zip(m.scores[p.full], (score, rot, low)):
                    h.Observe(v)
                self.score_histogram.Add(score)
                self.rotational_score_histogram.Add(rot)
                self.low_resolution_score_histogram.Add(low)
                self.rotational_scores.append(rot)
                self.low_resolution_scores.append(low)
                pose = refined.get(i, (tuple(float(v) for v in r["t"]),
                                       tuple(float(v) for v in r["q"])))
                self._constraints[p.slot] = Constraint3D(
                    submap_id=p.submap_id, node_id=p.node_id,
                    relative_pose=(tuple(pose[0]), tuple(pose[1])),
                    translation_weight=self.options.loop_closure_translation_weight,
                    rotation_weight=self.options.loop_closure_rotation_weight,
                    score=score, rotational_score=float(r["rotational_score"]),
                    low_resolution_score=float(r["low_resolution_score"]))
                if self.options.log_matches:
                    self._log_match(p, self._constraints[p.slot].relative_pose, score)
            if failed:
                print(f"ConstraintBuilder3D: {failed} of {len(pending)} pairs skipped "
                      f"({strerror(self.last_error)})", file=sys.stderr)

    def _log_match(self, p, constraint, score):
        """ComputeConstraint's log_matches line (:284-303): difference =
        global_node_pose^-1 * global_submap_pose * constraint, its angle
        transform::GetAngle."""
        info = (f"Node ({p.node_id[0]}, {p.node_id[1]}) with "
                f"{len(p.data.high_resolution_point_cloud)} points on submap "
                f"({p.submap_id[0]}, {p.submap_id[1]})")
        if p.full:
            info += " matches"
        else:
            d = rigid3d_compose(rigid3d_compose(rigid3d_inverse(p.node_pose), p.submap_pose),
                                constraint)
            q = d[1]
            angle = 2.0 * math.atan2(math.sqrt(q[1] ** 2 + q[2] ** 2 + q[3] ** 2), abs(q[0]))
            info += " differs by translation %.2f rotation %.3f" % (
                math.sqrt(sum(c * c for c in d[0])), angle)
        self.log_sink(info + " with score %.1f%%." % (100.0 * score))
