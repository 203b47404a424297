"""3D correlative scan matchers — Python mirror of the 3D C-ABI.

* :class:`HybridGrid` — a HybridGrid's known cells on the device
  (``mapping/3d/hybrid_grid.h:463-545``; cells as the iterator / ToProto yields them).
* :class:`RealTimeCorrelativeScanMatcher3D` — ``Match``
  (``real_time_correlative_scan_matcher_3d.h:47-50``).
* :class:`FastCorrelativeScanMatcher3D` — ``Match`` / ``MatchFullSubmap``
  (``fast_correlative_scan_matcher_3d.h:75-101``), results as
  ``FastCorrelativeScanMatcher3D::Result`` or ``None`` (the reference's nullptr).
* :func:`match_batch_3d` — the batched ConstraintBuilder3D search.

Every compute call runs the HIP kernels; there is no CPU fallback.
"""

from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import (CSM_OK, Context, Fast3DOptions, Node3D, Pair3D, Pose3D, Result3D, RtOptions,
               _check, _f32_points, _ptr, default_context)


class HybridGrid:
    """Known cells of a HybridGrid: ``indices`` (n, 3) int and uint16 ``values``."""

    def __init__(self, resolution: float, indices, values, grid_size: int = 0,
                 context: Optional[Context] = None):
        self.context = context or default_context()
        self._lib = self.context._lib
        self.resolution = float(resolution)
        idx = np.ascontiguousarray(np.asarray(indices, np.int32).reshape(-1, 3))
        val = np.ascontiguousarray(np.asarray(values, np.uint16).reshape(-1))
        if len(idx) != len(val):
            raise ValueError("indices and values differ in length")
        h = C.c_void_p()
        _check(self._lib.csm_hybrid_grid_create(self.context.handle, self.resolution,
                                                _ptr(idx, C.c_int32), _ptr(val, C.c_uint16),
                                                len(val), int(grid_size), C.byref(h)),
               "csm_hybrid_grid_create")
        self.handle = h

    @classmethod
    def create_batch(cls, resolution, cells, grid_sizes=None, context: Optional[Context] = None):
        """Many grids in one call (csm_hybrid_grid_create_batch): ``cells`` is a
        list of (indices, values) pairs, ``resolution`` one value or one per
        grid; returns the grids in order, each what the constructor returns."""
        context = context or default_context()
        lib = context._lib
        n = len(cells)
        res = np.broadcast_to(np.asarray(resolution, np.float32), (n,)).copy()
        idx = [np.ascontiguousarray(np.asarray(c[0], np.int32).reshape(-1, 3)) for c in cells]
        val = [np.ascontiguousarray(np.asarray(c[1], np.uint16).reshape(-1)) for c in cells]
        if any(len(i) != len(v) for i, v in zip(idx, val)):
            raise ValueError("indices and values differ in length")
        k = max(n, 1)
        iptr = (C.POINTER(C.c_int32) * k)(*[_ptr(i, C.c_int32) for i in idx])
        vptr = (C.POINTER(C.c_uint16) * k)(*[_ptr(v, C.c_uint16) for v in val])
        cnt = (C.c_int64 * k)(*[len(v) for v in val])
        gs = (C.c_int32 * k)(*([int(g) for g in grid_sizes] if grid_sizes is not None else [0] * n))
        out = (C.c_void_p * k)()
        _check(lib.csm_hybrid_grid_create_batch(context.handle, n, _ptr(res, C.c_float), iptr, vptr, cnt,
                                                gs, out), "csm_hybrid_grid_create_batch")
        made = []
        for i in range(n):
            g = cls.__new__(cls)
            g.context, g._lib, g.resolution = context, lib, float(res[i])
            g.handle = C.c_void_p(out[i])
            made.append(g)
        return made

    def device_bytes(self) -> int:
        """Device memory of the grid's bricks (csm_hybrid_grid_device_bytes)."""
        return int(self._lib.csm_hybrid_grid_device_bytes(self.handle))

    def info(self):
        o, d, g = (C.c_int32 * 3)(), (C.c_int32 * 3)(), C.c_int32()
        _check(self._lib.csm_hybrid_grid_info(self.handle, o, d, C.byref(g)), "csm_hybrid_grid_info")
        return tuple(o), tuple(d), g.value

    def get_probability(self, indices):
        """HybridGrid::GetProbability at cell indices (n, 3), on the device."""
        idx = np.ascontiguousarray(np.asarray(indices, np.int32).reshape(-1, 3))
        out = np.zeros(len(idx), np.float32)
        _check(self._lib.csm_hybrid_grid_get_probability(self.handle, _ptr(idx, C.c_int32), len(idx),
                                                         _ptr(out, C.c_float)),
               "csm_hybrid_grid_get_probability")
        return out

    def interpolate(self, points):
        """InterpolatedProbabilityGrid::GetInterpolatedValue at points (n, 3),
        on the device (the CeresScanMatcher3D kernel's interpolation)."""
        xyz = np.ascontiguousarray(np.asarray(points, np.float64).reshape(-1, 3))
        out = np.zeros(len(xyz), np.float64)
        _check(self._lib.csm_hybrid_grid_interpolate(self.handle, _ptr(xyz, C.c_double), len(xyz),
                                                     _ptr(out, C.c_double)),
               "csm_hybrid_grid_interpolate")
        return out

    def close(self):
        if getattr(self, "handle", None):
            self._lib.csm_hybrid_grid_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _pose(p) -> Pose3D:
    if isinstance(p, Pose3D):
        return p
    t, q = p
    return Pose3D.make(t, q)


class RealTimeCorrelativeScanMatcher3D:
    def __init__(self, options, context: Optional[Context] = None):
        self.context = context or default_context()
        self._lib = self.context._lib
        self.options = options

    def Match(self, initial_pose_estimate, point_cloud, grid: HybridGrid):
        """-> (score, ((tx, ty, tz), (qw, qx, qy, qz)))."""
        o = self.options
        opts = RtOptions(o.linear_search_window, o.angular_search_window,
                         o.translation_delta_cost_weight, o.rotation_delta_cost_weight)
        pts = _f32_points(point_cloud)
        init = _pose(initial_pose_estimate)
        score = C.c_float()
        out = Pose3D()
        _check(self._lib.csm_rt3d_match(self.context.handle, C.byref(opts), grid.handle,
                                        C.byref(init), _ptr(pts, C.c_float), len(pts),
                                        C.byref(score), C.byref(out)), "csm_rt3d_match")
        return float(score.value), out.as_tuple()

    def _opts(self):
        o = self.options
        return RtOptions(o.linear_search_window, o.angular_search_window,
                         o.translation_delta_cost_weight, o.rotation_delta_cost_weight)

    def window(self, point_cloud, resolution):
        """GenerateExhaustiveSearchTransforms' window: (num_translations,
        num_rotations); candidate index = t * num_rotations + r."""
        pts = _f32_points(point_cloud)
        nt, nr = C.c_int32(), C.c_int32()
        opts = self._opts()
        _check(self._lib.csm_rt3d_window(C.byref(opts), float(resolution), _ptr(pts, C.c_float),
                                         len(pts), C.byref(nt), C.byref(nr)), "csm_rt3d_window")
        return nt.value, nr.value

    def score_rotations(self, initial_pose_estimate, point_cloud, grid: HybridGrid, rotations):
        """Test-visible: ScoreCandidate of every translation for the given
        rotation indices, by Match's kernel -> (len(rotations), num_translations)."""
        pts = _f32_points(point_cloud)
        rot = np.ascontiguousarray(np.asarray(rotations, np.int32))
        nt, _ = self.window(pts, grid.resolution)
        out = np.zeros((len(rot), nt), np.float32)
        opts = self._opts()
        init = _pose(initial_pose_estimate)
        _check(self._lib.csm_rt3d_score_rotations(self.context.handle, C.byref(opts), grid.handle,
                                                  C.byref(init), _ptr(pts, C.c_float), len(pts),
                                                  _ptr(rot, C.c_int32), len(rot),
                                                  _ptr(out, C.c_float)),
               "csm_rt3d_score_rotations")
        return out


@dataclass
class FastCorrelativeScanMatcherOptions3D:
    """proto::FastCorrelativeScanMatcherOptions3D; defaults from
    configuration_files/pose_graph.lua:40-48."""
    branch_and_bound_depth: int = 8
    full_resolution_depth: int = 3
    min_rotational_score: float = 0.77
    min_low_resolution_score: float = 0.55
    linear_xy_search_window: float = 5.0
    linear_z_search_window: float = 1.0
    angular_search_window: float = math.radians(15.0)

    def to_c(self) -> Fast3DOptions:
        return Fast3DOptions(self.branch_and_bound_depth, self.full_resolution_depth,
                             self.min_rotational_score, self.min_low_resolution_score,
                             self.linear_xy_search_window, self.linear_z_search_window,
                             self.angular_search_window)


@dataclass
class NodeData3D:
    """The TrajectoryNode::Data fields the 3D matcher reads."""
    high_resolution_point_cloud: np.ndarray
    low_resolution_point_cloud: np.ndarray
    rotational_scan_matcher_histogram: np.ndarray
    gravity_alignment: tuple = (1.0, 0.0, 0.0, 0.0)
    _keep: list = field(default_factory=list, repr=False)

    def to_c(self) -> Node3D:
        hi = _f32_points(self.high_resolution_point_cloud)
        lo = _f32_points(self.low_resolution_point_cloud)
        hist = np.ascontiguousarray(np.asarray(self.rotational_scan_matcher_histogram, np.float32))
        self._keep = [hi, lo, hist]
        n = Node3D()
        n.high_resolution_xyz = _ptr(hi, C.c_float)
        n.num_high_resolution = len(hi)
        n.low_resolution_xyz = _ptr(lo, C.c_float)
        n.num_low_resolution = len(lo)
        n.histogram = _ptr(hist, C.c_float)
        n.histogram_size = len(hist)
        n.gravity_alignment[:] = [float(v) for v in self.gravity_alignment]
        return n


class NodeSet3D:
    """A node list converted once to the C-ABI's csm_node3d array (the clouds
    stay referenced, not copied). match_batch_3d / ceres_refine_batch_3d take
    it in place of a NodeData3D sequence when the same nodes are searched
    repeatedly, as a ConstraintBuilder's pending nodes are."""

    def __init__(self, nodes: Sequence[NodeData3D]):
        self.nodes = list(nodes)
        self.array = (Node3D * max(len(self.nodes), 1))(*[n.to_c() for n in self.nodes])

    def __len__(self):
        return len(self.nodes)


def _c_nodes(nodes):
    if isinstance(nodes, NodeSet3D):
        return nodes.array
    return (Node3D * max(len(nodes), 1))(*[n.to_c() for n in nodes])


@dataclass
class Result:
    """FastCorrelativeScanMatcher3D::Result."""
    score: float
    pose_estimate: tuple
    rotational_score: float
    low_resolution_score: float
    tie: int = 0  # csm_result3d.tie (TIE_*): how the pick among exactly tied leaves was made


def _result(r: Result3D) -> Optional[Result]:
    _check(r.status, "FastCorrelativeScanMatcher3D")
    if r.status != CSM_OK:
        return None
    return Result(float(r.score), r.pose.as_tuple(), float(r.rotational_score),
                  float(r.low_resolution_score), int(r.tie))


class FastCorrelativeScanMatcher3D:
    def __init__(self, hybrid_grid: HybridGrid, low_resolution_grid: HybridGrid,
                 histogram, options: FastCorrelativeScanMatcherOptions3D,
                 context: Optional[Context] = None):
        self.context = context or default_context()
        self._lib = self.context._lib
        self.options = options
        self.low_resolution_grid = low_resolution_grid  # must outlive the matcher
        hist = np.ascontiguousarray(np.asarray(histogram, np.float32))
        opts = options.to_c()
        h = C.c_void_p()
        _check(self._lib.csm_fast3d_create(self.context.handle, hybrid_grid.handle,
                                           low_resolution_grid.handle, _ptr(hist, C.c_float),
                                           len(hist), C.byref(opts), C.byref(h)),
               "csm_fast3d_create")
        self.handle = h

    @classmethod
    def create_batch(cls, grids, histograms, options: FastCorrelativeScanMatcherOptions3D,
                     context: Optional[Context] = None):
        """Many matchers in one call (csm_fast3d_create_batch): ``grids`` is a
        list of (high_resolution, low_resolution) HybridGrid pairs; returns
        the matchers in the same order, each what the constructor returns."""
        context = context or default_context()
        lib = context._lib
        n = len(grids)
        if n != len(histograms):
            raise ValueError("one histogram per grid pair")
        hists = [np.ascontiguousarray(np.asarray(h, np.float32)) for h in histograms]
        highs = (C.c_void_p * max(n, 1))(*[g[0].handle for g in grids])
        lows = (C.c_void_p * max(n, 1))(*[g[1].handle for g in grids])
        hptr = (C.POINTER(C.c_float) * max(n, 1))(*[_ptr(h, C.c_float) for h in hists])
        hsize = (C.c_int32 * max(n, 1))(*[len(h) for h in hists])
        out = (C.c_void_p * max(n, 1))()
        opts = options.to_c()
        _check(lib.csm_fast3d_create_batch(context.handle, n, highs, lows, hptr, hsize,
                                           C.byref(opts), out), "csm_fast3d_create_batch")
        made = []
        for i in range(n):
            m = cls.__new__(cls)
            m.context, m._lib, m.options = context, lib, options
            m.low_resolution_grid = grids[i][1]  # must outlive the matcher
            m.handle = C.c_void_p(out[i])
            made.append(m)
        return made

    def close(self):
        if getattr(self, "handle", None):
            self._lib.csm_fast3d_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_bytes(self) -> int:
        """Device memory of the pyramid (csm_fast3d_device_bytes)."""
        return int(self._lib.csm_fast3d_device_bytes(self.handle))

    def read_level(self, level: int):
        o, d = (C.c_int32 * 3)(), (C.c_int32 * 3)()
        _check(self._lib.csm_fast3d_read_level(self.handle, level, None, 0, o, d),
               "csm_fast3d_read_level")
        out = np.zeros(int(d[0]) * int(d[1]) * int(d[2]), np.uint8)
        _check(self._lib.csm_fast3d_read_level(self.handle, level, _ptr(out, C.c_uint8), out.size,
                                               o, d), "csm_fast3d_read_level")
        return tuple(o), out.reshape(int(d[2]), int(d[1]), int(d[0]))

    def Match(self, global_node_pose, global_submap_pose, node: NodeData3D, min_score: float):
        n = node.to_c()
        r = Result3D()
        _check(self._lib.csm_fast3d_match(self.handle, C.byref(_pose(global_node_pose)),
                                          C.byref(_pose(global_submap_pose)), C.byref(n),
                                          min_score, C.byref(r)), "csm_fast3d_match")
        return _result(r)

    def MatchFullSubmap(self, global_node_rotation, global_submap_rotation, node: NodeData3D,
                        min_score: float):
        n = node.to_c()
        a = (C.c_double * 4)(*[float(v) for v in global_node_rotation])
        b = (C.c_double * 4)(*[float(v) for v in global_submap_rotation])
        r = Result3D()
        _check(self._lib.csm_fast3d_match_full_submap(self.handle, a, b, C.byref(n), min_score,
                                                      C.byref(r)), "csm_fast3d_match_full_submap")
        return _result(r)


PAIR3_DTYPE = np.dtype([("submap", np.int32), ("node", np.int32), ("full_submap", np.int32),
                        ("min_score", np.float32), ("node_t", np.float64, 3),
                        ("node_q", np.float64, 4), ("submap_t", np.float64, 3),
                        ("submap_q", np.float64, 4)])
RESULT3_DTYPE = np.dtype([("status", np.int32), ("score", np.float32), ("t", np.float64, 3),
                          ("q", np.float64, 4), ("rotational_score", np.float32),
                          ("low_resolution_score", np.float32), ("tie", np.int32),
                          ("reserved", np.int32)])


def make_pairs_3d(submap, node, min_score, full_submap=True, node_q=None, node_t=None,
                  submap_q=None, submap_t=None) -> np.ndarray:
    """Vectorised csm_pair3d array (pose rotations as (w, x, y, z))."""
    submap = np.asarray(submap, np.int32)
    pairs = np.zeros(len(submap), PAIR3_DTYPE)
    pairs["submap"] = submap
    pairs["node"] = np.asarray(node, np.int32)
    pairs["full_submap"] = np.asarray(full_submap, np.int32)
    pairs["min_score"] = min_score
    pairs["node_q"] = (1.0, 0.0, 0.0, 0.0) if node_q is None else node_q
    pairs["submap_q"] = (1.0, 0.0, 0.0, 0.0) if submap_q is None else submap_q
    if node_t is not None:
        pairs["node_t"] = node_t
    if submap_t is not None:
        pairs["submap_t"] = submap_t
    return pairs


def match_batch_3d(matchers: Sequence[FastCorrelativeScanMatcher3D], nodes: Sequence[NodeData3D],
                   pairs, context: Optional[Context] = None):
    """Batched FastCSM3D search. `pairs` is a PAIR3_DTYPE array (make_pairs_3d)
    or a sequence of (submap, node, full_submap, min_score, node_pose,
    submap_pose) tuples. Returns a RESULT3_DTYPE array in pair order (tuple
    input: a list of Result3D records)."""
    ctx = context or (matchers[0].context if matchers else default_context())
    lib = ctx._lib
    assert PAIR3_DTYPE.itemsize == C.sizeof(Pair3D)
    assert RESULT3_DTYPE.itemsize == C.sizeof(Result3D)
    cnodes = _c_nodes(nodes)
    handles = (C.c_void_p * len(matchers))(*[m.handle for m in matchers])
    if isinstance(pairs, np.ndarray):
        arr = np.ascontiguousarray(pairs, PAIR3_DTYPE)
        out = np.zeros(len(arr), RESULT3_DTYPE)
        _check(lib.csm_fast3d_match_batch(ctx.handle, handles, len(matchers), cnodes, len(nodes),
                                          arr.ctypes.data_as(C.POINTER(Pair3D)), len(arr),
                                          out.ctypes.data_as(C.POINTER(Result3D))),
               "csm_fast3d_match_batch")
        return out
    cpairs = (Pair3D * len(pairs))()
    for i, (s, n, full, ms, npose, spose) in enumerate(pairs):
        cpairs[i].submap, cpairs[i].node, cpairs[i].full_submap = s, n, 1 if full else 0
        cpairs[i].min_score = ms
        cpairs[i].node_pose = _pose(npose)
        cpairs[i].submap_pose = _pose(spose)
    results = (Result3D * len(pairs))()
    _check(lib.csm_fast3d_match_batch(ctx.handle, handles, len(matchers), cnodes, len(nodes),
                                      cpairs, len(pairs), results), "csm_fast3d_match_batch")
    return list(results)


def ceres_refine_batch_3d(grids: Sequence[HybridGrid], nodes: Sequence[NodeData3D], items,
                          options=None, context: Optional[Context] = None):
    """CeresScanMatcher3D::Match on the device for each item
    (high_grid, low_grid, node, initial ((t), (w, x, y, z)), target (t))
    (ceres_scan_matcher_3d.cc:84-160): returns ([((t), (q)), ...], iterations)."""
    from . import CeresOptions3D, Refine3D
    ctx = context or (grids[0].context if grids else default_context())
    n = len(items)
    citems = (Refine3D * max(n, 1))()
    for i, (hg, lg, nd, init, target) in enumerate(items):
        citems[i].high_grid, citems[i].low_grid, citems[i].node = hg, lg, nd
        citems[i].initial = _pose(init)
        for a in range(3):
            citems[i].target[a] = float(target[a])
    cnodes = _c_nodes(nodes)
    handles = (C.c_void_p * max(len(grids), 1))(*[g.handle for g in grids])
    out = (Pose3D * max(n, 1))()
    iters = np.zeros(max(n, 1), np.int32)
    opts = options or CeresOptions3D.make()
    _check(ctx._lib.csm_ceres3d_refine_batch(ctx.handle, handles, len(grids), cnodes, len(nodes),
                                             citems, n, C.byref(opts), out,
                                             _ptr(iters, C.c_int32)),
           "csm_ceres3d_refine_batch")
    return [out[i].as_tuple() for i in range(n)], iters[:n]


# --------------------------------------------------------------------------
# Synthetic 3D world (bench / test inputs; not the matching path).

class SynthConfig3D(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("world_x", C.c_double), ("world_y", C.c_double),
                ("world_z", C.c_double), ("num_boxes", C.c_int32), ("num_nodes", C.c_int32),
                ("num_submaps", C.c_int32), ("scans_per_submap", C.c_int32),
                ("rings", C.c_int32), ("azimuths", C.c_int32), ("min_elevation", C.c_double),
                ("max_elevation", C.c_double), ("max_range", C.c_double),
                ("range_noise", C.c_double), ("high_resolution", C.c_double),
                ("low_resolution", C.c_double), ("high_resolution_max_range", C.c_double),
                ("high_voxel", C.c_double), ("low_voxel", C.c_double),
                ("high_max_range", C.c_double), ("high_min_points", C.c_int32),
                ("low_min_points", C.c_int32), ("low_max_range", C.c_double),
                ("histogram_size", C.c_int32),
                ("insert_voxel", C.c_double), ("threads", C.c_int32),
                ("submap_begin", C.c_int32), ("submap_count", C.c_int32)]


class SyntheticWorld3D:
    """Seeded warehouse, 64-ring lidar scans, submaps with high/low-resolution
    grids and rotational histograms."""

    def __init__(self, num_nodes=16, num_submaps=4, submap_range=None, **kw):
        """submap_range=(begin, count): build only those submaps of the
        num_submaps-submap world (a rank's shard); they are indexed 0..count-1
        here, with submap_ids the world indices."""
        from . import SYNTH_PATH
        lib = C.CDLL(SYNTH_PATH)
        lib.csm_synth3d_create.argtypes = [C.POINTER(SynthConfig3D), C.POINTER(C.c_void_p)]
        lib.csm_synth3d_destroy.argtypes = [C.c_void_p]
        lib.csm_synth3d_node_poses.restype = C.POINTER(C.c_double)
        lib.csm_synth3d_node_poses.argtypes = [C.c_void_p]
        lib.csm_synth3d_submap_nodes.restype = C.POINTER(C.c_int32)
        lib.csm_synth3d_submap_nodes.argtypes = [C.c_void_p]
        lib.csm_synth3d_cloud.restype = C.c_int64
        lib.csm_synth3d_cloud.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_float),
                                          C.c_int64]
        lib.csm_synth3d_node_histogram.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_float)]
        lib.csm_synth3d_submap_histogram.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_float)]
        lib.csm_synth3d_grid.restype = C.c_int64
        lib.csm_synth3d_grid.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_int32),
                                         C.POINTER(C.c_uint16), C.c_int64]
        cfg = SynthConfig3D()
        lib.csm_synth3d_default_config(C.byref(cfg))
        cfg.num_nodes, cfg.num_submaps = num_nodes, num_submaps
        if submap_range is not None:
            cfg.submap_begin, cfg.submap_count = int(submap_range[0]), int(submap_range[1])
        for k, v in kw.items():
            setattr(cfg, k, v)
        h = C.c_void_p()
        if lib.csm_synth3d_create(C.byref(cfg), C.byref(h)) != 0:
            raise ValueError("invalid synthetic 3D world config")
        try:
            n, hs = num_nodes, cfg.histogram_size
            s = cfg.submap_count if cfg.submap_count > 0 else num_submaps
            self.submap_ids = np.arange(s) + (cfg.submap_begin if cfg.submap_count > 0 else 0)
            self.node_poses = np.ctypeslib.as_array(lib.csm_synth3d_node_poses(h), (n * 4,)).reshape(-1, 4).copy()
            self.submap_nodes = np.ctypeslib.as_array(lib.csm_synth3d_submap_nodes(h), (max(s, 1),))[:s].copy()

            def cloud(i, kind):
                m = lib.csm_synth3d_cloud(h, i, kind, None, 0)
                out = np.zeros((m, 3), np.float32)
                lib.csm_synth3d_cloud(h, i, kind, _ptr(out, C.c_float), m)
                return out

            self.raw = [cloud(i, 0) for i in range(n)]
            self.high = [cloud(i, 1) for i in range(n)]
            self.low = [cloud(i, 2) for i in range(n)]
            self.node_hist = []
            for i in range(n):
                out = np.zeros(hs, np.float32)
                lib.csm_synth3d_node_histogram(h, i, _ptr(out, C.c_float))
                self.node_hist.append(out)
            self.submap_hist, self.high_cells, self.low_cells = [], [], []
            for j in range(s):
                out = np.zeros(hs, np.float32)
                lib.csm_synth3d_submap_histogram(h, j, _ptr(out, C.c_float))
                self.submap_hist.append(out)
                for grid, dst in ((0, self.high_cells), (1, self.low_cells)):
                    m = lib.csm_synth3d_grid(h, j, grid, None, None, 0)
                    ijk = np.zeros((m, 3), np.int32)
                    val = np.zeros(m, np.uint16)
                    lib.csm_synth3d_grid(h, j, grid, _ptr(ijk, C.c_int32), _ptr(val, C.c_uint16), m)
                    dst.append((ijk, val))
        finally:
            lib.csm_synth3d_destroy(h)
        self.high_resolution = cfg.high_resolution
        self.low_resolution = cfg.low_resolution
        self.num_nodes, self.num_submaps = num_nodes, s

    def node(self, i) -> NodeData3D:
        return NodeData3D(self.high[i], self.low[i], self.node_hist[i])

    def node_rotation(self, i):
        yaw = float(self.node_poses[i, 3])
        return (math.cos(0.5 * yaw), 0.0, 0.0, math.sin(0.5 * yaw))

    def node_in_submap(self, i, s):
        """Ground-truth node pose in submap s's frame: ((t), (q))."""
        c = int(self.submap_nodes[s])
        t = (float(self.node_poses[i, 0] - self.node_poses[c, 0]),
             float(self.node_poses[i, 1] - self.node_poses[c, 1]), 0.0)
        return t, self.node_rotation(i)
