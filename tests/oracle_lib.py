"""ctypes wrapper of the oracle (oracle/_build/liboracle.so) — test
infrastructure only: the checker the HIP path is compared against."""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "_build", "liboracle.so")

D, F, I32, I64, VP = C.c_double, C.c_float, C.c_int32, C.c_int64, C.c_void_p
P = C.POINTER


def _p(a, t):
    return a.ctypes.data_as(P(t))


class Oracle:
    def __init__(self, path=ORACLE_PATH):
        lib = C.CDLL(path)
        sig = {
            "oracle_fast2d_create": (VP, [D, D, D, I32, I32, P(C.c_uint16), D, D, I32]),
            "oracle_fast2d_destroy": (None, [VP]),
            "oracle_fast2d_level": (I64, [VP, I32, P(C.c_uint8), P(I32), P(I32)]),
            "oracle_fast2d_match_full_submap": (I32, [VP, P(F), I32, F, P(F), P(D), P(I64)]),
            "oracle_fast2d_match": (I32, [VP, P(D), P(F), I32, F, P(F), P(D), P(I64)]),
            "oracle_fast2d_score_candidate": (I32, [VP, I32, P(D), D, D, P(F), I32, I32, I32,
                                                    I32, I32, P(I32), P(F)]),
            "oracle_fast2d_tie_leaves": (I32, [VP, I32, P(D), P(F), I32, F, I32, P(I32), P(I32)]),
            "oracle_fast2d_match_pairs": (D, [P(VP), P(F), P(I64), P(I32), P(I32), I64, I32, F,
                                              P(F), P(D), P(I32), P(D)]),
            "oracle_fast2d_match_pairs_stats": (D, [P(VP), P(F), P(I64), P(I32), P(I32), I64, I32,
                                                    F, P(F), P(D), P(I32), P(D), P(I64)]),
            "oracle_rt2d_match": (D, [D, D, D, I32, I32, P(C.c_uint16), D, D, D, D, P(D), P(F),
                                      I32, P(D), P(I64)]),
            "oracle_rt2d_time": (D, [D, D, D, I32, I32, P(C.c_uint16), D, D, D, D, P(D), P(F),
                                     I32, I32]),
            "oracle_discretize": (I32, [D, D, D, I32, I32, P(D), D, D, P(F), I32, I32, P(I32),
                                        P(I32), P(I32), I64, P(D)]),
            "oracle_search_parameters": (I32, [D, D, P(F), I32, D, P(I32), P(D), P(I32), P(I32)]),
            "oracle_generate_rotated_scans": (I32, [P(F), I32, I32, I32, D, D, P(F)]),
            "oracle_discretize_scans": (I32, [D, D, D, I32, I32, P(F), I32, I32, F, F, P(I32)]),
            "oracle_rt2d_score_candidates": (I32, [D, D, D, I32, I32, P(C.c_uint16), D, D,
                                                   P(I32), I32, I32, I32, D, P(I32), I64, P(F)]),
            "oracle_rt2d_score_candidates_tsdf": (I32, [D, D, D, I32, I32, P(C.c_uint16),
                                                        P(C.c_uint16), F, F, D, D, P(I32), I32,
                                                        I32, I32, D, P(I32), I64, P(F)]),
            "oracle_grid_create": (VP, [D, D, D, I32, I32]),
            "oracle_grid_destroy": (None, [VP]),
            "oracle_grid_insert": (None, [VP, F, F, I32, P(F), P(F), I32]),
            "oracle_grid_set_probability": (None, [VP, I32, I32, F]),
            "oracle_grid_crop": (None, [VP]),
            "oracle_ceres2d_match": (I32, [D, D, D, I32, I32, P(C.c_uint16), F, F, P(D), P(D), P(D),
                                           P(F), I32, P(D)]),
            "oracle_grid_info": (None, [VP, P(D), P(I32)]),
            "oracle_grid_cells": (None, [VP, P(C.c_uint16)]),
            "oracle_transform_cloud_2d": (None, [P(F), P(F), I32, P(F)]),
            "oracle_tsdf_create": (VP, [D, D, D, I32, I32, F, F]),
            "oracle_tsdf_destroy": (None, [VP]),
            "oracle_tsdf_insert": (None, [VP, P(D), P(F), P(F), I32]),
            "oracle_tsdf_info": (None, [VP, P(D), P(I32)]),
            "oracle_tsdf_cells": (None, [VP, P(C.c_uint16), P(C.c_uint16)]),
            "oracle_voxel_filter": (I64, [P(F), P(I64), I32, F, P(C.c_uint8)]),
            "oracle_adaptive_voxel_filter": (I64, [P(F), P(I64), I32, F, F, F, P(C.c_uint8)]),
            "oracle_rt2d_match_tsdf": (D, [D, D, D, I32, I32, P(C.c_uint16), P(C.c_uint16), F,
                                           F, D, D, D, D, P(D), P(F), I32, P(D), P(I64)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        self.lib = lib

    # ---- grids ---------------------------------------------------------
    def grid_from_inserts(self, res, max_x, max_y, nx, ny, inserts, hit=0.7, miss=0.4,
                          crop=False):
        """Grid built with the restated ProbabilityGridRangeDataInserter2D.
        inserts: list of (origin xyz, returns (n,3)). Returns (limits, cells);
        crop=True finishes it like Submap2D::Finish (ComputeCroppedGrid)."""
        g = self.lib.oracle_grid_create(res, max_x, max_y, nx, ny)
        try:
            for origin, ret in inserts:
                o = np.asarray(origin, np.float32)
                r = np.ascontiguousarray(ret, np.float32)
                self.lib.oracle_grid_insert(g, hit, miss, 1, _p(o, F), _p(r, F), len(r))
            if crop:
                self.lib.oracle_grid_crop(g)
            return self._grid_out(g)
        finally:
            self.lib.oracle_grid_destroy(g)

    def grid_from_probabilities(self, res, max_x, max_y, nx, ny, cells_xy_p, crop=False):
        g = self.lib.oracle_grid_create(res, max_x, max_y, nx, ny)
        try:
            for x, y, p in cells_xy_p:
                self.lib.oracle_grid_set_probability(g, int(x), int(y), float(p))
            if crop:
                self.lib.oracle_grid_crop(g)
            return self._grid_out(g)
        finally:
            self.lib.oracle_grid_destroy(g)

    def _grid_out(self, g):
        info = np.zeros(3)
        cells = np.zeros(2, np.int32)
        self.lib.oracle_grid_info(g, _p(info, D), _p(cells, I32))
        out = np.zeros((cells[1], cells[0]), np.uint16)
        self.lib.oracle_grid_cells(g, _p(out, C.c_uint16))
        return (float(info[0]), float(info[1]), float(info[2])), out

    # ---- TSDF2D (restated TSDFRangeDataInserter2D) -----------------------
    # Inserter options in proto order: truncation_distance, maximum_weight,
    # update_free_space, num_normal_samples, sample_radius,
    # project_sdf_distance_to_scan_normal, update_weight_range_exponent,
    # angle bandwidth, distance bandwidth.
    TSDF_TEST_OPTIONS = (0.3, 10.0, 0, 4, 0.5, 1, 0, 0.5, 0.5)  # rtcsm_2d_test.cc:67-90

    def tsdf_from_inserts(self, res, max_x, max_y, nx, ny, truncation, max_weight, inserts,
                          options=TSDF_TEST_OPTIONS):
        """TSDF2D built by the restated inserter; inserts: list of (origin xyz,
        returns (n,3)). Returns (limits, tsd_cells, weight_cells)."""
        g = self.lib.oracle_tsdf_create(res, max_x, max_y, nx, ny, truncation, max_weight)
        try:
            opts = np.asarray(options, np.float64)
            for origin, ret in inserts:
                o = np.asarray(origin, np.float32)
                r = np.ascontiguousarray(ret, np.float32)
                self.lib.oracle_tsdf_insert(g, _p(opts, D), _p(o, F), _p(r, F), len(r))
            info = np.zeros(3)
            cells = np.zeros(2, np.int32)
            self.lib.oracle_tsdf_info(g, _p(info, D), _p(cells, I32))
            tsd = np.zeros((cells[1], cells[0]), np.uint16)
            wgt = np.zeros_like(tsd)
            self.lib.oracle_tsdf_cells(g, _p(tsd, C.c_uint16), _p(wgt, C.c_uint16))
            return (float(info[0]), float(info[1]), float(info[2])), tsd, wgt
        finally:
            self.lib.oracle_tsdf_destroy(g)

    def rt2d_match_tsdf(self, limits, tsd, wgt, truncation, max_weight, opts, initial, cloud):
        res, mx, my = limits
        tsd = np.ascontiguousarray(tsd, np.uint16)
        wgt = np.ascontiguousarray(wgt, np.uint16)
        init = np.asarray(initial, np.float64)
        pts = np.ascontiguousarray(cloud, np.float32)
        pose = np.zeros(3)
        ncand = C.c_int64()
        s = self.lib.oracle_rt2d_match_tsdf(res, mx, my, tsd.shape[1], tsd.shape[0],
                                            _p(tsd, C.c_uint16), _p(wgt, C.c_uint16), truncation,
                                            max_weight, *opts, _p(init, D), _p(pts, F), len(pts),
                                            _p(pose, D), C.byref(ncand))
        return s, tuple(pose), ncand.value

    def transform_cloud(self, pose_f, cloud):
        pose = np.asarray(pose_f, np.float32)
        c = np.ascontiguousarray(cloud, np.float32)
        out = np.zeros_like(c)
        self.lib.oracle_transform_cloud_2d(_p(pose, F), _p(c, F), len(c), _p(out, F))
        return out

    # ---- FastCSM2D -------------------------------------------------------
    def fast2d(self, limits, cells, lin, ang, depth):
        res, mx, my = limits
        cells = np.ascontiguousarray(cells, np.uint16)
        return OracleFast2D(self, self.lib.oracle_fast2d_create(
            res, mx, my, cells.shape[1], cells.shape[0], _p(cells, C.c_uint16), lin, ang, depth),
            limits, lin, ang)

    def rt2d_match(self, limits, cells, opts, initial, cloud):
        res, mx, my = limits
        cells = np.ascontiguousarray(cells, np.uint16)
        init = np.asarray(initial, np.float64)
        pts = np.ascontiguousarray(cloud, np.float32)
        pose = np.zeros(3)
        ncand = C.c_int64()
        s = self.lib.oracle_rt2d_match(res, mx, my, cells.shape[1], cells.shape[0],
                                       _p(cells, C.c_uint16), *opts, _p(init, D), _p(pts, F),
                                       len(pts), _p(pose, D), C.byref(ncand))
        return s, tuple(pose), ncand.value

    def rt2d_time(self, limits, cells, opts, initial, cloud, reps):
        res, mx, my = limits
        cells = np.ascontiguousarray(cells, np.uint16)
        init = np.asarray(initial, np.float64)
        pts = np.ascontiguousarray(cloud, np.float32)
        return self.lib.oracle_rt2d_time(res, mx, my, cells.shape[1], cells.shape[0],
                                         _p(cells, C.c_uint16), *opts, _p(init, D), _p(pts, F),
                                         len(pts), reps)


class OracleFast2D:
    def __init__(self, o, handle, limits, lin, ang):
        self.o, self.h, self.limits, self.lin, self.ang = o, handle, limits, lin, ang

    def __del__(self):
        try:
            self.o.lib.oracle_fast2d_destroy(self.h)
        except Exception:
            pass

    def level(self, d):
        wnx, wny = C.c_int32(), C.c_int32()
        n = self.o.lib.oracle_fast2d_level(self.h, d, None, C.byref(wnx), C.byref(wny))
        out = np.zeros((wny.value, wnx.value), np.uint8)
        self.o.lib.oracle_fast2d_level(self.h, d, _p(out, C.c_uint8), C.byref(wnx), C.byref(wny))
        assert out.size == n
        return out

    def match_full_submap(self, cloud, min_score):
        pts = np.ascontiguousarray(cloud, np.float32)
        score, pose, stats = C.c_float(), np.zeros(3), np.zeros(16, np.int64)
        r = self.o.lib.oracle_fast2d_match_full_submap(self.h, _p(pts, F), len(pts), min_score,
                                                       C.byref(score), _p(pose, D), _p(stats, I64))
        return r == 0, score.value, tuple(pose), stats

    def match(self, initial, cloud, min_score):
        pts = np.ascontiguousarray(cloud, np.float32)
        init = np.asarray(initial, np.float64)
        score, pose, stats = C.c_float(), np.zeros(3), np.zeros(16, np.int64)
        r = self.o.lib.oracle_fast2d_match(self.h, _p(init, D), _p(pts, F), len(pts), min_score,
                                           C.byref(score), _p(pose, D), _p(stats, I64))
        return r == 0, score.value, tuple(pose), stats

    def tie_leaves(self, full_submap, initial, cloud, min_score, max_out=4096):
        """Leaves tied at the maximum score as (scan, x_off, y_off) rows, and
        the reference's pick among them (None, None if no match)."""
        pts = np.ascontiguousarray(cloud, np.float32)
        init = np.asarray(initial if initial is not None else (0, 0, 0), np.float64)
        out = np.zeros((max_out, 3), np.int32)
        pick = np.zeros(3, np.int32)
        k = self.o.lib.oracle_fast2d_tie_leaves(self.h, 1 if full_submap else 0, _p(init, D),
                                                _p(pts, F), len(pts), min_score, max_out,
                                                _p(out, I32), _p(pick, I32))
        if k == 0:
            return None, None
        return out[:k].copy(), tuple(int(v) for v in pick)

    def score_candidate(self, full_submap, initial, cloud, scan_index, x_off, y_off, depth=0):
        pts = np.ascontiguousarray(cloud, np.float32)
        init = np.asarray(initial if initial is not None else (0, 0, 0), np.float64)
        s, sc = C.c_int32(), C.c_float()
        r = self.o.lib.oracle_fast2d_score_candidate(self.h, 1 if full_submap else 0, _p(init, D),
                                                     self.lin, self.ang, _p(pts, F), len(pts),
                                                     scan_index, x_off, y_off, depth, C.byref(s),
                                                     C.byref(sc))
        assert r == 0
        return s.value, sc.value


# ---------------------------------------------------------------------- 3D --
_SIG3D = {
    "oracle_hgrid_create": (VP, [F]),
    "oracle_hgrid_destroy": (None, [VP]),
    "oracle_hgrid_set_probability": (None, [VP, I32, I32, I32, F]),
    "oracle_hgrid_insert": (None, [VP, F, F, I32, P(F), P(F), I32]),
    "oracle_hgrid_set_values": (None, [VP, P(I32), P(C.c_uint16), I64]),
    "oracle_hgrid_cells": (I64, [VP, P(I32), P(C.c_uint16), I64]),
    "oracle_hgrid_grid_size": (I32, [VP]),
    "oracle_hgrid_probability": (F, [VP, I32, I32, I32]),
    "oracle_hgrid_interpolate": (None, [VP, P(D), I64, P(D)]),
    "oracle_hgrid_cell_index": (None, [VP, P(F), I64, P(I32)]),
    "oracle_histogram": (None, [P(F), I32, I32, P(F)]),
    "oracle_rotational_match": (None, [P(F), P(F), I32, F, P(F), I32, P(F)]),
    "oracle_fast3d_create": (VP, [VP, VP, P(F), I32, P(D)]),
    "oracle_fast3d_destroy": (None, [VP]),
    "oracle_fast3d_level": (I64, [VP, I32, P(I32), P(C.c_uint8), I64]),
    "oracle_fast3d_match": (None, [VP, P(D), P(D), P(F), I32, P(F), I32, P(F), I32, P(D), F,
                                   P(D)]),
    "oracle_fast3d_match_full_submap": (None, [VP, P(D), P(D), P(F), I32, P(F), I32, P(F), I32,
                                               P(D), F, P(D)]),
    "oracle_fast3d_evaluate_leaf": (I32, [VP, I32, P(D), P(D), P(F), I32, P(F), I32, P(F), I32,
                                          P(D), P(D), P(D)]),
    "oracle_rt3d_match": (None, [VP, P(D), P(D), P(F), I32, P(D)]),
    "oracle_rt3d_score": (F, [VP, P(D), P(D), P(F), I32, I64, P(D)]),
    "oracle_rt3d_window": (None, [P(D), F, P(F), I32, P(I32), P(F), P(I32)]),
    "oracle_fast3d_match_pairs": (D, [P(VP), P(F), P(I64), P(F), P(I64), P(F), I32, P(D),
                                      P(I32), P(I32), I64, I32, F, P(I32), P(D), P(D)]),
    "oracle_rt3d_time": (D, [VP, P(D), P(D), P(F), I32, I64, I64]),
}


def _pose7(t=(0, 0, 0), q=(1, 0, 0, 0)):
    return np.array(list(t) + list(q), np.float64)


class OracleHybridGrid:
    def __init__(self, o, resolution):
        self.o = o
        self.resolution = resolution
        self.h = o.lib.oracle_hgrid_create(resolution)

    def __del__(self):
        try:
            self.o.lib.oracle_hgrid_destroy(self.h)
        except Exception:
            pass

    def set_probability(self, x, y, z, p):
        self.o.lib.oracle_hgrid_set_probability(self.h, x, y, z, p)

    def insert(self, origin, returns, hit=0.7, miss=0.4, num_free_space_voxels=5):
        org = np.asarray(origin, np.float32)
        r = np.ascontiguousarray(returns, np.float32).reshape(-1, 3)
        self.o.lib.oracle_hgrid_insert(self.h, hit, miss, num_free_space_voxels, _p(org, F),
                                       _p(r, F), len(r))

    def set_values(self, ijk, values):
        ijk = np.ascontiguousarray(ijk, np.int32).reshape(-1, 3)
        v = np.ascontiguousarray(values, np.uint16)
        self.o.lib.oracle_hgrid_set_values(self.h, _p(ijk, I32), _p(v, C.c_uint16), len(v))

    def cells(self):
        n = self.o.lib.oracle_hgrid_cells(self.h, None, None, 0)
        ijk = np.zeros((n, 3), np.int32)
        v = np.zeros(n, np.uint16)
        self.o.lib.oracle_hgrid_cells(self.h, _p(ijk, I32), _p(v, C.c_uint16), n)
        return ijk, v

    @property
    def grid_size(self):
        return self.o.lib.oracle_hgrid_grid_size(self.h)

    def probability(self, x, y, z):
        return self.o.lib.oracle_hgrid_probability(self.h, x, y, z)

    def interpolate(self, points):
        xyz = np.ascontiguousarray(np.asarray(points, np.float64).reshape(-1, 3))
        out = np.zeros(len(xyz))
        self.o.lib.oracle_hgrid_interpolate(self.h, _p(xyz, D), len(xyz), _p(out, D))
        return out

    def cell_index(self, points):
        xyz = np.ascontiguousarray(np.asarray(points, np.float32).reshape(-1, 3))
        out = np.zeros((len(xyz), 3), np.int32)
        self.o.lib.oracle_hgrid_cell_index(self.h, _p(xyz, F), len(xyz), _p(out, I32))
        return out


class OracleFast3D:
    def __init__(self, o, high, low, histogram, options):
        self.o, self.high, self.low = o, high, low
        self.hist = np.ascontiguousarray(histogram, np.float32)
        opts = np.array(options, np.float64)
        self.h = o.lib.oracle_fast3d_create(high.h, low.h, _p(self.hist, F), len(self.hist),
                                            _p(opts, D))

    def __del__(self):
        try:
            self.o.lib.oracle_fast3d_destroy(self.h)
        except Exception:
            pass

    def level(self, d):
        n = self.o.lib.oracle_fast3d_level(self.h, d, None, None, 0)
        ijk = np.zeros((n, 3), np.int32)
        v = np.zeros(n, np.uint8)
        self.o.lib.oracle_fast3d_level(self.h, d, _p(ijk, I32), _p(v, C.c_uint8), n)
        return ijk, v

    @staticmethod
    def _node(node):
        hi = np.ascontiguousarray(node.high_resolution_point_cloud, np.float32).reshape(-1, 3)
        lo = np.ascontiguousarray(node.low_resolution_point_cloud, np.float32).reshape(-1, 3)
        hist = np.ascontiguousarray(node.rotational_scan_matcher_histogram, np.float32)
        g = np.asarray(node.gravity_alignment, np.float64)
        return hi, lo, hist, g

    @staticmethod
    def _out(out):
        return {"matched": bool(out[0]), "score": float(np.float32(out[1])),
                "rotational_score": float(np.float32(out[2])),
                "low_resolution_score": float(np.float32(out[3])),
                "pose": (tuple(out[4:7]), tuple(out[7:11])), "lookups": int(out[11]),
                "low_resolution_checks": int(out[12]), "num_discrete_scans": int(out[13])}

    def match(self, node_pose, submap_pose, node, min_score):
        hi, lo, hist, g = self._node(node)
        a = _pose7(*node_pose)
        b = _pose7(*submap_pose)
        out = np.zeros(14)
        self.o.lib.oracle_fast3d_match(self.h, _p(a, D), _p(b, D), _p(hi, F), len(hi), _p(lo, F),
                                       len(lo), _p(hist, F), len(hist), _p(g, D), min_score,
                                       _p(out, D))
        return self._out(out)

    def evaluate_leaf(self, full_submap, node_pose, submap_pose, node, pose):
        """The leaf behind `pose` ((t), (q)): dict like match(), or None."""
        hi, lo, hist, g = self._node(node)
        a = _pose7(*node_pose)
        b = _pose7(*submap_pose)
        p = _pose7(*pose)
        out = np.zeros(14)
        ok = self.o.lib.oracle_fast3d_evaluate_leaf(self.h, 1 if full_submap else 0, _p(a, D),
                                                    _p(b, D), _p(hi, F), len(hi), _p(lo, F),
                                                    len(lo), _p(hist, F), len(hist), _p(g, D),
                                                    _p(p, D), _p(out, D))
        return self._out(out) if ok else None

    def match_full_submap(self, node_q, submap_q, node, min_score):
        hi, lo, hist, g = self._node(node)
        a = np.asarray(node_q, np.float64)
        b = np.asarray(submap_q, np.float64)
        out = np.zeros(14)
        self.o.lib.oracle_fast3d_match_full_submap(self.h, _p(a, D), _p(b, D), _p(hi, F), len(hi),
                                                   _p(lo, F), len(lo), _p(hist, F), len(hist),
                                                   _p(g, D), min_score, _p(out, D))
        return self._out(out)


def _bind3d(lib):
    for name, (res, args) in _SIG3D.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args


def _o3_hgrid(self, resolution):
    if not getattr(self, "_bound3d", False):
        _bind3d(self.lib)
        self._bound3d = True
    return OracleHybridGrid(self, resolution)


def _o3_fast3d(self, high, low, histogram, options):
    _o3_hgrid(self, 1.0)  # binds
    return OracleFast3D(self, high, low, histogram, options)


def _o3_histogram(self, cloud, size):
    _o3_hgrid(self, 1.0)
    pts = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
    out = np.zeros(size, np.float32)
    self.lib.oracle_histogram(_p(pts, F), len(pts), size, _p(out, F))
    return out


def _o3_rt3d_match(self, grid, options, initial, cloud):
    _o3_hgrid(self, 1.0)
    pts = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
    o = np.asarray(options, np.float64)
    init = _pose7(*initial)
    out = np.zeros(10)
    self.lib.oracle_rt3d_match(grid.h, _p(o, D), _p(init, D), _p(pts, F), len(pts), _p(out, D))
    return (float(np.float32(out[0])), (tuple(out[1:4]), tuple(out[4:8])), int(out[8]),
            int(out[9]))


def _o3_rt3d_score(self, grid, options, initial, cloud, index):
    _o3_hgrid(self, 1.0)
    pts = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
    o = np.asarray(options, np.float64)
    init = _pose7(*initial)
    pose = np.zeros(7)
    s = self.lib.oracle_rt3d_score(grid.h, _p(o, D), _p(init, D), _p(pts, F), len(pts), index,
                                   _p(pose, D))
    return float(s), (tuple(pose[:3]), tuple(pose[3:]))


Oracle.hybrid_grid = _o3_hgrid
Oracle.fast3d = _o3_fast3d
Oracle.histogram = _o3_histogram
Oracle.rt3d_match = _o3_rt3d_match
Oracle.rt3d_score = _o3_rt3d_score


# ---- voxel filters (oracle/voxel_filter.cc) ------------------------------
def _pack_clouds(clouds):
    arrs = [np.ascontiguousarray(np.asarray(c, np.float32).reshape(-1, 3)) for c in clouds]
    offsets = np.zeros(len(arrs) + 1, np.int64)
    offsets[1:] = np.cumsum([len(a) for a in arrs])
    pts = np.ascontiguousarray(np.concatenate(arrs) if arrs else np.zeros((0, 3), np.float32))
    return pts, offsets


def _o_voxel_filter_masks(self, clouds, resolution):
    pts, offsets = _pack_clouds(clouds)
    keep = np.zeros(max(len(pts), 1), np.uint8)
    self.lib.oracle_voxel_filter(_p(pts, F), _p(offsets, I64), len(offsets) - 1,
                                 float(resolution), _p(keep, C.c_uint8))
    return keep[:len(pts)].astype(bool), offsets


def _o_adaptive_voxel_filter_masks(self, clouds, max_length, min_num_points, max_range):
    pts, offsets = _pack_clouds(clouds)
    keep = np.zeros(max(len(pts), 1), np.uint8)
    self.lib.oracle_adaptive_voxel_filter(_p(pts, F), _p(offsets, I64), len(offsets) - 1,
                                          float(max_length), float(min_num_points),
                                          float(max_range), _p(keep, C.c_uint8))
    return keep[:len(pts)].astype(bool), offsets


Oracle.voxel_filter_masks = _o_voxel_filter_masks
Oracle.adaptive_voxel_filter_masks = _o_adaptive_voxel_filter_masks


def _o_ceres2d_match(self, limits, cells, options, target, initial, cloud,
                     min_cc=None, max_cc=None):
    """CeresScanMatcher2D::Match restated (oracle/ceres2d.cc): (pose, iterations).
    options: (occupied, translation, rotation weights, max_num_iterations
    [, use_nonmonotonic_steps = True as pose_graph.lua:35])."""
    # probability_values.h: kMinCorrespondenceCost = 1.f - kMaxProbability,
    # kMaxCorrespondenceCost = 1.f - kMinProbability, in float.
    f32 = np.float32
    if min_cc is None:
        min_cc = f32(1.0) - (f32(1.0) - f32(0.1))
    if max_cc is None:
        max_cc = f32(1.0) - f32(0.1)
    cells = np.ascontiguousarray(cells, np.uint16)
    pts = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
    o = np.asarray(tuple(options) + ((1.0,) if len(options) == 4 else ()), np.float64)
    t = np.asarray(target, np.float64)
    i = np.asarray(initial, np.float64)
    out = np.zeros(3)
    it = self.lib.oracle_ceres2d_match(limits[0], limits[1], limits[2], cells.shape[1],
                                       cells.shape[0], _p(cells, C.c_uint16),
                                       float(np.float32(min_cc)), float(np.float32(max_cc)),
                                       _p(o, D), _p(t, D), _p(i, D), _p(pts, F), len(pts),
                                       _p(out, D))
    return tuple(out), int(it)


Oracle.ceres2d_match = _o_ceres2d_match


def _o_ceres3d_match(self, high, low, high_cloud, low_cloud, options, target, initial_t,
                     initial_q):
    """CeresScanMatcher3D::Match restated (oracle/ceres3d.cc): ((t, q), iterations).
    high / low: OracleHybridGrid objects; q as (w, x, y, z)."""
    _o3_hgrid(self, 1.0)  # binds the 3D signatures
    f = self.lib.oracle_ceres3d_match
    f.restype = I32
    f.argtypes = [VP, VP, P(F), I32, P(F), I32, P(D), P(D), P(D), P(D)]
    hc = np.ascontiguousarray(high_cloud, np.float32).reshape(-1, 3)
    lc = np.ascontiguousarray(low_cloud, np.float32).reshape(-1, 3)
    # (w0, w1, translation, rotation, max_num_iterations [, nonmonotonic = 0])
    o = np.asarray(tuple(options) + ((0.0,) if len(options) == 5 else ()), np.float64)
    t = np.asarray(target, np.float64)
    init = np.concatenate([np.asarray(initial_t, np.float64), np.asarray(initial_q, np.float64)])
    out = np.zeros(7)
    it = f(high.h, low.h, _p(hc, F), len(hc), _p(lc, F), len(lc), _p(o, D), _p(t, D),
           _p(init, D), _p(out, D))
    return (tuple(out[:3]), tuple(out[3:])), int(it)


Oracle.ceres3d_match = _o_ceres3d_match


def _o_search_parameters(self, lin, ang, cloud, res):
    """SearchParameters(lin, ang, cloud, res) restated: (num_angular, step,
    num_scans, first scan's bounds)."""
    pts = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
    na, ns = C.c_int32(), C.c_int32()
    step = C.c_double()
    b = np.zeros(4, np.int32)
    self.lib.oracle_search_parameters(lin, ang, _p(pts, F), len(pts), res, C.byref(na),
                                      C.byref(step), C.byref(ns), _p(b, I32))
    return na.value, step.value, ns.value, tuple(int(v) for v in b)


def _o_generate_rotated_scans(self, cloud, num_linear, num_angular, step, res):
    pts = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
    out = np.zeros((2 * num_angular + 1, len(pts), 3), np.float32)
    self.lib.oracle_generate_rotated_scans(_p(pts, F), len(pts), num_linear, num_angular, step,
                                           res, _p(out, F))
    return out


def _o_discretize_scans(self, limits, scans, tx, ty):
    """limits: (res, max_x, max_y, nx, ny); scans (num_scans, n, 3)."""
    sc = np.ascontiguousarray(scans, np.float32)
    out = np.zeros((sc.shape[0], sc.shape[1], 2), np.int32)
    self.lib.oracle_discretize_scans(limits[0], limits[1], limits[2], limits[3], limits[4],
                                     _p(sc, F), sc.shape[1], sc.shape[0], float(np.float32(tx)),
                                     float(np.float32(ty)), _p(out, I32))
    return out


def _o_rt2d_score_candidates(self, limits, cells, wt, wr, discrete, num_angular, step, cands,
                             tsdf=None):
    """ScoreCandidates restated; cands (k, 3) (scan, x_off, y_off). tsdf:
    (weight_cells, truncation, max_weight) for a TSDF2D (cells = tsd cells)."""
    d = np.ascontiguousarray(discrete, np.int32)
    c = np.ascontiguousarray(cands, np.int32).reshape(-1, 3)
    cells = np.ascontiguousarray(cells, np.uint16)
    out = np.zeros(len(c), np.float32)
    if tsdf is None:
        self.lib.oracle_rt2d_score_candidates(limits[0], limits[1], limits[2], limits[3],
                                              limits[4], _p(cells, C.c_uint16), wt, wr,
                                              _p(d, I32), d.shape[0], d.shape[1], num_angular,
                                              step, _p(c, I32), len(c), _p(out, F))
    else:
        w = np.ascontiguousarray(tsdf[0], np.uint16)
        self.lib.oracle_rt2d_score_candidates_tsdf(limits[0], limits[1], limits[2], limits[3],
                                                   limits[4], _p(cells, C.c_uint16),
                                                   _p(w, C.c_uint16), tsdf[1], tsdf[2], wt, wr,
                                                   _p(d, I32), d.shape[0], d.shape[1],
                                                   num_angular, step, _p(c, I32), len(c),
                                                   _p(out, F))
    return out


Oracle.search_parameters = _o_search_parameters
Oracle.generate_rotated_scans = _o_generate_rotated_scans
Oracle.discretize_scans = _o_discretize_scans
Oracle.rt2d_score_candidates = _o_rt2d_score_candidates


def _o_discretize(self, limits, cells, initial, lin, ang, cloud, rotated_sp=False):
    """The matchers' whole window pipeline restated (oracle_discretize):
    SearchParameters, rotated scans, DiscretizeScans at the initial pose and
    ShrinkToFit. Returns (num_scans, shrunk bounds (num_scans, 4),
    discrete scans (num_scans, n, 2), step)."""
    res, mx, my = limits
    pts = np.ascontiguousarray(cloud, np.float32).reshape(-1, 3)
    init = np.asarray(initial, np.float64)
    ns, step = C.c_int32(), C.c_double()
    args = (res, mx, my, cells.shape[1], cells.shape[0], _p(init, D), lin, ang, _p(pts, F),
            len(pts), int(rotated_sp), C.byref(ns))
    self.lib.oracle_discretize(*args, None, None, 0, C.byref(step))
    bounds = np.zeros((ns.value, 4), np.int32)
    out = np.zeros((ns.value, len(pts), 2), np.int32)
    rc = self.lib.oracle_discretize(*args, _p(bounds, I32), _p(out, I32), out.size,
                                    C.byref(step))
    assert rc == 0
    return ns.value, bounds, out, step.value


Oracle.discretize = _o_discretize
