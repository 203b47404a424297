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
            "oracle_fast2d_match_pairs": (D, [P(VP), P(F), P(I64), P(I32), P(I32), I64, I32, F,
                                              P(F), P(D), P(I32)]),
            "oracle_rt2d_match": (D, [D, D, D, I32, I32, P(C.c_uint16), D, D, D, D, P(D), P(F),
                                      I32, P(D), P(I64)]),
            "oracle_rt2d_time": (D, [D, D, D, I32, I32, P(C.c_uint16), D, D, D, D, P(D), P(F),
                                     I32, I32]),
            "oracle_discretize": (I32, [D, D, D, I32, I32, P(D), D, D, P(F), I32, I32, P(I32),
                                        P(I32), P(I32), I64, P(D)]),
            "oracle_grid_create": (VP, [D, D, D, I32, I32]),
            "oracle_grid_destroy": (None, [VP]),
            "oracle_grid_insert": (None, [VP, F, F, I32, P(F), P(F), I32]),
            "oracle_grid_set_probability": (None, [VP, I32, I32, F]),
            "oracle_grid_info": (None, [VP, P(D), P(I32)]),
            "oracle_grid_cells": (None, [VP, P(C.c_uint16)]),
            "oracle_transform_cloud_2d": (None, [P(F), P(F), I32, P(F)]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        self.lib = lib

    # ---- grids ---------------------------------------------------------
    def grid_from_inserts(self, res, max_x, max_y, nx, ny, inserts, hit=0.7, miss=0.4):
        """Grid built with the restated ProbabilityGridRangeDataInserter2D.
        inserts: list of (origin xyz, returns (n,3)). Returns (limits, cells)."""
        g = self.lib.oracle_grid_create(res, max_x, max_y, nx, ny)
        try:
            for origin, ret in inserts:
                o = np.asarray(origin, np.float32)
                r = np.ascontiguousarray(ret, np.float32)
                self.lib.oracle_grid_insert(g, hit, miss, 1, _p(o, F), _p(r, F), len(r))
            return self._grid_out(g)
        finally:
            self.lib.oracle_grid_destroy(g)

    def grid_from_probabilities(self, res, max_x, max_y, nx, ny, cells_xy_p):
        g = self.lib.oracle_grid_create(res, max_x, max_y, nx, ny)
        try:
            for x, y, p in cells_xy_p:
                self.lib.oracle_grid_set_probability(g, int(x), int(y), float(p))
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
