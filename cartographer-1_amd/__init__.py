"""MI355X-native correlative scan matching — Python host mirror.

Thin ctypes layer over ``libcsm_amd.so`` (C-ABI: ``include/csm_amd.h``) that
mirrors the reference's operator interface so tests and benchmarks read like
the reference's own code:

* :class:`FastCorrelativeScanMatcher2D` — ``Match`` / ``MatchFullSubmap``
  (reference ``mapping/internal/2d/scan_matching/fast_correlative_scan_matcher_2d.h:112-164``)
* :class:`RealTimeCorrelativeScanMatcher2D` — ``Match``
  (``real_time_correlative_scan_matcher_2d.h:53-85``)
* :func:`match_batch` — the batched constraint search that replaces one
  ``ConstraintBuilder2D`` task per (node, submap) pair
  (``constraints/constraint_builder_2d.cc:77-137``)

There is no CPU fallback: every compute call runs the HIP kernels, and loading
fails loudly when the extension is missing. PyTorch is not used here.
"""

from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass
from typing import Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CSM_AMD_LIB points experiments (e.g. a CSM_KPROF build) at another build of
# the same library; the default is the in-tree build.
LIB_PATH = os.environ.get("CSM_AMD_LIB") or os.path.join(_HERE, "libcsm_amd.so")
SYNTH_PATH = os.path.join(_HERE, "libcsm_synth.so")

CSM_OK = 0
CSM_NO_MATCH = 1
CSM_EINVAL = -1
CSM_EHIP = -2
CSM_ENOMEM = -3
CSM_ERANGE = -4


class CsmError(RuntimeError):
    """A negative return code from the C-ABI (the reference would CHECK-fail)."""


class MapLimits(C.Structure):
    _fields_ = [("resolution", C.c_double), ("max_x", C.c_double), ("max_y", C.c_double),
                ("num_x_cells", C.c_int32), ("num_y_cells", C.c_int32)]


class Pose2D(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("theta", C.c_double)]

    def as_tuple(self) -> Tuple[float, float, float]:
        return (self.x, self.y, self.theta)


class Fast2DOptions(C.Structure):
    _fields_ = [("linear_search_window", C.c_double), ("angular_search_window", C.c_double),
                ("branch_and_bound_depth", C.c_int32), ("search_depth", C.c_int32)]


class RtOptions(C.Structure):
    _fields_ = [("linear_search_window", C.c_double), ("angular_search_window", C.c_double),
                ("translation_delta_cost_weight", C.c_double),
                ("rotation_delta_cost_weight", C.c_double)]


class Pair2D(C.Structure):
    _fields_ = [("submap", C.c_int32), ("scan", C.c_int32), ("full_submap", C.c_int32),
                ("min_score", C.c_float), ("initial", Pose2D)]


class Result2D(C.Structure):
    _fields_ = [("status", C.c_int32), ("score", C.c_float), ("pose", Pose2D),
                ("tie", C.c_int32), ("reserved", C.c_int32)]


# csm_result2d.tie: how a result was picked among exactly tied maxima.
TIE_NONE, TIE_ANCESTORS, TIE_TOPLIST, TIE_WALK = 0, 1, 2, 3


class Timing(C.Structure):
    _fields_ = [("search_kernel_ms", C.c_double), ("search_launches", C.c_int64),
                ("search_lookups", C.c_double), ("search_candidates", C.c_double),
                ("other_kernel_ms", C.c_double), ("rt3d_kernel_ms", C.c_double),
                ("rt3d_lookups", C.c_double), ("fast3d_kernel_ms", C.c_double),
                ("fast3d_launches", C.c_int64), ("fast3d_lookups", C.c_double),
                ("search_errors", C.c_int64), ("stack_high_water", C.c_int64),
                ("tied_pairs", C.c_int64), ("ties_walked", C.c_int64),
                ("ties_toplist", C.c_int64), ("tied_pairs_3d", C.c_int64),
                ("ties_walked_3d", C.c_int64)]


class Pose3D(C.Structure):
    """transform::Rigid3d: t (x, y, z) and q (w, x, y, z)."""
    _fields_ = [("t", C.c_double * 3), ("q", C.c_double * 4)]

    @staticmethod
    def make(t=(0.0, 0.0, 0.0), q=(1.0, 0.0, 0.0, 0.0)) -> "Pose3D":
        p = Pose3D()
        p.t[:] = [float(v) for v in t]
        p.q[:] = [float(v) for v in q]
        return p

    def as_tuple(self):
        return tuple(self.t), tuple(self.q)


class Fast3DOptions(C.Structure):
    _fields_ = [("branch_and_bound_depth", C.c_int32), ("full_resolution_depth", C.c_int32),
                ("min_rotational_score", C.c_double), ("min_low_resolution_score", C.c_double),
                ("linear_xy_search_window", C.c_double), ("linear_z_search_window", C.c_double),
                ("angular_search_window", C.c_double)]


class Node3D(C.Structure):
    _fields_ = [("high_resolution_xyz", C.POINTER(C.c_float)),
                ("num_high_resolution", C.c_int32),
                ("low_resolution_xyz", C.POINTER(C.c_float)), ("num_low_resolution", C.c_int32),
                ("histogram", C.POINTER(C.c_float)), ("histogram_size", C.c_int32),
                ("gravity_alignment", C.c_double * 4)]


class Result3D(C.Structure):
    _fields_ = [("status", C.c_int32), ("score", C.c_float), ("pose", Pose3D),
                ("rotational_score", C.c_float), ("low_resolution_score", C.c_float),
                ("tie", C.c_int32), ("reserved", C.c_int32)]


class CeresOptions2D(C.Structure):
    """proto::CeresScanMatcherOptions2D; defaults pose_graph.lua:30-39
    (ceres_solver_options: max_num_iterations 10, use_nonmonotonic_steps)."""
    _fields_ = [("occupied_space_weight", C.c_double), ("translation_weight", C.c_double),
                ("rotation_weight", C.c_double), ("max_num_iterations", C.c_int32),
                ("use_nonmonotonic_steps", C.c_int32)]

    @staticmethod
    def make(occupied_space_weight=20.0, translation_weight=10.0, rotation_weight=1.0,
             max_num_iterations=10, use_nonmonotonic_steps=True) -> "CeresOptions2D":
        return CeresOptions2D(occupied_space_weight, translation_weight, rotation_weight,
                              max_num_iterations, int(bool(use_nonmonotonic_steps)))


class CeresOptions3D(C.Structure):
    """proto::CeresScanMatcherOptions3D; defaults pose_graph.lua:49-60
    (ceres_solver_options: max_num_iterations 10, monotonic steps)."""
    _fields_ = [("occupied_space_weight_0", C.c_double), ("occupied_space_weight_1", C.c_double),
                ("translation_weight", C.c_double), ("rotation_weight", C.c_double),
                ("max_num_iterations", C.c_int32), ("use_nonmonotonic_steps", C.c_int32)]

    @staticmethod
    def make(w0=5.0, w1=30.0, translation_weight=10.0, rotation_weight=1.0,
             max_num_iterations=10, use_nonmonotonic_steps=False) -> "CeresOptions3D":
        return CeresOptions3D(w0, w1, translation_weight, rotation_weight, max_num_iterations,
                              int(bool(use_nonmonotonic_steps)))


class Refine3D(C.Structure):
    _fields_ = [("high_grid", C.c_int32), ("low_grid", C.c_int32), ("node", C.c_int32),
                ("initial", Pose3D), ("target", C.c_double * 3)]


class Refine2D(C.Structure):
    _fields_ = [("submap", C.c_int32), ("scan", C.c_int32), ("initial", Pose2D),
                ("target_x", C.c_double), ("target_y", C.c_double)]


class AdaptiveVoxelFilterOptions(C.Structure):
    """proto::AdaptiveVoxelFilterOptions (all floats); defaults are
    trajectory_builder_2d.lua:25-29's adaptive_voxel_filter."""
    _fields_ = [("max_length", C.c_float), ("min_num_points", C.c_float),
                ("max_range", C.c_float)]

    @staticmethod
    def make(max_length=0.5, min_num_points=200, max_range=50.0) -> "AdaptiveVoxelFilterOptions":
        return AdaptiveVoxelFilterOptions(max_length, min_num_points, max_range)


class LinearBounds(C.Structure):
    """SearchParameters::LinearBounds (correlative_scan_matcher_2d.h:37-42)."""
    _fields_ = [("min_x", C.c_int32), ("max_x", C.c_int32), ("min_y", C.c_int32),
                ("max_y", C.c_int32)]

    def as_tuple(self):
        return (self.min_x, self.max_x, self.min_y, self.max_y)


class SearchParametersC(C.Structure):
    _fields_ = [("num_angular_perturbations", C.c_int32),
                ("angular_perturbation_step_size", C.c_double), ("resolution", C.c_double),
                ("num_scans", C.c_int32), ("num_linear_perturbations", C.c_int32)]


class Candidate2DC(C.Structure):
    _fields_ = [("scan_index", C.c_int32), ("x_index_offset", C.c_int32),
                ("y_index_offset", C.c_int32), ("score", C.c_float)]


class Pair3D(C.Structure):
    _fields_ = [("submap", C.c_int32), ("node", C.c_int32), ("full_submap", C.c_int32),
                ("min_score", C.c_float), ("node_pose", Pose3D), ("submap_pose", Pose3D)]


# Exported symbols and their signatures (include/csm_amd.h).
_SIGNATURES = {
    "csm_context_create": (C.c_int, [C.c_int32, C.POINTER(C.c_void_p)]),
    "csm_context_destroy": (None, [C.c_void_p]),
    "csm_context_stream": (C.c_void_p, [C.c_void_p]),
    "csm_context_enable_timing": (None, [C.c_void_p, C.c_int32]),
    "csm_context_get_timing": (None, [C.c_void_p, C.POINTER(Timing)]),
    "csm_context_reset_timing": (None, [C.c_void_p]),
    "csm_context_level_stats": (C.c_int32, [C.c_void_p, C.POINTER(C.c_double),
                                            C.POINTER(C.c_double), C.c_int32]),
    "csm_fast2d_create": (C.c_int, [C.c_void_p, C.POINTER(MapLimits), C.POINTER(C.c_uint16),
                                    C.c_float, C.c_float, C.POINTER(Fast2DOptions),
                                    C.POINTER(C.c_void_p)]),
    "csm_fast2d_destroy": (None, [C.c_void_p]),
    "csm_fast2d_match": (C.c_int, [C.c_void_p, C.POINTER(Pose2D), C.POINTER(C.c_float),
                                   C.c_int32, C.c_float, C.POINTER(C.c_float),
                                   C.POINTER(Pose2D)]),
    "csm_fast2d_match_full_submap": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.c_int32,
                                               C.c_float, C.POINTER(C.c_float),
                                               C.POINTER(Pose2D)]),
    "csm_fast2d_device_bytes": (C.c_int64, [C.c_void_p]),
    "csm_fast3d_device_bytes": (C.c_int64, [C.c_void_p]),
    "csm_hybrid_grid_device_bytes": (C.c_int64, [C.c_void_p]),
    "csm_fast2d_read_level": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_uint8), C.c_int64,
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "csm_scan_set_create": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int64),
                                      C.c_int32, C.POINTER(C.c_void_p)]),
    "csm_scan_set_destroy": (None, [C.c_void_p]),
    "csm_scan_set_append": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int64),
                                      C.c_int32, C.POINTER(C.c_int32)]),
    "csm_scan_set_size": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64)]),
    "csm_fast2d_match_batch": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                         C.c_void_p, C.POINTER(Pair2D), C.c_int64,
                                         C.POINTER(Result2D)]),
    "csm_rt2d_match": (C.c_int, [C.c_void_p, C.POINTER(RtOptions), C.POINTER(MapLimits),
                                 C.POINTER(C.c_uint16), C.c_float, C.c_float, C.POINTER(Pose2D),
                                 C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_double),
                                 C.POINTER(Pose2D)]),
    "csm_rt2d_match_tsdf": (C.c_int, [C.c_void_p, C.POINTER(RtOptions), C.POINTER(MapLimits),
                                      C.POINTER(C.c_uint16), C.POINTER(C.c_uint16), C.c_float,
                                      C.c_float, C.POINTER(Pose2D), C.POINTER(C.c_float),
                                      C.c_int32, C.POINTER(C.c_double), C.POINTER(Pose2D)]),
    "csm_search_parameters_init": (C.c_int, [C.c_double, C.c_double, C.POINTER(C.c_float),
                                             C.c_int32, C.c_double,
                                             C.POINTER(SearchParametersC)]),
    "csm_search_parameters_init_for_testing": (C.c_int, [C.c_int32, C.c_int32, C.c_double,
                                                         C.c_double,
                                                         C.POINTER(SearchParametersC)]),
    "csm_search_parameters_shrink_to_fit": (C.c_int, [C.POINTER(SearchParametersC),
                                                      C.POINTER(C.c_int32), C.c_int32, C.c_int32,
                                                      C.c_int32, C.POINTER(LinearBounds)]),
    "csm_generate_rotated_scans": (C.c_int, [C.POINTER(C.c_float), C.c_int32,
                                             C.POINTER(SearchParametersC), C.POINTER(C.c_float)]),
    "csm_discretize_scans": (C.c_int, [C.POINTER(MapLimits), C.POINTER(C.c_float), C.c_int32,
                                       C.c_int32, C.c_float, C.c_float, C.POINTER(C.c_int32)]),
    "csm_rt2d_score_candidates": (C.c_int, [C.c_void_p, C.POINTER(RtOptions),
                                            C.POINTER(MapLimits), C.POINTER(C.c_uint16),
                                            C.c_float, C.c_float, C.POINTER(C.c_int32),
                                            C.c_int32, C.c_int32, C.POINTER(SearchParametersC),
                                            C.POINTER(Candidate2DC), C.c_int64]),
    "csm_rt2d_score_candidates_tsdf": (C.c_int, [C.c_void_p, C.POINTER(RtOptions),
                                                 C.POINTER(MapLimits), C.POINTER(C.c_uint16),
                                                 C.POINTER(C.c_uint16), C.c_float, C.c_float,
                                                 C.POINTER(C.c_int32), C.c_int32, C.c_int32,
                                                 C.POINTER(SearchParametersC),
                                                 C.POINTER(Candidate2DC), C.c_int64]),
    "csm_hybrid_grid_create": (C.c_int, [C.c_void_p, C.c_float, C.POINTER(C.c_int32),
                                         C.POINTER(C.c_uint16), C.c_int64, C.c_int32,
                                         C.POINTER(C.c_void_p)]),
    "csm_hybrid_grid_create_batch": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_float),
                                               C.POINTER(C.POINTER(C.c_int32)),
                                               C.POINTER(C.POINTER(C.c_uint16)),
                                               C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                               C.POINTER(C.c_void_p)]),
    "csm_hybrid_grid_destroy": (None, [C.c_void_p]),
    "csm_hybrid_grid_get_probability": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.c_int64,
                                                  C.POINTER(C.c_float)]),
    "csm_hybrid_grid_interpolate": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_int64,
                                              C.POINTER(C.c_double)]),
    "csm_hybrid_grid_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                       C.POINTER(C.c_int32)]),
    "csm_rt3d_window": (C.c_int, [C.POINTER(RtOptions), C.c_float, C.POINTER(C.c_float),
                                  C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "csm_rt3d_score_rotations": (C.c_int, [C.c_void_p, C.POINTER(RtOptions), C.c_void_p,
                                           C.POINTER(Pose3D), C.POINTER(C.c_float), C.c_int32,
                                           C.POINTER(C.c_int32), C.c_int32,
                                           C.POINTER(C.c_float)]),
    "csm_rt3d_match": (C.c_int, [C.c_void_p, C.POINTER(RtOptions), C.c_void_p, C.POINTER(Pose3D),
                                 C.POINTER(C.c_float), C.c_int32, C.POINTER(C.c_float),
                                 C.POINTER(Pose3D)]),
    "csm_fast3d_create": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(C.c_float),
                                    C.c_int32, C.POINTER(Fast3DOptions), C.POINTER(C.c_void_p)]),
    "csm_fast3d_create_batch": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_void_p), C.POINTER(C.POINTER(C.c_float)),
                                          C.POINTER(C.c_int32), C.POINTER(Fast3DOptions),
                                          C.POINTER(C.c_void_p)]),
    "csm_fast3d_destroy": (None, [C.c_void_p]),
    "csm_fast3d_read_level": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_uint8), C.c_int64,
                                        C.POINTER(C.c_int32), C.POINTER(C.c_int32)]),
    "csm_fast3d_match": (C.c_int, [C.c_void_p, C.POINTER(Pose3D), C.POINTER(Pose3D),
                                   C.POINTER(Node3D), C.c_float, C.POINTER(Result3D)]),
    "csm_fast3d_match_full_submap": (C.c_int, [C.c_void_p, C.POINTER(C.c_double),
                                               C.POINTER(C.c_double), C.POINTER(Node3D),
                                               C.c_float, C.POINTER(Result3D)]),
    "csm_fast3d_match_batch": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                         C.POINTER(Node3D), C.c_int32, C.POINTER(Pair3D),
                                         C.c_int64, C.POINTER(Result3D)]),
    "csm_voxel_filter": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_int64),
                                   C.c_int32, C.c_float, C.POINTER(C.c_uint8),
                                   C.POINTER(C.c_int32)]),
    "csm_adaptive_voxel_filter": (C.c_int, [C.c_void_p, C.POINTER(C.c_float),
                                            C.POINTER(C.c_int64), C.c_int32,
                                            C.POINTER(AdaptiveVoxelFilterOptions),
                                            C.POINTER(C.c_uint8), C.POINTER(C.c_int32)]),
    "csm_voxel_filter_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                          C.c_int32, C.c_float, C.c_void_p, C.c_void_p]),
    "csm_adaptive_voxel_filter_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p,
                                                   C.c_int32, C.c_int32,
                                                   C.POINTER(AdaptiveVoxelFilterOptions),
                                                   C.c_void_p, C.c_void_p]),
    "csm_ceres2d_refine_batch": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                           C.c_void_p, C.POINTER(Refine2D), C.c_int64,
                                           C.POINTER(CeresOptions2D), C.POINTER(Pose2D),
                                           C.POINTER(C.c_int32)]),
    "csm_ceres3d_refine_batch": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.c_int32,
                                           C.POINTER(Node3D), C.c_int32, C.POINTER(Refine3D),
                                           C.c_int64, C.POINTER(CeresOptions3D),
                                           C.POINTER(Pose3D), C.POINTER(C.c_int32)]),
    "csm_grid2d_cropped_limits": (C.c_int, [C.POINTER(MapLimits), C.POINTER(C.c_uint16),
                                            C.POINTER(C.c_int32), C.POINTER(MapLimits)]),
    "csm_grid2d_crop": (C.c_int, [C.POINTER(MapLimits), C.POINTER(C.c_uint16),
                                  C.POINTER(MapLimits), C.POINTER(C.c_uint16), C.c_int64]),
    "csm_pbstream_open": (C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    "csm_pbstream_close": (None, [C.c_void_p]),
    "csm_pbstream_format_version": (C.c_uint32, [C.c_void_p]),
    "csm_pbstream_num_submaps2d": (C.c_int32, [C.c_void_p]),
    "csm_pbstream_num_nodes": (C.c_int32, [C.c_void_p]),
    "csm_pbstream_submap2d": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int32),
                                        C.POINTER(MapLimits), C.POINTER(C.c_float),
                                        C.POINTER(C.c_int32), C.POINTER(C.c_double),
                                        C.POINTER(C.c_uint16), C.c_int64]),
    "csm_pbstream_node": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int32),
                                    C.POINTER(C.c_int64), C.POINTER(C.c_double),
                                    C.POINTER(C.c_double), C.POINTER(C.c_float), C.c_int64,
                                    C.POINTER(C.c_int32)]),
    "csm_pbstream_node_cloud": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_float),
                                          C.c_int64, C.POINTER(C.c_int32)]),
    "csm_pbstream_node_histogram": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_float),
                                              C.c_int32, C.POINTER(C.c_int32)]),
    "csm_pbstream_num_submaps3d": (C.c_int32, [C.c_void_p]),
    "csm_pbstream_submap3d": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int32),
                                        C.POINTER(C.c_int32), C.POINTER(C.c_double),
                                        C.POINTER(C.c_int64), C.POINTER(C.c_int32)]),
    "csm_pbstream_submap3d_grid": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32,
                                             C.POINTER(C.c_float), C.POINTER(C.c_int32),
                                             C.POINTER(C.c_uint16), C.c_int64]),
    "csm_pbstream_submap3d_histogram": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_float),
                                                  C.c_int32]),
    "csm_comm_get_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "csm_comm_create_rccl": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(C.c_uint8),
                                       C.POINTER(C.c_void_p)]),
    "csm_comm_create_tcp": (C.c_int, [C.c_int32, C.c_int32, C.c_char_p, C.c_int32,
                                      C.POINTER(C.c_void_p)]),
    "csm_comm_destroy": (None, [C.c_void_p]),
    "csm_comm_rank": (C.c_int32, [C.c_void_p]),
    "csm_comm_size": (C.c_int32, [C.c_void_p]),
    "csm_comm_gather": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
    "csm_comm_gathered": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_int64)]),
    "csm_comm_allreduce_i64": (C.c_int, [C.c_void_p, C.POINTER(C.c_int64), C.c_int32, C.c_int32]),
    "csm_comm_barrier": (C.c_int, [C.c_void_p]),
    "csm_comm_claim_open": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32]),
    "csm_comm_fetch_add": (C.c_int, [C.c_void_p, C.c_int64, C.c_int64, C.POINTER(C.c_int64)]),
    "csm_strerror": (C.c_char_p, [C.c_int]),
}

_lib_handle = None


def load_library(path: str = LIB_PATH) -> C.CDLL:
    """Loads libcsm_amd.so; raises if it is missing (no CPU fallback exists)."""
    global _lib_handle
    if _lib_handle is not None:
        return _lib_handle
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build it with `make -C cartographer-1_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(path)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib_handle = lib
    return lib


def strerror(code: int) -> str:
    """csm_strerror: the text of a C-ABI status code."""
    return load_library().csm_strerror(code).decode()


def _check(code: int, what: str) -> int:
    if code < 0:
        msg = load_library().csm_strerror(code).decode()
        raise CsmError(f"{what}: {msg} ({code})")
    return code


def _f32_points(points) -> np.ndarray:
    pts = np.ascontiguousarray(np.asarray(points, dtype=np.float32))
    if pts.ndim == 1:
        pts = pts.reshape(-1, 3)
    if pts.shape[1] == 2:
        pts = np.ascontiguousarray(np.concatenate([pts, np.zeros((len(pts), 1), np.float32)], 1))
    if pts.shape[1] != 3:
        raise ValueError("point cloud must be (n, 3) or (n, 2)")
    return pts


def _ptr(a: np.ndarray, t):
    return a.ctypes.data_as(C.POINTER(t))


# kMinCorrespondenceCost / kMaxCorrespondenceCost (probability_values.h:64-67),
# evaluated in float like the reference's constexprs.
K_MIN_PROBABILITY = float(np.float32(0.1))
K_MAX_PROBABILITY = float(np.float32(1.0) - np.float32(0.1))
K_MIN_CORRESPONDENCE_COST = float(np.float32(1.0) - np.float32(K_MAX_PROBABILITY))
K_MAX_CORRESPONDENCE_COST = float(np.float32(1.0) - np.float32(0.1))


@dataclass
class ProbabilityGrid:
    """Grid2D data for the boundary: MapLimits + uint16 correspondence-cost cells
    (x fastest: ``cells[y, x]`` for a (num_y_cells, num_x_cells) array)."""
    resolution: float
    max_x: float
    max_y: float
    cells: np.ndarray  # shape (num_y_cells, num_x_cells), uint16
    min_correspondence_cost: float = K_MIN_CORRESPONDENCE_COST
    max_correspondence_cost: float = K_MAX_CORRESPONDENCE_COST

    @property
    def num_x_cells(self) -> int:
        return int(self.cells.shape[1])

    @property
    def num_y_cells(self) -> int:
        return int(self.cells.shape[0])

    def limits(self) -> MapLimits:
        return MapLimits(self.resolution, self.max_x, self.max_y, self.num_x_cells,
                         self.num_y_cells)


def ComputeCroppedGrid(grid: "ProbabilityGrid") -> "ProbabilityGrid":
    """Submap2D::Finish's crop (ProbabilityGrid::ComputeCroppedGrid,
    probability_grid.cc:91-106) through csm_grid2d_crop."""
    lib = load_library()
    cells = np.ascontiguousarray(grid.cells, np.uint16)
    lim = grid.limits()
    out_lim = MapLimits()
    out = np.zeros(max(cells.size, 1), np.uint16)
    _check(lib.csm_grid2d_crop(C.byref(lim), _ptr(cells, C.c_uint16), C.byref(out_lim),
                               _ptr(out, C.c_uint16), out.size), "csm_grid2d_crop")
    nx, ny = out_lim.num_x_cells, out_lim.num_y_cells
    return ProbabilityGrid(out_lim.resolution, out_lim.max_x, out_lim.max_y,
                           out[:nx * ny].reshape(ny, nx).copy())


@dataclass
class SerializedSubmap2D:
    """A Submap2D read from a pbstream (mapping/proto/submap.proto:24-29)."""
    trajectory_id: int
    submap_index: int
    local_pose: np.ndarray  # (tx, ty, tz, qw, qx, qy, qz)
    finished: bool
    grid: ProbabilityGrid


@dataclass
class SerializedNode:
    """A trajectory node read from a pbstream (trajectory_node_data.proto:23-32):
    ``points`` is the decompressed filtered_gravity_aligned_point_cloud."""
    trajectory_id: int
    node_index: int
    timestamp: int
    local_pose: np.ndarray  # (tx, ty, tz, qw, qx, qy, qz)
    gravity_alignment: np.ndarray  # (w, x, y, z)
    points: np.ndarray  # (n, 3) float32
    # 3D node data (trajectory_node_data.proto:28-30); empty for 2D nodes.
    high_resolution_points: np.ndarray = None
    low_resolution_points: np.ndarray = None
    rotational_scan_matcher_histogram: np.ndarray = None


@dataclass
class SerializedSubmap3D:
    """A Submap3D read from a pbstream (mapping/proto/submap.proto:32-39): each
    grid is (resolution, (n, 3) int32 indices, uint16 values), values as
    HybridGrid(proto) stores them (hybrid_grid.h:473-484)."""
    trajectory_id: int
    submap_index: int
    local_pose: np.ndarray
    finished: bool
    high_resolution_hybrid_grid: tuple
    low_resolution_hybrid_grid: tuple
    rotational_scan_matcher_histogram: np.ndarray


@dataclass
class PbStream:
    format_version: int
    submaps: list
    nodes: list
    submaps3d: list = None


def read_pbstream(path) -> PbStream:
    """Loads the Submap2D grids and node clouds of a serialized state file
    (io/proto_stream.cc, io/internal/mapping_state_serialization.cc) through
    csm_pbstream_*; other message kinds are skipped."""
    lib = load_library()
    h = C.c_void_p()
    _check(lib.csm_pbstream_open(os.fsencode(os.fspath(path)), C.byref(h)), "csm_pbstream_open")
    try:
        submaps, nodes = [], []
        for i in range(lib.csm_pbstream_num_submaps2d(h)):
            ids = (C.c_int32 * 2)()
            lim = MapLimits()
            cc = (C.c_float * 2)()
            fin = C.c_int32()
            pose = np.zeros(7, np.float64)
            _check(lib.csm_pbstream_submap2d(h, i, ids, C.byref(lim), cc, C.byref(fin),
                                             _ptr(pose, C.c_double), None, 0),
                   "csm_pbstream_submap2d")
            cells = np.zeros((lim.num_y_cells, lim.num_x_cells), np.uint16)
            _check(lib.csm_pbstream_submap2d(h, i, None, None, None, None, None,
                                             _ptr(cells, C.c_uint16), cells.size),
                   "csm_pbstream_submap2d")
            grid = ProbabilityGrid(lim.resolution, lim.max_x, lim.max_y, cells,
                                   float(cc[0]), float(cc[1]))
            submaps.append(SerializedSubmap2D(ids[0], ids[1], pose, bool(fin.value), grid))
        for i in range(lib.csm_pbstream_num_nodes(h)):
            ids = (C.c_int32 * 2)()
            ts = C.c_int64()
            pose = np.zeros(7, np.float64)
            grav = np.zeros(4, np.float64)
            n = C.c_int32()
            _check(lib.csm_pbstream_node(h, i, ids, C.byref(ts), _ptr(pose, C.c_double),
                                         _ptr(grav, C.c_double), None, 0, C.byref(n)),
                   "csm_pbstream_node")
            pts = np.zeros((n.value, 3), np.float32)
            _check(lib.csm_pbstream_node(h, i, None, None, None, None, _ptr(pts, C.c_float),
                                         n.value, None), "csm_pbstream_node")
            clouds = []
            for which in (1, 2):
                _check(lib.csm_pbstream_node_cloud(h, i, which, None, 0, C.byref(n)),
                       "csm_pbstream_node_cloud")
                c = np.zeros((n.value, 3), np.float32)
                _check(lib.csm_pbstream_node_cloud(h, i, which, _ptr(c, C.c_float), n.value, None),
                       "csm_pbstream_node_cloud")
                clouds.append(c)
            _check(lib.csm_pbstream_node_histogram(h, i, None, 0, C.byref(n)),
                   "csm_pbstream_node_histogram")
            hist = np.zeros(n.value, np.float32)
            _check(lib.csm_pbstream_node_histogram(h, i, _ptr(hist, C.c_float), n.value, None),
                   "csm_pbstream_node_histogram")
            nodes.append(SerializedNode(ids[0], ids[1], ts.value, pose, grav, pts, clouds[0],
                                        clouds[1], hist))
        submaps3d = []
        for i in range(lib.csm_pbstream_num_submaps3d(h)):
            ids = (C.c_int32 * 2)()
            fin = C.c_int32()
            pose = np.zeros(7, np.float64)
            cells = (C.c_int64 * 2)()
            hs = C.c_int32()
            _check(lib.csm_pbstream_submap3d(h, i, ids, C.byref(fin), _ptr(pose, C.c_double),
                                             cells, C.byref(hs)), "csm_pbstream_submap3d")
            grids = []
            for which in (0, 1):
                res = C.c_float()
                idx = np.zeros((cells[which], 3), np.int32)
                val = np.zeros(cells[which], np.uint16)
                _check(lib.csm_pbstream_submap3d_grid(h, i, which, C.byref(res),
                                                      _ptr(idx, C.c_int32), _ptr(val, C.c_uint16),
                                                      cells[which]), "csm_pbstream_submap3d_grid")
                grids.append((float(res.value), idx, val))
            hist = np.zeros(hs.value, np.float32)
            _check(lib.csm_pbstream_submap3d_histogram(h, i, _ptr(hist, C.c_float), hs.value),
                   "csm_pbstream_submap3d_histogram")
            submaps3d.append(SerializedSubmap3D(ids[0], ids[1], pose, bool(fin.value), grids[0],
                                                grids[1], hist))
        return PbStream(int(lib.csm_pbstream_format_version(h)), submaps, nodes, submaps3d)
    finally:
        lib.csm_pbstream_close(h)


@dataclass
class TSDF2D:
    """TSDF2D data for the boundary (mapping/internal/2d/tsdf_2d.h): MapLimits,
    the uint16 TSD cells (Grid2D correspondence_cost_cells) and weight cells,
    both ``[y, x]``, and the TSDValueConverter parameters."""
    resolution: float
    max_x: float
    max_y: float
    tsd_cells: np.ndarray     # shape (num_y_cells, num_x_cells), uint16
    weight_cells: np.ndarray  # same shape, uint16
    truncation_distance: float
    max_weight: float

    @property
    def num_x_cells(self) -> int:
        return int(self.tsd_cells.shape[1])

    @property
    def num_y_cells(self) -> int:
        return int(self.tsd_cells.shape[0])

    def limits(self) -> MapLimits:
        return MapLimits(self.resolution, self.max_x, self.max_y, self.num_x_cells,
                         self.num_y_cells)


class Context:
    """A device, a HIP stream and per-call scratch (one per calling thread)."""

    def __init__(self, device: int = 0):
        self._lib = load_library()
        h = C.c_void_p()
        _check(self._lib.csm_context_create(device, C.byref(h)), "csm_context_create")
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            self._lib.csm_context_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return self._lib.csm_context_stream(self.handle) or 0

    def enable_timing(self, on: bool = True):
        self._lib.csm_context_enable_timing(self.handle, 1 if on else 0)

    def reset_timing(self):
        self._lib.csm_context_reset_timing(self.handle)

    def level_stats(self):
        """(candidates, batches) scored per pyramid level while timing was on."""
        c = (C.c_double * 12)()
        b = (C.c_double * 12)()
        n = self._lib.csm_context_level_stats(self.handle, c, b, 12)
        return list(c)[:n], list(b)[:n]

    def timing(self) -> Timing:
        t = Timing()
        self._lib.csm_context_get_timing(self.handle, C.byref(t))
        return t


_default_contexts = {}


def default_context(device: int = 0) -> Context:
    if device not in _default_contexts:
        _default_contexts[device] = Context(device)
    return _default_contexts[device]


@dataclass
class FastCorrelativeScanMatcherOptions2D:
    """proto::FastCorrelativeScanMatcherOptions2D; defaults from
    configuration_files/pose_graph.lua:25-29."""
    linear_search_window: float = 7.0
    angular_search_window: float = math.radians(30.0)
    branch_and_bound_depth: int = 7
    search_depth: int = 0  # device pyramid depth (0 = automatic; exact either way)


@dataclass
class RealTimeCorrelativeScanMatcherOptions:
    """proto::RealTimeCorrelativeScanMatcherOptions; defaults from
    configuration_files/trajectory_builder_2d.lua:38-43."""
    linear_search_window: float = 0.1
    angular_search_window: float = math.radians(20.0)
    translation_delta_cost_weight: float = 1e-1
    rotation_delta_cost_weight: float = 1e-1


class FastCorrelativeScanMatcher2D:
    """Device pyramid of one submap grid; Match / MatchFullSubmap run on the GPU."""

    def __init__(self, grid: ProbabilityGrid, options: FastCorrelativeScanMatcherOptions2D,
                 context: Optional[Context] = None):
        self.context = context or default_context()
        self._lib = self.context._lib
        self.grid_limits = grid.limits()
        self.options = options
        cells = np.ascontiguousarray(grid.cells, dtype=np.uint16)
        opts = Fast2DOptions(options.linear_search_window, options.angular_search_window,
                             options.branch_and_bound_depth, options.search_depth)
        h = C.c_void_p()
        _check(self._lib.csm_fast2d_create(self.context.handle, C.byref(self.grid_limits),
                                           _ptr(cells, C.c_uint16),
                                           grid.min_correspondence_cost,
                                           grid.max_correspondence_cost, C.byref(opts),
                                           C.byref(h)), "csm_fast2d_create")
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            self._lib.csm_fast2d_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def Match(self, initial_pose_estimate, point_cloud, min_score: float):
        """fast_correlative_scan_matcher_2d.h:127-129 -> (matched, score, pose)."""
        pts = _f32_points(point_cloud)
        init = Pose2D(*initial_pose_estimate)
        score = C.c_float(0.0)
        pose = Pose2D()
        rc = _check(self._lib.csm_fast2d_match(self.handle, C.byref(init), _ptr(pts, C.c_float),
                                               len(pts), min_score, C.byref(score),
                                               C.byref(pose)), "csm_fast2d_match")
        return rc == CSM_OK, float(score.value), pose.as_tuple()

    def MatchFullSubmap(self, point_cloud, min_score: float):
        """fast_correlative_scan_matcher_2d.h:135-136 -> (matched, score, pose)."""
        pts = _f32_points(point_cloud)
        score = C.c_float(0.0)
        pose = Pose2D()
        rc = _check(self._lib.csm_fast2d_match_full_submap(
            self.handle, _ptr(pts, C.c_float), len(pts), min_score, C.byref(score),
            C.byref(pose)), "csm_fast2d_match_full_submap")
        return rc == CSM_OK, float(score.value), pose.as_tuple()

    def device_bytes(self) -> int:
        """Device memory the matcher holds (csm_fast2d_device_bytes)."""
        return int(self._lib.csm_fast2d_device_bytes(self.handle))

    def read_level(self, level: int) -> np.ndarray:
        """PrecomputationGrid2D level as (wide_ny, wide_nx) uint8."""
        wnx, wny = C.c_int32(), C.c_int32()
        _check(self._lib.csm_fast2d_read_level(self.handle, level, None, 0, C.byref(wnx),
                                               C.byref(wny)), "csm_fast2d_read_level")
        out = np.zeros((wny.value, wnx.value), np.uint8)
        _check(self._lib.csm_fast2d_read_level(self.handle, level, _ptr(out, C.c_uint8),
                                               out.size, C.byref(wnx), C.byref(wny)),
               "csm_fast2d_read_level")
        return out


class RealTimeCorrelativeScanMatcher2D:
    def __init__(self, options: RealTimeCorrelativeScanMatcherOptions,
                 context: Optional[Context] = None):
        self.context = context or default_context()
        self._lib = self.context._lib
        self.options = options
        o = options
        self._opts = RtOptions(o.linear_search_window, o.angular_search_window,
                               o.translation_delta_cost_weight, o.rotation_delta_cost_weight)

    def Match(self, initial_pose_estimate, point_cloud, grid):
        """real_time_correlative_scan_matcher_2d.h:66-68 -> (score, pose). ``grid`` is a
        ProbabilityGrid or a TSDF2D (ScoreCandidates switches on the grid type,
        .cc:155-168)."""
        pts = _f32_points(point_cloud)
        opts = self._opts
        lim = grid.limits()
        init = Pose2D(*initial_pose_estimate)
        score = C.c_double(0.0)
        pose = Pose2D()
        if isinstance(grid, TSDF2D):
            tsd = np.ascontiguousarray(grid.tsd_cells, dtype=np.uint16)
            wgt = np.ascontiguousarray(grid.weight_cells, dtype=np.uint16)
            if tsd.shape != wgt.shape:
                raise ValueError("TSDF2D tsd_cells and weight_cells differ in shape")
            _check(self._lib.csm_rt2d_match_tsdf(
                self.context.handle, C.byref(opts), C.byref(lim), _ptr(tsd, C.c_uint16),
                _ptr(wgt, C.c_uint16), grid.truncation_distance, grid.max_weight, C.byref(init),
                _ptr(pts, C.c_float), len(pts), C.byref(score), C.byref(pose)),
                "csm_rt2d_match_tsdf")
        else:
            cells = np.ascontiguousarray(grid.cells, dtype=np.uint16)
            _check(self._lib.csm_rt2d_match(self.context.handle, C.byref(opts), C.byref(lim),
                                            _ptr(cells, C.c_uint16), grid.min_correspondence_cost,
                                            grid.max_correspondence_cost, C.byref(init),
                                            _ptr(pts, C.c_float), len(pts), C.byref(score),
                                            C.byref(pose)), "csm_rt2d_match")
        return float(score.value), pose.as_tuple()

    def ScoreCandidates(self, grid, discrete_scans, search_parameters: "SearchParameters",
                        candidates):
        """real_time_correlative_scan_matcher_2d.h:75-78 (visible for testing):
        sets ``score`` on every Candidate2D of ``candidates`` (in place; also
        returned as a float32 array). ``discrete_scans``: (num_scans, n, 2)
        int cell indices as DiscretizeScans returns them."""
        d = np.ascontiguousarray(np.asarray(discrete_scans, np.int32))
        if d.ndim != 3 or d.shape[2] != 2:
            raise ValueError("discrete_scans must be (num_scans, points, 2)")
        o = self.options
        opts = RtOptions(o.linear_search_window, o.angular_search_window,
                         o.translation_delta_cost_weight, o.rotation_delta_cost_weight)
        lim = grid.limits()
        arr = (Candidate2DC * max(len(candidates), 1))()
        for i, c in enumerate(candidates):
            arr[i].scan_index, arr[i].x_index_offset, arr[i].y_index_offset = (
                c.scan_index, c.x_index_offset, c.y_index_offset)
        sp = search_parameters._c
        if isinstance(grid, TSDF2D):
            tsd = np.ascontiguousarray(grid.tsd_cells, dtype=np.uint16)
            wgt = np.ascontiguousarray(grid.weight_cells, dtype=np.uint16)
            _check(self._lib.csm_rt2d_score_candidates_tsdf(
                self.context.handle, C.byref(opts), C.byref(lim), _ptr(tsd, C.c_uint16),
                _ptr(wgt, C.c_uint16), grid.truncation_distance, grid.max_weight,
                _ptr(d, C.c_int32), d.shape[0], d.shape[1], C.byref(sp), arr, len(candidates)),
                "csm_rt2d_score_candidates_tsdf")
        else:
            cells = np.ascontiguousarray(grid.cells, dtype=np.uint16)
            _check(self._lib.csm_rt2d_score_candidates(
                self.context.handle, C.byref(opts), C.byref(lim), _ptr(cells, C.c_uint16),
                grid.min_correspondence_cost, grid.max_correspondence_cost, _ptr(d, C.c_int32),
                d.shape[0], d.shape[1], C.byref(sp), arr, len(candidates)),
                "csm_rt2d_score_candidates")
        scores = np.array([arr[i].score for i in range(len(candidates))], np.float32)
        for c, v in zip(candidates, scores):
            c.score = float(v)
        return scores


class SearchParameters:
    """correlative_scan_matcher_2d.h:35-61: SearchParameters(linear_search_window,
    angular_search_window, point_cloud, resolution), or the testing constructor
    ``SearchParameters.for_testing(num_linear, num_angular, step, resolution)``."""

    def __init__(self, linear_search_window, angular_search_window, point_cloud,
                 resolution, _c=None):
        lib = load_library()
        if _c is None:
            pts = _f32_points(point_cloud)
            _c = SearchParametersC()
            _check(lib.csm_search_parameters_init(linear_search_window, angular_search_window,
                                                  _ptr(pts, C.c_float), len(pts), resolution,
                                                  C.byref(_c)), "csm_search_parameters_init")
        self._c = _c
        L = _c.num_linear_perturbations
        self.linear_bounds = [LinearBounds(-L, L, -L, L) for _ in range(_c.num_scans)]

    @staticmethod
    def for_testing(num_linear_perturbations, num_angular_perturbations,
                    angular_perturbation_step_size, resolution) -> "SearchParameters":
        c = SearchParametersC()
        _check(load_library().csm_search_parameters_init_for_testing(
            num_linear_perturbations, num_angular_perturbations, angular_perturbation_step_size,
            resolution, C.byref(c)), "csm_search_parameters_init_for_testing")
        return SearchParameters(0, 0, None, resolution, _c=c)

    num_angular_perturbations = property(lambda self: self._c.num_angular_perturbations)
    angular_perturbation_step_size = property(lambda self: self._c.angular_perturbation_step_size)
    resolution = property(lambda self: self._c.resolution)
    num_scans = property(lambda self: self._c.num_scans)

    def ShrinkToFit(self, discrete_scans, num_x_cells, num_y_cells):
        """correlative_scan_matcher_2d.cc:68-91 (cell_limits as its two counts)."""
        d = np.ascontiguousarray(np.asarray(discrete_scans, np.int32))
        if d.shape[0] != self.num_scans or d.ndim != 3 or d.shape[2] != 2:
            raise ValueError("discrete_scans must be (num_scans, points, 2)")
        b = (LinearBounds * self.num_scans)(*self.linear_bounds)
        _check(load_library().csm_search_parameters_shrink_to_fit(
            C.byref(self._c), _ptr(d, C.c_int32), d.shape[1], num_x_cells, num_y_cells, b),
            "csm_search_parameters_shrink_to_fit")
        self.linear_bounds = [b[i] for i in range(self.num_scans)]


@dataclass
class Candidate2D:
    """correlative_scan_matcher_2d.h:71-98."""
    scan_index: int
    x_index_offset: int
    y_index_offset: int
    search_parameters: "SearchParameters"
    score: float = 0.0

    @property
    def x(self):
        return -self.y_index_offset * self.search_parameters.resolution

    @property
    def y(self):
        return -self.x_index_offset * self.search_parameters.resolution

    @property
    def orientation(self):
        sp = self.search_parameters
        return (self.scan_index - sp.num_angular_perturbations) * sp.angular_perturbation_step_size


def GenerateRotatedScans(point_cloud, search_parameters: SearchParameters) -> np.ndarray:
    """correlative_scan_matcher_2d.cc:93-108 -> (num_scans, n, 3) float32."""
    pts = _f32_points(point_cloud)
    out = np.zeros((search_parameters.num_scans, len(pts), 3), np.float32)
    _check(load_library().csm_generate_rotated_scans(_ptr(pts, C.c_float), len(pts),
                                                     C.byref(search_parameters._c),
                                                     _ptr(out, C.c_float)),
           "csm_generate_rotated_scans")
    return out


def DiscretizeScans(map_limits: MapLimits, scans, initial_translation) -> np.ndarray:
    """correlative_scan_matcher_2d.cc:110-127: (num_scans, n, 3) rotated clouds
    -> (num_scans, n, 2) int32 cell indices (x, y)."""
    sc = np.ascontiguousarray(np.asarray(scans, np.float32))
    if sc.ndim != 3 or sc.shape[2] != 3:
        raise ValueError("scans must be (num_scans, points, 3)")
    out = np.zeros((sc.shape[0], sc.shape[1], 2), np.int32)
    _check(load_library().csm_discretize_scans(C.byref(map_limits), _ptr(sc, C.c_float),
                                               sc.shape[1], sc.shape[0],
                                               float(np.float32(initial_translation[0])),
                                               float(np.float32(initial_translation[1])),
                                               _ptr(out, C.c_int32)),
           "csm_discretize_scans")
    return out


class ScanSet:
    """Node point clouds resident on the device (TrajectoryNode::Data clouds)."""

    def __init__(self, clouds: Sequence, context: Optional[Context] = None,
                 packed: Optional[Tuple[np.ndarray, np.ndarray]] = None):
        self.context = context or default_context()
        self._lib = self.context._lib
        if packed is not None:
            pts, offsets = packed
            pts = np.ascontiguousarray(pts, np.float32).reshape(-1, 3)
            offsets = np.ascontiguousarray(offsets, np.int64)
        else:
            arrs = [_f32_points(c) for c in clouds]
            offsets = np.zeros(len(arrs) + 1, np.int64)
            offsets[1:] = np.cumsum([len(a) for a in arrs])
            pts = np.ascontiguousarray(np.concatenate(arrs) if arrs else np.zeros((0, 3), np.float32))
        self.points, self.offsets = pts, offsets
        h = C.c_void_p()
        _check(self._lib.csm_scan_set_create(self.context.handle, _ptr(pts, C.c_float),
                                             _ptr(offsets, C.c_int64), len(offsets) - 1,
                                             C.byref(h)), "csm_scan_set_create")
        self.handle = h

    def __len__(self):
        return len(self.offsets) - 1

    def append(self, clouds: Sequence) -> int:
        """Adds clouds to the resident set (csm_scan_set_append); earlier
        scans keep their indices. Returns the first new scan's index."""
        arrs = [_f32_points(c) for c in clouds]
        offsets = np.zeros(len(arrs) + 1, np.int64)
        offsets[1:] = np.cumsum([len(a) for a in arrs])
        pts = np.ascontiguousarray(np.concatenate(arrs) if arrs else np.zeros((0, 3), np.float32))
        first = C.c_int32()
        _check(self._lib.csm_scan_set_append(self.handle, _ptr(pts, C.c_float),
                                             _ptr(offsets, C.c_int64), len(arrs),
                                             C.byref(first)), "csm_scan_set_append")
        # `points` stays the creation-time clouds (the device set and its C
        # host copy hold the rest); `offsets` covers every scan.
        self.offsets = np.concatenate([self.offsets, self.offsets[-1] + offsets[1:]])
        return int(first.value)

    def device_size(self) -> Tuple[int, int]:
        """(scans, points) the device set holds (csm_scan_set_size)."""
        n, p = C.c_int32(), C.c_int64()
        _check(self._lib.csm_scan_set_size(self.handle, C.byref(n), C.byref(p)),
               "csm_scan_set_size")
        return int(n.value), int(p.value)

    def close(self):
        if getattr(self, "handle", None):
            self._lib.csm_scan_set_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


PAIR_DTYPE = np.dtype([("submap", np.int32), ("scan", np.int32), ("full_submap", np.int32),
                       ("min_score", np.float32), ("x", np.float64), ("y", np.float64),
                       ("theta", np.float64)])
RESULT_DTYPE = np.dtype([("status", np.int32), ("score", np.float32), ("x", np.float64),
                         ("y", np.float64), ("theta", np.float64), ("tie", np.int32),
                         ("reserved", np.int32)])
assert PAIR_DTYPE.itemsize == C.sizeof(Pair2D)
assert RESULT_DTYPE.itemsize == C.sizeof(Result2D)


def make_pairs(submap, scan, min_score, full_submap=True, initial=None) -> np.ndarray:
    submap = np.asarray(submap, np.int32)
    pairs = np.zeros(len(submap), PAIR_DTYPE)
    pairs["submap"] = submap
    pairs["scan"] = np.asarray(scan, np.int32)
    pairs["full_submap"] = 1 if full_submap else 0
    pairs["min_score"] = min_score
    if initial is not None:
        initial = np.asarray(initial, np.float64).reshape(-1, 3)
        pairs["x"], pairs["y"], pairs["theta"] = initial[:, 0], initial[:, 1], initial[:, 2]
    return pairs


def match_batch(matchers: Sequence[FastCorrelativeScanMatcher2D], scans: ScanSet,
                pairs: np.ndarray, context: Optional[Context] = None) -> np.ndarray:
    """Batched Match / MatchFullSubmap over (submap, node) pairs; returns a
    RESULT_DTYPE array in pair order (status CSM_OK = constraint found)."""
    ctx = context or scans.context
    lib = ctx._lib
    pairs = np.ascontiguousarray(pairs, PAIR_DTYPE)
    results = np.zeros(len(pairs), RESULT_DTYPE)
    handles = (C.c_void_p * len(matchers))(*[m.handle for m in matchers])
    _check(lib.csm_fast2d_match_batch(ctx.handle, handles, len(matchers), scans.handle,
                                      pairs.ctypes.data_as(C.POINTER(Pair2D)), len(pairs),
                                      results.ctypes.data_as(C.POINTER(Result2D))),
           "csm_fast2d_match_batch")
    return results


REFINE_DTYPE = np.dtype([("submap", np.int32), ("scan", np.int32), ("x", np.float64),
                         ("y", np.float64), ("theta", np.float64), ("target_x", np.float64),
                         ("target_y", np.float64)])
POSE_DTYPE = np.dtype([("x", np.float64), ("y", np.float64), ("theta", np.float64)])
assert REFINE_DTYPE.itemsize == C.sizeof(Refine2D) and POSE_DTYPE.itemsize == C.sizeof(Pose2D)


def ceres_refine_batch(matchers: Sequence[FastCorrelativeScanMatcher2D], scans: ScanSet,
                       submap_idx, scan_idx, initial, target=None,
                       options: Optional["CeresOptions2D"] = None,
                       context: Optional[Context] = None):
    """CeresScanMatcher2D::Match for each (submap, scan) item on the device
    (ceres_scan_matcher_2d.cc:64-105): returns (poses (n, 3), iterations)."""
    ctx = context or scans.context
    n = len(submap_idx)
    initial = np.asarray(initial, np.float64).reshape(n, 3)
    target = initial[:, :2] if target is None else np.asarray(target, np.float64).reshape(n, 2)
    items = np.zeros(max(n, 1), REFINE_DTYPE)
    items["submap"][:n] = np.asarray(submap_idx, np.int32)
    items["scan"][:n] = np.asarray(scan_idx, np.int32)
    items["x"][:n], items["y"][:n], items["theta"][:n] = initial[:, 0], initial[:, 1], initial[:, 2]
    items["target_x"][:n], items["target_y"][:n] = target[:, 0], target[:, 1]
    out = np.zeros(max(n, 1), POSE_DTYPE)
    iters = np.zeros(max(n, 1), np.int32)
    handles = (C.c_void_p * len(matchers))(*[m.handle for m in matchers])
    opts = options or CeresOptions2D.make()
    _check(ctx._lib.csm_ceres2d_refine_batch(ctx.handle, handles, len(matchers), scans.handle,
                                             items.ctypes.data_as(C.POINTER(Refine2D)), n,
                                             C.byref(opts), out.ctypes.data_as(C.POINTER(Pose2D)),
                                             _ptr(iters, C.c_int32)),
           "csm_ceres2d_refine_batch")
    poses = np.stack([out["x"][:n], out["y"][:n], out["theta"][:n]], 1)
    return poses, iters[:n]


# --------------------------------------------------------------------------
# Synthetic world (bench / test inputs; not the matching path).

class SynthConfig(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("world_x", C.c_double), ("world_y", C.c_double),
                ("resolution", C.c_double), ("num_nodes", C.c_int32),
                ("num_submaps", C.c_int32), ("submap_cells", C.c_int32), ("beams", C.c_int32),
                ("fov", C.c_double), ("max_range", C.c_double), ("range_noise", C.c_double),
                ("decimate_to", C.c_int32), ("room_size", C.c_double),
                ("boxes_per_room", C.c_int32), ("threads", C.c_int32)]


class SyntheticWorld2D:
    """Seeded building world: node clouds + fixed-size submap grids."""

    def __init__(self, num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                 seed=20250127, decimate_to=0, max_range=30.0, threads=0, **kw):
        lib = C.CDLL(SYNTH_PATH)
        lib.csm_synth2d_create.argtypes = [C.POINTER(SynthConfig), C.POINTER(C.c_void_p)]
        for name, t in [("csm_synth2d_point_offsets", C.c_int64), ("csm_synth2d_points", C.c_float),
                        ("csm_synth2d_node_poses", C.c_double),
                        ("csm_synth2d_submap_max", C.c_double),
                        ("csm_synth2d_submap_nodes", C.c_int32),
                        ("csm_synth2d_submap_cells", C.c_uint16)]:
            getattr(lib, name).restype = C.POINTER(t)
            getattr(lib, name).argtypes = [C.c_void_p]
        lib.csm_synth2d_destroy.argtypes = [C.c_void_p]
        cfg = SynthConfig()
        lib.csm_synth2d_default_config(C.byref(cfg))
        cfg.num_nodes, cfg.num_submaps, cfg.submap_cells = num_nodes, num_submaps, submap_cells
        cfg.beams, cfg.seed, cfg.decimate_to, cfg.max_range = beams, seed, decimate_to, max_range
        cfg.threads = threads
        for k, v in kw.items():
            setattr(cfg, k, v)
        h = C.c_void_p()
        if lib.csm_synth2d_create(C.byref(cfg), C.byref(h)) != 0:
            raise ValueError("invalid synthetic world config")
        try:
            n, s, c = num_nodes, num_submaps, submap_cells
            self.offsets = np.ctypeslib.as_array(lib.csm_synth2d_point_offsets(h), (n + 1,)).copy()
            total = int(self.offsets[-1])
            self.points = np.ctypeslib.as_array(lib.csm_synth2d_points(h), (total * 3,)).reshape(-1, 3).copy() \
                if total else np.zeros((0, 3), np.float32)
            self.node_poses = np.ctypeslib.as_array(lib.csm_synth2d_node_poses(h), (n * 3,)).reshape(-1, 3).copy()
            self.submap_max = np.ctypeslib.as_array(lib.csm_synth2d_submap_max(h), (max(s, 1) * 2,)).reshape(-1, 2)[:s].copy()
            self.submap_nodes = np.ctypeslib.as_array(lib.csm_synth2d_submap_nodes(h), (max(s, 1),))[:s].copy()
            self.submap_cells = np.ctypeslib.as_array(lib.csm_synth2d_submap_cells(h), (max(s, 1) * c * c,)).reshape(-1, c, c)[:s].copy()
        finally:
            lib.csm_synth2d_destroy(h)
        self.resolution = cfg.resolution
        self.num_nodes, self.num_submaps, self.submap_size = num_nodes, num_submaps, submap_cells

    def cloud(self, node: int) -> np.ndarray:
        return self.points[self.offsets[node]:self.offsets[node + 1]]

    def grid(self, submap: int) -> ProbabilityGrid:
        # cells[j, i] holds cell (x=i, y=j): flat index i + j * num_x_cells.
        return ProbabilityGrid(self.resolution, float(self.submap_max[submap, 0]),
                               float(self.submap_max[submap, 1]), self.submap_cells[submap])


# 3D matchers (RealTimeCorrelativeScanMatcher3D, FastCorrelativeScanMatcher3D).
from .matching3d import (FastCorrelativeScanMatcher3D, FastCorrelativeScanMatcherOptions3D,  # noqa: E402,F401
                         HybridGrid, NodeData3D, NodeSet3D, PAIR3_DTYPE, RESULT3_DTYPE,
                         RealTimeCorrelativeScanMatcher3D, SyntheticWorld3D, ceres_refine_batch_3d,
                         make_pairs_3d, match_batch_3d)


# --------------------------------------------------------------------------
# Node clouds: voxel filters (sensor/internal/voxel_filter.cc).

def _pack_clouds(clouds):
    arrs = [_f32_points(c) for c in clouds]
    offsets = np.zeros(len(arrs) + 1, np.int64)
    offsets[1:] = np.cumsum([len(a) for a in arrs])
    pts = np.ascontiguousarray(np.concatenate(arrs) if arrs else np.zeros((0, 3), np.float32))
    return pts, offsets


def voxel_filter_masks(clouds, resolution: float, context: Optional[Context] = None):
    """sensor::VoxelFilter(cloud, resolution) for each cloud (voxel_filter.cc:212-232):
    returns (keep mask over the concatenated points, per-cloud counts, offsets).
    The survivors of cloud c are ``points[offsets[c]:offsets[c+1]][mask[...]]``."""
    ctx = context or default_context()
    pts, offsets = _pack_clouds(clouds)
    keep = np.zeros(len(pts), np.uint8)
    counts = np.zeros(len(offsets) - 1, np.int32)
    _check(ctx._lib.csm_voxel_filter(ctx.handle, _ptr(pts, C.c_float), _ptr(offsets, C.c_int64),
                                     len(offsets) - 1, float(resolution), _ptr(keep, C.c_uint8),
                                     _ptr(counts, C.c_int32)), "csm_voxel_filter")
    return keep.astype(bool), counts, offsets


def adaptive_voxel_filter_masks(clouds, options: AdaptiveVoxelFilterOptions,
                                context: Optional[Context] = None):
    """sensor::AdaptiveVoxelFilter(cloud, options) for each cloud
    (voxel_filter.cc:263-268): (keep mask, counts, offsets) as voxel_filter_masks."""
    ctx = context or default_context()
    pts, offsets = _pack_clouds(clouds)
    keep = np.zeros(len(pts), np.uint8)
    counts = np.zeros(len(offsets) - 1, np.int32)
    _check(ctx._lib.csm_adaptive_voxel_filter(ctx.handle, _ptr(pts, C.c_float),
                                              _ptr(offsets, C.c_int64), len(offsets) - 1,
                                              C.byref(options), _ptr(keep, C.c_uint8),
                                              _ptr(counts, C.c_int32)),
           "csm_adaptive_voxel_filter")
    return keep.astype(bool), counts, offsets


def VoxelFilter(point_cloud, resolution: float, intensities=None,
                context: Optional[Context] = None):
    """sensor::VoxelFilter(const PointCloud&, float) (voxel_filter.cc:212-232):
    the surviving points in input order (and their intensities, if given)."""
    pts = _f32_points(point_cloud)
    keep, _, _ = voxel_filter_masks([pts], resolution, context)
    if intensities is None:
        return pts[keep]
    return pts[keep], np.asarray(intensities, np.float32)[keep[:len(intensities)]]


def AdaptiveVoxelFilter(point_cloud, options: AdaptiveVoxelFilterOptions, intensities=None,
                        context: Optional[Context] = None):
    """sensor::AdaptiveVoxelFilter(const PointCloud&, options) (voxel_filter.cc:263-268)."""
    pts = _f32_points(point_cloud)
    keep, _, _ = adaptive_voxel_filter_masks([pts], options, context)
    if intensities is None:
        return pts[keep]
    return pts[keep], np.asarray(intensities, np.float32)[keep[:len(intensities)]]


# --------------------------------------------------------------------------
# Device buffers for the *_device entry points (bench / tests), allocated with
# the HIP runtime libcsm_amd.so itself links (same soname, same instance).

_hip_handle = None


def _hip():
    global _hip_handle
    if _hip_handle is None:
        load_library()
        h = C.CDLL("libamdhip64.so.7")
        h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        h.hipFree.argtypes = [C.c_void_p]
        h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        h.hipStreamSynchronize.argtypes = [C.c_void_p]
        _hip_handle = h
    return _hip_handle


class DeviceBuffer:
    """hipMalloc'd bytes holding a copy of a numpy array (or zeros)."""

    def __init__(self, array: np.ndarray = None, nbytes: int = 0):
        self.nbytes = int(array.nbytes if array is not None else nbytes)
        self.ptr = C.c_void_p()
        if _hip().hipMalloc(C.byref(self.ptr), max(self.nbytes, 1)) != 0:
            raise CsmError("hipMalloc failed")
        if array is not None and self.nbytes:
            a = np.ascontiguousarray(array)
            if _hip().hipMemcpy(self.ptr, a.ctypes.data, self.nbytes, 1) != 0:  # H2D
                raise CsmError("hipMemcpy failed")

    def to_numpy(self, dtype, count) -> np.ndarray:
        out = np.empty(count, dtype)
        if out.nbytes and _hip().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, 2) != 0:  # D2H
            raise CsmError("hipMemcpy failed")
        return out

    def free(self):
        if self.ptr:
            _hip().hipFree(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


COMM_ID_BYTES = 128
REDUCE_SUM, REDUCE_MAX = 0, 1


class Comm:
    """The C-ABI's multi-GPU hand-off (csm_comm_*): gather of per-rank byte
    blobs to rank 0 and small integer all-reduces, over RCCL (one process per
    GPU) or TCP between host processes (CPU tests / rehearsals)."""

    def __init__(self, handle, lib):
        self.h, self._lib = handle, lib

    @staticmethod
    def unique_id() -> bytes:
        lib = load_library()
        buf = (C.c_uint8 * COMM_ID_BYTES)()
        _check(lib.csm_comm_get_unique_id(buf), "csm_comm_get_unique_id")
        return bytes(buf)

    @classmethod
    def rccl(cls, context: "Context", rank: int, world_size: int, uid: bytes) -> "Comm":
        lib = load_library()
        if len(uid) != COMM_ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        _check(lib.csm_comm_create_rccl(context.handle, rank, world_size, buf, C.byref(h)),
               "csm_comm_create_rccl")
        return cls(h.value, lib)

    @classmethod
    def tcp(cls, rank: int, world_size: int, host: str = "127.0.0.1", port: int = 29601) -> "Comm":
        lib = load_library()
        h = C.c_void_p()
        _check(lib.csm_comm_create_tcp(rank, world_size, host.encode(), port, C.byref(h)),
               "csm_comm_create_tcp")
        return cls(h.value, lib)

    @property
    def rank(self) -> int:
        return int(self._lib.csm_comm_rank(self.h))

    @property
    def size(self) -> int:
        return int(self._lib.csm_comm_size(self.h))

    def gather(self, blob: bytes):
        """Collective. Rank 0 gets the list of every rank's blob (rank order);
        the other ranks get None."""
        data = C.create_string_buffer(blob, len(blob)) if blob else None
        total = C.c_int64()
        _check(self._lib.csm_comm_gather(self.h, data, len(blob), C.byref(total)), "csm_comm_gather")
        if self.rank != 0:
            return None
        out = C.create_string_buffer(max(total.value, 1))
        sizes = (C.c_int64 * self.size)()
        _check(self._lib.csm_comm_gathered(self.h, out, total.value, sizes), "csm_comm_gathered")
        raw, blobs, at = out.raw, [], 0
        for n in sizes:
            blobs.append(raw[at:at + n])
            at += n
        return blobs

    def allreduce(self, values, op: int = REDUCE_SUM) -> np.ndarray:
        v = np.ascontiguousarray(values, np.int64).copy()
        _check(self._lib.csm_comm_allreduce_i64(self.h, v.ctypes.data_as(C.POINTER(C.c_int64)),
                                                len(v), op), "csm_comm_allreduce_i64")
        return v

    def barrier(self):
        _check(self._lib.csm_comm_barrier(self.h), "csm_comm_barrier")

    def claim_open(self, host: str = "127.0.0.1", port: int = 29621):
        """Collective: starts the rank-0 counter table for fetch_add (the
        shared work queue of common::ThreadPool across ranks)."""
        _check(self._lib.csm_comm_claim_open(self.h, host.encode(), port), "csm_comm_claim_open")

    def fetch_add(self, key: int, delta: int = 1) -> int:
        """Counter `key` before adding `delta`, atomic across ranks."""
        old = C.c_int64()
        _check(self._lib.csm_comm_fetch_add(self.h, key, delta, C.byref(old)), "csm_comm_fetch_add")
        return int(old.value)

    def close(self):
        if self.h:
            self._lib.csm_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synchronize(context: "Context"):
    if _hip().hipStreamSynchronize(C.c_void_p(context.stream)) != 0:
        raise CsmError("hipStreamSynchronize failed")
