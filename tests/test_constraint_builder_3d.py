"""ConstraintBuilder3D drop-in: restates ConstraintBuilder3DTest (reference
mapping/internal/constraints/constraint_builder_3d_test.cc:40-116) for the
Python mirror and the C++ header, plus parity of the builder's constraints
with the oracle's FastCorrelativeScanMatcher3D on synthetic C5-shaped pairs.

CPU tests: option defaults, the C++ headers compile and link against
libcsm_amd.so. GPU tests: the builder runs the HIP batch path.
"""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

CPP_TEST = os.path.join(ROOT, "tests", "cpp", "constraint_builder_3d_test.cc")
CPP_BIN = os.path.join(ROOT, "tests", "cpp", "_build", "constraint_builder_3d_test")


@pytest.fixture(scope="session")
def cb(csm):
    import importlib
    return importlib.import_module("cartographer_amd.constraint_builder")


def test_option_defaults_3d(cb):
    o = cb.ConstraintBuilderOptions()  # configuration_files/pose_graph.lua:17-48
    f = o.fast_correlative_scan_matcher_options_3d
    assert (f.branch_and_bound_depth, f.full_resolution_depth) == (8, 3)
    assert (f.min_rotational_score, f.min_low_resolution_score) == (0.77, 0.55)
    assert (f.linear_xy_search_window, f.linear_z_search_window) == (5.0, 1.0)
    assert math.isclose(f.angular_search_window, math.radians(15.0))


def _build_cpp():
    os.makedirs(os.path.dirname(CPP_BIN), exist_ok=True)
    libdir = os.path.join(ROOT, "cartographer-1_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
                           "-I", os.path.join(ROOT, "include"), CPP_TEST, "-o", CPP_BIN,
                           "-L", libdir, "-lcsm_amd", "-Wl,-rpath," + libdir])


def test_cpp_headers_compile_and_link_3d(csm):
    _build_cpp()
    assert os.access(CPP_BIN, os.X_OK)


@pytest.mark.gpu
def test_cpp_constraint_builder_3d(csm, oracle):
    """The C++ restatement of ConstraintBuilder3DTest passes, and its
    FindsConstraints constraints (an empty submap, every leaf tied) are the
    oracle's Match / MatchFullSubmap picks refined by the CeresScanMatcher3D
    restatement (oracle/ceres3d.cc; parity with Ceres itself unpinned)."""
    import importlib
    cb = importlib.import_module("cartographer_amd.constraint_builder")
    from test_fast3d_gpu import opt_tuple
    _build_cpp()
    out = subprocess.run([CPP_BIN], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "OK" in out.stdout
    got = [tuple(float(v) for v in line.split()[1:]) for line in out.stdout.splitlines()
           if line.startswith("FINDS_CONSTRAINTS")]
    assert len(got) == 3
    f = csm.FastCorrelativeScanMatcherOptions3D(min_rotational_score=0.0,
                                                 min_low_resolution_score=0.0)
    og_h, og_l = oracle.hybrid_grid(0.1), oracle.hybrid_grid(0.1)
    om = oracle.fast3d(og_h, og_l, np.zeros(3, np.float32), opt_tuple(f))
    pt = np.array([[0.1, 0.2, 0.3]], np.float32)
    node = csm.NodeData3D(pt, pt, np.zeros(3, np.float32))
    ident = ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))
    refs = [om.match(ident, ident, node, 0.0)] * 2 + \
        [om.match_full_submap((1, 0, 0, 0), (1, 0, 0, 0), node, 0.0)]
    o3 = cb.ConstraintBuilderOptions().ceres_scan_matcher_options_3d
    copts = (o3.occupied_space_weight_0, o3.occupied_space_weight_1, o3.translation_weight,
             o3.rotation_weight, o3.max_num_iterations)
    for g, ref in zip(got, refs):
        assert ref["matched"] and np.float32(g[7]) == np.float32(ref["score"])
        t, q = ref["pose"]
        (rt, rq), _ = oracle.ceres3d_match(og_h, og_l, pt, pt, copts, t, t, q)
        assert np.allclose(g[0:3], rt, atol=1e-6), (g, rt)
        assert np.allclose(g[3:7], rq, atol=1e-6), (g, rq)


def _test_options(cb, csm):
    f = csm.FastCorrelativeScanMatcherOptions3D(min_rotational_score=0.0,
                                                 min_low_resolution_score=0.0)
    return cb.ConstraintBuilderOptions(sampling_ratio=1.0, min_score=0.0,
                                       global_localization_min_score=0.0,
                                       fast_correlative_scan_matcher_options_3d=f)


def _empty_submap(cb):
    # Submap3D(0.1, 0.1, Identity, VectorXf::Zero(3)) (:82-83): no cells.
    empty = (np.zeros((0, 3), np.int32), np.zeros(0, np.uint16))
    return cb.Submap3D(0.1, empty, 0.1, empty, np.zeros(3, np.float32))


@pytest.mark.gpu
def test_calls_back_3d(csm, cb):  # :61-71
    builder = cb.ConstraintBuilder3D(_test_options(cb, csm))
    assert builder.GetNumFinishedNodes() == 0
    got = []
    builder.NotifyEndOfNode()
    builder.WhenDone(got.append)
    assert got == [[]]
    assert builder.GetNumFinishedNodes() == 1


@pytest.mark.gpu
def test_finds_constraints_3d(csm, cb):  # :73-116
    node = csm.NodeData3D(np.array([[0.1, 0.2, 0.3]], np.float32),
                          np.array([[0.1, 0.2, 0.3]], np.float32), np.zeros(3, np.float32))
    submap = _empty_submap(cb)
    builder = cb.ConstraintBuilder3D(_test_options(cb, csm))
    ident = ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))
    expected_nodes = 0
    for _ in range(2):
        assert builder.GetNumFinishedNodes() == expected_nodes
        for _ in range(2):
            builder.MaybeAddConstraint((0, 1), submap, (0, 0), node, ident, ident)
        builder.MaybeAddGlobalConstraint((0, 1), submap, (0, 0), node, (1, 0, 0, 0),
                                         (1, 0, 0, 0))
        builder.NotifyEndOfNode()
        expected_nodes += 1
        assert builder.GetNumFinishedNodes() == expected_nodes
        builder.NotifyEndOfNode()
        expected_nodes += 1
        assert builder.GetNumFinishedNodes() == expected_nodes
        got = []
        builder.WhenDone(got.append)
        assert len(got[0]) == 3
        assert all(c.tag == "INTER_SUBMAP" for c in got[0])
        builder.DeleteScanMatcher((0, 1))
        assert builder.num_submap_scan_matchers == 0
    assert (builder.constraints_searched, builder.constraints_found) == (4, 4)
    assert (builder.global_constraints_searched, builder.global_constraints_found) == (2, 2)


@pytest.mark.gpu
def test_builder_matches_oracle_on_synthetic_pairs(csm, cb, oracle):
    """Local and global constraints on C5-shaped submaps: every constraint the
    builder emits equals the oracle's Match / MatchFullSubmap result for that
    pair (score and pose, or an exactly tied leaf), failures are dropped, and
    the distance filter and sampler act before any search."""
    from test_fast3d_gpu import assert_same_result, opt_tuple
    w = csm.SyntheticWorld3D(num_nodes=16, num_submaps=2, seed=41)
    o = cb.ConstraintBuilderOptions(sampling_ratio=0.5, refine_with_ceres=False)
    f3 = o.fast_correlative_scan_matcher_options_3d
    builder = cb.ConstraintBuilder3D(o)
    subs, oms = [], []
    for s in range(w.num_submaps):
        subs.append(cb.Submap3D(w.high_resolution, w.high_cells[s], w.low_resolution,
                                w.low_cells[s], w.submap_hist[s]))
        oh, ol = oracle.hybrid_grid(w.high_resolution), oracle.hybrid_grid(w.low_resolution)
        oh.set_values(*w.high_cells[s])
        ol.set_values(*w.low_cells[s])
        oms.append((oh, ol, oracle.fast3d(oh, ol, w.submap_hist[s], opt_tuple(f3))))
    submitted = []
    sampler = {s: cb.FixedRatioSampler(o.sampling_ratio) for s in range(w.num_submaps)}
    for n in range(w.num_nodes):
        node = w.node(n)
        for s in range(w.num_submaps):
            truth = w.node_in_submap(n, s)
            gnode = ((truth[0][0] + 0.2, truth[0][1] - 0.1, 0.05), truth[1])
            gsub = ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))
            builder.MaybeAddConstraint((0, s), subs[s], (0, n), node, gnode, gsub)
            if math.sqrt(sum(v * v for v in gnode[0])) <= o.max_constraint_distance and \
                    sampler[s].Pulse():
                submitted.append((s, n, False, gnode, gsub))
            if n % 5 == 0:
                builder.MaybeAddGlobalConstraint((0, s), subs[s], (0, n), node,
                                                 w.node_rotation(n), (1, 0, 0, 0))
                submitted.append((s, n, True, w.node_rotation(n), (1, 0, 0, 0)))
        builder.NotifyEndOfNode()
    got = []
    builder.WhenDone(got.append)
    got = got[0]
    expected = []
    for s, n, full, a, b in submitted:
        om = oms[s][2]
        node = w.node(n)
        ref = (om.match_full_submap(a, b, node, o.global_localization_min_score) if full
               else om.match(a, b, node, o.min_score))
        if ref["matched"]:
            expected.append((s, n, full, a, b, ref))
    assert len(got) == len(expected) and len(got) >= 3
    for c, (s, n, full, a, b, ref) in zip(got, expected):
        assert c.submap_id == (0, s) and c.node_id == (0, n)
        r = type("R", (), {})()
        r.score, r.pose_estimate = c.score, c.relative_pose
        r.rotational_score, r.low_resolution_score = c.rotational_score, c.low_resolution_score
        assert_same_result(r, ref, oms[s][2], full, a, b, w.node(n), f3.min_low_resolution_score)
        assert c.translation_weight == o.loop_closure_translation_weight
    assert builder.constraints_searched + builder.global_constraints_searched == len(submitted)


@pytest.mark.gpu
def test_builder_refines_accepted_matches_3d(csm, cb, oracle):
    """With refine_with_ceres (the reference's ComputeConstraint, :264-275) each
    3D constraint is the CeresScanMatcher3D refinement of the unrefined
    builder's match (oracle/ceres3d.cc, to 1e-6; parity with Ceres unpinned)."""
    w = csm.SyntheticWorld3D(num_nodes=10, num_submaps=2, seed=43)
    runs = {}
    for refine in (False, True):
        o = cb.ConstraintBuilderOptions(sampling_ratio=1.0, refine_with_ceres=refine)
        builder = cb.ConstraintBuilder3D(o)
        for node in range(w.num_nodes):
            for s in range(w.num_submaps):
                sub = cb.Submap3D(w.high_resolution, w.high_cells[s], w.low_resolution,
                                  w.low_cells[s], w.submap_hist[s])
                builder.MaybeAddGlobalConstraint((0, s), sub, (0, node), w.node(node),
                                                 w.node_rotation(node), (1.0, 0.0, 0.0, 0.0))
            builder.NotifyEndOfNode()
        got = []
        builder.WhenDone(got.append)
        runs[refine] = got[0]
    plain, refined = runs[False], runs[True]
    assert len(plain) == len(refined) and len(plain) > 0
    ogr = {}
    o3 = cb.ConstraintBuilderOptions().ceres_scan_matcher_options_3d
    opts = (o3.occupied_space_weight_0, o3.occupied_space_weight_1, o3.translation_weight,
            o3.rotation_weight, o3.max_num_iterations)
    for a, b in zip(plain, refined):
        assert a.submap_id == b.submap_id and a.node_id == b.node_id and a.score == b.score
        s, n = a.submap_id[1], a.node_id[1]
        if s not in ogr:
            hg, lg = oracle.hybrid_grid(w.high_resolution), oracle.hybrid_grid(w.low_resolution)
            hg.set_values(*w.high_cells[s])
            lg.set_values(*w.low_cells[s])
            ogr[s] = (hg, lg)
        t, q = a.relative_pose
        (rt, rq), _ = oracle.ceres3d_match(ogr[s][0], ogr[s][1], w.high[n], w.low[n], opts, t, t, q)
        assert np.allclose(b.relative_pose[0], rt, atol=1e-6)
        assert np.allclose(b.relative_pose[1], rq, atol=1e-6)
