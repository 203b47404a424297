"""ConstraintBuilder2D drop-in: restates ConstraintBuilder2DTest
(reference mapping/internal/constraints/constraint_builder_2d_test.cc:58-128)
for the Python mirror and the C++ header, plus parity of the builder's
constraints with the oracle on synthetic submaps.

CPU tests: sampler / pose algebra / option defaults, and that the C++ headers
compile and link against libcsm_amd.so. GPU tests: the builder runs the HIP
batch path.
"""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, assert_search_ok

CPP_TEST = os.path.join(ROOT, "tests", "cpp", "constraint_builder_2d_test.cc")
CPP_BIN = os.path.join(ROOT, "tests", "cpp", "_build", "constraint_builder_2d_test")


@pytest.fixture(scope="session")
def cb(csm):
    import importlib
    return importlib.import_module("cartographer_amd.constraint_builder")


def test_fixed_ratio_sampler(cb):
    # common/fixed_ratio_sampler_test.cc: ratio 0.5 alternates, ratio 1 keeps all,
    # ratio 0 drops all, and the sample count tracks ratio * pulses.
    s = cb.FixedRatioSampler(0.5)
    assert [s.Pulse() for _ in range(6)] == [True, False, True, False, True, False]
    assert all(cb.FixedRatioSampler(1.0).Pulse() for _ in range(10))
    assert not any(cb.FixedRatioSampler(0.0).Pulse() for _ in range(10))
    s = cb.FixedRatioSampler(0.3)
    kept = sum(s.Pulse() for _ in range(1000))
    assert kept == 300
    with pytest.raises(ValueError):
        cb.FixedRatioSampler(1.5)


def test_rigid2d_algebra(cb):
    a, b = (1.0, -2.0, 0.7), (0.3, 0.4, -1.9)
    ab = cb.rigid2d_compose(a, b)
    back = cb.rigid2d_compose(cb.rigid2d_inverse(a), ab)
    assert np.allclose(back, b, atol=1e-12)
    ident = cb.rigid2d_compose(a, cb.rigid2d_inverse(a))
    assert np.allclose(ident[:2], (0, 0), atol=1e-12) and abs(ident[2]) < 1e-12


def test_option_defaults(cb):
    o = cb.ConstraintBuilderOptions()  # configuration_files/pose_graph.lua:17-29
    assert (o.sampling_ratio, o.max_constraint_distance, o.min_score,
            o.global_localization_min_score) == (0.3, 15.0, 0.55, 0.6)
    f = o.fast_correlative_scan_matcher_options
    assert (f.linear_search_window, f.branch_and_bound_depth) == (7.0, 7)
    assert math.isclose(f.angular_search_window, math.radians(30.0))


def _build_cpp():
    os.makedirs(os.path.dirname(CPP_BIN), exist_ok=True)
    libdir = os.path.join(ROOT, "cartographer-1_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
                           "-I", os.path.join(ROOT, "include"), CPP_TEST, "-o", CPP_BIN,
                           "-L", libdir, "-lcsm_amd", "-Wl,-rpath," + libdir])


def test_cpp_headers_compile_and_link(csm):
    _build_cpp()
    assert os.access(CPP_BIN, os.X_OK)


@pytest.mark.gpu
def test_cpp_constraint_builder(csm, oracle):
    """The C++ restatement of ConstraintBuilder2DTest passes, and its
    FindsConstraints constraints (all-unknown grid, every leaf tied) are the
    oracle's picks refined by the CeresScanMatcher2D restatement
    (oracle/ceres2d.cc; parity with Ceres itself unpinned), in the submap frame."""
    import importlib
    cb = importlib.import_module("cartographer_amd.constraint_builder")
    _build_cpp()
    out = subprocess.run([CPP_BIN], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "OK" in out.stdout
    got = [tuple(float(v) for v in line.split()[1:]) for line in out.stdout.splitlines()
           if line.startswith("FINDS_CONSTRAINTS")]
    assert len(got) == 3
    cells = np.zeros((110, 100), np.uint16)
    limits = (1.0, 2.0, 3.0)
    f = cb.ConstraintBuilderOptions().fast_correlative_scan_matcher_options
    om = oracle.fast2d(limits, cells, f.linear_search_window, f.angular_search_window,
                       f.branch_and_bound_depth)
    cloud = np.array([[0.1, 0.2, 0.3]], np.float32)
    origin = (4.0, 5.0, 0.0)
    refs = [om.match(origin, cloud, 0.0)] * 2 + [om.match_full_submap(cloud, 0.0)]
    o = cb.ConstraintBuilderOptions().ceres_scan_matcher_options
    copts = (o.occupied_space_weight, o.translation_weight, o.rotation_weight, o.max_num_iterations)
    for g, ref in zip(got, refs):
        assert ref[0] and np.float32(g[3]) == np.float32(ref[1])
        want, _ = oracle.ceres2d_match(limits, cells, copts, ref[2][:2], ref[2], cloud)
        pose = cb.rigid2d_compose(origin, g[:3])
        assert np.allclose(pose, want, atol=1e-6), (pose, want)


def _unknown_submap(csm, cb):
    # MapLimits(1., (2., 3.), CellLimits(100, 110)); Submap2D origin (4, 5).
    grid = csm.ProbabilityGrid(1.0, 2.0, 3.0, np.zeros((110, 100), np.uint16))
    return cb.Submap2D(grid, (4.0, 5.0, 0.0))


def _test_options(cb):
    return cb.ConstraintBuilderOptions(sampling_ratio=1.0, min_score=0.0,
                                       global_localization_min_score=0.0)


@pytest.mark.gpu
def test_calls_back(csm, cb):
    builder = cb.ConstraintBuilder2D(_test_options(cb))
    assert builder.GetNumFinishedNodes() == 0
    builder.NotifyEndOfNode()
    got = []
    builder.WhenDone(got.append)
    assert got == [[]]
    assert builder.GetNumFinishedNodes() == 1


@pytest.mark.gpu
def test_finds_constraints(csm, cb):
    builder = cb.ConstraintBuilder2D(_test_options(cb))
    cloud = np.array([[0.1, 0.2, 0.3]], np.float32)
    submap = _unknown_submap(csm, cb)
    submap_id = (0, 1)
    expected_nodes = 0
    for _ in range(2):
        assert builder.GetNumFinishedNodes() == expected_nodes
        for _ in range(2):
            builder.MaybeAddConstraint(submap_id, submap, (0, 0), cloud, (0.0, 0.0, 0.0))
        builder.MaybeAddGlobalConstraint(submap_id, submap, (0, 0), cloud)
        builder.NotifyEndOfNode()
        expected_nodes += 1
        assert builder.GetNumFinishedNodes() == expected_nodes
        builder.NotifyEndOfNode()
        expected_nodes += 1
        assert builder.GetNumFinishedNodes() == expected_nodes
        got = []
        builder.WhenDone(got.append)
        assert len(got) == 1 and len(got[0]) == 3
        assert all(c.tag == "INTER_SUBMAP" for c in got[0])
        builder.DeleteScanMatcher(submap_id)
        assert builder.num_submap_scan_matchers == 0


@pytest.mark.gpu
def test_skips_unsearchable_pairs(csm, cb, capsys):
    """A cloud past the device limit (16448 points: CSM_ERANGE) yields no
    constraint and is counted in constraints_failed, exactly as the C++
    header does (tests/cpp/constraint_builder_2d_test.cc); the rest of the
    flush is unaffected and nothing raises."""
    builder = cb.ConstraintBuilder2D(_test_options(cb))
    submap = _unknown_submap(csm, cb)
    small = np.array([[0.1, 0.2, 0.3]], np.float32)
    i = np.arange(16449)
    huge = np.stack([0.001 * (i % 100), 0.001 * (i // 100), np.zeros(len(i))], 1).astype(np.float32)
    builder.MaybeAddGlobalConstraint((0, 1), submap, (0, 0), small)
    builder.MaybeAddGlobalConstraint((0, 1), submap, (0, 1), huge)
    builder.NotifyEndOfNode()
    got = []
    builder.WhenDone(got.append)
    assert len(got[0]) == 1 and got[0][0].node_id == (0, 0)
    assert builder.constraints_failed == 1 and builder.last_error == csm.CSM_ERANGE
    assert builder.global_constraints_searched == 1 and builder.global_constraints_found == 1
    assert "1 of 2 pairs skipped" in capsys.readouterr().err


@pytest.mark.gpu
def test_distance_filter_and_sampling(csm, cb):
    opts = _test_options(cb)
    opts.sampling_ratio = 0.5
    builder = cb.ConstraintBuilder2D(opts)
    submap = _unknown_submap(csm, cb)
    cloud = np.array([[0.1, 0.2, 0.3]], np.float32)
    builder.MaybeAddConstraint((0, 0), submap, (0, 0), cloud, (15.1, 0.0, 0.0))  # too far
    for _ in range(4):
        builder.MaybeAddConstraint((0, 0), submap, (0, 0), cloud, (1.0, 1.0, 0.0))
    builder.NotifyEndOfNode()
    got = []
    builder.WhenDone(got.append)
    assert len(got[0]) == 2  # 4 pulses at ratio 0.5
    assert builder.constraints_searched == 2


@pytest.mark.gpu
def test_builder_constraints_match_oracle(csm, cb, oracle):
    """Constraints from the builder equal the oracle's Match / MatchFullSubmap
    on the same pairs (score bit-identical, pose identical or an exact tie),
    expressed in the submap frame as ComputeConstraint does (:251-252)."""
    from test_fast2d_gpu import assert_fast_parity
    world = csm.SyntheticWorld2D(num_nodes=48, num_submaps=4, decimate_to=160, seed=7)
    fopts = csm.FastCorrelativeScanMatcherOptions2D()
    opts = cb.ConstraintBuilderOptions(sampling_ratio=1.0, min_score=0.4,
                                       global_localization_min_score=0.45,
                                       max_constraint_distance=1e9,
                                       fast_correlative_scan_matcher_options=fopts,
                                       refine_with_ceres=False)
    builder = cb.ConstraintBuilder2D(opts)
    rng = np.random.default_rng(3)
    # Non-trivial submap poses: the builder composes the search start with it
    # (:195-197) and expresses the result in the submap frame (:251-252).
    local = {s: (0.2 * s, -0.1 * s, 0.0) for s in range(world.num_submaps)}
    submaps = {s: cb.Submap2D(world.grid(s), local[s]) for s in range(world.num_submaps)}
    expected = []
    for node in range(0, world.num_nodes, 3):
        cloud = world.cloud(node)
        for s in range(world.num_submaps):
            if (node + s) % 4 == 0:
                builder.MaybeAddGlobalConstraint((0, s), submaps[s], (0, node), cloud)
                expected.append((s, node, None))
            else:
                pose = world.node_poses[node] + rng.normal(0, [0.3, 0.3, 0.05])
                rel = cb.rigid2d_compose(cb.rigid2d_inverse(local[s]), tuple(pose))
                builder.MaybeAddConstraint((0, s), submaps[s], (0, node), cloud, rel)
                expected.append((s, node, cb.rigid2d_compose(local[s], rel)))
        builder.NotifyEndOfNode()
    got = []
    builder.WhenDone(got.append)
    got = got[0]

    from test_fast2d_gpu import full_submap_center
    oms, want = {}, []
    for s, node, init in expected:
        g = world.grid(s)
        limits = (g.resolution, g.max_x, g.max_y)
        if s not in oms:
            oms[s] = oracle.fast2d(limits, g.cells, fopts.linear_search_window,
                                   fopts.angular_search_window, fopts.branch_and_bound_depth)
        cloud = world.cloud(node)
        if init is None:
            ref = oms[s].match_full_submap(cloud, opts.global_localization_min_score)
            ctr = full_submap_center(limits, g.cells)
        else:
            ref = oms[s].match(init, cloud, opts.min_score)
            ctr = init
        if ref[0]:  # failed searches are dropped (RunWhenDoneCallback :285-288)
            want.append((s, node, init is None, ctr, ref, limits, g.cells, cloud))
    assert len(got) == len(want) and len(want) > 5
    for c, (s, node, full, ctr, ref, limits, cells, cloud) in zip(got, want):
        assert c.submap_id == (0, s) and c.node_id == (0, node)
        assert c.tag == "INTER_SUBMAP"
        assert c.translation_weight == opts.loop_closure_translation_weight
        assert c.rotation_weight == opts.loop_closure_rotation_weight
        pose = cb.rigid2d_compose(local[s], c.relative_pose)
        assert_fast_parity(oracle, oms[s], limits, cells, (True, c.score, pose), ref, full,
                           ctr, cloud)


@pytest.mark.gpu
def test_builder_refines_accepted_matches(csm, cb, oracle):
    """With refine_with_ceres (the reference's ComputeConstraint, :245-249),
    each constraint is the CeresScanMatcher2D refinement of the branch-and-bound
    match: oracle/ceres2d.cc started from the builder's own match pose (the
    unrefined run), to 1e-6 (parity with Ceres itself unpinned)."""
    world = csm.SyntheticWorld2D(num_nodes=30, num_submaps=3, decimate_to=200, seed=17)
    base = dict(sampling_ratio=1.0, min_score=0.4, global_localization_min_score=0.4,
                max_constraint_distance=1e9)
    runs = {}
    for refine in (False, True):
        builder = cb.ConstraintBuilder2D(cb.ConstraintBuilderOptions(refine_with_ceres=refine,
                                                                     **base))
        local = {s: (0.1 * s, -0.2 * s, 0.05 * s) for s in range(world.num_submaps)}
        for node in range(0, world.num_nodes, 2):
            for s in range(world.num_submaps):
                sm = cb.Submap2D(world.grid(s), local[s])
                builder.MaybeAddGlobalConstraint((0, s), sm, (0, node), world.cloud(node))
            builder.NotifyEndOfNode()
        got = []
        builder.WhenDone(got.append)
        runs[refine] = (got[0], local)
    plain, local = runs[False]
    refined, _ = runs[True]
    assert len(plain) == len(refined) and len(plain) >= 3
    o = cb.ConstraintBuilderOptions().ceres_scan_matcher_options
    opts = (o.occupied_space_weight, o.translation_weight, o.rotation_weight,
            o.max_num_iterations)
    for a, b in zip(plain, refined):
        assert a.submap_id == b.submap_id and a.node_id == b.node_id and a.score == b.score
        s = a.submap_id[1]
        match = cb.rigid2d_compose(local[s], a.relative_pose)  # global CSM pose
        g = world.grid(s)
        ref, _ = oracle.ceres2d_match((g.resolution, g.max_x, g.max_y), g.cells, opts,
                                      match[:2], match, world.cloud(a.node_id[1]))
        got_pose = cb.rigid2d_compose(local[s], b.relative_pose)
        assert np.allclose(got_pose, ref, atol=1e-6), (got_pose, ref)


@pytest.mark.gpu
def test_scan_set_append_matches_fresh_set(csm):
    """csm_scan_set_append: scans appended in steps (the device buffer grows
    and keeps the resident clouds) give the same batch results as one set
    made from all clouds at once, and earlier indices stay valid."""
    world = csm.SyntheticWorld2D(num_nodes=40, num_submaps=3, decimate_to=300, seed=11)
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30), 7)
    mats = [csm.FastCorrelativeScanMatcher2D(world.grid(s), opts) for s in range(3)]
    clouds = [world.cloud(n) for n in range(world.num_nodes)]
    fresh = csm.ScanSet(clouds)
    grown = csm.ScanSet(clouds[:2])
    assert grown.append(clouds[2:5]) == 2
    assert grown.append([]) == 5
    assert grown.append(clouds[5:]) == 5  # past the initial capacity: device-to-device growth
    assert grown.device_size() == (len(clouds), sum(len(c) for c in clouds))
    assert len(grown) == len(clouds)
    sub = [n % 3 for n in range(world.num_nodes)] + [int(s) for s in range(3)]
    nodes = list(range(world.num_nodes)) + [int(world.submap_nodes[s]) for s in range(3)]
    pairs = csm.make_pairs(sub, nodes, 0.5)
    a = csm.match_batch(mats, fresh, pairs)
    b = csm.match_batch(mats, grown, pairs)
    assert_search_ok(csm, a["status"])
    assert (a == b).all()
    assert (a["status"] == 0).sum() >= 3
    # Malformed appends are refused and leave the set as it was.
    import ctypes as C
    lib, first = grown._lib, C.c_int32(-7)
    pts = np.zeros((4, 3), np.float32)
    bad_start = np.array([1, 4], np.int64)    # offsets[0] must be 0
    decreasing = np.array([0, 3, 2], np.int64)
    for offs in (bad_start, decreasing):
        rc = lib.csm_scan_set_append(grown.handle, pts.ctypes.data_as(C.POINTER(C.c_float)),
                                     offs.ctypes.data_as(C.POINTER(C.c_int64)), len(offs) - 1,
                                     C.byref(first))
        assert rc == csm.CSM_EINVAL and first.value == -7
    assert grown.device_size() == (len(clouds), sum(len(c) for c in clouds))


@pytest.mark.gpu
def test_builder_keeps_node_clouds_resident(csm, cb):
    """The 2D builder uploads a node's cloud once across flushes (the pattern
    of a finished submap matched against earlier nodes,
    pose_graph_2d.cc:379-392), also when the caller hands a fresh array with
    the same points; a node whose points change is uploaded again; results
    equal a builder that starts a new set every flush (cache limit 0)."""
    world = csm.SyntheticWorld2D(num_nodes=24, num_submaps=3, decimate_to=200, seed=5)
    fopts = csm.FastCorrelativeScanMatcherOptions2D()

    def run(cache_points):
        opts = cb.ConstraintBuilderOptions(sampling_ratio=1.0, min_score=0.4,
                                           global_localization_min_score=0.45,
                                           max_constraint_distance=1e9,
                                           fast_correlative_scan_matcher_options=fopts,
                                           refine_with_ceres=False,
                                           scan_cache_points=cache_points)
        b = cb.ConstraintBuilder2D(opts)
        submaps = {s: cb.Submap2D(world.grid(s), (0.0, 0.0, 0.0)) for s in range(3)}
        for s in range(3):  # each "finished submap" against every node so far
            for node in range(8 * (s + 1)):
                cloud = world.cloud(node)
                if s == 2 and node == 1:
                    cloud = cloud.copy()
                    cloud[0, 0] += 0.05  # changed points: uploaded again
                b.MaybeAddGlobalConstraint((0, s), submaps[s], (0, node), cloud)
            b.NotifyEndOfNode()
        got = []
        b.WhenDone(got.append)
        return b, got[0]

    b, got = run(1 << 25)
    # 8 + 8 + 8 new nodes, plus node 1's changed cloud.
    assert b._scans.device_size()[0] == 25
    ref_b, ref = run(0)
    assert len(got) == len(ref) > 3
    for c, r in zip(got, ref):
        assert (c.submap_id, c.node_id, c.score, c.relative_pose) == \
            (r.submap_id, r.node_id, r.score, r.relative_pose)
    assert b.global_constraints_searched == ref_b.global_constraints_searched == 48


@pytest.mark.gpu
def test_matcher_budget_2000_submap_sweep(csm, cb):
    """A 2000-submap sweep under a 4 GB matcher budget (about 160 of the
    ~25 MB 400x400 matchers; the unbounded run holds all 2000, ~50 GB): the
    cache drops and rebuilds matchers and cuts every flush into sub-batches
    that fit, and delivers the unbounded run's constraints in the same order
    (the reference keeps every matcher, constraint_builder_2d.cc:165-186)."""
    world = csm.SyntheticWorld2D(num_nodes=2000, num_submaps=2000, submap_cells=400, beams=1080,
                                 seed=20250127)
    submaps = [cb.Submap2D(world.grid(s), (0.0, 0.0, 0.0)) for s in range(world.num_submaps)]
    nodes = [int(world.submap_nodes[s]) for s in (3, 700, 1400)] + [1999]

    def run(budget):
        opts = cb.ConstraintBuilderOptions(max_constraint_distance=1e9, matcher_cache_bytes=budget)
        b = cb.ConstraintBuilder2D(opts, csm.Context(0))
        for n in nodes:
            for s in range(world.num_submaps):
                b.MaybeAddGlobalConstraint((0, s), submaps[s], (0, n), world.cloud(n))
            b.NotifyEndOfNode()
        got = []
        b.WhenDone(got.append)
        return b, got[0]

    ref_b, ref = run(0)
    assert ref_b.matcher_cache.evictions == 0 and len(ref_b.matcher_cache) == 2000
    budget = 4 << 30
    b, got = run(budget)
    cache = b.matcher_cache
    assert cache.evictions > 0 and cache.builds > 2000
    assert cache.bytes <= budget
    assert len(got) == len(ref) >= 3
    for c, r in zip(got, ref):
        assert (c.submap_id, c.node_id, c.score, c.relative_pose) == \
            (r.submap_id, r.node_id, r.score, r.relative_pose)
    assert b.global_constraints_searched == ref_b.global_constraints_searched == 4 * 2000
