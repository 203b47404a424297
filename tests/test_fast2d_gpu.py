"""GPU parity: FastCorrelativeScanMatcher2D on the MI355X vs the oracle.

Bar (north star): score identical (the branch-and-bound maximum is an integer
sum, so bit-identical float), pose identical — or, when another leaf has
exactly the same maximal sum (the reference's unstable std::sort makes its
pick among ties unspecified, fast_correlative_scan_matcher_2d.cc:331-332),
the GPU's leaf must score exactly that maximum in the oracle.

Scenarios restate the reference tests (fast_correlative_scan_matcher_2d_test.cc)
plus BASELINE-shaped synthetic pairs and edge cases.
"""
import math

import numpy as np
import pytest
from conftest import assert_search_ok

pytestmark = pytest.mark.gpu


def _window_of(oracle, limits, cells, init, lin, ang, cloud, sp_from_rotated=0):
    import ctypes as C
    res, mx, my = limits
    pts = np.ascontiguousarray(cloud, np.float32)
    init = np.asarray(init, np.float64)
    ns, step = C.c_int32(), C.c_double()
    oracle.lib.oracle_discretize(res, mx, my, cells.shape[1], cells.shape[0],
                                 init.ctypes.data_as(C.POINTER(C.c_double)), lin, ang,
                                 pts.ctypes.data_as(C.POINTER(C.c_float)), len(pts),
                                 sp_from_rotated, C.byref(ns), None, None, 0, C.byref(step))
    return ns.value, step.value


def full_submap_center(limits, cells):
    res, mx, my = limits
    half = 0.5 * res
    return (mx - half * cells.shape[0], my - half * cells.shape[1], 0.0)


def assert_fast_parity(oracle, om, limits, cells, gpu, ref, full, init, cloud, ties_ok=False):
    """Same match decision, bit-identical score and the reference's pose. The
    v4/v5 kernels restore the reference's pick among exactly tied leaves
    (csm_host.cc ResolveTies), so the pose must be identical; only the v1
    kernel (CSM_SEARCH_KERNEL=1, never chosen by default) keeps the smallest tied leaf
    (ties_ok=True), which is then checked to score exactly the maximum."""
    g_ok, g_score, g_pose = gpu
    o_ok, o_score, o_pose = ref[:3]
    assert g_ok == o_ok, (gpu, ref[:3])
    if not o_ok:
        return "nomatch"
    assert np.float32(g_score) == np.float32(o_score), (g_score, o_score)
    if tuple(g_pose) == tuple(o_pose):
        return "exact"
    assert ties_ok, ("pose differs from the reference's pick", g_pose, o_pose)
    # Exact tie: recover the GPU leaf (scan index, offsets) and score it.
    res = limits[0]
    lin, ang = (1e6 * res, math.pi) if full else (om.lin, om.ang)
    ns, step = _window_of(oracle, limits, cells, init, lin, ang, cloud)
    n_ang = (ns - 1) // 2
    k = int(round((g_pose[2] - init[2]) / step)) + n_ang
    x_off = int(round(-(g_pose[1] - init[1]) / res))
    y_off = int(round(-(g_pose[0] - init[0]) / res))
    assert 0 <= k < ns, (k, ns, g_pose, o_pose)
    _, s = om.score_candidate(full, None if full else init, cloud, k, x_off, y_off, 0)
    assert np.float32(s) == np.float32(o_score), ("GPU leaf is not a tied maximum", g_pose, o_pose)
    return "tie"


def test_precomputation_levels_match_oracle(csm, oracle):
    """PrecomputationGridTest.CorrectValues grid (:37-77): every level bit-exact."""
    rng = np.random.RandomState(42)
    cells = np.zeros((250, 250), np.uint16)
    cells[50:, 50:] = rng.randint(1, 32768, size=(200, 200))
    limits = (0.05, 5.0, 5.0)
    grid = csm.ProbabilityGrid(*limits, cells)
    opts = csm.FastCorrelativeScanMatcherOptions2D(3.0, 1.0, 7, search_depth=9)
    m = csm.FastCorrelativeScanMatcher2D(grid, opts)
    om = oracle.fast2d(limits, cells, 3.0, 1.0, 9)
    for d in range(9):
        np.testing.assert_array_equal(m.read_level(d), om.level(d), err_msg=f"level {d}")


def test_tiny_grid_levels(csm, oracle):
    """TinyProbabilityGrid (:79-117): windows wider than the grid."""
    rng = np.random.RandomState(7)
    cells = rng.randint(0, 32768, size=(4, 4)).astype(np.uint16)
    limits = (0.05, 0.1, 0.1)
    m = csm.FastCorrelativeScanMatcher2D(csm.ProbabilityGrid(*limits, cells),
                                         csm.FastCorrelativeScanMatcherOptions2D(3.0, 1.0, 8))
    om = oracle.fast2d(limits, cells, 3.0, 1.0, 8)
    for d in range(8):
        np.testing.assert_array_equal(m.read_level(d), om.level(d), err_msg=f"level {d}")


def _rigid2f(x, y, a):
    return np.array([x, y, a], np.float32)


def test_correct_pose_match(csm, oracle, search_kernel):
    """FastCorrelativeScanMatcherTest.CorrectPose (:144-192): Match() with
    depth 3 recovers random poses; GPU == oracle on every case."""
    rng = np.random.RandomState(42)
    cloud = np.array([[-2.5, 0.5, 0], [-2.0, 0.5, 0], [0.0, -0.5, 0], [0.5, -1.6, 0],
                      [2.5, 0.5, 0], [2.5, 1.7, 0]], np.float32)
    kinds = []
    for i in range(50):
        d = rng.uniform(-1, 1, 3).astype(np.float32)
        expected = _rigid2f(2 * d[0], 2 * d[1], 0.5 * d[2])
        returns = oracle.transform_cloud(expected, cloud)
        limits, cells = oracle.grid_from_inserts(0.05, 5.0, 5.0, 200, 200,
                                                 [((expected[0], expected[1], 0), returns)])
        grid = csm.ProbabilityGrid(*limits, cells)
        m = csm.FastCorrelativeScanMatcher2D(grid, csm.FastCorrelativeScanMatcherOptions2D(3.0, 1.0, 3))
        om = oracle.fast2d(limits, cells, 3.0, 1.0, 3)
        init = (0.0, 0.0, 0.0)
        gpu = m.Match(init, cloud, 0.1)
        ref = om.match(init, cloud, 0.1)
        kinds.append(assert_fast_parity(oracle, om, limits, cells, gpu, ref, False, init, cloud,
                                        ties_ok=search_kernel == "v1"))
        assert gpu[0] and gpu[1] > 0.1
        # The reference test's own acceptance: pose within IsNearly 0.03.
        assert abs(gpu[2][0] - expected[0]) < 0.1 and abs(gpu[2][1] - expected[1]) < 0.1
    assert kinds.count("exact") + kinds.count("tie") == 50


def test_full_submap_matching(csm, oracle, search_kernel):
    """FastCorrelativeScanMatcherTest.FullSubmapMatching (:194-246), depth 6."""
    rng = np.random.RandomState(42)
    base = np.array([[-2.5, 0.5, 0], [-2.25, 0.5, 0], [0.0, 0.5, 0], [0.25, 1.6, 0],
                     [2.5, 0.5, 0], [2.0, 1.8, 0]], np.float32)
    for i in range(20):
        d = rng.uniform(-1, 1, 6).astype(np.float32)
        pert = _rigid2f(10 * d[0], 10 * d[1], 1.6 * d[2])
        cloud = oracle.transform_cloud(pert, base)
        local = _rigid2f(2 * d[3], 2 * d[4], 0.5 * d[5])
        # expected = local * pert^-1; the grid is built from the scan at `local`.
        c, s = math.cos(local[2]), math.sin(local[2])
        returns = oracle.transform_cloud(local, base)
        limits, cells = oracle.grid_from_inserts(0.05, 5.0, 5.0, 200, 200,
                                                 [((local[0], local[1], 0), returns)])
        grid = csm.ProbabilityGrid(*limits, cells)
        m = csm.FastCorrelativeScanMatcher2D(grid, csm.FastCorrelativeScanMatcherOptions2D(3.0, 1.0, 6))
        om = oracle.fast2d(limits, cells, 3.0, 1.0, 6)
        gpu = m.MatchFullSubmap(cloud, 0.1)
        ref = om.match_full_submap(cloud, 0.1)
        init = full_submap_center(limits, cells)
        assert_fast_parity(oracle, om, limits, cells, gpu, ref, True, init, cloud,
                           ties_ok=search_kernel == "v1")
        assert gpu[0]


@pytest.fixture(scope="module")
def world(csm):
    return csm.SyntheticWorld2D(num_nodes=64, num_submaps=8, decimate_to=200, seed=20250127)


SEARCH_KERNELS = {"v5": {}, "v5-all-hex": {"CSM_SEARCH_KERNEL": "5"},
                  "v5-mixed-lifo": {"CSM_HEX_LEVELS": "8,6,3", "CSM_SEARCH_ORDER": "lifo"},
                  "v4": {"CSM_SEARCH_KERNEL": "4"},
                  "v4-lifo": {"CSM_SEARCH_KERNEL": "4", "CSM_SEARCH_ORDER": "lifo"},
                  "v1": {"CSM_SEARCH_KERNEL": "1"}}


@pytest.fixture(params=list(SEARCH_KERNELS))
def search_kernel(request, monkeypatch):
    """Every search kernel and node order: v5 (the default: hex planes for the
    top level and the one two below, quad planes elsewhere, FIFO node order),
    v5 with every even level hex, hex levels mixed into quad ones under the
    depth-first LIFO order, v4 (quad planes only) in both orders, and v1
    (lanes = points, row-major pyramid; only when forced). The plane
    layout is fixed when a matcher is created, so the variables are set
    before."""
    for var in ("CSM_SEARCH_KERNEL", "CSM_HEX_LEVELS", "CSM_SEARCH_ORDER"):
        monkeypatch.delenv(var, raising=False)
    for var, val in SEARCH_KERNELS[request.param].items():
        monkeypatch.setenv(var, val)
    return request.param


@pytest.mark.parametrize("depth_mode", ["auto", "configured"])
def test_synthetic_full_submap_pairs(csm, oracle, world, depth_mode, search_kernel):
    """BASELINE-shaped 400x400 submaps, N~200 clouds, depth 7, min_score 0.55:
    GPU batch == oracle MatchFullSubmap on every pair."""
    search_depth = 0 if depth_mode == "auto" else 7
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30), 7, search_depth)
    mats = [csm.FastCorrelativeScanMatcher2D(world.grid(s), opts) for s in range(world.num_submaps)]
    scans = csm.ScanSet(None, packed=(world.points, world.offsets))
    pairs_sn = [(s, int(world.submap_nodes[s])) for s in range(8)] + [(1, 3), (2, 40), (5, 17), (7, 0)]
    pairs = csm.make_pairs([p[0] for p in pairs_sn], [p[1] for p in pairs_sn], 0.55)
    res = csm.match_batch(mats, scans, pairs)
    assert_search_ok(csm, res["status"])
    matched = 0
    for k, (s, n) in enumerate(pairs_sn):
        g = world.grid(s)
        limits = (g.resolution, g.max_x, g.max_y)
        om = oracle.fast2d(limits, g.cells, 7.0, math.radians(30), 7)
        cloud = world.cloud(n)
        ref = om.match_full_submap(cloud, 0.55)
        gpu = (res[k]["status"] == 0, float(res[k]["score"]),
               (res[k]["x"], res[k]["y"], res[k]["theta"]))
        assert_fast_parity(oracle, om, limits, g.cells, gpu, ref, True,
                           full_submap_center(limits, g.cells), cloud, ties_ok=search_kernel == "v1")
        matched += int(gpu[0])
    assert matched >= 3


def test_batch_equals_single_calls(csm, world):
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30), 7)
    mats = [csm.FastCorrelativeScanMatcher2D(world.grid(s), opts) for s in range(4)]
    scans = csm.ScanSet(None, packed=(world.points, world.offsets))
    sub = [0, 1, 2, 3, 0, 2]
    nodes = [int(world.submap_nodes[0]), int(world.submap_nodes[1]), 5, 9,
             int(world.submap_nodes[0]) + 1, 30]
    res = csm.match_batch(mats, scans, csm.make_pairs(sub, nodes, 0.5))
    assert_search_ok(csm, res["status"])
    for k, (s, n) in enumerate(zip(sub, nodes)):
        ok, score, pose = mats[s].MatchFullSubmap(world.cloud(n), 0.5)
        assert ok == (res[k]["status"] == 0)
        if ok:
            assert np.float32(score) == res[k]["score"]
            assert pose == (res[k]["x"], res[k]["y"], res[k]["theta"])


def test_match_window_mode_parity(csm, oracle, world, search_kernel):
    """Match() with an initial pose near the truth (the local constraint
    search of ConstraintBuilder2D::ComputeConstraint, :221-235)."""
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30), 7)
    rng = np.random.RandomState(3)
    for s in range(3):
        g = world.grid(s)
        limits = (g.resolution, g.max_x, g.max_y)
        m = csm.FastCorrelativeScanMatcher2D(g, opts)
        om = oracle.fast2d(limits, g.cells, 7.0, math.radians(30), 7)
        n = int(world.submap_nodes[s])
        truth = world.node_poses[n]
        init = (truth[0] + rng.uniform(-1, 1), truth[1] + rng.uniform(-1, 1),
                truth[2] + rng.uniform(-0.3, 0.3))
        cloud = world.cloud(n)
        gpu = m.Match(init, cloud, 0.55)
        ref = om.match(init, cloud, 0.55)
        assert_fast_parity(oracle, om, limits, g.cells, gpu, ref, False, init, cloud,
                           ties_ok=search_kernel == "v1")


def test_edge_cases(csm, oracle, search_kernel):
    cells = np.zeros((20, 30), np.uint16)
    cells[5:8, 10:20] = 30000
    limits = (0.05, 1.0, 1.5)
    g = csm.ProbabilityGrid(*limits, cells)
    m = csm.FastCorrelativeScanMatcher2D(g, csm.FastCorrelativeScanMatcherOptions2D(0.5, 0.3, 4))
    # Empty cloud: never a match (score of an empty scan cannot exceed min_score).
    assert m.MatchFullSubmap(np.zeros((0, 3), np.float32), 0.0)[0] is False
    # A single point and min_score 0: matched, parity with the oracle.
    cloud = np.array([[0.3, -0.2, 0.0]], np.float32)
    om = oracle.fast2d(limits, cells, 0.5, 0.3, 4)
    gpu = m.MatchFullSubmap(cloud, 0.0)
    ref = om.match_full_submap(cloud, 0.0)
    assert_fast_parity(oracle, om, limits, cells, gpu, ref, True, full_submap_center(limits, cells), cloud,
                       ties_ok=search_kernel == "v1")
    # min_score above every attainable score: no match.
    assert m.MatchFullSubmap(cloud, 0.95)[0] is False
    # 1x1 grid.
    one = csm.ProbabilityGrid(0.05, 0.05, 0.05, np.full((1, 1), 20000, np.uint16))
    m1 = csm.FastCorrelativeScanMatcher2D(one, csm.FastCorrelativeScanMatcherOptions2D(0.2, 0.1, 1))
    om1 = oracle.fast2d((0.05, 0.05, 0.05), np.full((1, 1), 20000, np.uint16), 0.2, 0.1, 1)
    gpu = m1.Match((0.0, 0.0, 0.0), cloud, 0.0)
    ref = om1.match((0.0, 0.0, 0.0), cloud, 0.0)
    assert_fast_parity(oracle, om1, (0.05, 0.05, 0.05), np.full((1, 1), 20000, np.uint16), gpu, ref,
                       False, (0.0, 0.0, 0.0), cloud, ties_ok=search_kernel == "v1")


def _run_list_clouds(world):
    """Clouds whose run lists stress the compaction: long runs (split at 255),
    runs crossing 64-point blocks, no runs, and ragged sizes around 64."""
    rng = np.random.default_rng(23)
    base = world.cloud(0)
    a, b = base[10], base[len(base) // 2]
    clouds = [
        np.concatenate([np.repeat(a[None], 600, 0), base[:300]]),          # one run of 600
        np.concatenate([np.repeat(a[None], 70, 0), np.repeat(b[None], 70, 0),
                        np.repeat(a[None], 130, 0)]),                        # runs across blocks
        np.stack([a, b] * 100),                                              # alternating, no runs
        np.repeat(b[None], 256, 0),                                          # exactly 256 in one cell
    ]
    for n in (1, 2, 63, 64, 65, 129):
        clouds.append(base[rng.choice(len(base), n, replace=False)])
    return [np.ascontiguousarray(c, np.float32) for c in clouds]


def test_run_lists_parity(csm, oracle, world, search_kernel):
    """Run-list compaction (consecutive points in one cell scored once with
    their count) leaves every score and pose unchanged, through the batch path
    with ragged clouds in one batch."""
    s = 0
    g = world.grid(s)
    limits = (g.resolution, g.max_x, g.max_y)
    opts = csm.FastCorrelativeScanMatcherOptions2D()
    m = csm.FastCorrelativeScanMatcher2D(g, opts)
    om = oracle.fast2d(limits, g.cells, opts.linear_search_window, opts.angular_search_window,
                       opts.branch_and_bound_depth)
    clouds = _run_list_clouds(world)
    scans = csm.ScanSet(clouds)
    pairs = csm.make_pairs(np.zeros(len(clouds), np.int32), np.arange(len(clouds), dtype=np.int32),
                           0.3, full_submap=True)
    res = csm.match_batch([m], scans, pairs)
    assert_search_ok(csm, res["status"])
    kinds = []
    for k, c in enumerate(clouds):
        gpu = (int(res[k]["status"]) == csm.CSM_OK, float(res[k]["score"]),
               (float(res[k]["x"]), float(res[k]["y"]), float(res[k]["theta"])))
        ref = om.match_full_submap(c, 0.3)
        kinds.append(assert_fast_parity(oracle, om, limits, g.cells, gpu, ref, True,
                                        full_submap_center(limits, g.cells), c,
                                        ties_ok=search_kernel == "v1"))
    assert kinds.count("nomatch") < len(kinds)


def _large_cloud(world, n_points, seed):
    """n_points points: node clouds repeated with a few centimetres of jitter
    (every copy after the first), so cells hold many points and runs split."""
    rng = np.random.default_rng(seed)
    base = world.cloud(int(world.submap_nodes[0]))
    reps = -(-n_points // len(base))
    c = np.concatenate([base] * reps)[:n_points].astype(np.float64)
    jitter = rng.uniform(-0.03, 0.03, c.shape)
    jitter[:len(base)] = 0.0
    c[:, :2] += jitter[:, :2]
    return np.ascontiguousarray(c, np.float32)


@pytest.mark.parametrize("kernel", ["v5", "v4", "v1"])
def test_large_clouds_match_oracle(csm, oracle, world, kernel, monkeypatch):
    """Clouds past 8192 points, up to the boundary's limit kMaxPoints = 16448
    (csm_device.h): Match() with a local window, in one batch with a small
    cloud. v5 (the default for every size) runs one rotation per workgroup
    here, its 16448-point scan and lists in ~128 KB of LDS; v4 and the forced
    v1 kernel too."""
    for var in ("CSM_SEARCH_KERNEL", "CSM_HEX_LEVELS", "CSM_SEARCH_ORDER"):
        monkeypatch.delenv(var, raising=False)
    if kernel != "v5":
        monkeypatch.setenv("CSM_SEARCH_KERNEL", kernel[1:])
    opts = csm.FastCorrelativeScanMatcherOptions2D(1.0, 0.15, 5)
    s = 0
    g = world.grid(s)
    limits = (g.resolution, g.max_x, g.max_y)
    m = csm.FastCorrelativeScanMatcher2D(g, opts)
    om = oracle.fast2d(limits, g.cells, 1.0, 0.15, 5)
    n = int(world.submap_nodes[s])
    truth = world.node_poses[n]
    init = (truth[0] + 0.3, truth[1] - 0.2, truth[2] + 0.05)
    clouds = [_large_cloud(world, 9000, 1), _large_cloud(world, 16448, 2), world.cloud(n)]
    scans = csm.ScanSet(clouds)
    pairs = csm.make_pairs(np.zeros(3, np.int32), np.arange(3, dtype=np.int32), 0.3,
                           full_submap=False, initial=[init] * 3)
    res = csm.match_batch([m], scans, pairs)
    assert_search_ok(csm, res["status"])
    matched = 0
    for k, c in enumerate(clouds):
        gpu = (int(res[k]["status"]) == csm.CSM_OK, float(res[k]["score"]),
               (float(res[k]["x"]), float(res[k]["y"]), float(res[k]["theta"])))
        ref = om.match(init, c, 0.3)
        assert_fast_parity(oracle, om, limits, g.cells, gpu, ref, False, init, c,
                           ties_ok=kernel == "v1")
        matched += int(gpu[0])
    assert matched == 3
    # One point past the limit is refused, not searched.
    big = csm.ScanSet([_large_cloud(world, 16449, 3)])
    r = csm.match_batch([m], big, csm.make_pairs([0], [0], 0.3, full_submap=False, initial=[init]))
    assert int(r[0]["status"]) == csm.CSM_ERANGE
