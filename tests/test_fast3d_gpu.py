"""GPU parity: FastCorrelativeScanMatcher3D and RealTimeCorrelativeScanMatcher3D
on the MI355X vs the oracle.

Bar: pyramid levels byte-identical; FastCSM3D score, rotational score and
low-resolution score identical floats, pose identical (including the
reference's pick among exactly tied leaves); RTCSM3D score within 1e-6 relative (the double exp() penalty may
differ from glibc in the last ulps) and the same winning candidate.

Scenarios restate fast_correlative_scan_matcher_3d_test.cc:36-204 and
real_time_correlative_scan_matcher_3d_test.cc:34-117, plus variants with
half-resolution levels (full_resolution_depth < branch_and_bound_depth) and
non-trivial rotational histograms.
"""
import math

import numpy as np
import pytest
from conftest import assert_search_ok

pytestmark = pytest.mark.gpu

TEST_CLOUD = np.array([[4, 0, 0], [4.5, 0, 0], [5, 0, 0], [5.5, 0, 0], [0, 4, 0], [0, 4.5, 0],
                       [0, 5, 0], [0, 5.5, 0], [0, 0, 4], [0, 0, 4.5], [0, 0, 5], [0, 0, 5.5]],
                      np.float32)


def quat_z(theta):
    return (math.cos(0.5 * theta), 0.0, 0.0, math.sin(0.5 * theta))


def transform(cloud, t, q):
    w, x, y, z = q
    r = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                  [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                  [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
    return (np.asarray(cloud, np.float64) @ r.T + np.asarray(t)).astype(np.float32)


def gpu_grid(csm, og):
    ijk, v = og.cells()
    return csm.HybridGrid(og.resolution, ijk, v, grid_size=og.grid_size)


def assert_same_result(gpu, ref, om=None, full=False, node_pose=None, submap_pose=None,
                       node=None, min_low=0.15):
    """Identical result: match decision, score, pose, rotational and
    low-resolution scores. Among leaves that tie at the maximum and pass the
    low-resolution check the reference returns the first its depth-first
    search reaches (fast_correlative_scan_matcher_3d.cc:332-355, :377-440);
    the GPU restores that pick (host3d.cc ResolveTies3d), so the pose must be
    the oracle's in every case. Returns "tie" when the GPU reported resolving
    a tie (csm_result3d.tie), else "exact"."""
    assert (gpu is not None) == ref["matched"], (gpu, ref)
    if gpu is None:
        return "nomatch"
    assert np.float32(gpu.score) == np.float32(ref["score"])
    (gt, gq), (rt, rq) = gpu.pose_estimate, ref["pose"]
    assert tuple(gt) == tuple(rt) and tuple(gq) == tuple(rq), \
        ("pose differs from the reference's pick", gpu, ref)
    assert np.float32(gpu.rotational_score) == np.float32(ref["rotational_score"])
    assert np.float32(gpu.low_resolution_score) == np.float32(ref["low_resolution_score"])
    return "tie" if getattr(gpu, "tie", 0) else "exact"


def options(csm, depth, full_depth, **kw):
    o = csm.FastCorrelativeScanMatcherOptions3D(depth, full_depth, 0.1, 0.15, 0.8, 0.8, 0.3)
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def opt_tuple(o):
    return (o.branch_and_bound_depth, o.full_resolution_depth, o.min_rotational_score,
            o.min_low_resolution_score, o.linear_xy_search_window, o.linear_z_search_window,
            o.angular_search_window)


def fixture(csm, oracle, pose_t, pose_q, o, histogram=None):
    og = oracle.hybrid_grid(0.05)
    og.insert(pose_t, transform(TEST_CLOUD, pose_t, pose_q), 0.7, 0.4, 5)
    hist = np.zeros(10, np.float32) if histogram is None else histogram
    om = oracle.fast3d(og, og, hist, opt_tuple(o))
    g = gpu_grid(csm, og)
    gm = csm.FastCorrelativeScanMatcher3D(g, g, hist, o)
    return og, om, g, gm


@pytest.mark.parametrize("depth,full_depth", [(6, 6), (6, 3), (8, 3)])
def test_levels_match_oracle(csm, oracle, depth, full_depth):
    o = options(csm, depth, full_depth)
    og, om, g, gm = fixture(csm, oracle, (0.3, -0.2, 0.1), quat_z(0.1), o)
    for d in range(depth):
        ijk, v = om.level(d)
        origin, brick = gm.read_level(d)
        assert np.count_nonzero(brick) == np.count_nonzero(v)
        loc = ijk - np.asarray(origin)
        assert np.all(brick[loc[:, 2], loc[:, 1], loc[:, 0]] == v), d


@pytest.mark.parametrize("depth,full_depth", [(6, 6), (8, 3)])
def test_correct_pose_for_match(csm, oracle, depth, full_depth):
    """fast_correlative_scan_matcher_3d_test.cc:144-177, GPU vs oracle."""
    rng = np.random.default_rng(42)
    o = options(csm, depth, full_depth)
    for _ in range(10):
        x, y, z, th = rng.uniform(-1, 1, 4) * [0.7, 0.7, 0.7, 0.2]
        og, om, g, gm = fixture(csm, oracle, (x, y, z), quat_z(th), o)
        node = csm.NodeData3D(TEST_CLOUD, TEST_CLOUD, np.zeros(10, np.float32))
        ident = ((0, 0, 0), (1, 0, 0, 0))
        ref = om.match(ident, ident, node, 0.1)
        gpu = gm.Match(ident, ident, node, 0.1)
        assert_same_result(gpu, ref, om, False, ident, ident, node)
        if depth == 6:  # the reference test's own expectation (IsNearly 0.05)
            assert gpu is not None and gpu.score > 0.1 and gpu.low_resolution_score > 0.14
            assert np.allclose(gpu.pose_estimate[0], (x, y, z), atol=0.06)
        far = csm.NodeData3D(TEST_CLOUD, np.array([[42, 42, 42]], np.float32),
                             np.zeros(10, np.float32))
        assert gm.Match(ident, ident, far, 0.1) is None
        assert not om.match(ident, ident, far, 0.1)["matched"]


@pytest.mark.parametrize("depth,full_depth", [(6, 6), (8, 3)])
def test_correct_pose_for_match_full_submap(csm, oracle, depth, full_depth):
    """fast_correlative_scan_matcher_3d_test.cc:179-204, GPU vs oracle."""
    rng = np.random.default_rng(7)
    o = options(csm, depth, full_depth)
    for _ in range(3):
        x, y, z, th = rng.uniform(-1, 1, 4) * [0.7, 0.7, 0.7, 0.2]
        og, om, g, gm = fixture(csm, oracle, (x, y, z), quat_z(th), o)
        node = csm.NodeData3D(TEST_CLOUD, TEST_CLOUD, np.zeros(10, np.float32))
        ident = (1, 0, 0, 0)
        ref = om.match_full_submap(ident, ident, node, 0.1)
        gpu = gm.MatchFullSubmap(ident, ident, node, 0.1)
        assert_same_result(gpu, ref, om, True, ident, ident, node)
        far = csm.NodeData3D(TEST_CLOUD, np.array([[42, 42, 42]], np.float32),
                             np.zeros(10, np.float32))
        assert gm.MatchFullSubmap(ident, ident, far, 0.1) is None


def test_rotational_filter_and_poses(csm, oracle):
    """Non-zero histograms (ComputeHistogram of the clouds): the yaw filter,
    gravity alignment and non-identity global poses."""
    rng = np.random.default_rng(3)
    cloud = np.concatenate([TEST_CLOUD,
                            rng.uniform(-6, 6, (200, 3)).astype(np.float32) * [1, 1, 0.3]])
    cloud = cloud.astype(np.float32)
    o = options(csm, 7, 3, min_rotational_score=0.5, linear_xy_search_window=1.0,
                angular_search_window=0.4)
    og = oracle.hybrid_grid(0.05)
    og.insert((0.2, 0.1, 0.0), transform(cloud, (0.2, 0.1, 0.0), quat_z(0.15)), 0.7, 0.4, 5)
    hist_submap = oracle.histogram(transform(cloud, (0.2, 0.1, 0.0), quat_z(0.15)), 120)
    hist_node = oracle.histogram(cloud, 120)
    om = oracle.fast3d(og, og, hist_submap, opt_tuple(o))
    g = gpu_grid(csm, og)
    gm = csm.FastCorrelativeScanMatcher3D(g, g, hist_submap, o)
    grav = (math.cos(0.01), math.sin(0.01), 0.0, 0.0)
    node = csm.NodeData3D(cloud, cloud[::3], hist_node, grav)
    for node_pose, submap_pose in [(((0, 0, 0), (1, 0, 0, 0)), ((0, 0, 0), (1, 0, 0, 0))),
                                   (((0.1, 0.0, 0.05), quat_z(0.1)), ((-0.1, 0.1, 0.0), quat_z(-0.05)))]:
        ref = om.match(node_pose, submap_pose, node, 0.3)
        gpu = gm.Match(node_pose, submap_pose, node, 0.3)
        assert ref["num_discrete_scans"] > 0
        assert_same_result(gpu, ref, om, False, node_pose, submap_pose, node)
    ref = om.match_full_submap(quat_z(0.05), (1, 0, 0, 0), node, 0.3)
    gpu = gm.MatchFullSubmap(quat_z(0.05), (1, 0, 0, 0), node, 0.3)
    assert_same_result(gpu, ref, om, True, quat_z(0.05), (1, 0, 0, 0), node)


def test_batch_equals_single_calls(csm, oracle):
    o = options(csm, 6, 6)
    mats, nodes, pairs, refs = [], [], [], []
    rng = np.random.default_rng(11)
    keep = []
    for s in range(3):
        x, y, z, th = rng.uniform(-1, 1, 4) * [0.7, 0.7, 0.7, 0.2]
        og, om, g, gm = fixture(csm, oracle, (x, y, z), quat_z(th), o)
        keep.append((og, om, g))
        mats.append(gm)
    nodes = [csm.NodeData3D(TEST_CLOUD, TEST_CLOUD, np.zeros(10, np.float32)),
             csm.NodeData3D(TEST_CLOUD[:8], TEST_CLOUD[:8], np.zeros(10, np.float32))]
    ident = ((0, 0, 0), (1, 0, 0, 0))
    for s in range(3):
        for n in range(2):
            pairs.append((s, n, n == 1, 0.1, ident, ident))
    results = csm.match_batch_3d(mats, nodes, pairs)
    assert_search_ok(csm, [r.status for r in results])
    for (s, n, full, ms, npose, spose), r in zip(pairs, results):
        single = (mats[s].MatchFullSubmap((1, 0, 0, 0), (1, 0, 0, 0), nodes[n], ms) if full
                  else mats[s].Match(npose, spose, nodes[n], ms))
        assert (single is not None) == (r.status == csm.CSM_OK)
        if single is not None:
            assert np.float32(single.score) == np.float32(r.score)
            assert single.pose_estimate == r.pose.as_tuple()


# ------------------------------------------------------------------ RTCSM3D --
RT_CLOUD = np.array([[-3, 2, 0], [-4, 2, 0], [-5, 2, 0], [-6, 2, 0], [-6, 3, 1], [-6, 4, 2],
                     [-7, 3, 1]], np.float32)


# Every RTCSM3D kernel the host can select (host3d.cc RunRt3d): v5 (column
# gathers, the default for 3-, 5- and 7-step z columns), v4 (rotation lanes,
# other windows), v3 / v2 (bricks too large for v4's / v3's float byte
# offsets) and v1 (bricks past v2's 2^29 cells). The variables force the
# fallbacks on small inputs; the last two tests reach v4 and v2 unforced.
RT3D_KERNELS = {"v5": None, "v4": "CSM_RT3D_V4", "v3": "CSM_RT3D_V3", "v2": "CSM_RT3D_V2",
                "v1": "CSM_RT3D_V1"}


@pytest.fixture(params=list(RT3D_KERNELS))
def rt3d_kernel(request, monkeypatch):
    for var in RT3D_KERNELS.values():
        if var:
            monkeypatch.delenv(var, raising=False)
    if RT3D_KERNELS[request.param]:
        monkeypatch.setenv(RT3D_KERNELS[request.param], "1")
    return request.param


@pytest.mark.parametrize("initial", [
    ((-1.0, 0.0, 0.0), (1, 0, 0, 0)),        # PerfectEstimate
    ((-0.8, 0.0, 0.0), (1, 0, 0, 0)),        # AlongX
    ((-1.0, 0.0, -0.2), (1, 0, 0, 0)),       # AlongZ
    ((-0.9, -0.2, 0.2), (1, 0, 0, 0)),       # AlongXYZ
    ((-1.0, 0.0, 0.0), (math.cos(0.4 / 180 * math.pi), math.sin(0.4 / 180 * math.pi), 0, 0)),
    ((-1.0, 0.0, 0.0), (math.cos(0.4 / 180 * math.pi), 0, math.sin(0.4 / 180 * math.pi), 0)),
    ((-1.0, 0.0, 0.0), (math.cos(0.4 / 180 * math.pi), 0, math.sin(0.4 / 180 * math.pi),
                        math.sin(0.4 / 180 * math.pi))),  # unnormalized axis (0, 1, 1)
])
def test_rt3d_reference_cases(csm, oracle, initial, rt3d_kernel):
    """real_time_correlative_scan_matcher_3d_test.cc:34-117 on the GPU."""
    og = oracle.hybrid_grid(0.1)
    for p in RT_CLOUD:
        c = np.rint((p + [-1, 0, 0]) / np.float32(0.1)).astype(int)
        og.set_probability(int(c[0]), int(c[1]), int(c[2]), 1.0)
    opts = (0.3, math.radians(1.0), 0.1, 1.0)
    g = gpu_grid(csm, og)
    m = csm.RealTimeCorrelativeScanMatcher3D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    score, pose = m.Match(initial, RT_CLOUD, g)
    ref_score, ref_pose, _, _ = oracle.rt3d_match(og, opts, initial, RT_CLOUD)
    assert math.isclose(score, ref_score, rel_tol=1e-6), (score, ref_score)
    assert pose == ref_pose
    assert np.allclose(pose[0], (-1, 0, 0), atol=1e-3)


def test_rt3d_dense_scene(csm, oracle, rt3d_kernel):
    """A few hundred points, a 0.1 m grid built by the 3D inserter, and a
    +-0.2 m / +-2 deg window: many candidates, every one scored in float in
    the reference order."""
    rng = np.random.default_rng(5)
    cloud = rng.uniform(-4, 4, (300, 3)).astype(np.float32) * np.float32([1, 1, 0.4])
    og = oracle.hybrid_grid(0.1)
    og.insert((0, 0, 0), cloud, 0.7, 0.4, 5)
    opts = (0.2, math.radians(2.0), 0.1, 0.1)
    g = gpu_grid(csm, og)
    m = csm.RealTimeCorrelativeScanMatcher3D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    for initial in [((0.05, -0.03, 0.02), quat_z(0.01)), ((0.0, 0.0, 0.0), (1, 0, 0, 0))]:
        score, pose = m.Match(initial, cloud, g)
        ref_score, ref_pose, idx, n = oracle.rt3d_match(og, opts, initial, cloud)
        assert math.isclose(score, ref_score, rel_tol=1e-6), (score, ref_score)
        assert pose == ref_pose


@pytest.mark.parametrize("window", [0.1, 0.2, 0.3])
def test_rt3d_column_kernel_tilted_initial(csm, oracle, window, rt3d_kernel):
    """The column-gather kernel (rt3d_score5, 3-, 5- and 7-step z columns)
    under an initial pose with roll and pitch: the translation lattice's z
    columns drift in x and y, so many lookups fail the column test and take
    the per-step exact path. Same score and pose as the oracle."""
    rng = np.random.default_rng(11)
    cloud = rng.uniform(-4, 4, (400, 3)).astype(np.float32) * np.float32([1, 1, 0.4])
    og = oracle.hybrid_grid(0.1)
    og.insert((0, 0, 0), cloud, 0.7, 0.4, 5)
    opts = (window, math.radians(1.5), 0.1, 0.1)
    g = gpu_grid(csm, og)
    m = csm.RealTimeCorrelativeScanMatcher3D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    roll, pitch = math.radians(8.0), math.radians(-5.0)
    q = (math.cos(roll / 2) * math.cos(pitch / 2), math.sin(roll / 2) * math.cos(pitch / 2),
         math.cos(roll / 2) * math.sin(pitch / 2), -math.sin(roll / 2) * math.sin(pitch / 2))
    for initial in [((0.04, -0.02, 0.03), q), ((0.0, 0.0, 0.0), quat_z(0.2))]:
        score, pose = m.Match(initial, cloud, g)
        ref_score, ref_pose, idx, n = oracle.rt3d_match(og, opts, initial, cloud)
        assert math.isclose(score, ref_score, rel_tol=1e-6), (score, ref_score)
        assert pose == ref_pose


@pytest.mark.parametrize("steps", [9, 11, 13])
def test_rt3d_wide_z_windows(csm, oracle, rt3d_kernel, steps):
    """+-0.4 / 0.5 / 0.6 m at 0.1 m: 9-, 11- and 13-step z columns, which v5
    takes with three or four 16-byte loads per column (rt3d_score5<9..13>),
    under a tilted and a yawed initial pose (real_time_correlative_scan_
    matcher_3d.cc:55-113 generates the same lattice)."""
    rng = np.random.default_rng(19)
    cloud = rng.uniform(-4, 4, (300, 3)).astype(np.float32) * np.float32([1, 1, 0.4])
    og = oracle.hybrid_grid(0.1)
    og.insert((0, 0, 0), cloud, 0.7, 0.4, 5)
    opts = (round((steps // 2) * 0.1, 10), math.radians(1.0), 0.1, 0.1)
    g = gpu_grid(csm, og)
    m = csm.RealTimeCorrelativeScanMatcher3D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    nt, _ = m.window(cloud, 0.1)
    assert nt == steps ** 3
    roll = math.radians(6.0)
    for initial in [((0.05, -0.03, 0.02), (math.cos(roll / 2), math.sin(roll / 2), 0.0, 0.0)),
                    ((0.0, 0.0, 0.0), quat_z(0.1))]:
        score, pose = m.Match(initial, cloud, g)
        ref_score, ref_pose, _, _ = oracle.rt3d_match(og, opts, initial, cloud)
        assert math.isclose(score, ref_score, rel_tol=1e-6), (score, ref_score)
        assert pose == ref_pose


@pytest.mark.parametrize("kernel", ["v2", "v1"])
def test_rt3d_large_brick(csm, oracle, kernel, monkeypatch):
    """A HybridGrid whose known cells span 30 x 30 x 6 m at 0.1 m (5.5e6
    voxels, a 22 MB float brick): past v4's and v3's 2^24-byte float offsets,
    so the host selects v2 unforced (and v1 when forced)."""
    for var in RT3D_KERNELS.values():
        if var:
            monkeypatch.delenv(var, raising=False)
    if kernel == "v1":
        monkeypatch.setenv("CSM_RT3D_V1", "1")
    rng = np.random.default_rng(29)
    cloud = rng.uniform(-4, 4, (250, 3)).astype(np.float32) * np.float32([1, 1, 0.4])
    og = oracle.hybrid_grid(0.1)
    og.insert((0, 0, 0), cloud, 0.7, 0.4, 5)
    og.set_probability(-150, -150, -30, 0.6)
    og.set_probability(150, 150, 30, 0.6)
    g = gpu_grid(csm, og)
    opts = (0.2, math.radians(1.0), 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher3D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    for initial in [((0.04, -0.02, 0.03), quat_z(0.02)), ((0.0, 0.0, 0.0), (1, 0, 0, 0))]:
        score, pose = m.Match(initial, cloud, g)
        ref_score, ref_pose, _, _ = oracle.rt3d_match(og, opts, initial, cloud)
        assert math.isclose(score, ref_score, rel_tol=1e-6), (score, ref_score)
        assert pose == ref_pose


# ------------------------------------------------- synthetic world (C5 shape) --
@pytest.fixture(scope="module")
def world3d(csm):
    return csm.SyntheticWorld3D(num_nodes=24, num_submaps=3, seed=99)


def test_synthetic_pairs_match_oracle(csm, oracle, world3d):
    """C5-shaped inputs: 0.10 m high / 0.45 m low resolution grids built from
    64-ring scans, ~200-point node clouds, 120-bucket histograms, the
    pose_graph.lua 3D options; MatchFullSubmap and Match on the same pairs."""
    w = world3d
    o = csm.FastCorrelativeScanMatcherOptions3D()  # pose_graph.lua:40-48
    stats = {"exact": 0, "tie": 0, "nomatch": 0}
    for s in range(w.num_submaps):
        oh, ol = oracle.hybrid_grid(w.high_resolution), oracle.hybrid_grid(w.low_resolution)
        oh.set_values(*w.high_cells[s])
        ol.set_values(*w.low_cells[s])
        om = oracle.fast3d(oh, ol, w.submap_hist[s], opt_tuple(o))
        gh = csm.HybridGrid(w.high_resolution, *w.high_cells[s])
        gl = csm.HybridGrid(w.low_resolution, *w.low_cells[s])
        assert gh.info()[2] == oh.grid_size
        gm = csm.FastCorrelativeScanMatcher3D(gh, gl, w.submap_hist[s], o)
        c = int(w.submap_nodes[s])
        for n in [c, (c + 1) % w.num_nodes, (c + 7) % w.num_nodes]:
            node = w.node(n)
            ref = om.match_full_submap(w.node_rotation(n), (1, 0, 0, 0), node, 0.6)
            gpu = gm.MatchFullSubmap(w.node_rotation(n), (1, 0, 0, 0), node, 0.6)
            stats[assert_same_result(gpu, ref, om, True, w.node_rotation(n), (1, 0, 0, 0), node,
                                     o.min_low_resolution_score)] += 1
            truth = w.node_in_submap(n, s)
            init = ((truth[0][0] + 0.3, truth[0][1] - 0.2, 0.1), truth[1])
            ref = om.match(init, ((0, 0, 0), (1, 0, 0, 0)), node, 0.55)
            gpu = gm.Match(init, ((0, 0, 0), (1, 0, 0, 0)), node, 0.55)
            stats[assert_same_result(gpu, ref, om, False, init, ((0, 0, 0), (1, 0, 0, 0)), node,
                                     o.min_low_resolution_score)] += 1
    assert stats["exact"] + stats["tie"] >= 3, stats


def test_grid_create_batch_equals_single_creates(csm, world3d):
    """csm_hybrid_grid_create_batch (one upload and one launch per build step
    for all grids) makes what csm_hybrid_grid_create makes grid by grid: the
    same brick boxes and grid sizes, the same probabilities at every known
    cell and at unknown ones, the same interpolation, and matchers built on
    the batch grids search exactly like matchers on single-created grids. An
    empty grid inside the batch stays empty."""
    w = world3d
    S = w.num_submaps
    single = [(csm.HybridGrid(w.high_resolution, *w.high_cells[s]),
               csm.HybridGrid(w.low_resolution, *w.low_cells[s])) for s in range(S)]
    empty = (np.zeros((0, 3), np.int32), np.zeros(0, np.uint16))
    hi = csm.HybridGrid.create_batch(w.high_resolution, [w.high_cells[s] for s in range(S)] + [empty])
    lo = csm.HybridGrid.create_batch([w.low_resolution] * S, [w.low_cells[s] for s in range(S)])
    assert hi[-1].info()[1] == (0, 0, 0)
    rng = np.random.default_rng(7)
    for s in range(S):
        for b, g, cells in ((hi[s], single[s][0], w.high_cells[s]), (lo[s], single[s][1], w.low_cells[s])):
            assert b.info() == g.info(), s
            ijk = np.asarray(cells[0], np.int32).reshape(-1, 3)
            probe = np.concatenate([ijk, ijk[rng.integers(0, len(ijk), 500)] + rng.integers(-3, 4, (500, 3))])
            assert np.array_equal(b.get_probability(probe), g.get_probability(probe)), s
            pts = (ijk[rng.integers(0, len(ijk), 200)] + rng.random((200, 3)) - 0.5) * b.resolution
            assert np.array_equal(b.interpolate(pts), g.interpolate(pts)), s
    o = csm.FastCorrelativeScanMatcherOptions3D()
    mb = csm.FastCorrelativeScanMatcher3D.create_batch(list(zip(hi[:S], lo)), list(w.submap_hist[:S]), o)
    ms = csm.FastCorrelativeScanMatcher3D.create_batch(single, list(w.submap_hist[:S]), o)
    for s in range(S):
        for lvl in range(o.branch_and_bound_depth):
            ob, vb = mb[s].read_level(lvl)
            os_, vs = ms[s].read_level(lvl)
            assert ob == os_ and np.array_equal(vb, vs), (s, lvl)
    nodes = csm.NodeSet3D([w.node(i) for i in range(w.num_nodes)])
    sub = np.repeat(np.arange(S), w.num_nodes)
    nod = np.tile(np.arange(w.num_nodes), S)
    rot = np.array([w.node_rotation(n) for n in range(w.num_nodes)])
    pairs = csm.make_pairs_3d(sub, nod, 0.6, True, node_q=rot[nod])
    rb = csm.match_batch_3d(mb, nodes, pairs)
    rs = csm.match_batch_3d(ms, nodes, pairs)
    assert (rb["status"] == rs["status"]).all()
    ok = rb["status"] == csm.CSM_OK
    assert ok.sum() >= 3
    for f in ("score", "rotational_score", "low_resolution_score", "t", "q"):
        assert np.array_equal(rb[f][ok], rs[f][ok]), f
    for m in mb + ms:
        m.close()
    for g in hi + lo + [x for pair in single for x in pair]:
        g.close()


def test_create_batch_equals_single_creates(csm, oracle, world3d):
    """csm_fast3d_create_batch builds every level of every matcher in one
    launch per level: the levels are byte-identical to the oracle's
    (PrecomputationGridStack3D) and to single creates', and a batch search
    over the batch-built matchers returns what the single-built ones do."""
    w = world3d
    o = csm.FastCorrelativeScanMatcherOptions3D()
    grids = [(csm.HybridGrid(w.high_resolution, *w.high_cells[s]),
              csm.HybridGrid(w.low_resolution, *w.low_cells[s])) for s in range(w.num_submaps)]
    batch = csm.FastCorrelativeScanMatcher3D.create_batch(grids, list(w.submap_hist[:w.num_submaps]), o)
    single = [csm.FastCorrelativeScanMatcher3D(g[0], g[1], w.submap_hist[s], o)
              for s, g in enumerate(grids)]
    for s in range(w.num_submaps):
        oh, ol = oracle.hybrid_grid(w.high_resolution), oracle.hybrid_grid(w.low_resolution)
        oh.set_values(*w.high_cells[s])
        ol.set_values(*w.low_cells[s])
        om = oracle.fast3d(oh, ol, w.submap_hist[s], opt_tuple(o))
        for lvl in range(o.branch_and_bound_depth):
            ob, vb = batch[s].read_level(lvl)
            os_, vs = single[s].read_level(lvl)
            assert ob == os_ and np.array_equal(vb, vs), (s, lvl)
            ijk, v = om.level(lvl)
            assert np.count_nonzero(vb) == np.count_nonzero(v), (s, lvl)
            loc = ijk - np.asarray(ob)
            assert np.all(vb[loc[:, 2], loc[:, 1], loc[:, 0]] == v), (s, lvl)
    nodes = csm.NodeSet3D([w.node(i) for i in range(w.num_nodes)])
    sub = np.repeat(np.arange(w.num_submaps), w.num_nodes)
    nod = np.tile(np.arange(w.num_nodes), w.num_submaps)
    rot = np.array([w.node_rotation(n) for n in range(w.num_nodes)])
    pairs = csm.make_pairs_3d(sub, nod, 0.6, True, node_q=rot[nod])
    rb = csm.match_batch_3d(batch, nodes, pairs)
    rs = csm.match_batch_3d(single, nodes, pairs)
    assert (rb["status"] == rs["status"]).all()
    ok = rb["status"] == csm.CSM_OK
    assert ok.sum() >= 3
    for f in ("score", "rotational_score", "low_resolution_score", "t", "q"):
        assert np.array_equal(rb[f][ok], rs[f][ok]), f
    for m in batch + single:
        m.close()


def test_large_clouds_match_oracle(csm, oracle, world3d):
    """Clouds past the small build's LDS capacity (2048 points) take the
    large-cloud build (up to 8192); a batch mixing both is split over the
    two launches and results come back in pair order. Past 8192: CSM_ERANGE."""
    w = world3d
    o = csm.FastCorrelativeScanMatcherOptions3D()
    s = 0
    oh, ol = oracle.hybrid_grid(w.high_resolution), oracle.hybrid_grid(w.low_resolution)
    oh.set_values(*w.high_cells[s])
    ol.set_values(*w.low_cells[s])
    om = oracle.fast3d(oh, ol, w.submap_hist[s], opt_tuple(o))
    gm = csm.FastCorrelativeScanMatcher3D(csm.HybridGrid(w.high_resolution, *w.high_cells[s]),
                                          csm.HybridGrid(w.low_resolution, *w.low_cells[s]),
                                          w.submap_hist[s], o)
    c = int(w.submap_nodes[s])
    small = w.node(c)
    rng = np.random.default_rng(5)
    pts = small.high_resolution_point_cloud
    reps = 2100 // len(pts) + 1
    big_cloud = np.concatenate([pts + rng.uniform(-0.03, 0.03, pts.shape).astype(np.float32)
                                for _ in range(reps)]).astype(np.float32)
    assert 2048 < len(big_cloud) <= 8192
    big = csm.NodeData3D(big_cloud, small.low_resolution_point_cloud,
                         small.rotational_scan_matcher_histogram, small.gravity_alignment)
    rot = w.node_rotation(c)
    ref = om.match_full_submap(rot, (1, 0, 0, 0), big, 0.55)
    gpu = gm.MatchFullSubmap(rot, (1, 0, 0, 0), big, 0.55)
    assert assert_same_result(gpu, ref, om, True, rot, (1, 0, 0, 0), big,
                              o.min_low_resolution_score) in ("exact", "tie")
    truth = w.node_in_submap(c, s)
    init = ((truth[0][0] + 0.3, truth[0][1] - 0.2, 0.1), truth[1])
    ident = ((0, 0, 0), (1, 0, 0, 0))
    ref = om.match(init, ident, big, 0.55)
    gpu = gm.Match(init, ident, big, 0.55)
    assert_same_result(gpu, ref, om, False, init, ident, big, o.min_low_resolution_score)
    # Mixed batch, large first in input order.
    huge = csm.NodeData3D(np.tile(big_cloud, (4, 1)), small.low_resolution_point_cloud,
                          small.rotational_scan_matcher_histogram, small.gravity_alignment)
    pairs = [(0, 1, False, 0.55, init, ident), (0, 0, False, 0.55, init, ident),
             (0, 1, True, 0.55, ((0, 0, 0), rot), ident),
             (0, 2, False, 0.55, init, ident)]
    res = csm.match_batch_3d([gm], [small, big, huge], pairs)
    for (sub, n, full, ms, npose, spose), r in zip(pairs[:3], res[:3]):
        node = [small, big][n]
        single = (gm.MatchFullSubmap(npose[1], spose[1], node, ms) if full
                  else gm.Match(npose, spose, node, ms))
        assert (single is not None) == (r.status == csm.CSM_OK)
        if single is not None:
            assert np.float32(single.score) == np.float32(r.score)
            assert single.pose_estimate == r.pose.as_tuple()
    assert res[3].status == csm.CSM_ERANGE


def test_search_tiers_match_oracle(csm, oracle, world3d):
    """One batch over the three search builds (Search3dTier: <= 512 points,
    <= 2048, <= 8192; each its own launch over its item range) against the
    oracle and against single calls, clouds listed largest first."""
    w = world3d
    o = csm.FastCorrelativeScanMatcherOptions3D()
    s = 0
    oh, ol = oracle.hybrid_grid(w.high_resolution), oracle.hybrid_grid(w.low_resolution)
    oh.set_values(*w.high_cells[s])
    ol.set_values(*w.low_cells[s])
    om = oracle.fast3d(oh, ol, w.submap_hist[s], opt_tuple(o))
    gm = csm.FastCorrelativeScanMatcher3D(csm.HybridGrid(w.high_resolution, *w.high_cells[s]),
                                          csm.HybridGrid(w.low_resolution, *w.low_cells[s]),
                                          w.submap_hist[s], o)
    c = int(w.submap_nodes[s])
    small = w.node(c)
    pts = small.high_resolution_point_cloud
    assert len(pts) <= 512
    rng = np.random.default_rng(11)

    def grown(target):
        reps = target // len(pts) + 1
        cloud = np.concatenate([pts + rng.uniform(-0.03, 0.03, pts.shape).astype(np.float32)
                                for _ in range(reps)]).astype(np.float32)
        return csm.NodeData3D(cloud, small.low_resolution_point_cloud,
                              small.rotational_scan_matcher_histogram, small.gravity_alignment)

    mid, big = grown(900), grown(2300)
    assert 512 < len(mid.high_resolution_point_cloud) <= 2048
    assert 2048 < len(big.high_resolution_point_cloud) <= 8192
    nodes = [big, mid, small]
    rot = w.node_rotation(c)
    truth = w.node_in_submap(c, s)
    init = ((truth[0][0] + 0.3, truth[0][1] - 0.2, 0.1), truth[1])
    ident = ((0, 0, 0), (1, 0, 0, 0))
    pairs = [(0, n, full, 0.55, ((0, 0, 0), rot) if full else init, ident)
             for n in range(3) for full in (True, False)]
    res = csm.match_batch_3d([gm], nodes, pairs)
    matched = 0
    for (sub, n, full, ms, npose, spose), r in zip(pairs, res):
        node = nodes[n]
        if full:
            ref = om.match_full_submap(npose[1], spose[1], node, ms)
            single = gm.MatchFullSubmap(npose[1], spose[1], node, ms)
        else:
            ref = om.match(npose, spose, node, ms)
            single = gm.Match(npose, spose, node, ms)
        assert assert_same_result(single, ref, om, full, npose[1] if full else npose,
                                  spose[1] if full else spose, node,
                                  o.min_low_resolution_score) in ("exact", "tie", "nomatch")
        matched += single is not None
        assert (single is not None) == (r.status == csm.CSM_OK), (n, full)
        if single is not None:
            assert np.float32(single.score) == np.float32(r.score)
            assert single.pose_estimate == r.pose.as_tuple()
    assert matched >= 3


def _qmul(a, b):
    return (a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
            a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
            a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
            a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0])


def test_rt3d_c4_full_window(csm, oracle):
    """BASELINE config C4 at its full size: the bench's 64-ring scan (~55k
    points) against a 0.10 m HybridGrid, +-0.3 m / +-15 deg (343 translations x
    ~420k rotations, 1.45e8 candidates), yawed initial pose. The whole window
    is searched on the device; the oracle cannot score 1.45e8 candidates
    (~27 h), so parity is checked (1) on the winner: the oracle scores the
    winning candidate index to the same float (exp penalty: 1e-6 relative);
    (2) on 16 whole rotations scored by Match's kernel (the winner's, the two
    window corners and 13 seeded ones, 5488 candidates): every one of them
    equals the oracle's score on a 400-candidate sample including the full
    winner row, and none beats the winner."""
    w = csm.SyntheticWorld3D(num_nodes=2, num_submaps=1, world_x=20.0, world_y=20.0, world_z=5.0,
                             num_boxes=8, max_range=14.0, seed=20250127 + 3)
    c = int(w.submap_nodes[0])
    cloud = np.ascontiguousarray(w.raw[c], np.float32)
    grid = csm.HybridGrid(w.high_resolution, *w.high_cells[0])
    (tx, ty, tz), q = w.node_in_submap(c, 0)
    dyaw = math.radians(4.0)
    q0 = (q[0] * math.cos(dyaw / 2) - q[3] * math.sin(dyaw / 2), 0.0, 0.0,
          q[3] * math.cos(dyaw / 2) + q[0] * math.sin(dyaw / 2))
    init = ((tx + 0.12, ty - 0.08, tz + 0.05), q0)
    opts = (0.3, math.radians(15.0), 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher3D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    nt, nr = m.window(cloud, w.high_resolution)
    assert len(cloud) > 40000 and nt == 343 and nr > 100000
    score, pose = m.Match(init, cloud, grid)
    # Recover the winner's (t, r): translations are init * (x, y, z) * res,
    # rotations init.q * AngleAxis((rx, ry, rz) * step).
    og = oracle.hybrid_grid(w.high_resolution)
    og.set_values(*w.high_cells[0])
    import ctypes as C
    Lw, Aw, stepw = C.c_int(), C.c_int(), C.c_float()
    oo = np.asarray(opts, np.float64)
    oracle.lib.oracle_rt3d_window(oo.ctypes.data_as(C.POINTER(C.c_double)),
                                  float(w.high_resolution),
                                  cloud.ctypes.data_as(C.POINTER(C.c_float)), len(cloud),
                                  C.byref(Lw), C.byref(stepw), C.byref(Aw))
    L, A, step = Lw.value, Aw.value, float(stepw.value)
    nl, na = 2 * L + 1, 2 * A + 1
    assert nl ** 3 == nt and na ** 3 == nr
    qi = tuple(float(v) for v in init[1])
    nq = math.sqrt(sum(v * v for v in qi))
    qi = tuple(v / nq for v in qi)
    qinv = (qi[0], -qi[1], -qi[2], -qi[3])
    d = np.asarray(pose[0]) - np.asarray(init[0])
    v = _qmul(_qmul(qinv, (0.0,) + tuple(d)), qi)[1:]
    x, y, z = (int(round(c_ / w.high_resolution)) for c_ in v)
    t = ((z + L) * nl + (y + L)) * nl + (x + L)
    qs = _qmul(qinv, pose[1])
    s_ = math.sqrt(sum(c_ * c_ for c_ in qs[1:]))
    ang = 2 * math.atan2(s_, qs[0])
    axis = [c_ / s_ for c_ in qs[1:]] if s_ > 0 else [0.0, 0.0, 0.0]
    rx, ry, rz = (int(round(a_ * ang / step)) for a_ in axis)
    r = ((rz + A) * na + (ry + A)) * na + (rx + A)
    win_index = t * nr + r
    ref_score, ref_pose = oracle.rt3d_score(og, opts, init, cloud, win_index)
    assert np.allclose(ref_pose[0], pose[0], atol=1e-6) and np.allclose(ref_pose[1], pose[1],
                                                                        atol=1e-6)
    assert math.isclose(score, ref_score, rel_tol=1e-6), (score, ref_score)
    rng = np.random.RandomState(17)
    rots = [r, 0, nr - 1] + [int(v) for v in rng.randint(0, nr, 13)]
    scores = m.score_rotations(init, cloud, grid, rots)
    assert scores.shape == (16, nt)
    assert scores[0, t] == np.float32(score)
    # Nothing in the subset beats the winner (ties: the smaller index wins).
    for k, rr in enumerate(rots):
        for tt in np.nonzero(scores[k] >= np.float32(score))[0]:
            assert scores[k, tt] == np.float32(score) and int(tt) * nr + rr >= win_index
    sample = [(0, tt) for tt in range(nt)] + [(int(k), int(tt)) for k, tt in
                                              zip(rng.randint(1, 16, 57), rng.randint(0, nt, 57))]
    exact = 0
    for k, tt in sample:
        ref, _ = oracle.rt3d_score(og, opts, init, cloud, tt * nr + rots[k])
        assert math.isclose(float(scores[k, tt]), ref, rel_tol=1e-6), (k, tt, scores[k, tt], ref)
        exact += float(scores[k, tt]) == ref
    assert exact >= 0.95 * len(sample)


# ----------------------------------------------------------- exact ties ------
def _tied_world(oracle, csm, shifts, depth):
    """A sparse pattern of voxels copied at each shift (cells never collide):
    the pattern's own points then reach the same sum at every copy, an exact
    tie between leaves that all pass the low-resolution check."""
    rng = np.random.RandomState(3)
    base = np.unique(rng.randint(-4, 4, (40, 3)) * 3, axis=0)
    vals = rng.randint(20000, 32768, len(base)).astype(np.uint16)
    ijk = np.concatenate([base + np.array(s) for s in shifts])
    og = oracle.hybrid_grid(0.05)
    og.set_values(ijk, np.concatenate([vals] * len(shifts)))
    o = options(csm, depth, 3)
    hist = np.zeros(10, np.float32)
    om = oracle.fast3d(og, og, hist, opt_tuple(o))
    g = gpu_grid(csm, og)
    gm = csm.FastCorrelativeScanMatcher3D(g, g, hist, o)
    cloud = (base * 0.05).astype(np.float32)
    return om, gm, g, csm.NodeData3D(cloud, cloud, hist)


TIE_SHIFTS = [[(1, 0, 0), (0, 0, 1)], [(1, 1, 0), (0, 0, 1)], [(-9, 0, 0), (9, 0, 0)],
              [(-7, 2, 1), (7, -2, -1)], [(2, 0, 0), (0, 0, 1)], [(0, 1, 0), (0, 0, 1)],
              [(-1, 0, 1), (1, 0, 0)], [(0, 0, 0), (3, 0, 0), (0, 0, 3)]]


@pytest.mark.parametrize("depth", [4, 6])
def test_exact_ties_take_the_reference_pick(csm, oracle, depth):
    """Leaves that tie at the maximum and all pass the low-resolution check:
    the reference returns the first one its DFS reaches (sorted children,
    generation order z, y, x among equal scores, the lowest-resolution list in
    std::sort's order), which is often not the smallest (yaw, x, y, z) key
    (e.g. (1, 0, 0) before (0, 0, 1) under one parent; +9 before -9 when the
    two top-level candidates tie at depth 6). The GPU must return exactly the
    oracle's pose, through Match and MatchFullSubmap, and report the tie."""
    ident = ((0, 0, 0), (1, 0, 0, 0))
    ties = 0
    for shifts in TIE_SHIFTS:
        om, gm, g, node = _tied_world(oracle, csm, shifts, depth)
        for init in [(0.0, 0.0, 0.0), (0.01, -0.02, 0.0)]:
            ref = om.match((init, (1, 0, 0, 0)), ident, node, 0.1)
            gpu = gm.Match((init, (1, 0, 0, 0)), ident, node, 0.1)
            ties += assert_same_result(gpu, ref) == "tie"
        ref = om.match_full_submap((1, 0, 0, 0), (1, 0, 0, 0), node, 0.1)
        gpu = gm.MatchFullSubmap((1, 0, 0, 0), (1, 0, 0, 0), node, 0.1)
        ties += assert_same_result(gpu, ref) == "tie"
    assert ties >= len(TIE_SHIFTS), ties


def test_exact_ties_in_batches(csm, oracle):
    """The same tied pairs inside one batch next to untied ones (the collect
    search and the score queries index pairs and yaws of a whole batch)."""
    ident = ((0, 0, 0), (1, 0, 0, 0))
    mats, nodes, refs, keep = [], [], [], []
    for shifts in TIE_SHIFTS[:4]:
        om, gm, g, node = _tied_world(oracle, csm, shifts, 6)
        keep.append((g, om))
        mats.append(gm)
        nodes.append(node)
    pairs = []
    for s in range(len(mats)):
        for n in range(len(nodes)):
            pairs.append((s, n, False, 0.1, ((0.0, 0.0, 0.0), (1, 0, 0, 0)), ident))
            refs.append(keep[s][1].match(((0.0, 0.0, 0.0), (1, 0, 0, 0)), ident, nodes[n], 0.1))
    res = csm.match_batch_3d(mats, nodes, pairs)
    assert_search_ok(csm, [r.status for r in res])
    tied = 0
    for (s, n, *_), r, ref in zip(pairs, res, refs):
        gpu = None if r.status != csm.CSM_OK else type("R", (), {
            "score": r.score, "pose_estimate": r.pose.as_tuple(), "rotational_score": r.rotational_score,
            "low_resolution_score": r.low_resolution_score, "tie": r.tie})()
        tied += assert_same_result(gpu, ref) == "tie"
    assert tied >= 4
