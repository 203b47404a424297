"""GPU parity: RealTimeCorrelativeScanMatcher2D::Match on the MI355X vs the oracle.

Every candidate score is a float sum taken in the reference's point order, so
the best score is expected bit-identical and the pose identical (first max in
(scan, x, y) order, real_time_correlative_scan_matcher_2d.cc:142-143). The
exp/hypot penalty is evaluated in double on the device (OCML) and on the host
(glibc); a last-ulp difference there could move a float score by one ulp, so
the score tolerance written here is 1e-6 relative, and the pose must match.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_reference_seven_point_grid(csm, oracle):
    """RealTimeCorrelativeScanMatcherTest probability-grid fixture (:72-96)."""
    cloud = np.array([[0.025, 0.175, 0], [-0.025, 0.175, 0], [-0.075, 0.175, 0],
                      [-0.125, 0.175, 0], [-0.125, 0.125, 0], [-0.125, 0.075, 0],
                      [-0.125, 0.025, 0]], np.float32)
    limits, cells = oracle.grid_from_inserts(0.05, 0.05, 0.25, 6, 6, [((0, 0, 0), cloud)])
    opts = (0.6, 0.16, 0.0, 0.0)
    m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    g = csm.ProbabilityGrid(*limits, cells)
    for init in [(0.0, 0.0, 0.0), (0.05, -0.05, 0.1), (-0.1, 0.02, -0.05)]:
        score, pose = m.Match(init, cloud, g)
        ref_score, ref_pose, _ = oracle.rt2d_match(limits, cells, opts, init, cloud)
        assert abs(score - ref_score) <= 1e-6 * abs(ref_score)
        assert pose == ref_pose


def test_c1_shaped_synthetic(csm, oracle):
    """BASELINE config C1: 1080-beam scan vs 200x200 @5cm, +-0.2 m / +-10 deg,
    translation/rotation weights 0.1."""
    world = csm.SyntheticWorld2D(num_nodes=6, num_submaps=6, submap_cells=200, seed=11)
    opts = (0.2, math.radians(10.0), 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    rng = np.random.RandomState(5)
    for s in range(6):
        g = world.grid(s)
        n = int(world.submap_nodes[s])
        t = world.node_poses[n]
        init = (t[0] + rng.uniform(-0.15, 0.15), t[1] + rng.uniform(-0.15, 0.15),
                t[2] + math.radians(rng.uniform(-8, 8)))
        cloud = world.cloud(n)
        score, pose = m.Match(init, cloud, g)
        ref_score, ref_pose, ncand = oracle.rt2d_match((g.resolution, g.max_x, g.max_y), g.cells,
                                                       opts, init, cloud)
        assert ncand > 1000
        assert abs(score - ref_score) <= 1e-6 * abs(ref_score)
        assert pose == ref_pose


# ---- TSDF2D grids (real_time_correlative_scan_matcher_2d.cc:38-59) ----------
SEVEN = np.array([[0.025, 0.175, 0], [-0.025, 0.175, 0], [-0.075, 0.175, 0],
                  [-0.125, 0.175, 0], [-0.125, 0.125, 0], [-0.125, 0.075, 0],
                  [-0.125, 0.025, 0]], np.float32)


def _seven_point_tsdf(oracle):
    """RealTimeCorrelativeScanMatcherTest TSDF fixture (:67-92): TSDF2D over
    MapLimits(0.05, (0.3, 0.5), 20x20), truncation 0.3, max weight 1.0, one
    insert from origin (0.5, -0.5) with the test's inserter options."""
    return oracle.tsdf_from_inserts(0.05, 0.3, 0.5, 20, 20, 0.3, 1.0, [((0.5, -0.5, 0), SEVEN)])


def test_reference_seven_point_tsdf(csm, oracle):
    limits, tsd, wgt = _seven_point_tsdf(oracle)
    g = csm.TSDF2D(*limits, tsd, wgt, 0.3, 1.0)
    for opts in [(0.6, 0.16, 0.0, 0.0), (0.6, 0.16, 0.1, 0.1)]:
        m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
        for init in [(0.0, 0.0, 0.0), (0.05, -0.05, 0.1), (-0.1, 0.02, -0.05)]:
            score, pose = m.Match(init, SEVEN, g)
            ref_score, ref_pose, _ = oracle.rt2d_match_tsdf(limits, tsd, wgt, 0.3, 1.0, opts,
                                                            init, SEVEN)
            assert abs(score - ref_score) <= 1e-6 * abs(ref_score)
            assert pose == ref_pose


def test_tsdf_cloud_off_the_grid(csm, oracle):
    """Every point reads (-truncation, 0) outside the limits: summed weight 0,
    every candidate scores 0 and the first candidate wins (max_element)."""
    limits, tsd, wgt = _seven_point_tsdf(oracle)
    g = csm.TSDF2D(*limits, tsd, wgt, 0.3, 1.0)
    opts = (0.2, 0.1, 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    init = (50.0, -40.0, 0.3)
    score, pose = m.Match(init, SEVEN, g)
    ref_score, ref_pose, _ = oracle.rt2d_match_tsdf(limits, tsd, wgt, 0.3, 1.0, opts, init, SEVEN)
    assert score == ref_score == 0.0
    assert pose == ref_pose


def test_tsdf_c1_shaped_synthetic(csm, oracle):
    """C1 shape on TSDF2D windows built by the restated inserter from the
    synthetic world's scans (trajectory_builder_2d.lua:100-112 options)."""
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_golden_tsdf as mg
    world = csm.SyntheticWorld2D(num_nodes=400, num_submaps=3, submap_cells=200, seed=23)
    opts = (0.2, math.radians(10.0), 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    rng = np.random.RandomState(9)
    checked = 0
    for s in range(3):
        inside = mg.nodes_inside(world, s)
        if not inside:
            continue
        limits, tsd, wgt = mg.build_tsdf(oracle, world, s, inside[:6])
        g = csm.TSDF2D(*limits, tsd, wgt, mg.TRUNCATION, mg.MAX_WEIGHT)
        for n in inside[:2]:
            t = world.node_poses[n]
            init = (t[0] + rng.uniform(-0.15, 0.15), t[1] + rng.uniform(-0.15, 0.15),
                    t[2] + math.radians(rng.uniform(-8, 8)))
            cloud = world.cloud(n)
            score, pose = m.Match(init, cloud, g)
            ref_score, ref_pose, ncand = oracle.rt2d_match_tsdf(
                limits, tsd, wgt, mg.TRUNCATION, mg.MAX_WEIGHT, opts, init, cloud)
            assert ncand > 1000
            assert abs(score - ref_score) <= 1e-6 * abs(ref_score)
            assert pose == ref_pose
            checked += 1
    assert checked >= 2


@pytest.mark.parametrize("lin,ang_deg", [(0.5, 10.0), (3.5, 2.0)])
def test_wide_windows(csm, oracle, lin, ang_deg):
    """Windows whose candidates' gathered values do not fit one LDS stage
    (+-0.5 m: 21 x offsets x 1080 points, staged in segments) or span several
    64-offset chunks (+-3.5 m: 141 x offsets)."""
    world = csm.SyntheticWorld2D(num_nodes=6, num_submaps=6, submap_cells=200, seed=13)
    opts = (lin, math.radians(ang_deg), 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    rng = np.random.RandomState(3)
    for s in range(2):
        g = world.grid(s)
        n = int(world.submap_nodes[s])
        t = world.node_poses[n]
        init = (t[0] + rng.uniform(-0.3, 0.3), t[1] + rng.uniform(-0.3, 0.3),
                t[2] + math.radians(rng.uniform(-1, 1)))
        cloud = world.cloud(n)
        score, pose = m.Match(init, cloud, g)
        ref_score, ref_pose, _ = oracle.rt2d_match((g.resolution, g.max_x, g.max_y), g.cells,
                                                   opts, init, cloud)
        assert abs(score - ref_score) <= 1e-6 * abs(ref_score)
        assert pose == ref_pose


def test_tsdf_wide_window(csm, oracle):
    """TSDF2D with a window past one LDS stage (+-0.6 m: 25 x offsets of
    8-byte terms) and a cloud past the staged point indices."""
    limits, tsd, wgt = _seven_point_tsdf(oracle)
    g = csm.TSDF2D(*limits, tsd, wgt, 0.3, 1.0)
    # 5005 points: the point indices are read from global memory (> 4096).
    cloud = np.repeat(SEVEN, 715, axis=0) + np.float32(1e-5) * np.arange(5005, dtype=np.float32)[:, None]
    cloud[:, 2] = 0
    opts = (0.6, 0.05, 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    init = (0.02, -0.03, 0.01)
    score, pose = m.Match(init, cloud, g)
    ref_score, ref_pose, _ = oracle.rt2d_match_tsdf(limits, tsd, wgt, 0.3, 1.0, opts, init, cloud)
    assert abs(score - ref_score) <= 1e-6 * abs(ref_score)
    assert pose == ref_pose
