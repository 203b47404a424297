"""CeresScanMatcher2D refinement (ceres_scan_matcher_2d.cc:64-105, called by
ConstraintBuilder2D::ComputeConstraint at constraint_builder_2d.cc:245-249).

Ceres is absent from this image, so the oracle (oracle/ceres2d.cc) restates
the cost (OccupiedSpaceCostFunction2D with ceres::BiCubicInterpolator, the
translation and rotation delta functors) and Ceres 1.13's trust-region LM
(the version scripts/install_ceres.sh pins), non-monotonic steps included.
The restatement is pinned by the reference's own ceres_scan_matcher_2d_test.cc
and occupied_space_cost_function_2d_test.cc (oracle/ref_tests.cc, and the
four cases again below through the device path) to those tests' tolerances.
The HIP batch path must agree with the restatement to 1e-6 m / 1e-6 rad
(double arithmetic, different summation order and libm)."""
import math

import numpy as np
import pytest

OPTS = (20.0, 10.0, 1.0, 10)  # pose_graph.lua:30-39


# ceres_scan_matcher_2d_test.cc:35-96: MapLimits(1, (10, 10), 20 x 20), the
# cell of (-3.5, 2.5) at kMaxProbability (correspondence-cost value 1), one
# point at (-3, 2); options occupied 1, translation 0.1, rotation 1.5, 50
# iterations, non-monotonic steps. Expected Translation(-0.5, 0.5).
REF_OPTS = (1.0, 0.1, 1.5, 50, True)
REF_STARTS = [(-0.5, 0.5), (-0.3, 0.5), (-0.45, 0.3), (-0.3, 0.3)]


def _ref_grid(csm):
    cells = np.zeros((20, 20), np.uint16)  # unknown: kMaxCorrespondenceCost
    cells[13, 7] = 1  # GetCellIndex(-3.5, 2.5) = (x 7, y 13); cost 0.1 -> value 1
    return csm.ProbabilityGrid(1.0, 10.0, 10.0, cells)


def is_nearly_2d(a, b, eps):
    """transform::IsNearly (rigid_transform_test_helpers.h:42-46): Eigen
    isApprox of the 3x3 affine matrices."""
    def m(p):
        c, s = math.cos(p[2]), math.sin(p[2])
        return np.array([[c, -s, p[0]], [s, c, p[1]], [0.0, 0.0, 1.0]])
    ma, mb = m(a), m(b)
    return ((ma - mb) ** 2).sum() <= eps * eps * min((ma ** 2).sum(), (mb ** 2).sum())


def test_oracle_passes_reference_ceres_cases(csm, oracle):
    g = _ref_grid(csm)
    cloud = np.array([[-3.0, 2.0, 0.0]], np.float32)
    for st in REF_STARTS:
        pose, _ = oracle.ceres2d_match((1.0, 10.0, 10.0), g.cells, REF_OPTS[:4] + (1.0,), st,
                                       (st[0], st[1], 0.0), cloud)
        assert is_nearly_2d(pose, (-0.5, 0.5, 0.0), 1e-2), (st, pose)


@pytest.mark.gpu
def test_gpu_passes_reference_ceres_cases(csm, oracle):
    """The reference's four CeresScanMatcherTest cases through
    csm_ceres2d_refine_batch: the reference's expectation (IsNearly 1e-2) and
    the oracle's pose to 1e-6."""
    g = _ref_grid(csm)
    cloud = np.array([[-3.0, 2.0, 0.0]], np.float32)
    m = csm.FastCorrelativeScanMatcher2D(g, csm.FastCorrelativeScanMatcherOptions2D())
    scans = csm.ScanSet([cloud])
    n = len(REF_STARTS)
    init = [(x, y, 0.0) for x, y in REF_STARTS]
    poses, iters = csm.ceres_refine_batch([m], scans, [0] * n, [0] * n, init, REF_STARTS,
                                          csm.CeresOptions2D.make(*REF_OPTS))
    for k, st in enumerate(REF_STARTS):
        assert is_nearly_2d(poses[k], (-0.5, 0.5, 0.0), 1e-2), (st, poses[k])
        ref, ref_it = oracle.ceres2d_match((1.0, 10.0, 10.0), g.cells, REF_OPTS[:4] + (1.0,), st,
                                           init[k], cloud)
        assert np.allclose(poses[k], ref, atol=1e-6), (k, poses[k], ref)
        assert abs(int(iters[k]) - ref_it) <= 1


def _world(csm):
    return csm.SyntheticWorld2D(num_nodes=24, num_submaps=3, submap_cells=200, decimate_to=200,
                                seed=5)


def test_oracle_refinement_reduces_the_occupied_cost(csm, oracle):
    """The refined pose sits where the grid's cost is lower than at a
    perturbed start (a property Ceres' solution has as well)."""
    w = _world(csm)
    g = w.grid(0)
    lim = (g.resolution, g.max_x, g.max_y)
    n = int(w.submap_nodes[0])
    truth = tuple(float(v) for v in w.node_poses[n])
    cloud = w.cloud(n)
    start = (truth[0] + 0.04, truth[1] - 0.03, truth[2] + 0.02)
    pose, iters = oracle.ceres2d_match(lim, g.cells, OPTS, start[:2], start, cloud)
    assert 1 <= iters <= 10
    assert math.dist(pose[:2], truth[:2]) < math.dist(start[:2], truth[:2])
    # Zero iterations returns the start.
    pose0, it0 = oracle.ceres2d_match(lim, g.cells, OPTS[:3] + (0,), start[:2], start, cloud)
    assert it0 == 0 and pose0 == start


@pytest.mark.gpu
def test_gpu_refinement_matches_oracle(csm, oracle):
    w = _world(csm)
    fopts = csm.FastCorrelativeScanMatcherOptions2D()
    matchers = [csm.FastCorrelativeScanMatcher2D(w.grid(s), fopts) for s in range(w.num_submaps)]
    scans = csm.ScanSet([w.cloud(i) for i in range(w.num_nodes)])
    rng = np.random.default_rng(9)
    sub, scn, init, tgt = [], [], [], []
    for i in range(w.num_nodes):
        s = i % w.num_submaps
        t = w.node_poses[i]
        p = (t[0] + rng.normal(0, 0.05), t[1] + rng.normal(0, 0.05), t[2] + rng.normal(0, 0.03))
        sub.append(s)
        scn.append(i)
        init.append(p)
        tgt.append((p[0] + rng.normal(0, 0.01), p[1] + rng.normal(0, 0.01)))
    for opts in [OPTS, (5.0, 1.0, 0.5, 25), (20.0, 10.0, 1.0, 1), OPTS + (False,)]:
        poses, iters = csm.ceres_refine_batch(matchers, scans, sub, scn, init, tgt,
                                              csm.CeresOptions2D.make(*opts))
        for k in range(len(sub)):
            g = w.grid(sub[k])
            ref, ref_it = oracle.ceres2d_match((g.resolution, g.max_x, g.max_y), g.cells, opts,
                                               tgt[k], init[k], w.cloud(scn[k]))
            assert np.allclose(poses[k], ref, atol=1e-6), (k, poses[k], ref)
            assert iters[k] == ref_it or abs(iters[k] - ref_it) <= 1


@pytest.mark.gpu
def test_gpu_refinement_off_grid_and_rejects_bad_options(csm):
    """Points far outside the grid read kMaxCorrespondenceCost (flat cost):
    only the delta terms act, so the pose stays at the target. Non-positive
    weights are rejected like the reference's CHECK_GTs."""
    w = _world(csm)
    m = csm.FastCorrelativeScanMatcher2D(w.grid(0), csm.FastCorrelativeScanMatcherOptions2D())
    far = np.array([[500.0, 500.0, 0.0], [501.0, 499.0, 0.0]], np.float32)
    scans = csm.ScanSet([far])
    poses, _ = csm.ceres_refine_batch([m], scans, [0], [0], [(1.0, 2.0, 0.3)], [(1.0, 2.0)])
    assert np.allclose(poses[0], (1.0, 2.0, 0.3), atol=1e-9)
    with pytest.raises(csm.CsmError):
        csm.ceres_refine_batch([m], scans, [0], [0], [(1.0, 2.0, 0.3)],
                               options=csm.CeresOptions2D.make(0.0, 10.0, 1.0, 10))
