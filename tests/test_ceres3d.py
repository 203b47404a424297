"""CeresScanMatcher3D refinement (ceres_scan_matcher_3d.cc:84-160, called by
ConstraintBuilder3D::ComputeConstraint at constraint_builder_3d.cc:264-275).

Ceres is absent from this image: the oracle (oracle/ceres3d.cc) restates the
cost (two OccupiedSpaceCostFunction3D blocks over InterpolatedGrid, the
translation and rotation delta functors), the quaternion parameterization and
Ceres 1.13's LM. Its analytic Jacobians are checked against finite
differences of the same cost, and the restatement is pinned by the reference's
rotation_delta_cost_functor_3d_test.cc and the upstream
ceres_scan_matcher_3d_test.cc (the fork's .bak copy; restated in
oracle/ref_tests_3d.cc without its intensity block, which ConstraintBuilder3D
never passes), whose five cases run below through the device path too. The
HIP path must agree with the restatement to 1e-6."""
import math

import numpy as np
import pytest

OPTS = (5.0, 30.0, 10.0, 1.0, 10)  # pose_graph.lua:49-60


@pytest.fixture(scope="module")
def world3(csm):
    return csm.SyntheticWorld3D(num_nodes=8, num_submaps=2, seed=11)


def _oracle_grids(oracle, w, s):
    hg = oracle.hybrid_grid(w.high_resolution)
    hg.set_values(*w.high_cells[s])
    lg = oracle.hybrid_grid(w.low_resolution)
    lg.set_values(*w.low_cells[s])
    return hg, lg


def test_oracle_refinement_runs_and_zero_iterations_is_identity(csm, oracle, world3):
    hg, lg = _oracle_grids(oracle, world3, 0)
    t, q = world3.node_in_submap(0, 0)
    start = (t[0] + 0.05, t[1] - 0.04, t[2] + 0.03)
    (tr, qr), it = oracle.ceres3d_match(hg, lg, world3.high[0], world3.low[0], OPTS, start, start, q)
    assert 1 <= it <= 10
    assert abs(math.sqrt(sum(v * v for v in qr)) - 1.0) < 1e-9  # the Plus keeps |q| = 1
    (t0, q0), it0 = oracle.ceres3d_match(hg, lg, world3.high[0], world3.low[0], OPTS[:4] + (0,),
                                         start, start, q)
    assert it0 == 0 and t0 == start and q0 == tuple(q)


@pytest.mark.gpu
def test_gpu_refinement_matches_oracle(csm, oracle, world3):
    grids, ogrids = [], []
    for s in range(world3.num_submaps):
        grids.append(csm.HybridGrid(world3.high_resolution, *world3.high_cells[s]))
        grids.append(csm.HybridGrid(world3.low_resolution, *world3.low_cells[s]))
        ogrids.append(_oracle_grids(oracle, world3, s))
    nodes = [world3.node(i) for i in range(world3.num_nodes)]
    rng = np.random.default_rng(4)
    items = []
    for i in range(world3.num_nodes):
        s = i % world3.num_submaps
        t, q = world3.node_in_submap(i, s)
        tt = tuple(float(v) for v in np.asarray(t) + rng.normal(0, 0.05, 3))
        yaw = rng.normal(0, 0.02)
        dq = (math.cos(yaw / 2), 0.0, 0.0, math.sin(yaw / 2))
        qq = (dq[0] * q[0] - dq[3] * q[3], 0.0, 0.0, dq[0] * q[3] + dq[3] * q[0])
        items.append((2 * s, 2 * s + 1, i, (tt, qq), tt))
    for opts in [OPTS, (5.0, 30.0, 10.0, 1.0, 1), (1.0, 2.0, 0.5, 0.3, 20), OPTS + (True,)]:
        poses, iters = csm.ceres_refine_batch_3d(grids, nodes, items, csm.CeresOptions3D.make(*opts))
        for k, (hgi, lgi, nd, (tt, qq), tgt) in enumerate(items):
            hg, lg = ogrids[hgi // 2]
            (rt, rq), rit = oracle.ceres3d_match(hg, lg, world3.high[nd], world3.low[nd], opts,
                                                 tgt, tt, qq)
            assert np.allclose(poses[k][0], rt, atol=1e-6), (k, poses[k], rt)
            assert np.allclose(poses[k][1], rq, atol=1e-6), (k, poses[k], rq)
            assert abs(int(iters[k]) - rit) <= 1


# ceres_scan_matcher_3d_test.cc.bak:34-136 (upstream CeresScanMatcher3DTest):
# seven points at probability 1 in a 1 m HybridGrid, shifted by the expected
# pose Translation(-1, 0, 0); occupied weight 1, translation 0.01, rotation
# 0.1, 10 iterations, non-monotonic steps; IsNearly(expected, 3e-2).
REF_POINTS = np.array([[-3, 2, 0], [-4, 2, 0], [-5, 2, 0], [-6, 2, 0], [-6, 3, 1], [-6, 4, 2],
                       [-7, 3, 1]], np.float32)


def _qmul(a, b):
    return (a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
            a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
            a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
            a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0])


def is_nearly_3d(t, q, te, qe, eps):
    """transform::IsNearly: Eigen isApprox of the 4x4 affine matrices."""
    def m(t, q):
        w, x, y, z = q
        r = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        out = np.eye(4)
        out[:3, :3], out[:3, 3] = r, t
        return out
    a, b = m(t, q), m(te, qe)
    return ((a - b) ** 2).sum() <= eps * eps * min((a ** 2).sum(), (b ** 2).sum())


def _ref_cases():
    """(cloud, initial (t, q), expected (t, q)) of the five reference cases."""
    ident = (1.0, 0.0, 0.0, 0.0)
    exp = ((-1.0, 0.0, 0.0), ident)
    cases = [(REF_POINTS, ((-1.0, 0.0, 0.0), ident), exp),
             (REF_POINTS, ((-0.8, 0.0, 0.0), ident), exp),
             (REF_POINTS, ((-1.0, 0.0, -0.2), ident), exp),
             (REF_POINTS, ((-0.9, -0.2, 0.2), ident), exp)]
    c, s = math.cos(0.05), math.sin(0.05)
    turned = np.stack([c * REF_POINTS[:, 0].astype(np.float64) - s * REF_POINTS[:, 1],
                       s * REF_POINTS[:, 0].astype(np.float64) + c * REF_POINTS[:, 1],
                       REF_POINTS[:, 2]], 1).astype(np.float32)
    qz = (math.cos(0.025), 0.0, 0.0, math.sin(0.025))
    qx = (math.cos(0.025), math.sin(0.025), 0.0, 0.0)
    cases.append((turned, ((-0.95, -0.05, 0.05), qx),
                  ((-1.0, 0.0, 0.0), (qz[0], -qz[1], -qz[2], -qz[3]))))
    return cases


def _ref_cells():
    return np.rint((REF_POINTS + np.array([-1.0, 0.0, 0.0], np.float32)) / 1.0).astype(np.int32)


# One (cloud, grid) block of weight 1 is the device's two-block form with the
# same grid and cloud in both blocks at weight 1/sqrt(2) each: the same cost
# and normal equations.
REF_OPTS3 = (math.sqrt(0.5), math.sqrt(0.5), 0.01, 0.1, 10, True)


def test_oracle_passes_reference_ceres3d_cases(oracle):
    g = oracle.hybrid_grid(1.0)
    g.set_values(_ref_cells(), np.full(len(REF_POINTS), 32767, np.uint16))
    for cloud, (t0, q0), (te, qe) in _ref_cases():
        (t, q), _ = oracle.ceres3d_match(g, g, cloud, cloud, REF_OPTS3, t0, t0, q0)
        assert is_nearly_3d(t, q, te, qe, 3e-2), (t0, t, q)


@pytest.mark.gpu
def test_gpu_passes_reference_ceres3d_cases(csm, oracle):
    g = csm.HybridGrid(1.0, _ref_cells(), np.full(len(REF_POINTS), 32767, np.uint16))
    og = oracle.hybrid_grid(1.0)
    og.set_values(_ref_cells(), np.full(len(REF_POINTS), 32767, np.uint16))
    cases = _ref_cases()
    nodes = [csm.NodeData3D(c, c, np.zeros(8, np.float32)) for c, _, _ in cases]
    items = [(0, 0, k, (t0, q0), t0) for k, (_, (t0, q0), _) in enumerate(cases)]
    poses, iters = csm.ceres_refine_batch_3d([g], nodes, items, csm.CeresOptions3D.make(*REF_OPTS3))
    for k, (cloud, (t0, q0), (te, qe)) in enumerate(cases):
        assert is_nearly_3d(poses[k][0], poses[k][1], te, qe, 3e-2), (k, poses[k])
        (rt, rq), rit = oracle.ceres3d_match(og, og, cloud, cloud, REF_OPTS3, t0, t0, q0)
        assert np.allclose(poses[k][0], rt, atol=1e-6), (k, poses[k], rt)
        assert np.allclose(poses[k][1], rq, atol=1e-6), (k, poses[k], rq)
        assert abs(int(iters[k]) - rit) <= 1


@pytest.mark.gpu
def test_gpu_refinement_rejects_bad_options(csm, world3):
    g = csm.HybridGrid(world3.high_resolution, *world3.high_cells[0])
    t, q = world3.node_in_submap(0, 0)
    with pytest.raises(csm.CsmError):
        csm.ceres_refine_batch_3d([g, g], [world3.node(0)], [(0, 1, 0, (t, q), t)],
                                  csm.CeresOptions3D.make(0.0))
