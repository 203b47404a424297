"""CeresScanMatcher3D refinement (ceres_scan_matcher_3d.cc:84-160, called by
ConstraintBuilder3D::ComputeConstraint at constraint_builder_3d.cc:264-275).

Ceres is absent from this image: the oracle (oracle/ceres3d.cc) restates the
cost (two OccupiedSpaceCostFunction3D blocks over InterpolatedGrid, the
translation and rotation delta functors), the quaternion parameterization and
Ceres' LM defaults — PARITY UNPINNED against Ceres. Its analytic Jacobians are
checked against finite differences of the same cost (the oracle's own
functions). The HIP path must agree with the restatement to 1e-6."""
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
    for opts in [OPTS, (5.0, 30.0, 10.0, 1.0, 1), (1.0, 2.0, 0.5, 0.3, 20)]:
        poses, iters = csm.ceres_refine_batch_3d(grids, nodes, items, csm.CeresOptions3D.make(*opts))
        for k, (hgi, lgi, nd, (tt, qq), tgt) in enumerate(items):
            hg, lg = ogrids[hgi // 2]
            (rt, rq), rit = oracle.ceres3d_match(hg, lg, world3.high[nd], world3.low[nd], opts,
                                                 tgt, tt, qq)
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
