"""Exactly tied maxima of any size: the ordered walk (csm_host.cc ResolveTies
step 4, `fast2d_walk`; host3d.cc ResolveTies3d, `fast3d_walk`).

The reference returns the first maximal leaf its depth-first search visits
(fast_correlative_scan_matcher_2d.cc:276-312, :335-378;
fast_correlative_scan_matcher_3d.cc:377-440), however many leaves tie. The
collect pass records at most 4096 tied leaves per pair; past that the device
walks the reference's visiting order itself (CSM_TIE_WALK). These tests drive
pairs far past that cap and require the oracle's pose exactly:

* the inputs of the reference's own ConstraintBuilder2DTest.FindsConstraints
  (constraint_builder_2d_test.cc:70-112: all-unknown 100 x 110 grid at 1 m,
  one point, min_score 0, where every leaf ties), through the matcher and
  through the builder, whose constraint poses are compared with the oracle;
* MatchFullSubmap on an all-unknown grid at min_score 0;
* a plateau world with more than 10^4 tied leaves, where lowest-resolution
  candidates at the plateau's border bound the maximum without holding a
  leaf at it, so the walk has to back out of them.
"""
import math

import numpy as np
import pytest

from conftest import assert_search_ok

pytestmark = pytest.mark.gpu

KERNELS = {"v5": {}, "v4-lifo": {"CSM_SEARCH_KERNEL": "4", "CSM_SEARCH_ORDER": "lifo"}}


@pytest.fixture(params=list(KERNELS))
def kernel(request, monkeypatch):
    for var in ("CSM_SEARCH_KERNEL", "CSM_HEX_LEVELS", "CSM_SEARCH_ORDER"):
        monkeypatch.delenv(var, raising=False)
    for var, val in KERNELS[request.param].items():
        monkeypatch.setenv(var, val)
    return request.param


def _unknown_grid(csm):
    # MapLimits(1., (2., 3.), CellLimits(100, 110)) (constraint_builder_2d_test.cc:76-79).
    cells = np.zeros((110, 100), np.uint16)
    return (1.0, 2.0, 3.0), cells, csm.ProbabilityGrid(1.0, 2.0, 3.0, cells)


def _center(limits, cells):
    res, mx, my = limits
    return (mx - 0.5 * res * cells.shape[0], my - 0.5 * res * cells.shape[1], 0.0)


def _run(csm, mats, clouds, pairs_spec):
    """pairs_spec: (submap, scan, full, min_score, initial) -> batch results."""
    scans = csm.ScanSet(clouds)
    pairs = np.zeros(len(pairs_spec), dtype=csm.make_pairs([0], [0], 0.0).dtype)
    for k, (s, n, full, ms, init) in enumerate(pairs_spec):
        p = csm.make_pairs([s], [n], ms, full_submap=full, initial=None if full else [init])
        pairs[k] = p[0]
    ctx = csm.default_context(0)
    ctx.reset_timing()
    res = csm.match_batch(mats, scans, pairs)
    return res, ctx.timing()


def _assert_exact(res_k, ref):
    ok, score, pose = ref[:3]
    assert (res_k["status"] == 0) == ok
    if ok:
        assert np.float32(res_k["score"]) == np.float32(score)
        got = (res_k["x"], res_k["y"], res_k["theta"])
        assert got == tuple(pose), ("pose differs from the reference's pick", got, pose)


def test_finds_constraints_inputs_match_oracle(csm, oracle, kernel):
    """The FindsConstraints pairs: Match at the node pose (the two
    MaybeAddConstraint calls) and MatchFullSubmap (MaybeAddGlobalConstraint),
    min_score 0, default options (linear 7 m, angular 30 deg, depth 7)."""
    limits, cells, grid = _unknown_grid(csm)
    opts = csm.FastCorrelativeScanMatcherOptions2D()
    m = csm.FastCorrelativeScanMatcher2D(grid, opts)
    om = oracle.fast2d(limits, cells, opts.linear_search_window, opts.angular_search_window,
                       opts.branch_and_bound_depth)
    cloud = np.array([[0.1, 0.2, 0.3]], np.float32)
    # The submap sits at (4, 5) and the node at the origin: the search start
    # is the node's pose in the submap frame (constraint_builder_2d.cc:195-197).
    init = (-4.0, -5.0, 0.0)
    res, tm = _run(csm, [m], [cloud], [(0, 0, False, 0.0, init), (0, 0, True, 0.0, None)])
    assert_search_ok(csm, res["status"])
    _assert_exact(res[0], om.match(init, cloud, 0.0))
    _assert_exact(res[1], om.match_full_submap(cloud, 0.0))
    assert (res["tie"] == csm.TIE_WALK).all(), res["tie"]
    assert tm.ties_walked == 2
    # The single-call drop-ins take the same path.
    assert m.Match(init, cloud, 0.0) == (True, float(res[0]["score"]),
                                         (res[0]["x"], res[0]["y"], res[0]["theta"]))
    assert m.MatchFullSubmap(cloud, 0.0) == (True, float(res[1]["score"]),
                                             (res[1]["x"], res[1]["y"], res[1]["theta"]))


def test_unknown_grid_full_submap_clouds(csm, oracle, kernel):
    """MatchFullSubmap on an all-unknown grid at min_score 0 with clouds of 1,
    7 and 60 points and two depths: every leaf inside the grid ties."""
    limits, cells, grid = _unknown_grid(csm)
    rng = np.random.default_rng(5)
    clouds = [np.array([[0.1, 0.2, 0.3]], np.float32),
              rng.uniform(-3, 3, (7, 3)).astype(np.float32),
              rng.uniform(-6, 6, (60, 3)).astype(np.float32)]
    for depth in (7, 3):
        opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30), depth)
        m = csm.FastCorrelativeScanMatcher2D(grid, opts)
        om = oracle.fast2d(limits, cells, 7.0, math.radians(30), depth)
        res, tm = _run(csm, [m], clouds, [(0, i, True, 0.0, None) for i in range(len(clouds))])
        assert_search_ok(csm, res["status"])
        for i, c in enumerate(clouds):
            _assert_exact(res[i], om.match_full_submap(c, 0.0))
        assert tm.ties_walked == len(clouds)


def _plateau_world(csm, seed):
    """A 5 cm grid of random known cells (probability 0.15-0.6) with a square
    plateau of one higher value, and a small cloud that fits on it many ways."""
    rng = np.random.default_rng(seed)
    n = 120
    p = rng.uniform(0.15, 0.6, (n, n))
    p[30:90, 25:85] = 0.8
    # ProbabilityToCorrespondenceCost, then the uint16 value (probability_values.h).
    cc = 1.0 - p
    cells = (1 + np.round((cc - 0.1) / 0.8 * 32766)).astype(np.uint16)
    limits = (0.05, 3.0, 3.0)
    ang = rng.uniform(0, 2 * math.pi, 24)
    rad = rng.uniform(0.05, 0.35, 24)
    cloud = np.stack([rad * np.cos(ang), rad * np.sin(ang), np.zeros(24)], 1).astype(np.float32)
    return limits, cells, csm.ProbabilityGrid(*limits, cells), cloud


@pytest.mark.parametrize("seed", [1, 2])
def test_plateau_ties_past_the_record(csm, oracle, kernel, seed):
    """More than 10^4 leaves at the maximum (counted by the oracle): the
    reference's pick, through the batch and the single call."""
    limits, cells, grid, cloud = _plateau_world(csm, seed)
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30), 5)
    m = csm.FastCorrelativeScanMatcher2D(grid, opts)
    om = oracle.fast2d(limits, cells, 7.0, math.radians(30), 5)
    ref = om.match_full_submap(cloud, 0.5)
    assert ref[0]
    leaves, pick = om.tie_leaves(True, None, cloud, 0.5, max_out=1 << 20)
    assert len(leaves) > 10_000, len(leaves)
    res, tm = _run(csm, [m], [cloud], [(0, 0, True, 0.5, None)])
    assert_search_ok(csm, res["status"])
    _assert_exact(res[0], ref)
    assert res[0]["tie"] == csm.TIE_WALK and tm.ties_walked == 1
    assert m.MatchFullSubmap(cloud, 0.5) == (True, float(res[0]["score"]),
                                             (res[0]["x"], res[0]["y"], res[0]["theta"]))
