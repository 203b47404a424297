"""The test-visible entry points of the 2D correlative scan matchers through the
C-ABI: SearchParameters (both constructors), ShrinkToFit, GenerateRotatedScans,
DiscretizeScans (correlative_scan_matcher_2d.{h,cc}) and
RealTimeCorrelativeScanMatcher2D::ScoreCandidates
(real_time_correlative_scan_matcher_2d.h:75-78).

The host helpers need no GPU: they are checked here against the oracle
bit-for-bit and against the reference's own correlative_scan_matcher_test.cc
cases. ScoreCandidates runs on the device (gpu marker): float sums in point
order, so scores are bit-identical to the oracle's except through the double
exp penalty (OCML vs glibc), allowed 1e-6 relative as in test_rt2d_gpu.py."""
import math

import numpy as np
import pytest


def _cloud(rng, n, spread=8.0):
    xy = rng.uniform(-spread, spread, (n, 2)).astype(np.float32)
    return np.concatenate([xy, rng.uniform(-0.2, 0.2, (n, 1)).astype(np.float32)], 1)


# ---- reference cases (correlative_scan_matcher_test.cc) ---------------------

def test_search_parameters_construction(csm):
    """correlative_scan_matcher_test.cc:26-40."""
    sp = csm.SearchParameters.for_testing(4, 5, 0.03, 0.05)
    assert sp.num_angular_perturbations == 5
    assert abs(sp.angular_perturbation_step_size - 0.03) < 1e-9
    assert abs(sp.resolution - 0.05) < 1e-9
    assert sp.num_scans == 11
    assert len(sp.linear_bounds) == 11
    assert all(b.as_tuple() == (-4, 4, -4, 4) for b in sp.linear_bounds)


def test_candidate_construction(csm):
    """correlative_scan_matcher_test.cc:42-56."""
    sp = csm.SearchParameters.for_testing(4, 5, 0.03, 0.05)
    c = csm.Candidate2D(3, 4, -5, sp)
    assert (c.scan_index, c.x_index_offset, c.y_index_offset) == (3, 4, -5)
    assert abs(c.x - 0.25) < 1e-9 and abs(c.y + 0.2) < 1e-9
    assert abs(c.orientation + 0.06) < 1e-9 and c.score == 0.0


def test_generate_rotated_scans_reference_case(csm):
    """correlative_scan_matcher_test.cc:58-70."""
    scans = csm.GenerateRotatedScans(np.array([[-1.0, 1.0, 0.0]], np.float32),
                                     csm.SearchParameters.for_testing(0, 1, math.pi / 2, 0.0))
    assert scans.shape == (3, 1, 3)
    for s, (x, y) in enumerate([(1.0, 1.0), (-1.0, 1.0), (-1.0, -1.0)]):
        assert abs(scans[s, 0, 0] - x) < 1e-6 and abs(scans[s, 0, 1] - y) < 1e-6


SEVEN = np.array([[0.025, 0.175, 0], [-0.025, 0.175, 0], [-0.075, 0.175, 0],
                  [-0.125, 0.175, 0], [-0.125, 0.125, 0], [-0.125, 0.075, 0],
                  [-0.125, 0.025, 0]], np.float32)


def test_discretize_scans_reference_case(csm):
    """correlative_scan_matcher_test.cc:72-96: exact cell indices."""
    limits = csm.MapLimits(0.05, 0.05, 0.25, 6, 6)
    sp = csm.SearchParameters.for_testing(0, 0, 0.0, 0.0)
    d = csm.DiscretizeScans(limits, csm.GenerateRotatedScans(SEVEN, sp), (0.0, 0.0))
    assert d.shape == (1, 7, 2)
    assert [tuple(v) for v in d[0]] == [(1, 0), (1, 1), (1, 2), (1, 3), (2, 3), (3, 3), (4, 3)]


# ---- against the oracle -----------------------------------------------------

def test_search_parameters_match_oracle(csm, oracle):
    rng = np.random.RandomState(3)
    for trial in range(20):
        cloud = _cloud(rng, rng.randint(1, 400), spread=rng.uniform(0.01, 30.0))
        res = float(rng.choice([0.05, 0.1, 0.025, 1.0]))
        lin, ang = float(rng.uniform(0, 8)), float(rng.uniform(0, math.pi))
        sp = csm.SearchParameters(lin, ang, cloud, res)
        na, step, ns, b = oracle.search_parameters(lin, ang, cloud, res)
        assert (sp.num_angular_perturbations, sp.num_scans) == (na, ns)
        assert sp.angular_perturbation_step_size == step  # same double arithmetic
        assert all(x.as_tuple() == b for x in sp.linear_bounds)


def test_rotated_scans_and_discretization_match_oracle(csm, oracle):
    rng = np.random.RandomState(4)
    for trial in range(10):
        cloud = _cloud(rng, 300)
        na, step = int(rng.randint(0, 12)), float(rng.uniform(1e-3, 0.05))
        res = float(rng.choice([0.05, 0.1]))
        sp = csm.SearchParameters.for_testing(7, na, step, res)
        scans = csm.GenerateRotatedScans(cloud, sp)
        ref = oracle.generate_rotated_scans(cloud, 7, na, step, res)
        assert np.array_equal(scans.view(np.uint32), ref.view(np.uint32))  # bit-identical
        limits = csm.MapLimits(res, float(rng.uniform(-5, 5)), float(rng.uniform(-5, 5)), 200, 180)
        t = (float(rng.uniform(-3, 3)), float(rng.uniform(-3, 3)))
        d = csm.DiscretizeScans(limits, scans, t)
        dref = oracle.discretize_scans((res, limits.max_x, limits.max_y, 200, 180), ref, *t)
        assert np.array_equal(d, dref)


def test_shrink_to_fit_matches_oracle(csm, oracle):
    """ShrinkToFit after the FastCSM pipeline (SearchParameters from the input
    cloud, rotated scans, discretization at the initial translation)."""
    world = csm.SyntheticWorld2D(num_nodes=4, num_submaps=2, submap_cells=200, decimate_to=300,
                                 seed=8)
    for s in range(2):
        g = world.grid(s)
        cloud = world.cloud(int(world.submap_nodes[s]))
        init = (float(g.max_x) - 4.0, float(g.max_y) - 6.0, 0.0)
        sp = csm.SearchParameters(7.0, math.radians(30.0), cloud, g.resolution)
        d = csm.DiscretizeScans(g.limits(), csm.GenerateRotatedScans(cloud, sp), init[:2])
        sp.ShrinkToFit(d, g.num_x_cells, g.num_y_cells)
        ns, bounds, dref, _ = oracle.discretize((g.resolution, g.max_x, g.max_y), g.cells, init,
                                                7.0, math.radians(30.0), cloud, rotated_sp=False)
        assert ns == sp.num_scans
        assert np.array_equal(d.reshape(-1, 2), np.asarray(dref).reshape(-1, 2))
        assert [b.as_tuple() for b in sp.linear_bounds] == [tuple(b) for b in bounds]


# ---- RealTimeCorrelativeScanMatcher2D::ScoreCandidates on the device --------

@pytest.mark.gpu
def test_score_perfect_candidate_reference_case(csm, oracle):
    """real_time_correlative_scan_matcher_2d_test.cc:127-145
    (ScorePerfectHighResolutionCandidateProbabilityGrid)."""
    limits, cells = oracle.grid_from_inserts(0.05, 0.05, 0.25, 6, 6, [((0, 0, 0), SEVEN)])
    g = csm.ProbabilityGrid(*limits, cells)
    sp = csm.SearchParameters.for_testing(0, 0, 0.0, 0.0)
    d = csm.DiscretizeScans(g.limits(), csm.GenerateRotatedScans(SEVEN, sp), (0.0, 0.0))
    m = csm.RealTimeCorrelativeScanMatcher2D(
        csm.RealTimeCorrelativeScanMatcherOptions(0.6, 0.16, 0.0, 0.0))
    cands = [csm.Candidate2D(0, 0, 0, sp)]
    m.ScoreCandidates(g, d, sp, cands)
    assert (cands[0].scan_index, cands[0].x_index_offset, cands[0].y_index_offset) == (0, 0, 0)
    assert abs(cands[0].score - 0.7) <= 1e-2


def _random_candidates(csm, rng, sp, k, reach):
    return [csm.Candidate2D(int(rng.randint(0, sp.num_scans)), int(rng.randint(-reach, reach + 1)),
                            int(rng.randint(-reach, reach + 1)), sp) for _ in range(k)]


@pytest.mark.gpu
def test_score_candidates_match_oracle(csm, oracle):
    world = csm.SyntheticWorld2D(num_nodes=4, num_submaps=2, submap_cells=200, seed=12)
    rng = np.random.RandomState(7)
    for opts in [(0.2, math.radians(10.0), 0.1, 0.1), (0.6, 0.16, 0.0, 0.0)]:
        m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
        for s in range(2):
            g = world.grid(s)
            cloud = world.cloud(int(world.submap_nodes[s]))
            sp = csm.SearchParameters(opts[0], opts[1], cloud, g.resolution)
            t = world.node_poses[int(world.submap_nodes[s])]
            d = csm.DiscretizeScans(g.limits(), csm.GenerateRotatedScans(cloud, sp), t[:2])
            # Offsets reach far past the window and the grid (outside cells).
            cands = _random_candidates(csm, rng, sp, 500, 300)
            scores = m.ScoreCandidates(g, d, sp, cands)
            ref = oracle.rt2d_score_candidates(
                (g.resolution, g.max_x, g.max_y, g.num_x_cells, g.num_y_cells), g.cells, opts[2],
                opts[3], d, sp.num_angular_perturbations, sp.angular_perturbation_step_size,
                [(c.scan_index, c.x_index_offset, c.y_index_offset) for c in cands])
            assert np.allclose(scores, ref, rtol=1e-6, atol=0.0)
            assert np.mean(scores == ref) > 0.99


@pytest.mark.gpu
def test_score_candidates_tsdf_match_oracle(csm, oracle):
    limits, tsd, wgt = oracle.tsdf_from_inserts(0.05, 0.3, 0.5, 20, 20, 0.3, 1.0,
                                                [((0.5, -0.5, 0), SEVEN)])
    g = csm.TSDF2D(*limits, tsd, wgt, 0.3, 1.0)
    rng = np.random.RandomState(1)
    opts = (0.6, 0.16, 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher2D(csm.RealTimeCorrelativeScanMatcherOptions(*opts))
    sp = csm.SearchParameters(opts[0], opts[1], SEVEN, 0.05)
    d = csm.DiscretizeScans(g.limits(), csm.GenerateRotatedScans(SEVEN, sp), (0.02, -0.03))
    cands = _random_candidates(csm, rng, sp, 400, 12)
    scores = m.ScoreCandidates(g, d, sp, cands)
    assert np.count_nonzero(scores) > 40
    ref = oracle.rt2d_score_candidates(
        (limits[0], limits[1], limits[2], tsd.shape[1], tsd.shape[0]), tsd, opts[2], opts[3], d,
        sp.num_angular_perturbations, sp.angular_perturbation_step_size,
        [(c.scan_index, c.x_index_offset, c.y_index_offset) for c in cands],
        tsdf=(wgt, 0.3, 1.0))
    assert np.allclose(scores, ref, rtol=1e-6, atol=0.0)
