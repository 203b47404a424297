"""HybridGrid / InterpolatedProbabilityGrid parity against the fork's captured
output (tests/golden/hybrid_test_fork.json, made from
/root/reference/hybrid_test.txt by tests/golden/make_hybrid_fixture.py) and
interpolated_grid_test.cc on the device.

CPU: the oracle's HybridGrid (GetCellIndex in float with lround, the iterator
order of DynamicGrid -> NestedGrid -> FlatGrid, hybrid_grid.h:40-545) and
InterpolatedGrid (interpolated_grid.h:48-105) reproduce every cell index,
probability and interpolated value the fork printed (6 significant digits:
tolerance 1e-6). GPU: the device brick made from that grid
(csm_hybrid_grid_create) returns the same probabilities, and the
CeresScanMatcher3D kernel's interpolation (csm_hybrid_grid_interpolate)
equals the oracle's and the fork's values.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = json.load(open(os.path.join(HERE, "golden", "hybrid_test_fork.json")))
PRINT_TOL = 1e-6  # values were printed with 6 significant digits


def sample_points(section):
    """point + Vector3f(float(0.2 * i), 0, 0) in float (hybrid_grid_test.cc:142)."""
    o = np.asarray(FIXTURE["sample_origin"], np.float32)
    pts = []
    for s in section["samples"]:
        step = np.float32(FIXTURE["sample_step"] * s["i"])
        pts.append(np.array([o[0] + step, o[1], o[2]], np.float32))
    return np.stack(pts)


def oracle_grid(oracle, res):
    og = oracle.hybrid_grid(res)
    for p in FIXTURE["points"]:
        i, j, k = og.cell_index(np.asarray(p, np.float32))[0]
        og.set_probability(int(i), int(j), int(k), FIXTURE["probability_set"])
    return og


@pytest.mark.parametrize("section", FIXTURE["sections"], ids=lambda s: f"res{s['resolution']}")
def test_oracle_matches_fork_output(oracle, section):
    og = oracle_grid(oracle, section["resolution"])
    ijk, v = og.cells()
    expected = [c["index"] for c in section["cells"]]
    assert ijk.tolist() == expected  # same cells, in the iterator's order
    for (i, j, k), c in zip(ijk, section["cells"]):
        assert abs(og.probability(int(i), int(j), int(k)) - c["probability"]) <= PRINT_TOL
    pts = sample_points(section)
    for p, s in zip(pts, section["samples"]):
        np.testing.assert_allclose(p, s["printed_point"], atol=5e-6)
    cells = og.cell_index(pts)
    interp = og.interpolate(pts.astype(np.float64))
    for (i, j, k), val, s in zip(cells, interp, section["samples"]):
        assert abs(og.probability(int(i), int(j), int(k)) - s["cell_probability"]) <= PRINT_TOL
        assert abs(val - s["interpolated"]) <= PRINT_TOL, (val, s)


@pytest.mark.gpu
@pytest.mark.parametrize("section", FIXTURE["sections"], ids=lambda s: f"res{s['resolution']}")
def test_device_grid_matches_fork_output(csm, oracle, section):
    og = oracle_grid(oracle, section["resolution"])
    ijk, v = og.cells()
    g = csm.HybridGrid(section["resolution"], ijk, v, grid_size=og.grid_size)
    probs = g.get_probability(np.asarray([c["index"] for c in section["cells"]]))
    assert np.all(np.abs(probs - [c["probability"] for c in section["cells"]]) <= PRINT_TOL)
    pts = sample_points(section)
    cell_probs = g.get_probability(og.cell_index(pts))
    assert np.all(np.abs(cell_probs - [s["cell_probability"] for s in section["samples"]]) <= PRINT_TOL)
    dev = g.interpolate(pts.astype(np.float64))
    ref = og.interpolate(pts.astype(np.float64))
    np.testing.assert_allclose(dev, ref, rtol=0, atol=1e-12)
    assert np.all(np.abs(dev - [s["interpolated"] for s in section["samples"]]) <= PRINT_TOL)


@pytest.mark.gpu
def test_device_interpolated_grid_reference_cases(csm, oracle):
    """interpolated_grid_test.cc:28-85 on the device: at grid points the
    interpolation equals the cell probability (1e-6), and between grid
    points it moves monotonically in x, over the test's whole lattice."""
    og = oracle.hybrid_grid(0.1)
    for p in [(-3, 2, 0), (-4, 2, 0), (-5, 2, 0), (-6, 2, 0), (-6, 3, 1), (-6, 4, 2), (-7, 3, 1)]:
        i, j, k = og.cell_index(np.asarray(p, np.float32))[0]
        og.set_probability(int(i), int(j), int(k), 1.0)
    ijk, v = og.cells()
    g = csm.HybridGrid(0.1, ijk, v, grid_size=og.grid_size)
    res = float(np.float32(0.1))

    def axis(lo, hi):  # for (double t = lo; t < hi; t += res), as the test accumulates
        out, t = [], lo
        while t < hi:
            out.append(t)
            t += res
        return np.asarray(out)

    zs, ys, xs = axis(-1.0, 3.0), axis(1.0, 5.0), axis(-8.0, -2.0)
    Z, Y, X = np.meshgrid(zs, ys, xs, indexing="ij")
    pts = np.stack([X.ravel(), Y.ravel(), Z.ravel()], 1)
    interp = g.interpolate(pts)
    cell_p = g.get_probability(og.cell_index(pts.astype(np.float32)))
    np.testing.assert_allclose(interp, cell_p, rtol=0, atol=1e-6)
    np.testing.assert_allclose(interp, og.interpolate(pts), rtol=0, atol=1e-12)
    # Monotonic between grid points in x (the test's sample loop).
    step = res / 10.0
    nxt = g.get_probability(og.cell_index((pts + [res, 0, 0]).astype(np.float32)))
    diff = nxt - cell_p
    rows = np.nonzero(np.abs(diff) >= 1e-6)[0]
    assert len(rows) > 0
    samples = []
    s = step
    while s < res - 2 * step:
        samples.append(s)
        s += step
    for r in rows:
        q = np.array([[pts[r, 0] + s_, pts[r, 1], pts[r, 2]] for s_ in samples + [samples[-1] + step]])
        vals = g.interpolate(q)
        assert np.all(diff[r] * np.diff(vals) > 0), (pts[r], vals)
