"""Submap2D::Finish's crop (ProbabilityGrid::ComputeCroppedGrid,
probability_grid.cc:91-106; Grid2D::ComputeCroppedLimits, grid_2d.cc:110-120)
through csm_grid2d_crop (host side of the boundary, no GPU), against the
oracle, which crops to the known box its updates tracked (ExtendBox on every
update) rather than to the nonzero cells: the two must agree exactly."""
import numpy as np


def _crop(csm, limits, cells):
    g = csm.ProbabilityGrid(*limits, cells)
    return csm.ComputeCroppedGrid(g)


def test_crop_matches_oracle_on_inserted_scans(csm, oracle):
    rng = np.random.RandomState(3)
    for trial in range(6):
        inserts = []
        for _ in range(3):
            origin = (rng.uniform(-1, 1), rng.uniform(-1, 1), 0.0)
            ang = np.linspace(-np.pi, np.pi, 180)
            r = rng.uniform(0.5, 2.5, size=len(ang))
            pts = np.stack([origin[0] + r * np.cos(ang), origin[1] + r * np.sin(ang),
                            np.zeros_like(r)], 1).astype(np.float32)
            inserts.append((origin, pts))
        # A generous fixed grid (no growth) and a small one the inserter grows.
        for lim in [(0.05, 4.0, 4.0, 160, 160), (0.05, 0.5, 0.5, 20, 20)]:
            full_limits, full = oracle.grid_from_inserts(*lim, inserts)
            ref_limits, ref = oracle.grid_from_inserts(*lim, inserts, crop=True)
            out = _crop(csm, full_limits, full)
            assert (out.resolution, out.max_x, out.max_y) == ref_limits
            np.testing.assert_array_equal(out.cells, ref)


def test_every_value_survives_the_crop_round_trip(csm, oracle):
    """SetProbability(GetProbability(v)) == v for v in 1..32767."""
    table = np.arange(1, 32768, dtype=np.uint16)
    cells = np.zeros((130, 256), np.uint16)
    cells.flat[256:256 + len(table)] = table
    out = _crop(csm, (0.05, 10.0, 10.0), cells)
    assert out.cells.shape == (128, 256)
    np.testing.assert_array_equal(out.cells.flat[:len(table)], table)


def test_crop_of_an_unknown_grid_is_one_cell(csm):
    out = _crop(csm, (0.05, 1.0, 2.0), np.zeros((7, 9), np.uint16))
    assert out.cells.shape == (1, 1) and out.cells[0, 0] == 0
    assert (out.max_x, out.max_y) == (1.0, 2.0)


def test_crop_limits_follow_the_offset(csm):
    cells = np.zeros((40, 30), np.uint16)
    cells[11, 5] = 1000
    cells[20, 17] = 30000
    out = _crop(csm, (0.05, 3.0, 2.0), cells)
    assert out.cells.shape == (10, 13)
    assert out.max_x == 3.0 - 0.05 * 11 and out.max_y == 2.0 - 0.05 * 5
    assert out.cells[0, 0] == 1000 and out.cells[9, 12] == 30000
