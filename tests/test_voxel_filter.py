"""Voxel filters (sensor/internal/voxel_filter.cc): the oracle against the
reference's own tests (restated in oracle/ref_tests_voxel.cc, run by
test_oracle.py) and an independent pure-Python restatement of the reservoir
draws; the HIP batch kernel (csm_voxel_filter / csm_adaptive_voxel_filter)
against the oracle, bit-exact on the kept set.

Edge cases the reference tests hold: several points per voxel, intensities
following their points, large coordinates, identical points (IgnoresTime).
Added here: empty clouds, clouds at the 8192-point limit, a single voxel of
2000 points (std::uniform_int_distribution rejects minstd output 1311 of its
stream, shifting every later draw), negative coordinates whose keys wrap, and
AdaptiveVoxelFilter's range filter and edge-length search with the 2D and 3D
option sets of configuration_files/trajectory_builder_{2d,3d}.lua.
"""
import numpy as np
import pytest

MINSTD_M = 2147483647
URNG_RANGE = 2147483645


def py_voxel_filter(cloud, resolution):
    """Pure-Python restatement of RandomizedVoxelFilterIndices (:136-162), for
    small clouds: minstd_rand0 (seed 1) and libstdc++'s downscaling
    uniform_int_distribution, in point order."""
    res = np.float32(resolution)
    state = 1
    voxels = {}
    for i, p in enumerate(np.asarray(cloud, np.float32)):
        q = [np.float32(v) / res for v in p]
        idx = []
        for v in q:
            r = int(np.floor(abs(float(v)) + 0.5)) * (1 if v >= 0 else -1)  # lround
            r = ((r + 2**31) % 2**32) - 2**31  # narrowed to int
            idx.append(r % 2**64)
        key = ((idx[0] << 42) + (idx[1] << 21) + idx[2]) % 2**64
        cnt, sel = voxels.get(key, (0, -1))
        cnt += 1
        if cnt == 1:
            sel = i
        else:
            scaling = URNG_RANGE // cnt
            past = cnt * scaling
            while True:
                state = state * 16807 % MINSTD_M
                ret = state - 1
                if ret < past:
                    break
            if ret // scaling + 1 == cnt:
                sel = i
        voxels[key] = (cnt, sel)
    keep = np.zeros(len(cloud), bool)
    for _, sel in voxels.values():
        keep[sel] = True
    return keep


def rejection_cloud(n=2000):
    """n points in one voxel: draw k = r + 1 at stream position r - 1."""
    rng = np.random.RandomState(7)
    return (0.2 + 0.05 * rng.rand(n, 3)).astype(np.float32)


def scan_like_clouds(count, n, seed):
    rng = np.random.RandomState(seed)
    out = []
    for _ in range(count):
        ang = np.linspace(-2.3, 2.3, n)
        r = 2.0 + 8.0 * rng.rand() + 3.0 * np.abs(np.sin(3 * ang + rng.rand() * 6)) \
            + 0.01 * rng.randn(n)
        out.append(np.stack([r * np.cos(ang), r * np.sin(ang), np.zeros(n)], 1).astype(np.float32))
    return out


def cloud3d(n, seed, scale=20.0):
    rng = np.random.RandomState(seed)
    pts = rng.randn(n, 3) * np.array([scale, scale, scale / 6])
    return pts.astype(np.float32)


# ---------------------------------------------------------------- CPU ----

def test_oracle_matches_python_restatement(oracle):
    clouds = [np.zeros((5, 3), np.float32), cloud3d(300, 1, 1.0), scan_like_clouds(1, 200, 2)[0],
              rejection_cloud(1400), cloud3d(200, 3, 1e4)]
    for res in (0.3, 0.05, 0.025):
        keep, _ = oracle.voxel_filter_masks(clouds, res)
        off = 0
        for c in clouds:
            np.testing.assert_array_equal(keep[off:off + len(c)], py_voxel_filter(c, res))
            off += len(c)


def test_rejection_is_in_the_stream():
    """Output 1311 of minstd_rand0 (draw with k = 1312) is rejected by the
    downscaling loop: the case the kernel's in-order replay exists for."""
    state, rejected = 1, []
    for pos in range(2000):
        state = state * 16807 % MINSTD_M
        k = pos + 2
        if state - 1 >= k * (URNG_RANGE // k):
            rejected.append(pos)
    assert rejected == [1310]


def test_oracle_one_point_per_voxel(oracle):
    cloud = cloud3d(3000, 5, 3.0)
    keep, _ = oracle.voxel_filter_masks([cloud], 0.2)
    keys = np.round(cloud / np.float32(0.2)).astype(np.int64)
    kept = {tuple(k) for k in keys[keep]}
    assert len(kept) == keep.sum() == len({tuple(k) for k in keys})


# ---------------------------------------------------------------- GPU ----

def _check_batch(csm, oracle, clouds, resolution):
    keep, counts, offsets = csm.voxel_filter_masks(clouds, resolution)
    ref, ref_off = oracle.voxel_filter_masks(clouds, resolution)
    np.testing.assert_array_equal(offsets, ref_off)
    np.testing.assert_array_equal(keep, ref)
    for c in range(len(clouds)):
        assert counts[c] == ref[offsets[c]:offsets[c + 1]].sum()


def _check_adaptive(csm, oracle, clouds, max_length, min_num_points, max_range):
    opts = csm.AdaptiveVoxelFilterOptions.make(max_length, min_num_points, max_range)
    keep, counts, offsets = csm.adaptive_voxel_filter_masks(clouds, opts)
    ref, _ = oracle.adaptive_voxel_filter_masks(clouds, max_length, min_num_points, max_range)
    np.testing.assert_array_equal(keep, ref)
    for c in range(len(clouds)):
        assert counts[c] == ref[offsets[c]:offsets[c + 1]].sum()
    return keep, counts


@pytest.mark.gpu
def test_reference_cases_on_gpu(csm):
    """voxel_filter_test.cc's four cases through the HIP path."""
    cloud = np.array([[0, 0, 0], [0.1, -0.1, 0.1], [0.3, -0.1, 0], [0, 0, 0.1]], np.float32)
    out = csm.VoxelFilter(cloud, 0.3)
    assert len(out) == 2 and any((out == cloud[2]).all(1))
    pts = np.array([[-100.0, 0.3, 0.1 * i] for i in range(100)], np.float32)
    inten = (np.float32(0.1) * np.arange(100, dtype=np.float32)).astype(np.float32)
    out, oi = csm.VoxelFilter(pts, 0.3, intensities=inten)
    assert len(out) == len(oi) and np.allclose(out[:, 2], oi, atol=1e-6)
    big = np.array([[100000.0, 0, 0], [100000.001, -0.0001, 0.0001], [100000.003, -0.0001, 0],
                    [-200000.0, 0, 0]], np.float32)
    out = csm.VoxelFilter(big, 0.01)
    assert len(out) == 2 and any((out == big[3]).all(1))
    same = np.tile(np.array([[-100.0, 0.3, 0.4]], np.float32), (100, 1))
    assert len(csm.VoxelFilter(same, 0.3)) == 1


@pytest.mark.gpu
def test_voxel_filter_scans_match_oracle(csm, oracle):
    clouds = scan_like_clouds(64, 1080, 11)
    for res in (0.025, 0.05, 0.3):
        _check_batch(csm, oracle, clouds, res)


@pytest.mark.gpu
def test_voxel_filter_3d_and_edge_cases(csm, oracle):
    clouds = [cloud3d(8192, 1), cloud3d(5000, 2, 2.0), np.zeros((0, 3), np.float32),
              cloud3d(1, 3), rejection_cloud(2000), rejection_cloud(8192),
              cloud3d(777, 4, 1e4), -np.abs(cloud3d(900, 5, 0.5)),
              np.tile(np.array([[1e5, -2e5, 3.0]], np.float32), (300, 1))]
    for res in (0.15, 0.01, 1.0):
        _check_batch(csm, oracle, clouds, res)


@pytest.mark.gpu
def test_adaptive_voxel_filter_2d_options(csm, oracle):
    clouds = scan_like_clouds(48, 1080, 21) + [scan_like_clouds(1, 150, 22)[0],
                                               np.zeros((0, 3), np.float32)]
    # adaptive_voxel_filter and loop_closure_adaptive_voxel_filter
    # (trajectory_builder_2d.lua:25-35).
    keep, counts = _check_adaptive(csm, oracle, clouds, 0.5, 200, 50.0)
    assert (counts[:48] >= 200).all()
    _check_adaptive(csm, oracle, clouds, 0.9, 100, 50.0)
    # A tight range filter and a minimum no length reaches.
    _check_adaptive(csm, oracle, clouds, 0.5, 900, 6.0)


@pytest.mark.gpu
def test_adaptive_voxel_filter_3d_options(csm, oracle):
    clouds = [cloud3d(n, 30 + n % 7, s) for n, s in
              [(8192, 10.0), (6000, 4.0), (3000, 30.0), (150, 5.0), (151, 5.0), (2000, 60.0)]]
    # high / low resolution filters (trajectory_builder_3d.lua:24-34).
    _check_adaptive(csm, oracle, clouds, 2.0, 150, 15.0)
    _check_adaptive(csm, oracle, clouds, 4.0, 200, 60.0)


@pytest.mark.gpu
def test_voxel_filter_rejects_oversized_clouds(csm):
    with pytest.raises(csm.CsmError):
        csm.voxel_filter_masks([cloud3d(8193, 1)], 0.1)
