"""pbstream ingest (csm_pbstream_*, cartographer-1_amd/csrc/pbstream.cc).

Parity unpinned: the reference ships no .pbstream file and the image has no
protobuf runtime, so these tests write streams with a small encoder that
follows the reference's framing (io/proto_stream.cc:26-66: little-endian magic,
then per message a little-endian size and a gzip member), the proto3 wire
format of the messages it serializes (mapping/proto/serialization.proto,
submap.proto, grid_2d.proto, trajectory_node_data.proto, sensor.proto,
transform.proto) and CompressedPointCloud's block encoding
(sensor/compressed_point_cloud.cc:99-146). The reader must return the same
grids, poses and ids, and clouds bit-exact with the reference's decode
arithmetic (compressed_point_cloud.cc:79-97) restated in numpy float32.
"""
import gzip
import math
import struct

import numpy as np
import pytest

MAGIC = 0x7B1D1F7B5BF501DB


# ---- proto3 wire encoder ---------------------------------------------------
def varint(v):
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def key(f, w):
    return varint(f << 3 | w)


def f_int(f, v):
    return key(f, 0) + varint(int(v))


def f_dbl(f, v):
    return key(f, 1) + struct.pack("<d", v)


def f_flt(f, v):
    return key(f, 5) + struct.pack("<f", v)


def f_msg(f, body):
    return key(f, 2) + varint(len(body)) + body


def f_packed(f, vals):
    return f_msg(f, b"".join(varint(int(v)) for v in vals))


def quaternion(wxyz):
    w, x, y, z = wxyz
    return f_dbl(1, x) + f_dbl(2, y) + f_dbl(3, z) + f_dbl(4, w)


def rigid3d(pose7):
    t = f_dbl(1, pose7[0]) + f_dbl(2, pose7[1]) + f_dbl(3, pose7[2])
    return f_msg(1, t) + f_msg(2, quaternion(pose7[3:]))


def grid2d(resolution, max_x, max_y, cells, min_cc=None, max_cc=None, packed=True):
    ny, nx = cells.shape
    limits = (f_dbl(1, resolution) + f_msg(2, f_dbl(1, max_x) + f_dbl(2, max_y)) +
              f_msg(3, f_int(1, nx) + f_int(2, ny)))
    flat = cells.reshape(-1).astype(np.int64)
    body = f_msg(1, limits)
    body += f_packed(2, flat) if packed else b"".join(f_int(2, c) for c in flat)
    body += f_msg(3, f_int(1, 0) + f_int(2, 0) + f_int(3, nx - 1) + f_int(4, ny - 1))
    body += f_msg(4, b"")  # probability_grid_2d {}
    if min_cc is not None:
        body += f_flt(6, min_cc) + f_flt(7, max_cc)
    return body


def submap2d_msg(traj, index, pose7, grid_body, finished=True):
    sid = f_int(1, traj) + f_int(2, index)
    s2d = f_msg(1, rigid3d(pose7)) + f_int(2, 90) + f_int(3, int(finished)) + f_msg(4, grid_body)
    return f_msg(3, f_msg(1, sid) + f_msg(2, s2d))


def submap3d_msg(traj, index):
    sid = f_int(1, traj) + f_int(2, index)
    s3d = f_msg(1, rigid3d([0, 0, 0, 1, 0, 0, 0])) + f_int(2, 10) + f_msg(4, f_dbl(1, 0.1))
    return f_msg(3, f_msg(1, sid) + f_msg(3, s3d))


def compress(points):
    """CompressedPointCloud(const PointCloud&) (compressed_point_cloud.cc:99-146):
    blocks of 1024 raster cells at 1 mm. Blocks are emitted in first-seen
    order (the reference iterates its HybridGrid; the format allows any
    block order). Returns (point_data, decoded points in stream order, input
    index of each decoded point)."""
    p = np.asarray(points, np.float32)
    v = p / np.float32(0.001)
    raster = (np.sign(v) * np.floor(np.abs(v.astype(np.float64)) + 0.5)).astype(np.int64)
    block = raster >> 10
    rp = raster & 1023
    order = {}
    for i, b in enumerate(map(tuple, block)):
        order.setdefault(b, []).append(i)
    data, decoded, perm = [], [], []
    for b, idx in order.items():
        perm += idx
        data += [len(idx), *b]
        for i in idx:
            data.append(((int(rp[i, 2]) << 10) + int(rp[i, 1])) << 10 | int(rp[i, 0]))
            c = (np.array(b, np.int64) << 10) + rp[i]
            decoded.append(c.astype(np.int32).astype(np.float32) * np.float32(0.001))
    return data, np.array(decoded, np.float32).reshape(-1, 3), np.array(perm, np.int64)


def node_msg(traj, index, timestamp, pose7, gravity, points):
    data, decoded, _ = compress(points)
    cloud = f_int(1, len(points)) + f_packed(3, data)
    nd = (f_int(1, timestamp) + f_msg(2, quaternion(gravity)) + f_msg(3, cloud) +
          f_msg(7, rigid3d(pose7)))
    return f_msg(4, f_msg(1, f_int(1, traj) + f_int(2, index)) + f_msg(5, nd)), decoded


def write_stream(path, messages, magic=MAGIC, header=f_int(1, 2)):
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", magic))
        for m in ([header] if header is not None else []) + list(messages):
            z = gzip.compress(m)
            f.write(struct.pack("<Q", len(z)))
            f.write(z)


# ---- tests -----------------------------------------------------------------
def test_round_trip(csm, tmp_path):
    rng = np.random.default_rng(7)
    cells_a = rng.integers(0, 32768, size=(37, 53)).astype(np.uint16)
    cells_b = rng.integers(0, 32768, size=(5, 4)).astype(np.uint16)
    pose_a = [1.5, -2.25, 0.0, math.cos(0.2), 0.0, 0.0, math.sin(0.2)]
    pose_b = [-3.0, 4.0, 0.5, 1.0, 0.0, 0.0, 0.0]
    cloud0 = rng.uniform(-30.0, 30.0, size=(500, 3)).astype(np.float32)
    cloud0[:, 2] = rng.uniform(-0.5, 0.5, 500)
    cloud1 = np.array([[0.0005, -0.0005, 0.0], [-1.0236, 1.0244, 2.0]], np.float32)
    g0 = [math.cos(0.05), 0.05, -0.02, 0.0]
    n0, d0 = node_msg(0, 3, 638000000000000000, pose_a, g0, cloud0)
    n1, d1 = node_msg(1, 0, -12, pose_b, [1, 0, 0, 0], cloud1)
    n2, d2 = node_msg(1, 1, 5, pose_b, [1, 0, 0, 0], np.zeros((0, 3), np.float32))
    msgs = [
        f_msg(1, f_msg(1, f_int(1, 2))),  # pose_graph (skipped)
        submap2d_msg(0, 4, pose_a, grid2d(0.05, 12.5, -3.0, cells_a, 0.1, 0.9)),
        submap3d_msg(0, 5),  # 3D submap (skipped)
        submap2d_msg(1, 0, pose_b, grid2d(0.1, 1.0, 2.0, cells_b, 0.2, 0.8), finished=False),
        n0, n1, n2,
        f_msg(6, f_int(1, 0)),  # imu_data (skipped)
    ]
    path = tmp_path / "state.pbstream"
    write_stream(path, msgs)
    st = csm.read_pbstream(path)
    assert st.format_version == 2
    assert len(st.submaps) == 2 and len(st.nodes) == 3
    a, b = st.submaps
    assert (a.trajectory_id, a.submap_index, a.finished) == (0, 4, True)
    assert (b.trajectory_id, b.submap_index, b.finished) == (1, 0, False)
    np.testing.assert_array_equal(a.local_pose, pose_a)
    np.testing.assert_array_equal(b.local_pose, pose_b)
    assert (a.grid.resolution, a.grid.max_x, a.grid.max_y) == (0.05, 12.5, -3.0)
    np.testing.assert_array_equal(a.grid.cells, cells_a)
    np.testing.assert_array_equal(b.grid.cells, cells_b)
    assert a.grid.min_correspondence_cost == float(np.float32(0.1))
    assert b.grid.max_correspondence_cost == float(np.float32(0.8))
    for node, (traj, idx, ts, pose, grav, dec) in zip(st.nodes, [
            (0, 3, 638000000000000000, pose_a, g0, d0), (1, 0, -12, pose_b, [1, 0, 0, 0], d1),
            (1, 1, 5, pose_b, [1, 0, 0, 0], d2)]):
        assert (node.trajectory_id, node.node_index, node.timestamp) == (traj, idx, ts)
        np.testing.assert_array_equal(node.local_pose, pose)
        np.testing.assert_array_equal(node.gravity_alignment, grav)
        assert node.points.shape == dec.shape
        assert node.points.tobytes() == dec.tobytes()  # bit-exact decode
    # Decoded clouds are the inputs rounded to the 1 mm raster.
    perm = compress(cloud0)[2]
    np.testing.assert_allclose(st.nodes[0].points, cloud0[perm], rtol=0, atol=6e-4)


def test_legacy_costs_and_unpacked_cells(csm, tmp_path):
    """Grid2D(proto) loads 0/0 correspondence costs as kMin/kMaxCorrespondenceCost
    (grid_2d.cc:22-44); cells may be written one per key."""
    cells = np.array([[0, 1, 65535], [32768, 7, 0]], np.uint16)
    path = tmp_path / "legacy.pbstream"
    write_stream(path, [submap2d_msg(0, 0, [0, 0, 0, 1, 0, 0, 0],
                                     grid2d(0.05, 1.0, 1.0, cells, packed=False))])
    st = csm.read_pbstream(path)
    g = st.submaps[0].grid
    np.testing.assert_array_equal(g.cells, cells)
    assert g.min_correspondence_cost == csm.K_MIN_CORRESPONDENCE_COST
    assert g.max_correspondence_cost == csm.K_MAX_CORRESPONDENCE_COST


def test_empty_stream(csm, tmp_path):
    path = tmp_path / "empty.pbstream"
    write_stream(path, [])
    st = csm.read_pbstream(path)
    assert st.submaps == [] and st.nodes == []


@pytest.mark.parametrize("case", ["magic", "no_header", "truncated", "cell_range", "cell_count",
                                  "cost_order", "missing", "garbage", "num_points", "inflate_limit"])
def test_malformed_streams_fail(csm, tmp_path, case, monkeypatch):
    path = tmp_path / f"{case}.pbstream"
    cells = np.zeros((2, 2), np.uint16)
    good = submap2d_msg(0, 0, [0, 0, 0, 1, 0, 0, 0], grid2d(0.05, 1.0, 1.0, cells))
    if case == "magic":
        write_stream(path, [good], magic=MAGIC ^ 1)
    elif case == "no_header":
        write_stream(path, [], header=None)
    elif case == "truncated":
        write_stream(path, [good])
        data = path.read_bytes()
        path.write_bytes(data[:-5])
    elif case == "cell_range":
        body = grid2d(0.05, 1.0, 1.0, cells)
        body = body.replace(f_packed(2, [0, 0, 0, 0]), f_packed(2, [0, 70000, 0, 0]))
        write_stream(path, [submap2d_msg(0, 0, [0, 0, 0, 1, 0, 0, 0], body)])
    elif case == "cell_count":
        write_stream(path, [submap2d_msg(0, 0, [0, 0, 0, 1, 0, 0, 0],
                                         grid2d(0.05, 1.0, 1.0, cells).replace(
                                             f_packed(2, [0, 0, 0, 0]), f_packed(2, [0, 0, 0])))])
    elif case == "cost_order":
        write_stream(path, [submap2d_msg(0, 0, [0, 0, 0, 1, 0, 0, 0],
                                         grid2d(0.05, 1.0, 1.0, cells, 0.9, 0.1))])
    elif case == "missing":
        path = tmp_path / "does_not_exist.pbstream"
    elif case == "garbage":
        with open(path, "wb") as f:
            f.write(struct.pack("<Q", MAGIC))
            f.write(struct.pack("<Q", 4))
            f.write(b"\x1f\x8b\x00\x00")
    elif case == "num_points":
        # A node cloud declaring 2^31 - 1 points over a few words of data is
        # rejected before the loader allocates for the declared count.
        data, _, _ = compress(np.array([[0.1, 0.2, 0.0]], np.float32))
        cloud = f_int(1, 2**31 - 1) + f_packed(3, data)
        nd = (f_int(1, 0) + f_msg(2, quaternion([1, 0, 0, 0])) + f_msg(3, cloud) +
              f_msg(7, rigid3d([0, 0, 0, 1, 0, 0, 0])))
        write_stream(path, [f_msg(4, f_msg(1, f_int(1, 0) + f_int(2, 0)) + f_msg(5, nd))])
    elif case == "inflate_limit":
        # A message that inflates past the per-message limit (lowered here;
        # 256 MiB by default) fails instead of filling host memory.
        monkeypatch.setenv("CSM_PBSTREAM_MAX_MESSAGE_BYTES", "4096")
        big = submap2d_msg(0, 0, [0, 0, 0, 1, 0, 0, 0],
                           grid2d(0.05, 1.0, 1.0, np.zeros((64, 64), np.uint16)))
        assert len(big) > 4096
        write_stream(path, [big])
    with pytest.raises(csm.CsmError):
        csm.read_pbstream(path)


@pytest.mark.gpu
def test_stream_loaded_submap_matches_oracle(csm, oracle, tmp_path):
    """A submap grid and a node cloud that went through a pbstream feed the GPU
    MatchFullSubmap; the result has parity with the oracle on the same
    (decoded) inputs."""
    from test_fast2d_gpu import assert_fast_parity, full_submap_center
    world = csm.SyntheticWorld2D(num_nodes=16, num_submaps=2, decimate_to=200, seed=4242)
    g = world.grid(1)
    node = int(world.submap_nodes[1])
    cloud = np.asarray(world.cloud(node), np.float32)
    n_msg, decoded = node_msg(0, node, 1, [0, 0, 0, 1, 0, 0, 0], [1, 0, 0, 0], cloud)
    path = tmp_path / "world.pbstream"
    write_stream(path, [submap2d_msg(0, 1, [0, 0, 0, 1, 0, 0, 0],
                                     grid2d(g.resolution, g.max_x, g.max_y, g.cells,
                                            g.min_correspondence_cost,
                                            g.max_correspondence_cost)), n_msg])
    st = csm.read_pbstream(path)
    lg = st.submaps[0].grid
    np.testing.assert_array_equal(lg.cells, g.cells)
    pts = st.nodes[0].points
    assert pts.tobytes() == decoded.tobytes()
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30), 7)
    gpu = csm.FastCorrelativeScanMatcher2D(lg, opts).MatchFullSubmap(pts, 0.55)
    limits = (lg.resolution, lg.max_x, lg.max_y)
    om = oracle.fast2d(limits, lg.cells, 7.0, math.radians(30), 7)
    ref = om.match_full_submap(pts, 0.55)
    assert_fast_parity(oracle, om, limits, lg.cells, gpu, ref, True,
                       full_submap_center(limits, lg.cells), pts)
    assert gpu[0]


# ---- 3D: Submap3D HybridGrids, node clouds and histograms -------------------
def f_sint_packed(f, vals):
    return f_msg(f, b"".join(varint((int(v) << 1) ^ (int(v) >> 31)) for v in vals))


def f_floats_packed(f, vals):
    return f_msg(f, np.asarray(vals, "<f4").tobytes())


def hybrid_grid(resolution, idx, values):
    idx = np.asarray(idx, np.int64).reshape(-1, 3)
    return (f_flt(1, resolution) + f_sint_packed(3, idx[:, 0]) + f_sint_packed(4, idx[:, 1]) +
            f_sint_packed(5, idx[:, 2]) + f_packed(6, values))


def submap3d_full_msg(traj, index, pose7, high, low, hist, finished=True):
    sid = f_int(1, traj) + f_int(2, index)
    s3d = (f_msg(1, rigid3d(pose7)) + f_int(2, 20) + f_int(3, int(finished)) +
           f_msg(4, hybrid_grid(*high)) + f_msg(5, hybrid_grid(*low)) + f_floats_packed(6, hist))
    return f_msg(3, f_msg(1, sid) + f_msg(3, s3d))


def node3d_msg(traj, index, gravity, filtered, high, low, hist):
    parts = []
    decoded = []
    for fld, pts in ((3, filtered), (4, high), (5, low)):
        data, dec, _ = compress(pts)
        parts.append(f_msg(fld, f_int(1, len(pts)) + f_packed(3, data)))
        decoded.append(dec)
    nd = (f_int(1, 1) + f_msg(2, quaternion(gravity)) + b"".join(parts) +
          f_floats_packed(6, hist) + f_msg(7, rigid3d([0, 0, 0, 1, 0, 0, 0])))
    return f_msg(4, f_msg(1, f_int(1, traj) + f_int(2, index)) + f_msg(5, nd)), decoded


def loaded_value(v):
    """ProbabilityToValue(ValueToProbability(v)) in float32
    (probability_values.cc:27-49, probability_values.h:32-93)."""
    f = np.float32
    v = np.asarray(v, np.int64)
    kmin = f(0.1)
    kmax = f(f(1.0) - kmin)
    scale = f((kmax - kmin) / f(32766.0))
    low = (v & 0x7FFF).astype(np.float32)
    p = np.where((v & 0x7FFF) == 0, kmin, (low * scale + f(kmin - scale)).astype(np.float32))
    c = np.clip(p.astype(np.float32), kmin, kmax)
    x = ((c - kmin) * f(f(32766.0) / f(kmax - kmin))).astype(np.float32)
    return (np.floor(x.astype(np.float64) + 0.5) + 1).astype(np.uint16)


def test_round_trip_3d(csm, tmp_path):
    rng = np.random.default_rng(11)
    hi_idx = rng.integers(-300, 300, size=(400, 3))
    lo_idx = rng.integers(-60, 60, size=(90, 3))
    hi_val = rng.integers(1, 32768, size=400)
    hi_val[:4] = [0, 32768 + 5, 65535, 32767]  # unknown and update-marked values
    lo_val = rng.integers(1, 32768, size=90)
    hist = rng.uniform(0, 50, 120).astype(np.float32)
    pose = [0.5, -1.0, 2.0, math.cos(0.3), 0.0, math.sin(0.3), 0.0]
    sub = submap3d_full_msg(2, 7, pose, (0.1, hi_idx, hi_val), (0.45, lo_idx, lo_val), hist)
    clouds = [rng.uniform(-20, 20, size=(k, 3)).astype(np.float32) for k in (300, 150, 60)]
    nhist = rng.uniform(0, 5, 120).astype(np.float32)
    nd, decoded = node3d_msg(2, 9, [1, 0, 0, 0], *clouds, nhist)
    path = tmp_path / "state3d.pbstream"
    write_stream(path, [sub, nd])
    st = csm.read_pbstream(path)
    assert st.submaps == [] and len(st.submaps3d) == 1 and len(st.nodes) == 1
    s3 = st.submaps3d[0]
    assert (s3.trajectory_id, s3.submap_index, s3.finished) == (2, 7, True)
    np.testing.assert_array_equal(s3.local_pose, pose)
    for (res, idx, val), (eres, eidx, evals) in ((s3.high_resolution_hybrid_grid, (0.1, hi_idx, hi_val)),
                                                 (s3.low_resolution_hybrid_grid, (0.45, lo_idx, lo_val))):
        assert res == float(np.float32(eres))
        np.testing.assert_array_equal(idx, eidx)
        np.testing.assert_array_equal(val, loaded_value(evals))
    # Known values round-trip unchanged; 0 loads as 1, the marker is dropped.
    assert list(s3.high_resolution_hybrid_grid[2][:4]) == [1, 5, 32767, 32767]
    np.testing.assert_array_equal(loaded_value(np.arange(1, 32768)), np.arange(1, 32768))
    np.testing.assert_array_equal(s3.rotational_scan_matcher_histogram, hist)
    n = st.nodes[0]
    for got, dec in zip((n.points, n.high_resolution_points, n.low_resolution_points), decoded):
        assert got.tobytes() == dec.tobytes()
    np.testing.assert_array_equal(n.rotational_scan_matcher_histogram, nhist)


def test_hybrid_grid_length_mismatch_fails(csm, tmp_path):
    """HybridGrid(proto) CHECKs equal index and value counts (hybrid_grid.h:475-477)."""
    body = (f_flt(1, 0.1) + f_sint_packed(3, [1, 2]) + f_sint_packed(4, [1, 2]) +
            f_sint_packed(5, [1]) + f_packed(6, [5, 6]))
    sub = f_msg(3, f_msg(1, f_int(1, 0)) + f_msg(3, f_msg(4, body)))
    path = tmp_path / "bad3d.pbstream"
    write_stream(path, [sub])
    with pytest.raises(csm.CsmError):
        csm.read_pbstream(path)


@pytest.mark.gpu
def test_stream_loaded_3d_world_matches_direct(csm):
    """C5-shaped submaps and nodes written to a pbstream and read back give the
    same FastCorrelativeScanMatcher3D results as the in-memory grids and
    histograms (both sides use the 1 mm-decoded clouds)."""
    import tempfile
    import os
    w = csm.SyntheticWorld3D(num_nodes=12, num_submaps=2, seed=77)
    msgs = []
    for s in range(w.num_submaps):
        msgs.append(submap3d_full_msg(0, s, [0, 0, 0, 1, 0, 0, 0],
                                      (w.high_resolution, *w.high_cells[s]),
                                      (w.low_resolution, *w.low_cells[s]), w.submap_hist[s]))
    decoded_nodes = []
    for i in range(w.num_nodes):
        m, dec = node3d_msg(0, i, w.node(i).gravity_alignment, w.raw[i], w.high[i], w.low[i],
                            w.node_hist[i])
        msgs.append(m)
        decoded_nodes.append(dec)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "world3d.pbstream")
        write_stream(path, msgs)
        st = csm.read_pbstream(path)
    opts = csm.FastCorrelativeScanMatcherOptions3D()
    direct, loaded = [], []
    for s in range(w.num_submaps):
        direct.append(csm.FastCorrelativeScanMatcher3D(
            csm.HybridGrid(w.high_resolution, *w.high_cells[s]),
            csm.HybridGrid(w.low_resolution, *w.low_cells[s]), w.submap_hist[s], opts))
        s3 = st.submaps3d[s]
        loaded.append(csm.FastCorrelativeScanMatcher3D(
            csm.HybridGrid(*s3.high_resolution_hybrid_grid),
            csm.HybridGrid(*s3.low_resolution_hybrid_grid),
            s3.rotational_scan_matcher_histogram, opts))
    nodes_direct = [csm.NodeData3D(dec[1], dec[2], w.node_hist[i], w.node(i).gravity_alignment)
                    for i, dec in enumerate(decoded_nodes)]
    nodes_loaded = [csm.NodeData3D(n.high_resolution_points, n.low_resolution_points,
                                   n.rotational_scan_matcher_histogram, tuple(n.gravity_alignment))
                    for n in st.nodes]
    sub_idx = [s for s in range(w.num_submaps) for _ in range(w.num_nodes)]
    node_idx = [i for _ in range(w.num_submaps) for i in range(w.num_nodes)]
    pairs = csm.make_pairs_3d(sub_idx, node_idx, 0.3)
    a = csm.match_batch_3d(direct, nodes_direct, pairs)
    b = csm.match_batch_3d(loaded, nodes_loaded, pairs)
    for name in a.dtype.names:
        np.testing.assert_array_equal(a[name], b[name])
    assert (a["status"] == 0).sum() >= 2
