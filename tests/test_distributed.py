"""Multi-rank path on CPU (gloo, world_size 2): submap sharding, the rank-0
gather of accepted constraints in submission order (constraint_builder_2d.cc
:285-288), and max-over-ranks timing. The same functions run over RCCL in
bench.py; only the tensor device differs."""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, load_package


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_submaps(csm):
    d = __import__("cartographer_amd.distributed", fromlist=["x"])
    assert d.shard_submaps(10, 1, 4) == [1, 5, 9]
    assert d.shard_submaps(100, 1, 2, per_rank=50) == list(range(50, 100))
    shards = [d.shard_submaps(23, r, 3) for r in range(3)]
    assert sorted(sum(shards, [])) == list(range(23))
    with pytest.raises(ValueError):
        d.shard_submaps(10, 3, 3)
    with pytest.raises(ValueError):
        d.shard_submaps(10, 0, 3, per_rank=4)


def _fake_results(csm, n, seed):
    rng = np.random.default_rng(seed)
    res = np.zeros(n, csm.RESULT_DTYPE)
    res["status"] = np.where(rng.random(n) < 0.4, 0, 1)
    res["score"] = rng.random(n).astype(np.float32)
    res["x"], res["y"], res["theta"] = rng.normal(size=(3, n))
    return res


def _worker(rank, world_size, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        csm = load_package()
        import importlib
        d = importlib.import_module("cartographer_amd.distributed")
        nodes, per_rank = 7, 3
        mine = d.shard_submaps(per_rank * world_size, rank, world_size, per_rank)
        sub = np.repeat(np.asarray(mine, np.int64), nodes)
        node = np.tile(np.arange(nodes), per_rank)
        submission = rank * len(sub) + np.arange(len(sub))
        res = _fake_results(csm, len(sub), seed=rank)
        rec = d.make_records(res, submission, sub, node)
        got = d.gather_records(rec, dist, rank, world_size)
        t = d.max_over_ranks(float(rank + 1), dist)
        if rank == 0:
            np.save(os.path.join(out_dir, "gathered.npy"), got)
            np.save(os.path.join(out_dir, "tmax.npy"), np.array([t]))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_gather_two_ranks_gloo(csm, tmp_path):
    import torch.multiprocessing as mp
    world_size = 2
    mp.spawn(_worker, args=(world_size, _free_port(), str(tmp_path)), nprocs=world_size,
             join=True)
    got = np.load(tmp_path / "gathered.npy")
    assert float(np.load(tmp_path / "tmax.npy")[0]) == 2.0
    # Expected: every rank's accepted rows, in global submission order.
    d = __import__("cartographer_amd.distributed", fromlist=["x"])
    want = []
    for r in range(world_size):
        mine = d.shard_submaps(3 * world_size, r, world_size, 3)
        sub = np.repeat(np.asarray(mine, np.int64), 7)
        node = np.tile(np.arange(7), 3)
        res = _fake_results(csm, len(sub), seed=r)
        want.append(d.make_records(res, r * len(sub) + np.arange(len(sub)), sub, node))
    want = np.concatenate(want)
    assert np.array_equal(got, want)
    assert np.all(np.diff(got[:, 0]) > 0)
    assert set(got[:, 2].astype(int)) <= set(range(6))


# ---------------------------------------------------------------- 3D (C5) --
def _fake_results_3d(csm, n, seed, accept=0.4):
    rng = np.random.default_rng(seed)
    res = np.zeros(n, csm.RESULT3_DTYPE)
    res["status"] = np.where(rng.random(n) < accept, 0, 1)
    res["score"] = rng.random(n).astype(np.float32)
    res["t"] = rng.normal(size=(n, 3))
    q = rng.normal(size=(n, 4))
    res["q"] = q / np.linalg.norm(q, axis=1, keepdims=True)
    return res


def _worker3d(rank, world_size, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world_size)
    try:
        csm = load_package()
        import importlib
        d = importlib.import_module("cartographer_amd.distributed")
        nodes, per_rank = 5, 2
        sub = np.repeat(np.arange(per_rank, dtype=np.int64) + rank * per_rank, nodes)
        node = np.tile(np.arange(nodes), per_rank)
        submission = rank * len(sub) + np.arange(len(sub))
        # Rank 1 accepts nothing: the gather pads and still agrees on width.
        res = _fake_results_3d(csm, len(sub), seed=rank, accept=0.5 if rank == 0 else 0.0)
        got = d.gather_records(d.make_records_3d(res, submission, sub, node), dist, rank,
                               world_size)
        if rank == 0:
            np.save(os.path.join(out_dir, "gathered3d.npy"), got)
    finally:
        dist.destroy_process_group()


def test_gather_3d_two_ranks_gloo(csm, tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker3d, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    got = np.load(tmp_path / "gathered3d.npy")
    d = __import__("cartographer_amd.distributed", fromlist=["x"])
    res = _fake_results_3d(csm, 10, seed=0, accept=0.5)
    sub = np.repeat(np.arange(2, dtype=np.int64), 5)
    want = d.make_records_3d(res, np.arange(10), sub, np.tile(np.arange(5), 2))
    assert got.shape[1] == d.RECORD3_WIDTH == 13
    assert np.array_equal(got, want)
    ok = res["status"] == 0
    assert np.allclose(got[:, 5:8], res["t"][ok]) and np.allclose(got[:, 8:12], res["q"][ok])


def test_synthetic_3d_shard_is_the_full_worlds_submaps(csm):
    """bench.py's C5 sharding: a rank building submaps [b, b + k) of the world
    gets exactly those submaps (grids, histograms, centre nodes) and the same
    nodes as a rank building the whole world."""
    kw = dict(num_nodes=8, num_submaps=4, seed=11, scans_per_submap=3, azimuths=240)
    full = csm.SyntheticWorld3D(**kw)
    part = csm.SyntheticWorld3D(submap_range=(2, 2), **kw)
    assert part.num_submaps == 2 and list(part.submap_ids) == [2, 3]
    assert np.array_equal(part.submap_nodes, full.submap_nodes[2:4])
    for j in range(2):
        for a, b in ((full.high_cells[2 + j], part.high_cells[j]),
                     (full.low_cells[2 + j], part.low_cells[j])):
            assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
        assert np.array_equal(full.submap_hist[2 + j], part.submap_hist[j])
    for i in range(8):
        assert np.array_equal(full.high[i], part.high[i])


# ---- the C++ sharded ConstraintBuilder2D over the C-ABI communicator -------

DIST_SRC = os.path.join(ROOT, "tests", "cpp", "distributed_builder_test.cc")
DIST_BIN = os.path.join(ROOT, "tests", "cpp", "_build", "distributed_builder_test")


def _build_dist():
    import subprocess
    os.makedirs(os.path.dirname(DIST_BIN), exist_ok=True)
    libdir = os.path.join(ROOT, "cartographer-1_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror",
                           "-I", os.path.join(ROOT, "include"), DIST_SRC, "-o", DIST_BIN,
                           "-L", libdir, "-lcsm_amd", "-Wl,-rpath," + libdir])


@pytest.mark.parametrize("world", [2, 3])
def test_cpp_record_gather_tcp(csm, world):
    """GatherConstraintRecords over the TCP transport, <world> forked ranks:
    rank 0 gets every rank's records in slot (submission) order."""
    import subprocess
    _build_dist()
    out = subprocess.run([DIST_BIN, "gather", str(world), str(_free_port())],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "gather OK" in out.stdout


@pytest.mark.parametrize("world", [2, 3])
def test_cpp_record_gather_3d_tcp(csm, world):
    """GatherRecords<ConstraintRecord3D> (the sharded ConstraintBuilder3D's
    hand-off) over TCP: rank 0 gets every rank's 3D records in slot order."""
    import subprocess
    _build_dist()
    out = subprocess.run([DIST_BIN, "gather3d", str(world), str(_free_port())],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "gather3d OK" in out.stdout


@pytest.mark.parametrize("world", [2, 3])
def test_cpp_claim_loop_tcp(csm, world):
    """Sharding::kClaim's queue without a device: <world> forked ranks claim
    the chunks of three flushes (ClaimChunks groups pending pairs by submap)
    through csm_comm_fetch_add; rank 0 receives every pair exactly once, in
    submission order, each from the chunk that holds its submap."""
    import subprocess
    _build_dist()
    out = subprocess.run([DIST_BIN, "claimloop", str(world), str(_free_port())],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "claimloop OK" in out.stdout


def test_cpp_diverging_submissions_abort(csm):
    """A rank that submits a different pair sequence makes WhenDone abort on
    every rank (CheckSameSubmissions), instead of rank 0 mixing constraints."""
    import subprocess
    _build_dist()
    out = subprocess.run([DIST_BIN, "diverge", "3", str(_free_port())],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "diverge OK" in out.stdout
    assert out.stderr.count("ranks submitted different pair sequences") == 3, out.stderr


STANDIN = os.path.join(ROOT, "tests", "comm_standin", "librccl_standin.so")


def _build_standin():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.dirname(STANDIN)])


def _run_ranks(mode, world, transport="tcp", tmp_path=None):
    """Runs <world> ranks of the C++ test. transport "rccl": the library's
    RCCL code path (csm_comm_create_rccl, RcclGather / RcclAllreduce) over the
    test stand-in library (tests/comm_standin), since one GPU box cannot make
    a multi-rank RCCL world."""
    import subprocess
    port = str(_free_port())
    env = dict(os.environ)
    if transport == "rccl":
        _build_standin()
        env.update(CSM_TEST_COMM="rccl", CSM_RCCL_LIB=STANDIN,
                   CSM_TEST_RCCL_ID=str(tmp_path / "rccl_id"))
    procs = [subprocess.Popen([DIST_BIN, mode, str(r), str(world), port], stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True, env=env) for r in range(world)]
    outs = [p.communicate(timeout=180) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
        if transport == "rccl":
            assert "transport rccl" in e, e
    if mode.endswith("-claim"):
        claimed = [int(l.split()[1]) for _, e in outs for l in e.splitlines() if l.startswith("claimed ")]
        assert len(claimed) == world and sum(claimed) > 0, [e for _, e in outs]
    return outs


@pytest.mark.gpu
@pytest.mark.parametrize("mode,world,transport", [("builder3d", 2, "tcp"),
                                                  ("builder3d-claim", 2, "tcp"),
                                                  ("builder3d", 3, "rccl")])
def test_cpp_sharded_builder_3d_matches_single_rank(csm, mode, world, transport, tmp_path):
    """The C++ ConstraintBuilder3D sharded over 2 ranks (two processes on the
    one GPU, TCP transport; by submap owner, or by chunks claimed through
    csm_comm_fetch_add) delivers on rank 0 what the single-rank builder
    delivers: same constraints in submission order, same summed counters and
    the same score metric lists (constraint_builder_3d.cc:200-305)."""
    import subprocess
    _build_dist()
    single = subprocess.run([DIST_BIN, "builder3d", "0", "1", "0"], capture_output=True, text=True,
                            timeout=120)
    assert single.returncode == 0, single.stderr
    outs = _run_ranks(mode, world, transport, tmp_path)
    lines = single.stdout.strip().splitlines()
    assert sum(1 for l in lines if l.startswith("c ")) >= 4, single.stdout
    assert any(l.startswith("c ") and l.endswith(" 1") for l in lines), single.stdout  # a global one
    assert outs[0][0].strip().splitlines() == lines
    assert all(o.strip() == "" for o, _ in outs[1:])


@pytest.mark.gpu
@pytest.mark.parametrize("mode,world,transport", [("builder", 2, "tcp"), ("builder-claim", 2, "tcp"),
                                                  ("builder-claim", 3, "tcp"),
                                                  ("builder", 2, "rccl"),
                                                  ("builder-claim", 3, "rccl")])
def test_cpp_sharded_builder_matches_single_rank(csm, mode, world, transport, tmp_path):
    """The C++ ConstraintBuilder2D sharded over 2-3 ranks (processes on the
    one GPU, TCP transport; Sharding::kStatic by submap owner, or
    Sharding::kClaim with one-submap chunks claimed dynamically) delivers on
    rank 0 exactly what the single-rank builder delivers: same constraints,
    same (submission) order, same summed counters."""
    import subprocess
    _build_dist()
    single = subprocess.run([DIST_BIN, "builder", "0", "1", "0"], capture_output=True, text=True,
                            timeout=120)
    assert single.returncode == 0, single.stderr
    outs = _run_ranks(mode, world, transport, tmp_path)
    lines = single.stdout.strip().splitlines()
    assert sum(1 for l in lines if l.startswith("c ")) >= 5, single.stdout
    assert outs[0][0].strip().splitlines() == lines
    assert all(o.strip() == "" for o, _ in outs[1:])
