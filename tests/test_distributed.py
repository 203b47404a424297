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
