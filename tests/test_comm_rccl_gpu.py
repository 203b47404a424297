"""comm.cc's RCCL code paths with 2 and 3 ranks on the one-GPU box.

Real RCCL cannot make a multi-rank world on one GPU, so CSM_RCCL_LIB points
comm.cc's dlopen at tests/comm_standin/librccl_standin.so, a test-only
stand-in with the same entry points over TCP with host staging. What runs is
the library's own RCCL path: csm_comm_create_rccl (world-size check, count
buffer), RcclGather (the count AllGather, the root's staging agreement, the
grouped Send / Recv of the exact sizes into d_recv, the copy-out in rank
order) and RcclAllreduce (64-word chunks), with the payloads every rank
hands over checked on rank 0.
"""
import multiprocessing as mp
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

STANDIN = os.path.join(ROOT, "tests", "comm_standin", "librccl_standin.so")


def _blob(rank, k, n):
    return ((np.arange(n, dtype=np.int64) * (rank + 3) + 7 * k + rank) % 251).astype(np.uint8).tobytes()


def _rank(rank, world, uid_q, out_q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_package
    csm = load_package()
    try:
        ctx = csm.Context(0)
        if rank == 0:
            uid = csm.Comm.unique_id()
            for _ in range(world - 1):
                uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=90)
        comm = csm.Comm.rccl(ctx, rank, world, uid)
        res = {"rank": rank, "size": comm.size}
        # Gathers of uneven sizes: rank 0 sends nothing in the first, one rank
        # nothing in the second, then payloads that regrow the root's staging.
        sizes = [[0, 3000, 17][r % 3] for r in range(world)], \
                [[512, 0, 4096][r % 3] for r in range(world)], \
                [200000 + 13 * r for r in range(world)]
        res["gathers"] = [comm.gather(_blob(rank, k, s[rank])) for k, s in enumerate(sizes)]
        v = np.arange(150, dtype=np.int64) * (rank + 1) - 40 * rank
        res["sum"] = comm.allreduce(v, csm.REDUCE_SUM).tolist()
        res["max"] = comm.allreduce(v, csm.REDUCE_MAX).tolist()
        comm.barrier()
        comm.close()
        out_q.put(res)
    except Exception as e:  # reported to the parent, which fails the test
        out_q.put({"rank": rank, "error": repr(e)})


@pytest.mark.parametrize("world", [2, 3])
def test_rccl_gather_and_allreduce_multi_rank(world):
    import subprocess
    subprocess.check_call(["make", "-s", "-C", os.path.dirname(STANDIN)])
    os.environ["CSM_RCCL_LIB"] = STANDIN  # inherited by the spawned ranks
    try:
        ctx = mp.get_context("spawn")
        uid_q, out_q = ctx.Queue(), ctx.Queue()
        procs = [ctx.Process(target=_rank, args=(r, world, uid_q, out_q)) for r in range(world)]
        for p in procs:
            p.start()
        outs = {}
        for _ in range(world):
            o = out_q.get(timeout=100)
            outs[o["rank"]] = o
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        os.environ.pop("CSM_RCCL_LIB", None)
    for r, o in outs.items():
        assert "error" not in o, o
        assert o["size"] == world
    sizes = [[[0, 3000, 17][r % 3] for r in range(world)],
             [[512, 0, 4096][r % 3] for r in range(world)],
             [200000 + 13 * r for r in range(world)]]
    for k, s in enumerate(sizes):
        got = outs[0]["gathers"][k]
        assert [len(b) for b in got] == s
        for r in range(world):
            assert got[r] == _blob(r, k, s[r]), (k, r)
        for r in range(1, world):
            assert outs[r]["gathers"][k] is None
    vs = [np.arange(150, dtype=np.int64) * (r + 1) - 40 * r for r in range(world)]
    for r in range(world):
        assert outs[r]["sum"] == np.sum(vs, axis=0).tolist()
        assert outs[r]["max"] == np.max(vs, axis=0).tolist()


def _real_rank(out_q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_package
    csm = load_package()
    try:
        ctx = csm.Context(0)
        comm = csm.Comm.rccl(ctx, 0, 1, csm.Comm.unique_id())
        res = {"size": comm.size, "rank": comm.rank,
               "gather": [len(b) for b in comm.gather(b"\x05" * 1234)],
               "sum": comm.allreduce(np.arange(6, dtype=np.int64), csm.REDUCE_SUM).tolist()}
        comm.barrier()
        comm.close()
        out_q.put(res)
    except Exception as e:  # reported to the parent, which fails the test
        out_q.put({"error": repr(e)})


def test_real_rccl_single_rank():
    """The installed librccl (no stand-in) through csm_comm_create_rccl:
    ncclGetUniqueId, ncclCommInitRank with the 128-byte id by value, and
    ncclCommDestroy, in a world of one (RCCL refuses two ranks on one GPU,
    tools/probe_rccl_real.py; N > 1 is the driver's scaling run)."""
    assert "CSM_RCCL_LIB" not in os.environ
    ctx = mp.get_context("spawn")
    out_q = ctx.Queue()
    p = ctx.Process(target=_real_rank, args=(out_q,))
    p.start()
    o = out_q.get(timeout=100)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert "error" not in o, o
    assert o == {"size": 1, "rank": 0, "gather": [1234], "sum": list(range(6))}
