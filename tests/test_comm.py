"""The C-ABI communicator (csm_comm_*, cartographer-1_amd/csrc/comm.cc) over
its TCP transport: world_size 2 and 3 host processes gather their accepted
constraint records to rank 0, which restores ConstraintBuilder2D::WhenDone's
submission order (constraint_builder_2d.cc:279-300). CPU only; the RCCL
transport of the same calls runs in bench.py at N > 1 and in
test_distributed_gpu (world_size 1 on the GPU box)."""
import multiprocessing as mp
import os
import socket
import sys
import traceback

import numpy as np
import pytest

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _records(rank, world):
    # Rank r owns submaps r, r + world, ...: its records carry the global
    # submission indices of its pairs (interleaved across ranks).
    rng = np.random.RandomState(100 + rank)
    sub = np.arange(rank, 40, world)
    n = len(sub) * 3
    rec = np.zeros((n, 9))
    rec[:, 0] = np.sort(rng.choice(np.arange(rank, 400, world), n, replace=False))
    rec[:, 2] = np.repeat(sub, 3)
    rec[:, 4] = rng.randint(0, 50, n)
    rec[:, 5:8] = rng.randn(n, 3)
    rec[:, 8] = rng.rand(n)
    if rank == world - 1:
        rec = rec[:0]  # a rank with nothing accepted
    return rec


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        import __graft_entry__ as ge
        csm = ge._load_package()
        from cartographer_amd import distributed as cdist
        comm = csm.Comm.tcp(rank, world, "127.0.0.1", port)
        assert (comm.rank, comm.size) == (rank, world)
        out = cdist.gather_records_comm(_records(rank, world), comm)
        s = comm.allreduce([rank + 1, 10 * rank], csm.REDUCE_SUM)
        m = comm.allreduce([rank, -rank], csm.REDUCE_MAX)
        comm.barrier()
        blobs = comm.gather(bytes([rank]) * (rank + 2))
        comm.close()
        q.put((rank, None if out is None else out.tolist(), s.tolist(), m.tolist(),
               blobs, None))
    except Exception:
        q.put((rank, None, None, None, None, traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_tcp_gather_restores_submission_order(csm, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, out, s, m, blobs, err = q.get(timeout=120)
        assert err is None, err
        got[rank] = (out, s, m, blobs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect = np.concatenate([_records(r, world) for r in range(world)])
    expect = expect[np.argsort(expect[:, 0], kind="stable")]
    assert np.array_equal(np.asarray(got[0][0]).reshape(-1, 9), expect)
    assert np.all(np.diff(expect[:, 0]) > 0)
    for r in range(1, world):
        assert got[r][0] is None and got[r][3] is None
    for r in range(world):
        assert got[r][1] == [sum(k + 1 for k in range(world)), sum(10 * k for k in range(world))]
        assert got[r][2] == [world - 1, 0]
    assert got[0][3] == [bytes([k]) * (k + 2) for k in range(world)]


def test_single_rank_comm(csm):
    comm = csm.Comm.tcp(0, 1, "127.0.0.1", _free_port())
    assert comm.gather(b"abc") == [b"abc"]
    assert comm.allreduce([3, 4]).tolist() == [3, 4]
    comm.close()


def test_comm_rejects_bad_arguments(csm):
    lib = csm.load_library()
    import ctypes as C
    h = C.c_void_p()
    assert lib.csm_comm_create_tcp(2, 2, b"127.0.0.1", 1234, C.byref(h)) == csm.CSM_EINVAL
    assert lib.csm_comm_create_tcp(0, 0, b"127.0.0.1", 1234, C.byref(h)) == csm.CSM_EINVAL
    assert lib.csm_comm_create_tcp(1, 2, None, 1234, C.byref(h)) == csm.CSM_EINVAL
    assert lib.csm_comm_gather(None, None, 0, None) == csm.CSM_EINVAL


@pytest.mark.gpu
def test_rccl_single_rank(csm):
    """The RCCL transport on the box's one GPU: loading librccl through
    dlopen and ncclCommInitRank at world_size 1 (the collectives themselves
    short-circuit at one rank; N > 1 runs them in bench.py)."""
    ctx = csm.Context(0)
    comm = csm.Comm.rccl(ctx, 0, 1, csm.Comm.unique_id())
    assert (comm.rank, comm.size) == (0, 1)
    assert comm.gather(b"\x01\x02\x03") == [b"\x01\x02\x03"]
    assert comm.allreduce([5, -2], csm.REDUCE_MAX).tolist() == [5, -2]
    comm.barrier()
    comm.close()
