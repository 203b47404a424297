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


# ---- dynamic work claiming (csm_comm_claim_open / csm_comm_fetch_add) -------

def _chunk_cost(c):
    # Deliberately skewed per-chunk costs: every 7th chunk is 8x the others.
    return 0.08 if c % 7 == 0 else 0.01


def _claim_worker(rank, world, port, q, n_chunks, skew_rank_delay):
    try:
        import time
        sys.path.insert(0, ROOT)
        import __graft_entry__ as ge
        csm = ge._load_package()
        from cartographer_amd import distributed as cdist
        comm = csm.Comm.tcp(rank, world, "127.0.0.1", port)
        comm.claim_open("127.0.0.1", port + 1)
        if rank == 1:
            time.sleep(skew_rank_delay)  # a rank that starts late still balances
        t0 = time.perf_counter()
        mine, recs = [], []
        while True:
            c = comm.fetch_add(7, 1)  # key 7: this sweep's queue head
            if c >= n_chunks:
                break
            time.sleep(_chunk_cost(c))
            mine.append(c)
            # Records of the chunk's pairs (3 per chunk), submission = queue order.
            r = np.zeros((3, 9))
            r[:, 0] = 3 * c + np.arange(3)
            r[:, 2] = c
            r[:, 8] = c / n_chunks
            recs.append(r)
        finish = time.perf_counter() - t0 + (skew_rank_delay if rank == 1 else 0.0)
        out = cdist.gather_records_comm(np.concatenate(recs) if recs else np.zeros((0, 9)), comm)
        other = comm.fetch_add(8, rank + 1)  # an independent key
        comm.barrier()
        comm.close()
        q.put((rank, mine, finish, None if out is None else out.tolist(), other, None))
    except Exception:
        q.put((rank, None, None, None, None, traceback.format_exc()))


def test_claiming_balances_skewed_chunks(csm):
    """Three ranks claim chunks of one queue through the rank-0 counter
    table (the reference's shared ThreadPool queue, thread_pool.cc:80-106):
    every chunk is taken exactly once, a rank that starts late or draws the
    costly chunks still finishes within about one chunk of the others, and
    rank 0's gathered records equal the single-rank sweep in submission
    order."""
    world, n_chunks = 3, 84
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_claim_worker, args=(r, world, port, q, n_chunks, 0.3))
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, mine, finish, out, other, err = q.get(timeout=120)
        assert err is None, err
        got[rank] = (mine, finish, out, other)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    claimed = sorted(c for r in range(world) for c in got[r][0])
    assert claimed == list(range(n_chunks))
    total = sum(_chunk_cost(c) for c in range(n_chunks))
    finishes = [got[r][1] for r in range(world)]
    # Balanced: nobody idles while work remains, so finish times differ by at
    # most one chunk (plus scheduling noise), against ~1/3 of the total each.
    assert max(finishes) - min(finishes) < 0.08 + 0.15, finishes
    assert max(finishes) < total / world + 0.3 + 0.2, (finishes, total)
    assert len(got[1][0]) < len(got[0][0]) + len(got[2][0])
    expect = np.zeros((3 * n_chunks, 9))
    expect[:, 0] = np.arange(3 * n_chunks)
    expect[:, 2] = np.repeat(np.arange(n_chunks), 3)
    expect[:, 8] = expect[:, 2] / n_chunks
    assert np.array_equal(np.asarray(got[0][2]).reshape(-1, 9), expect)
    # Key 8: each rank added rank + 1 once; the olds are the prefix sums in
    # arrival order, so they are distinct and the last one plus its delta is 6.
    olds = {r: got[r][3] for r in range(world)}
    assert len(set(olds.values())) == world and min(olds.values()) == 0
    assert max(o + r + 1 for r, o in olds.items()) == sum(range(1, world + 1))


def test_single_rank_claims(csm):
    comm = csm.Comm.tcp(0, 1, "127.0.0.1", _free_port())
    comm.claim_open()
    assert [comm.fetch_add(3) for _ in range(4)] == [0, 1, 2, 3]
    assert comm.fetch_add(3, 10) == 4 and comm.fetch_add(3, 0) == 14
    assert comm.fetch_add(-5, 2) == 0
    comm.close()


def _late_worker(rank, world, port, q, delay, timeout_ms):
    try:
        import time
        if timeout_ms:
            os.environ["CSM_COMM_TIMEOUT_MS"] = str(timeout_ms)
        sys.path.insert(0, ROOT)
        import __graft_entry__ as ge
        csm = ge._load_package()
        comm = csm.Comm.tcp(rank, world, "127.0.0.1", port)
        if rank == world - 1:
            time.sleep(delay)  # this rank's share of the search ran longer
        try:
            blobs = comm.gather(bytes([rank + 1]) * 4)
            err = None
        except Exception as e:  # noqa: BLE001
            blobs, err = None, str(e)
        q.put((rank, blobs, err, None))
        if err is None:
            comm.close()
    except Exception:
        q.put((rank, None, None, traceback.format_exc()))


@pytest.mark.parametrize("timeout_ms,delay,ok", [(0, 2.5, True), (8000, 2.5, True), (400, 2.5, False)])
def test_gather_waits_for_a_late_rank(csm, timeout_ms, delay, ok):
    """A rank that reaches the gather long after rank 0 (its search share ran
    longer) is waited for: data receives have no limit unless
    CSM_COMM_TIMEOUT_MS sets one, and then the root fails with an error
    instead of hanging."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_late_worker, args=(r, world, port, q, delay, timeout_ms))
             for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, blobs, err, tb = q.get(timeout=120)
        assert tb is None, tb
        got[rank] = (blobs, err)
    for p in procs:
        p.join(timeout=60)
    if ok:
        assert got[0] == ([bytes([1]) * 4, bytes([2]) * 4], None)
    else:
        assert got[0][0] is None and "csm_comm_gather" in got[0][1]
