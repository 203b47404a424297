"""Real RCCL (no stand-in) through the library's csm_comm on the one-GPU box:
W ranks on device 0, each through the unique id, init, a gather of uneven
payloads and an all-reduce. RCCL may refuse two ranks on one GPU; the
probe reports what happens per rank.

    python tools/probe_rccl_real.py W"""
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, uid_q, out_q):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_package
    import numpy as np
    csm = load_package()
    try:
        ctx = csm.Context(0)
        if rank == 0:
            uid = csm.Comm.unique_id()
            for _ in range(world - 1):
                uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        comm = csm.Comm.rccl(ctx, rank, world, uid)
        res = {"rank": rank, "size": comm.size}
        g = comm.gather(bytes([rank + 1]) * (1000 + 7 * rank))
        res["gather"] = None if g is None else [len(b) for b in g]
        v = np.arange(8, dtype=np.int64) * (rank + 1)
        res["sum"] = comm.allreduce(v).tolist()
        comm.barrier()
        comm.close()
        out_q.put(res)
    except Exception as e:  # noqa: BLE001
        out_q.put({"rank": rank, "error": repr(e)})


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    uid_q, out_q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, uid_q, out_q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = []
    for _ in range(world):
        try:
            outs.append(out_q.get(timeout=90))
        except Exception as e:  # noqa: BLE001
            outs.append({"error": "no answer: " + repr(e)})
    for p in procs:
        p.join(timeout=30)
        if p.exitcode is None:
            p.kill()
    print(json.dumps({"world": world, "ranks": outs, "exitcodes": [p.exitcode for p in procs]}))


if __name__ == "__main__":
    main()
