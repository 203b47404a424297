"""Multi-GPU constraint search: submap sharding and the rank-0 gather.

The reference runs one ``common::Task`` per (node, submap) pair on a thread
pool (``constraint_builder_2d.cc:102-111``) and hands every accepted
constraint to the pose-graph solve through ``WhenDone`` in submission order
(``:285-288``). Here the pair queue is sharded by submap across ranks (one
process per GPU): every rank builds the pyramids of its own submaps only and
searches its pairs with no data-path collective. The single exchange is the
gather of accepted constraints to rank 0, which restores submission order
(SURVEY.md 8(e)).

Record layout (float64, one row per accepted constraint): 2D (x 9)
``submission_index, submap_trajectory, submap_index, node_trajectory,
node_index, x, y, theta, score``; 3D (x 13, ConstraintBuilder3D) the same ids,
then ``tx, ty, tz, qw, qx, qy, qz, score``.
"""

from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

RECORD_FIELDS = ("submission", "submap_traj", "submap_index", "node_traj", "node_index",
                 "x", "y", "theta", "score")
RECORD_WIDTH = len(RECORD_FIELDS)
RECORD3_FIELDS = ("submission", "submap_traj", "submap_index", "node_traj", "node_index",
                  "tx", "ty", "tz", "qw", "qx", "qy", "qz", "score")
RECORD3_WIDTH = len(RECORD3_FIELDS)


def shard_submaps(num_submaps: int, rank: int, world_size: int,
                  per_rank: Optional[int] = None) -> List[int]:
    """Submaps owned by ``rank``: contiguous blocks of ``per_rank`` when given
    (weak scaling, each rank a fixed share), else striped ``s % world_size``."""
    if not 0 <= rank < world_size:
        raise ValueError("rank out of range")
    if per_rank is not None:
        if per_rank * world_size > num_submaps:
            raise ValueError("not enough submaps for per_rank x world_size")
        return list(range(rank * per_rank, (rank + 1) * per_rank))
    return list(range(rank, num_submaps, world_size))


def make_records(results: np.ndarray, submission: np.ndarray, submap_ids: np.ndarray,
                 node_ids: np.ndarray, submap_traj: int = 0, node_traj: int = 0) -> np.ndarray:
    """Accepted rows of a ``match_batch`` result as gather records."""
    ok = results["status"] == 0
    rec = np.zeros((int(ok.sum()), RECORD_WIDTH), np.float64)
    rec[:, 0] = submission[ok]
    rec[:, 1] = submap_traj
    rec[:, 2] = submap_ids[ok]
    rec[:, 3] = node_traj
    rec[:, 4] = node_ids[ok]
    rec[:, 5] = results["x"][ok]
    rec[:, 6] = results["y"][ok]
    rec[:, 7] = results["theta"][ok]
    rec[:, 8] = results["score"][ok]
    return rec


def make_records_3d(results: np.ndarray, submission: np.ndarray, submap_ids: np.ndarray,
                    node_ids: np.ndarray, submap_traj: int = 0, node_traj: int = 0) -> np.ndarray:
    """Accepted rows of a ``match_batch_3d`` (RESULT3_DTYPE) result as records."""
    ok = results["status"] == 0
    rec = np.zeros((int(ok.sum()), RECORD3_WIDTH), np.float64)
    rec[:, 0] = submission[ok]
    rec[:, 1] = submap_traj
    rec[:, 2] = submap_ids[ok]
    rec[:, 3] = node_traj
    rec[:, 4] = node_ids[ok]
    rec[:, 5:8] = results["t"][ok]
    rec[:, 8:12] = results["q"][ok]
    rec[:, 12] = results["score"][ok]
    return rec


def gather_records(rec: np.ndarray, dist=None, rank: int = 0, world_size: int = 1,
                   device=None) -> Optional[np.ndarray]:
    """Gathers every rank's records to rank 0, sorted by submission index.

    Two collectives: an all-gather of the per-rank counts, then a gather of
    count-padded fixed-width record blocks. ``device`` is the tensor device of
    the process group's backend (``cuda:<local_rank>`` for RCCL, cpu for gloo).
    Returns the sorted records on rank 0 and None elsewhere."""
    if dist is None or world_size == 1:
        return rec[np.argsort(rec[:, 0], kind="stable")]
    import torch
    dev = torch.device("cpu") if device is None else device
    cnt = torch.tensor([rec.shape[0]], dtype=torch.int64, device=dev)
    cnts = [torch.zeros_like(cnt) for _ in range(world_size)]
    dist.all_gather(cnts, cnt)
    counts = [int(c.item()) for c in cnts]
    mx = max(max(counts), 1)
    buf = torch.zeros((mx, rec.shape[1]), dtype=torch.float64, device=dev)
    if rec.shape[0]:
        buf[:rec.shape[0]] = torch.from_numpy(np.ascontiguousarray(rec)).to(dev)
    bufs = [torch.zeros_like(buf) for _ in range(world_size)] if rank == 0 else None
    dist.gather(buf, bufs, dst=0)
    if rank != 0:
        return None
    allrec = np.concatenate([b[:c].cpu().numpy() for b, c in zip(bufs, counts)])
    return allrec[np.argsort(allrec[:, 0], kind="stable")]


def gather_records_comm(rec: np.ndarray, comm) -> Optional[np.ndarray]:
    """gather_records over the C-ABI communicator (csm_comm_gather: RCCL or
    TCP): each rank's float64 record block as one blob; rank 0 concatenates
    them in rank order and sorts by submission index. None on other ranks."""
    width = rec.shape[1]
    blobs = comm.gather(np.ascontiguousarray(rec, np.float64).tobytes())
    if blobs is None:
        return None
    allrec = np.concatenate([np.frombuffer(b, np.float64).reshape(-1, width) for b in blobs])
    return allrec[np.argsort(allrec[:, 0], kind="stable")]


def make_comm(csm, context, rank: int, world_size: int, store=None, backend: str = "rccl",
              port: int = 29611):
    """The C-ABI communicator of this rank: RCCL with rank 0's unique id
    shared through ``store`` (torch.distributed's TCPStore), or TCP to
    127.0.0.1:``port`` (host processes, gloo rehearsals)."""
    if backend == "rccl":
        if rank == 0:
            uid = csm.Comm.unique_id()
            if store is not None:
                store.set("csm_comm_id", uid)
        else:
            uid = bytes(store.get("csm_comm_id"))
        return csm.Comm.rccl(context, rank, world_size, uid)
    return csm.Comm.tcp(rank, world_size, "127.0.0.1", port)


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """The slowest rank's wall time (bench timing contract)."""
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64,
                     device=torch.device("cpu") if device is None else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(value: float, dist=None, device=None) -> float:
    """Sum of a per-rank count (e.g. pairs that returned an error)."""
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64,
                     device=torch.device("cpu") if device is None else device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())
