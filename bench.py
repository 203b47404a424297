"""Benchmark: loop-closure constraint search throughput on MI355X.

Metric (BASELINE.json): loop-closure constraint candidates/sec (node x submap
pairs) + ms/scan-match, 2D 5 cm grid.

Headline workload (default, BASELINE config C3 = the north-star queue):
ConstraintBuilder2D's global loop-closure sweep, 2000 synthetic 1080-beam
nodes x 1000 submaps (400x400 @ 5 cm), FastCorrelativeScanMatcher2D::
MatchFullSubmap, branch_and_bound_depth 7, min_score 0.55: one fixed queue of
2 M pairs. A step is one twentieth of it (50 submaps x 2000 nodes = 100,000
pairs), so `--steps 20` covers the whole queue once. Inside the timed region
the ranks claim chunks of submaps from the queue dynamically (csm_comm's
rank-0 counter table, the reference's shared ThreadPool queue), build each
chunk's pyramids on their GPU, search it as one batch, and finally gather
the accepted constraints to rank 0 in submission order (RCCL). Node clouds
are resident in HBM before timing; submap pyramids are built inside it.

Secondary lines (rank 0, one GPU): C2 (500 x 50), the same C2 queue at
min_score 0.65 (a low-acceptance sweep), C1 RTCSM2D ms/scan-match,
the drop-in's call patterns, voxel filter, Ceres refinement, C4 RTCSM3D and
C5 FastCSM3D (500 nodes x 200 submaps, split over the ranks).

Prints ONE JSON line on rank 0.
"""
import argparse
import importlib
import json
import math
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
# Version tag of the search kernel the committed PMC traffic figures belong to
# (a traffic file recorded on another kernel version is not reported).
KERNEL_TAG = "v5-align8"
# fast3d_search version whose PMC passes TRAFFIC3D_FILE holds.
KERNEL3D_TAG = "f3-tiny5-r64-b32-box"
TRAFFIC3D_FILE = os.path.join("profiles", "r6ba", "traffic_c5.json")


def load_pkg():
    sys.path.insert(0, ROOT)
    import __graft_entry__ as ge
    return ge._load_package()


# Rank 0's gathered constraint records per workload (--dump-records).
DUMP = {}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--workload", default="c3", choices=["c2", "c3"],
                   help="c3 (default): the fixed 2000-node x 1000-submap queue, a step = one "
                        "--c3-slice of it, claimed dynamically over the ranks; c2: 500 x 50 "
                        "submaps per GPU (weak scaling)")
    p.add_argument("--nodes", type=int, default=500)
    p.add_argument("--submaps-per-rank", type=int, default=50)
    p.add_argument("--min-score", type=float, default=0.55)
    p.add_argument("--search-depth", type=int, default=0, help="0 = automatic (exact)")
    p.add_argument("--cpu-seconds", type=float, default=20.0)
    p.add_argument("--cpu-threads", type=int, default=0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-rt", action="store_true",
                   help="skip the secondary legs (C2, C2 strict, C1, C4); C5 runs unless --no-3d")
    p.add_argument("--seed", type=int, default=20250127)
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    p.add_argument("--no-3d", action="store_true")
    p.add_argument("--nodes3d", type=int, default=500)
    p.add_argument("--submaps3d", type=int, default=200,
                   help="C5 submaps in total, split over the ranks")
    p.add_argument("--steps3d", type=int, default=3)
    p.add_argument("--c5-groups", type=int, default=12,
                   help="C5: submap groups per step; group g + 1 builds while group g is searched "
                        "(1: build all, then search all)")
    p.add_argument("--c5-search-streams", type=int, default=1,
                   help="C5: contexts (streams) the groups' searches alternate over, one host "
                        "thread each, so one group's host phases overlap another's kernel "
                        "(1 since round 6: 231-235 ms per step against 236-239 with 2, whose "
                        "overlapping searches contend; profiles/r6an/)")
    p.add_argument("--c5-dropin-calls", type=int, default=4000,
                   help="C5: single MatchFullSubmap calls from 16 threads (Option A), 0: skip")
    p.add_argument("--c5-first-group", type=int, default=6,
                   help="C5: submaps in the first group (its build is exposed; 0: an even split)")
    p.add_argument("--c5-grids", choices=("single", "batch"), default="batch",
                   help="C5: one csm_hybrid_grid_create per grid, or one csm_hybrid_grid_create_batch "
                        "per group and resolution")
    p.add_argument("--c5-create", choices=("single", "batch"), default="batch",
                   help="C5: one csm_fast3d_create per submap, or one csm_fast3d_create_batch per group")
    p.add_argument("--c3-nodes", type=int, default=2000)
    p.add_argument("--c3-submaps", type=int, default=1000)
    p.add_argument("--c3-slice", type=int, default=50, help="submaps of the queue per step")
    p.add_argument("--c3-chunk", type=int, default=0,
                   help="submaps per claimed chunk (0: 4 on one GPU, 2 on several, so the "
                        "ranks' last claims end closer together)")
    p.add_argument("--c3-workers", type=int, default=1,
                   help="host threads per rank, each with its own context (stream): a chunk's "
                        "host work (tie resolution, records) overlaps the next chunk's search")
    p.add_argument("--c3-tie-log", default="",
                   help="write the C3 queue's exactly tied pairs (submap, node, branch) to "
                        "<path>.rank<r>.json (input of tools/c3_tie_fixture.py)")
    p.add_argument("--comm-backend", default="auto", choices=["auto", "rccl", "tcp"],
                   help="csm_comm transport at N > 1 (auto: RCCL with --dist-backend nccl, TCP "
                        "with gloo); rccl with gloo rehearses the RCCL branch on one GPU against "
                        "a library named by CSM_RCCL_LIB (tests/test_bench_multirank_gpu.py)")
    p.add_argument("--dump-records", default="",
                   help="rank 0 writes the gathered C3 and C5 constraint records to this .npz")
    p.add_argument("--cpu-pairs", type=int, default=0,
                   help="CPU baseline sample size (0: 2000 for C3, sized to --cpu-seconds for C2)")
    p.add_argument("--parity-pairs", type=int, default=-1,
                   help="C3 pairs of the timed run compared with the oracle afterwards (-1: the "
                        "CPU baseline's 2000 at N = 1, 500 at N > 1; 0: none). At N > 1 the rank "
                        "that claims a sampled pair keeps its result; rank 0 gathers and checks them")
    return p.parse_args()


def launch_ranks(args):
    """`bench.py --gpus N` (N > 1) run without a launcher: start N ranks under
    torch.distributed.run as a child process, before this process touches the
    GPU, and exit with its status. Under a launcher WORLD_SIZE must equal
    --gpus, so a scaling line can never silently measure fewer GPUs."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is None:
        if args.gpus <= 1:
            return
        import socket
        import subprocess
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
               "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
        print(f"bench: --gpus {args.gpus} without a launcher: starting {args.gpus} ranks "
              "(torch.distributed.run)", file=sys.stderr, flush=True)
        sys.exit(subprocess.call(cmd, env=env))
    if int(ws) != args.gpus:
        print(f"bench: WORLD_SIZE={ws} but --gpus {args.gpus}: refusing to report a {ws}-rank "
              f"run as {args.gpus} GPUs", file=sys.stderr, flush=True)
        sys.exit(2)


def main():
    args = parse()
    launch_ranks(args)
    rank = int(os.environ.get("RANK", "0"))
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local_rank
    coll_dev = None
    if world_size > 1:
        import torch
        import torch.distributed as tdist
        # --dist-backend gloo (CPU tensors) lets ranks share one GPU for rehearsal;
        # the production path is RCCL ("nccl"), one rank per GPU.
        device = local_rank % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(device)
        tdist.init_process_group(args.dist_backend)
        dist = tdist
        coll_dev = torch.device("cuda", device) if args.dist_backend == "nccl" else None

    csm = load_pkg()
    ctx = csm.Context(device)
    comm, transport, comm_ranks = make_comm_checked(csm, ctx, args, rank, world_size, dist,
                                                    coll_dev)
    cdist = importlib.import_module("cartographer_amd.distributed")
    if comm is not None:
        def gather(rec):
            return cdist.gather_records_comm(rec, comm)
    else:
        def gather(rec):
            return cdist.gather_records(rec)

    def barrier_sync():
        if dist is not None:
            dist.barrier()
            import torch
            torch.cuda.synchronize()

    if args.workload == "c3":
        out, errors = c3_run(csm, ctx, args, rank, world_size, dist, coll_dev, comm, gather,
                             transport, barrier_sync)
        out["comm_ranks"] = comm_ranks
    else:
        out, errors = c2_run(csm, ctx, args, rank, world_size, dist, coll_dev, gather, transport,
                             barrier_sync, headline=True)
    if rank == 0 and world_size == 1 and not args.no_rt:
        if args.workload == "c3":
            c2, c2_errors = c2_run(csm, ctx, args, rank, world_size, dist, coll_dev, gather,
                                   transport, barrier_sync, headline=False)
            errors += c2_errors
            out["c2"] = c2
            # The same C2 queue at a stricter min_score: a low-acceptance sweep,
            # closer to a real loop-closure queue where most pairs fail.
            strict = argparse.Namespace(**{**vars(args), "min_score": 0.65})
            c2s, c2s_errors = c2_run(csm, ctx, strict, rank, world_size, dist, coll_dev, gather,
                                     transport, barrier_sync, headline=False, extras=False)
            errors += c2s_errors
            out["c2_strict"] = {k: c2s[k] for k in ("value", "unit", "ms_per_step", "config",
                                                    "accepted_constraints_per_step",
                                                    "errors_per_step")}
            out["c2_strict"]["kernel_ms"] = c2s["roofline"]["kernel_ms_avg"]
        out["rt2d"] = rt2d_bench(csm, ctx, args)
    if rank == 0 and world_size == 1 and not args.no_3d and not args.no_rt:
        out["rt3d"] = rt3d_bench(csm, ctx, args)
    if not args.no_3d:  # collective over ranks: the C5 sweep, submap-sharded
        f3 = fast3d_bench(csm, ctx, args, rank, world_size, dist, coll_dev, barrier_sync, cdist,
                          gather)
        if rank == 0:
            out["fast3d"] = f3
    if rank == 0:
        print(json.dumps(out), flush=True)
        if args.dump_records:
            np.savez(args.dump_records, **DUMP)
    if dist is not None:
        dist.barrier()
    if comm is not None:
        comm.close()
    if dist is not None:
        dist.destroy_process_group()
    f3 = out.get("fast3d", {}) if rank == 0 else {}
    failed = errors + f3.get("errors_per_step", 0) + f3.get("parity_failures", 0)
    if failed:
        print(f"bench: {failed} pair searches returned an error status or differ from the oracle "
              "in a parity sample", file=sys.stderr)
        sys.exit(3)


def c2_run(csm, ctx, args, rank, world_size, dist, coll_dev, gather, transport, barrier_sync,
           headline, extras=True):
    """Config C2: 500 scans x 50 submaps per GPU, submap-sharded (weak
    scaling). As the headline (--workload c2) it carries the roofline and its
    CPU baseline; as a secondary line (default run) one step, plus the
    drop-in's call patterns, the voxel filter and the Ceres refinement on its
    world. Returns (result dict, pairs with error statuses per step)."""
    cdist = importlib.import_module("cartographer_amd.distributed")
    steps = args.steps if headline else 1
    warmup = args.warmup if headline else 1
    t0 = time.time()
    world = csm.SyntheticWorld2D(num_nodes=args.nodes,
                                 num_submaps=args.submaps_per_rank * world_size,
                                 submap_cells=400, beams=1080, seed=args.seed)
    gen_s = time.time() - t0
    my_submaps = cdist.shard_submaps(world.num_submaps, rank, world_size, args.submaps_per_rank)
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30.0), 7, args.search_depth)
    t0 = time.time()
    matchers = [csm.FastCorrelativeScanMatcher2D(world.grid(s), opts, ctx) for s in my_submaps]
    scans = csm.ScanSet(None, ctx, packed=(world.points, world.offsets))
    build_s = time.time() - t0
    sub_local = np.repeat(np.arange(len(my_submaps), dtype=np.int32), args.nodes)
    node_idx = np.tile(np.arange(args.nodes, dtype=np.int32), len(my_submaps))
    pairs = csm.make_pairs(sub_local, node_idx, args.min_score, full_submap=True)
    # Submission index = global queue position (submap-major), used to restore
    # ConstraintBuilder2D::WhenDone ordering on rank 0 (constraint_builder_2d.cc:285-288).
    submission = (np.int64(rank) * len(pairs) + np.arange(len(pairs), dtype=np.int64))
    n_pairs = len(pairs)
    sub_global = np.asarray(my_submaps, np.int64)[sub_local]

    def gather_constraints(res):
        return gather(cdist.make_records(res, submission, sub_global, node_idx))

    # ---- warmup + timed steps ------------------------------------------------
    for _ in range(warmup):
        res = csm.match_batch(matchers, scans, pairs, ctx)
        gather_constraints(res)
    ctx.reset_timing()
    ctx.enable_timing(True)
    barrier_sync()
    t_start = time.perf_counter()
    accepted = 0
    errors = 0  # pairs whose search returned an error status (never counted as work)
    for _ in range(steps):
        res = csm.match_batch(matchers, scans, pairs, ctx)
        errors += int((res["status"] < 0).sum())
        rec = gather_constraints(res)
        if rank == 0:
            accepted = len(rec)
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    ctx.enable_timing(False)
    tm = ctx.timing()
    lv_cands, lv_batches = ctx.level_stats()
    elapsed = cdist.max_over_ranks(elapsed, dist, coll_dev)
    errors = int(cdist.sum_over_ranks(errors, dist, coll_dev))
    total_pairs = n_pairs * world_size * steps
    value = total_pairs / elapsed

    # Roofline of the dominant kernel (fast2d_search_v4): issued bytes per
    # launch (4 B per quad-dword gather) over its HIP-event duration.
    kernel_ms_avg = tm.search_kernel_ms / max(tm.search_launches, 1)
    bytes_per_launch = tm.search_lookups / max(tm.search_launches, 1)
    achieved = bytes_per_launch / (kernel_ms_avg * 1e-3) / 1e9 if kernel_ms_avg > 0 else 0.0
    peak = 8000.0
    traffic = committed_traffic(args, world_size) if headline else None

    out = {
        "metric": "loop-closure constraint candidates/sec (node x submap pairs) + ms/scan-match, 2D 5cm grid",
        "value": value,
        "unit": "pairs/s",
        "n_gpus": world_size,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": elapsed / steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded building world, 1080-beam scans, ray-cast submaps)",
        "config": {"workload": "C2: FastCorrelativeScanMatcher2D::MatchFullSubmap, "
                               f"{args.nodes} scans x {args.submaps_per_rank} submaps per GPU "
                               "(400x400 @5cm), branch_and_bound_depth=7, min_score=%.2f" % args.min_score,
                   "pairs_per_step_per_gpu": n_pairs, "search_depth": matchers[0].options.search_depth,
                   "parallelism": f"submap-sharded x{world_size}",
                   "gather": transport},
        "roofline": roofline_fields(tm, achieved, peak, traffic, kernel_ms_avg, bytes_per_launch,
                                    tm.search_candidates / max(tm.search_launches, 1) *
                                    float(np.diff(world.offsets).mean())),
        "accepted_constraints_per_step": accepted,
        "errors_per_step": errors / steps,
        "stack_high_water": int(tm.stack_high_water),
        "tied_pairs": int(tm.tied_pairs), "ties_walked": int(tm.ties_walked),
        "search_levels": {"candidates_per_pair": [c / max(n_pairs * steps, 1) for c in lv_cands],
                          "mean_lanes_per_batch": [c / b if b else 0 for c, b in zip(lv_cands, lv_batches)]},
        "setup_s": {"world": gen_s, "pyramids_and_upload": build_s},
    }
    if not headline:
        for k in ("metric", "higher_is_better", "vs_baseline", "dtype", "data"):
            out.pop(k)
    if rank == 0 and world_size == 1 and headline and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(world, my_submaps, args)
    if rank == 0 and world_size == 1 and not args.no_rt and extras:
        out["dropin"] = dropin_bench(csm, ctx, matchers, scans, world, args)
        out["voxel_filter"] = voxel_filter_bench(csm, ctx, world, args)
        out["ceres2d"] = ceres_bench(csm, ctx, world, matchers, scans, pairs, res, my_submaps,
                                     node_idx, sub_local, args)
    for m in matchers:
        m.close()
    scans.close()
    return out, errors


def roofline_fields(tm, achieved, peak, traffic, kernel_ms_avg, bytes_per_launch,
                    candidate_bytes):
    return {"bound": "hbm", "achieved": achieved, "peak": peak, "unit": "GB/s",
            "frac": achieved / peak,
            **traffic_fields(traffic, kernel_ms_avg, peak),
            "kernel": "fast2d_search", "kernel_ms_avg": kernel_ms_avg,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "bytes_definition": "4 B per quad-dword gather and 16 B per hex gather the "
                                "search issues (one per node x scan entry: 4 children or "
                                "16 grandchildren each)",
            # SURVEY §8(d)'s figure: candidates scored x N points x 1 B
            "candidate_equivalent_bytes_per_launch": candidate_bytes}


TRAFFIC_FILES = {"c2": os.path.join("profiles", "r6f", "traffic_c2.json"),
                 "c3": os.path.join("profiles", "r6f", "traffic_c3.json")}


def traffic_fields(traffic, kernel_ms_avg, peak):
    """roofline.traffic (HBM-side bytes per launch from the committed PMC
    pass) and the rate / fraction of peak it implies at this run's measured
    launch duration, next to the algorithmic figures."""
    if not traffic or not kernel_ms_avg:
        return {"traffic": None, "traffic_source": None, "traffic_GBps": None, "traffic_frac": None}
    gbps = traffic["traffic_bytes_per_launch"] / (kernel_ms_avg * 1e-3) / 1e9
    return {"traffic": traffic["traffic_bytes_per_launch"], "traffic_source": traffic["source"],
            "traffic_GBps": gbps, "traffic_frac": gbps / peak}


def sum_timing(csm, tms):
    """Adds the timing records of several contexts (the high-water mark: max)."""
    out = csm.Timing()
    for name, _ in csm.Timing._fields_:
        vals = [getattr(t, name) for t in tms]
        setattr(out, name, max(vals) if name == "stack_high_water" else sum(vals))
    return out


GATHER_FILE = os.path.join("profiles", "r6f", "gather_c3.json")


def gather_roofline(kernel_ms):
    """The C3 kernel against its texture-path ceiling: the
    distinct 128-byte lines its gathers touch per launch (a CSM_KPROF pass)
    at the gather microbenchmark's floor of TD cycles per line, spread over
    every CU's TD at the engine clock, against this run's launch time; with
    the measured TD cycles per line from a PMC pass of the same kernel tag
    (tools/gather_roofline.py). None when no committed pass matches."""
    try:
        t = json.load(open(os.path.join(ROOT, GATHER_FILE)))
    except (OSError, ValueError):
        return None
    if t.get("commit_kernel") != KERNEL_TAG or not kernel_ms:
        return None
    return {"bound": "texture data path: TD cycles per distinct 128-byte line a gather touches",
            "line_touches_per_launch": t["line_touches_per_launch"],
            "floor_td_cycles_per_line": t["floor_td_cycles_per_line"],
            "floor_ms": t["floor_ms_per_launch"], "kernel_ms": kernel_ms,
            "frac": t["floor_ms_per_launch"] / kernel_ms,
            "td_cycles_per_line_measured": t["td_cycles_per_line_measured"],
            "source": GATHER_FILE}


def committed_traffic(args, world_size, workload="c2"):
    """HBM-side bytes per search launch from the committed PMC pass
    (profiles/*/traffic_*.json: rocprofv3 --pmc FETCH_SIZE, x2 gfx950
    correction). PMC counters cannot be read from inside this process, so the
    figure is reported only when this run's workload is the profiled one."""
    path = os.path.join(ROOT, TRAFFIC_FILES[workload])
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    if workload == "c3":
        # Per-launch traffic of chunk launches (chunk x all nodes); the PMC
        # pass may cover the first chunks of the queue only.
        same = (args.c3_nodes == t["nodes"] and args.c3_chunk == t["chunk"] and abs(args.min_score - t["min_score"]) < 1e-9 and
                args.search_depth == t["search_depth"] and t.get("commit_kernel") == KERNEL_TAG)
        return t if same else None
    same = (world_size == 1 and args.nodes == t["nodes"] and
            args.submaps_per_rank == t["submaps_per_rank"] and
            abs(args.min_score - t["min_score"]) < 1e-9 and args.search_depth == t["search_depth"]
            and t.get("commit_kernel") == KERNEL_TAG)
    return t if same else None


def make_comm_checked(csm, ctx, args, rank, world_size, dist, coll_dev):
    """The C-ABI communicator for N > 1 (csm_comm over RCCL; TCP for gloo
    rehearsals), with its work-claiming table opened. Rank 0 makes the RCCL
    unique id and hands it out through torch.distributed's store (an error
    sentinel if it cannot, so peers do not wait out the store's timeout).
    Every rank reports whether its communicator came up, and the ranks agree
    (all_reduce MIN) before any of them uses it: if one failed, ALL exit
    non-zero. There is no fallback transport, so a scaling run either
    measures the product path or fails visibly.
    Once up, the communicator must report world_size ranks, and an
    all-reduce over it (RCCL at N > 1 in production) must count every rank:
    that count is the line's comm_ranks.
    Returns (comm or None at N = 1, transport name, ranks the communicator spans)."""
    if dist is None:
        return None, "local", 1
    import torch
    from torch.distributed import distributed_c10d
    store = distributed_c10d._get_default_store()
    backend = args.comm_backend if args.comm_backend != "auto" else \
        ("rccl" if args.dist_backend == "nccl" else "tcp")
    base = int(os.environ.get("MASTER_PORT", "29500"))
    comm, err = None, None
    try:
        if backend == "rccl":
            if rank == 0:
                try:
                    uid = csm.Comm.unique_id()
                except Exception:
                    store.set("csm_comm_id", b"ERROR")
                    raise
                store.set("csm_comm_id", uid)
            else:
                uid = bytes(store.get("csm_comm_id"))
                if uid == b"ERROR":
                    raise RuntimeError("rank 0 could not make the RCCL unique id")
            comm = csm.Comm.rccl(ctx, rank, world_size, uid)
        else:
            comm = csm.Comm.tcp(rank, world_size, "127.0.0.1", base + 17)
        comm.claim_open("127.0.0.1", base + 19)
    except Exception as e:  # noqa: BLE001 - reported below, then every rank exits
        err = e
    ok = torch.tensor([0 if err else 1], dtype=torch.int64,
                      device=coll_dev if coll_dev is not None else torch.device("cpu"))
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if int(ok.item()) != 1:
        print(f"bench: rank {rank}: csm_comm ({backend}) not available on every rank"
              + (f": {err}" if err else ""), file=sys.stderr, flush=True)
        sys.exit(4)
    ranks = int(comm.allreduce(np.ones(1, np.int64))[0])
    if comm.size != world_size or comm.rank != rank or ranks != world_size:
        print(f"bench: rank {rank}: csm_comm spans {ranks} ranks (size {comm.size}, rank "
              f"{comm.rank}), expected {world_size}", file=sys.stderr, flush=True)
        sys.exit(4)
    return comm, f"csm_comm_{backend}", ranks


def rt2d_bench(csm, ctx, args):
    """Config C1: 1080-beam scan vs 200x200 @5cm, +-0.2 m / +-10 deg window."""
    w = csm.SyntheticWorld2D(num_nodes=4, num_submaps=4, submap_cells=200, seed=args.seed + 1)
    opts = csm.RealTimeCorrelativeScanMatcherOptions(0.2, math.radians(10.0), 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher2D(opts, ctx)
    g = w.grid(0)
    n = int(w.submap_nodes[0])
    t = w.node_poses[n]
    init = (t[0] + 0.1, t[1] - 0.07, t[2] + math.radians(5.0))
    cloud = w.cloud(n)
    for _ in range(10):
        m.Match(init, cloud, g)
    # Same grid every call (the device keeps its converted copy), then a grid
    # that changes between calls as local SLAM's matching submap does after
    # every insertion (one cell toggled: the whole grid is re-uploaded and
    # re-converted).
    g2 = csm.ProbabilityGrid(g.resolution, g.max_x, g.max_y, g.cells.copy())
    g2.cells[0, 0] ^= 1
    times, times_changed = [], []
    ctx.reset_timing()
    ctx.enable_timing(True)
    for _ in range(100):
        a = time.perf_counter()
        m.Match(init, cloud, g)
        times.append(time.perf_counter() - a)
    ctx.enable_timing(False)
    kernel_ms = ctx.timing().other_kernel_ms / 100
    for k in range(100):
        a = time.perf_counter()
        m.Match(init, cloud, g2 if k % 2 == 0 else g)
        times_changed.append(time.perf_counter() - a)
    # The same call through the C-ABI with its arguments built once: what a
    # C++ caller (the reference's LocalTrajectoryBuilder2D) pays per Match.
    import ctypes as C
    lib = ctx._lib
    opts_c = csm.RtOptions(opts.linear_search_window, opts.angular_search_window,
                           opts.translation_delta_cost_weight, opts.rotation_delta_cost_weight)
    lim = g.limits()
    cells = np.ascontiguousarray(g.cells, dtype=np.uint16)
    pts = np.ascontiguousarray(np.asarray(cloud, np.float32)[:, :3])
    init_c = csm.Pose2D(*init)
    score_c, pose_c = C.c_double(0.0), csm.Pose2D()
    args_c = (ctx.handle, C.byref(opts_c), C.byref(lim), cells.ctypes.data_as(C.POINTER(C.c_uint16)),
              g.min_correspondence_cost, g.max_correspondence_cost, C.byref(init_c),
              pts.ctypes.data_as(C.POINTER(C.c_float)), len(pts), C.byref(score_c), C.byref(pose_c))
    times_c = []
    for _ in range(100):
        a = time.perf_counter()
        rc = lib.csm_rt2d_match(*args_c)
        times_c.append(time.perf_counter() - a)
        if rc < 0:
            raise RuntimeError(f"csm_rt2d_match: {rc}")
    res = {"gpu_ms_per_scan_match_median": 1e3 * float(np.median(times)),
           "cabi_ms_per_scan_match_median": 1e3 * float(np.median(times_c)),
           "gpu_ms_per_scan_match_median_grid_changed": 1e3 * float(np.median(times_changed)),
           "kernel_ms_per_scan_match": kernel_ms,
           "points": len(cloud)}
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib
    o = oracle_lib.Oracle()
    cpu_s = o.rt2d_time((g.resolution, g.max_x, g.max_y), g.cells,
                        (0.2, math.radians(10.0), 0.1, 0.1), init, cloud, 20)
    res["cpu_ms_per_scan_match"] = cpu_s * 1e3
    res["cpu_threads"] = 1
    return res


def dropin_bench(csm, ctx, matchers, scans, world, args):
    """The drop-in's real call patterns on the C2 world (pyramids resident):
    ConstraintBuilder2D flushing one finished node against every submap (one
    batch of len(matchers) MatchFullSubmap pairs per node, INTEGRATION.md
    Option B), and Option A's single MatchFullSubmap calls (one pair per
    call, the reference's Task granularity)."""
    nodes = min(20, args.nodes)
    k = len(matchers)
    sub = np.arange(k, dtype=np.int32)
    for _ in range(2):  # warm-up
        csm.match_batch(matchers, scans, csm.make_pairs(sub, np.zeros(k, np.int32), args.min_score,
                                                        full_submap=True), ctx)
    flush_ms = []
    for nd in range(nodes):
        pairs = csm.make_pairs(sub, np.full(k, nd, np.int32), args.min_score, full_submap=True)
        a = time.perf_counter()
        csm.match_batch(matchers, scans, pairs, ctx)
        flush_ms.append((time.perf_counter() - a) * 1e3)
    single_ms = []
    for j in range(20):
        m, cloud = matchers[j % k], world.cloud(j % args.nodes)
        a = time.perf_counter()
        m.MatchFullSubmap(cloud, args.min_score)
        single_ms.append((time.perf_counter() - a) * 1e3)
    # Option A as the reference runs it: T pool threads calling MatchFullSubmap
    # on shared matchers concurrently (constraint_builder_2d.cc:100-111), each
    # call on its own call context (stream + scratch).
    from concurrent.futures import ThreadPoolExecutor
    threaded = {}
    calls = 400
    for T in (1, 4, 8, 16):
        def one(j):
            return matchers[j % k].MatchFullSubmap(world.cloud(j % args.nodes), args.min_score)
        with ThreadPoolExecutor(max_workers=T) as ex:
            list(ex.map(one, range(2 * T)))  # warm-up: one call context per thread
            a = time.perf_counter()
            list(ex.map(one, range(calls)))
            wall = time.perf_counter() - a
        threaded[str(T)] = {"calls": calls, "pairs_per_s": calls / wall}
    # The same pattern from C++ threads (tools/dropin_threads.cc, no GIL):
    # what the reference's ThreadPool sees through the C-ABI.
    threaded_cpp = None
    exe = os.path.join(ROOT, "tools", "dropin_threads")
    if os.path.exists(exe):
        import subprocess
        try:
            out = subprocess.run([exe, "2000", str(args.min_score)], capture_output=True, text=True,
                                 timeout=300, check=True).stdout
            threaded_cpp = json.loads(out.strip().splitlines()[-1])
        except (subprocess.SubprocessError, ValueError) as e:
            threaded_cpp = {"error": str(e)[:200]}
    return {"per_node_flush": {"pairs_per_flush": k, "flushes": nodes,
                               "ms_per_flush_median": float(np.median(flush_ms)),
                               "pairs_per_s": k / (float(np.median(flush_ms)) * 1e-3)},
            "single_call": {"calls": len(single_ms),
                            "ms_per_match_full_submap_median": float(np.median(single_ms)),
                            "pairs_per_s": 1e3 / float(np.median(single_ms))},
            "single_call_threads": threaded,
            "single_call_threads_cpp": threaded_cpp,
            "note": "through the Python ctypes mirror; a batch uploads its pair descriptors, the "
                    "scan set's rotation tables are built once and kept on the device"}


def voxel_filter_bench(csm, ctx, world, args):
    """AdaptiveVoxelFilter (trajectory_builder_2d.lua:25-29 options) over the
    C2 node clouds as one device-resident batch: the step that makes the
    clouds the loop-closure search uses (local_trajectory_builder_2d.cc:229-231)."""
    import ctypes as C
    clouds = [world.cloud(n) for n in range(args.nodes)]
    pts = np.ascontiguousarray(np.concatenate(clouds), np.float32)
    offsets = np.zeros(len(clouds) + 1, np.int64)
    offsets[1:] = np.cumsum([len(c) for c in clouds])
    d_pts, d_off = csm.DeviceBuffer(pts), csm.DeviceBuffer(offsets)
    d_keep = csm.DeviceBuffer(nbytes=len(pts))
    d_cnt = csm.DeviceBuffer(nbytes=4 * len(clouds))
    opts = csm.AdaptiveVoxelFilterOptions.make(0.5, 200, 50.0)
    lib = ctx._lib
    max_pts = int(np.diff(offsets).max())

    def launch():
        csm._check(lib.csm_adaptive_voxel_filter_device(
            ctx.handle, d_pts.ptr, d_off.ptr, len(clouds), max_pts, C.byref(opts), d_keep.ptr,
            d_cnt.ptr), "csm_adaptive_voxel_filter_device")

    for _ in range(3):
        launch()
    csm.synchronize(ctx)
    reps = 20
    a = time.perf_counter()
    for _ in range(reps):
        launch()
    csm.synchronize(ctx)
    gpu_s = (time.perf_counter() - a) / reps
    counts = d_cnt.to_numpy(np.int32, len(clouds))
    keep = d_keep.to_numpy(np.uint8, len(pts)).astype(bool)
    res = {"workload": f"AdaptiveVoxelFilter(max_length 0.5, min_num_points 200, max_range 50) "
                       f"over {len(clouds)} clouds x {max_pts} points",
           "gpu_ms_per_batch": gpu_s * 1e3, "clouds_per_s": len(clouds) / gpu_s,
           "mean_kept_points": float(counts.mean())}
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        o = oracle_lib.Oracle()
        a = time.perf_counter()
        ref, _ = o.adaptive_voxel_filter_masks(clouds, 0.5, 200, 50.0)
        cpu_s = time.perf_counter() - a
        res["cpu_clouds_per_s"] = len(clouds) / cpu_s
        res["cpu_threads"] = 1
        res["matches_oracle"] = bool((ref == keep).all())
    except OSError as e:  # the checker must be there: fail loudly
        raise RuntimeError(f"oracle (CPU baseline) unavailable: {e}") from e
    return res


def ceres_bench(csm, ctx, world, matchers, scans, pairs, res, my_submaps, node_idx, sub_local,
                args):
    """CeresScanMatcher2D refinement of one C2 step's accepted matches (what
    ComputeConstraint does next, constraint_builder_2d.cc:245-249), as one
    device batch; CPU: the oracle restatement on a sample, one thread."""
    ok = np.nonzero(res["status"] == csm.CSM_OK)[0]
    if len(ok) == 0:
        return {"accepted": 0}
    init = np.stack([res["x"][ok], res["y"][ok], res["theta"][ok]], 1)
    sub, scn = sub_local[ok], node_idx[ok]
    opts = csm.CeresOptions2D.make()
    csm.ceres_refine_batch(matchers, scans, sub, scn, init, None, opts, ctx)  # warm-up
    a = time.perf_counter()
    poses, iters = csm.ceres_refine_batch(matchers, scans, sub, scn, init, None, opts, ctx)
    gpu_s = time.perf_counter() - a
    out = {"workload": f"CeresScanMatcher2D::Match on the {len(ok)} accepted matches of one C2 "
                       "step (pose_graph.lua options), 1080-point clouds",
           "accepted": int(len(ok)), "gpu_ms": gpu_s * 1e3,
           "refinements_per_s": len(ok) / gpu_s, "mean_iterations": float(iters.mean())}
    try:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        o = oracle_lib.Oracle()
        k = min(len(ok), 64)
        a = time.perf_counter()
        for j in range(k):
            g = world.grid(int(my_submaps[int(sub[j])]))
            o.ceres2d_match((g.resolution, g.max_x, g.max_y), g.cells, (20.0, 10.0, 1.0, 10),
                            init[j][:2], init[j], world.cloud(int(scn[j])))
        cpu_s = (time.perf_counter() - a) / k
        out["cpu_baseline"] = {"value": 1.0 / cpu_s, "unit": "refinements/s", "cores": 1,
                               "kind": "port", "sample": f"{k} of the accepted matches (oracle "
                                                         "restatement, includes grid copy-in)"}
    except OSError as e:  # the checker must be there: fail loudly
        raise RuntimeError(f"oracle (CPU baseline) unavailable: {e}") from e
    return out


def rt3d_bench(csm, ctx, args):
    """Config C4: RealTimeCorrelativeScanMatcher3D, one 64-ring scan (~55k
    points, R <= 14 m) vs the 0.10 m HybridGrid of a 20x20x5 m box world,
    +-0.3 m / +-15 deg, weights 0.1. Every candidate is scored (exhaustive, as
    the reference); the CPU figure extrapolates the oracle's per-candidate
    time (one thread, like Match) measured on a spread sample of candidates."""
    w = csm.SyntheticWorld3D(num_nodes=2, num_submaps=1, world_x=20.0, world_y=20.0,
                             world_z=5.0, num_boxes=8, max_range=14.0, seed=args.seed + 3)
    c = int(w.submap_nodes[0])
    cloud = w.raw[c]
    grid = csm.HybridGrid(w.high_resolution, *w.high_cells[0], context=ctx)
    (tx, ty, tz), q = w.node_in_submap(c, 0)
    dyaw = math.radians(4.0)
    q0 = (q[0] * math.cos(dyaw / 2) - q[3] * math.sin(dyaw / 2), 0.0, 0.0,
          q[3] * math.cos(dyaw / 2) + q[0] * math.sin(dyaw / 2))
    init = ((tx + 0.12, ty - 0.08, tz + 0.05), q0)
    opts = (0.3, math.radians(15.0), 0.1, 0.1)
    m = csm.RealTimeCorrelativeScanMatcher3D(csm.RealTimeCorrelativeScanMatcherOptions(*opts), ctx)
    m.Match(init, cloud[:64], grid)  # warm-up (module load), tiny
    ctx.reset_timing()
    ctx.enable_timing(True)
    t0 = time.perf_counter()
    score, pose = m.Match(init, cloud, grid)
    wall = time.perf_counter() - t0
    tm = ctx.timing()
    ctx.enable_timing(False)
    lookups = tm.rt3d_lookups
    n = len(cloud)
    res = {"config": "C4: 64-ring scan vs 0.10 m HybridGrid, +-0.3 m / +-15 deg, wt=wr=0.1",
           "points": n, "candidates": lookups / n, "gpu_ms_per_scan_match": wall * 1e3,
           "kernel_ms": tm.rt3d_kernel_ms, "lookups": lookups,
           "lookups_per_s": lookups / (tm.rt3d_kernel_ms * 1e-3) if tm.rt3d_kernel_ms else 0.0,
           "algorithmic_GBps": 2.0 * lookups / (tm.rt3d_kernel_ms * 1e-3) / 1e9
           if tm.rt3d_kernel_ms else 0.0, "score": score,
           "pose_error_m": math.dist(pose[0], (tx, ty, tz))}
    if not args.no_cpu:
        try:
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            import ctypes as C

            import oracle_lib
            o = oracle_lib.Oracle()
            og = o.hybrid_grid(w.high_resolution)
            og.set_values(*w.high_cells[0])
            total = int(round(lookups / n))
            P = C.POINTER
            oo = np.asarray(opts, np.float64)
            ii = oracle_lib._pose7(*init)
            pts = np.ascontiguousarray(cloud, np.float32)

            def timed(k):
                return o.lib.oracle_rt3d_time(og.h, oo.ctypes.data_as(P(C.c_double)),
                                              ii.ctypes.data_as(P(C.c_double)),
                                              pts.ctypes.data_as(P(C.c_float)), n, k,
                                              max(1, total // k))

            probe = timed(16)
            sample = int(min(50000, max(16, 10.0 / max(probe / 16, 1e-6))))
            sec = timed(sample)
            res["cpu_baseline"] = {
                "value": sec / sample * total * 1e3, "unit": "ms/scan-match", "cores": 1,
                "kind": "port",
                "sample": f"{sample} candidates spread over the {total} of one match, "
                          f"{sec:.2f} s, extrapolated to all candidates (oracle, -O3)"}
        except OSError as e:  # the checker must be there: fail loudly
            raise RuntimeError(f"oracle (CPU baseline) unavailable: {e}") from e
    return res


def fast3d_bench(csm, ctx, args, rank=0, world_size=1, dist=None, coll_dev=None,
                 barrier_sync=lambda: None, cdist=None, gather=None):
    """C5 (BASELINE.json configs[4]): FastCorrelativeScanMatcher3D::MatchFullSubmap
    over nodes3d nodes x submaps3d submaps (500 x 200) of one world, split by
    submap over the ranks (strong scaling): rank r builds and searches
    submaps [r S / N, (r + 1) S / N) against every node, pose_graph.lua 3D
    options, global_localization_min_score 0.6. Accepted constraints are
    gathered to rank 0 each step in submission order; value = all pairs / the
    slowest rank's time."""
    t0 = time.time()
    S3 = args.submaps3d
    b0, b1 = rank * S3 // world_size, (rank + 1) * S3 // world_size
    w = csm.SyntheticWorld3D(num_nodes=args.nodes3d, num_submaps=S3,
                             submap_range=(b0, b1 - b0), seed=args.seed + 5)
    gen = time.time() - t0
    o = csm.FastCorrelativeScanMatcherOptions3D()

    # Builds run on their own context (stream), issued by a helper thread: a
    # step's submaps go in --c5-groups groups, and group g + 1's grids and
    # pyramids are issued while group g is searched (the reference's matcher
    # construction tasks run ahead of the constraint tasks that depend on
    # them, constraint_builder_3d.cc:170-198). The search waits for each
    # matcher's build (its ready event).
    bctx = csm.Context(ctx.device) if args.c5_groups > 1 else ctx
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(max_workers=1) if args.c5_groups > 1 else None
    # Searches: group g on sctxs[g % K], from K host threads (the builder's
    # constraint tasks run on a thread pool, constraint_builder_3d.cc:200-230).
    nsearch = max(1, args.c5_search_streams) if pool is not None else 1
    sctxs = [ctx] + [csm.Context(ctx.device) for _ in range(nsearch - 1)]
    spool = ThreadPoolExecutor(max_workers=nsearch) if nsearch > 1 else None

    # CSM_C5_TRACE=1: host timestamps of each group's build and search
    # (stderr), to see what the step waits on.
    c5_trace = [] if os.environ.get("CSM_C5_TRACE") else None

    def build(subs=None, bc=None):
        """The submaps' HybridGrids and PrecomputationGridStack3D pyramids
        (DispatchScanMatcherConstruction, constraint_builder_3d.cc:170-198)."""
        if c5_trace is not None:
            c5_trace.append(("build+", len(c5_trace), time.perf_counter()))
            try:
                return build_(subs, bc)
            finally:
                c5_trace.append(("build-", len(c5_trace), time.perf_counter()))
        return build_(subs, bc)

    def build_(subs=None, bc=None):
        bc = bc or ctx
        subs = range(w.num_submaps) if subs is None else subs
        if args.c5_grids == "batch":  # one csm_hybrid_grid_create_batch per resolution
            hi = csm.HybridGrid.create_batch(w.high_resolution, [w.high_cells[s] for s in subs], context=bc)
            lo = csm.HybridGrid.create_batch(w.low_resolution, [w.low_cells[s] for s in subs], context=bc)
            g = list(zip(hi, lo))
        else:
            g = [(csm.HybridGrid(w.high_resolution, *w.high_cells[s], context=bc),
                  csm.HybridGrid(w.low_resolution, *w.low_cells[s], context=bc))
                 for s in subs]
        if c5_trace is not None:
            c5_trace.append(("grids", len(c5_trace), time.perf_counter()))
        # A group's matchers in one csm_fast3d_create_batch (one launch per
        # level for the whole group), or one create per submap (--c5-create
        # single). With the builds pipelined against the searches, the batch
        # form's ~20 launches per group beat ~18 per submap (profiles/r5n/).
        if args.c5_create == "batch":
            m = csm.FastCorrelativeScanMatcher3D.create_batch(g, [w.submap_hist[s] for s in subs], o, bc)
        else:
            m = [csm.FastCorrelativeScanMatcher3D(gg[0], gg[1], w.submap_hist[s], o, bc)
                 for s, gg in zip(subs, g)]
        return g, m

    def close(g, m):
        for x in m:
            x.close()
        for pair in g:
            for x in pair:
                x.close()

    # Node clouds converted to csm_node3d once, like inputs resident before the timed region.
    nodes = csm.NodeSet3D([w.node(i) for i in range(w.num_nodes)])
    sub = np.repeat(np.arange(w.num_submaps), w.num_nodes)
    nod = np.tile(np.arange(w.num_nodes), w.num_submaps)
    rot = np.array([w.node_rotation(n) for n in range(w.num_nodes)])
    pairs = csm.make_pairs_3d(sub, nod, 0.6, True, node_q=rot[nod])
    sub_global = w.submap_ids[sub].astype(np.int64)
    submission = sub_global * w.num_nodes + nod  # queue order: submap-major

    # A step is the whole C5 queue as a sweep runs it: every submap's grids and
    # pyramid are built (once per sweep, as the builder's matcher cache does),
    # then all its pairs are searched; the builds are inside the timed region
    # like C3's pyramids, and also reported on their own. Releasing the
    # matchers afterwards (to the context's pool, where the next step's builds
    # find them) is outside it, reported as release_ms_per_step.
    phase = {"build": 0.0, "search": 0.0, "release": 0.0}

    ids = np.arange(w.num_submaps)
    f = min(args.c5_first_group, w.num_submaps) if args.c5_groups > 1 else 0
    groups = [g for g in ([ids[:f]] if f else []) +
              np.array_split(ids[f:], max(1, args.c5_groups - (1 if f else 0))) if len(g)]

    def step():
        a = time.perf_counter()
        if pool is None:
            g, m = build()
            b = time.perf_counter()
            res = csm.match_batch_3d(m, nodes, pairs, ctx)
        elif spool is None:
            g, m, parts, waited = [], [], [], 0.0
            fut = pool.submit(build, groups[0], bctx)
            for gi, grp in enumerate(groups):
                t = time.perf_counter()
                gg, mm = fut.result()
                waited += time.perf_counter() - t
                if gi + 1 < len(groups):
                    fut = pool.submit(build, groups[gi + 1], bctx)
                g += gg
                m += mm
                lo, hi = int(grp[0]) * w.num_nodes, (int(grp[-1]) + 1) * w.num_nodes
                gp = pairs[lo:hi].copy()
                gp["submap"] -= int(grp[0])
                parts.append(csm.match_batch_3d(mm, nodes, gp, ctx))
            res = np.concatenate(parts)
            b = a + waited  # the builds' exposed time (the rest overlaps the searches)
        else:
            # Every group's build queued in order on the build thread; group
            # g's search starts on its own thread once its build is issued.
            bfuts = [pool.submit(build, grp, bctx) for grp in groups]

            def search(gi):
                grp = groups[gi]
                _, mm = bfuts[gi].result()
                lo, hi = int(grp[0]) * w.num_nodes, (int(grp[-1]) + 1) * w.num_nodes
                gp = pairs[lo:hi].copy()
                gp["submap"] -= int(grp[0])
                if c5_trace is not None:
                    c5_trace.append(("search+", gi, time.perf_counter()))
                r = csm.match_batch_3d(mm, nodes, gp, sctxs[gi % nsearch])
                if c5_trace is not None:
                    c5_trace.append(("search-", gi, time.perf_counter()))
                return r

            sfuts = [spool.submit(search, gi) for gi in range(len(groups))]
            bfuts[0].result()
            b = time.perf_counter()  # the first group's build is exposed
            parts = [f.result() for f in sfuts]
            g, m = [], []
            for f in bfuts:
                gg, mm = f.result()
                g += gg
                m += mm
            res = np.concatenate(parts)
        rec = cdist.make_records_3d(res, submission, sub_global, nod) if cdist else None
        if cdist is not None:
            rec = gather(rec) if gather is not None else \
                cdist.gather_records(rec, dist, rank, world_size, coll_dev)
        c = time.perf_counter()
        if c5_trace is not None:
            print("c5 trace:", " ".join(f"{k}{i}@{(t - a) * 1e3:.1f}" for k, i, t in c5_trace),
                  file=sys.stderr)
            c5_trace.clear()
        phase["build"] += b - a
        phase["search"] += c - b
        return res, rec, (g, m)

    _, _, kept = step()  # warm-up at full size (staging buffers, the pool)
    close(*kept)
    phase["build"] = phase["search"] = 0.0
    for c in sctxs:
        c.reset_timing()
        c.enable_timing(True)
    reps = max(1, args.steps3d)
    errors3 = 0
    wall = 0.0
    for k in range(reps):
        barrier_sync()
        t0 = time.perf_counter()
        res3, rec, kept = step()
        barrier_sync()
        wall += time.perf_counter() - t0
        errors3 += int((res3["status"] < 0).sum())
        if k + 1 < reps:
            t0 = time.perf_counter()
            close(*kept)
            phase["release"] += time.perf_counter() - t0
    grids, mats = kept
    if pool is not None:
        pool.shutdown()
    if spool is not None:
        spool.shutdown()
    if rank == 0 and rec is not None:
        DUMP["c5"] = np.asarray(rec)
    tm = merged_timing(sctxs)
    for c in sctxs:
        c.enable_timing(False)
    if cdist is not None:
        wall = cdist.max_over_ranks(wall, dist, coll_dev)
    total = w.num_nodes * S3 * reps
    out = {"config": f"C5: MatchFullSubmap, {w.num_nodes} nodes x {S3} submaps split over "
                     f"{world_size} GPU(s) (0.10/0.45 m grids, ~200-point clouds, "
                     "120-bucket histograms), branch_and_bound_depth 8, full_resolution_depth 3; a step "
                     "builds every submap's HybridGrids and pyramid, then searches all pairs",
           "pairs_per_step": w.num_nodes * S3, "steps": reps, "value": total / wall,
           "unit": "pairs/s", "n_gpus": world_size, "scaling": "strong",
           "accepted_per_step": int(len(rec)) if rec is not None else int((res3["status"] == 0).sum()),
           "ms_per_step": wall / reps * 1e3,
           "errors_per_step": errors3 / reps, "stack_high_water": int(tm.stack_high_water),
           # Pairs whose maximum more than one passing leaf reached (resolved to
           # the reference's pick, host3d.cc ResolveTies3d), per step.
           "tied_pairs_per_step": tm.tied_pairs_3d / reps,
           "ties_walked_per_step": tm.ties_walked_3d / reps,
           "ties_by_branch_last_step": {name: int(((res3["status"] == 0) & (res3["tie"] == code)).sum())
                                        for name, code in (("ancestors", csm.TIE_ANCESTORS),
                                                           ("toplist", csm.TIE_TOPLIST),
                                                           ("walk", csm.TIE_WALK))},
           "c5_groups": len(groups), "c5_group_sizes": [len(g) for g in groups],
           "c5_search_streams": nsearch,
           "c5_create": args.c5_create,
           # Builds' exposed time: all of it with one group; with several, the
           # first group's build and any wait for a later one.
           "build_ms_per_step": phase["build"] / reps * 1e3,
           "release_ms_per_step": phase["release"] / max(reps - 1, 1) * 1e3,
           "search_ms_per_step": phase["search"] / reps * 1e3,
           "value_search_only": total / phase["search"] if phase["search"] else 0.0,
           "roofline": roofline_3d(tm),
           "kernel_ms_per_step": tm.fast3d_kernel_ms / reps, "lookups_per_step": tm.fast3d_lookups / reps,
           "algorithmic_GBps": tm.fast3d_lookups / (tm.fast3d_kernel_ms * 1e-3) / 1e9
           if tm.fast3d_kernel_ms else 0.0, "setup_s": gen}
    if world_size > 1:
        # Parity at N > 1: every rank checks a uniform sample of its own share
        # (its submaps x every node) of the last timed step against the
        # oracle on its host, and the counts are summed over the ranks.
        total_k = args.parity_pairs if args.parity_pairs > 0 else 512
        if args.parity_pairs != 0:
            k = max(1, -(-total_k // world_size))
            _, _, sampled = oracle3d_runner(w, o, args.cpu_threads or host_cpu()["usable_cpus"])(k)
            mine = parity_3d(res3, sampled, w.num_nodes)
            summed = {key: int(cdist.sum_over_ranks(mine[key], dist, coll_dev))
                      for key in ("pairs", "compared", "matched_oracle", "mismatched_decision",
                                  "mismatched_score", "mismatched_pose", "gpu_errors")}
            summed["ranks"] = world_size
            summed["what"] = ("each rank's uniform sample of its own share of the last timed step, "
                              "its GPU results vs the oracle's on that rank's host; counts summed")
            out["parity_sample"] = summed
            out["parity_failures"] = parity_failures(summed)
        return out
    if rank != 0:
        return out
    # CeresScanMatcher3D refinement of the last step's accepted matches
    # (constraint_builder_3d.cc:264-275), one device batch.
    ok = np.nonzero(res3["status"] == csm.CSM_OK)[0]
    if len(ok):
        flat = [g for pair in grids for g in pair]
        items = [(2 * int(sub[i]), 2 * int(sub[i]) + 1, int(nod[i]),
                  (tuple(res3["t"][i]), tuple(res3["q"][i])), tuple(res3["t"][i])) for i in ok]
        csm.ceres_refine_batch_3d(flat, nodes, items, context=ctx)  # warm-up
        a = time.perf_counter()
        _, it3 = csm.ceres_refine_batch_3d(flat, nodes, items, context=ctx)
        out["ceres3d"] = {"accepted": int(len(ok)), "gpu_ms": (time.perf_counter() - a) * 1e3,
                          "mean_iterations": float(np.mean(it3)),
                          "workload": "CeresScanMatcher3D::Match on one C5 step's accepted "
                                      "matches (pose_graph.lua options)"}
    if args.c5_dropin_calls > 0:
        out["dropin"] = dropin_3d(csm, w, mats, sub, nod, rot, res3, args.c5_dropin_calls)
    if not args.no_cpu:
        cpu = host_cpu()
        threads = args.cpu_threads or cpu["usable_cpus"]
        run = oracle3d_runner(w, o, threads)
        probe, _, _ = run(threads)
        k = min(20000, max(threads, int(threads * 10.0 / max(probe, 1e-3))))
        sec, task, sampled = run(k)
        cb = summarize_cpu(k, sec, task, threads, cpu, [], "uniformly sampled pairs of the same queue")
        cb["sample"] = (f"{k} uniformly sampled pairs of the same queue, {sec:.1f} s on "
                        f"{threads} threads (oracle, -O3)")
        out["cpu_baseline"] = cb
        # The same pairs' GPU results from the last timed step, against
        # the oracle's (fast_correlative_scan_matcher_3d.cc:148-199).
        out["parity_sample"] = parity_3d(res3, sampled, w.num_nodes)
        out["parity_failures"] = parity_failures(out["parity_sample"])
    return out


def oracle3d_runner(w, o, threads):
    """run(k) -> (wall s, per-task s, (submaps, nodes, results)): the oracle's
    MatchFullSubmap on k uniformly drawn (submap, node) pairs of world `w`
    (this rank's submaps x every node), `threads` tasks at a time."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C

    import oracle_lib
    orc = oracle_lib.Oracle()
    opt = (o.branch_and_bound_depth, o.full_resolution_depth, o.min_rotational_score,
           o.min_low_resolution_score, o.linear_xy_search_window,
           o.linear_z_search_window, o.angular_search_window)
    keep = []
    handles = []
    for s in range(w.num_submaps):
        oh, ol = orc.hybrid_grid(w.high_resolution), orc.hybrid_grid(w.low_resolution)
        oh.set_values(*w.high_cells[s])
        ol.set_values(*w.low_cells[s])
        om = orc.fast3d(oh, ol, w.submap_hist[s], opt)
        keep.append((oh, ol, om))
        handles.append(om.h)
    hoff = np.zeros(w.num_nodes + 1, np.int64)
    hoff[1:] = np.cumsum([len(x) for x in w.high])
    loff = np.zeros(w.num_nodes + 1, np.int64)
    loff[1:] = np.cumsum([len(x) for x in w.low])
    high = np.ascontiguousarray(np.concatenate(w.high), np.float32)
    low = np.ascontiguousarray(np.concatenate(w.low), np.float32)
    hists = np.ascontiguousarray(np.stack(w.node_hist), np.float32)
    nq = np.ascontiguousarray([w.node_rotation(i) for i in range(w.num_nodes)], np.float64)
    rng = np.random.RandomState(777)
    P = C.POINTER
    hv = (C.c_void_p * len(handles))(*handles)

    def run(k):
        ps = rng.randint(0, w.num_submaps, k).astype(np.int32)
        pn = rng.randint(0, w.num_nodes, k).astype(np.int32)
        matched = np.zeros(k, np.int32)
        results = np.zeros((k, 14))
        task = np.zeros(k)
        wall = orc.lib.oracle_fast3d_match_pairs(
            hv, high.ctypes.data_as(P(C.c_float)), hoff.ctypes.data_as(P(C.c_int64)),
            low.ctypes.data_as(P(C.c_float)), loff.ctypes.data_as(P(C.c_int64)),
            hists.ctypes.data_as(P(C.c_float)), hists.shape[1],
            nq.ctypes.data_as(P(C.c_double)), ps.ctypes.data_as(P(C.c_int32)),
            pn.ctypes.data_as(P(C.c_int32)), k, threads, 0.6,
            matched.ctypes.data_as(P(C.c_int32)), results.ctypes.data_as(P(C.c_double)),
            task.ctypes.data_as(P(C.c_double)))
        _ = len(keep)  # the oracle's grids and matchers live as long as run()
        return wall, task, (ps, pn, results)
    return run


def cpu_baseline(world, my_submaps, args):
    """C2 CPU baseline: the oracle restatement (the reference's algorithm and
    data structures) on host threads, one pair per task as ConstraintBuilder2D
    schedules them, on a bounded uniform random sample of the same queue."""
    rng = np.random.RandomState(12345)
    k = 100000
    ps = np.asarray(my_submaps)[rng.randint(0, len(my_submaps), k)]
    pn = rng.randint(0, world.num_nodes, k)
    return cpu_pairs_2d(world, ps, pn, args, "uniformly sampled (submap, scan) pairs of the same C2 queue")[0]


def host_cpu():
    """The host the CPU baseline runs on: CPU model, logical CPUs, the CPUs
    this process may run on (affinity) and the cgroup CPU quota."""
    info = {"model": None, "logical_cpus": os.cpu_count(), "affinity_cpus": None,
            "cgroup_quota_cpus": None}
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["model"] = line.split(":", 1)[1].strip()
                break
    except OSError as e:  # the checker must be there: fail loudly
        raise RuntimeError(f"oracle (CPU baseline) unavailable: {e}") from e
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity_cpus"] = os.cpu_count()
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            info["cgroup_quota_cpus"] = int(quota) / int(period)
    except (OSError, ValueError):
        pass
    usable = info["affinity_cpus"] or 1
    if info["cgroup_quota_cpus"]:
        usable = min(usable, max(1, int(math.ceil(info["cgroup_quota_cpus"]))))
    info["usable_cpus"] = usable
    return info


def timed_pool(run, threads_options, probe_pairs_per_thread=2):
    """Picks the thread count for the CPU baseline: a short probe at each
    candidate (the usable CPUs, and every logical CPU when more are visible);
    the faster per-pair rate wins. run(k, threads) -> (wall_s, task_seconds)."""
    best = None
    probes = []
    for t in threads_options:
        k = max(t * probe_pairs_per_thread, 4)
        wall, _ = run(k, t)
        probes.append({"threads": t, "pairs": k, "pairs_per_s": k / wall})
        if best is None or k / wall > best[1]:
            best = (t, k / wall)
    return best, probes


def summarize_cpu(k, wall, task_s, threads, cpu, probes, what):
    """pairs/s on the sample, with a 95% interval from the spread of per-pair
    costs: value * mean / (mean +- 1.96 * sd / sqrt(k))."""
    mu = float(np.mean(task_s))
    half = 1.96 * float(np.std(task_s, ddof=1)) / math.sqrt(k) if k > 1 else 0.0
    value = k / wall
    lo = value * mu / (mu + half)
    hi = value * mu / (mu - half) if mu > half else float("inf")
    return {"value": value, "ci95": [lo, hi], "unit": "pairs/s", "cores": threads,
            "threads": threads, "kind": "port",
            "host": {"cpu_model": cpu["model"], "logical_cpus": cpu["logical_cpus"],
                     "affinity_cpus": cpu["affinity_cpus"],
                     "cgroup_quota_cpus": cpu["cgroup_quota_cpus"]},
            "thread_probes": probes,
            "mean_pair_cpu_s": mu,
            "sample": f"{k} {what}, {wall:.1f} s wall on {threads} threads "
                      f"(oracle restatement, -O3 -DNDEBUG, one pair per task)"}


def oracle_submaps_2d(o, world, submaps, threads):
    """Oracle FastCorrelativeScanMatcher2D per submap, built on a thread pool
    (ctypes releases the GIL; setup, outside any timed region)."""
    from concurrent.futures import ThreadPoolExecutor

    def make(s):
        return o.fast2d((world.resolution, world.submap_max[s, 0], world.submap_max[s, 1]),
                        world.submap_cells[s], 7.0, math.radians(30.0), 7)
    with ThreadPoolExecutor(max_workers=max(1, threads)) as ex:
        return list(ex.map(make, submaps))


def cpu_pairs_2d(world, pair_sub, pair_node, args, what):
    """CPU baseline on the given (submap, node) pairs: the oracle's
    MatchFullSubmap, one pair per task on a pool of host threads
    (ConstraintBuilder2D on common::ThreadPool, thread_pool.cc:80-106)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import ctypes as C

    import oracle_lib
    o = oracle_lib.Oracle()
    cpu = host_cpu()
    uniq, inv = np.unique(pair_sub, return_inverse=True)
    subs = oracle_submaps_2d(o, world, uniq, cpu["usable_cpus"])
    handles = (C.c_void_p * len(subs))(*[m.h for m in subs])
    pts = np.ascontiguousarray(world.points, np.float32)
    offs = np.ascontiguousarray(world.offsets, np.int64)
    P = C.POINTER
    cursor = [0]
    # The oracle's result for every sample index it ran (probes and the main
    # run): the bench's parity check against the GPU's results of the same
    # pairs (c3_run).
    # Per pair also the oracle's work counters (lookups, candidates per
    # level; oracle_fast2d_match_pairs_stats): work_ratio's reference side.
    ores = {"done": np.zeros(len(inv), bool), "matched": np.zeros(len(inv), bool),
            "score": np.zeros(len(inv), np.float32), "pose": np.zeros((len(inv), 3)),
            "stats": np.zeros((len(inv), 16), np.int64)}

    def run(k, threads):
        # Consecutive slices of the (shuffled) sample: probes and the main
        # run see different pairs of the same distribution. Slices of
        # 64 pairs per thread keep every thread busy and let a long sample
        # print progress (a silent minute-long call looks hung).
        wall, tasks, done, t0 = 0.0, [], 0, time.time()
        while done < k:
            kk = min(k - done, 64 * threads)
            idx = np.arange(cursor[0], cursor[0] + kk) % len(inv)
            cursor[0] += kk
            ps = np.ascontiguousarray(inv[idx], np.int32)
            pn = np.ascontiguousarray(pair_node[idx], np.int32)
            scores, poses = np.zeros(kk, np.float32), np.zeros(3 * kk)
            matched, task = np.zeros(kk, np.int32), np.zeros(kk)
            st = np.zeros((kk, 16), np.int64)
            wall += o.lib.oracle_fast2d_match_pairs_stats(
                handles, pts.ctypes.data_as(P(C.c_float)), offs.ctypes.data_as(P(C.c_int64)),
                ps.ctypes.data_as(P(C.c_int32)), pn.ctypes.data_as(P(C.c_int32)), kk, threads,
                args.min_score, scores.ctypes.data_as(P(C.c_float)),
                poses.ctypes.data_as(P(C.c_double)), matched.ctypes.data_as(P(C.c_int32)),
                task.ctypes.data_as(P(C.c_double)), st.ctypes.data_as(P(C.c_int64)))
            ores["stats"][idx] = st
            tasks.append(task)
            ores["done"][idx] = True
            ores["matched"][idx] = matched != 0
            ores["score"][idx] = scores
            ores["pose"][idx] = poses.reshape(-1, 3)
            done += kk
            if k > 64 * threads:
                print(f"cpu baseline: {done}/{k} pairs, {time.time() - t0:.0f} s", file=sys.stderr,
                      flush=True)
        return wall, np.concatenate(tasks)

    # Thread counts to probe: the usable CPUs (affinity and cgroup quota);
    # every logical CPU as well only when no quota caps the process.
    options = [args.cpu_threads] if args.cpu_threads else sorted(
        {cpu["usable_cpus"]} | ({cpu["logical_cpus"]} if cpu["logical_cpus"] and
                                not cpu["cgroup_quota_cpus"] else set()))
    (threads, rate), probes = timed_pool(run, options)
    k = args.cpu_pairs or max(4 * threads, int(rate * args.cpu_seconds))
    wall, task = run(k, threads)
    return summarize_cpu(k, wall, task, threads, cpu, probes, what), ores


def gather_sample(sample, comm, csm):
    """The sampled pairs' GPU results held by every rank (each kept the
    results of the chunks it claimed) to rank 0 over the C-ABI communicator
    (csm_comm_gather): (sample index, csm_result2d) rows; rank 0 fills its
    sample table with them. Every sampled pair must come back from some rank
    (parity_failures counts the missing)."""
    row = np.dtype([("i", "<i8"), ("r", csm.RESULT_DTYPE)])
    have = np.nonzero(sample["have"])[0]
    mine = np.zeros(len(have), row)
    mine["i"] = have
    mine["r"] = sample["gpu"][have]
    blobs = comm.gather(mine.tobytes())
    if blobs is None:  # not rank 0
        return
    for b in blobs:
        rows = np.frombuffer(b, row)
        sample["gpu"][rows["i"]] = rows["r"]
        sample["have"][rows["i"]] = True


def work_ratio(csm, ctx, world, opts, sample, ores, args, queue_levels):
    """SURVEY §8(d)'s reference lookup count next to the GPU's work, on the
    same sampled pairs. Reference side: the oracle's counters from the parity
    run (GetValue calls, fast_correlative_scan_matcher_2d.cc:319-330, and
    candidates scored per level, :335-378). GPU side: the sampled pairs
    searched again after the timed region, grouped by submap, with the
    kernel's counters (gpu_sample_work)."""
    done = ores["done"]
    g_lv, g_cand, g_vals = gpu_sample_work(csm, ctx, world, opts, sample["sub"][done],
                                           sample["node"][done], args.min_score)
    return work_ratio_fields(ores["stats"][done], g_lv, g_cand, g_vals, queue_levels)


def gpu_sample_work(csm, ctx, world, opts, subs, nodes, min_score):
    """The GPU search's work on the given (submap, node) pairs: candidates
    scored per level (12), all candidates, and candidate values its gathers
    fetch (1 B each: 4 per quad entry, 16 per hex entry, an entry being a
    point or a weighted cluster; the kernel's issued bytes), summed over the
    pairs. Searched in groups of up to 32 submaps on `ctx`, untimed."""
    uniq = np.unique(subs)
    g_lv = np.zeros(12)
    g_cand = g_vals = 0.0
    scans = csm.ScanSet(None, ctx, packed=(world.points, world.offsets))
    ctx.enable_timing(True)
    for a in range(0, len(uniq), 32):
        grp = uniq[a:a + 32]
        mats = [csm.FastCorrelativeScanMatcher2D(world.grid(int(s)), opts, ctx) for s in grp]
        pos = {int(s): i for i, s in enumerate(grp)}
        sel = np.nonzero(np.isin(subs, grp))[0]
        sub_local = np.array([pos[int(s)] for s in subs[sel]], np.int32)
        pairs = csm.make_pairs(sub_local, np.asarray(nodes)[sel].astype(np.int32), min_score,
                               full_submap=True)
        ctx.reset_timing()
        csm.match_batch(mats, scans, pairs, ctx)
        tm = ctx.timing()
        lv, _ = ctx.level_stats()
        g_lv[:len(lv)] += np.asarray(lv, np.float64)[:12]
        g_cand += tm.search_candidates
        g_vals += tm.search_lookups
        for m in mats:
            m.close()
    ctx.enable_timing(False)
    ctx.reset_timing()
    scans.close()
    return g_lv, g_cand, g_vals


def work_ratio_fields(stats, gpu_levels, gpu_candidates, gpu_values, queue_levels):
    """work_ratio's line fields from the oracle's per-pair counters (rows of
    16: lookups, scans, lowest-resolution candidates, candidates per level
    0..12) and the GPU's totals over the same pairs. Both count a candidate at
    the level it is scored at; the GPU's pyramid is deeper (automatic depth),
    its hex levels skip the level between, and its inner bounds are the
    looser clustered ones, so levels differ and the totals are
    what compare."""
    stats = np.asarray(stats, np.int64).reshape(-1, 16)
    k = max(len(stats), 1)
    o_lv = stats[:, 3:16].sum(0) / k
    o_cand = float(o_lv.sum())
    o_look = float(stats[:, 0].sum()) / k
    g_lv = np.asarray(gpu_levels, np.float64) / k
    g_cand, g_vals = gpu_candidates / k, gpu_values / k
    return {"pairs": len(stats),
            "oracle": {"candidates_per_pair": o_cand, "candidates_per_pair_by_level": o_lv.tolist(),
                       "lookups_per_pair": o_look,
                       "what": "reference algorithm (oracle restatement): candidates scored at "
                               "each level and GetValue calls (candidates x points)"},
            "gpu_same_pairs": {"candidates_per_pair": g_cand,
                               "candidates_per_pair_by_level": g_lv.tolist(),
                               "candidate_values_per_pair": g_vals,
                               "what": "the same pairs searched again after the timed region: "
                                       "candidates scored per level, and candidate values the "
                                       "gathers fetch (1 B each: 4 per quad entry, 16 per hex "
                                       "entry, an entry being a point or a weighted cluster)"},
            "gpu_queue_candidates_per_pair": float(np.sum(queue_levels)),
            "candidates_ratio": g_cand / o_cand if o_cand else None,
            "leaf_candidates_ratio": float(g_lv[0] / o_lv[0]) if o_lv[0] else None,
            "lookups_ratio": g_vals / o_look if o_look else None}


def parity_2d(sample, ores):
    """The GPU's results of the sampled pairs (from the timed run) against the
    oracle's MatchFullSubmap of the same pairs: the match decision, the score
    (bit-identical float) and the pose (identical doubles, the reference's pick
    among exact ties included; fast_correlative_scan_matcher_2d.cc:210-262)."""
    both = sample["have"] & ores["done"]
    g = sample["gpu"][both]
    gm = g["status"] == 0
    om = ores["matched"][both]
    dec = gm != om
    ok = gm & om
    gpose = np.stack([g["x"], g["y"], g["theta"]], 1)
    score_bad = ok & (g["score"].astype(np.float32) != ores["score"][both])
    pose_bad = ok & np.any(gpose != ores["pose"][both], axis=1)
    return {"pairs": int(len(both)), "compared": int(both.sum()), "matched_oracle": int(om.sum()),
            "mismatched_decision": int(dec.sum()), "mismatched_score": int(score_bad.sum()),
            "mismatched_pose": int(pose_bad.sum()), "gpu_errors": int((g["status"] < 0).sum()),
            "what": "the CPU baseline's sampled pairs: the GPU's results from the timed run vs the "
                    "oracle's (decision, float score bit-exact, pose exact)"}


def dropin_3d(csm, w, mats, sub, nod, rot, res3, calls, threads=16):
    """Option A in 3D: single MatchFullSubmap calls on the last C5 step's
    matchers from `threads` host threads, as the builder's thread pool issues
    them (constraint_builder_3d.cc:200-230); the library coalesces concurrent
    calls into batches (host3d.cc SingleMatch3). Each result must equal the
    timed batch's result of the same pair."""
    from concurrent.futures import ThreadPoolExecutor
    pick = np.random.RandomState(7).randint(0, len(sub), calls)
    node_objs = [w.node(i) for i in range(w.num_nodes)]
    ident = (1.0, 0.0, 0.0, 0.0)

    def one(i):
        n = int(nod[i])
        return mats[int(sub[i])].MatchFullSubmap(rot[n], ident, node_objs[n], 0.6)

    with ThreadPoolExecutor(max_workers=threads) as ex:
        list(ex.map(one, pick[:64]))  # warm-up: call contexts, staging
        a = time.perf_counter()
        got = list(ex.map(one, pick))
        el = time.perf_counter() - a
    mism = 0
    for i, g in zip(pick, got):
        ok = res3["status"][i] == csm.CSM_OK
        if (g is not None) != ok or (ok and (np.float32(g.score) != np.float32(res3["score"][i]) or
                                            g.pose_estimate != (tuple(res3["t"][i]), tuple(res3["q"][i])))):
            mism += 1
    if mism:
        raise RuntimeError(f"C5 single calls: {mism} of {calls} differ from the batch's results")
    # The same call pattern from C++ threads (tools/dropin_threads3d.cc, no
    # GIL) on a C5 slice: what ConstraintBuilder3D's ThreadPool sees through
    # the C-ABI, with every result checked against the batch's.
    threaded_cpp = None
    exe = os.path.join(ROOT, "tools", "dropin_threads3d")
    if os.path.exists(exe):
        import subprocess
        try:
            res = subprocess.run([exe, "4000", "8", "200"], capture_output=True, text=True, timeout=300)
            threaded_cpp = json.loads(res.stdout.strip().splitlines()[-1])
            if res.returncode != 0:
                raise RuntimeError(f"dropin_threads3d: exit {res.returncode}, {threaded_cpp}")
        except (subprocess.SubprocessError, ValueError, IndexError) as e:
            threaded_cpp = {"error": str(e)[:200]}
    return {"calls": int(calls), "threads": threads, "pairs_per_s": calls / el,
            "matched": int(sum(g is not None for g in got)), "mismatches_vs_batch": mism,
            "single_call_threads_cpp": threaded_cpp,
            "note": "single csm_fast3d_match_full_submap calls from Python threads (GIL-bound), "
                    "coalesced by the library; single_call_threads_cpp: C++ threads on a C5 slice"}


def merged_timing(contexts):
    """The contexts' csm_timing summed field by field (the high-water mark
    as a maximum)."""
    ts = [c.timing() for c in contexts]
    out = type(ts[0])()
    for name, _ in out._fields_:
        vals = [getattr(t, name) for t in ts]
        setattr(out, name, max(vals) if name == "stack_high_water" else sum(vals))
    return out


def roofline_3d(tm):
    """C5's fast3d_search against the HBM roofline, as C3's: achieved =
    algorithmic bytes per launch (1 B per precomputation-grid lookup, 8 per
    octet gather; the kernel counts them) / the launch time from HIP events;
    traffic = FETCH_SIZE x 1024 x 2 per dispatch from the committed PMC pass
    of the same kernel tag (tools/traffic3d_json.py), with the rate it
    implies at this run's launch time."""
    launches = max(int(tm.fast3d_launches), 1)
    kernel_ms = tm.fast3d_kernel_ms / launches
    per_launch = tm.fast3d_lookups / launches
    achieved = per_launch / (kernel_ms * 1e-3) / 1e9 if kernel_ms else 0.0
    out = {"bound": "hbm", "achieved": achieved, "peak": 8000.0, "unit": "GB/s",
           "frac": achieved / 8000.0, "bytes_per_launch": per_launch, "kernel_ms_avg": kernel_ms,
           "launches": launches, "traffic": None, "traffic_frac": None}
    try:
        t = json.load(open(os.path.join(ROOT, TRAFFIC3D_FILE)))
    except (OSError, ValueError):
        return out
    if t.get("commit_kernel") == KERNEL3D_TAG and t.get("traffic_bytes_per_launch") and kernel_ms:
        # Launches of another size than the PMC run's (the step's groups):
        # its traffic per algorithmic byte times this run's bytes per launch.
        ratio = t.get("traffic_bytes_per_algorithmic_byte")
        out["traffic"] = ratio * per_launch if ratio else t["traffic_bytes_per_launch"]
        out["traffic_GBps"] = out["traffic"] / (kernel_ms * 1e-3) / 1e9
        out["traffic_frac"] = out["traffic_GBps"] / 8000.0
        out["traffic_source"] = TRAFFIC3D_FILE
    return out


def parity_3d(res3, sampled, num_nodes):
    """C5's CPU sample: the GPU's MatchFullSubmap results of the sampled pairs
    (pair index = submap x nodes + node, the last timed step) against the
    oracle's: decision, score, rotational and low-resolution scores
    (bit-identical floats) and pose (identical, ties included)."""
    ps, pn, o = sampled
    g = res3[ps.astype(np.int64) * num_nodes + pn]
    gm = g["status"] == 0
    om = o[:, 0] != 0
    ok = gm & om
    score_bad = ok & ((g["score"].astype(np.float32) != o[:, 1].astype(np.float32)) |
                      (g["rotational_score"].astype(np.float32) != o[:, 2].astype(np.float32)) |
                      (g["low_resolution_score"].astype(np.float32) != o[:, 3].astype(np.float32)))
    gpose = np.concatenate([np.asarray(g["t"], np.float64), np.asarray(g["q"], np.float64)], 1)
    pose_bad = ok & np.any(gpose != o[:, 4:11], axis=1)
    return {"pairs": int(len(ps)), "compared": int(len(ps)), "matched_oracle": int(om.sum()),
            "mismatched_decision": int((gm != om).sum()), "mismatched_score": int(score_bad.sum()),
            "mismatched_pose": int(pose_bad.sum()), "gpu_errors": int((g["status"] < 0).sum()),
            "what": "the CPU baseline's sampled pairs: the GPU's results from the last timed step vs "
                    "the oracle's (decision, float scores bit-exact, pose exact)"}


def parity_failures(p):
    """Pairs of a parity sample that differ from the oracle, plus any sampled
    pair the GPU did not return (the check must cover the whole sample)."""
    return (p["mismatched_decision"] + p["mismatched_score"] + p["mismatched_pose"] +
            p["gpu_errors"] + (p["pairs"] - p["compared"]))


def c3_run(csm, ctx, args, rank, world_size, dist, coll_dev, comm, gather, transport,
           barrier_sync):
    """C3 (BASELINE.json configs[2], the north-star queue): ConstraintBuilder2D's
    global sweep, 2000 nodes x 1000 submaps = 2 M MatchFullSubmap pairs,
    min_score 0.55, as ONE fixed queue (constraint_builder_2d.cc:102-111, swept
    by pose_graph_2d.cc:379-392). Step k is the queue's slice of --c3-slice
    submaps starting at submap k * slice (mod 1000): 20 steps = the whole
    queue. The timed region's K slices are cut into chunks of --c3-chunk
    submaps x all nodes; every rank claims chunks through csm_comm_fetch_add
    (the rank-0 counter table: the shared queue of common::ThreadPool,
    thread_pool.cc:80-106), builds the chunk's pyramids on its GPU, searches it
    as one batch and keeps the accepted constraints; at the end the records
    go to rank 0 in submission order (constraint_builder_2d.cc:279-300) over
    RCCL. Warmup steps run one chunk each, untimed."""
    cdist = importlib.import_module("cartographer_amd.distributed")
    N, S = args.c3_nodes, args.c3_submaps
    K = args.c3_chunk = args.c3_chunk or (4 if world_size == 1 else 2)
    t0 = time.time()
    world = csm.SyntheticWorld2D(num_nodes=N, num_submaps=S, submap_cells=400, beams=1080,
                                 seed=args.seed)
    gen_s = time.time() - t0
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30.0), 7, args.search_depth)
    # One context (stream + scratch) and scan set per host worker.
    ctxs = [ctx] + [csm.Context(ctx.device) for _ in range(max(args.c3_workers, 1) - 1)]
    scan_sets = [csm.ScanSet(None, c, packed=(world.points, world.offsets)) for c in ctxs]
    slice_ = args.c3_slice
    # The timed queue: steps x slice submaps, in queue order (wrapping after S).
    queue = (np.arange(args.steps * slice_) % S).astype(np.int64)
    chunks = [queue[i:i + K] for i in range(0, len(queue), K)]
    n_chunks = len(chunks)

    phase = {"pyramids": 0.0, "search": 0.0, "close": 0.0, "records": 0.0}
    profile = bool(os.environ.get("C3_PROFILE"))

    def run_chunk(subs, base, w=0):
        ctx, scans = ctxs[w], scan_sets[w]
        t0 = time.perf_counter()
        mats = [csm.FastCorrelativeScanMatcher2D(world.grid(int(s)), opts, ctx) for s in subs]
        sub_local = np.repeat(np.arange(len(subs), dtype=np.int32), N)
        node = np.tile(np.arange(N, dtype=np.int32), len(subs))
        pairs = csm.make_pairs(sub_local, node, args.min_score, full_submap=True)
        t1 = time.perf_counter()
        res = csm.match_batch(mats, scans, pairs, ctx)
        t2 = time.perf_counter()
        for m in mats:
            m.close()
        t3 = time.perf_counter()
        sub_global = np.asarray(subs, np.int64)[sub_local]
        submission = base + np.arange(len(pairs), dtype=np.int64)  # queue order: submap-major
        rec = cdist.make_records(res, submission, sub_global, node)
        if profile:
            phase["pyramids"] += t1 - t0
            phase["search"] += t2 - t1
            phase["close"] += t3 - t2
            phase["records"] += time.perf_counter() - t3
        return res, rec

    claim_lock = threading.Lock()  # one claim in flight per rank (the comm's socket)

    def claim(key):
        with claim_lock:
            if comm is None:
                claim.local[key] = claim.local.get(key, 0) + 1
                return claim.local[key] - 1
            return comm.fetch_add(key, 1)
    claim.local = {}

    # The parity sample of the queue, drawn up front (the same seed on every
    # rank, so every rank holds rank 0's draw): the timed run keeps the GPU's
    # result of each sampled pair on whichever rank claims it; afterwards the
    # results are gathered to rank 0 and compared with the oracle's result of
    # the same pair (parity_sample). At N = 1 the oracle's run on the sample is
    # also the CPU baseline.
    sample = None
    k_s = args.parity_pairs
    if k_s < 0:
        k_s = 0 if (world_size == 1 and args.no_cpu) else \
            (args.cpu_pairs or 2000) if world_size == 1 else 500
    if k_s > 0:
        rng = np.random.RandomState(12345)
        # Submaps of the timed queue (all of them when it covers the queue).
        s_sub = np.unique(queue)[rng.randint(0, len(np.unique(queue)), k_s)]
        s_node = rng.randint(0, N, k_s)
        want = {}
        for i, (a, b) in enumerate(zip(s_sub, s_node)):
            want.setdefault(int(a), []).append((i, int(b)))
        sample = {"sub": s_sub, "node": s_node, "want": want,
                  "gpu": np.zeros(k_s, csm.RESULT_DTYPE), "have": np.zeros(k_s, bool)}
    for w in range(args.warmup):  # one chunk each: module load, staging buffers
        for i in range(len(ctxs)):
            run_chunk(chunks[(rank + w) % n_chunks], 0, i)
    for c in ctxs:
        c.reset_timing()
        c.enable_timing(True)
    barrier_sync()
    t_start = time.perf_counter()
    done = {"errors": 0, "mine": 0, "recs": [], "ties": []}

    def worker(w):
        while True:
            c = claim(1)  # key 1: the timed queue's head
            if c >= n_chunks:
                return
            res, rec = run_chunk(chunks[c], np.int64(c) * K * N, w)
            tied = np.nonzero((res["status"] == 0) & (res["tie"] != 0))[0]
            if sample is not None:
                for j, sm in enumerate(chunks[c]):
                    for i, n in sample["want"].get(int(sm), ()):
                        sample["gpu"][i] = res[j * N + n]
                        sample["have"][i] = True
            with claim_lock:
                done["errors"] += int((res["status"] < 0).sum())
                done["recs"].append(rec)
                done["mine"] += 1
                for k in tied:  # (submap, node, csm_result2d.tie) of exactly tied pairs
                    done["ties"].append((int(chunks[c][k // N]), int(k % N), int(res["tie"][k])))
            if rank == 0 and (c % 10 == 0 or world_size == 1):
                print(f"c3: chunk {c + 1}/{n_chunks} {time.perf_counter() - t_start:.1f} s",
                      file=sys.stderr, flush=True)

    if len(ctxs) == 1:
        worker(0)
    else:
        threads = [threading.Thread(target=worker, args=(w,)) for w in range(len(ctxs))]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
    errors, mine, recs = done["errors"], done["mine"], done["recs"]
    tms = [c.timing() for c in ctxs]
    if profile:
        print("c3 host phases (s): " + ", ".join(f"{k} {v:.2f}" for k, v in phase.items())
              + f"; kernel {sum(t.search_kernel_ms for t in tms) * 1e-3:.2f}",
              file=sys.stderr, flush=True)
    allrec = gather(np.concatenate(recs) if recs else np.zeros((0, cdist.RECORD_WIDTH)))
    barrier_sync()
    elapsed = time.perf_counter() - t_start
    if sample is not None and comm is not None:
        # After the timed region: every rank's results of sampled pairs to rank 0.
        gather_sample(sample, comm, csm)
    for c in ctxs:
        c.enable_timing(False)
    tm = sum_timing(csm, [c.timing() for c in ctxs])
    lv_cands, lv_batches = (list(map(sum, zip(*v))) for v in zip(*[c.level_stats() for c in ctxs]))
    accepted = len(allrec) if rank == 0 else 0
    if rank == 0:
        DUMP["c3"] = np.asarray(allrec)
    elapsed = cdist.max_over_ranks(elapsed, dist, coll_dev)
    errors = int(cdist.sum_over_ranks(errors, dist, coll_dev))
    total_pairs = len(queue) * N
    kernel_ms_avg = tm.search_kernel_ms / max(tm.search_launches, 1)
    bytes_per_launch = tm.search_lookups / max(tm.search_launches, 1)
    achieved = bytes_per_launch / (kernel_ms_avg * 1e-3) / 1e9 if kernel_ms_avg else 0.0
    traffic = committed_traffic(args, world_size, "c3")
    claimed = cdist.sum_over_ranks(mine, dist, coll_dev)
    chunks_max = cdist.max_over_ranks(mine, dist, coll_dev)
    out = {
        "metric": "loop-closure constraint candidates/sec (node x submap pairs) + ms/scan-match, 2D 5cm grid",
        "value": total_pairs / elapsed, "unit": "pairs/s", "n_gpus": world_size,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (seeded building world, 1080-beam scans, ray-cast submaps)",
        "config": {"workload": f"C3: ConstraintBuilder2D global sweep, {N} nodes x {S} submaps "
                               f"(400x400 @5cm) = {N * S} MatchFullSubmap pairs in one fixed queue; "
                               f"a step = {slice_} submaps x {N} nodes of it ({slice_ * N} pairs), "
                               f"chunks of {K} submaps claimed dynamically by the ranks, pyramids "
                               f"built inside the timed region, branch_and_bound_depth=7, "
                               f"min_score={args.min_score:.2f}",
                   "pairs_per_step": slice_ * N, "queue_pairs_timed": total_pairs,
                   "covers_whole_queue": bool(len(np.unique(queue)) == S),
                   "search_depth": args.search_depth,
                   "parallelism": f"dynamic chunk claiming x{world_size}",
                   "gather": transport},
        "roofline": roofline_fields(tm, achieved, 8000.0, traffic, kernel_ms_avg, bytes_per_launch,
                                    tm.search_candidates / max(tm.search_launches, 1) *
                                    float(np.diff(world.offsets).mean())),
        "gather_roofline": gather_roofline(kernel_ms_avg),
        "accepted_constraints": accepted,
        "errors_per_step": errors / args.steps,
        "stack_high_water": int(tm.stack_high_water),
        "chunks": n_chunks, "chunks_claimed": int(claimed), "chunks_max_rank": int(chunks_max),
        # Pairs with exactly tied maxima (resolved to the reference's pick,
        # csm_host.cc ResolveTies) and any left at the smallest-key leaf.
        "tied_pairs_rank0": int(tm.tied_pairs), "ties_walked_rank0": int(tm.ties_walked),
        # Per resolution branch (csm_result2d.tie): under one top-level
        # candidate, through the whole top-level list's introsort, unresolved.
        "ties_by_branch_rank0": {name: sum(1 for t in done["ties"] if t[2] == code)
                                 for name, code in (("ancestors", csm.TIE_ANCESTORS),
                                                    ("toplist", csm.TIE_TOPLIST),
                                                    ("walk", csm.TIE_WALK))},
        "kernel_s_rank0": tm.search_kernel_ms * 1e-3, "search_launches_rank0": int(tm.search_launches),
        "search_levels": {"candidates_per_pair": [c / max(mine * K * N, 1) for c in lv_cands],
                          "mean_lanes_per_batch": [c / b if b else 0 for c, b in zip(lv_cands, lv_batches)]},
        "setup_s": {"world": gen_s},
    }
    if args.c3_tie_log:  # the tied pairs, for tools/c3_tie_fixture.py
        with open(f"{args.c3_tie_log}.rank{rank}.json", "w") as f:
            json.dump({"seed": args.seed, "nodes": N, "submaps": S, "min_score": args.min_score,
                       "ties": sorted(done["ties"])}, f)
    if sample is not None and rank == 0:
        args_c = argparse.Namespace(**vars(args))
        args_c.cpu_pairs = len(sample["sub"])
        cb, ores = cpu_pairs_2d(world, sample["sub"], sample["node"], args_c,
                                "uniformly sampled (submap, node) pairs of the C3 queue")
        if world_size == 1 and not args.no_cpu:
            out["cpu_baseline"] = cb
            out["speedup_vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
        out["parity_sample"] = parity_2d(sample, ores)
        out["parity_sample"]["ranks"] = world_size
        out["work_ratio"] = work_ratio(csm, ctx, world, opts, sample, ores, args,
                                       out["search_levels"]["candidates_per_pair"])
        bad = parity_failures(out["parity_sample"])
        if bad:
            print(f"bench: C3 parity sample: {bad} of {out['parity_sample']['compared']} pairs differ "
                  "from the oracle", file=sys.stderr, flush=True)
            errors += bad
    for sc, c in zip(scan_sets, ctxs):
        sc.close()
        if c is not ctx:
            c.close()
    return out, errors


if __name__ == "__main__":
    main()
