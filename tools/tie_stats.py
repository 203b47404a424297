"""Tie statistics of the 2D FastCSM search ("settle tie parity").

For every pair: the oracle's maximum leaf score, every leaf tied at it
(oracle TiedMaxLeaves: the reference's tree, all leaves whose score equals the
maximum) and the reference's own pick (its DFS's first-visited maximum,
fast_correlative_scan_matcher_2d.cc:331-332, 370-374). The device's pick
among the same tie set is the smallest (rotation, x, y) key
(csm_device.h PackLeafKey). Reports how often a pair has a tie, how often the
two picks differ and how far apart they are (cells, rotation steps).

CPU only (the oracle); the device pick follows from the tie set exactly,
because the device search scores every leaf whose bound reaches the best sum
(DESIGN.md §2).

    python tools/tie_stats.py [--c3-pairs 200] [--synthetic-pairs 96] > profiles/r3a/tie_stats.json
"""
import argparse
import json
import math
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def device_pick(ties):
    key = ((ties[:, 0].astype(np.int64) << 28) | ((ties[:, 1].astype(np.int64) + 8192) << 14) |
           (ties[:, 2].astype(np.int64) + 8192))
    return tuple(int(v) for v in ties[int(np.argmin(key))])


def run_cases(o, cases, threads):
    """cases: (name, limits, cells, cloud, full, initial, min_score, lin, ang, depth)."""
    def one(c):
        name, limits, cells, cloud, full, init, ms, lin, ang, depth = c
        om = o.fast2d(limits, cells, lin, ang, depth)
        ties, ref = om.tie_leaves(full, init, cloud, ms)
        if ties is None:
            return {"case": name, "matched": False}
        dev = device_pick(ties)
        out = {"case": name, "matched": True, "tied_leaves": int(len(ties)),
               "same_pick": dev == ref}
        if dev != ref:
            out.update({"reference_pick": ref, "device_pick": dev,
                        "d_rotation_steps": dev[0] - ref[0],
                        "d_cells": max(abs(dev[1] - ref[1]), abs(dev[2] - ref[2]))})
        return out
    with ThreadPoolExecutor(max_workers=threads) as ex:
        return list(ex.map(one, cases))


def golden_cases(path, label):
    d = np.load(path)
    opt = d["options"]
    out = []
    for k, p in enumerate(d["pairs"]):
        s, c, full = int(p[0]), int(p[1]), bool(p[2])
        lim = tuple(float(v) for v in d["limits"][s])
        cloud = d["points"][d["offsets"][c]:d["offsets"][c + 1]]
        out.append((f"{label}[{k}]", lim, d["cells"][s], cloud, full, tuple(p[3:6]), float(p[6]),
                    float(opt[0]), float(opt[1]), int(opt[2])))
    return out


def world_cases(csm, world, pairs, label, ms=0.55):
    out = []
    for s, n in pairs:
        g = world.grid(int(s))
        out.append((f"{label}({int(s)},{int(n)})", (g.resolution, g.max_x, g.max_y), g.cells,
                    world.cloud(int(n)), True, None, ms, 7.0, math.radians(30.0), 7))
    return out


def summarize(rows):
    m = [r for r in rows if r["matched"]]
    tied = [r for r in m if r["tied_leaves"] > 1]
    diff = [r for r in m if not r["same_pick"]]
    return {"pairs": len(rows), "matched": len(m), "matched_with_ties": len(tied),
            "picks_differ": len(diff),
            "max_d_cells": max([r["d_cells"] for r in diff], default=0),
            "max_abs_d_rotation_steps": max([abs(r["d_rotation_steps"]) for r in diff], default=0),
            "differ_beyond_one_cell": sum(1 for r in diff if r["d_cells"] > 1 or r["d_rotation_steps"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c3-pairs", type=int, default=200)
    ap.add_argument("--synthetic-pairs", type=int, default=96)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    args = ap.parse_args()
    import __graft_entry__ as ge
    import oracle_lib
    csm = ge._load_package()
    o = oracle_lib.Oracle()
    report = {}
    for f, label in (("fast2d_c2.npz", "golden_c2"), ("fast2d_local.npz", "golden_local")):
        rows = run_cases(o, golden_cases(os.path.join(ROOT, "tests", "golden", f), label), args.threads)
        report[label] = {"summary": summarize(rows), "rows": rows}
        print(label, report[label]["summary"], file=sys.stderr, flush=True)
    # The reference's own 2D tests (fast_correlative_scan_matcher_2d_test.cc):
    # CorrectPose (:144-192, Match, depth 3) and FullSubmapMatching (:194-246,
    # depth 6), 6-point clouds, the draws tests/test_fast2d_gpu.py makes.
    cases = []
    rng = np.random.RandomState(42)
    cloud = np.array([[-2.5, 0.5, 0], [-2.0, 0.5, 0], [0.0, -0.5, 0], [0.5, -1.6, 0],
                      [2.5, 0.5, 0], [2.5, 1.7, 0]], np.float32)
    for i in range(50):
        d = rng.uniform(-1, 1, 3).astype(np.float32)
        exp = np.array([2 * d[0], 2 * d[1], 0.5 * d[2]], np.float32)
        ret = o.transform_cloud(exp, cloud)
        lim, cells = o.grid_from_inserts(0.05, 5.0, 5.0, 200, 200, [((exp[0], exp[1], 0), ret)])
        cases.append((f"correct_pose[{i}]", lim, cells, cloud, False, (0.0, 0.0, 0.0), 0.1, 3.0, 1.0, 3))
    rng = np.random.RandomState(42)
    base = np.array([[-2.5, 0.5, 0], [-2.25, 0.5, 0], [0.0, 0.5, 0], [0.25, 1.6, 0],
                     [2.5, 0.5, 0], [2.0, 1.8, 0]], np.float32)
    for i in range(20):
        d = rng.uniform(-1, 1, 6).astype(np.float32)
        pert = np.array([10 * d[0], 10 * d[1], 1.6 * d[2]], np.float32)
        local = np.array([2 * d[3], 2 * d[4], 0.5 * d[5]], np.float32)
        lim, cells = o.grid_from_inserts(0.05, 5.0, 5.0, 200, 200,
                                         [((local[0], local[1], 0), o.transform_cloud(local, base))])
        cases.append((f"full_submap[{i}]", lim, cells, o.transform_cloud(pert, base), True, None, 0.1,
                      3.0, 1.0, 6))
    rows = run_cases(o, cases, args.threads)
    report["reference_tests"] = {"summary": summarize(rows), "rows": rows}
    print("reference_tests", report["reference_tests"]["summary"], file=sys.stderr, flush=True)
    # The GPU tests' synthetic world (N ~ 200 clouds), matched and uniform pairs.
    w = csm.SyntheticWorld2D(num_nodes=64, num_submaps=8, decimate_to=200, seed=20250127)
    rng = np.random.RandomState(1)
    pairs = [(s, int(w.submap_nodes[s])) for s in range(8)]
    pairs += list(zip(rng.randint(0, 8, args.synthetic_pairs - 8), rng.randint(0, 64, args.synthetic_pairs - 8)))
    rows = run_cases(o, world_cases(csm, w, pairs, "synthetic200"), args.threads)
    report["synthetic200"] = {"summary": summarize(rows), "rows": rows}
    print("synthetic200", report["synthetic200"]["summary"], file=sys.stderr, flush=True)
    # The C3 world (bench.py's seed): pairs near each submap's own node
    # (matches) and uniform pairs of the queue.
    w3 = csm.SyntheticWorld2D(num_nodes=2000, num_submaps=1000, submap_cells=400, beams=1080,
                              seed=20250127)
    rng = np.random.RandomState(3)
    half = args.c3_pairs // 2
    near = rng.choice(w3.num_submaps, half, replace=False)
    pairs = [(int(s), int(min(w3.num_nodes - 1, w3.submap_nodes[s] + d)))
             for s, d in zip(near, rng.randint(0, 3, half))]
    pairs += list(zip(rng.randint(0, w3.num_submaps, args.c3_pairs - half),
                      rng.randint(0, w3.num_nodes, args.c3_pairs - half)))
    rows = run_cases(o, world_cases(csm, w3, pairs, "c3"), args.threads)
    report["c3"] = {"summary": summarize(rows), "rows": rows}
    print("c3", report["c3"]["summary"], file=sys.stderr, flush=True)
    print(json.dumps(report, indent=1))


if __name__ == "__main__":
    main()
