"""Option A in 3D (single FastCorrelativeScanMatcher3D::MatchFullSubmap
calls, the reference's one Task per pair, constraint_builder_3d.cc:200-230):
latency of one call alone and throughput from T host threads, on a slice of
the C5 world (matchers built once, pyramids resident).

    python tools/probe_dropin3d.py [--submaps 8] [--nodes 200] [--calls 2000]
With CSM_PROFILE3D=1 the library prints each batch's host phases."""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--submaps", type=int, default=8)
    p.add_argument("--nodes", type=int, default=200)
    p.add_argument("--calls", type=int, default=2000)
    p.add_argument("--threads", default="1,4,16,32")
    p.add_argument("--seed", type=int, default=20250127 + 5)
    a = p.parse_args()
    csm = bench.load_pkg()
    ctx = csm.Context(0)
    w = csm.SyntheticWorld3D(num_nodes=a.nodes, num_submaps=a.submaps, seed=a.seed)
    o = csm.FastCorrelativeScanMatcherOptions3D()
    grids = [(csm.HybridGrid(w.high_resolution, *w.high_cells[s], context=ctx),
              csm.HybridGrid(w.low_resolution, *w.low_cells[s], context=ctx)) for s in range(w.num_submaps)]
    mats = [csm.FastCorrelativeScanMatcher3D(g[0], g[1], w.submap_hist[s], o, ctx)
            for s, g in enumerate(grids)]
    nodes = [w.node(i) for i in range(w.num_nodes)]
    rot = [w.node_rotation(i) for i in range(w.num_nodes)]
    ident = (1.0, 0.0, 0.0, 0.0)
    rng = np.random.RandomState(3)
    pick = [(int(rng.randint(w.num_submaps)), int(rng.randint(w.num_nodes))) for _ in range(a.calls)]

    def one(sn):
        s, n = sn
        return mats[s].MatchFullSubmap(rot[n], ident, nodes[n], 0.6)

    for sn in pick[:32]:
        one(sn)
    lat = []
    for sn in pick[:200]:
        t = time.perf_counter()
        one(sn)
        lat.append((time.perf_counter() - t) * 1e3)
    out = {"single_call_ms": {"median": float(np.median(lat)), "p10": float(np.percentile(lat, 10)),
                              "p90": float(np.percentile(lat, 90))}, "threads": {}}
    # The same pairs as one batch (the batch API's rate on these pairs).
    sub = np.array([s for s, _ in pick], np.int32)
    nod = np.array([n for _, n in pick], np.int32)
    ns = csm.NodeSet3D(nodes)
    pairs = csm.make_pairs_3d(sub, nod, 0.6, True, node_q=np.array(rot)[nod])
    csm.match_batch_3d(mats, ns, pairs, ctx)
    t = time.perf_counter()
    csm.match_batch_3d(mats, ns, pairs, ctx)
    out["batch_pairs_per_s"] = len(pick) / (time.perf_counter() - t)
    for T in [int(x) for x in a.threads.split(",")]:
        with ThreadPoolExecutor(max_workers=T) as ex:
            list(ex.map(one, pick[:2 * T]))
            t = time.perf_counter()
            list(ex.map(one, pick))
            el = time.perf_counter() - t
        out["threads"][str(T)] = {"pairs_per_s": len(pick) / el}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
