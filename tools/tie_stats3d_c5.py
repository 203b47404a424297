"""FastCSM3D picks among exactly tied maxima on the C5 workload: the C5
world's first submaps (bench.py's fast3d leg, seed + 5) x all 500 nodes,
MatchFullSubmap on the GPU (one batch) and, for every pair either side
accepts, on the pinned oracle restatement; counts pairs whose score matches
but whose pose differs (an exact tie the device resolved to its smallest
(yaw, x, y, z) leaf). GPU; prints one JSON line.

    python tools/tie_stats3d_c5.py [submaps]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    from test_fast3d_gpu import opt_tuple
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 25
    w = csm.SyntheticWorld3D(num_nodes=500, num_submaps=200, submap_range=(0, S), seed=20250127 + 5)
    o = csm.FastCorrelativeScanMatcherOptions3D()
    grids = [(csm.HybridGrid(w.high_resolution, *w.high_cells[s]),
              csm.HybridGrid(w.low_resolution, *w.low_cells[s])) for s in range(w.num_submaps)]
    mats = [csm.FastCorrelativeScanMatcher3D(g[0], g[1], w.submap_hist[s], o)
            for s, g in enumerate(grids)]
    nodes = csm.NodeSet3D([w.node(i) for i in range(w.num_nodes)])
    sub = np.repeat(np.arange(w.num_submaps), w.num_nodes)
    nod = np.tile(np.arange(w.num_nodes), w.num_submaps)
    rot = np.array([w.node_rotation(n) for n in range(w.num_nodes)])
    pairs = csm.make_pairs_3d(sub, nod, 0.6, True, node_q=rot[nod])
    res = csm.match_batch_3d(mats, nodes, pairs)
    oracle = oracle_lib.Oracle()
    out = {"pairs": int(len(pairs)), "gpu_accepted": int((res["status"] == csm.CSM_OK).sum()),
           "compared": 0, "same_pose": 0, "tie_differs": 0, "mismatch": 0}
    oms = {}
    for i in range(len(pairs)):
        s, n = int(sub[i]), int(nod[i])
        if res["status"][i] != csm.CSM_OK:
            continue
        if s not in oms:
            oh, ol = oracle.hybrid_grid(w.high_resolution), oracle.hybrid_grid(w.low_resolution)
            oh.set_values(*w.high_cells[s])
            ol.set_values(*w.low_cells[s])
            oms[s] = (oh, ol, oracle.fast3d(oh, ol, w.submap_hist[s], opt_tuple(o)))
        ref = oms[s][2].match_full_submap(w.node_rotation(n), (1, 0, 0, 0), w.node(n), 0.6)
        out["compared"] += 1
        if not ref["matched"] or np.float32(ref["score"]) != np.float32(res["score"][i]):
            out["mismatch"] += 1
            continue
        gpose = (tuple(res["t"][i]), tuple(res["q"][i]))
        if gpose == (tuple(ref["pose"][0]), tuple(ref["pose"][1])):
            out["same_pose"] += 1
        else:
            out["tie_differs"] += 1
    print(json.dumps(out))


if __name__ == "__main__":
    main()
