"""How often the FastCSM3D device search returns a different (exactly tied)
leaf than the reference's pick: the C5 golden pairs (tests/golden/fast3d_c5.npz,
reference poses from the pinned oracle) and a synthetic C5-shaped sweep
compared against the oracle. GPU; prints one JSON line."""
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
    from test_golden import _load, _cells3, _node3, _pair3
    from test_fast3d_gpu import opt_tuple
    d = _load("fast3d_c5.npz")
    o = csm.FastCorrelativeScanMatcherOptions3D(*[int(v) if i < 2 else float(v)
                                                   for i, v in enumerate(d["options"])])
    mats = []
    for s in range(len(d["submap_hist"])):
        gh = csm.HybridGrid(float(d["high_resolution"]), *_cells3(d, "high", s))
        gl = csm.HybridGrid(float(d["low_resolution"]), *_cells3(d, "low", s))
        mats.append((gh, gl, csm.FastCorrelativeScanMatcher3D(gh, gl, d["submap_hist"][s], o)))
    nodes = [_node3(csm, d, n) for n in range(len(d["node_hist"]))]
    out = {"golden": {"matched": 0, "same_pose": 0, "differs": []}}
    for i, row in enumerate(d["pairs"]):
        s, n, full, ms, npose, spose = _pair3(row)
        m = mats[s][2]
        r = m.MatchFullSubmap(npose[1], spose[1], nodes[n], ms) if full else m.Match(npose, spose, nodes[n], ms)
        if r is None or not d["matched"][i]:
            continue
        out["golden"]["matched"] += 1
        ref = (tuple(d["t"][i]), tuple(d["q"][i]))
        if r.pose_estimate == ref:
            out["golden"]["same_pose"] += 1
        else:
            dt = float(np.linalg.norm(np.subtract(r.pose_estimate[0], ref[0])))
            out["golden"]["differs"].append({"pair": i, "d_translation_m": dt})
    # Synthetic sweep against the oracle.
    o2 = csm.FastCorrelativeScanMatcherOptions3D()
    w = csm.SyntheticWorld3D(num_nodes=40, num_submaps=4, seed=7)
    oracle = oracle_lib.Oracle()
    syn = {"matched": 0, "same_pose": 0, "differs": 0}
    for s in range(w.num_submaps):
        oh, ol = oracle.hybrid_grid(w.high_resolution), oracle.hybrid_grid(w.low_resolution)
        oh.set_values(*w.high_cells[s])
        ol.set_values(*w.low_cells[s])
        om = oracle.fast3d(oh, ol, w.submap_hist[s], opt_tuple(o2))
        gh = csm.HybridGrid(w.high_resolution, *w.high_cells[s])
        gl = csm.HybridGrid(w.low_resolution, *w.low_cells[s])
        gm = csm.FastCorrelativeScanMatcher3D(gh, gl, w.submap_hist[s], o2)
        for n in range(w.num_nodes):
            node = w.node(n)
            ref = om.match_full_submap(w.node_rotation(n), (1, 0, 0, 0), node, 0.55)
            gpu = gm.MatchFullSubmap(w.node_rotation(n), (1, 0, 0, 0), node, 0.55)
            if gpu is None or not ref["matched"]:
                continue
            syn["matched"] += 1
            if tuple(map(tuple, gpu.pose_estimate)) == tuple(map(tuple, ref["pose"])):
                syn["same_pose"] += 1
            else:
                syn["differs"] += 1
    out["synthetic_full_submap"] = syn
    print(json.dumps(out))


if __name__ == "__main__":
    main()
