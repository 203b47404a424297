"""Generates the 3D golden vectors in this directory from the pinned oracle
(same contract as make_golden.py: the oracle must first pass the restated
reference unit tests, oracle/_build/ref_tests, which include the 3D ones).

Fixtures (numpy .npz, no pickles):
* fast3d_c5.npz — BASELINE config C5 shape, scaled to stay small: 0.10 m /
  0.45 m HybridGrids built from 32-ring scans of a 20x20x5 m world,
  ~160-point high-resolution node clouds, 120-bucket rotational histograms,
  the pose_graph.lua 3D options; MatchFullSubmap at min_score 0.55 down to 0.3,
  and Match(initial = truth + offset) at 0.45 (the scaled world scores lower
  than C5's, so lower thresholds keep accepted matches in the set).
* rt3d_c4.npz — BASELINE config C4 shape, scaled: RealTimeCorrelativeScanMatcher3D
  on the same 0.10 m grids, 1500-point scans, +-0.1 m / +-2 deg, weights 0.1.

Usage: python tests/golden/make_golden3d.py   (from the repo root)
"""
import math
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))

WORLD = dict(world_x=20., world_y=20., world_z=5., num_boxes=12, rings=32, azimuths=360,
             scans_per_submap=4, max_range=15.)


def _pack(clouds):
    offs = np.zeros(len(clouds) + 1, np.int64)
    offs[1:] = np.cumsum([len(c) for c in clouds])
    return np.concatenate(clouds).astype(np.float32), offs


def _pack_cells(cells):
    offs = np.zeros(len(cells) + 1, np.int64)
    offs[1:] = np.cumsum([len(v) for _, v in cells])
    return (np.concatenate([i for i, _ in cells]).astype(np.int32),
            np.concatenate([v for _, v in cells]).astype(np.uint16), offs)


def main():
    from conftest import ensure_built, load_package
    ensure_built()
    rc = subprocess.call([os.path.join(ROOT, "oracle", "_build", "ref_tests")],
                         stdout=subprocess.DEVNULL)
    if rc != 0:
        raise SystemExit("oracle fails the restated reference tests; not writing fixtures")
    import oracle_lib
    csm = load_package()  # synthetic-world generator only (no GPU needed)
    o = oracle_lib.Oracle()
    w = csm.SyntheticWorld3D(num_nodes=16, num_submaps=3, seed=20250127, **WORLD)
    f = csm.FastCorrelativeScanMatcherOptions3D()  # pose_graph.lua:40-48
    opts = (f.branch_and_bound_depth, f.full_resolution_depth, f.min_rotational_score,
            f.min_low_resolution_score, f.linear_xy_search_window, f.linear_z_search_window,
            f.angular_search_window)
    oms = []
    for s in range(w.num_submaps):
        oh, ol = o.hybrid_grid(w.high_resolution), o.hybrid_grid(w.low_resolution)
        oh.set_values(*w.high_cells[s])
        ol.set_values(*w.low_cells[s])
        oms.append((oh, ol, o.fast3d(oh, ol, w.submap_hist[s], opts)))

    # ---- C5-shaped pairs ----------------------------------------------------
    ident = ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))
    rows = []  # submap, node, full, min_score, node_t(3), node_q(4), submap_t(3), submap_q(4)
    for s in range(w.num_submaps):
        c = int(w.submap_nodes[s])
        for n, ms in [(c, 0.55), ((c + 1) % 16, 0.5), ((c + 5) % 16, 0.45), ((c + 9) % 16, 0.3)]:
            rows.append((s, n, 1, ms, (0, 0, 0), w.node_rotation(n), ident[0], ident[1]))
        for n in [c, (c + 2) % 16]:
            truth = w.node_in_submap(n, s)
            init = ((truth[0][0] + 0.3, truth[0][1] - 0.2, 0.1), truth[1])
            rows.append((s, n, 0, 0.45, init[0], init[1], ident[0], ident[1]))
    out = {k: [] for k in ("matched", "score", "t", "q", "rotational_score",
                           "low_resolution_score", "lookups")}
    for s, n, full, ms, nt, nq, st, sq in rows:
        om = oms[s][2]
        r = (om.match_full_submap(nq, sq, w.node(n), ms) if full
             else om.match((nt, nq), (st, sq), w.node(n), ms))
        out["matched"].append(int(r["matched"]))
        out["score"].append(r["score"])
        out["t"].append(r["pose"][0])
        out["q"].append(r["pose"][1])
        out["rotational_score"].append(r["rotational_score"])
        out["low_resolution_score"].append(r["low_resolution_score"])
        out["lookups"].append(r["lookups"])
    hi_idx, hi_val, hi_off = _pack_cells(w.high_cells)
    lo_idx, lo_val, lo_off = _pack_cells(w.low_cells)
    hpts, hoff = _pack(w.high)
    lpts, loff = _pack(w.low)
    pairs = np.array([(s, n, full, ms, *nt, *nq, *st, *sq)
                      for s, n, full, ms, nt, nq, st, sq in rows], np.float64)
    np.savez_compressed(
        os.path.join(HERE, "fast3d_c5.npz"),
        high_resolution=np.float64(w.high_resolution), low_resolution=np.float64(w.low_resolution),
        high_idx=hi_idx, high_val=hi_val, high_off=hi_off,
        low_idx=lo_idx, low_val=lo_val, low_off=lo_off,
        submap_hist=np.stack(w.submap_hist).astype(np.float32),
        high_points=hpts, high_offsets=hoff, low_points=lpts, low_offsets=loff,
        node_hist=np.stack(w.node_hist).astype(np.float32),
        options=np.array(opts, np.float64),
        pairs=pairs,  # submap, node, full, min_score, node t3 q4, submap t3 q4
        matched=np.array(out["matched"], np.int32), score=np.array(out["score"], np.float32),
        t=np.array(out["t"]), q=np.array(out["q"]),
        rotational_score=np.array(out["rotational_score"], np.float32),
        low_resolution_score=np.array(out["low_resolution_score"], np.float32),
        reference_lookups=np.array(out["lookups"], np.int64))

    # ---- C4-shaped RTCSM3D ----------------------------------------------------
    rt_opts = (0.1, math.radians(2.0), 0.1, 0.1)
    rng = np.random.default_rng(7)
    cases = []
    for s in range(2):
        c = int(w.submap_nodes[s])
        raw = w.raw[c]
        cloud = raw[rng.choice(len(raw), 1500, replace=False)].astype(np.float32)
        for k in range(2):
            truth = w.node_in_submap(c, s)
            init = ((truth[0][0] + rng.uniform(-0.08, 0.08), truth[0][1] + rng.uniform(-0.08, 0.08),
                     rng.uniform(-0.05, 0.05)), truth[1])
            sc, pose, idx, ncand = o.rt3d_match(oms[s][0], rt_opts, init, cloud)
            cases.append((s, cloud, init, sc, pose, idx, ncand))
    cpts, coff = _pack([c[1] for c in cases])
    np.savez_compressed(
        os.path.join(HERE, "rt3d_c4.npz"),
        options=np.array(rt_opts), grid=np.array([c[0] for c in cases], np.int32),
        points=cpts, offsets=coff,
        initial=np.array([(*c[2][0], *c[2][1]) for c in cases]),
        score=np.array([c[3] for c in cases], np.float32),
        pose=np.array([(*c[4][0], *c[4][1]) for c in cases]),
        candidate=np.array([c[5] for c in cases], np.int64),
        candidates=np.array([c[6] for c in cases], np.int64))
    for name in ("fast3d_c5.npz", "rt3d_c4.npz"):
        print(name, os.path.getsize(os.path.join(HERE, name)), "bytes")
    print("matched", sum(out["matched"]), "of", len(rows))


if __name__ == "__main__":
    main()
