"""Generates the golden vectors in this directory from the pinned oracle.

The reference ships no golden vectors for this path and cannot be built here
(DESIGN.md §2), so the vectors are the oracle's outputs. The oracle is
trusted only after it passes the restated reference unit tests
(oracle/_build/ref_tests). This script checks that first and refuses to write
otherwise.

Fixtures (numpy .npz, no pickles):
* fast2d_c2.npz — BASELINE config C2 shape: 1080-beam scans vs 400x400 @5cm
  submaps, MatchFullSubmap, depth 7, min_score 0.55 (plus a few pairs at
  min_score 0.3 so that failures and weak matches are covered).
* fast2d_local.npz — Match(initial) with the pose_graph.lua window (7 m, 30 deg)
  on decimated (200-point) clouds, initial = truth + noise.
* rt2d_c1.npz — BASELINE config C1 shape: RealTimeCorrelativeScanMatcher2D on
  200x200 @5cm, +-0.2 m / +-10 deg, weights 0.1.

Usage: python tests/golden/make_golden.py   (from the repo root)
"""
import math
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _pack(clouds):
    offs = np.zeros(len(clouds) + 1, np.int64)
    offs[1:] = np.cumsum([len(c) for c in clouds])
    return np.concatenate(clouds).astype(np.float32), offs


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

    # ---- C2-shaped MatchFullSubmap pairs ----------------------------------
    w = csm.SyntheticWorld2D(num_nodes=600, num_submaps=3, submap_cells=400, beams=1080,
                             seed=20250127)
    inside = [_nodes_inside(w, s)[:4] for s in range(3)]
    nodes = sorted(set(sum(inside, [])) | {1, 2})
    rows = []
    for s in range(3):
        for n in inside[s] + [1, 2]:
            rows.append((s, nodes.index(n), 1, 0.0, 0.0, 0.0, 0.55))
    for s in range(3):  # a weaker threshold: the outside nodes' best leaves
        rows.append((s, nodes.index(1), 1, 0.0, 0.0, 0.0, 0.3))
    _write_fast(o, w, [w.cloud(n) for n in nodes], [0, 1, 2], rows, 7.0, math.radians(30.0), 7,
                os.path.join(HERE, "fast2d_c2.npz"), nodes)

    # ---- local Match(initial) pairs ----------------------------------------
    w2 = csm.SyntheticWorld2D(num_nodes=600, num_submaps=2, submap_cells=400, decimate_to=200,
                              seed=4242)
    rng = np.random.default_rng(5)
    inside2 = [_nodes_inside(w2, s)[:6] for s in range(2)]
    nodes2 = sorted(set(sum(inside2, [])) | {3})
    rows2 = []
    for s in range(2):
        for n in inside2[s] + [3]:
            t = w2.node_poses[n] + rng.normal(0, [0.5, 0.5, 0.1])
            rows2.append((s, nodes2.index(n), 0, t[0], t[1], t[2], 0.45))
    _write_fast(o, w2, [w2.cloud(n) for n in nodes2], [0, 1], rows2, 7.0, math.radians(30.0), 7,
                os.path.join(HERE, "fast2d_local.npz"), nodes2)

    # ---- C1-shaped RTCSM2D -------------------------------------------------
    w3 = csm.SyntheticWorld2D(num_nodes=8, num_submaps=2, submap_cells=200, seed=20250128)
    opts = np.array([0.2, math.radians(10.0), 0.1, 0.1])
    clouds, inits, grids, scores, poses, which = [], [], [], [], [], []
    rng = np.random.default_rng(11)
    for s in range(2):
        g = w3.grid(s)
        n = int(w3.submap_nodes[s])
        for k in range(3):
            t = w3.node_poses[n] + rng.uniform(-1, 1, 3) * [0.15, 0.15, math.radians(8)]
            sc, pose, _ = o.rt2d_match((g.resolution, g.max_x, g.max_y), g.cells, tuple(opts),
                                       tuple(t), w3.cloud(n))
            clouds.append(w3.cloud(n))
            inits.append(t)
            scores.append(sc)
            poses.append(pose)
            which.append(s)
    pts, offs = _pack(clouds)
    np.savez_compressed(
        os.path.join(HERE, "rt2d_c1.npz"),
        cells=np.stack([w3.grid(s).cells for s in range(2)]),
        limits=np.array([[w3.grid(s).resolution, w3.grid(s).max_x, w3.grid(s).max_y]
                         for s in range(2)]),
        points=pts, offsets=offs, grid=np.array(which, np.int32), initial=np.array(inits),
        options=opts, score=np.array(scores), pose=np.array(poses))
    for f in ("fast2d_c2.npz", "fast2d_local.npz", "rt2d_c1.npz"):
        print(f, os.path.getsize(os.path.join(HERE, f)), "bytes")


def _nodes_inside(w, s):
    """Nodes whose pose lies inside submap s's window (those can match)."""
    mx, my = w.submap_max[s]
    size = w.submap_size * w.resolution
    p = w.node_poses
    ok = (p[:, 0] < mx - 1) & (p[:, 0] > mx - size + 1) & (p[:, 1] < my - 1) & (p[:, 1] > my - size + 1)
    return [int(i) for i in np.nonzero(ok)[0]]


def _write_fast(o, w, clouds, submaps, rows, lin, ang, depth, path, node_ids):
    rows = np.array(rows, np.float64)
    grids = [w.grid(s) for s in submaps]
    oms = [o.fast2d((g.resolution, g.max_x, g.max_y), g.cells, lin, ang, depth) for g in grids]
    matched, score, pose, lookups = [], [], [], []
    for r in rows:
        s, c, full = int(r[0]), int(r[1]), int(r[2])
        if full:
            ok, sc, p, stats = oms[s].match_full_submap(clouds[c], float(r[6]))
        else:
            ok, sc, p, stats = oms[s].match(tuple(r[3:6]), clouds[c], float(r[6]))
        matched.append(ok)
        score.append(sc)
        pose.append(p)
        lookups.append(int(stats[0]))
    pts, offs = _pack(clouds)
    np.savez_compressed(
        path,
        cells=np.stack([g.cells for g in grids]),
        limits=np.array([[g.resolution, g.max_x, g.max_y] for g in grids]),
        points=pts, offsets=offs, node_ids=np.array(node_ids, np.int32),
        options=np.array([lin, ang, depth]),
        pairs=rows,  # submap, cloud, full_submap, init x, y, theta, min_score
        matched=np.array(matched, np.int32), score=np.array(score, np.float32),
        pose=np.array(pose), reference_lookups=np.array(lookups, np.int64))


if __name__ == "__main__":
    main()
