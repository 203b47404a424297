"""Generates tests/golden/rt2d_tsdf.npz from the pinned oracle.

RealTimeCorrelativeScanMatcher2D over TSDF2D grids in the C1 shape: 1080-beam
scans vs 200x200 @5cm windows, +-0.2 m / +-10 deg, weights 0.1. The grids are
built with the restated TSDFRangeDataInserter2D and the
trajectory_builder_2d.lua:100-112 inserter options (truncation 0.3 m, max
weight 10, normal projection, 0.5 kernel bandwidths) from the synthetic
world's node scans (hits outside the window are dropped so the grid keeps its
200x200 limits). Written only after the oracle passes the restated reference
tests, TSDF ones included.

Usage: python tests/golden/make_golden_tsdf.py   (from the repo root)
"""
import math
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))

TRUNCATION, MAX_WEIGHT = 0.3, 10.0
INSERTER = (TRUNCATION, MAX_WEIGHT, 0, 4, 0.5, 1, 0, 0.5, 0.5)


def world_scan(w, n):
    """Node n's scan in the world frame (origin, returns)."""
    x, y, th = w.node_poses[n]
    c = w.cloud(n).astype(np.float64)
    ct, st = math.cos(th), math.sin(th)
    out = np.stack([ct * c[:, 0] - st * c[:, 1] + x, st * c[:, 0] + ct * c[:, 1] + y,
                    np.zeros(len(c))], axis=1)
    return (x, y, 0.0), out.astype(np.float32)


def build_tsdf(o, w, s, nodes):
    mx, my = w.submap_max[s]
    size = w.submap_size * w.resolution
    inserts = []
    for n in nodes:
        origin, pts = world_scan(w, n)
        keep = ((pts[:, 0] < mx - 0.4) & (pts[:, 0] > mx - size + 0.4) &
                (pts[:, 1] < my - 0.4) & (pts[:, 1] > my - size + 0.4))
        inserts.append((origin, pts[keep]))
    return o.tsdf_from_inserts(w.resolution, float(mx), float(my), w.submap_size, w.submap_size,
                               TRUNCATION, MAX_WEIGHT, inserts, INSERTER)


def nodes_inside(w, s, margin=1.0):
    mx, my = w.submap_max[s]
    size = w.submap_size * w.resolution
    p = w.node_poses
    ok = ((p[:, 0] < mx - margin) & (p[:, 0] > mx - size + margin) &
          (p[:, 1] < my - margin) & (p[:, 1] > my - size + margin))
    return [int(i) for i in np.nonzero(ok)[0]]


def main():
    from conftest import ensure_built, load_package
    ensure_built()
    rc = subprocess.call([os.path.join(ROOT, "oracle", "_build", "ref_tests")],
                         stdout=subprocess.DEVNULL)
    if rc != 0:
        raise SystemExit("oracle fails the restated reference tests; not writing fixtures")
    import oracle_lib
    csm = load_package()
    o = oracle_lib.Oracle()
    w = csm.SyntheticWorld2D(num_nodes=600, num_submaps=2, submap_cells=200, seed=20250129)
    opts = np.array([0.2, math.radians(10.0), 0.1, 0.1])
    rng = np.random.default_rng(17)
    out = {"options": opts, "truncation": np.float32(TRUNCATION),
           "max_weight": np.float32(MAX_WEIGHT)}
    clouds, inits, scores, poses, which = [], [], [], [], []
    for s in range(2):
        inside = nodes_inside(w, s)
        assert len(inside) >= 2, inside
        lim, tsd, wgt = build_tsdf(o, w, s, inside[:8])
        out[f"limits_{s}"] = np.array(lim)
        out[f"tsd_{s}"] = tsd
        out[f"wgt_{s}"] = wgt
        for n in inside[:3]:
            t = w.node_poses[n] + rng.uniform(-1, 1, 3) * [0.15, 0.15, math.radians(8)]
            sc, pose, _ = o.rt2d_match_tsdf(lim, tsd, wgt, TRUNCATION, MAX_WEIGHT, tuple(opts),
                                            tuple(t), w.cloud(n))
            clouds.append(w.cloud(n))
            inits.append(t)
            scores.append(sc)
            poses.append(pose)
            which.append(s)
    offs = np.zeros(len(clouds) + 1, np.int64)
    offs[1:] = np.cumsum([len(c) for c in clouds])
    out.update(points=np.concatenate(clouds).astype(np.float32), offsets=offs,
               grid=np.array(which, np.int32), initial=np.array(inits), score=np.array(scores),
               pose=np.array(poses))
    path = os.path.join(HERE, "rt2d_tsdf.npz")
    np.savez_compressed(path, **out)
    print(path, os.path.getsize(path), "bytes", "scores", np.round(scores, 4))


if __name__ == "__main__":
    main()
