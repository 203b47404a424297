"""Design study: can a cheap per-rotation bound find the best rotation early?

For matched C2-world pairs: every rotation's best top-level bound (level-L
nodes of the search lattice scored with the k-cell cluster list, as the
device does) and the rank of the rotation holding the pair's best leaf in
that order. If it ranks near the top, searching the top rotations first would
give the pair's final best as the incumbent for the rest.

    python tools/rotation_rank_sim.py [--pairs 8] [--level 8]
"""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    from scipy.ndimage import maximum_filter
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=8)
    ap.add_argument("--levels", default="8,6")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--depth", type=int, default=9)
    ap.add_argument("--min-score", type=float, default=0.55)
    args = ap.parse_args()
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(5)
    subs = rng.choice(50, args.pairs, replace=False)
    for s in subs:
        nd = int(world.submap_nodes[s])
        g = world.grid(int(s))
        limits = (g.resolution, g.max_x, g.max_y)
        om = o.fast2d(limits, g.cells, 7.0, math.radians(30.0), args.depth)
        cloud = world.cloud(nd)
        ok, score, pose, _ = om.match_full_submap(cloud, args.min_score)
        if not ok:
            print(f"submap {s} node {nd}: unmatched")
            continue
        G0 = om.level(0).astype(np.int64)
        PAD = 600
        Gp = np.zeros((G0.shape[0] + 2 * PAD, G0.shape[1] + 2 * PAD), np.int64)
        Gp[PAD:PAD + G0.shape[0], PAD:PAD + G0.shape[1]] = G0
        cx = g.max_x - 0.5 * g.resolution * g.cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * g.cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, g.cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        n_ang = (ns - 1) // 2
        th = math.atan2(math.sin(pose[2]), math.cos(pose[2]))
        r_star = int(round(th / step)) + n_ang
        k = args.k
        line = f"submap {s} node {nd}: score {score:.3f} rotations {ns} best rotation {r_star}"
        for L in [int(v) for v in args.levels.split(",")]:
            w = (1 << L) + k - 1
            A = maximum_filter(Gp, size=(w, w), origin=(-(w // 2), -(w // 2)), mode="constant", cval=0)
            B = np.zeros(ns)
            for r in range(ns):
                ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
                qx, qy = (ix // k) * k, (iy // k) * k
                key = qx * 100000 + qy
                head = np.ones(len(key), bool)
                head[1:] = key[1:] != key[:-1]
                idx = np.nonzero(head)[0]
                cnt = np.diff(np.append(idx, len(key)))
                qx, qy = qx[idx], qy[idx]
                bx0, bx1, by0, by1 = bounds[r]
                st = 1 << L
                fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                         np.arange(by0, by1 + 1, st), indexing="ij")]
                lx = qx[None, :] + fx[:, None] + PAD
                ly = qy[None, :] + fy[:, None] + PAD
                v = A[np.clip(ly, 0, A.shape[0] - 1), np.clip(lx, 0, A.shape[1] - 1)]
                B[r] = (v * cnt[None, :]).sum(1).max()
            order = np.argsort(-B, kind="stable")
            rank = int(np.nonzero(order == r_star)[0][0])
            near = min(int(np.nonzero(np.abs(order - r_star) <= 2)[0][0]), rank)
            S = (score - 0.1) / 0.8 * 255 * len(cloud)
            line += (f" | level {L}: rank {rank} ({rank / ns:.1%}), a rotation within 2 at {near},"
                     f" bound/S {B[r_star] / S:.3f} (mirror {B[ns - 1 - r_star] / S:.3f}, max {B.max() / S:.3f})")
        print(line, flush=True)


if __name__ == "__main__":
    main()
