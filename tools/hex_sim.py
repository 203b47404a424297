"""CPU model of the FastCSM2D search with two-level ("hex") expansions
(design study for the 16-byte grandchild planes).

A node at level d expanded in quad mode scores its 4 children at level d-1
(one dword gather per child-level list entry); in hex mode it scores its 16
grandchildren at level d-2 directly (one dwordx4 gather per entry of the
level d-2 list), skipping the pruning at level d-1. Threshold-only pruning
(min_score, no incumbent), clustered lists as the kernel (k per child level).
Reports gather instructions (lane-entries) per rotation by mode set.

    python tools/hex_sim.py [--pairs 3] [--rots 12] [--hex 8,6] [--k 1,2,2,4,4,8,8,8,8]
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
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--rots", type=int, default=12)
    ap.add_argument("--k", default="1,2,2,4,4,8,8,8,8", help="k per child level 0..8")
    ap.add_argument("--hex", default="", help="node levels expanded two levels at once; "
                    "several sets separated by ';'")
    ap.add_argument("--depth", type=int, default=9)
    args = ap.parse_args()
    ks = [int(v) for v in args.k.split(",")]
    sets = [[int(v) for v in h.split(",") if v] for h in args.hex.split(";")]
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(5)
    D = args.depth
    tot = {tuple(h): {"quad": 0, "hex": 0, "nodes": [0] * (D + 1)} for h in sets}
    R = 0
    for pi in range(args.pairs):
        s = int(rng.randint(world.num_submaps))
        nd = int(rng.randint(world.num_nodes))
        g = world.grid(s)
        cells = g.cells
        limits = (g.resolution, g.max_x, g.max_y)
        om = o.fast2d(limits, cells, 7.0, math.radians(30.0), D)
        G0 = om.level(0).astype(np.int64)
        PAD = 600
        Gp = np.zeros((G0.shape[0] + 2 * PAD, G0.shape[1] + 2 * PAD), np.int64)
        Gp[PAD:PAD + G0.shape[0], PAD:PAD + G0.shape[1]] = G0
        cache = {}

        def M(w):
            if w not in cache:
                cache[w] = maximum_filter(Gp, size=(w, w), origin=(-(w // 2), -(w // 2)),
                                          mode="constant", cval=0) if w > 1 else Gp
            return cache[w]

        def score(e, fx, fy):
            qx, qy, cnt, w = e
            A = M(w)
            lx = qx[None, :] + fx[:, None] + PAD
            ly = qy[None, :] + fy[:, None] + PAD
            ok = (lx >= 0) & (lx < A.shape[1]) & (ly >= 0) & (ly < A.shape[0])
            v = np.where(ok, A[np.clip(ly, 0, A.shape[0] - 1), np.clip(lx, 0, A.shape[1] - 1)], 0)
            return (v * cnt[None, :]).sum(1)

        cloud = world.cloud(nd)
        n = len(cloud)
        cx = g.max_x - 0.5 * g.resolution * cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        s_min = int(math.floor((0.55 - 0.1) / 0.8 * 255 * n))
        for r in np.linspace(0, ns - 1, args.rots).astype(int):
            R += 1
            ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
            ent = []
            for c in range(D):
                k = ks[c]
                if c == 0:
                    ent.append((ix, iy, np.ones(n, np.int64), 1))
                    continue
                qx, qy = (ix // k) * k, (iy // k) * k
                key = qx * 100000 + qy
                # run list (consecutive equal keys), as the kernel builds it
                head = np.ones(n, bool)
                head[1:] = key[1:] != key[:-1]
                idx = np.nonzero(head)[0]
                cnt = np.diff(np.append(idx, n))
                ent.append((qx[idx], qy[idx], cnt.astype(np.int64), (1 << c) + k - 1))
            bx0, bx1, by0, by1 = bounds[r]
            st = 1 << (D - 1)
            for h in sets:
                T = tot[tuple(h)]
                # virtual roots at level D scoring level D-1 children
                fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                         np.arange(by0, by1 + 1, st), indexing="ij")]
                T["quad"] += ((len(fx) + 3) // 4) * len(ent[D - 1][0])
                d = D - 1
                while len(fx):
                    sc = score(ent[d], fx, fy)
                    keep = sc > s_min
                    fx, fy = fx[keep], fy[keep]
                    if d == 0:
                        break
                    T["nodes"][d] += len(fx)
                    two = d in h and d >= 2
                    step_ = 2 if two else 1
                    hh = 1 << (d - step_)
                    m = 1 << step_
                    cx_ = np.concatenate([fx + a * hh for a in range(m) for b in range(m)])
                    cy_ = np.concatenate([fy + b * hh for a in range(m) for b in range(m)])
                    if two:
                        T["hex"] += len(fx) * len(ent[d - 2][0])
                    else:
                        T["quad"] += len(fx) * len(ent[d - 1][0])
                    ok = (cx_ <= bx1) & (cy_ <= by1)
                    fx, fy = cx_[ok], cy_[ok]
                    d -= step_
        print(f"pair {pi} done ({ns} rotations)", flush=True)
    for h in sets:
        T = tot[tuple(h)]
        print(f"hex levels {h or 'none'}: quad gathers/rot {T['quad'] / R:.0f}, hex gathers/rot "
              f"{T['hex'] / R:.0f}, total {(T['quad'] + T['hex']) / R:.0f}; expanded/rot "
              f"{[round(v / R, 1) for v in T['nodes']]}")


if __name__ == "__main__":
    main()
