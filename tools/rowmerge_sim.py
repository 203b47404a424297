"""CPU model of row-merged quad scoring (design study, round 5).

A quad node at level d scores its 4 children with one dword gather per entry
of its list from quad plane Q_{d-1}. Its x-siblings (the same parent, the
same row b) sit in the next dwords of that plane (polyphase, period 2^d), so
one lane could score a whole surviving row of siblings with one 8-byte (quad
parent: rows of 2) or 16-byte (hex parent: rows of 4) load. This counts, per
child level, the gather instructions' lane-entries with and without merging
under threshold-only pruning (the node set of a non-matching pair), with the
kernel's default hex levels and cluster sizes.

    python tools/rowmerge_sim.py [--pairs 3] [--rots 12]
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
    ap.add_argument("--k", default="1,1,4,4,4,8,8,8,8", help="k per child level 0..8")
    ap.add_argument("--hex", default="8,6")
    ap.add_argument("--depth", type=int, default=9)
    ap.add_argument("--min-score", type=float, default=0.55)
    args = ap.parse_args()
    ks = [int(v) for v in args.k.split(",")]
    hexl = [int(v) for v in args.hex.split(",") if v]
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(5)
    D = args.depth
    plain = np.zeros(D + 1)   # lane-entries per child level, one node per lane
    merged = np.zeros(D + 1)  # one surviving sibling row per lane
    nodes = np.zeros(D + 1)
    rows = np.zeros(D + 1)
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
            out = np.zeros(len(fx), np.int64)
            for a in range(0, len(fx), 4096):
                lx = qx[None, :] + fx[a:a + 4096, None] + PAD
                ly = qy[None, :] + fy[a:a + 4096, None] + PAD
                ok = (lx >= 0) & (lx < A.shape[1]) & (ly >= 0) & (ly < A.shape[0])
                v = np.where(ok, A[np.clip(ly, 0, A.shape[0] - 1), np.clip(lx, 0, A.shape[1] - 1)], 0)
                out[a:a + 4096] = (v * cnt[None, :]).sum(1)
            return out

        cloud = world.cloud(nd)
        n = len(cloud)
        cx = g.max_x - 0.5 * g.resolution * cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        s_min = int(math.floor((args.min_score - 0.1) / 0.8 * 255 * n))
        for r in np.linspace(0, ns - 1, args.rots).astype(int):
            R += 1
            ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
            ent = []
            for c in range(D):
                k = ks[c]
                if k == 1:
                    ent.append((ix, iy, np.ones(n, np.int64), 1 << c))
                    continue
                qx, qy = (ix // k) * k, (iy // k) * k
                key = qx * 100000 + qy
                head = np.ones(n, bool)
                head[1:] = key[1:] != key[:-1]
                idx = np.nonzero(head)[0]
                cnt = np.diff(np.append(idx, n))
                ent.append((qx[idx], qy[idx], cnt.astype(np.int64), (1 << c) + k - 1))
            bx0, bx1, by0, by1 = bounds[r]
            st = 1 << (D - 1)
            fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                     np.arange(by0, by1 + 1, st), indexing="ij")]
            gid = np.arange(len(fx))
            d = D - 1
            while len(fx):
                sc = score(ent[d], fx, fy)
                keep = sc > s_min
                fx, fy, gid = fx[keep], fy[keep], gid[keep]
                if d == 0:
                    break
                two = d in hexl and d >= 2
                m = 4 if two else 2
                hh = 1 << (d - (2 if two else 1))
                if not two:
                    L = len(ent[d - 1][0])
                    plain[d - 1] += len(fx) * L
                    merged[d - 1] += len(np.unique(gid)) * L
                    nodes[d - 1] += len(fx)
                    rows[d - 1] += len(np.unique(gid))
                par = np.repeat(np.arange(len(fx)), 1)
                cx_ = np.concatenate([fx + a * hh for b in range(m) for a in range(m)])
                cy_ = np.concatenate([fy + b * hh for b in range(m) for a in range(m)])
                cg = np.concatenate([par * m + b for b in range(m) for a in range(m)])
                ok = (cx_ <= bx1) & (cy_ <= by1)
                fx, fy, gid = cx_[ok], cy_[ok], cg[ok]
                d -= 2 if two else 1
        print(f"pair {pi} done ({ns} rotations)", flush=True)
    print("child level: nodes/rot, rows/rot, quad lane-entries/rot plain -> merged")
    for c in range(D):
        if plain[c]:
            print(f"  L{c}: {nodes[c] / R:9.1f} {rows[c] / R:9.1f}  {plain[c] / R:12.0f} -> "
                  f"{merged[c] / R:12.0f} ({merged[c] / plain[c]:.2f})")
    print(f"  all quad: {plain.sum() / R:.0f} -> {merged.sum() / R:.0f} "
          f"({merged.sum() / plain.sum():.2f})")


if __name__ == "__main__":
    main()
