"""CPU model of the FastCSM2D device search: how much of its work an early
incumbent would save (design study).

Per pair (C2 world): the quad-mode search's gather count (lane-entries,
clustered lists as the kernel builds them, tools/hex_sim.py) on a sample of
rotations, with nodes pruned at bound <= s_min (no incumbent: what every
rotation chunk starts from) and at bound < S, S = the pair's final best sum
(a perfect incumbent from the start). Matched and unmatched pairs apart.

    python tools/incumbent_sim.py [--pairs 24] [--rots 16]
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
    ap.add_argument("--pairs", type=int, default=24)
    ap.add_argument("--rots", type=int, default=16)
    ap.add_argument("--k", default="1,2,2,4,4,8,8,8,8")
    ap.add_argument("--depth", type=int, default=9)
    ap.add_argument("--min-score", type=float, default=0.55)
    ap.add_argument("--dive", type=int, default=0,
                    help="greedy dive incumbent from every n-th rotation (0: off)")
    args = ap.parse_args()
    ks = [int(v) for v in args.k.split(",")]
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(11)
    D = args.depth
    half = args.pairs // 2
    pairs = [(s, int(world.submap_nodes[s])) for s in rng.choice(50, half, replace=False)]
    pairs += list(zip(rng.randint(0, 50, args.pairs - half), rng.randint(0, 500, args.pairs - half)))
    tot = {"matched": [0, 0, 0, 0], "unmatched": [0, 0, 0, 0]}  # gathers at s_min, at S, pairs, at dive
    for pi, (s, nd) in enumerate(pairs):
        g = world.grid(int(s))
        cells = g.cells
        limits = (g.resolution, g.max_x, g.max_y)
        om = o.fast2d(limits, cells, 7.0, math.radians(30.0), D)
        cloud = world.cloud(int(nd))
        n = len(cloud)
        ok, score, _, _ = om.match_full_submap(cloud, args.min_score)
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

        def score_e(e, fx, fy):
            qx, qy, cnt, w = e
            A = M(w)
            lx = qx[None, :] + fx[:, None] + PAD
            ly = qy[None, :] + fy[:, None] + PAD
            okm = (lx >= 0) & (lx < A.shape[1]) & (ly >= 0) & (ly < A.shape[0])
            v = np.where(okm, A[np.clip(ly, 0, A.shape[0] - 1), np.clip(lx, 0, A.shape[1] - 1)], 0)
            return (v * cnt[None, :]).sum(1)

        cx = g.max_x - 0.5 * g.resolution * cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        s_min = int(math.floor((args.min_score - 0.1) / 0.8 * 255 * n))
        while 0.1 + (s_min + 1) / n * (0.8 / 255) <= args.min_score:
            s_min += 1
        S = int(round((score - 0.1) / 0.8 * 255 * n)) if ok else None
        kind = "matched" if ok else "unmatched"

        def entries(r):
            ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
            ent = []
            for c in range(D):
                k = ks[c]
                if c == 0:
                    ent.append((ix, iy, np.ones(n, np.int64), 1))
                    continue
                qx, qy = (ix // k) * k, (iy // k) * k
                key = qx * 100000 + qy
                head = np.ones(n, bool)
                head[1:] = key[1:] != key[:-1]
                idx = np.nonzero(head)[0]
                cnt = np.diff(np.append(idx, n))
                ent.append((qx[idx], qy[idx], cnt.astype(np.int64), (1 << c) + k - 1))
            return ent

        # Greedy dive per rotation: from the best top-level node, the best
        # child at every level down to a leaf (exact leaf sum).
        S_dive = 0
        if args.dive:
            for r in range(0, ns, args.dive):
                ent = entries(r)
                bx0, bx1, by0, by1 = bounds[r]
                st = 1 << (D - 1)
                fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                         np.arange(by0, by1 + 1, st), indexing="ij")]
                d = D - 1
                while True:
                    sc = score_e(ent[d], fx, fy)
                    b = int(np.argmax(sc))
                    if d == 0:
                        S_dive = max(S_dive, int(sc[b]))
                        break
                    hh = 1 << (d - 1)
                    cx_ = np.array([fx[b] + a * hh for a in range(2) for bb in range(2)])
                    cy_ = np.array([fy[b] + bb * hh for a in range(2) for bb in range(2)])
                    okc = (cx_ <= bx1) & (cy_ <= by1)
                    fx, fy = cx_[okc], cy_[okc]
                    d -= 1
        for r in np.linspace(0, ns - 1, args.rots).astype(int):
            ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
            ent = []
            for c in range(D):
                k = ks[c]
                if c == 0:
                    ent.append((ix, iy, np.ones(n, np.int64), 1))
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
            for slot, thr in ((0, s_min), (1, None if S is None else S - 1),
                              (3, max(s_min, S_dive - 1) if args.dive else None)):
                if thr is None:
                    continue
                fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                         np.arange(by0, by1 + 1, st), indexing="ij")]
                gathers = ((len(fx) + 3) // 4) * len(ent[D - 1][0])
                d = D - 1
                while len(fx):
                    sc = score_e(ent[d], fx, fy)
                    keep = sc > thr
                    fx, fy = fx[keep], fy[keep]
                    if d == 0:
                        break
                    hh = 1 << (d - 1)
                    cx_ = np.concatenate([fx + a * hh for a in range(2) for b in range(2)])
                    cy_ = np.concatenate([fy + b * hh for a in range(2) for b in range(2)])
                    gathers += len(fx) * len(ent[d - 1][0])
                    okc = (cx_ <= bx1) & (cy_ <= by1)
                    fx, fy = cx_[okc], cy_[okc]
                    d -= 1
                tot[kind][slot] += gathers * ns / args.rots
            if S is None:
                tot[kind][1] += 0
        tot[kind][2] += 1
        print(f"pair {pi} ({s},{nd}) {kind} score {score:.3f} rotations {ns} S {S} dive {S_dive} "
              f"s_min {s_min}", flush=True)
    for kind, (a, b, npairs, dv) in tot.items():
        if npairs:
            print(f"{kind}: {npairs} pairs, gathers/pair at s_min {a / npairs:.3g}"
                  + (f", at S {b / npairs:.3g} ({b / a:.2f}x)" if b else "")
                  + (f", at the best dive {dv / npairs:.3g} ({dv / a:.2f}x)" if dv else ""))


if __name__ == "__main__":
    main()
