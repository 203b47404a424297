"""CPU model of split-list scoring (design study, round 5).

Each scan's entry lists are cut at point index n * f into a head and a tail
(a run crossing the cut becomes two entries). A node carries its head and
tail sums from its parent's scoring. Its children are first scored over the
head lists only; child head + the node's own tail sum bounds each child
(the node's tail entries cover the child's at every level: clusters nest and
a coarser level's max covers the finer window), so a node whose children
all fall to <= min_sum on that bound skips the tail gathers. Counts lane-
entries (gather work) per child level with and without the cut, under
threshold-only pruning with the kernel's hex levels and cluster sizes.

    python tools/split_bound_sim.py [--pairs 2] [--rots 8] [--cut 0.5]
"""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def runs(ix, iy, k, lo, hi):
    qx, qy = (ix[lo:hi] // k) * k, (iy[lo:hi] // k) * k
    m = hi - lo
    if m == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64)
    key = qx * 100000 + qy
    head = np.ones(m, bool)
    head[1:] = key[1:] != key[:-1]
    idx = np.nonzero(head)[0]
    cnt = np.diff(np.append(idx, m))
    return qx[idx], qy[idx], cnt.astype(np.int64)


def main():
    from scipy.ndimage import maximum_filter
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2)
    ap.add_argument("--rots", type=int, default=8)
    ap.add_argument("--k", default="1,1,4,4,4,8,8,8,8", help="k per child level 0..8")
    ap.add_argument("--hex", default="8,6")
    ap.add_argument("--depth", type=int, default=9)
    ap.add_argument("--cut", default="0.5", help="head fraction(s), comma separated")
    ap.add_argument("--min-score", type=float, default=0.55)
    ap.add_argument("--frac-bits", type=int, default=0, help="node tail sum kept as a rounded-up "
                    "fraction of the node's sum with this many bits (0: exact)")
    args = ap.parse_args()
    ks = [int(v) for v in args.k.split(",")]
    hexl = [int(v) for v in args.hex.split(",") if v]
    cuts = [float(c) for c in args.cut.split(",")]
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(5)
    D = args.depth
    base = np.zeros(D + 1)
    split = {c: np.zeros(D + 1) for c in cuts}
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

        def score(e, w, fx, fy):
            qx, qy, cnt = e
            A = M(w)
            out = np.zeros(len(fx), np.int64)
            if len(qx) == 0:
                return out
            for a in range(0, len(fx), 2048):
                lx = qx[None, :] + fx[a:a + 2048, None] + PAD
                ly = qy[None, :] + fy[a:a + 2048, None] + PAD
                ok = (lx >= 0) & (lx < A.shape[1]) & (ly >= 0) & (ly < A.shape[0])
                v = np.where(ok, A[np.clip(ly, 0, A.shape[0] - 1), np.clip(lx, 0, A.shape[1] - 1)], 0)
                out[a:a + 2048] = (v * cnt[None, :]).sum(1)
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
            W = [(1 << c) + ks[c] - 1 for c in range(D)]
            full = [runs(ix, iy, ks[c], 0, n) for c in range(D)]
            bx0, bx1, by0, by1 = bounds[r]
            st = 1 << (D - 1)
            for variant in [None] + cuts:
                h = n if variant is None else int(round(n * variant))
                head = [runs(ix, iy, ks[c], 0, h) for c in range(D)]
                tail = [runs(ix, iy, ks[c], h, n) for c in range(D)]
                fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                         np.arange(by0, by1 + 1, st), indexing="ij")]
                d = D - 1
                A = score(head[d], W[d], fx, fy)
                B = score(tail[d], W[d], fx, fy)
                keep = A + B > s_min
                fx, fy, A, B = fx[keep], fy[keep], A[keep], B[keep]
                acc = base if variant is None else split[variant]
                while len(fx) and d > 0:
                    two = d in hexl and d >= 2
                    m = 4 if two else 2
                    c = d - (2 if two else 1)
                    hh = 1 << c
                    par = np.concatenate([np.arange(len(fx))] * (m * m))
                    cx_ = np.concatenate([fx + a * hh for b in range(m) for a in range(m)])
                    cy_ = np.concatenate([fy + b * hh for b in range(m) for a in range(m)])
                    ok = (cx_ <= bx1) & (cy_ <= by1)
                    if variant is None:
                        acc[c] += len(fx) * len(full[c][0])
                        sc = score(full[c], W[c], cx_, cy_)
                        keep = ok & (sc > s_min)
                        fx, fy = cx_[keep], cy_[keep]
                        A = B = np.zeros(len(fx), np.int64)
                    else:
                        ca = score(head[c], W[c], cx_, cy_)
                        Bn = B[par]
                        if args.frac_bits:
                            q = 1 << args.frac_bits
                            S = np.maximum(A + B, 1)[par]
                            fr = np.maximum(0, -(-Bn * q // S) - 1)
                            Bn = -(-S * (fr + 1) // q)
                        bound = ca + Bn
                        live = np.zeros(len(fx), bool)
                        np.logical_or.at(live, par[ok & (bound > s_min)], True)
                        acc[c] += len(fx) * len(head[c][0]) + live.sum() * len(tail[c][0])
                        sel = ok & live[par]
                        cb = np.zeros(len(cx_), np.int64)
                        cb[sel] = score(tail[c], W[c], cx_[sel], cy_[sel])
                        keep = sel & (ca + cb > s_min)
                        fx, fy, A, B = cx_[keep], cy_[keep], ca[keep], cb[keep]
                    d = c
        print(f"pair {pi} done ({ns} rotations)", flush=True)
    print("child level: lane-entries per rotation, full lists -> split at each cut")
    for c in range(D):
        if base[c]:
            row = "  ".join(f"{cut}: {split[cut][c] / R:10.0f} ({split[cut][c] / base[c]:.2f})" for cut in cuts)
            print(f"  L{c}: {base[c] / R:10.0f}   {row}")
    row = "  ".join(f"{cut}: {split[cut].sum() / base.sum():.3f}" for cut in cuts)
    print(f"  all: {base.sum() / R:.0f}   {row}")


if __name__ == "__main__":
    main()
