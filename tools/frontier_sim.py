"""CPU model of the FastCSM2D full-submap search frontier (design study).

For a few C2 pairs it runs the branch and bound level by level with the
min_score threshold only (the node set every non-matching pair explores,
whatever the traversal order), over a sample of rotations, and reports per
level: nodes expanded, lattice density, and the distinct 128-byte lines one
64-lane gather touches when 64 frontier nodes x 1 run-list entry are issued
together under several orderings / plane layouts.

    python tools/frontier_sim.py [--pairs 4] [--rots 24]
"""
import argparse
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def morton(x, y):
    def spread(v):
        v = v.astype(np.int64) & 0xffff
        v = (v | (v << 8)) & 0x00ff00ff
        v = (v | (v << 4)) & 0x0f0f0f0f
        v = (v | (v << 2)) & 0x33333333
        v = (v | (v << 1)) & 0x55555555
        return v
    return spread(x) | (spread(y) << 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--rots", type=int, default=24)
    ap.add_argument("--depth", type=int, default=9)
    args = ap.parse_args()
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(5)
    D = args.depth
    tot = {}
    for pi in range(args.pairs):
        s = int(rng.randint(world.num_submaps))
        nd = int(rng.randint(world.num_nodes))
        g = world.grid(s)
        cells = g.cells
        limits = (g.resolution, g.max_x, g.max_y)
        om = o.fast2d(limits, cells, 7.0, math.radians(30.0), D)
        levels = [om.level(d).astype(np.int64) for d in range(D)]
        cloud = world.cloud(nd)
        n = len(cloud)
        # MatchFullSubmap: window centred on the submap, 1e6 m / pi.
        cx = g.max_x - 0.5 * g.resolution * cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        s_min = int(math.floor((0.55 - 0.1) / 0.8 * 255 * n))  # ToScore(s / n) > 0.55, approx.
        rsel = np.linspace(0, ns - 1, args.rots).astype(int)
        for r in rsel:
            ix, iy = disc[r, :, 0], disc[r, :, 1]
            bx0, bx1, by0, by1 = bounds[r]
            top = D - 1
            st = 1 << top
            xs = np.arange(bx0, bx1 + 1, st)
            ys = np.arange(by0, by1 + 1, st)
            fx, fy = [a.ravel() for a in np.meshgrid(xs, ys, indexing="ij")]
            d = top
            while True:
                G = levels[d]
                b = (1 << d) - 1
                lx = ix[None, :] + fx[:, None] + b
                ly = iy[None, :] + fy[:, None] + b
                ok = (lx >= 0) & (lx < G.shape[1]) & (ly >= 0) & (ly < G.shape[0])
                v = np.where(ok, G[np.clip(ly, 0, G.shape[0] - 1), np.clip(lx, 0, G.shape[1] - 1)], 0)
                sc = v.sum(1)
                keep = sc > s_min
                fx, fy = fx[keep], fy[keep]
                if d == 0 or len(fx) == 0:
                    break
                # These nodes are expanded: children scored through Q_{d-1}
                # (polyphase period P = 2^d: node lattice entries adjacent).
                h = 1 << (d - 1)
                P = 2 * h
                rec = tot.setdefault(d, {"nodes": 0, "lattice": 0, "lines": {}})
                rec["nodes"] += len(fx)
                rec["lattice"] += len(np.arange(bx0, bx1 + 1, P)) * len(np.arange(by0, by1 + 1, P))
                # Node lattice coordinates.
                ex = (fx - bx0) // P
                ey = (fy - by0) // P
                pws = (400 + 2 * P) // P + 2  # plane row stride (entries)
                # Sample entries (points) for the line count.
                pk = rng.randint(0, n, 8)
                for name, order, tiled in (("rowmajor_yx", np.lexsort((ex, ey)), False),
                                          ("tiled8x4_morton", np.argsort(morton(ex, ey)), True),
                                          ("tiled8x8_morton", np.argsort(morton(ex, ey)), "8x8")):
                    oxs, oys = ex[order], ey[order]
                    lines, inst = 0, 0
                    for k0 in range(0, len(oxs), 64):
                        bx_, by_ = oxs[k0:k0 + 64], oys[k0:k0 + 64]
                        for p in pk:
                            X = ix[p] // P + bx_ + 10  # entry coords within the plane
                            Y = iy[p] // P + by_ + 10
                            if tiled is True:   # 8 x 4 dwords per 128 B line
                                lid = (Y // 4) * 1000 + X // 8
                            elif tiled == "8x8":  # 8x8 dword tiles, 2 lines each (4 rows)
                                lid = (Y // 4) * 1000 + X // 8
                            else:
                                lid = Y * 1000 + (X * 4) // 128
                            lines += len(np.unique(lid))
                            inst += 1
                    L = rec["lines"].setdefault(name, [0, 0])
                    L[0] += lines
                    L[1] += inst
                # children
                cx_ = np.concatenate([fx, fx, fx + h, fx + h])
                cy_ = np.concatenate([fy, fy + h, fy, fy + h])
                m = (cx_ <= bx1) & (cy_ <= by1)
                fx, fy = cx_[m], cy_[m]
                d -= 1
        print(f"pair {pi}: submap {s} node {nd} n={n} rotations={ns}", flush=True)
    print("level  nodes/rot  density  lines/instr (per ordering)")
    for d in sorted(tot, reverse=True):
        rec = tot[d]
        dens = rec["nodes"] / max(rec["lattice"], 1)
        ls = "  ".join(f"{k}={v[0] / max(v[1], 1):.2f}" for k, v in rec["lines"].items())
        print(f"{d:5d}  {rec['nodes'] / (args.pairs * args.rots):9.1f}  {dens:7.3f}  {ls}")




def rotation_coherence(argv=None):
    """Lines per gather when a batch's lanes are (rotation, node) with the
    SAME raw point index k: R consecutive rotations' frontiers at one level,
    grouped by node offset, then Morton order of the offset."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2)
    ap.add_argument("--chunks", type=int, default=6)
    ap.add_argument("--R", type=int, default=8)
    ap.add_argument("--depth", type=int, default=9)
    args = ap.parse_args(argv)
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(5)
    D = args.depth
    stats = {}
    for pi in range(args.pairs):
        s = int(rng.randint(world.num_submaps))
        nd = int(rng.randint(world.num_nodes))
        g = world.grid(s)
        cells = g.cells
        limits = (g.resolution, g.max_x, g.max_y)
        om = o.fast2d(limits, cells, 7.0, math.radians(30.0), D)
        levels = [om.level(d).astype(np.int64) for d in range(D)]
        cloud = world.cloud(nd)
        n = len(cloud)
        cx = g.max_x - 0.5 * g.resolution * cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        s_min = int(math.floor((0.55 - 0.1) / 0.8 * 255 * n))
        for c0 in np.linspace(0, ns - args.R - 1, args.chunks).astype(int):
            fronts = {}  # level -> list of (r, fx, fy)
            for r in range(c0, c0 + args.R):
                ix, iy = disc[r, :, 0], disc[r, :, 1]
                bx0, bx1, by0, by1 = bounds[r]
                st = 1 << (D - 1)
                xs = np.arange(bx0, bx1 + 1, st)
                ys = np.arange(by0, by1 + 1, st)
                fx, fy = [a.ravel() for a in np.meshgrid(xs, ys, indexing="ij")]
                d = D - 1
                while d >= 1 and len(fx):
                    G = levels[d]
                    b = (1 << d) - 1
                    lx = ix[None, :] + fx[:, None] + b
                    ly = iy[None, :] + fy[:, None] + b
                    ok = (lx >= 0) & (lx < G.shape[1]) & (ly >= 0) & (ly < G.shape[0])
                    v = np.where(ok, G[np.clip(ly, 0, G.shape[0] - 1), np.clip(lx, 0, G.shape[1] - 1)], 0)
                    keep = v.sum(1) > s_min
                    fx, fy = fx[keep], fy[keep]
                    fronts.setdefault(d, []).append((r, fx.copy(), fy.copy()))
                    h = 1 << (d - 1)
                    cx_ = np.concatenate([fx, fx, fx + h, fx + h])
                    cy_ = np.concatenate([fy, fy + h, fy, fy + h])
                    m = (cx_ <= bx1) & (cy_ <= by1)
                    fx, fy = cx_[m], cy_[m]
                    d -= 1
            for d, fl in fronts.items():
                P = 1 << d
                rr = np.concatenate([np.full(len(a), r) for r, a, _ in fl])
                xx = np.concatenate([a for _, a, _ in fl])
                yy = np.concatenate([b for _, _, b in fl])
                if len(rr) == 0:
                    continue
                uniq = len(np.unique(xx * 100000 + yy))
                order = np.lexsort((rr, morton((xx + 2000) // P, (yy + 2000) // P)))
                rr, xx, yy = rr[order], xx[order], yy[order]
                lines = inst = 0
                for k0 in range(0, len(rr), 64):
                    br, bxx, byy = rr[k0:k0 + 64], xx[k0:k0 + 64], yy[k0:k0 + 64]
                    for p in rng.randint(0, n, 6):
                        cxp = disc[br, p, 0] + bxx + 4000
                        cyp = disc[br, p, 1] + byy + 4000
                        X, Y = cxp // P, cyp // P
                        plane = (cyp % P) * P + (cxp % P)
                        lid = plane * 10 ** 8 + (Y // 4) * 10000 + X // 8
                        lines += len(np.unique(lid))
                        inst += 1
                st_ = stats.setdefault(d, [0, 0, 0, 0])
                st_[0] += len(rr)
                st_[1] += uniq
                st_[2] += lines
                st_[3] += inst
        print(f"pair {pi} done", flush=True)
    print(f"R={args.R}: level  nodes  distinct-offsets  lines/instr (lanes = rot x node, same point)")
    for d in sorted(stats, reverse=True):
        a = stats[d]
        print(f"{d:5d}  {a[0]:7d}  {a[1]:7d}  {a[2] / max(a[3], 1):.2f}")


def rotation_groups(argv=None):
    """Node expansions (one quad lookup per entry each) when R consecutive
    rotations share one search tree down to level S, with bounds from
    dilated max grids (width 2^d + 2*delta, delta = the group's largest
    per-point deviation from its middle rotation), split into per-rotation
    nodes below S. Threshold-only pruning (non-matching pairs)."""
    from scipy.ndimage import maximum_filter
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=2)
    ap.add_argument("--chunks", type=int, default=6)
    ap.add_argument("--R", type=int, default=8)
    ap.add_argument("--split", type=int, default=5)
    ap.add_argument("--depth", type=int, default=9)
    args = ap.parse_args(argv)
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(5)
    D = args.depth
    base_units = grp_units = 0
    deltas = []
    for pi in range(args.pairs):
        s = int(rng.randint(world.num_submaps))
        nd = int(rng.randint(world.num_nodes))
        g = world.grid(s)
        cells = g.cells
        limits = (g.resolution, g.max_x, g.max_y)
        om = o.fast2d(limits, cells, 7.0, math.radians(30.0), D)
        levels = [om.level(d).astype(np.int64) for d in range(D)]
        G0 = levels[0]  # (ny, nx) values, no padding at level 0
        PAD = 600
        Gp = np.zeros((G0.shape[0] + 2 * PAD, G0.shape[1] + 2 * PAD), np.int64)
        Gp[PAD:PAD + G0.shape[0], PAD:PAD + G0.shape[1]] = G0
        cloud = world.cloud(nd)
        n = len(cloud)
        cx = g.max_x - 0.5 * g.resolution * cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        s_min = int(math.floor((0.55 - 0.1) / 0.8 * 255 * n))
        dil_cache = {}

        def dilated(w):
            if w not in dil_cache:
                # M[c] = max G0 over [c, c + w) per axis (origin-shifted filter).
                dil_cache[w] = maximum_filter(Gp, size=(w, w), origin=(-(w // 2), -(w // 2)),
                                              mode="constant", cval=0)
            return dil_cache[w]

        def score_block(px, py, fx, fy, d, dl):
            # sum_k max G0 over [p + o - dl, p + o - dl + 2^d + 2 dl)
            w = (1 << d) + 2 * dl
            M = dilated(w)
            lx = px[None, :] + fx[:, None] - dl + PAD
            ly = py[None, :] + fy[:, None] - dl + PAD
            ok = (lx >= 0) & (lx < M.shape[1]) & (ly >= 0) & (ly < M.shape[0])
            return np.where(ok, M[np.clip(ly, 0, M.shape[0] - 1), np.clip(lx, 0, M.shape[1] - 1)], 0).sum(1)

        for c0 in np.linspace(0, ns - args.R - 1, args.chunks).astype(int):
            rots = list(range(c0, c0 + args.R))
            # --- baseline: per-rotation trees
            for r in rots:
                ix, iy = disc[r, :, 0], disc[r, :, 1]
                bx0, bx1, by0, by1 = bounds[r]
                st = 1 << (D - 1)
                fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                         np.arange(by0, by1 + 1, st), indexing="ij")]
                d = D - 1
                while d >= 1 and len(fx):
                    keep = score_block(ix, iy, fx, fy, d, 0) > s_min
                    fx, fy = fx[keep], fy[keep]
                    base_units += len(fx)
                    h = 1 << (d - 1)
                    cx_ = np.concatenate([fx, fx, fx + h, fx + h])
                    cy_ = np.concatenate([fy, fy + h, fy, fy + h])
                    m = (cx_ <= bx1) & (cy_ <= by1)
                    fx, fy = cx_[m], cy_[m]
                    d -= 1
            # --- grouped: one tree for the group down to the split level
            mid = rots[len(rots) // 2]
            mx, my = disc[mid, :, 0], disc[mid, :, 1]
            dl = int(max(np.abs(disc[rots, :, 0] - mx[None]).max(),
                         np.abs(disc[rots, :, 1] - my[None]).max()))
            deltas.append(dl)
            bx0 = min(bounds[r][0] for r in rots); bx1 = max(bounds[r][1] for r in rots)
            by0 = min(bounds[r][2] for r in rots); by1 = max(bounds[r][3] for r in rots)
            st = 1 << (D - 1)
            fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                     np.arange(by0, by1 + 1, st), indexing="ij")]
            d = D - 1
            while d > args.split and len(fx):
                keep = score_block(mx, my, fx, fy, d, dl) > s_min
                fx, fy = fx[keep], fy[keep]
                grp_units += len(fx)
                h = 1 << (d - 1)
                cx_ = np.concatenate([fx, fx, fx + h, fx + h])
                cy_ = np.concatenate([fy, fy + h, fy, fy + h])
                m = (cx_ <= bx1) & (cy_ <= by1)
                fx, fy = cx_[m], cy_[m]
                d -= 1
            # below the split: per rotation, starting from the group's level-S nodes
            gfx, gfy = fx, fy
            for r in rots:
                ix, iy = disc[r, :, 0], disc[r, :, 1]
                rb = bounds[r]
                m = (gfx >= rb[0]) & (gfx <= rb[1]) & (gfy >= rb[2]) & (gfy <= rb[3])
                fx, fy = gfx[m], gfy[m]
                # Per-rotation scores of the group's level-S nodes: one quad
                # lookup per (parent, rotation) (siblings share the dword).
                par = np.unique(((fx - rb[0]) >> (args.split + 1)) * 100000 + ((fy - rb[2]) >> (args.split + 1)))
                grp_units += len(par)
                d = args.split
                while d >= 1 and len(fx):
                    keep = score_block(ix, iy, fx, fy, d, 0) > s_min
                    fx, fy = fx[keep], fy[keep]
                    grp_units += len(fx)
                    h = 1 << (d - 1)
                    cx_ = np.concatenate([fx, fx, fx + h, fx + h])
                    cy_ = np.concatenate([fy, fy + h, fy, fy + h])
                    mm = (cx_ <= rb[1]) & (cy_ <= rb[3])
                    fx, fy = cx_[mm], cy_[mm]
                    d -= 1
        print(f"pair {pi}: rotations {ns}; units base {base_units} grouped {grp_units}", flush=True)
    print(f"R={args.R} split={args.split}: expansions base {base_units}, grouped {grp_units} "
          f"({grp_units / max(base_units, 1):.3f}x); delta mean {np.mean(deltas):.1f} max {max(deltas)}")


def clustered_scan(argv=None):
    """Lookups when the scan is clustered per level: at child level c the
    points are grouped into k_c x k_c cell clusters (one entry per occupied
    cluster, weighted by its point count) and scored against a max grid of
    width 2^c + k_c - 1 (a valid, looser bound). k_0 = 1 (exact leaves).
    Threshold-only pruning; cost = sum over expanded nodes of the entries of
    their children's level."""
    from scipy.ndimage import maximum_filter
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=3)
    ap.add_argument("--rots", type=int, default=12)
    ap.add_argument("--k", default="1,1,1,2,4,8,8,8,8", help="k per child level 0..8")
    ap.add_argument("--depth", type=int, default=9)
    args = ap.parse_args(argv)
    ks = [int(v) for v in args.k.split(",")]
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    rng = np.random.RandomState(5)
    D = args.depth
    tot = {"base_lookups": 0, "clu_lookups": 0, "base_nodes": [0] * D, "clu_nodes": [0] * D,
           "runs": 0, "entries": [0] * D, "rot": 0}
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

        def score(qx, qy, cnt, fx, fy, w):
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
            ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
            code = ix * 100000 + iy
            runs = 1 + int((code[1:] != code[:-1]).sum())
            tot["runs"] += runs
            tot["rot"] += 1
            ent = []
            for c in range(D):
                k = ks[c]
                qx, qy = (ix // k) * k, (iy // k) * k
                key = qx * 100000 + qy
                u, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
                first = np.zeros(len(u), np.int64)
                first[inv[::-1]] = np.arange(len(key))[::-1]
                ent.append((qx[first], qy[first], cnt.astype(np.int64), (1 << c) + k - 1))
                tot["entries"][c] += len(u)
            ones = np.ones(n, np.int64)
            bx0, bx1, by0, by1 = bounds[r]
            st = 1 << (D - 1)
            for mode in ("base", "clu"):
                fx, fy = [a.ravel() for a in np.meshgrid(np.arange(bx0, bx1 + 1, st),
                                                         np.arange(by0, by1 + 1, st), indexing="ij")]
                d = D - 1
                while len(fx):
                    if mode == "base":
                        sc = score(ix, iy, ones, fx, fy, 1 << d)
                    else:
                        e = ent[d]
                        sc = score(e[0], e[1], e[2], fx, fy, e[3])
                    keep = sc > s_min
                    fx, fy = fx[keep], fy[keep]
                    if d == 0:
                        break
                    tot[f"{mode}_nodes"][d] += len(fx)
                    tot[f"{mode}_lookups"] += len(fx) * (runs if mode == "base" else len(ent[d - 1][0]))
                    h = 1 << (d - 1)
                    cx_ = np.concatenate([fx, fx, fx + h, fx + h])
                    cy_ = np.concatenate([fy, fy + h, fy, fy + h])
                    m = (cx_ <= bx1) & (cy_ <= by1)
                    fx, fy = cx_[m], cy_[m]
                    d -= 1
        print(f"pair {pi} done ({ns} rotations)", flush=True)
    R = max(tot["rot"], 1)
    print(f"k={args.k}: runs/rot {tot['runs'] / R:.0f}; entries/rot per child level "
          f"{[round(e / R) for e in tot['entries']]}")
    print(f"  expanded nodes/rot base {[round(v / R, 1) for v in tot['base_nodes']]}")
    print(f"  expanded nodes/rot clu  {[round(v / R, 1) for v in tot['clu_nodes']]}")
    print(f"  lookups base {tot['base_lookups'] / R:.0f}/rot, clustered {tot['clu_lookups'] / R:.0f}/rot "
          f"({tot['clu_lookups'] / max(tot['base_lookups'], 1):.3f}x)")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "rot":
        rotation_coherence(sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "cluster":
        clustered_scan(sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] == "groups":
        rotation_groups(sys.argv[2:])
    else:
        main()
