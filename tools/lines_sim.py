"""Design study: distinct 128-byte lines per wave-wide gather instruction in
the FastCSM2D search, for the current lane mapping (64 nodes x 1 entry, hex /
quad planes polyphase with period 4h / 2h) against entry-major lanes (G nodes x
64/G consecutive entries of each node's list) over planes split by the cluster
residue (X mod k, Y mod k) and tiled in 2-D per line.

tools/gather_bench2.hip: an instruction costs ~2.2 texture cycles per distinct
line it touches, L1 hit or not, so lines per instruction is the kernel's cost
model. Uses the C2 world's scans (oracle discretization) and every in-bounds
node of a level for each sampled rotation.

    python tools/lines_sim.py
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run_list(ix, iy, k):
    qx, qy = (ix // k) * k, (iy // k) * k
    key = qx * 100000 + qy
    head = np.ones(len(key), bool)
    head[1:] = key[1:] != key[:-1]
    return qx[head], qy[head]


def lines_current(ex, ey, nx_, ny_, P, es, W):
    # polyphase period P: plane (X mod P, Y mod P), entry (X/P, Y/P), row width W/P
    pw = W // P + 2
    X = ex[None, :] + nx_[:, None] + 3 * P
    Y = ey[None, :] + ny_[:, None] + 3 * P
    plane = (Y % P) * P + (X % P)
    addr = plane * (pw * pw * es) + ((Y // P) * pw + X // P) * es
    return addr >> 7  # [node, entry]


def lines_polytile(ex, ey, nx_, ny_, P, es, W, tx, ty):
    # polyphase period P as lines_current, each plane tiled tx x ty entries per line
    pw = W // P + 2
    X = ex[None, :] + nx_[:, None] + 3 * P
    Y = ey[None, :] + ny_[:, None] + 3 * P
    plane = (Y % P) * P + (X % P)
    u, v = X // P, Y // P
    tpr = pw // tx + 2
    addr = plane * (tpr * tpr * 128 * 4) + ((v // ty) * tpr + u // tx) * 128 + ((v % ty) * tx + u % tx) * es
    return addr >> 7


def lines_residue(ex, ey, nx_, ny_, k, es, tx, ty, W):
    X = ex[None, :] + nx_[:, None] + 3 * 64
    Y = ey[None, :] + ny_[:, None] + 3 * 64
    u, v = X // k, Y // k
    tpr = (W // k) // tx + 2
    plane = (Y % k) * k + (X % k)
    tiles = (v // ty) * tpr + (u // tx)
    addr = plane * (tpr * tpr * 128 * 4) + tiles * 128 + ((v % ty) * tx + (u % tx)) * es
    return addr >> 7


def per_instruction(lines, nodes_per_instr):
    # lines[node, entry]; current: instruction = all nodes (<= 64) x one entry;
    # entry-major: nodes in groups of G, 64/G consecutive entries each.
    n, m = lines.shape
    G = nodes_per_instr
    E = 64 // G
    tot, cnt = 0, 0
    for g0 in range(0, n, G):
        blk = lines[g0:g0 + G]
        for e0 in range(0, m, E):
            tot += len(np.unique(blk[:, e0:e0 + E]))
            cnt += 1
    return tot, cnt


def survivors(ent_lists, M, fx0, fy0, top, s_min, stop_level, PAD):
    """Level-by-level search of one rotation with clustered bounds (as the
    kernel: hex from levels 8 and 6, quad below); returns the node sets that
    get expanded at each level >= stop_level."""
    expanded = {}
    fx, fy = fx0, fy0
    d = top
    while len(fx) and d >= stop_level:
        expanded[d] = (fx, fy)
        hexp = d in (8, 6)
        c = d - 2 if hexp else d - 1
        hh = 1 << c
        m = 4 if hexp else 2
        cx_ = np.concatenate([fx + a * hh for a in range(m) for b in range(m)])
        cy_ = np.concatenate([fy + b * hh for a in range(m) for b in range(m)])
        qx, qy, cnt, w = ent_lists[c]
        A = M(w)
        lx = qx[None, :] + cx_[:, None] + PAD
        ly = qy[None, :] + cy_[:, None] + PAD
        v = A[np.clip(ly, 0, A.shape[0] - 1), np.clip(lx, 0, A.shape[1] - 1)]
        sc = (v * cnt[None, :]).sum(1)
        keep = sc > s_min
        fx, fy = cx_[keep], cy_[keep]
        order = np.lexsort((fx, fy))
        fx, fy = fx[order], fy[order]
        d = c
    return expanded


def main_survivors():
    from scipy.ndimage import maximum_filter
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    W = 700
    ks = [1, 1, 4, 4, 4, 8, 8, 8, 8]
    res = {}
    for s, nd in [(3, 30), (10, 100), (20, 200), (5, 400), (12, 33)]:
        g = world.grid(s)
        cloud = world.cloud(nd)
        limits = (g.resolution, g.max_x, g.max_y)
        om = o.fast2d(limits, g.cells, 7.0, math.radians(30.0), 9)
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
        cx = g.max_x - 0.5 * g.resolution * g.cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * g.cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, g.cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        n = len(cloud)
        s_min = int(math.floor((0.55 - 0.1) / 0.8 * 255 * n))
        for r in range(0, ns, 101):
            ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
            ent = []
            for c in range(9):
                k = ks[c]
                qx, qy = run_list(ix, iy, k)
                key = (ix // k) * k * 100000 + (iy // k) * k
                head = np.ones(n, bool)
                head[1:] = key[1:] != key[:-1]
                idx = np.nonzero(head)[0]
                cnt = np.diff(np.append(idx, n))
                ent.append((qx, qy, cnt, (1 << c) + k - 1))
            b0, b1, b2, b3 = bounds[r]
            fx, fy = [a.ravel() for a in np.meshgrid(np.arange(b0, b1 + 1, 256),
                                                     np.arange(b2, b3 + 1, 256), indexing="ij")]
            exp = survivors(ent, M, fx, fy, 8, s_min, 2, PAD)
            for L, hexp in ((6, True), (4, False), (3, False)):
                if L not in exp:
                    continue
                nx_, ny_ = exp[L]
                c = L - 2 if hexp else L - 1
                k = ks[c]
                ex, ey = ent[c][0], ent[c][1]
                P = (4 << (L - 2)) if hexp else (2 << (L - 1))
                es = 16 if hexp else 4
                tiles = (4, 2) if hexp else (8, 4)
                for key, lines, G in [
                        ("current", lines_current(ex, ey, nx_, ny_, P, es, W), 64),
                        ("current lanes, polyphase planes tiled 4x2 / 8x4",
                         lines_polytile(ex, ey, nx_, ny_, P, es, W, *tiles), 64),
                        ("residue 4x2/8x4 tiles, 8 nodes x 8 entries",
                         lines_residue(ex, ey, nx_, ny_, k, es, *((4, 2) if hexp else (8, 4)), W), 8),
                        ("residue 4x2/8x4 tiles, 4 nodes x 16 entries",
                         lines_residue(ex, ey, nx_, ny_, k, es, *((4, 2) if hexp else (8, 4)), W), 4)]:
                    t, cnt_ = per_instruction(lines, min(G, len(nx_)))
                    a = res.setdefault((L, key), [0, 0, 0])
                    a[0] += t
                    a[1] += cnt_
                    a[2] += lines.size
    for (L, key), (t, c, lanes) in sorted(res.items()):
        print(f"level-{L} nodes, {key}: {t / c:.1f} lines per instruction, "
              f"{t / lanes:.3f} lines per lane-gather")


def main():
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    W = 700
    cases = [  # (name, cluster k, node level L, hex?)
        ("hex: level-6 nodes -> level-4 grandchildren, k=4", 4, 6, True),
        ("quad: level-4 nodes -> level-3 children, k=4", 4, 4, False),
    ]
    for name, k, L, hexp in cases:
        res = {}
        for s, nd in [(3, 30), (10, 100), (20, 200), (5, 400)]:
            g = world.grid(s)
            cloud = world.cloud(nd)
            limits = (g.resolution, g.max_x, g.max_y)
            cx = g.max_x - 0.5 * g.resolution * g.cells.shape[0]
            cy = g.max_y - 0.5 * g.resolution * g.cells.shape[1]
            ns, bounds, disc, step = o.discretize(limits, g.cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
            for r in range(0, ns, 211):
                ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
                ex, ey = run_list(ix, iy, k)
                b0, b1, b2, b3 = bounds[r]
                st = 1 << L
                nx_, ny_ = [a.ravel() for a in np.meshgrid(np.arange(b0, b1 + 1, st),
                                                           np.arange(b2, b3 + 1, st), indexing="ij")]
                order = np.lexsort((nx_, ny_))  # x fastest, as the ring order
                nx_, ny_ = nx_[order], ny_[order]
                P = (4 << (L - 2)) if hexp else (2 << (L - 1))
                es = 16 if hexp else 4
                cur = lines_current(ex, ey, nx_, ny_, P, es, W)
                variants = {"current (64 nodes x 1 entry, polyphase)": (cur, 64)}
                for tx, ty in ([(8, 1), (4, 2)] if hexp else [(32, 1), (8, 4)]):
                    lr = lines_residue(ex, ey, nx_, ny_, k, es, tx, ty, W)
                    for G in (8, 4):
                        variants[f"residue planes, {tx}x{ty} tiles, {G} nodes x {64 // G} entries"] = (lr, G)
                for key, (lines, G) in variants.items():
                    t, c = per_instruction(lines, min(G, len(nx_)))
                    a = res.setdefault(key, [0, 0, 0])
                    a[0] += t
                    a[1] += c
                    a[2] += lines.size
        print(name)
        for key, (t, c, lanes) in res.items():
            print(f"  {key}: {t / c:.1f} lines per instruction, {t / lanes:.3f} lines per lane-gather")


if __name__ == "__main__":
    main_survivors() if "--survivors" in sys.argv else main()
