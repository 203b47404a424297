"""Design study: how many entries of the search kernel's run lists repeat an
earlier entry's cluster key, and how far back (C2 world, sampled rotations).

A run list merges consecutive points with the same k x k cluster key; a key
that recurs later stays a separate entry. The fraction caught within a window
of W entries tells which merge the kernel can afford. On C2 every repeat is
two entries back (a scan zig-zagging across a cluster boundary). A wave-level
merge of those chains (9% fewer k = 4 / k = 8 entries) was built and measured
slower on the GPU (C3 chunk 626 -> 644 ms, profiles/r3y/), so it was dropped.

    python tools/list_repeats.py
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    o = oracle_lib.Oracle()
    world = csm.SyntheticWorld2D(num_nodes=500, num_submaps=50, submap_cells=400, beams=1080,
                                 seed=20250127)
    windows = [1, 2, 4, 8, 16, 64, 1 << 20]
    tot = {k: np.zeros(len(windows) + 1) for k in (1, 4, 8)}
    for s, nd in [(3, 30), (10, 100), (20, 200), (5, 400), (40, 77), (7, 250)]:
        g = world.grid(s)
        cloud = world.cloud(nd)
        limits = (g.resolution, g.max_x, g.max_y)
        cx = g.max_x - 0.5 * g.resolution * g.cells.shape[0]
        cy = g.max_y - 0.5 * g.resolution * g.cells.shape[1]
        ns, bounds, disc, step = o.discretize(limits, g.cells, (cx, cy, 0.0), 1e6, math.pi, cloud)
        for r in range(0, ns, 97):
            ix, iy = disc[r, :, 0].astype(np.int64), disc[r, :, 1].astype(np.int64)
            for k in tot:
                key = (ix // k) * 100000 + (iy // k)
                head = np.ones(len(key), bool)
                head[1:] = key[1:] != key[:-1]
                runs = key[head]
                tot[k][0] += len(runs)
                for wi, w in enumerate(windows):
                    tot[k][wi + 1] += sum(1 for i in range(len(runs))
                                          if runs[i] in runs[max(0, i - w):i])
    for k, v in tot.items():
        print(f"k = {k}: {int(v[0])} run entries; repeats of a key within W entries back: " +
              ", ".join(f"W={w if w < 1 << 20 else 'all'} {x / v[0]:.3f}"
                        for w, x in zip(windows, v[1:])))


if __name__ == "__main__":
    main()
