"""Design study for RTCSM3D (C4): how many rotations could an exact
rotation-level bound discard?

For each sampled rotation r of the C4 window, bound_r = sum over points of
the max probability within reach of every translation of the window (a max
filter of the probability brick, widths from the translation lattice's
extent), divided by n. A rotation whose bound is below the best score cannot
hold the winner. Prints the distribution of bound_r against the best score.

    python tools/rt3d_prune_sim.py [--samples 3000]
"""
import argparse
import math
import os
import sys

import numpy as np
from scipy.ndimage import maximum_filter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def quat_mul(a, b):
    w1, x1, y1, z1 = a
    w2, x2, y2, z2 = b
    return np.array([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2])


def quat_to_mat(q):
    w, x, y, z = q / np.linalg.norm(q)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=3000)
    ap.add_argument("--best", type=float, default=0.6055)
    args = ap.parse_args()
    import __graft_entry__ as ge
    csm = ge._load_package()
    seed = 20250127 + 3
    w = csm.SyntheticWorld3D(num_nodes=2, num_submaps=1, world_x=20.0, world_y=20.0, world_z=5.0,
                             num_boxes=8, max_range=14.0, seed=seed)
    c = int(w.submap_nodes[0])
    cloud = w.raw[c].astype(np.float64)
    res = w.high_resolution
    ijk, val = w.high_cells[0]
    lo = ijk.min(0)
    hi = ijk.max(0)
    dims = hi - lo + 1
    kmin, kmax = 0.1, 0.9
    scale = (kmax - kmin) / (32768 - 2.0)
    prob = np.full(dims[::-1], 0.1)
    p = np.where(val == 0, 0.1, val * scale + (kmin - scale))
    prob[ijk[:, 2] - lo[2], ijk[:, 1] - lo[1], ijk[:, 0] - lo[0]] = p
    (tx, ty, tz), q = w.node_in_submap(c, 0)
    dyaw = math.radians(4.0)
    q0 = np.array([q[0] * math.cos(dyaw / 2) - q[3] * math.sin(dyaw / 2), 0.0, 0.0,
                   q[3] * math.cos(dyaw / 2) + q[0] * math.sin(dyaw / 2)])
    t0 = np.array([tx + 0.12, ty - 0.08, tz + 0.05])
    R0 = quat_to_mat(q0)
    L = 3
    reach = np.ceil(L * np.abs(R0).sum(1)).astype(int) + 1  # cells per axis (x, y, z)
    pad = int(reach.max()) + 2
    P = np.pad(prob, pad, constant_values=0.1)
    M = maximum_filter(P, size=(2 * reach[2] + 1, 2 * reach[1] + 1, 2 * reach[0] + 1), mode="nearest")
    max_range = max(3 * res, float(np.linalg.norm(cloud, axis=1).max()))
    step = (1 - 1e-3) * math.acos(1 - res * res / (2 * max_range * max_range))
    A = int(round(math.radians(15.0) / step))
    rng = np.random.RandomState(1)
    n = len(cloud)
    bounds = []
    for _ in range(args.samples):
        r = rng.randint(-A, A + 1, 3) * step
        ang = np.linalg.norm(r)
        qs = np.array([1.0, 0, 0, 0]) if ang == 0 else np.concatenate(
            [[math.cos(ang / 2)], math.sin(ang / 2) * r / ang])
        Rq = quat_to_mat(quat_mul(q0, qs))
        pts = cloud @ Rq.T + t0
        cell = np.rint(pts / res).astype(int) - lo + pad
        inb = np.all((cell >= 0) & (cell < np.array(P.shape[::-1])), axis=1)
        v = np.full(n, 0.9)
        v[inb] = M[cell[inb, 2], cell[inb, 1], cell[inb, 0]]
        bounds.append(v.sum() / n)
    b = np.array(bounds)
    print(f"points {n}, A {A} ({(2 * A + 1) ** 3} rotations), translation reach {reach.tolist()} cells")
    for thr in (args.best, args.best * 1.05):
        print(f"rotations with bound >= {thr:.4f}: {np.mean(b >= thr):.3f}")
    print("bound quantiles", np.quantile(b, [0.01, 0.1, 0.5, 0.9, 0.99]).round(4).tolist())


if __name__ == "__main__":
    main()
