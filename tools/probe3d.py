"""Probe: 3D matcher timings on the GPU (not part of the bench contract)."""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

csm = ge._load_package()
p = argparse.ArgumentParser()
p.add_argument("--nodes", type=int, default=100)
p.add_argument("--submaps", type=int, default=10)
p.add_argument("--rt", action="store_true")
p.add_argument("--rt-lin", type=float, default=0.3)
p.add_argument("--rt-ang", type=float, default=15.0)
p.add_argument("--rt-points", type=int, default=0)
a = p.parse_args()
ctx = csm.Context(0)
t = time.time()
w = csm.SyntheticWorld3D(num_nodes=a.nodes, num_submaps=a.submaps)
gen = time.time() - t
o = csm.FastCorrelativeScanMatcherOptions3D()
t = time.time()
grids = [(csm.HybridGrid(w.high_resolution, *w.high_cells[s], context=ctx),
          csm.HybridGrid(w.low_resolution, *w.low_cells[s], context=ctx)) for s in range(a.submaps)]
mats = [csm.FastCorrelativeScanMatcher3D(g[0], g[1], w.submap_hist[s], o, ctx) for s, g in enumerate(grids)]
build = time.time() - t
nodes = [w.node(i) for i in range(a.nodes)]
ident = ((0, 0, 0), (1, 0, 0, 0))
sub = np.repeat(np.arange(a.submaps), a.nodes)
nod = np.tile(np.arange(a.nodes), a.submaps)
pairs = csm.make_pairs_3d(sub, nod, 0.6, True, node_q=np.array([w.node_rotation(n) for n in nod]))
csm.match_batch_3d(mats, nodes, pairs, ctx)  # warm: staging buffers at full size
ctx.reset_timing()
ctx.enable_timing(True)
t = time.time()
res = csm.match_batch_3d(mats, nodes, pairs, ctx)
dt = time.time() - t
tm = ctx.timing()
acc = int((res["status"] == 0).sum())
out = {"pairs": len(pairs), "s": dt, "pairs_per_s": len(pairs) / dt, "accepted": acc,
       "kernel_ms": tm.fast3d_kernel_ms, "lookups": tm.fast3d_lookups,
       "GBps_alg": tm.fast3d_lookups / (tm.fast3d_kernel_ms * 1e-3) / 1e9 if tm.fast3d_kernel_ms else 0,
       "gen_s": gen, "build_s": build,
       "mean_high_pts": float(np.mean([len(x) for x in w.high])),
       "mean_raw_pts": float(np.mean([len(x) for x in w.raw]))}
print(json.dumps(out), flush=True)
if a.rt:
    s = 0
    c = int(w.submap_nodes[s])
    truth = w.node_in_submap(c, s)
    init = ((truth[0][0] + 0.1, truth[0][1] - 0.05, 0.05), truth[1])
    m = csm.RealTimeCorrelativeScanMatcher3D(
        csm.RealTimeCorrelativeScanMatcherOptions(a.rt_lin, math.radians(a.rt_ang), 0.1, 0.1), ctx)
    cloud = w.raw[c] if a.rt_points == 0 else w.raw[c][:a.rt_points]
    ctx.reset_timing()
    t = time.time()
    score, pose = m.Match(init, cloud, grids[s][0])
    dt = time.time() - t
    tm = ctx.timing()
    print(json.dumps({"rt3d_s": dt, "score": score, "pose": pose, "points": len(cloud),
                      "kernel_ms": tm.rt3d_kernel_ms, "lookups": tm.rt3d_lookups,
                      "Glookups_per_s": tm.rt3d_lookups / (tm.rt3d_kernel_ms * 1e-3) / 1e9 if tm.rt3d_kernel_ms else 0}),
          flush=True)
