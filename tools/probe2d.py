"""Small-probe of the 2D search kernel: a few pairs, kernel time, candidates and
batches per level, and agreement with the default policy. Experiments only."""
import math
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge

csm = ge._load_package()
nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 20
subs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ctx = csm.Context(0)
w = csm.SyntheticWorld2D(num_nodes=nodes, num_submaps=subs, submap_cells=400, beams=1080, seed=20250127)
opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30.0), 7, 0)
ms = [csm.FastCorrelativeScanMatcher2D(w.grid(s), opts, ctx) for s in range(subs)]
scans = csm.ScanSet(None, ctx, packed=(w.points, w.offsets))
sub = np.repeat(np.arange(subs, dtype=np.int32), nodes)
nd = np.tile(np.arange(nodes, dtype=np.int32), subs)
pairs = csm.make_pairs(sub, nd, 0.55, full_submap=True)
ctx.reset_timing()
ctx.enable_timing(True)
t0 = time.time()
res = csm.match_batch(ms, scans, pairs, ctx)
wall = time.time() - t0
tm = ctx.timing()
c, b = ctx.level_stats()
print("mode", os.environ.get("CSM_MIXED_LEVELS", "1"), "pairs", len(pairs), "kernel_ms", round(tm.search_kernel_ms, 2),
      "wall_s", round(wall, 3), "lookups", tm.search_lookups)
print("cands/level", [int(x) for x in c])
print("batches/level", [int(x) for x in b])
np.save(os.environ.get("PROBE_OUT", "/tmp/probe.npy"), np.stack([res["status"].astype(np.float64), res["score"].astype(np.float64)]))
print("accepted", int(np.sum(res["status"] == 0)))
