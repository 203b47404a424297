"""Per-node flush cost of the Python ConstraintBuilder2D drop-in on the C2
world (50 submaps of 400 x 400 at 5 cm, 1080-beam clouds): each node ends
with a MatchFullSubmap pair against every submap, as a global sweep does
(pose_graph_2d.cc:379-392), then a second pass re-matches the same nodes
(a finished submap against earlier nodes). Compares node clouds kept
resident across flushes (the default) with a new scan set every flush
(scan_cache_points=0). Prints one JSON line."""
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_package  # noqa: E402

csm = load_package()
import importlib  # noqa: E402
cb = importlib.import_module("cartographer_amd.constraint_builder")

world = csm.SyntheticWorld2D(num_nodes=40, num_submaps=50, seed=20250127)
fopts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30), 7)


def run(cache_points, passes=2, nodes=20):
    opts = cb.ConstraintBuilderOptions(sampling_ratio=1.0, min_score=0.55,
                                       global_localization_min_score=0.55,
                                       max_constraint_distance=1e9,
                                       fast_correlative_scan_matcher_options=fopts,
                                       refine_with_ceres=False, scan_cache_points=cache_points)
    b = cb.ConstraintBuilder2D(opts)
    submaps = {s: cb.Submap2D(world.grid(s), (0.0, 0.0, 0.0)) for s in range(world.num_submaps)}
    for s in range(world.num_submaps):  # matchers built outside the timed flushes
        b.MaybeAddGlobalConstraint((0, s), submaps[s], (0, 39), world.cloud(39))
    b.NotifyEndOfNode()
    ms = []
    for _ in range(passes):
        for node in range(nodes):
            cloud = world.cloud(node)
            for s in range(world.num_submaps):
                b.MaybeAddGlobalConstraint((0, s), submaps[s], (0, node), cloud)
            a = time.perf_counter()
            b.NotifyEndOfNode()
            ms.append((time.perf_counter() - a) * 1e3)
    got = []
    b.WhenDone(got.append)
    half = len(ms) // passes
    return {"ms_per_flush_median_first_pass": float(np.median(ms[:half])),
            "ms_per_flush_median_revisit": float(np.median(ms[half:])),
            "pairs_per_flush": world.num_submaps, "constraints": len(got[0])}


out = {"resident": run(1 << 25), "new_set_every_flush": run(0)}
print(json.dumps(out))
