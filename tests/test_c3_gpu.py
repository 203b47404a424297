"""GPU parity on the north-star C3 world (BASELINE.json configs[2]): the
2000-node x 1000-submap ConstraintBuilder2D sweep bench.py --workload c3
runs, same generator and seed. A sample of its (submap, node) pairs goes
through the batch path in chunk-shaped batches (several submaps x nodes per
launch, as c3_main issues them) and every pair is compared with the oracle's
MatchFullSubmap (fast_correlative_scan_matcher_2d.cc:220-235) at the bench's
options (7 m, 30 deg, depth 7, min_score 0.55).
"""
import math
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
from conftest import assert_search_ok
from test_fast2d_gpu import assert_fast_parity, full_submap_center

pytestmark = pytest.mark.gpu

SEED = 20250127  # bench.py's default --seed


@pytest.fixture(scope="module")
def c3_world(csm):
    return csm.SyntheticWorld2D(num_nodes=2000, num_submaps=1000, submap_cells=400, beams=1080,
                                seed=SEED)


def test_c3_world_pairs_match_oracle(csm, oracle, c3_world):
    w = c3_world
    rng = np.random.RandomState(7)
    # Pairs that should close a loop (the node the submap was built around
    # and its neighbours) and uniform pairs of the queue (mostly no match).
    near = rng.choice(w.num_submaps, 12, replace=False)
    pairs_sn = [(int(s), int(min(w.num_nodes - 1, w.submap_nodes[s] + d)))
                for s, d in zip(near, rng.randint(0, 3, 12))]
    pairs_sn += [(int(s), int(n)) for s, n in zip(rng.randint(0, w.num_submaps, 12),
                                                  rng.randint(0, w.num_nodes, 12))]
    subs = sorted({s for s, _ in pairs_sn})
    local = {s: i for i, s in enumerate(subs)}
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30.0), 7, 0)
    mats = [csm.FastCorrelativeScanMatcher2D(w.grid(s), opts) for s in subs]
    scans = csm.ScanSet(None, packed=(w.points, w.offsets))
    pairs = csm.make_pairs([local[s] for s, _ in pairs_sn], [n for _, n in pairs_sn], 0.55,
                           full_submap=True)
    res = csm.match_batch(mats, scans, pairs)
    assert_search_ok(csm, res["status"])

    def ref(sn):
        s, n = sn
        g = w.grid(s)
        limits = (g.resolution, g.max_x, g.max_y)
        om = oracle.fast2d(limits, g.cells, 7.0, math.radians(30.0), 7)
        cloud = w.cloud(n)
        return om, limits, g.cells, cloud, om.match_full_submap(cloud, 0.55)

    with ThreadPoolExecutor(max_workers=8) as ex:
        refs = list(ex.map(ref, pairs_sn))
    kinds = []
    for k, (om, limits, cells, cloud, r) in enumerate(refs):
        gpu = (res[k]["status"] == 0, float(res[k]["score"]),
               (res[k]["x"], res[k]["y"], res[k]["theta"]))
        kinds.append(assert_fast_parity(oracle, om, limits, cells, gpu, r, True,
                                        full_submap_center(limits, cells), cloud))
    assert kinds.count("nomatch") < len(kinds), kinds
    assert kinds.count("exact") + kinds.count("tie") >= 6, kinds
