"""Builds tests/golden/fast2d_c3_ties.npz: exactly tied pairs of the C3 queue
(BASELINE.json configs[2]) with the oracle's MatchFullSubmap result.

Input: the tied-pair log of a GPU run of the whole C3 queue
(`bench.py --c3-tie-log PATH`, which writes PATH.rank0.json: the (submap,
node, csm_result2d.tie) of every accepted pair whose maximum more than one
leaf reached). The GPU only says WHICH pairs tie; the expected results come
from the oracle (test infrastructure, oracle/match2d.cc, the reference's
MatchFullSubmap restated, fast_correlative_scan_matcher_2d.cc:210-225 and
:276-378), run here on the CPU on the same seeded world
(libcsm_synth.so, the generator bench.py and tests/test_c3_gpu.py use).

Every pair of the TOPLIST branch (two lowest-resolution candidates share the
highest score, so the reference's introsort permutation decides) is kept, and
pairs of the ANCESTORS branch fill the fixture to --count. A fingerprint of
each used submap grid and node cloud is stored so that a change of the
generator fails the fixture's CPU test instead of the GPU parity test.

    python tools/c3_tie_fixture.py gpurun_out/r4a/c3ties.rank0.json
"""
import argparse
import json
import math
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

OUT = os.path.join(ROOT, "tests", "golden", "fast2d_c3_ties.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log", help="bench.py --c3-tie-log output (PATH.rank0.json)")
    ap.add_argument("--count", type=int, default=32, help="pairs in the fixture (>= 20)")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=OUT)
    a = ap.parse_args()
    import __graft_entry__ as ge
    import oracle_lib
    from c3_fixture_fp import fingerprint
    csm = ge._load_package()
    log = json.load(open(a.log))
    ties = [tuple(t) for t in log["ties"]]
    top = [t for t in ties if t[2] == csm.TIE_TOPLIST]
    anc = [t for t in ties if t[2] == csm.TIE_ANCESTORS]
    rng = np.random.RandomState(4)
    pick = list(top[:a.count // 2])
    if anc:
        pick += [anc[i] for i in sorted(rng.choice(len(anc), min(len(anc), a.count - len(pick)),
                                                   replace=False))]
    print(f"{len(ties)} tied pairs in the log ({len(top)} toplist, {len(anc)} ancestors); "
          f"{len(pick)} picked", flush=True)
    world = csm.SyntheticWorld2D(num_nodes=log["nodes"], num_submaps=log["submaps"],
                                 submap_cells=400, beams=1080, seed=log["seed"])
    oracle = oracle_lib.Oracle()
    min_score = float(log["min_score"])

    def ref(t):
        s, n, _ = t
        g = world.grid(s)
        om = oracle.fast2d((g.resolution, g.max_x, g.max_y), g.cells, 7.0, math.radians(30.0), 7)
        return om.match_full_submap(world.cloud(n), min_score)

    t0 = time.time()
    with ThreadPoolExecutor(max_workers=a.threads) as ex:
        refs = list(ex.map(ref, pick))
    print(f"oracle: {len(pick)} pairs in {time.time() - t0:.1f} s", flush=True)
    ok = np.array([r[0] for r in refs], np.int32)
    if not ok.all():
        raise SystemExit("a tied GPU match is not a match in the oracle")
    np.savez_compressed(
        a.out,
        seed=np.int64(log["seed"]), nodes=np.int64(log["nodes"]), submaps=np.int64(log["submaps"]),
        min_score=np.float32(min_score),
        submap=np.array([t[0] for t in pick], np.int32), node=np.array([t[1] for t in pick], np.int32),
        branch=np.array([t[2] for t in pick], np.int32),
        score=np.array([r[1] for r in refs], np.float32),
        pose=np.array([r[2] for r in refs], np.float64).reshape(-1, 3),
        grid_fp=np.array([fingerprint(world.submap_cells[t[0]]) for t in pick], np.int64),
        cloud_fp=np.array([fingerprint(world.cloud(t[1])) for t in pick], np.int64),
        queue_ties=np.array([len(ties), len(top), len(anc)], np.int64))
    print(f"wrote {a.out}")


if __name__ == "__main__":
    main()
