"""Tie parity at BASELINE scale: exactly tied pairs of the C3 queue.

When several leaves reach a pair's maximum the reference returns the first
one its depth-first search visits (fast_correlative_scan_matcher_2d.cc:
276-312 orders the lowest-resolution candidates with std::sort, :331-332 and
:344-376 visit children by descending score and keep the incumbent on equal
scores). The device search keeps the smallest (rotation, x, y) leaf and
csm_host.cc ResolveTies restores the reference's pick. This file pins that on
real 1080-point C3 pairs: tests/golden/fast2d_c3_ties.npz holds tied pairs
found by a GPU run of the whole 2 M-pair queue with the oracle's
MatchFullSubmap result for each (tools/c3_tie_fixture.py), including pairs
whose two highest lowest-resolution candidates tie, which take the branch
that scores and introsorts the pair's whole lowest-resolution list
(csm_result2d.tie == CSM_TIE_TOPLIST).
"""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "fast2d_c3_ties.npz")


@pytest.fixture(scope="module")
def ties():
    return dict(np.load(FIXTURE))


@pytest.fixture(scope="module")
def c3_world(csm, ties):
    return csm.SyntheticWorld2D(num_nodes=int(ties["nodes"]), num_submaps=int(ties["submaps"]),
                                submap_cells=400, beams=1080, seed=int(ties["seed"]))


def test_fixture_covers_both_branches(csm, ties):
    assert len(ties["submap"]) >= 20
    assert (ties["branch"] == csm.TIE_TOPLIST).sum() >= 1
    assert (ties["branch"] == csm.TIE_ANCESTORS).sum() >= 1


def test_fixture_world_unchanged(c3_world, ties):
    """The generator still makes the world the fixture was computed on."""
    from c3_fixture_fp import fingerprint
    w = c3_world
    for s, n, gfp, cfp in zip(ties["submap"], ties["node"], ties["grid_fp"], ties["cloud_fp"]):
        assert fingerprint(w.submap_cells[s]) == gfp, f"submap {s} changed"
        assert fingerprint(w.cloud(n)) == cfp, f"node {n} changed"


@pytest.mark.gpu
@pytest.mark.parametrize("batch", ["chunk", "single", "threads"])
def test_c3_tied_pairs_match_oracle(csm, c3_world, ties, batch):
    """Every tied pair: bit-identical score and the oracle's (the reference's)
    pose, searched inside chunk-shaped batches (the pair's submap x many
    nodes, as bench.py's C3 leg issues them) and as single MatchFullSubmap
    calls, sequentially and from 8 threads at once (the reference's pool
    workers sharing the matchers, constraint_builder_2d.cc:100-111). A batch
    result must report the branch the GPU run recorded."""
    import math
    from conftest import assert_search_ok
    w = c3_world
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30.0), 7, 0)
    min_score = float(ties["min_score"])
    subs = sorted(set(int(s) for s in ties["submap"]))
    mats = {s: csm.FastCorrelativeScanMatcher2D(w.grid(s), opts) for s in subs}
    n_pairs = len(ties["submap"])
    got = []
    if batch == "chunk":
        scans = csm.ScanSet(None, packed=(w.points, w.offsets))
        # The tied pairs among 256 other nodes of their submaps per launch.
        rng = np.random.RandomState(11)
        extra = rng.choice(w.num_nodes, 256, replace=False)
        local = {s: i for i, s in enumerate(subs)}
        sub_idx, node_idx = [], []
        for s in subs:
            nodes = sorted(set(extra.tolist()) | {int(n) for t, n in zip(ties["submap"], ties["node"])
                                                   if int(t) == s})
            sub_idx += [local[s]] * len(nodes)
            node_idx += nodes
        pairs = csm.make_pairs(sub_idx, node_idx, min_score, full_submap=True)
        res = csm.match_batch([mats[s] for s in subs], scans, pairs)
        assert_search_ok(csm, res["status"])
        where = {(subs[si], ni): k for k, (si, ni) in enumerate(zip(sub_idx, node_idx))}
        for k in range(n_pairs):
            r = res[where[(int(ties["submap"][k]), int(ties["node"][k]))]]
            got.append((int(r["status"]), float(r["score"]), (r["x"], r["y"], r["theta"]),
                        int(r["tie"])))
    else:
        def single(k):
            m = mats[int(ties["submap"][k])]
            ok, score, pose = m.MatchFullSubmap(w.cloud(int(ties["node"][k])), min_score)
            return (0 if ok else 1, score, tuple(pose), None)
        if batch == "single":
            got = [single(k) for k in range(n_pairs)]
        else:
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=8) as ex:
                got = list(ex.map(single, range(n_pairs)))
    for k, (status, score, pose, tie) in enumerate(got):
        s, n = int(ties["submap"][k]), int(ties["node"][k])
        assert status == csm.CSM_OK, (s, n, status)
        assert np.float32(score) == ties["score"][k], (s, n, score, ties["score"][k])
        assert tuple(pose) == tuple(ties["pose"][k]), (s, n, pose, tuple(ties["pose"][k]))
        if tie is not None:
            assert tie == ties["branch"][k], (s, n, tie, ties["branch"][k])
