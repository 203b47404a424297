"""Golden vectors (tests/golden/*.npz, written by tests/golden/make_golden.py
from the pinned oracle).

CPU: the oracle still reproduces them (guards against oracle drift; the
cheapest C2 pairs plus every local and RTCSM case).
GPU: the HIP path reproduces them through the C-ABI, both batched
(csm_fast2d_match_batch) and single-call (Match / MatchFullSubmap).
"""
import math
import os

import numpy as np
import pytest
from conftest import assert_search_ok

from conftest import ROOT

GOLDEN = os.path.join(ROOT, "tests", "golden")


def _load(name):
    return dict(np.load(os.path.join(GOLDEN, name)))


def _cloud(d, c):
    return d["points"][d["offsets"][c]:d["offsets"][c + 1]]


def _limits(d, s):
    res, mx, my = d["limits"][s]
    return float(res), float(mx), float(my)


def _full_center(d, s):
    res, mx, my = _limits(d, s)
    cells = d["cells"][s]
    return (mx - 0.5 * res * cells.shape[0], my - 0.5 * res * cells.shape[1], 0.0)


@pytest.mark.parametrize("name", ["fast2d_c2.npz", "fast2d_local.npz"])
def test_oracle_reproduces_fast2d_golden(oracle, name):
    d = _load(name)
    lin, ang, depth = d["options"]
    oms = {}
    cheap = np.argsort(d["reference_lookups"])
    budget = 2.5e9  # lookups, ~ a few seconds of oracle time
    checked = 0
    for i in cheap:
        if d["reference_lookups"][i] > budget and checked >= 3:
            break
        budget -= d["reference_lookups"][i]
        s, c, full = int(d["pairs"][i, 0]), int(d["pairs"][i, 1]), int(d["pairs"][i, 2])
        if s not in oms:
            oms[s] = oracle.fast2d(_limits(d, s), d["cells"][s], float(lin), float(ang), int(depth))
        ms = float(d["pairs"][i, 6])
        r = (oms[s].match_full_submap(_cloud(d, c), ms) if full
             else oms[s].match(tuple(d["pairs"][i, 3:6]), _cloud(d, c), ms))
        assert int(r[0]) == d["matched"][i]
        if r[0]:
            assert np.float32(r[1]) == d["score"][i]
            assert tuple(r[2]) == tuple(d["pose"][i])
        checked += 1
    assert checked >= 3


def test_oracle_reproduces_rt2d_golden(oracle):
    d = _load("rt2d_c1.npz")
    for i in range(len(d["score"])):
        s = int(d["grid"][i])
        sc, pose, _ = oracle.rt2d_match(_limits(d, s), d["cells"][s], tuple(d["options"]),
                                        tuple(d["initial"][i]), _cloud(d, i))
        assert sc == d["score"][i]
        assert tuple(pose) == tuple(d["pose"][i])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["fast2d_c2.npz", "fast2d_local.npz"])
def test_gpu_matches_fast2d_golden(csm, oracle, name):
    d = _load(name)
    lin, ang, depth = float(d["options"][0]), float(d["options"][1]), int(d["options"][2])
    opts = csm.FastCorrelativeScanMatcherOptions2D(lin, ang, depth)
    grids = [csm.ProbabilityGrid(*_limits(d, s), d["cells"][s]) for s in range(len(d["cells"]))]
    mats = [csm.FastCorrelativeScanMatcher2D(g, opts) for g in grids]
    scans = csm.ScanSet(None, packed=(d["points"], d["offsets"]))
    p = d["pairs"]
    pairs = csm.make_pairs(p[:, 0].astype(np.int32), p[:, 1].astype(np.int32), 0.0)
    pairs["full_submap"] = p[:, 2].astype(np.int32)
    pairs["min_score"] = p[:, 6]
    pairs["x"], pairs["y"], pairs["theta"] = p[:, 3], p[:, 4], p[:, 5]
    res = csm.match_batch(mats, scans, pairs)
    assert_search_ok(csm, res["status"])
    matched = 0
    for i in range(len(p)):
        s, c, full = int(p[i, 0]), int(p[i, 1]), bool(p[i, 2])
        ok = res["status"][i] == csm.CSM_OK
        assert int(ok) == d["matched"][i], (name, i)
        if full:
            single = mats[s].MatchFullSubmap(_cloud(d, c), float(p[i, 6]))
        else:
            single = mats[s].Match(tuple(p[i, 3:6]), _cloud(d, c), float(p[i, 6]))
        assert single[0] == ok
        if not ok:
            continue
        assert np.float32(res["score"][i]) == d["score"][i]
        assert np.float32(single[1]) == d["score"][i]
        gp = (float(res["x"][i]), float(res["y"][i]), float(res["theta"][i]))
        assert tuple(single[2]) == gp  # batch == single call
        matched += 1
        # The reference's pose, including its pick among exactly tied
        # leaves (csm_host.cc ResolveTies).
        assert gp == tuple(d["pose"][i]), (name, i, gp, tuple(d["pose"][i]))
        print(f"{name}: {matched} matched pairs, poses identical")


@pytest.mark.gpu
def test_gpu_matches_rt2d_golden(csm):
    d = _load("rt2d_c1.npz")
    o = d["options"]
    m = csm.RealTimeCorrelativeScanMatcher2D(
        csm.RealTimeCorrelativeScanMatcherOptions(*[float(v) for v in o]))
    for i in range(len(d["score"])):
        s = int(d["grid"][i])
        g = csm.ProbabilityGrid(*_limits(d, s), d["cells"][s])
        sc, pose = m.Match(tuple(d["initial"][i]), _cloud(d, i), g)
        # float sum in reference order; the double exp() penalty may differ from
        # glibc in the last ulps: 1e-6 relative (north star: 1e-4).
        assert math.isclose(sc, d["score"][i], rel_tol=1e-6, abs_tol=0), (i, sc, d["score"][i])
        assert tuple(pose) == tuple(d["pose"][i])


def _tsdf_case(d, i):
    s = int(d["grid"][i])
    return (tuple(float(v) for v in d[f"limits_{s}"]), d[f"tsd_{s}"], d[f"wgt_{s}"])


def test_oracle_reproduces_rt2d_tsdf_golden(oracle):
    d = _load("rt2d_tsdf.npz")
    for i in range(len(d["score"])):
        lim, tsd, wgt = _tsdf_case(d, i)
        sc, pose, _ = oracle.rt2d_match_tsdf(lim, tsd, wgt, float(d["truncation"]),
                                             float(d["max_weight"]), tuple(d["options"]),
                                             tuple(d["initial"][i]), _cloud(d, i))
        assert sc == d["score"][i]
        assert tuple(pose) == tuple(d["pose"][i])


@pytest.mark.gpu
def test_gpu_matches_rt2d_tsdf_golden(csm):
    d = _load("rt2d_tsdf.npz")
    m = csm.RealTimeCorrelativeScanMatcher2D(
        csm.RealTimeCorrelativeScanMatcherOptions(*[float(v) for v in d["options"]]))
    for i in range(len(d["score"])):
        lim, tsd, wgt = _tsdf_case(d, i)
        g = csm.TSDF2D(*lim, tsd, wgt, float(d["truncation"]), float(d["max_weight"]))
        sc, pose = m.Match(tuple(d["initial"][i]), _cloud(d, i), g)
        # TSDF sums are float, in reference order, so bit-identical; the double
        # exp() penalty may differ from glibc in the last ulps: 1e-6 relative.
        assert math.isclose(sc, d["score"][i], rel_tol=1e-6, abs_tol=0), (i, sc, d["score"][i])
        assert tuple(pose) == tuple(d["pose"][i])


# ------------------------------------------------------------------ 3D (C4/C5) --
def _cells3(d, kind, s):
    o = d[kind + "_off"]
    return d[kind + "_idx"][o[s]:o[s + 1]], d[kind + "_val"][o[s]:o[s + 1]]


def _node3(csm_or_none, d, n):
    from types import SimpleNamespace
    hi = d["high_points"][d["high_offsets"][n]:d["high_offsets"][n + 1]]
    lo = d["low_points"][d["low_offsets"][n]:d["low_offsets"][n + 1]]
    if csm_or_none is None:
        return SimpleNamespace(high_resolution_point_cloud=hi, low_resolution_point_cloud=lo,
                               rotational_scan_matcher_histogram=d["node_hist"][n],
                               gravity_alignment=(1.0, 0.0, 0.0, 0.0))
    return csm_or_none.NodeData3D(hi, lo, d["node_hist"][n])


def _pair3(row):
    s, n, full, ms = int(row[0]), int(row[1]), bool(row[2]), float(row[3])
    return s, n, full, ms, (tuple(row[4:7]), tuple(row[7:11])), (tuple(row[11:14]), tuple(row[14:18]))


def _oracle3(oracle, d):
    oms = []
    for s in range(len(d["submap_hist"])):
        oh, ol = oracle.hybrid_grid(float(d["high_resolution"])), oracle.hybrid_grid(float(d["low_resolution"]))
        oh.set_values(*_cells3(d, "high", s))
        ol.set_values(*_cells3(d, "low", s))
        oms.append((oh, ol, oracle.fast3d(oh, ol, d["submap_hist"][s],
                                          tuple(float(v) if i >= 2 else int(v)
                                                for i, v in enumerate(d["options"])))))
    return oms


def test_oracle_reproduces_fast3d_golden(oracle):
    d = _load("fast3d_c5.npz")
    oms = _oracle3(oracle, d)
    for i, row in enumerate(d["pairs"]):
        s, n, full, ms, npose, spose = _pair3(row)
        node = _node3(None, d, n)
        om = oms[s][2]
        r = om.match_full_submap(npose[1], spose[1], node, ms) if full else om.match(npose, spose, node, ms)
        assert int(r["matched"]) == d["matched"][i], i
        assert r["lookups"] == d["reference_lookups"][i]
        if r["matched"]:
            assert np.float32(r["score"]) == d["score"][i]
            assert r["pose"] == (tuple(d["t"][i]), tuple(d["q"][i]))
            assert np.float32(r["rotational_score"]) == d["rotational_score"][i]
            assert np.float32(r["low_resolution_score"]) == d["low_resolution_score"][i]


def test_oracle_reproduces_rt3d_golden(oracle):
    d = _load("rt3d_c4.npz")
    f = _load("fast3d_c5.npz")
    grids = {}
    for i in range(len(d["score"])):
        s = int(d["grid"][i])
        if s not in grids:
            grids[s] = oracle.hybrid_grid(float(f["high_resolution"]))
            grids[s].set_values(*_cells3(f, "high", s))
        init = (tuple(d["initial"][i][:3]), tuple(d["initial"][i][3:]))
        sc, pose, idx, ncand = oracle.rt3d_match(grids[s], tuple(d["options"]), init, _cloud(d, i))
        assert np.float32(sc) == d["score"][i]
        assert (tuple(pose[0]), tuple(pose[1])) == (tuple(d["pose"][i][:3]), tuple(d["pose"][i][3:]))
        assert (idx, ncand) == (d["candidate"][i], d["candidates"][i])


@pytest.mark.gpu
@pytest.mark.parametrize("yaw_build", ["device", "host", "retry"])
def test_gpu_matches_fast3d_golden(csm, oracle, yaw_build, monkeypatch):
    """Every discrete-scan pose path: built on the device (yaw_build, flag
    count read back with the results), the rerun with the flag check before
    the search that a flagged yaw triggers (libm fix-ups; CSM_YAW_FORCE_RETRY
    forces it) and the host path that a flag-list overflow falls back to
    (CSM_YAW_HOST_BUILD forces it)."""
    if yaw_build == "host":
        monkeypatch.setenv("CSM_YAW_HOST_BUILD", "1")
    if yaw_build == "retry":
        monkeypatch.setenv("CSM_YAW_FORCE_RETRY", "1")
    from test_fast3d_gpu import assert_same_result
    d = _load("fast3d_c5.npz")
    o = csm.FastCorrelativeScanMatcherOptions3D(*[int(v) if i < 2 else float(v)
                                                   for i, v in enumerate(d["options"])])
    grids, mats = [], []
    for s in range(len(d["submap_hist"])):
        gh = csm.HybridGrid(float(d["high_resolution"]), *_cells3(d, "high", s))
        gl = csm.HybridGrid(float(d["low_resolution"]), *_cells3(d, "low", s))
        grids.append((gh, gl))
        mats.append(csm.FastCorrelativeScanMatcher3D(gh, gl, d["submap_hist"][s], o))
    nodes = [_node3(csm, d, n) for n in range(len(d["node_hist"]))]
    rows = [_pair3(r) for r in d["pairs"]]
    res = csm.match_batch_3d(mats, nodes, [(s, n, full, ms, npose, spose)
                                           for s, n, full, ms, npose, spose in rows])
    assert_search_ok(csm, [r.status for r in res])
    oms = None
    for i, (s, n, full, ms, npose, spose) in enumerate(rows):
        single = (mats[s].MatchFullSubmap(npose[1], spose[1], nodes[n], ms) if full
                  else mats[s].Match(npose, spose, nodes[n], ms))
        assert (single is not None) == bool(d["matched"][i]) == (res[i].status == csm.CSM_OK), i
        if single is None:
            continue
        assert np.float32(single.score) == d["score"][i] == np.float32(res[i].score)
        assert single.pose_estimate == res[i].pose.as_tuple()  # batch == single call
        ref = {"matched": True, "score": float(d["score"][i]),
               "pose": (tuple(d["t"][i]), tuple(d["q"][i])),
               "rotational_score": float(d["rotational_score"][i]),
               "low_resolution_score": float(d["low_resolution_score"][i])}
        if single.pose_estimate != ref["pose"] and oms is None:
            oms = _oracle3(oracle, d)
        assert_same_result(single, ref, oms[s][2] if oms else None, full,
                           npose[1] if full else npose, spose[1] if full else spose,
                           _node3(None, d, n), o.min_low_resolution_score)


@pytest.mark.gpu
def test_gpu_matches_rt3d_golden(csm):
    d = _load("rt3d_c4.npz")
    f = _load("fast3d_c5.npz")
    m = csm.RealTimeCorrelativeScanMatcher3D(
        csm.RealTimeCorrelativeScanMatcherOptions(*[float(v) for v in d["options"]]))
    grids = {}
    for i in range(len(d["score"])):
        s = int(d["grid"][i])
        if s not in grids:
            grids[s] = csm.HybridGrid(float(f["high_resolution"]), *_cells3(f, "high", s))
        init = (tuple(d["initial"][i][:3]), tuple(d["initial"][i][3:]))
        score, pose = m.Match(init, _cloud(d, i), grids[s])
        # float sums in reference order; the double exp() penalty may differ
        # from glibc in the last ulps: 1e-6 relative (north star: 1e-4).
        assert math.isclose(score, float(d["score"][i]), rel_tol=1e-6), (i, score)
        assert pose == (tuple(d["pose"][i][:3]), tuple(d["pose"][i][3:]))
