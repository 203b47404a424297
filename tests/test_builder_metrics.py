"""Observability of the constraint-builder drop-ins (C++ headers and Python
mirror): the metric families (constraint_builder_2d.cc:46-53, :318-343;
constraint_builder_3d.cc:46-59, :351-386), the score histograms
(common/histogram.cc:27-75; :239, :257-259) and the log_matches lines
(:260-300; 3D :284-326).

CPU: common::Histogram::ToString restated twice (metrics.h, metrics.py) and
pinned on a hand-worked case; the metric interfaces. GPU: a scripted sweep
through the C++ builders (tests/cpp/builder_metrics_test.cc) and the same
script through the Python mirror: counters, gauges and histogram buckets
against the script's own counts, and the two implementations against each
other (constraints, ToString, every log line).
"""
import json
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

CPP_SRC = os.path.join(ROOT, "tests", "cpp", "builder_metrics_test.cc")
CPP_BIN = os.path.join(ROOT, "tests", "cpp", "_build", "builder_metrics_test")


@pytest.fixture(scope="module")
def bin_path(csm):
    os.makedirs(os.path.dirname(CPP_BIN), exist_ok=True)
    libdir = os.path.join(ROOT, "cartographer-1_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I",
                           os.path.join(ROOT, "include"), CPP_SRC, "-o", CPP_BIN, "-L", libdir,
                           "-lcsm_amd", "-Wl,-rpath," + libdir])
    return CPP_BIN


@pytest.fixture(scope="module")
def mt(csm):
    import importlib
    return importlib.import_module("cartographer_amd.metrics")


@pytest.fixture(scope="module")
def cb(csm):
    import importlib
    return importlib.import_module("cartographer_amd.constraint_builder")


def _cpp_hist(bin_path, values):
    return subprocess.run([bin_path, "hist", *[repr(float(v)) for v in values]],
                          capture_output=True, text=True, check=True).stdout


def test_histogram_hand_worked_case(mt, bin_path):
    """Values {0, 1}, 10 buckets: the string common::Histogram::ToString
    builds for them, worked by hand from histogram.cc:27-75."""
    want = "Count: 2  Min: 0  Max: 1  Mean: 0.5"
    total = 0
    for i in range(10):
        lo, hi = i / 10, (i + 1) / 10
        c = 1 if i in (0, 9) else 0
        total += c
        bar = " " * 10 + "#" * 10 if c else " " * 20
        want += "\n[%f, %f%s\t%s\tCount: %d (%s%%)\tTotal: %d (%s%%)" % (
            lo, hi, "]" if i == 9 else ")", bar, c, "50" if c else "0", total,
            "50" if total == 1 else "100")
    h = mt.ScoreHistogram()
    h.Add(0.0)
    h.Add(1.0)
    assert h.ToString(10) == want
    assert _cpp_hist(bin_path, [0.0, 1.0]) == want


def test_histogram_cpp_and_python_agree(mt, bin_path):
    rng = np.random.default_rng(3)
    cases = [[], [0.7], [0.55, 0.55, 0.55], list(rng.uniform(0.5, 0.9, 37)),
             list(rng.uniform(0.0, 1.0, 500)), [0.1, 0.9, 0.9, 0.1, 0.5]]
    for vals in cases:
        vals = [float(np.float32(v)) for v in vals]
        h = mt.ScoreHistogram()
        for v in vals:
            h.Add(v)
        assert h.ToString(10) == _cpp_hist(bin_path, vals), vals


def test_metric_interfaces(mt):
    assert mt.Histogram.FixedWidth(0.05, 20) == pytest.approx([0.05 * k for k in range(1, 21)])
    assert mt.Histogram.ScaledPowersOf(2, 1, 10) == [1, 2, 4, 8]
    mt.Counter.Null().Increment()
    mt.Gauge.Null().Set(3)
    mt.Histogram.Null().Observe(0.5)
    f = mt.InMemoryFamilyFactory()
    c = f.NewCounterFamily("c", "d").Add({"a": "1"})
    c.Increment()
    c.Increment(2.5)
    assert f.get("c", {"a": "1"}).value == 3.5 and f.get("c", {"a": "2"}) is None
    h = f.NewHistogramFamily("h", "d", [0.5, 1.0]).Add({})
    for v in (0.2, 0.5, 0.7, 1.0, 3.0):
        h.Observe(v)
    assert h.counts == [2, 2, 1] and h.count == 5  # bucket k: <= boundaries[k]


# ------------------------------------------------------------- GPU sweep --

def _sweep_cells():
    cells = np.zeros((80, 80), np.uint16)
    ring = np.zeros((80, 80), bool)
    ring[20:61, 20:61] = True
    inner = np.zeros((80, 80), bool)
    inner[21:60, 21:60] = True
    cells[ring] = 1
    cells[inner] = 32767
    return cells


def _sweep_cloud(k):
    def coord(i):
        return np.float32(2.0 - (i + 0.5) * 0.05)
    pts = []
    for j in range(10):
        i = 22 + 4 * j
        pts += [(coord(20), coord(i)), (coord(60), coord(i)), (coord(i), coord(20)),
                (coord(i), coord(60))]
    for j in range(5 * k):
        pts.append((coord(30 + (j * 7) % 21), coord(30 + (j * 3) % 19)))
    return np.array([(x, y, 0.0) for x, y in pts], np.float32)


def _python_sweep(csm, cb, mt):
    """tests/cpp/builder_metrics_test.cc Sweep(), through the Python mirror."""
    factory = mt.InMemoryFamilyFactory()
    cb.ConstraintBuilder2D.RegisterMetrics(factory)
    cb.ConstraintBuilder3D.RegisterMetrics(factory)
    log = []
    m2, m3 = "mapping_constraints_constraint_builder_2d_", "mapping_constraints_constraint_builder_3d_"

    def counter(name, region, what):
        c = factory.get(name, {"search_region": region, "matcher": what})
        return c.value if c else -1.0

    def gauge(name):
        g = factory.get(name, {})
        return g.value if g else -1.0

    def hist(name, labels):
        h = factory.get(name, labels)
        return None if h is None else list(h.counts)

    out = {}
    o = cb.ConstraintBuilderOptions(sampling_ratio=1.0, min_score=np.float32(0.3),
                                    global_localization_min_score=np.float32(0.35))
    b = cb.ConstraintBuilder2D(o)
    b.log_sink = lambda line: log.append("2d " + line)
    grid = csm.ProbabilityGrid(0.05, 2.0, 2.0, _sweep_cells())
    s0 = cb.Submap2D(grid, (0.0, 0.0, 0.0))
    s1 = cb.Submap2D(grid, (0.3, -0.2, 0.1))
    clouds = [_sweep_cloud(k) for k in range(6)]
    for k in range(6):
        b.MaybeAddConstraint((0, 0), s0, (0, k), clouds[k], (0.02 * k, -0.01 * k, 0.01))
        b.MaybeAddConstraint((0, 1), s1, (0, k), clouds[k],
                             cb.rigid2d_compose(cb.rigid2d_inverse(s1.local_pose),
                                                (0.03, 0.02 * k, -0.02)))
        if k % 2 == 0:
            b.MaybeAddGlobalConstraint((0, 1), s1, (0, k), clouds[k])
        b.NotifyEndOfNode()
    b.MaybeAddConstraint((0, 0), s0, (0, 9), clouds[0], (20.0, 0.0, 0.0))  # filtered
    out["queue_2d"] = gauge(m2 + "queue_length")
    out["matchers_2d"] = gauge(m2 + "num_submap_scan_matchers")
    got = []
    b.WhenDone(got.append)
    out["constraints_2d"] = [[c.submap_id[1], c.node_id[1], float(np.float32(c.score)),
                              *c.relative_pose] for c in got[0]]
    out["queue_2d_after"] = gauge(m2 + "queue_length")
    b.DeleteScanMatcher((0, 0))
    out["matchers_2d_after_delete"] = gauge(m2 + "num_submap_scan_matchers")
    out["counters_2d"] = [counter(m2 + "constraints", r, w) for r, w in
                          (("local", "searched"), ("local", "found"), ("global", "searched"),
                           ("global", "found"))]
    out["hist_2d_local"] = hist(m2 + "scores", {"search_region": "local"})
    out["hist_2d_global"] = hist(m2 + "scores", {"search_region": "global"})
    out["tostring_2d"] = b.score_histogram.ToString(10)

    f3 = csm.FastCorrelativeScanMatcherOptions3D(min_rotational_score=0.0,
                                                  min_low_resolution_score=0.0)
    o3 = cb.ConstraintBuilderOptions(sampling_ratio=1.0, min_score=0.0,
                                     global_localization_min_score=0.0,
                                     fast_correlative_scan_matcher_options_3d=f3)
    b3 = cb.ConstraintBuilder3D(o3)
    b3.log_sink = lambda line: log.append("3d " + line)
    empty = (np.zeros((0, 3), np.int32), np.zeros(0, np.uint16))
    sub3 = cb.Submap3D(0.1, empty, 0.1, empty, np.zeros(3, np.float32))
    pt = np.array([[0.1, 0.2, 0.3]], np.float32)
    node = csm.NodeData3D(pt, pt, np.zeros(3, np.float32))
    ident = ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))
    for rnd in range(2):
        for _ in range(2):
            b3.MaybeAddConstraint((0, 1), sub3, (0, 0), node, ident, ident)
        b3.MaybeAddGlobalConstraint((0, 1), sub3, (0, 0), node, (1, 0, 0, 0), (1, 0, 0, 0))
        b3.NotifyEndOfNode()
        if rnd == 0:
            out["queue_3d"] = gauge(m3 + "queue_length")
        b3.WhenDone(lambda r: None)
    out["queue_3d_after"] = gauge(m3 + "queue_length")
    out["counters_3d"] = [counter(m3 + "constraints", r, w) for r, w in
                          (("local", "searched"), ("local", "found"), ("global", "searched"),
                           ("global", "found"))]
    for region in ("local", "global"):
        for kind in ("score", "rotational_score", "low_resolution_score"):
            out[f"hist_3d_{region}_{kind}"] = hist(m3 + "scores",
                                                   {"search_region": region, "kind": kind})
    out["log"] = log
    return out


def _bucket(v, bounds):
    return sum(1 for b in bounds if v > b)


@pytest.mark.gpu
def test_scripted_sweep_cpp_and_python(csm, cb, mt, bin_path):
    r = subprocess.run([bin_path, "sweep"], capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    cpp = json.loads(r.stdout)
    py = _python_sweep(csm, cb, mt)
    # The script's own counts: 12 local and 3 global pairs queued (the far
    # pair filtered), every node matching its ring.
    for got in (cpp, py):
        cons = got["constraints_2d"]
        assert got["queue_2d"] == 15 and got["queue_2d_after"] == 0
        assert got["matchers_2d"] == 2 and got["matchers_2d_after_delete"] == 1
        searched_l, found_l, searched_g, found_g = got["counters_2d"]
        assert (searched_l, searched_g) == (12, 3)
        assert found_l + found_g == len(cons) and found_l >= 6 and found_g >= 1
        bounds = [0.05 * k for k in range(1, 21)]
        hl, hg = got["hist_2d_local"], got["hist_2d_global"]
        assert sum(hl) == found_l and sum(hg) == found_g
        want = np.zeros(21, int)
        for c in cons:
            want[_bucket(c[2], bounds)] += 1
        assert (np.array(hl) + np.array(hg) == want).all()
        assert got["tostring_2d"].startswith(f"Count: {len(cons)}  Min: ")
        # 3D FindsConstraints inputs: 3 pairs a round, all found (score 0.1).
        assert got["queue_3d"] == 3 and got["queue_3d_after"] == 0
        assert got["counters_3d"] == [4, 4, 2, 2]
        assert got["hist_3d_local_score"][_bucket(float(np.float32(0.1)), bounds)] == 4
        assert sum(got["hist_3d_global_low_resolution_score"]) == 2
        log = got["log"]
        lines_2d = [x for x in log if x.startswith("2d Node")]
        assert len(lines_2d) == len(cons)
        assert sum(" matches with score " in x for x in lines_2d) == found_g
        assert f"2d 15 computations resulted in {len(cons)} additional constraints." in log
        assert "2d Score histogram:\n" + got["tostring_2d"] in log
        assert sum(x.startswith("3d 3 computations resulted in 3 additional constraints.\n"
                                "Score histogram:\nCount: ") for x in log) == 2
    # The two implementations agree line for line.
    assert cpp["log"] == py["log"]
    assert cpp["tostring_2d"] == py["tostring_2d"]
    # Same matches and the same refinement (the Ceres kernel's reductions are
    # deterministic): only the Rigid2d algebra's last bits may differ.
    for a, b in zip(cpp["constraints_2d"], py["constraints_2d"]):
        assert a[:3] == b[:3] and np.allclose(a[3:], b[3:], rtol=0, atol=1e-12), (a, b)
    for k in cpp:
        if k not in ("log", "constraints_2d"):
            assert cpp[k] == py[k], k
    # A global line and a local one, as the reference formats them (:260-276).
    g = next(x for x in cpp["log"] if " matches " in x)
    assert g.startswith("2d Node (0, 0) with 40 points on submap (0, 1) matches with score ")
    loc = next(x for x in cpp["log"] if "differs by translation" in x)
    assert loc.startswith("2d Node (0, 0) with 40 points on submap (0, 0) differs by translation ")
