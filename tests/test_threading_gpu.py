"""The §8(b) threading contract: single Match / MatchFullSubmap calls from
many host threads at once.

The reference schedules one common::Task per (node, submap) pair on its
ThreadPool and every worker calls the const Match methods of a shared
FastCorrelativeScanMatcher2D concurrently (constraint_builder_2d.cc:100-111,
:169-170, :213-228; fast_correlative_scan_matcher_2d.h:127-136). Here each
call takes a call context of the matcher's context (own stream and scratch,
csm_internal.h), so concurrent calls must give exactly the results of the
oracle (2D) or of the already oracle-checked batch path (3D), whatever the
interleaving. ctypes releases the GIL during the C calls, so the Python
threads really overlap in the library.
"""
import math
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = 8
# Low enough that most of the cases below match (18 of 28 in the oracle).
MIN_SCORE = 0.3


@pytest.fixture(scope="module")
def world(csm):
    return csm.SyntheticWorld2D(num_nodes=40, num_submaps=4, decimate_to=200, seed=20250127)


@pytest.fixture(scope="module")
def cases(csm, oracle, world):
    """(submap, node, full, initial) cases with the oracle's results."""
    w = world
    rng = np.random.RandomState(3)
    out = []
    for s in range(w.num_submaps):
        c = int(w.submap_nodes[s])
        for n in sorted({c, min(c + 1, w.num_nodes - 1), int(rng.randint(w.num_nodes)),
                         int(rng.randint(w.num_nodes))}):
            out.append((s, n, True, None))
            # Match() near the node's pose in the submap frame (the synthetic
            # world's submap frame is the map frame).
            p = w.node_poses[n]
            out.append((s, n, False, (p[0] + 0.12, p[1] - 0.08, p[2] + 0.03)))
    opts = (7.0, math.radians(30.0), 7)
    oms = {}
    for s in range(w.num_submaps):
        g = w.grid(s)
        oms[s] = oracle.fast2d((g.resolution, g.max_x, g.max_y), g.cells, *opts)

    def ref(case):
        s, n, full, init = case
        om = oms[s]
        r = (om.match_full_submap(w.cloud(n), MIN_SCORE) if full
             else om.match(init, w.cloud(n), MIN_SCORE))
        return r[:3]

    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        refs = list(ex.map(ref, out))
    return out, refs


def _mats(csm, world, ctx=None):
    opts = csm.FastCorrelativeScanMatcherOptions2D(7.0, math.radians(30.0), 7)
    return [csm.FastCorrelativeScanMatcher2D(world.grid(s), opts, ctx)
            for s in range(world.num_submaps)]


def _run(mats, world, case):
    s, n, full, init = case
    m = mats[s]
    return (m.MatchFullSubmap(world.cloud(n), MIN_SCORE) if full
            else m.Match(init, world.cloud(n), MIN_SCORE))


def _check(got, refs, cases):
    matched = 0
    for case, g, r in zip(cases, got, refs):
        assert g[0] == r[0], (case, g, r)
        if r[0]:
            matched += 1
            assert np.float32(g[1]) == np.float32(r[1]), (case, g, r)
            assert tuple(g[2]) == tuple(r[2]), (case, g, r)
    assert matched >= 4


def test_threads_on_one_handle(csm, world, cases):
    """8 threads calling MatchFullSubmap / Match on ONE matcher."""
    cs, refs = cases
    mats = _mats(csm, world, csm.Context(0))
    one = [c for c in cs if c[0] == 0] * 3   # every submap-0 case, three times over
    one_refs = [r for c, r in zip(cs, refs) if c[0] == 0] * 3
    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        got = list(ex.map(lambda c: _run(mats, world, c), one))
    _check(got, one_refs, one)


def test_threads_on_several_handles(csm, world, cases):
    """8 threads over every case, the matchers of one context, twice over
    with timing enabled: single calls are counted in the owner's timing, and
    concurrent ones share launches."""
    cs, refs = cases
    ctx = csm.Context(0)
    mats = _mats(csm, world, ctx)
    ctx.reset_timing()
    ctx.enable_timing(True)
    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        got = list(ex.map(lambda c: _run(mats, world, c), cs + cs))
    ctx.enable_timing(False)
    _check(got, refs + refs, cs + cs)
    t = ctx.timing()
    # Concurrent calls are coalesced into batches (csm_host.cc SingleMatch):
    # fewer launches than calls, every call counted once among them.
    assert 1 <= t.search_launches < 2 * len(cs), t.search_launches
    assert t.search_errors == 0


def test_threads_mixed_with_batches(csm, world, cases):
    """Single calls on one context's matchers while another thread runs batch
    searches over the same matchers on the same context."""
    cs, refs = cases
    ctx = csm.Context(0)
    mats = _mats(csm, world, ctx)
    scans = csm.ScanSet(None, ctx, packed=(world.points, world.offsets))
    full = [(k, c) for k, c in enumerate(cs) if c[2]]
    pairs = csm.make_pairs([c[0] for _, c in full], [c[1] for _, c in full], MIN_SCORE, True)

    def batch(_):
        return csm.match_batch(mats, scans, pairs, ctx)

    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        fb = [ex.submit(batch, i) for i in range(3)]
        fs = [ex.submit(_run, mats, world, c) for c in cs]
        got = [f.result() for f in fs]
        batches = [f.result() for f in fb]
    _check(got, refs, cs)
    for res in batches:
        for (k, c), r in zip(full, res):
            ref = refs[k]
            assert (r["status"] == csm.CSM_OK) == ref[0], (c, r, ref)
            if ref[0]:
                assert np.float32(r["score"]) == np.float32(ref[1])
                assert (r["x"], r["y"], r["theta"]) == tuple(ref[2])


def test_threads_3d_single_calls(csm):
    """FastCorrelativeScanMatcher3D: 8 threads calling MatchFullSubmap and
    Match on one matcher give the batch path's results (the batch is checked
    against the oracle in test_fast3d_gpu.py)."""
    w = csm.SyntheticWorld3D(num_nodes=16, num_submaps=1, seed=99)
    o = csm.FastCorrelativeScanMatcherOptions3D()
    gm = csm.FastCorrelativeScanMatcher3D(csm.HybridGrid(w.high_resolution, *w.high_cells[0]),
                                          csm.HybridGrid(w.low_resolution, *w.low_cells[0]),
                                          w.submap_hist[0], o)
    ident = ((0, 0, 0), (1, 0, 0, 0))
    nodes = [w.node(n) for n in range(w.num_nodes)]
    pairs = []
    for n in range(w.num_nodes):
        truth = w.node_in_submap(n, 0)
        pairs.append((0, n, True, 0.55, ((0, 0, 0), w.node_rotation(n)), ident))
        pairs.append((0, n, False, 0.55, ((truth[0][0] + 0.3, truth[0][1] - 0.2, 0.1), truth[1]),
                      ident))
    batch = csm.match_batch_3d([gm], nodes, pairs)

    def single(p):
        _, n, full, ms, npose, spose = p
        return (gm.MatchFullSubmap(npose[1], spose[1], nodes[n], ms) if full
                else gm.Match(npose, spose, nodes[n], ms))

    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        got = list(ex.map(single, pairs * 2))
    matched = 0
    for p, g, r in zip(pairs * 2, got, batch * 2):
        assert (g is not None) == (r.status == csm.CSM_OK), (p, g, r.status)
        if g is not None:
            matched += 1
            assert np.float32(g.score) == np.float32(r.score)
            assert g.pose_estimate == r.pose.as_tuple()
    assert matched >= 2


def test_threads_3d_single_calls_several_matchers(csm):
    """Concurrent single 3D calls on three matchers of one context are
    coalesced into shared batches (host3d.cc SingleMatch3): 16 threads, each
    result equal to the batch path's for the same pair."""
    w = csm.SyntheticWorld3D(num_nodes=24, num_submaps=3, seed=7)
    o = csm.FastCorrelativeScanMatcherOptions3D()
    ctx = csm.Context(0)
    ms = [csm.FastCorrelativeScanMatcher3D(csm.HybridGrid(w.high_resolution, *w.high_cells[s], context=ctx),
                                           csm.HybridGrid(w.low_resolution, *w.low_cells[s], context=ctx),
                                           w.submap_hist[s], o, ctx)
          for s in range(w.num_submaps)]
    ident = ((0, 0, 0), (1, 0, 0, 0))
    nodes = [w.node(n) for n in range(w.num_nodes)]
    pairs = [(s, n, True, 0.55, ((0, 0, 0), w.node_rotation(n)), ident)
             for s in range(w.num_submaps) for n in range(w.num_nodes)]
    batch = csm.match_batch_3d(ms, nodes, pairs, ctx)

    def single(p):
        s, n, _, ms_, npose, spose = p
        return ms[s].MatchFullSubmap(npose[1], spose[1], nodes[n], ms_)

    with ThreadPoolExecutor(max_workers=16) as ex:
        got = list(ex.map(single, pairs * 2))
    matched = 0
    for p, g, r in zip(pairs * 2, got, batch * 2):
        assert (g is not None) == (r.status == csm.CSM_OK), (p, g, r.status)
        if g is not None:
            matched += 1
            assert np.float32(g.score) == np.float32(r.score)
            assert g.pose_estimate == r.pose.as_tuple()
    assert matched >= 4


def test_cpp_threads_match_single_thread_results():
    """The threading contract from C++ threads (no GIL): 16 threads call
    csm_fast2d_match_full_submap on shared matchers at once; every result
    equals the single-threaded one (tools/dropin_threads.cc --check)."""
    import json
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                       "dropin_threads")
    assert os.path.exists(exe), "build() makes tools/dropin_threads"
    out = subprocess.run([exe, "0", "0.55", "--check"], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, (out.stdout, out.stderr)
    r = json.loads(out.stdout.strip().splitlines()[-1])
    assert r["mismatches"] == 0 and r["matched"] > 0, r
