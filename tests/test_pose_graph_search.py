"""PoseGraph2D's constraint-search enumeration (pose_graph_2d.cc:260-425) in
the C++ header (include/cartographer_amd/pose_graph_2d_search.h) and its
Python mirror, with a recording builder (no GPU). The small cases restate the
reference's control flow; the scripted random scenario runs both mirrors and
compares every builder call. Parity unpinned against the reference binary
(it cannot be built here): the anchors are the reference's
code paths cited below."""
import math
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

CPP_TEST = os.path.join(ROOT, "tests", "cpp", "pose_graph_search_test.cc")
CPP_BIN = os.path.join(ROOT, "tests", "cpp", "_build", "pose_graph_search_test")


@pytest.fixture(scope="session")
def pg(csm):
    import importlib
    return importlib.import_module("cartographer_amd.pose_graph")


class Recorder:
    def __init__(self):
        self.log = []

    def MaybeAddConstraint(self, s, submap, n, cloud, rel):
        self.log.append(("L", tuple(n), tuple(s), tuple(round(v, 9) for v in rel)))

    def MaybeAddGlobalConstraint(self, s, submap, n, cloud):
        self.log.append(("G", tuple(n), tuple(s)))

    def NotifyEndOfNode(self):
        self.log.append(("E",))


class _C:
    def __init__(self, n, s):
        self.node_id, self.submap_id = n, s


def test_same_trajectory_is_local_with_relative_pose(pg):
    r = Recorder()
    g = pg.PoseGraph2DConstraintSearch(pg.PoseGraphSearchOptions(), r)
    g.AddSubmap((0, 0), None, (1.0, 2.0, 0.5))
    g.AddNode((0, 0), 0.0, (1.0, 2.0, 0.5), None, [(0, 0)], True)  # finishes (0,0)
    g.AddNode((0, 1), 1.0, (3.0, 1.0, 0.1), None, [], False)
    calls = [c for c in r.log if c[0] != "E"]
    assert len(calls) == 1 and calls[0][:3] == ("L", (0, 1), (0, 0))
    # submap.global_pose.inverse() * node.global_pose (:293-297)
    c, s = math.cos(-0.5), math.sin(-0.5)
    exp = (c * 2.0 - s * -1.0, s * 2.0 + c * -1.0, 0.1 - 0.5)
    assert np.allclose(calls[0][3], exp, atol=1e-9)


def test_unconnected_trajectory_early_node_is_local(pg):
    """A never-connected trajectory pair reads the epoch (0) as its last
    connection time (trajectory_connectivity_state.cc:67-70), so a node of
    another trajectory earlier than global_constraint_search_after_n_seconds
    gets a local search (pose_graph_2d.cc:276-282), a later one a global one.
    Both mirrors run the same script."""
    ops = [("S", (0, 0), (0.0, 0.0, 0.0)),
           ("N", (0, 0), 0.0, (0.0, 0.0, 0.0), 1, [(0, 0)]),
           ("N", (1, 0), 5.0, (0.0, 0.0, 0.0), 0, []),     # t < 10 s: local
           ("N", (1, 1), 12.0, (0.0, 0.0, 0.0), 0, [])]    # t >= 10 s: global
    want = [("L", (1, 0), (0, 0)), ("G", (1, 1), (0, 0))]
    py = _run_python(pg, ops, 1.0, 10.0)
    assert [c[:3] for c in py if c[0] != "E"] == want
    _build_cpp_search()
    out = subprocess.run([CPP_BIN, "1.0", "10.0"], input=_script(ops), capture_output=True,
                         text=True, timeout=60, check=True).stdout
    assert [c[:3] for c in _parse_cpp(out) if c[0] != "E"] == want
    assert pg.TrajectoryConnectivityState().LastConnectionTime(0, 1) == 0.0


def test_order_finished_submaps_then_old_nodes(pg):
    """:364-393: the node against every finished submap in SubmapId order, then
    the newly finished submap against older nodes in NodeId order, skipping
    the nodes inserted into it."""
    r = Recorder()
    g = pg.PoseGraph2DConstraintSearch(pg.PoseGraphSearchOptions(), r)
    for i in range(3):
        g.AddSubmap((0, i), None, (float(i), 0.0, 0.0))
    g.AddNode((0, 0), 0.0, (0, 0, 0), None, [(0, 0)], False)
    g.AddNode((0, 1), 1.0, (0, 0, 0), None, [(0, 0), (0, 1)], True)   # (0,0) finished
    g.AddNode((0, 2), 2.0, (0, 0, 0), None, [(0, 1), (0, 2)], False)
    g.AddNode((0, 3), 3.0, (0, 0, 0), None, [(0, 1), (0, 2)], True)   # (0,1) finished
    seq = [(c[0], c[1], c[2]) if c[0] != "E" else ("E",) for c in r.log]
    assert seq == [("E",), ("E",),
                   ("L", (0, 2), (0, 0)), ("E",),
                   ("L", (0, 3), (0, 0)), ("L", (0, 0), (0, 1)), ("E",)]


def test_other_trajectory_global_sampled_until_connected(pg):
    """:276-290: another trajectory is searched globally when its sampler
    pulses; after a loop closure the search is local for
    global_constraint_search_after_n_seconds past the connection time."""
    r = Recorder()
    g = pg.PoseGraph2DConstraintSearch(pg.PoseGraphSearchOptions(0.5, 10.0), r)
    g.AddSubmap((0, 0), None, (0, 0, 0))
    g.AddNode((0, 0), 0.0, (0, 0, 0), None, [(0, 0)], True)
    g.AddSubmap((1, 0), None, (0, 0, 0))
    for i in range(4):
        g.AddNode((1, i), 100.0 + i, (0, 0, 0), None, [(1, 0)], False)
    kinds = [c[0] for c in r.log if c[0] != "E"]
    assert kinds == ["G", "G"]  # ratio 0.5: pulses 1 and 3 of 4
    g.HandleConstraints([_C((1, 3), (0, 0))])
    # Latest node time of ((1,3), (0,0)) = max(103, time of (0,0)'s last node) = 103.
    assert g.connectivity.LastConnectionTime(0, 1) == 103.0
    r.log.clear()
    g.AddNode((1, 4), 112.5, (0, 0, 0), None, [(1, 0)], False)
    g.AddNode((1, 5), 113.5, (0, 0, 0), None, [(1, 0)], False)
    kinds = [c[0] for c in r.log if c[0] != "E"]
    assert kinds[0] == "L" and (len(kinds) == 1 or kinds[1] == "G")


def test_connectivity_joins_components(pg):
    """trajectory_connectivity_state.cc:25-52: joining two components stamps
    every bipartite pair; within a component only the pair is updated."""
    t = pg.TrajectoryConnectivityState()
    for i in range(4):
        t.Add(i)
    t.Connect(0, 1, 5.0)
    t.Connect(2, 3, 6.0)
    t.Connect(1, 2, 7.0)
    assert t.LastConnectionTime(0, 3) == 7.0 and t.LastConnectionTime(0, 1) == 5.0
    t.Connect(0, 3, 9.0)
    assert t.LastConnectionTime(0, 3) == 9.0 and t.LastConnectionTime(1, 3) == 7.0
    assert t.LastConnectionTime(0, 9) == 0.0  # the epoch: never connected
    assert t.TransitivelyConnected(0, 3) and not t.TransitivelyConnected(0, 9)


def _scenario(seed):
    rng = np.random.RandomState(seed)
    lines, ops = [], []
    node_idx = {0: 0, 1: 0, 2: 0}
    sub_idx = {0: 0, 1: 0, 2: 0}
    active = {}
    t = 0.0
    found = []
    for step in range(240):
        traj = int(rng.choice(3, p=[0.5, 0.3, 0.2]))
        if traj not in active or rng.rand() < 0.1:
            s = (traj, sub_idx[traj])
            sub_idx[traj] += 1
            pose = tuple(float(v) for v in np.round(rng.uniform(-20, 20, 3), 6))
            ops.append(("S", s, pose))
            active.setdefault(traj, []).append([s, 0])
        t += float(np.round(rng.uniform(0.1, 3.0), 3))
        n = (traj, node_idx[traj])
        node_idx[traj] += 1
        ins = [a[0] for a in active[traj][-2:]]
        for a in active[traj][-2:]:
            a[1] += 1
        fin = len(active[traj]) >= 2 and active[traj][-2][1] >= 4
        if fin:
            ins = [active[traj][-2][0]] + [a[0] for a in active[traj][-1:]]
            active[traj].pop(-2)
        pose = tuple(float(v) for v in np.round(rng.uniform(-20, 20, 3), 6))
        ops.append(("N", n, t, pose, int(fin), ins))
        found.append(n)
        if rng.rand() < 0.05 and step > 20:
            other = int(rng.choice([k for k in sub_idx if sub_idx[k] > 0]))
            ops.append(("C", n, (other, 0)))
    return ops


def _run_python(pg, ops, ratio, after):
    r = Recorder()
    g = pg.PoseGraph2DConstraintSearch(pg.PoseGraphSearchOptions(ratio, after), r)
    for op in ops:
        if op[0] == "S":
            g.AddSubmap(op[1], None, op[2])
        elif op[0] == "N":
            g.AddNode(op[1], op[2], op[3], None, op[5], bool(op[4]))
        else:
            g.HandleConstraints([_C(op[1], op[2])])
    return r.log


def _script(ops):
    out = []
    for op in ops:
        if op[0] == "S":
            out.append("S %d %d %r %r %r" % (*op[1], *op[2]))
        elif op[0] == "N":
            ins = " ".join("%d %d" % s for s in op[5])
            out.append("N %d %d %r %r %r %r %d %d %s" % (*op[1], op[2], *op[3], op[4],
                                                         len(op[5]), ins))
        else:
            out.append("C %d %d %d %d" % (*op[1], *op[2]))
    return "\n".join(out) + "\n"


def _parse_cpp(text):
    log = []
    for line in text.splitlines():
        f = line.split()
        if f[0] == "E":
            log.append(("E",))
        elif f[0] == "G":
            log.append(("G", (int(f[1]), int(f[2])), (int(f[3]), int(f[4]))))
        else:
            log.append(("L", (int(f[1]), int(f[2])), (int(f[3]), int(f[4])),
                        tuple(round(float(v), 9) for v in f[5:8])))
    return log


def _build_cpp_search():
    os.makedirs(os.path.dirname(CPP_BIN), exist_ok=True)
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I",
                           os.path.join(ROOT, "include"), CPP_TEST, "-o", CPP_BIN,
                           "-L", os.path.join(ROOT, "cartographer-1_amd"), "-lcsm_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "cartographer-1_amd")])


def test_cpp_header_and_python_mirror_agree(pg):
    _build_cpp_search()
    for seed, ratio, after in [(1, 0.003, 10.0), (2, 0.3, 10.0), (3, 1.0, 5.0)]:
        ops = _scenario(seed)
        py = _run_python(pg, ops, ratio, after)
        out = subprocess.run([CPP_BIN, repr(ratio), repr(after)], input=_script(ops),
                             capture_output=True, text=True, timeout=60, check=True).stdout
        cpp = _parse_cpp(out)
        assert len(py) == len(cpp)
        for a, b in zip(py, cpp):
            assert a[:3] == b[:3]
            if a[0] == "L":
                assert np.allclose(a[3], b[3], atol=2e-9)
        assert sum(1 for c in py if c[0] == "G") > 0 or ratio < 0.01


@pytest.mark.gpu
def test_sweep_through_the_gpu_builder(csm, pg):
    """Two trajectories over the synthetic world: trajectory 0 builds and
    finishes submaps (local searches), trajectory 1 localizes against them
    (global MatchFullSubmap searches, sampler ratio 1). The real
    ConstraintBuilder2D receives exactly the recorder's pairs, and the loop
    closures it finds connect the trajectories."""
    import importlib
    cb = importlib.import_module("cartographer_amd.constraint_builder")
    world = csm.SyntheticWorld2D(num_nodes=40, num_submaps=4, decimate_to=200, seed=11)
    opts = cb.ConstraintBuilderOptions(sampling_ratio=1.0, max_constraint_distance=1e9,
                                       min_score=0.5, global_localization_min_score=0.55)
    builder = cb.ConstraintBuilder2D(opts)
    rec = Recorder()
    sopts = pg.PoseGraphSearchOptions(1.0, 10.0)
    graphs = [pg.PoseGraph2DConstraintSearch(sopts, builder),
              pg.PoseGraph2DConstraintSearch(sopts, rec)]
    submaps = {s: cb.Submap2D(world.grid(s)) for s in range(4)}
    for g in graphs:
        for s in range(4):
            g.AddSubmap((0, s), submaps[s], (0.0, 0.0, 0.0))
        g.AddSubmap((1, 0), submaps[0], (0.0, 0.0, 0.0))
        for i in range(40):
            traj, idx = (0, i) if i < 20 else (1, i - 20)
            pose = tuple(float(v) for v in world.node_poses[i])
            ins = [(0, idx // 5)] if traj == 0 else [(1, 0)]
            g.AddNode((traj, idx), float(i), pose, world.cloud(i), ins,
                      traj == 0 and idx % 5 == 4)
    got = []
    builder.WhenDone(got.append)
    got = got[0]
    searched = [c for c in rec.log if c[0] != "E"]
    assert builder.constraints_searched == sum(1 for c in searched if c[0] == "L")
    assert builder.global_constraints_searched == sum(1 for c in searched if c[0] == "G")
    assert builder.global_constraints_searched > 0 and builder.constraints_searched > 0
    found_global = [c for c in got if c.node_id[0] == 1]
    assert len(got) > 0
    graphs[0].HandleConstraints(got)
    if found_global:
        assert graphs[0].connectivity.TransitivelyConnected(0, 1)
