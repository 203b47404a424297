"""bench.py's host logic that needs no GPU (CPU only):

* the rank contract: under a launcher, WORLD_SIZE must equal --gpus, checked
  before anything touches the GPU (VERDICT r5 Next 1);
* the reference lookup count: the oracle's per-pair work
  counters that work_ratio reports next to the GPU's, and the line fields
  work_ratio builds from them (VERDICT r5 Next 4).
"""
import argparse
import math
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, load_package, ensure_built

sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_world_size_must_equal_gpus():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr
    assert not r.stdout.strip()  # no line printed


def test_single_gpu_needs_no_launcher(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert bench.launch_ranks(argparse.Namespace(gpus=1)) is None


def test_oracle_work_counters_and_work_ratio_fields():
    """The oracle's counters per pair (oracle_fast2d_match_pairs_stats, the
    run bench.py's parity sample and CPU baseline make) are the reference's
    own work: every candidate scored costs one GetValue per point
    (fast_correlative_scan_matcher_2d.cc:319-330), so lookups = candidates x
    points, and the lowest-resolution candidates are the top level's."""
    ensure_built()
    csm = load_package()
    world = csm.SyntheticWorld2D(num_nodes=3, num_submaps=2, submap_cells=120, decimate_to=150,
                                 seed=99)
    subs = np.array([0, 1, 1, 0, 1], np.int64)
    nodes = np.array([0, 1, 2, 2, 0], np.int64)
    args = argparse.Namespace(min_score=0.55, cpu_threads=2, cpu_pairs=len(subs), cpu_seconds=1.0)
    _, ores = bench.cpu_pairs_2d(world, subs, nodes, args, "test pairs")
    assert ores["done"].all()
    st = ores["stats"]
    npts = np.diff(world.offsets)[nodes]
    assert np.array_equal(st[:, 0], st[:, 3:16].sum(1) * npts)
    assert np.all(st[:, 2] == st[:, 3 + 6])  # depth 7: levels 0..6, the lowest resolution is 6
    wr = bench.work_ratio_fields(st, np.arange(12) * 10.0, 500.0, 4000.0, [1.0, 2.0])
    assert wr["pairs"] == len(subs)
    assert math.isclose(wr["oracle"]["lookups_per_pair"], st[:, 0].mean())
    assert math.isclose(wr["oracle"]["candidates_per_pair"], st[:, 3:16].sum(1).mean())
    assert math.isclose(wr["candidates_ratio"], 100.0 / wr["oracle"]["candidates_per_pair"])
    assert math.isclose(wr["lookups_ratio"], 800.0 / wr["oracle"]["lookups_per_pair"])
    assert wr["leaf_candidates_ratio"] == (0.0 if st[:, 3].any() else None)
    assert wr["gpu_queue_candidates_per_pair"] == 3.0


@pytest.mark.parametrize("bad", [{"gpus": 3}])
def test_launch_ranks_rejects_mismatch(monkeypatch, bad):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit) as e:
        bench.launch_ranks(argparse.Namespace(**bad))
    assert e.value.code == 2


def test_gather_sample_merges_every_ranks_results():
    """At N > 1 each rank keeps the sampled pairs of the chunks it claimed;
    rank 0 receives every rank's (index, result) rows through csm_comm_gather
    and fills its table (bench.gather_sample). A fake communicator stands in
    for the 2-rank gather."""
    ensure_built()
    csm = load_package()
    k = 10

    def table(have):
        t = {"gpu": np.zeros(k, csm.RESULT_DTYPE), "have": np.zeros(k, bool)}
        for i in have:
            t["gpu"][i]["status"] = 0
            t["gpu"][i]["score"] = 0.5 + i / 100
            t["have"][i] = True
        return t

    r0, r1 = table([0, 3, 4]), table([1, 2, 7, 9])

    class FakeComm:
        def __init__(self, blobs):
            self.blobs = blobs

        def gather(self, blob):
            return None if self.blobs is None else [blob] + self.blobs

    row = np.dtype([("i", "<i8"), ("r", csm.RESULT_DTYPE)])
    have1 = np.nonzero(r1["have"])[0]
    other = np.zeros(len(have1), row)
    other["i"], other["r"] = have1, r1["gpu"][have1]
    bench.gather_sample(r0, FakeComm([other.tobytes()]), csm)
    assert r0["have"].tolist() == [i in (0, 1, 2, 3, 4, 7, 9) for i in range(k)]
    for i in (1, 2, 7, 9):
        assert r0["gpu"][i]["score"] == np.float32(0.5 + i / 100)
    bench.gather_sample(r1, FakeComm(None), csm)  # a non-root rank: its table is untouched
    assert r1["have"].sum() == 4
