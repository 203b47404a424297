"""Pre-flight of bench.py's N > 1 path on the one-GPU box (VERDICT r4 Next 5).

The driver's scaling run launches bench.py with torch.distributed.run, one
rank per GPU, and csm_comm over RCCL. Here two ranks share the one GPU: the
process group is gloo (torch's RCCL cannot put two ranks on one device) and
csm_comm takes its RCCL branch (--comm-backend rccl) through CSM_RCCL_LIB =
tests/comm_standin/librccl_standin.so, a test-only library with RCCL's entry
points over TCP. What runs is bench.py's own multi-rank code: the store-based
unique-id exchange and the all-ranks agreement (make_comm_checked), the C3
chunk claims through csm_comm_fetch_add, the record gathers over
csm_comm_gather (C3 and C5), the max-over-ranks timing and the strong-scaling
accounting. The gathered records must equal a single-rank run's, in
submission order (ConstraintBuilder2D::WhenDone, constraint_builder_2d.cc:
279-300).

The two ranks are started the way a bare `bench.py --gpus 2` starts them
(no launcher: bench.py runs torch.distributed.run itself), so a scaling
command can never silently measure one rank; the line must report the
communicator's rank count (comm_ranks) and a parity sample of the timed
run, gathered from whichever rank claimed each sampled pair and compared
with the oracle on rank 0 (VERDICT r5 Next 1).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

STANDIN = os.path.join(ROOT, "tests", "comm_standin", "librccl_standin.so")
SMALL = ["--workload", "c3", "--c3-nodes", "48", "--c3-submaps", "12", "--c3-slice", "4",
         "--steps", "3", "--warmup", "1", "--no-rt", "--no-cpu", "--nodes3d", "40",
         "--submaps3d", "6", "--steps3d", "1", "--parity-pairs", "24"]


def _json_line(out):
    return json.loads([line for line in out.splitlines() if line.startswith("{")][-1])


def test_two_ranks_rccl_branch_equal_single_rank(tmp_path):
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONUNBUFFERED="1")
    one = tmp_path / "one.npz"
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *SMALL,
                         "--dump-records", str(one)], capture_output=True, text=True, timeout=240,
                        cwd=ROOT, env=env)
    assert r1.returncode == 0, r1.stderr[-3000:]
    j1 = _json_line(r1.stdout)
    two = tmp_path / "two.npz"
    env2 = dict(env, CSM_RCCL_LIB=STANDIN)
    for var in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env2.pop(var, None)
    r2 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *SMALL,
                         "--dist-backend", "gloo", "--comm-backend", "rccl",
                         "--dump-records", str(two)], capture_output=True, text=True,
                        timeout=300, cwd=ROOT, env=env2)
    assert r2.returncode == 0, r2.stderr[-3000:]
    assert "starting 2 ranks" in r2.stderr
    j2 = _json_line(r2.stdout)
    assert j2["config"]["gather"] == "csm_comm_rccl" and j2["n_gpus"] == 2
    assert j1["comm_ranks"] == 1 and j2["comm_ranks"] == 2
    for j in (j1, j2):  # the timed run's sampled pairs, against the oracle
        p = j["parity_sample"]
        assert p["pairs"] == p["compared"] == 24, p
        assert p["mismatched_decision"] == p["mismatched_score"] == p["mismatched_pose"] == 0, p
        assert p["gpu_errors"] == 0
        assert j["work_ratio"]["pairs"] == 24 and j["work_ratio"]["oracle"]["lookups_per_pair"] > 0
    assert j2["parity_sample"]["ranks"] == 2
    p3 = j2["fast3d"]["parity_sample"]  # each rank's C5 share against the oracle, summed
    assert p3["ranks"] == 2 and p3["pairs"] == p3["compared"] == 24, p3
    assert p3["mismatched_decision"] == p3["mismatched_score"] == p3["mismatched_pose"] == 0, p3
    a, b = np.load(one), np.load(two)
    for key in ("c3", "c5"):
        assert a[key].shape == b[key].shape and len(a[key]) > 0, key
        assert np.array_equal(a[key], b[key]), key          # same records, submission order
        assert np.all(np.diff(b[key][:, 0]) > 0), key
    # Strong-scaling accounting: the same fixed queue, every chunk claimed
    # once over the ranks, value = all pairs / the slowest rank's time.
    for j in (j1, j2):
        assert j["scaling"] == "strong"
        assert j["config"]["queue_pairs_timed"] == 3 * 4 * 48
        assert j["chunks_claimed"] == j["chunks"]
        assert abs(j["value"] - j["config"]["queue_pairs_timed"] / (j["ms_per_step"] * 1e-3 * 3)) \
            < 1e-6 * j["value"]
        assert j["accepted_constraints"] == len(a["c3"])
        assert j["fast3d"]["pairs_per_step"] == 40 * 6
        assert j["fast3d"]["accepted_per_step"] == len(a["c5"])
    assert j2["chunks_max_rank"] < j2["chunks"]  # both ranks claimed chunks
