"""Every committed profile summary is rebuilt from the committed per-dispatch
reductions alone (tools/profiles.py, manifests under profiles/<round>/) and
must equal the committed file; and the summaries bench.py reads name their
committed inputs, not gpurun_out/ scratch (VERDICT r5 Next 6). CPU only."""
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import profiles  # noqa: E402

MANIFESTS = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "manifest.json")))


@pytest.mark.parametrize("manifest", MANIFESTS, ids=[os.path.basename(os.path.dirname(m)) for m in MANIFESTS])
def test_summary_rebuilds_from_committed_inputs(manifest):
    assert profiles.check(manifest) == []


def test_bench_summaries_come_from_manifests():
    files = list(bench.TRAFFIC_FILES.values()) + [bench.GATHER_FILE, bench.TRAFFIC3D_FILE]
    built = set()
    for m in MANIFESTS:
        base = os.path.relpath(os.path.dirname(m), ROOT)
        built |= {os.path.join(base, name) for name in json.load(open(m))["outputs"]}
    for rel in files:
        assert rel in built, f"{rel} has no manifest"
        src = json.load(open(os.path.join(ROOT, rel)))["source"]
        assert "gpurun_out" not in src, (rel, src)


def test_cited_profile_paths_exist():
    """Every profiles/ path the documents cite is committed (ADVICE r5:
    evidence trails must not dangle)."""
    import re
    missing = []
    for doc in ("DESIGN.md", "EXPERIMENTS.md", "INTEGRATION.md", "README.md"):
        path = os.path.join(ROOT, doc)
        if not os.path.exists(path):
            continue
        for cite in set(re.findall(r"profiles/r[0-9a-z]+(?:/[A-Za-z0-9_./-]*[A-Za-z0-9_])?", open(path).read())):
            if not os.path.exists(os.path.join(ROOT, cite)):
                missing.append((doc, cite))
    assert not missing, missing
