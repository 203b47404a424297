"""The committed PMC summaries bench.py reports next to its own timings
(FETCH traffic, the C3 gather roofline, the C5 traffic) exist and belong to
the kernel versions bench.py names, so a kernel change cannot silently keep
reporting an older kernel's counters (CPU only)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _load(rel):
    path = os.path.join(ROOT, rel)
    assert os.path.isfile(path), rel
    with open(path) as f:
        return json.load(f)


def test_2d_traffic_files_match_kernel_tag():
    for workload, rel in bench.TRAFFIC_FILES.items():
        t = _load(rel)
        assert t["commit_kernel"] == bench.KERNEL_TAG, (workload, rel)
        assert t["traffic_bytes_per_launch"] > 0
        assert t["gfx950_fetch_correction"] == 2.0


def test_gather_roofline_file_matches_kernel_tag():
    t = _load(bench.GATHER_FILE)
    assert t["commit_kernel"] == bench.KERNEL_TAG
    assert 0 < t["floor_ms_per_launch"] and t["line_touches_per_launch"] > 0


def test_c5_traffic_file_matches_kernel_tag():
    t = _load(bench.TRAFFIC3D_FILE)
    assert t["commit_kernel"] == bench.KERNEL3D_TAG
    # Per-dispatch averages over the C5 step's search launches only: the
    # traffic is of the order of the issued bytes (the single-call leg's
    # small dispatches once pulled the average down 20x, profiles/r5ay).
    ratio = t["traffic_bytes_per_algorithmic_byte"]
    assert 0.1 < ratio < 10.0
