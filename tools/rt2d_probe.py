"""C1 probe: the bench's rt2d leg alone (for kernel-trace profiling)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--seed", type=int, default=20250127)
    args = p.parse_args()
    csm = bench.load_pkg()
    ctx = csm.default_context(0)
    print(json.dumps(bench.rt2d_bench(csm, ctx, args)), flush=True)


if __name__ == "__main__":
    main()
