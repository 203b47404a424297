"""C5 leg alone (bench.fast3d_bench, no CPU baseline), for host/kernel
phase profiling: CSM_PROFILE3D=1 python tools/probe_c5.py [bench C5 flags]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0], "--no-cpu"] + sys.argv[1:]
    args = bench.parse()
    csm = bench.load_pkg()
    ctx = csm.Context(0)
    out = bench.fast3d_bench(csm, ctx, args)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
