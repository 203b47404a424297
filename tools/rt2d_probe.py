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
    res = bench.rt2d_bench(csm, ctx, args)
    res["ctypes_call_us"] = ctypes_overhead_us(csm, ctx)
    print(json.dumps(res), flush=True)


def ctypes_overhead_us(csm, ctx):
    """Median cost of the ctypes call alone: csm_rt2d_match with the same
    argument list and a null context (rejected before any work)."""
    import ctypes as C
    import time
    import numpy as np
    lib = ctx._lib
    lim = csm.MapLimits(0.05, 10.0, 10.0, 200, 200)
    opts = csm.RtOptions(0.2, 0.17, 0.1, 0.1)
    cells = np.zeros((200, 200), np.uint16)
    pts = np.zeros((1080, 3), np.float32)
    init = csm.Pose2D(0.0, 0.0, 0.0)
    score, pose = C.c_double(0.0), csm.Pose2D()
    times = []
    for _ in range(2000):
        a = time.perf_counter()
        lib.csm_rt2d_match(None, C.byref(opts), C.byref(lim),
                           cells.ctypes.data_as(C.POINTER(C.c_uint16)), 0.1, 0.9, C.byref(init),
                           pts.ctypes.data_as(C.POINTER(C.c_float)), len(pts), C.byref(score),
                           C.byref(pose))
        times.append(time.perf_counter() - a)
    return 1e6 * float(np.median(times))


if __name__ == "__main__":
    main()
