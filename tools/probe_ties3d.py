"""Times ConstraintBuilder3DTest.FindsConstraints' inputs (an all-unknown
submap, a one-point node, min scores 0: every leaf ties) on the GPU path
(search, collect pass, ordered walk) and on the oracle, per call, with the
host-phase print of CSM_PROFILE3D if set. Run on the GPU box."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import __graft_entry__ as ge
    csm = ge._load_package()
    import oracle_lib
    from test_ties_walk import _matchers3d
    oracle = oracle_lib.Oracle()
    f = csm.FastCorrelativeScanMatcherOptions3D(min_rotational_score=0.0, min_low_resolution_score=0.0)
    hist = np.zeros(3, np.float32)
    og_h, og_l = oracle.hybrid_grid(0.1), oracle.hybrid_grid(0.1)
    om, gm, keep = _matchers3d(csm, oracle, og_h, og_l, hist, f)
    pt = np.array([[0.1, 0.2, 0.3]], np.float32)
    node = csm.NodeData3D(pt, pt, hist)
    ident = ((0.0, 0.0, 0.0), (1.0, 0.0, 0.0, 0.0))
    ctx = csm.default_context(0)
    for name, g, o in (("Match", lambda: gm.Match(ident, ident, node, 0.0), lambda: om.match(ident, ident, node, 0.0)),
                       ("MatchFullSubmap", lambda: gm.MatchFullSubmap((1, 0, 0, 0), (1, 0, 0, 0), node, 0.0),
                        lambda: om.match_full_submap((1, 0, 0, 0), (1, 0, 0, 0), node, 0.0))):
        ctx.reset_timing()
        ctx.enable_timing(True)
        a = time.perf_counter()
        r = g()
        b = time.perf_counter()
        o()
        c = time.perf_counter()
        t = ctx.timing()
        print(f"{name}: gpu {1e3 * (b - a):.1f} ms (tie {r.tie}, fast3d kernel {t.fast3d_kernel_ms:.1f} ms), "
              f"oracle {1e3 * (c - b):.1f} ms", flush=True)


if __name__ == "__main__":
    main()
