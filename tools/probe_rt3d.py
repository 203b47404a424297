"""C4 RTCSM3D timing per scoring-loop unroll (CSM_RT3D_UNROLL) and kernel
version (CSM_RT3D_V1): prints kernel ms and the best score for each setting."""
import importlib.util
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bench)
csm = bench.load_pkg()
ctx = csm.Context(0)
args = SimpleNamespace(seed=20250127, no_cpu=True)
for setting in sys.argv[1:]:
    for kv in setting.split(","):
        k, v = kv.split("=")
        if v == "-":
            os.environ.pop(k, None)
        else:
            os.environ[k] = v
    r = bench.rt3d_bench(csm, ctx, args)
    print(setting, "kernel_ms %.1f" % r["kernel_ms"], "score", r["score"], flush=True)
