"""Reads a rocprofv3 kernel trace of a default bench.py run and reports
(1) the C3 chunk launches of fast2d_search_v4 (dispatches over --c3-min-ms)
against the bench line's kernel_ms_avg, and (2) the timeline of each C5 step:
wall from its first to its last kernel, the union of busy time, the time
fast3d_search kernels run, the builds' kernel time, and the idle gaps.

    python tools/trace_c5.py TRACE.csv [BENCH.json]
"""
import csv
import json
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    out = {}
    c3 = [(r["e"] - r["s"]) / 1e6 for r in rows
          if "fast2d_search_v4<true, true, false>" in r["Kernel_Name"] and (r["e"] - r["s"]) > 300e6]
    out["c3_chunk_launches"] = len(c3)
    out["c3_chunk_launch_ms_avg"] = sum(c3) / len(c3) if c3 else None
    if len(sys.argv) > 2:
        line = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
        out["bench_kernel_ms_avg"] = line["roofline"]["kernel_ms_avg"]
    # C5 steps: clusters of fast3d_search dispatches separated by > 50 ms of no fast3d_search.
    f3 = [r for r in rows if "fast3d_search" in r["Kernel_Name"]]
    steps, cur = [], []
    for r in f3:
        if cur and r["s"] - cur[-1]["e"] > 50e6:
            steps.append(cur)
            cur = []
        cur.append(r)
    if cur:
        steps.append(cur)
    rep = []
    for st in steps:
        if len(st) < 8:  # the single-call and drop-in legs
            continue
        t0, t1 = st[0]["s"], st[-1]["e"]
        # the step's builds start before its first search: include kernels from
        # 400 ms before the first search that are not fast2d/rt kernels
        win = [r for r in rows if t0 - 400e6 <= r["s"] <= t1 and "fast2d" not in r["Kernel_Name"]
               and "rt2d" not in r["Kernel_Name"] and "rt3d" not in r["Kernel_Name"]]
        start = min(r["s"] for r in win)
        kinds = defaultdict(float)
        for r in win:
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            kinds[name] += (r["e"] - r["s"]) / 1e6
        search = [(r["s"], r["e"]) for r in st]
        other = [(r["s"], r["e"]) for r in win if "fast3d_search" not in r["Kernel_Name"]]
        rep.append({"wall_ms": (t1 - start) / 1e6, "search_launches": len(st),
                    "search_kernel_ms_sum": sum(e - s for s, e in search) / 1e6,
                    "search_busy_ms": union(search) / 1e6,
                    "other_busy_ms": union(other) / 1e6,
                    "busy_ms": union(search + other) / 1e6,
                    "kernel_ms_by_name": {k: round(v, 2) for k, v in sorted(kinds.items(), key=lambda x: -x[1])[:10]}})
    out["c5_steps"] = rep
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
