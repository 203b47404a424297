"""Writes profiles/<round>/gather_c3.json: the texture-path (TD) ceiling of
the C3 search kernel, which bench.py reports next to the HBM roofline.

Inputs, all from one 16-submap slice of the C3 queue (4 chunk launches):
  KPROF_ERR  stderr of a CSM_KPROF build run with CSM_PROFILE2D=1: per launch,
             the distinct 128-byte lines and gather instructions by child
             level ("fast2d lines per gather by child level: L0 a (b instr) ...")
  PMC_DIR    rocprofv3 --pmc TD_TD_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum pass
             of the default build (counters summed over the TD/TA instances)
The floor is FLOOR_CYCLES TD cycles per distinct line (the gather
microbenchmark's cost when lanes sharing a line are adjacent, L2-resident set:
profiles/r4g/gather_pattern.txt, 2.3), spread over every CU's TD at the
engine clock.

    python tools/gather_roofline.py KPROF_ERR PMC_DIR OUT_JSON KERNEL_TAG [FLOOR_CYCLES]
"""
import collections
import csv
import glob
import json
import re
import sys

NUM_CUS = 256
CLOCK_HZ = 2.4e9  # MI355X peak engine clock (MI355X_MICROARCH.md)


def kprof_lines(path):
    launches = []
    for line in open(path):
        if "fast2d lines per gather by child level:" not in line:
            continue
        levels = {}
        for lv, lpi, instr in re.findall(r"L(\d+) ([\d.]+) \(([\deE.+-]+) instr\)", line):
            levels[int(lv)] = (float(lpi) * float(instr), float(instr))
        launches.append(levels)
    if not launches:
        sys.exit(f"no KPROF line counts in {path}")
    return launches


def pmc(pmc_dir):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{pmc_dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if "fast2d_search_v4" in name and "true>" not in name.split(",")[2]:
                per[r.get("Dispatch_Id", "0")][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        sys.exit(f"no fast2d_search_v4 counters in {pmc_dir}")
    keys = set().union(*[set(v) for v in per.values()])
    return {k: sum(v[k] for v in per.values()) / len(per) for k in keys}, len(per)


def main():
    kerr, pdir, out, tag = sys.argv[1:5]
    floor = float(sys.argv[5]) if len(sys.argv) > 5 else 2.3
    launches = kprof_lines(kerr)
    lines = sum(sum(v[0] for v in lv.values()) for lv in launches) / len(launches)
    instr = sum(sum(v[1] for v in lv.values()) for lv in launches) / len(launches)
    by_level = {}
    for lv in sorted({k for x in launches for k in x}):
        t = sum(x.get(lv, (0, 0))[0] for x in launches) / len(launches)
        n = sum(x.get(lv, (0, 0))[1] for x in launches) / len(launches)
        by_level[f"L{lv}"] = {"line_touches": t, "instructions": n,
                              "lines_per_instruction": t / n if n else 0.0, "share": t / lines}
    counters, n_pmc = pmc(pdir)
    td = counters.get("TD_TD_BUSY_sum") or counters.get("TD_TD_BUSY")
    ta_wf = counters.get("TA_BUFFER_READ_WAVEFRONTS_sum") or counters.get("TA_BUFFER_READ_WAVEFRONTS")
    floor_ms = lines * floor / (NUM_CUS * CLOCK_HZ) * 1e3
    t = {"kernel": "fast2d_search_v4", "commit_kernel": tag,
         "workload": "C3 chunk launches (4-submap chunks x 2000 nodes), the first 16 submaps of the queue",
         "kprof_launches": len(launches), "pmc_launches": n_pmc,
         "line_touches_per_launch": lines, "gather_instructions_per_launch": instr,
         "by_child_level": by_level,
         "floor_td_cycles_per_line": floor,
         "floor_source": "profiles/r4g/gather_pattern.txt (adjacent lanes sharing a line, L2-resident)",
         "num_cus": NUM_CUS, "clock_hz": CLOCK_HZ, "floor_ms_per_launch": floor_ms,
         "td_busy_cycles_per_launch": td, "ta_buffer_read_wavefronts_per_launch": ta_wf,
         "td_cycles_per_line_measured": td / lines if td else None,
         "source": f"KPROF {kerr}; PMC {pdir}"}
    json.dump(t, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in t.items() if k != "by_child_level"}))


if __name__ == "__main__":
    main()
