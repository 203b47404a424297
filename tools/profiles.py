"""The profile pipeline behind every roofline number bench.py reports.

rocprofv3's raw output (per-counter rows of every dispatch, whole kernel
traces) stays in gpurun_out/ scratch. What is committed under
profiles/<round>/ is its reduction: per-dispatch CSVs of the kernels that
matter (a few KB), the CSM_KPROF line counts, the bench lines of the same
runs, and a manifest.json naming, for every summary JSON bench.py reads
(traffic_c3.json, gather_c3.json, traffic_c5.json, trace_summary.json ...),
the committed inputs and parameters it is built from. `build` writes the
summaries from those inputs alone; `check` rebuilds them in memory and
compares them with the committed files (tests/test_profiles.py runs it on
every manifest, CPU only).

    python tools/profiles.py reduce-pmc RAW_DIR OUT_CSV KERNEL [KERNEL...]
    python tools/profiles.py reduce-trace RAW_TRACE_CSV OUT_CSV KERNEL [KERNEL...]
    python tools/profiles.py build  profiles/<round>/manifest.json
    python tools/profiles.py check  profiles/<round>/manifest.json

KERNEL is a key of KERNELS (the search kernels' own instantiations: the
2D tie-collect launches are a different instantiation and are left out).
Counter units and corrections follow MI355X_MICROARCH.md's rocprofv3
section: FETCH_SIZE is in KB, x 1024 x 2 for gfx950's HBM bytes.
"""
import collections
import csv
import glob
import json
import math
import os
import re
import sys

KERNELS = {
    "fast2d_search": "fast2d_search_v4<true, true, false>",
    "fast3d_search": "fast3d_search<",
}
NUM_CUS = 256
CLOCK_HZ = 2.4e9  # MI355X peak engine clock (MI355X_MICROARCH.md)
FETCH_CORRECTION = 2.0
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rel(base, name):
    """A committed input as the repo-relative path the summaries cite."""
    return os.path.relpath(os.path.abspath(os.path.join(base, name)), REPO)


def _key(name, keys):
    for k in keys:
        if KERNELS[k] in name:
            return k
    return None


# ---------------------------------------------------------------- reduce --

def reduce_pmc(raw_dir, out_csv, keys):
    """Every counter_collection.csv under raw_dir (one subdirectory per pass
    when several) -> rows (pass, dispatch, kernel, counter, value), the
    counter summed over its instances, for the kernels in `keys`."""
    acc = collections.OrderedDict()
    files = sorted(glob.glob(os.path.join(raw_dir, "**", "*counter_collection.csv"), recursive=True))
    if not files:
        sys.exit(f"no counter_collection.csv under {raw_dir}")
    for f in files:
        rel = os.path.relpath(f, raw_dir)
        pass_id = rel.split(os.sep)[0] if os.sep in rel else "."
        for r in csv.DictReader(open(f)):
            k = _key(r.get("Kernel_Name", ""), keys)
            if k is None:
                continue
            key = (pass_id, int(r.get("Dispatch_Id", 0)), k, r["Counter_Name"])
            acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
    with open(out_csv, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["pass", "dispatch", "kernel", "counter", "value"])
        for (p, d, k, c), v in acc.items():
            w.writerow([p, d, k, c, repr(v)])
    return len(acc)


def reduce_trace(trace_csv, out_csv, keys):
    """A kernel_trace.csv -> rows (order, dispatch, kernel, start_ns, duration_ns)
    of the kernels in `keys`, in start order, start relative to the first."""
    rows = []
    for r in csv.DictReader(open(trace_csv)):
        k = _key(r.get("Kernel_Name", ""), keys)
        if k is None:
            continue
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        rows.append((s, int(r["Dispatch_Id"]), k, e - s))
    rows.sort()
    t0 = rows[0][0] if rows else 0
    with open(out_csv, "w", newline="") as fo:
        w = csv.writer(fo)
        w.writerow(["order", "dispatch", "kernel", "start_ns", "duration_ns"])
        for i, (s, d, k, dur) in enumerate(rows):
            w.writerow([i, d, k, s - t0, dur])
    return len(rows)


# ----------------------------------------------------------------- read --

def read_pmc(path, kernel):
    """{(pass, dispatch): {counter: value}} of one kernel."""
    per = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        if r["kernel"] == kernel:
            per[(r["pass"], int(r["dispatch"]))][r["counter"]] = float(r["value"])
    if not per:
        raise ValueError(f"no {kernel} rows in {path}")
    return per


def pmc_average(per):
    """Each counter averaged over the dispatches of the pass(es) that
    collected it."""
    sums, counts = collections.defaultdict(float), collections.defaultdict(int)
    for cs in per.values():
        for c, v in cs.items():
            sums[c] += v
            counts[c] += 1
    return {c: sums[c] / counts[c] for c in sums}, max(counts.values())


def read_trace(path, kernel):
    return [(int(r["order"]), int(r["dispatch"]), int(r["duration_ns"]))
            for r in csv.DictReader(open(path)) if r["kernel"] == kernel]


def kprof_lines(path):
    """Per launch {child level: (line touches, gather instructions)} from the
    stderr of a CSM_KPROF build run with CSM_PROFILE2D=1."""
    launches = []
    for line in open(path):
        if "fast2d lines per gather by child level:" not in line:
            continue
        levels = {}
        for lv, lpi, instr in re.findall(r"L(\d+) ([\d.]+) \(([\deE.+-]+) instr\)", line):
            levels[int(lv)] = (float(lpi) * float(instr), float(instr))
        launches.append(levels)
    if not launches:
        raise ValueError(f"no KPROF line counts in {path}")
    return launches


def bench_line(path):
    return json.loads([ln for ln in open(path) if ln.startswith("{")][-1])


# ---------------------------------------------------------------- build --

def build_traffic2d(base, spec):
    """traffic_c3.json / traffic_c2.json: HBM-side bytes per search launch
    from a FETCH_SIZE pass (KB x 1024 x 2)."""
    avg, n = pmc_average(read_pmc(os.path.join(base, spec["pmc"]), "fast2d_search"))
    kb = avg["FETCH_SIZE"]
    t = {"kernel": "fast2d_search_v4 (v5: FIFO order, hex planes, scan clusters)",
         "commit_kernel": spec["tag"], "workload": spec["workload"], "nodes": spec["nodes"]}
    for k in ("submaps_per_rank", "chunk", "submaps"):
        if k in spec:
            t[k] = spec[k]
    t.update({"min_score": spec.get("min_score", 0.55), "search_depth": spec.get("search_depth", 0),
              "launches": n, "fetch_size_kb_per_launch": kb,
              "gfx950_fetch_correction": FETCH_CORRECTION,
              "traffic_bytes_per_launch": kb * 1024 * FETCH_CORRECTION,
              "launch_ms": spec["launch_ms"],
              "source": f"rocprofv3 --pmc FETCH_SIZE (own pass, no tracing), per dispatch: "
                        f"{_rel(base, spec['pmc'])}"})
    return t


def build_gather(base, spec):
    """gather_c3.json: the texture-path ceiling of the C3 search kernel, from
    the KPROF line counts (distinct 128-byte lines per gather, by child level)
    and a TD_TD_BUSY / TA_BUFFER_READ_WAVEFRONTS pass of the same slice."""
    floor = spec.get("floor_td_cycles_per_line", 2.3)
    launches = kprof_lines(os.path.join(base, spec["kprof"]))
    lines = sum(sum(v[0] for v in lv.values()) for lv in launches) / len(launches)
    instr = sum(sum(v[1] for v in lv.values()) for lv in launches) / len(launches)
    by_level = {}
    for lv in sorted({k for x in launches for k in x}):
        t_ = sum(x.get(lv, (0, 0))[0] for x in launches) / len(launches)
        n_ = sum(x.get(lv, (0, 0))[1] for x in launches) / len(launches)
        by_level[f"L{lv}"] = {"line_touches": t_, "instructions": n_,
                              "lines_per_instruction": t_ / n_ if n_ else 0.0, "share": t_ / lines}
    avg, n_pmc = pmc_average(read_pmc(os.path.join(base, spec["pmc"]), "fast2d_search"))
    td = avg.get("TD_TD_BUSY_sum")
    ta_wf = avg.get("TA_BUFFER_READ_WAVEFRONTS_sum")
    floor_ms = lines * floor / (NUM_CUS * CLOCK_HZ) * 1e3
    out = {"kernel": "fast2d_search_v4", "commit_kernel": spec["tag"], "workload": spec["workload"],
           "kprof_launches": len(launches), "pmc_launches": n_pmc,
           "line_touches_per_launch": lines, "gather_instructions_per_launch": instr,
           "by_child_level": by_level, "floor_td_cycles_per_line": floor,
           "floor_source": "profiles/r4g/gather_pattern.txt (adjacent lanes sharing a line, L2-resident)",
           "num_cus": NUM_CUS, "clock_hz": CLOCK_HZ, "floor_ms_per_launch": floor_ms,
           "td_busy_cycles_per_launch": td, "ta_buffer_read_wavefronts_per_launch": ta_wf,
           "td_cycles_per_line_measured": td / lines if td else None,
           "source": f"KPROF {_rel(base, spec['kprof'])}; PMC {_rel(base, spec['pmc'])}"}
    for c in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_REQ_sum", "TA_TA_BUSY_sum", "FETCH_SIZE"):
        if c in avg:
            out.setdefault("counters_per_launch", {})[c] = avg[c]
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / (avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    return out


def build_traffic3d(base, spec):
    """traffic_c5.json: fast3d_search's counters per dispatch (each counter
    over its own pass), HBM bytes = FETCH_SIZE x 1024 x 2, and the traffic per
    algorithmic byte of the probe run (so bench.py can scale it to the C5
    step's launches)."""
    avg, _ = pmc_average(read_pmc(os.path.join(base, spec["pmc"]), "fast3d_search"))
    kb = avg.get("FETCH_SIZE")
    t = {"kernel": "fast3d_search (octet child levels, root cell lists)", "commit_kernel": spec["tag"],
         "workload": spec["workload"], "counters_per_dispatch": avg,
         "gfx950_fetch_correction": FETCH_CORRECTION,
         "traffic_bytes_per_launch": kb * 1024 * FETCH_CORRECTION if kb else None,
         "source": f"rocprofv3 --pmc passes (own passes, no tracing), per dispatch: "
                   f"{_rel(base, spec['pmc'])}"}
    if spec.get("probe") and kb:
        probe = bench_line(os.path.join(base, spec["probe"]))
        launches_per_step = probe["roofline"]["launches"] / max(probe["steps"], 1)
        lookups_per_launch = probe["lookups_per_step"] / launches_per_step
        t["algorithmic_bytes_per_launch"] = lookups_per_launch
        t["traffic_bytes_per_algorithmic_byte"] = t["traffic_bytes_per_launch"] / lookups_per_launch
    return t


def build_trace_summary(base, spec):
    """trace_summary.json: the timed C3 chunk launches' average duration in
    the kernel trace of a default bench.py run, next to the run's own
    HIP-event figure. The timed launches are the search dispatches longer
    than min_ms, less the first `skip_first` (warm-up chunks) and the last
    `skip_last` (the C2 legs' launches)."""
    d = [dur / 1e6 for _, _, dur in read_trace(os.path.join(base, spec["trace"]), "fast2d_search")
         if dur / 1e6 > spec.get("min_ms", 300.0)]
    timed = d[spec.get("skip_first", 2):len(d) - spec.get("skip_last", 4)]
    line = bench_line(os.path.join(base, spec["bench"]))
    out = {"source": f"rocprofv3 --kernel-trace --stats of the default bench.py run, per-dispatch "
                     f"durations: {_rel(base, spec['trace'])}",
           "c3_timed_chunk_launches": len(timed),
           "c3_chunk_launch_ms_avg_trace": sum(timed) / len(timed),
           "c3_chunk_launch_ms_avg_bench_events": line["roofline"]["kernel_ms_avg"],
           "c3_note": spec.get("note", ""),
           "bench_value_pairs_per_s": line["value"], "c5_pairs_per_s": line["fast3d"]["value"]}
    return out


BUILDERS = {"traffic2d": build_traffic2d, "gather": build_gather, "traffic3d": build_traffic3d,
            "trace_summary": build_trace_summary}


def build(manifest):
    base = os.path.dirname(manifest)
    spec = json.load(open(manifest))
    return {name: BUILDERS[s["kind"]](base, s) for name, s in spec["outputs"].items()}


def _close(a, b, path=""):
    if isinstance(a, dict) and isinstance(b, dict):
        if set(a) != set(b):
            return f"{path}: keys {sorted(set(a) ^ set(b))}"
        for k in a:
            e = _close(a[k], b[k], f"{path}.{k}")
            if e:
                return e
        return None
    if isinstance(a, (int, float)) and isinstance(b, (int, float)) and not isinstance(a, bool):
        return None if math.isclose(a, b, rel_tol=1e-9, abs_tol=1e-12) else f"{path}: {a} != {b}"
    return None if a == b else f"{path}: {a!r} != {b!r}"


def check(manifest):
    """Rebuilds every output of the manifest and compares it with the
    committed file. Returns a list of differences (empty: all equal)."""
    base = os.path.dirname(manifest)
    errs = []
    for name, got in build(manifest).items():
        want = json.load(open(os.path.join(base, name)))
        e = _close(got, want, name)
        if e:
            errs.append(e)
    return errs


def main():
    cmd = sys.argv[1]
    if cmd == "reduce-pmc":
        print(reduce_pmc(sys.argv[2], sys.argv[3], sys.argv[4:]), "rows")
    elif cmd == "reduce-trace":
        print(reduce_trace(sys.argv[2], sys.argv[3], sys.argv[4:]), "rows")
    elif cmd == "build":
        base = os.path.dirname(sys.argv[2])
        for name, t in build(sys.argv[2]).items():
            json.dump(t, open(os.path.join(base, name), "w"), indent=1)
            print("wrote", os.path.join(base, name))
    elif cmd == "check":
        errs = check(sys.argv[2])
        print("\n".join(errs) if errs else "ok")
        sys.exit(1 if errs else 0)
    else:
        sys.exit(__doc__)


if __name__ == "__main__":
    main()
