# Round 5, final HEAD: the default bench.py run under
# rocprofv3 --kernel-trace --stats; the traced C3 chunk launches of
# fast2d_search_v4 against the bench's HIP-event kernel_ms_avg of the same run.
set -u
O=gpurun_out/r5bf
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $O
date +%T
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 780 rocprofv3 --kernel-trace --stats -d $R/$O/trace -o bench \
  --output-format csv -- python3 $R/bench.py > $R/$O/bench_full.json 2> $R/$O/bench_full.err) \
  || { tail -30 $O/bench_full.err; exit 1; }
date +%T
# The timed C3 chunk launches: dispatches of the search over 300 ms, less the
# 2 warm-up chunks and the last 4 (the C2 and C2-strict launches).
python3 - <<'PY'
import csv, json
O = "gpurun_out/r5bf"
rows = list(csv.DictReader(open(f"{O}/trace/bench_kernel_trace.csv")))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
c3 = [(r["e"] - r["s"]) / 1e6 for r in rows
      if "fast2d_search_v4<true, true, false>" in r["Kernel_Name"] and (r["e"] - r["s"]) > 300e6]
timed = c3[2:-4]
line = json.loads([l for l in open(f"{O}/bench_full.json") if l.startswith("{")][-1])
out = {"source": "rocprofv3 --kernel-trace --stats of the default bench.py run at the final round-5 HEAD "
                 "(tools/sessions/r5bf_session.sh); per-dispatch durations from its kernel trace",
       "c3_timed_chunk_launches": len(timed),
       "c3_chunk_launch_ms_avg_trace": sum(timed) / len(timed),
       "c3_chunk_launch_ms_avg_bench_events": line["roofline"]["kernel_ms_avg"],
       "c3_note": "the first 2 dispatches over 300 ms are the warm-up chunks; the last 4 are C2 and "
                  "C2-strict launches (25,000-pair batches)",
       "bench_value_pairs_per_s": line["value"], "c5_pairs_per_s": line["fast3d"]["value"]}
json.dump(out, open(f"{O}/trace_summary.json", "w"), indent=1)
print(json.dumps(out))
PY
