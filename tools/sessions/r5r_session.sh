# Round 5: Option A coalescing, second pass: per-batch host phases at 16
# threads (CSM_PROFILE2D "fast2d batch host" lines), and the grid share of
# a coalesced batch (CSM_COALESCE_SHARE) against leaders 2-3.
set -u
O=gpurun_out/r5r
mkdir -p $O
run() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 ./tools/dropin_threads 2000 0.55 > $O/d.json 2> $O/d.err || { tail -5 $O/d.err; exit 1; }
  echo "$label $(tail -1 $O/d.json)" | tee -a $O/dropin_summary.txt
}
date +%T
CSM_PROFILE2D=1 timeout -k 10 240 ./tools/dropin_threads 2000 0.55 > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
tail -1 $O/prof.json
grep "fast2d batch host" $O/prof.err | tail -400 > $O/prof_last400.txt
python3 - <<'PY'
import re
rows=[list(map(float,re.findall(r"\d+\.\d+|\d+", l.split(":",1)[1]))) for l in open("gpurun_out/r5r/prof_last400.txt")]
# prep, search, kernel, ties, tied, decode, pairs
import statistics as st
for i,name in enumerate(["prep","search+readback","kernel","ties","tied","decode","pairs"]):
    print(name, round(st.mean(r[i] for r in rows),3))
PY
for sh in 1 2 4; do run share=$sh CSM_COALESCE_SHARE=$sh; done
run leaders3-share1 CSM_COALESCE_LEADERS=3 CSM_COALESCE_SHARE=1
run leaders3 CSM_COALESCE_LEADERS=3
date +%T
