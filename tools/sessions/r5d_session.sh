# Round 5: Option A's single calls coalesced into batches (csm_host.cc
# SingleMatch): tools/dropin_threads (C++ threads, C2 world) with coalescing
# off, and with 1-4 leaders and 0-400 us windows.
set -u
O=gpurun_out/r5d
mkdir -p $O
run() {  # label, then env assignments
  local label=$1; shift
  env "$@" timeout -k 10 240 ./tools/dropin_threads 2000 0.55 > $O/d.json 2> $O/d.err || { tail -5 $O/d.err; exit 1; }
  echo "$label $(tail -1 $O/d.json)" | tee -a $O/dropin_summary.txt
}
date +%T
run off CSM_SINGLE_COALESCE=0
for l in 1 2 3 4; do run leaders=$l CSM_COALESCE_LEADERS=$l; done
for w in 0 50 400; do run window=$w CSM_COALESCE_WINDOW_US=$w; done
timeout -k 10 240 ./tools/dropin_threads 0 0.55 --check > $O/check.json 2>&1 || { cat $O/check.json; exit 1; }
tail -1 $O/check.json | tee -a $O/dropin_summary.txt
date +%T
