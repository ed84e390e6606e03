#!/bin/bash
# Round-3 session o: warm-up admission spread over waves (GRM_OPT_WARMUP_SPREAD) and the shared child queue (GRM_OPT_WARMUP_SHARE)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for v in "" "20=1" "19=4" "20=1,19=4"; do
  t="${v:-default}"; t="${t//=/_}"
  GRM_BENCH_OPTS="$v" timeout -k 10 200 python -u tools/pass_phases.py 4 1e6 > gpurun_out/r3o_adm_$t.log 2>&1 || { tail -5 gpurun_out/r3o_adm_$t.log; exit 1; }
  echo "== $t"; cat gpurun_out/r3o_adm_$t.log
done
rm -f gpurun_out/*.dump
