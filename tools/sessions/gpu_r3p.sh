#!/bin/bash
# Round-3 session p: warm-up spread sweep (GRM_OPT_WARMUP_SPREAD = 19) at photon_n = 1e6, 12 passes each:
# warm-up end time, dominant launch and recorded per pass
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for v in "" "19=1" "19=2" "19=4" "19=8" "19=16"; do
  t="${v:-default}"; t="${t//=/_}"
  GRM_BENCH_OPTS="$v" timeout -k 10 200 python -u tools/pass_phases.py 12 1e6 > gpurun_out/r3p_spread_$t.log 2>&1 || { tail -5 gpurun_out/r3p_spread_$t.log; exit 1; }
  echo "== $t"; grep -v admissions gpurun_out/r3p_spread_$t.log
done
rm -f gpurun_out/*.dump
