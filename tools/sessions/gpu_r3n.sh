#!/bin/bash
# Round-3 session n: the warm-up's admission log at photon_n = 1e6 (default, and larger first batches)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for v in "" "14=256" "14=1024"; do
  t="${v:-default}"; t="${t//=/_}"
  GRM_BENCH_OPTS="$v" timeout -k 10 200 python -u tools/pass_phases.py 4 1e6 > gpurun_out/r3n_adm_$t.log 2>&1 || { tail -5 gpurun_out/r3n_adm_$t.log; exit 1; }
  echo "== $t"; cat gpurun_out/r3n_adm_$t.log
done
rm -f gpurun_out/*.dump
