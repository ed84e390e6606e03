#!/bin/bash
# warm-up cost: pass wall time with the default warm-up, none, and looser slack / larger first batch
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
run() { # name, env...
  local n=$1; shift
  env "$@" DEV_EMIT=1 DIAG_REPS=3 SEED=126 timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/r3f_$n.log 2>&1 || { tail -5 gpurun_out/r3f_$n.log; exit 1; }
  echo "$n: $(grep -oE 'wall [0-9.]+s kernel [0-9.]+ms' gpurun_out/r3f_$n.log | tr '\n' ' ') scatt $(grep -oE 'scatt [0-9]+ ' gpurun_out/r3f_$n.log | tr '\n' ' ')"
}
for r in 1 2; do
run default_$r X=1
run nowarm_$r WARMUP=0
run slack3_$r SLACK=3
run slack2_$r SLACK=2
run b0_256_$r WARMUP_BATCH=256
done
rm -f gpurun_out/*.dump
