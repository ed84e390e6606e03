#!/bin/bash
# scheduler strategies (cur = iterative-ilp, dflt, maxilp, maxmem), then early-worker hand-over threshold
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
VARIANTS="cur dflt maxilp maxmem" ROUNDS=2 STEPS=6 TAG=r3o bash tools/ab_bench.sh || exit 1
for st in 2000 5000 1000; do
  GRM_BENCH_OPTS="15=$st" VARIANTS="cur" ROUNDS=1 STEPS=10 TAG=r3o_early$st bash tools/ab_bench.sh || exit 1
done
rm -f gpurun_out/*.dump
