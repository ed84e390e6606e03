#!/bin/bash
# one laundered kernarg pointer for Params and Ctl (one) vs two (pc); lone-kernel laundering (onel)
# on the deterministic lone-latency probe
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for v in one onel pc; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" timeout -k 10 200 python tools/lone_bench.py 512 3 > gpurun_out/r3m_lone_$v.log 2>&1 || { tail -5 gpurun_out/r3m_lone_$v.log; exit 1; }
  echo "$v $(grep rep gpurun_out/r3m_lone_$v.log | tail -2 | cut -c1-150)"
done
VARIANTS="one pc" ROUNDS=2 STEPS=6 TAG=r3m bash tools/ab_bench.sh || exit 1
rm -f gpurun_out/*.dump
