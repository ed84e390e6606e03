#!/bin/bash
# machine-scheduler strategy for the lone pipeline's serial chain: lone-latency probe, twice each
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for r in 1 2; do for v in cur maxilp maxmem; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" timeout -k 10 200 python tools/lone_bench.py 512 3 > gpurun_out/r3y_lone_${v}_$r.log 2>&1 || { tail -5 gpurun_out/r3y_lone_${v}_$r.log; exit 1; }
  echo "$v $(grep 'rep 2' gpurun_out/r3y_lone_${v}_$r.log | cut -c1-150)"
done; done
rm -f gpurun_out/*.dump
