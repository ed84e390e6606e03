#!/bin/bash
# lone pipeline latency (one long photon alone in lone_kernel): current tree vs a built revision
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for v in cur base; do
  echo "== $v"
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" timeout -k 10 200 python -u tools/lone_bench.py 20000 5 > gpurun_out/r3h_$v.log 2>&1 || { tail -5 gpurun_out/r3h_$v.log; exit 1; }
  grep rep gpurun_out/r3h_$v.log
done
rm -f gpurun_out/*.dump
