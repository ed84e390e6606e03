#!/bin/bash
# Round-3 session f: push latency microbenchmark (push_attempt vs push_attempt_rows), long-photon chain
# with and without the row-parallel push.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3f
timeout -k 10 120 ./tools/microbench/push_lat > gpurun_out/${T}_push_lat.txt 2>&1 || { cat gpurun_out/${T}_push_lat.txt; exit 1; }
cat gpurun_out/${T}_push_lat.txt
for v in vnorows vrows vnorows vrows; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 > gpurun_out/${T}_long_$v.log 2>&1 || { tail -5 gpurun_out/${T}_long_$v.log; exit 1; }
  echo "== $v $(grep rep gpurun_out/${T}_long_$v.log)"
done
rm -f gpurun_out/*.dump
