#!/bin/bash
# Round-3 session s3j: long-photon chain with the lone translation unit scheduled by each machine
# scheduler strategy (the bulk unit unchanged)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for round in 1 2; do
  echo "== default ($round)"; timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
  for v in max-ilp iterative-ilp iterative-minreg max-memory-clause; do echo "== $v ($round)"
    GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_vs_$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
  done
done
