#!/bin/bash
# round-4 A/B: the current tree (vr4b) against bab96d7 (vr4a) -- the long-photon chain and the bench
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
V=${VARIANTS:-"r4a r4b"}
for round in 1 2; do for v in $V; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 120 python -u tools/long_photon_bench.py 2 > gpurun_out/r04g_long_${v}_$round.log 2>&1 || { tail -3 gpurun_out/r04g_long_${v}_$round.log; exit 1; }
  echo "$v chain: $(grep rep gpurun_out/r04g_long_${v}_$round.log | tail -1 | sed 's/.*-> //')"
done; done
VARIANTS="$V" ROUNDS=2 STEPS=6 TAG=r04g bash tools/ab_bench.sh
rm -f gpurun_out/*.dump
