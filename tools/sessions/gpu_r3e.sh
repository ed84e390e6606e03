#!/bin/bash
# scheduler-strategy A/B of the transport kernel: bulk steps/s over 3 passes each, interleaved twice
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for round in 1 2; do for v in new max-memory-clause iterative-maxocc max-ilp; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" DIAG_REPS=3 SEED=124 timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/r3e_${v}_$round.log 2>&1 || { tail -5 gpurun_out/r3e_${v}_$round.log; exit 1; }
  echo "$v $round: $(grep -oE 'kernel [0-9.]+ms' gpurun_out/r3e_${v}_$round.log | tr '\n' ' ') $(grep -oE 'bulk [0-9.]+ Msteps/s' gpurun_out/r3e_${v}_$round.log | tr '\n' ' ')"
done; done
rm -f gpurun_out/*.dump
