#!/bin/bash
# A/B of the batched-refill threshold (one process per setting, each under its own time limit)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for rm in ${REFILLS:-1 8 16 32}; do
  REFILL_MIN=$rm DIAG_REPS=2 timeout -k 10 200 python tools/gpu_diag.py ${DIAG:-192 1e5} > gpurun_out/ab_refill_$rm.log 2>&1
  rc=$?; echo "refill_min=$rm rc=$rc"; grep -E "^rep" gpurun_out/ab_refill_$rm.log | tail -1
  [ $rc -eq 0 ] || exit $rc
done
if [ -n "$TIMING" ]; then
  GRMONTY_AMD_LIB=$R/cuda-grmonty_amd/variants/libgrmonty_amd_timing.so REFILL_MIN=${TIMING} DIAG_REPS=1 \
    timeout -k 10 200 python tools/gpu_diag.py ${DIAG:-192 1e5} > gpurun_out/diag_timing.log 2>&1
  rc=$?; echo "timing rc=$rc"; cat gpurun_out/diag_timing.log; [ $rc -eq 0 ] || exit $rc
fi
exit 0
