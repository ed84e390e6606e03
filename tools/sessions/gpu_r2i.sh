#!/bin/bash
# capture the seed-125 tail photon's state (watchdog abandons the launch after 1.5 s); timing breakdown
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
DEV_EMIT=1 DIAG_REPS=1 SEED=125 WATCHDOG_MS=1500 timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/diag_stuck125.log 2>&1
rc=$?; cat gpurun_out/diag_stuck125.log; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
DEV_EMIT=1 DIAG_REPS=2 SEED=124 GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_timing.so" timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/r02b_timing.log 2>&1
rc=$?; cat gpurun_out/r02b_timing.log | grep -E "rep|timing"; exit $rc
