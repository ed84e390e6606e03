#!/bin/bash
# capture the seed-123 tail photon's state (watchdog abandons the launch after 1.5 s)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
DEV_EMIT=1 DIAG_REPS=1 SEED=123 WATCHDOG_MS=1500 timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/diag_stuck.log 2>&1
rc=$?; cat gpurun_out/diag_stuck.log; [ $rc -eq 0 ] || [ $rc -eq 3 ]
