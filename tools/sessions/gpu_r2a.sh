#!/bin/bash
# round-2 first check: GPU tests, then single passes at distinct seeds (tail census)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
DEV_EMIT=1 DIAG_REPS=${REPS:-8} SEED=123 timeout -k 10 400 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/diag_seeds.log 2>&1
rc=$?; cat gpurun_out/diag_seeds.log | grep -v "^  timing"; exit $rc
