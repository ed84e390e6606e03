#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_gpu.log | head; exit $rc; }
VARIANTS="prev lone" SEED=123 DIAG_REPS=6 bash tools/sessions/gpu_ab2.sh
