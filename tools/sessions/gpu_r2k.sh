#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transport.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_transport.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_transport.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_transport.log | head; exit $rc; }
VARIANTS="time0 time1" SEED=125 DIAG_REPS=2 DIAG="192 1e6" bash tools/sessions/gpu_ab2.sh
grep -h "lone" gpurun_out/ab_vtime*_1.log
