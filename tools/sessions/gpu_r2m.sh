#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transport.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_transport.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_transport.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/pytest_transport.log | head; exit $rc; }
bash tools/sessions/gpu_r2l.sh
DEV_EMIT=1 DIAG_REPS=1 SEED=125 timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > gpurun_out/lone_main.log 2>&1
rc=$?; grep -E "rep" gpurun_out/lone_main.log | cut -c1-400; exit $rc
