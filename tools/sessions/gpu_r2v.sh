#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 150 python -u -m pytest tests/test_gpu_transport.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_transport.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|Error|Timeout" gpurun_out/pytest_transport.log | tail -6; [ $rc -eq 0 ] || exit $rc
VARIANTS="tnew tsplit" bash tools/sessions/gpu_r2u.sh
