#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_probes.py tests/test_gpu_transport.py -x -v -s --timeout 250 --timeout-method thread > gpurun_out/pytest_probes.log 2>&1
rc=$?; grep -E "fsincospi max|PASS|FAIL|passed|failed|Error" gpurun_out/pytest_probes.log | tail -8; [ $rc -eq 0 ] || exit $rc
VARIANTS="base new" SEED=123 DIAG_REPS=3 bash tools/sessions/gpu_ab2.sh
