#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity_192.py tests/test_gpu_transport.py -x -v -s --timeout 250 --timeout-method thread > gpurun_out/pytest_parity.log 2>&1
rc=$?; grep -E "device:|oracle:|theta bin None|passed|failed" gpurun_out/pytest_parity.log; [ $rc -eq 0 ] || exit $rc
TAG=r02i bash tools/sessions/gpu_bench.sh
