#!/bin/bash
# round-4: job-wide warm-up gate (emulated ranks) + flight ratio 96: the parity tests
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity_192.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r04k_pytest_parity.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04k_pytest_parity.log | tail -1; grep -E " SE" gpurun_out/r04k_pytest_parity.log | cut -c1-200 | head -40
exit $rc
