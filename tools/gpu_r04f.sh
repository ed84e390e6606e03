#!/bin/bash
# round-4: live-bias parity tests (single GPU, emulated ranks) after the job-wide warm-up change
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity_192.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r04f_pytest_parity.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04f_pytest_parity.log | tail -2; grep -E " SE" gpurun_out/r04f_pytest_parity.log | head -40; rm -f gpurun_out/*.dump; exit $rc
