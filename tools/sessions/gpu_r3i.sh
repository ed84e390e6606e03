#!/bin/bash
# transport + parity tests on the current tree, then the lone latency probe
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_transport.py tests/test_gpu_parity_192.py > gpurun_out/r3i_pytest.log 2>&1 || { tail -20 gpurun_out/r3i_pytest.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r3i_pytest.log | cut -c1-120
bash tools/sessions/gpu_r3h.sh
