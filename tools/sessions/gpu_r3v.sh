#!/bin/bash
# interaction uniform drawn while the zone gather is in flight (edraw) vs cur: transport parity, A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_vedraw.so" timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_transport.py > gpurun_out/r3v_pytest.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3v_pytest.log | head -20; exit 1; }
grep -cE "PASSED" gpurun_out/r3v_pytest.log; grep -E "matching" gpurun_out/r3v_pytest.log | head -5
VARIANTS="cur edraw" ROUNDS=3 STEPS=6 TAG=r3v bash tools/ab_bench.sh || exit 1
rm -f gpurun_out/*.dump
