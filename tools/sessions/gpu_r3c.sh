#!/bin/bash
# lone-pipeline: transport tests, then timing (GRM_TIMING variant) of the seed-125 pass
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_transport.py > gpurun_out/r3c_pytest.log 2>&1 || { tail -20 gpurun_out/r3c_pytest.log; exit 1; }
tail -2 gpurun_out/r3c_pytest.log
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_timing.so" DEV_EMIT=1 DIAG_REPS=1 SEED=125 timeout -k 10 300 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/r3c_timing.log 2>&1 || { tail -5 gpurun_out/r3c_timing.log; exit 1; }
grep -E "rep|lone" gpurun_out/r3c_timing.log
rm -f gpurun_out/*.dump
