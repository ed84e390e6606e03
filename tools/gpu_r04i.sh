#!/bin/bash
# round-4: parity tests with the in-flight cap (GRM_OPT_FLIGHT_RATIO), then the A/B of this round's
# kernel changes (vr4b) against bab96d7 (vr4a): long-photon chain + bench; then a GRM_TIMING diag
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity_192.py -v -s --timeout 400 --timeout-method thread > gpurun_out/r04i_pytest_parity.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04i_pytest_parity.log | tail -1; grep -E " SE" gpurun_out/r04i_pytest_parity.log | grep -v "f\"" | head -40
bash tools/gpu_r04g.sh || exit 1
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_timing.so" DEV_EMIT=1 DIAG_REPS=2 timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/r04i_timing_diag.log 2>&1; tail -6 gpurun_out/r04i_timing_diag.log | cut -c1-400
rm -f gpurun_out/*.dump
exit $rc
