#!/bin/bash
# A/B helper: gpu tests + bench at JOBS, then the timing-instrumented variant's per-phase breakdown.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
JOBS="${JOBS:-8}" bash tools/sessions/gpu_check.sh || exit $?
DEV_EMIT=1 DIAG_REPS=2 GRMONTY_AMD_LIB=cuda-grmonty_amd/variants/libgrmonty_amd_timing.so \
  timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > gpurun_out/diag_timing.log 2>&1 || exit 1
grep -E "rep|timing" gpurun_out/diag_timing.log
