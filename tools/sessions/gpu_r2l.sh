#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
DEV_EMIT=1 DIAG_REPS=2 SEED=${SEED:-125} GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_vtime1.so" \
    timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > gpurun_out/lone_t1.log 2>&1
rc=$?; grep -E "rep|lone" gpurun_out/lone_t1.log | cut -c1-400; exit $rc
