#!/bin/bash
# timing breakdown with and without the live-bias warm-up
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for wu in 32768 0; do
DEV_EMIT=1 DIAG_REPS=2 SEED=123 WARMUP=$wu GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_vtime1.so" \
    timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > gpurun_out/warm_$wu.log 2>&1 || exit 1
grep -E "rep|timing|waves" gpurun_out/warm_$wu.log | cut -c1-420
done
