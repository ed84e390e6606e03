#!/bin/bash
# lone-kernel per-step timing, two builds, seed 125 (a ~5e5-step photon)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for v in ${VARIANTS:-tbase tnew}; do
DEV_EMIT=1 DIAG_REPS=1 SEED=125 GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" \
    timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > gpurun_out/lone_$v.log 2>&1 || exit 1
echo "== $v"; grep -E "^rep|lone geometry wave, photons" gpurun_out/lone_$v.log | cut -c1-260
done
