#!/bin/bash
# Round-3 session s3i: timing build on the long photon (geometry / interaction balance after the
# two-row quad push); bulk A/B: s_setprio 3 around the zone gather's issue (vprio) vs current (vcur)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_timing.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
VARIANTS="cur prio" ROUNDS=3 STEPS=6 TAG=s3i bash tools/ab_bench.sh
