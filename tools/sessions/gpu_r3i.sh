#!/bin/bash
# Round-3 session i: what the live-bias warm-up costs inside the dominant launch at photon_n = 1e6
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
OPTS="base 8=0 8=1024 14=512 8=16384" ROUNDS=2 STEPS=5 TAG=r3i bash tools/ab_opts.sh || exit 1
rm -f gpurun_out/*.dump
