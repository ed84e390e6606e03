#!/bin/bash
# which argument block to read through the kernarg pointer: both (cur), Params only, Ctl only
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
VARIANTS="cur ponly conly" ROUNDS=2 STEPS=6 TAG=r3s bash tools/ab_bench.sh || exit 1
rm -f gpurun_out/*.dump
