#!/bin/bash
# Round-3 session s3m: bulk A/B -- touch the step end's zone rows right after the kick (vpf) vs current
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
VARIANTS="cur pf" ROUNDS=3 STEPS=6 TAG=s3m bash tools/ab_bench.sh
