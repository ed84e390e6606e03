#!/bin/bash
# Round-3 session s3k: bulk unit machine scheduler A/B (default = vcur, max-ilp, iterative-minreg);
# the lone unit keeps max-ilp in all three
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
VARIANTS="cur bmaxilp bminreg" ROUNDS=3 STEPS=6 TAG=s3k bash tools/ab_bench.sh
