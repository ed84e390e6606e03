#!/bin/bash
# GPU tests on the current build, then A/B of engine variants over distinct-seed single passes
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
SEED=${SEED:-123} DIAG_REPS=${DIAG_REPS:-4} VARIANTS="${VARIANTS:-base walk}" bash tools/sessions/ab_libs.sh
