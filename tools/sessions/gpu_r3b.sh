#!/bin/bash
# Round-3 session b: strided multi-rank parity, the guard test, the engine-stash gloo test; then an
# interleaved A/B of the bulk with and without the spectrum atomics (experiment build GRM_X_NOSPEC).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3b
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_safety.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop rc=$rc"; exit $rc; }
VARIANTS="base nospec" ROUNDS=2 STEPS=6 TAG=${T}ab bash tools/ab_bench.sh || exit 1
rm -f gpurun_out/*.dump
