#!/bin/bash
# Round-3 session j: (1) end-of-pass hand-over of up to K photons per wave to lone pairs
# (GRM_OPT_LONE_K = 18; a full queue now falls back to the lane loop); (2) the warm-up's barrier
# slack (GRM_OPT_WARMUP_SLACK = 12, log2) and size (GRM_OPT_WARMUP = 8).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_transport.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/r3j_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r3j_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
OPTS="base 18=8 18=16 18=64" ROUNDS=2 STEPS=5 TAG=r3j bash tools/ab_opts.sh || exit 1
OPTS="12=2 12=1 8=16384,12=2 8=16384,12=1 8=65536,12=1" ROUNDS=2 STEPS=5 TAG=r3k bash tools/ab_opts.sh || exit 1
rm -f gpurun_out/*.dump
