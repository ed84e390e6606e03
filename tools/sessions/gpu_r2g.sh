#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bias_probe.py live > gpurun_out/bias_probe.log 2>&1; rc=$?; cat gpurun_out/bias_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; grep -E "matching|KS D|device:|oracle:|spectrum cells|recorded:" gpurun_out/pytest_gpu.log | head -30; exit $rc
