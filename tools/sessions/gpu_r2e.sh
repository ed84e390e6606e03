#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bias_probe.py "$@" > gpurun_out/bias_probe.log 2>&1; rc=$?; cat gpurun_out/bias_probe.log; exit $rc
