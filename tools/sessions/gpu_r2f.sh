#!/bin/bash
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bias_chunks.py "$@" > gpurun_out/bias_chunks.log 2>&1; rc=$?; cat gpurun_out/bias_chunks.log; exit $rc
