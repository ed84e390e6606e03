#!/bin/bash
# exec-mask issue-rate microbenchmark, then the round-end measurement set on the current tree (r02q)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 60 tools/microbench/exec_rate > gpurun_out/r02q_exec_rate.txt 2>&1 || { cat gpurun_out/r02q_exec_rate.txt; exit 1; }
cat gpurun_out/r02q_exec_rate.txt
TAG=r02q bash tools/gpu_final2.sh
