#!/bin/bash
# blit-free passes: GPU tests, then a rocprof kernel-trace of a short default bench
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_gpu.log | head; exit $rc; }
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2n -o run -- python3 bench.py --steps 4 --warmup 1 > gpurun_out/bench_prof_r2n.log 2>&1
rc=$?; tail -2 gpurun_out/bench_prof_r2n.log; exit $rc
