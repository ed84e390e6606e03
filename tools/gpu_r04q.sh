#!/bin/bash
# round-4: N-rank offset -- independent concurrent jobs (no sharding, no linked counters)
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
( timeout -k 10 300 python -u tools/concurrent_jobs.py 8 6 && timeout -k 10 300 python -u tools/concurrent_jobs.py 1 48 && \
  timeout -k 10 300 python -u tools/concurrent_jobs.py 8 6 20=0 ) > gpurun_out/r04q_concurrent.log 2>&1
rc=$?; cat gpurun_out/r04q_concurrent.log | tail -5; exit $rc
