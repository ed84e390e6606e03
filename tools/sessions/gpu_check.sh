#!/bin/bash
# GPU check used during development: the -m gpu tests, then bench.py at a few --jobs values.
# Every GPU step has its own time limit; the script stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_gpu.log
grep -E "recorded:|KS D|emitted oracle|agreement" gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for j in ${JOBS:-1 4}; do
  timeout -k 10 240 python bench.py --steps ${STEPS:-8} --warmup 1 --jobs $j --cpu-seconds 0 > gpurun_out/bench_j$j.log 2>&1 || exit 1
  python tools/bench_brief.py gpurun_out/bench_j$j.log
done
exit 0
