#!/bin/bash
# round-4 session: full GPU suite (incl. the configs[3] shard test), then the live-bias grid sweep
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r04e_pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04e_pytest_gpu.log | tail -2; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r04e_pytest_gpu.log | head; exit $rc; }
timeout -k 10 400 python -u tools/live_bias_grid_sweep.py --grids 8,32,256 --seeds 123-146 --out gpurun_out/r04_grid_sweep.jsonl > gpurun_out/r04_grid_sweep.log 2>&1
rc=$?; tail -c 300 gpurun_out/r04_grid_sweep.log; rm -f gpurun_out/*.dump; exit $rc
