#!/bin/bash
# round-4: live-bias counters vs photons in flight, 96 seeds per grid (the parity test's seeds)
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 700 python -u tools/live_bias_grid_sweep.py --grids 256,32,8 --seeds 123-218 --out gpurun_out/r04h_grid_sweep96.jsonl > gpurun_out/r04h_grid_sweep96.log 2>&1
rc=$?; tail -c 300 gpurun_out/r04h_grid_sweep96.log; rm -f gpurun_out/*.dump; exit $rc
