export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_config3.py -v -s --timeout 280 --timeout-method thread > gpurun_out/r04_config3.log 2>&1
rc=$?; tail -5 gpurun_out/r04_config3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/live_bias_grid_sweep.py --grids 8,32,256 --seeds 123-146 --out gpurun_out/r04_grid_sweep.jsonl > gpurun_out/r04_grid_sweep.log 2>&1
rc=$?; tail -c 400 gpurun_out/r04_grid_sweep.log; rm -f gpurun_out/*.dump; exit $rc
