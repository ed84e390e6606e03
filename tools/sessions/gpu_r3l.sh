#!/bin/bash
# kernarg reads through the kernarg segment pointer: transport tests, then A/B (base = HEAD behaviour,
# pc = track_kernel Params+Ctl, all = + lone/early kernels), then the full GPU suite
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_transport.py > gpurun_out/r3l_pytest_transport.log 2>&1 || { tail -20 gpurun_out/r3l_pytest_transport.log; exit 1; }
grep -cE "PASSED" gpurun_out/r3l_pytest_transport.log
VARIANTS="base pc all" ROUNDS=2 STEPS=6 TAG=r3l bash tools/ab_bench.sh || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02q_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/r02q_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/r02q_pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02q_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/r02q_smoke.log; exit 1; }
tail -1 gpurun_out/r02q_smoke.log
rm -f gpurun_out/*.dump
