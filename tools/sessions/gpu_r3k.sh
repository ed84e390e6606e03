#!/bin/bash
# Re-entry check of the restored tree: GPU tests, smoke, default bench line.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
T=r02q
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${T}_pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${T}_smoke.log; exit 1; }
cat gpurun_out/${T}_smoke.log | tail -2
timeout -k 10 600 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail -5 gpurun_out/${T}_bench.err; exit 1; }
tail -c 900 gpurun_out/${T}_bench.json
