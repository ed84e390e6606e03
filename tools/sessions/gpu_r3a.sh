#!/bin/bash
# Round-3 session a: the GPU suite with the new multi-seed / multi-rank / guard tests, smoke, one bench.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3a
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop rc=$rc"; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --overlap 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail -5 gpurun_out/${T}_bench.err; exit 1; }
tail -c 1500 gpurun_out/${T}_bench.json
rm -f gpurun_out/*.dump
exit $rc
