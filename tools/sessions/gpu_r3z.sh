#!/bin/bash
# stash-and-reduce-once API (1-rank RCCL), full GPU suite, smoke, default bench on the final tree
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r02v
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${T}_pytest_gpu.log | head; exit $rc; }
grep -E "stash" gpurun_out/${T}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail -5 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M/s', d['roofline']['frac'], d['detail']['pass_s']['all'], d['config']['parallelism'])"
rm -f gpurun_out/*.dump
