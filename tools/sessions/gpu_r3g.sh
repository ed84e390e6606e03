#!/bin/bash
# early worker under kernel serialisation: transport tests (incl. the serialised mode), then a PMC pass
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_transport.py > gpurun_out/r3g_pytest.log 2>&1 || { tail -20 gpurun_out/r3g_pytest.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r3g_pytest.log | cut -c1-120
( cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/r3g_pmc" -o run \
    -- python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-seconds 0 --overlap 0 ) > gpurun_out/r3g_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r3g_pmc.log; exit 1; }
grep -h '^{"metric"' gpurun_out/r3g_pmc.log | cut -c1-200
rm -f gpurun_out/*.dump
