#!/bin/bash
# Round-3 session s3a: warm-up spread 4 (default): full GPU suite (parity at 1e5 / 1e6, emulated
# ranks), smoke, and two bench lines.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=s3a
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop rc=$rc"; exit $rc; }
grep -E "ranks (recorded|scattered|steps|luminosity)|^(1e6 )?(recorded|scattered|steps|luminosity) |FAILED" gpurun_out/${T}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --cpu-seconds 0 --overlap 0 > gpurun_out/${T}_bench_$i.json 2> gpurun_out/${T}_bench_$i.err || { echo bench failed; tail -5 gpurun_out/${T}_bench_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench_$i.json').read().strip().splitlines()[-1]); t=d['detail']; r=d['roofline']
print('bench', round(d['value']/1e6,2), 'M/s frac', round(r['frac'],4), 'dominant', round(t['dominant_launch_ms_per_pass'],1), 'ms passes', t['pass_s']['all'], 'recorded/pass', t['recorded_per_pass'])"
done
rm -f gpurun_out/*.dump
exit $rc
