#!/bin/bash
# small relaunches through the lone pipeline: transport tests, then bench A/B vs HEAD
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_transport.py > gpurun_out/r3j_pytest.log 2>&1 || { tail -20 gpurun_out/r3j_pytest.log; exit 1; }
grep -cE "PASSED" gpurun_out/r3j_pytest.log
for round in 1 2; do for v in cur base; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" timeout -k 10 300 python bench.py --cpu-seconds 0 --overlap 0 > gpurun_out/r3j_${v}_$round.json 2> gpurun_out/r3j_${v}_$round.err || { tail -3 gpurun_out/r3j_${v}_$round.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r3j_${v}_$round.json').read().strip().splitlines()[-1]); t=d['detail']
print('$v', round(d['value']/1e6,2), 'M/s kernel_ms/pass', round(t['kernel_ms_per_pass'],1), 'dominant', round(t['dominant_launch_ms_per_pass'],1), 'passes', t['pass_s']['all'])"
done; done
rm -f gpurun_out/*.dump
