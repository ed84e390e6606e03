#!/bin/bash
# early worker (full grid + liveness word): transport tests, diag waves, bench A/B
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_transport.py > gpurun_out/r3b_pytest.log 2>&1 || { tail -20 gpurun_out/r3b_pytest.log; exit 1; }
tail -2 gpurun_out/r3b_pytest.log
DIAG_REPS=4 SEED=124 timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/r3b_diag.log 2>&1 || { tail -5 gpurun_out/r3b_diag.log; exit 1; }
grep -E "rep|waves" gpurun_out/r3b_diag.log
for round in 1 2; do for v in early noearly; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" timeout -k 10 300 python bench.py --cpu-seconds 0 --overlap 0 > gpurun_out/benchab_${v}_$round.json 2> gpurun_out/benchab_${v}_$round.err || { tail -3 gpurun_out/benchab_${v}_$round.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/benchab_${v}_$round.json').read().strip().splitlines()[-1])
print('$v', round(d['value']/1e6,2), 'M/s passes', d['detail']['pass_s']['all'], 'longest', d['detail']['longest_photon_life_steps'])"
done; done
rm -f gpurun_out/*.dump
