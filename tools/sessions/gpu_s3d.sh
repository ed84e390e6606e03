#!/bin/bash
# Round-3 session s3d: lone kernels in their own translation unit (machine LICM on, plain fma):
# photon-by-photon tests of every device path, long-photon chain against the LICM-off build of the
# same split (vlicmoff), the timing build's geometry / interaction split, one bench line.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=s3d
timeout -k 10 600 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_safety.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|agreement" gpurun_out/${T}_pytest.log | head; exit $rc; }
for round in 1 2; do
  echo "== long photon, current ($round)"; timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
  echo "== long photon, vlicmoff ($round)"
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_vlicmoff.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
done
echo "== long photon, GRM_TIMING build"
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_timing.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --overlap 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail -5 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]); t=d['detail']; r=d['roofline']
print('bench', round(d['value']/1e6,2), 'M/s frac', round(r['frac'],4), 'dominant', round(t['dominant_launch_ms_per_pass'],1), 'ms passes', t['pass_s']['all'])"
