#!/bin/bash
# Round-3 session f: push latency microbenchmark (push_attempt vs push_attempt_rows), long-photon chain
# with and without the row-parallel push.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3f
timeout -k 10 120 ./tools/microbench/push_lat > gpurun_out/${T}_push_lat.txt 2>&1 || { cat gpurun_out/${T}_push_lat.txt; exit 1; }
cat gpurun_out/${T}_push_lat.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_transport.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop rc=$rc"; exit $rc; }
for v in vnorows vrows vvec vnorows vrows vvec; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 > gpurun_out/${T}_long_$v.log 2>&1 || { tail -5 gpurun_out/${T}_long_$v.log; exit 1; }
  echo "== $v $(grep rep gpurun_out/${T}_long_$v.log)"
done
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_timing.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 > gpurun_out/${T}_long_timing.log 2>&1 || { tail -5 gpurun_out/${T}_long_timing.log; exit 1; }
grep -E "rep|wave" gpurun_out/${T}_long_timing.log
rm -f gpurun_out/*.dump
