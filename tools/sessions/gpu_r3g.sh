#!/bin/bash
# Round-3 session g: the metric's uniform factors precomputed (vpar) vs HEAD (vhead): transport tests,
# long-photon chain, interleaved bulk A/B.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3g
timeout -k 10 400 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_probes.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop rc=$rc"; exit $rc; }
for v in vhead vpar vhead vpar; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 > gpurun_out/${T}_long_$v.log 2>&1 || { tail -5 gpurun_out/${T}_long_$v.log; exit 1; }
  echo "== $v $(grep rep gpurun_out/${T}_long_$v.log)"
done
VARIANTS="head par" ROUNDS=3 STEPS=6 TAG=${T}ab bash tools/ab_bench.sh || exit 1
timeout -k 10 120 ./tools/microbench/push_lat > gpurun_out/${T}_push_lat.txt 2>&1 || exit 1
head -8 gpurun_out/${T}_push_lat.txt
rm -f gpurun_out/*.dump
exit $rc
