#!/bin/bash
# polynomial coefficients from SGPRs (fma_k) + ocml-identical fexp/fexp10: probe + transport tests,
# then bench A/B against HEAD (base) and the lone-latency probe
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_probes.py tests/test_gpu_transport.py > gpurun_out/r3q_pytest.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3q_pytest.log | head -20; tail -30 gpurun_out/r3q_pytest.log; exit 1; }
grep -cE "PASSED" gpurun_out/r3q_pytest.log; grep -E "max ulp" gpurun_out/r3q_pytest.log | head
for v in new base; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" timeout -k 10 200 python tools/lone_bench.py 512 3 > gpurun_out/r3q_lone_$v.log 2>&1 || { tail -5 gpurun_out/r3q_lone_$v.log; exit 1; }
  echo "$v $(grep 'rep 2' gpurun_out/r3q_lone_$v.log | cut -c1-150)"
done
VARIANTS="new base" ROUNDS=2 STEPS=6 TAG=r3q bash tools/ab_bench.sh || exit 1
rm -f gpurun_out/*.dump
