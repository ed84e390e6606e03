#!/bin/bash
# spectrum slices shared by workgroups (8 / 32, flushed by a kernel after each launch) vs one per
# workgroup: transport parity with the shared slices, bench A/B, L2 hit rate + HBM write bytes
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_vs8.so" timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_transport.py > gpurun_out/r3t_pytest.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/r3t_pytest.log | head -20; exit 1; }
grep -cE "PASSED" gpurun_out/r3t_pytest.log
VARIANTS="cur s8 s32" ROUNDS=2 STEPS=6 TAG=r3t bash tools/ab_bench.sh || exit 1
for v in cur s8; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" PMC_SETS="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum;WRITE_SIZE" PROF_TAG=r3t$v DIAG="192 1e6" bash tools/gpu_pmc.sh > gpurun_out/r3t_pmc_$v.txt 2>&1 || exit 1
  echo "$v: $(grep -E 'L2 hit|TCC_MISS|WRITE_SIZE|HBM' gpurun_out/r3t_pmc_$v.txt | tr '\n' ' ')"
done
rm -f gpurun_out/*.dump
