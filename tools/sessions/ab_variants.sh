#!/bin/bash
# A/B of kernel build variants in one session (same box): occupancy 1 vs 2
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"
for v in ${VARIANTS:-1 2}; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_w$v.so" timeout -k 10 300 python tools/gpu_diag.py ${DIAG:-192 1e5} > gpurun_out/ab_w$v.log 2>&1
  rc=$?; echo "variant w$v rc=$rc"; tail -2 gpurun_out/ab_w$v.log
  [ $rc -eq 0 ] || exit $rc
done
