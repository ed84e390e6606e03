#!/bin/bash
# round-4: occupancy experiment -- 768-lane workgroups (three waves per SIMD, VGPRs capped at 168,
# spills) with the two state copies in HBM (w768g), the state copies in HBM alone (w512g), and the
# product build (base): photon-by-photon check of the variants, then an interleaved bench A/B
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for v in w768g w512g; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 300 python -u -m pytest tests/test_gpu_transport.py -k "lane-loop" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04l_pbp_$v.log 2>&1 || { echo "pbp $v failed"; tail -5 gpurun_out/r04l_pbp_$v.log; exit 1; }
  tail -1 gpurun_out/r04l_pbp_$v.log
done
VARIANTS="base w768g w512g" ROUNDS=2 STEPS=6 TAG=r04l bash tools/ab_bench.sh 2>&1 | tee gpurun_out/r04l_ab.txt
