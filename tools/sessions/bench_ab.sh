#!/bin/bash
# bench.py A/B of engine builds on one box: VARIANTS names variants/libgrmonty_amd_v<name>.so ("main" =
# the in-tree library); each run is the default pipelined bench without the CPU baseline.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
i=0
for v in ${VARIANTS:-main}; do
  i=$((i+1))
  if [ "$v" = main ]; then lib=""; else lib="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so"; fi
  GRMONTY_AMD_LIB=$lib timeout -k 10 ${T_BENCH:-300} python bench.py --steps ${STEPS:-16} --warmup 1 --cpu-seconds 0 ${BENCH_ARGS} \
    > gpurun_out/bench_ab_${i}_$v.log 2>&1 || { echo "bench $v failed"; tail -3 gpurun_out/bench_ab_${i}_$v.log; exit 1; }
  echo "== $v: $(python tools/bench_brief.py gpurun_out/bench_ab_${i}_$v.log | cut -d: -f2-)"
done
