#!/bin/bash
# warm-up size / slack sweep: counters at 192^2 photon_n=1e5 (vs the oracle spread) and pass time at 1e6
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
SEEDS=123,124,125,126 timeout -k 10 400 python tools/bias_probe.py warm:0 warm:2048 warm:4096 warm:8192 warm:8192:2 warm:32768 warm:32768:2 > gpurun_out/warm_sweep.log 2>&1
rc=$?; cat gpurun_out/warm_sweep.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
for wu in 32768 8192 4096 2048; do
DEV_EMIT=1 DIAG_REPS=3 SEED=123 WARMUP=$wu timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > gpurun_out/warm_t_$wu.log 2>&1 || exit 1
echo "warmup $wu"; grep -E "^rep" gpurun_out/warm_t_$wu.log | cut -c1-120
done
