#!/bin/bash
# first warm-up batch sweep: counters at 192^2 photon_n=1e5 (vs the oracle spread) and kernel time at 1e6
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
SEEDS=123,124,125,126 timeout -k 10 400 python tools/bias_probe.py warm:4096:4:64 warm:4096:4:256 warm:4096:4:1024 warm:4096:3:256 > gpurun_out/warmb_sweep.log 2>&1
rc=$?; cut -c1-160 gpurun_out/warmb_sweep.log; [ $rc -eq 0 ] || exit $rc
for b in 64 256 1024 64; do
DEV_EMIT=1 DIAG_REPS=3 SEED=123 WARMUP_BATCH=$b timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > gpurun_out/warmb_t_$b.log 2>&1 || exit 1
echo "batch0 $b"; grep -E "^rep" gpurun_out/warmb_t_$b.log | cut -c1-110
done
