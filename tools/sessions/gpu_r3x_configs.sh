#!/bin/bash
# Round-3 session x (final tree): BASELINE configs[4] (512^2) and configs[2] (photon_n = 1e7) bench lines on the final kernels.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3x
timeout -k 10 400 python -u bench.py --grid 512 --steps 5 --warmup 1 --cpu-seconds 0 --overlap 0 > gpurun_out/${T}_bench_grid512.json 2> gpurun_out/${T}_bench_grid512.err || { tail -5 gpurun_out/${T}_bench_grid512.err; exit 1; }
tail -c 400 gpurun_out/${T}_bench_grid512.json
timeout -k 10 500 python -u bench.py --photon-n 1e7 --steps 3 --warmup 1 --cpu-seconds 0 --overlap 0 > gpurun_out/${T}_bench_pn1e7.json 2> gpurun_out/${T}_bench_pn1e7.err || { tail -5 gpurun_out/${T}_bench_pn1e7.err; exit 1; }
tail -c 400 gpurun_out/${T}_bench_pn1e7.json
rm -f gpurun_out/*.dump
