#!/bin/bash
# Round-3 session c: counter systematic vs warm-up size and rank count (tools/warmup_sweep2.py)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3c
timeout -k 10 500 python -u tools/warmup_sweep2.py --photon-n 1e5 --seeds 16 --warmups 4096,16384,65536,-1 --worlds 1,8 > gpurun_out/${T}_sweep_1e5.log 2>&1 || { tail -5 gpurun_out/${T}_sweep_1e5.log; exit 1; }
cat gpurun_out/${T}_sweep_1e5.log
timeout -k 10 500 python -u tools/warmup_sweep2.py --photon-n 1e6 --seeds 6 --warmups 4096,65536,-1 --worlds 1 --golden oracle_synth192_pn1e6 > gpurun_out/${T}_sweep_1e6.log 2>&1 || { tail -5 gpurun_out/${T}_sweep_1e6.log; exit 1; }
cat gpurun_out/${T}_sweep_1e6.log
rm -f gpurun_out/*.dump
