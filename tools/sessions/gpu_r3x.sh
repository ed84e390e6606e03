#!/bin/bash
# max_n_step photons of the seed-126 pass (frozen bias, traced) for an oracle replay
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/maxstep_probe.py 126 > gpurun_out/r3x_maxstep_126.log 2>&1 || { tail -20 gpurun_out/r3x_maxstep_126.log; exit 1; }
cat gpurun_out/r3x_maxstep_126.log | head -40
rm -f gpurun_out/*.dump
