#!/bin/bash
# Round-3 session m: timeline of the main launch (warm-up end, pool drained, last exit), 1e6 and 1e7
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pass_phases.py 5 1e6 > gpurun_out/r3m_phases_1e6.log 2>&1 || { tail -5 gpurun_out/r3m_phases_1e6.log; exit 1; }
cat gpurun_out/r3m_phases_1e6.log
timeout -k 10 300 python -u tools/pass_phases.py 2 1e7 > gpurun_out/r3m_phases_1e7.log 2>&1 || { tail -5 gpurun_out/r3m_phases_1e7.log; exit 1; }
cat gpurun_out/r3m_phases_1e7.log
rm -f gpurun_out/*.dump
