#!/bin/bash
# instruction-cache behaviour of the transport kernel (100 KB of code): SQC counters, one small set per pass
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
PMC_SETS="SQC_ICACHE_HITS SQC_ICACHE_MISSES;SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_MISSES;SQ_IFETCH SQ_WAVE_CYCLES" \
  PROF_TAG=r02u DIAG="192 1e6" bash tools/gpu_pmc.sh > gpurun_out/r02u_icache.txt 2>&1 || { cat gpurun_out/r02u_icache.txt | tail; exit 1; }
tail -20 gpurun_out/r02u_icache.txt
rm -f gpurun_out/*.dump
