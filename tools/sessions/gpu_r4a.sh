#!/bin/bash
# memory-side latency of the transport kernel: L1->L2 read latency, LDS bank conflicts, TA busy
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
PMC_SETS="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES;TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum;TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_sum" \
  PROF_TAG=r02w DIAG="192 1e6" bash tools/gpu_pmc.sh > gpurun_out/r02w_memlat.txt 2>&1 || { tail gpurun_out/r02w_memlat.txt; exit 1; }
tail -24 gpurun_out/r02w_memlat.txt
rm -f gpurun_out/*.dump
