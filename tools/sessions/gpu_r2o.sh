#!/bin/bash
# 512^2 (BASELINE config[4]) measurement: bench, rocprof kernel stats, PMC passes (L2 hit/miss,
# HBM traffic, instruction mix) at 512^2 and, for comparison, 192^2
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --grid 512 --steps 5 --warmup 1 --cpu-seconds 0 --overlap 0 > gpurun_out/r2o_bench512.json 2> gpurun_out/r2o_bench512.err
rc=$?; tail -c 600 gpurun_out/r2o_bench512.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/r2o_bench512.err; exit $rc; }
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r2o_prof512" -o run -- python3 $R/bench.py --grid 512 --steps 3 --warmup 1 --cpu-seconds 0 --overlap 0 ) > gpurun_out/r2o_prof512.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cut -c1-150 gpurun_out/r2o_prof512/run_kernel_stats.csv
PMC_SETS="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum;FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" PROF_TAG=g512 DIAG="512 1e6" bash tools/gpu_pmc.sh || exit 1
PMC_SETS="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum;FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" PROF_TAG=g192 DIAG="192 1e6" bash tools/gpu_pmc.sh || exit 1
python3 tools/pmc_summary.py gpurun_out g512 > gpurun_out/r2o_pmc512.txt; python3 tools/pmc_summary.py gpurun_out g192 > gpurun_out/r2o_pmc192.txt
rm -f gpurun_out/*.dump; rm -rf gpurun_out/pmc_g*_*/run_agent_info.csv
du -sh gpurun_out
