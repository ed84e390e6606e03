#!/bin/bash
# Round-2 measurement session: GPU tests, default bench, rocprof kernel stats of the bench, PMC
# traffic of the bench, PMC instruction mix + timing breakdown of one pass.  Every GPU step has
# its own time limit; the script stops at the first failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-r02b}
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest_gpu.log; grep -E "matching|KS D|device:|oracle:|spectrum cells" gpurun_out/${T}_pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err
rc=$?; tail -c 1500 gpurun_out/${T}_bench_default.json; echo; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
BCMD="$R/bench.py --steps ${PSTEPS:-4} --warmup 1 --cpu-seconds 0 --overlap 0"
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_prof" -o run -- python3 $BCMD ) > gpurun_out/${T}_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/${T}_pmc_$c" -o run -- python3 $BCMD ) > gpurun_out/${T}_pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic_summary.py gpurun_out/${T}_pmc_FETCH_SIZE/run_counter_collection.csv gpurun_out/${T}_pmc_WRITE_SIZE/run_counter_collection.csv gpurun_out/${T}_pmc_FETCH_SIZE.log gpurun_out/${T}_pmc_traffic.json
DEV_EMIT=1 DIAG="192 1e6" SEED=124 PROF_TAG=${T}_mix PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32;SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH;TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" bash tools/gpu_pmc.sh
rc=$?; [ $rc -eq 0 ] || exit $rc
DEV_EMIT=1 DIAG_REPS=2 SEED=124 GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_timing.so" timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/${T}_timing.log 2>&1
rc=$?; cat gpurun_out/${T}_timing.log | grep -E "rep|timing"; exit $rc
