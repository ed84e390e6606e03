#!/bin/bash
# One GPU measurement session (TAG names the outputs under gpurun_out/).  Every GPU step has its own
# time limit and the session stops at the first failure.  STEPS (default "tests smoke pmc bench prof
# cfg3 mix") selects:
#   tests  pytest -m gpu (TESTS = pytest selection, default the whole suite)
#   smoke  __graft_entry__.smoke()
#   pmc    PMC traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs) of a short bench -> pmc_traffic.json
#   bench  the default bench command (with that traffic when pmc ran)
#   prof   rocprofv3 --kernel-trace --stats of the same passes run alone
#   cfg3   BASELINE configs[3] rehearsal line: rank 0's shard of the 8-rank photon_n = 1e8 job
#   mix    PMC instruction mix / VALU utilisation (diag pass, 192^2 photon_n=1e6)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r05x}
S=" ${STEPS:-tests smoke pmc bench prof cfg3 mix} "
export TREE_REV=$(cat .tree_rev 2>/dev/null || echo "?")
has() { [[ "$S" == *" $1 "* ]]; }
if has tests; then
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -s -x --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/${T}_pytest_gpu.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/${T}_pytest_gpu.log | head; exit $rc; }
fi
if has smoke; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
fi
PMC_CMD="--steps 4 --warmup 1 --cpu-seconds 0 --overlap 0"
F="$R/gpurun_out/${T}_pmc_FETCH_SIZE/run_counter_collection.csv"; W="$R/gpurun_out/${T}_pmc_WRITE_SIZE/run_counter_collection.csv"
PS=""
if has pmc; then
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/${T}_pmc_$c" -o run \
      -- python3 "$R/bench.py" $PMC_CMD ) > "$R/gpurun_out/${T}_pmc_$c.log" 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 tools/traffic_summary.py "$F" "$W" "gpurun_out/${T}_pmc_FETCH_SIZE.log" gpurun_out/${T}_pmc_traffic.json || exit 1
PS="--pmc-summary $F,$W"
fi
if has bench; then
timeout -k 10 900 python3 -u bench.py $PS $BENCH_ARGS > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail -5 gpurun_out/${T}_bench.err; exit 1; }
tail -c 600 gpurun_out/${T}_bench.json
fi
if has prof; then
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_prof" -o run \
    -- python3 "$R/bench.py" --steps 10 --warmup 1 --cpu-seconds 0 --overlap 0 $PS ) > gpurun_out/${T}_prof.log 2>&1 || { echo "prof failed"; exit 1; }
grep -h '^{"metric"' gpurun_out/${T}_prof.log | tail -1 > gpurun_out/${T}_bench_under_rocprof.json
python3 tools/prof_summary.py gpurun_out/${T}_prof gpurun_out/${T}_bench_under_rocprof.json > gpurun_out/${T}_rocprof_summary.txt || exit 1
head -12 gpurun_out/${T}_rocprof_summary.txt | cut -c1-160
fi
if has cfg3; then
timeout -k 10 300 python3 -u bench.py --photon-n 1.25e7 --shard-of 0/8 --steps 3 --warmup 1 --cpu-seconds 0 --overlap 0 > gpurun_out/${T}_bench_config3_shard0of8.json 2> gpurun_out/${T}_bench_config3.err || { echo "config3 bench failed"; tail -5 gpurun_out/${T}_bench_config3.err; exit 1; }
tail -c 300 gpurun_out/${T}_bench_config3_shard0of8.json
fi
if has mix; then
PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU;SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS;TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
  PROF_TAG=${T}mix DIAG="192 1e6" bash tools/gpu_pmc.sh > gpurun_out/${T}_pmc_mix.txt 2>&1 || exit 1
tail -14 gpurun_out/${T}_pmc_mix.txt
fi
rm -f gpurun_out/*.dump
exit 0
