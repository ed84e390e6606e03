#!/bin/bash
# Round-end measurement: PMC traffic passes (FETCH_SIZE, WRITE_SIZE; one counter block per run),
# then the default bench with that traffic folded in, then the same bench command under
# rocprofv3 --kernel-trace --stats.  Every GPU step has its own time limit; stop at a failure.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-final}
PMC_CMD="--steps 2 --warmup 1 --jobs 1 --cpu-seconds 0"
for c in FETCH_SIZE WRITE_SIZE; do
  ( cd /tmp && timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$c" -o run \
      -- python3 "$R/bench.py" $PMC_CMD ) > "$R/gpurun_out/pmc_${TAG}_$c.log" 2>&1 || { echo "pmc $c failed"; exit 1; }
done
CSV="$R/gpurun_out/pmc_${TAG}_FETCH_SIZE/run_counter_collection.csv,$R/gpurun_out/pmc_${TAG}_WRITE_SIZE/run_counter_collection.csv"
timeout -k 10 500 python3 bench.py --pmc-summary "$CSV" > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${TAG}" -o run \
    -- python3 "$R/bench.py" --pmc-summary "$CSV" ) > gpurun_out/prof_${TAG}.log 2>&1 || { echo "prof failed"; exit 1; }
grep -h '^{' gpurun_out/prof_${TAG}.log | tail -1 > gpurun_out/bench_${TAG}_under_rocprof.json
python3 tools/prof_summary.py gpurun_out/prof_${TAG} gpurun_out/bench_${TAG}_under_rocprof.json > gpurun_out/prof_${TAG}_summary.txt
cat gpurun_out/prof_${TAG}_summary.txt
exit 0
