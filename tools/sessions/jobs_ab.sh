cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for j in 16 24 30 12 24 16; do
  timeout -k 10 240 python bench.py --steps 48 --warmup 1 --cpu-seconds 0 --jobs $j > gpurun_out/jobs_$j.log 2>&1 || { echo "jobs $j failed"; exit 1; }
  echo "jobs=$j $(python tools/bench_brief.py gpurun_out/jobs_$j.log)"
done
