#!/bin/bash
# round-4: write-traffic A/B of the record alignment (Cold 80 -> 64 B, SReq 208 -> 192 B): WRITE_SIZE
# per dominant track_kernel launch, the revision before (prealign, 2c40af6) against the product build,
# interleaved, one PMC pass per process
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for round in 1 2; do for v in prealign base; do
  d="$R/gpurun_out/r04m_write_${v}_$round"
  ( cd /tmp && GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$d" -o run \
      -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-seconds 0 --overlap 0 ) > "$d.log" 2>&1 || { echo "pmc $v failed"; tail -3 "$d.log"; exit 1; }
  python3 - "$d/run_counter_collection.csv" "$v" <<'PY'
import csv, sys
v = {}
for r in csv.DictReader(open(sys.argv[1])):
    if "track_kernel" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE":
        d = int(r["Dispatch_Id"]); v[d] = v.get(d, 0.0) + float(r["Counter_Value"])
w = sorted(v.values())[-4:]
print(sys.argv[2], "WRITE_SIZE per dominant launch (GB):", [round(x * 1024 / 1e9, 3) for x in w], "mean", round(sum(w) / len(w) * 1024 / 1e9, 3))
PY
done; done | tee gpurun_out/r04m_write_ab.txt
