#!/bin/bash
# kernel trace of early-worker passes: dispatch start/end of track/early/lone kernels
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
( cd /tmp && DEV_EMIT=1 DIAG_REPS=4 SEED=124 EARLY_STEPS=20000 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/ktrace" -o run -- python3 "$R/tools/gpu_diag.py" 192 1e6 ) > gpurun_out/ktrace.log 2>&1 || { tail -5 gpurun_out/ktrace.log; exit 1; }
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/ktrace/run_kernel_trace.csv")))
t0 = min(int(r["Start_Timestamp"]) for r in rows)
for r in rows:
    n = r["Kernel_Name"]
    if any(k in n for k in ("track_kernel", "early_kernel", "lone_kernel")):
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e6, (int(r["End_Timestamp"]) - t0) / 1e6
        print(f"{n.split('(')[0].split('::')[-1]:14s} grid {r.get('Grid_Size_X', r.get('Grid_Size',''))} wg {r.get('Workgroup_Size_X','')} start {s:9.1f} end {e:9.1f} dur {e - s:8.1f} ms")
PY
grep -E "^rep" gpurun_out/ktrace.log | sed 's/ tracked.*longest life/ ... longest life/' | cut -c1-160
