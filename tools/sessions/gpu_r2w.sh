#!/bin/bash
# refill / child-batch sweep on the current build (diag, 192^2 photon_n=1e6, seeds 123-124)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for cfg in "8 2" "16 2" "24 2" "8 4" "16 4" "4 2" "8 2"; do
  set -- $cfg
  DEV_EMIT=1 DIAG_REPS=2 SEED=123 CHILD_MIN=$1 REFILL_MIN=$2 timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > gpurun_out/sweep_$1_$2.log 2>&1 || exit 1
  python3 - "$1" "$2" gpurun_out/sweep_$1_$2.log <<'PY'
import re, sys
t = open(sys.argv[3]).read()
k = [float(x) for x in re.findall(r"kernel ([\d.]+)ms", t)]
st = [int(x) for x in re.findall(r"steps (\d+) \(", t)]
print(f"child_min {sys.argv[1]:>3} refill_min {sys.argv[2]}: kernel ms {k} G steps/s {[round(s / m / 1e6, 3) for s, m in zip(st, k)]}")
PY
done
