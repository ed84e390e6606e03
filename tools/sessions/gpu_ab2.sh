#!/bin/bash
# A/B of engine variants: DIAG_REPS passes each at seeds SEED.., interleaved twice (A B A B)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for round in 1 2; do
for v in ${VARIANTS:-base}; do
  DEV_EMIT=1 DIAG_REPS=${DIAG_REPS:-4} SEED=${SEED:-124} GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" \
    timeout -k 10 ${T_AB:-240} python tools/gpu_diag.py ${DIAG:-192 1e6} > gpurun_out/ab_v${v}_$round.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/ab_v${v}_$round.log; exit $rc; }
  python3 - "$v" "gpurun_out/ab_v${v}_$round.log" <<'PY'
import re, sys
v, f = sys.argv[1], sys.argv[2]
t = open(f).read()
walls = [float(x) for x in re.findall(r"wall ([\d.]+)s", t)]
kms = [float(x) for x in re.findall(r"kernel ([\d.]+)ms", t)]
steps = [int(x) for x in re.findall(r"steps (\d+) \(", t)]
bulk = re.findall(r"bulk ([\d.e+]+) Msteps/s", t)
rate = [s / k / 1e3 for s, k in zip(steps, kms)]
print(f"{v:8s} walls {['%.3f' % w for w in walls]} kernel-rate G steps/s {['%.2f' % r for r in rate]} bulk {bulk}")
PY
done
done
