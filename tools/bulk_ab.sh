#!/bin/bash
# Interleaved A/B of the bulk rate (transport steps per ms of the dominant launch, tools/pass_phases.py,
# PASSES passes of photon_n = 1e6 each) over variant libraries cuda-grmonty_amd/ab/libgrmonty_amd_v<name>.so:
#   VARIANTS="base x" ROUNDS=3 PASSES=6 TAG=t bash tools/bulk_ab.sh
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-bulk}
for round in $(seq 1 ${ROUNDS:-3}); do for v in $VARIANTS; do
  o=gpurun_out/${T}_${v}_$round.log
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 300 python tools/pass_phases.py ${PASSES:-6} > $o 2>&1 || { tail -3 $o; exit 1; }
  python3 - "$o" "$v" <<'PY'
import re, sys
t = open(sys.argv[1]).read()
d = [float(x) for x in re.findall(r"dominant ([0-9.]+) ms", t)]
st = [float(x) for x in re.findall(r"steps ([0-9.e+]+);", t)]
w = [float(x) for x in re.findall(r"warm-up ends ([0-9.]+) ms", t)]
bulk = [s / ((dd - ww) * 1e-3) / 1e9 for s, dd, ww in zip(st, d, w)]
print(f"{sys.argv[2]:6s} G steps/s over the launch {sum(st) / sum(d) * 1e3 / 1e9:.3f}  after the warm-up "
      f"{sum(bulk) / len(bulk):.3f} ({' '.join(f'{x:.2f}' for x in bulk)})  dominant {sum(d) / len(d):.1f} ms")
PY
done; done
