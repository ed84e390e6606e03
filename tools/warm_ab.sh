#!/bin/bash
# Interleaved A/B of the warm-up phase (tools/pass_phases.py, PASSES passes of photon_n = 1e6 each) over
# variant libraries cuda-grmonty_amd/ab/libgrmonty_amd_v<name>.so:
#   VARIANTS="base x" ROUNDS=2 PASSES=6 TAG=t bash tools/warm_ab.sh
# prints per run: mean warm-up end, mean dominant launch, mean recorded per pass.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-warm}
for round in $(seq 1 ${ROUNDS:-2}); do for v in $VARIANTS; do
  o=gpurun_out/${T}_${v}_$round.log
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 300 python tools/pass_phases.py ${PASSES:-6} > $o 2>&1 || { tail -3 $o; exit 1; }
  python3 - "$o" "$v" <<'PY'
import re, sys
t = open(sys.argv[1]).read()
w = [float(x) for x in re.findall(r"warm-up ends ([0-9.]+) ms", t)]
d = [float(x) for x in re.findall(r"dominant ([0-9.]+) ms", t)]
r = [int(x) for x in re.findall(r"recorded (\d+)", t)]
print(f"{sys.argv[2]:8s} warm-up end {sum(w) / len(w):.1f} ms ({' '.join(f'{x:.1f}' for x in w)})  dominant "
      f"{sum(d) / len(d):.1f} ms  recorded/pass {sum(r) / len(r) / 1e6:.3f} M")
PY
done; done
