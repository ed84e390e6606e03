#!/bin/bash
# Interleaved bench A/B of variant libraries (cuda-grmonty_amd/ab/libgrmonty_amd_v<name>.so):
#   VARIANTS="base cur" ROUNDS=2 STEPS=6 TAG=x bash tools/ab_bench.sh
# prints per run: value, dominant-launch (bulk) transport rate, dominant ms per pass, pass times
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-ab}
for round in $(seq 1 ${ROUNDS:-2}); do for v in $VARIANTS; do
  o=gpurun_out/${T}_${v}_$round
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 300 python bench.py --steps ${STEPS:-6} --cpu-seconds 0 --overlap 0 > $o.json 2> $o.err || { tail -3 $o.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$o.json').read().strip().splitlines()[-1]); t=d['detail']; r=d['roofline']
print('$v', round(d['value']/1e6,2), 'M/s  bulk', round(r['achieved']/r['flops_per_step']*1e12/1e9,3), 'G steps/s  dominant', round(t['dominant_launch_ms_per_pass'],1), 'ms  passes', t['pass_s']['all'])"
done; done
