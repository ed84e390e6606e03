#!/bin/bash
# Interleaved bench A/B of engine OPTIONS (GRM_BENCH_OPTS, grmonty_amd.OPT_* = value, comma-separated):
#   OPTS="base 14=512 8=2048" ROUNDS=2 STEPS=6 TAG=x bash tools/ab_opts.sh    ("base" = defaults)
# prints per run: value, bulk rate, dominant-launch ms per pass, recorded per pass, median pass
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-abo}
for round in $(seq 1 ${ROUNDS:-2}); do for o in $OPTS; do
  f=gpurun_out/${T}_$(echo $o | tr '=,' '__')_$round
  if [ "$o" = base ]; then ov=""; else ov="$o"; fi
  GRM_BENCH_OPTS="$ov" timeout -k 10 300 python bench.py --steps ${STEPS:-6} --cpu-seconds 0 --overlap 0 > $f.json 2> $f.err || { tail -3 $f.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); t=d['detail']; r=d['roofline']
print('$o', round(d['value']/1e6,2), 'M/s  bulk', round(r['achieved']/r['flops_per_step']*1e12/1e9,3), 'G steps/s  dominant', round(t['dominant_launch_ms_per_pass'],1), 'ms  recorded/pass', t['recorded_per_pass'], ' median pass', round(t['pass_s']['median'],4))"
done; done
