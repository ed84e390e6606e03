#!/bin/bash
# Round-3 session s3g: which waves take the warm-up's admission batches (GRM_OPT_WARMUP_BLOCKS = 20,
# GRM_OPT_WARMUP_WAVES = 21, with the spread GRM_OPT_WARMUP_SPREAD = 19) at photon_n = 1e6, 8 passes
# each: warm-up end, dominant launch, recorded per pass
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for v in "" "20=256,21=4,19=2" "20=256,21=4,19=1" "20=256,21=8,19=1" "20=128,21=4,19=4" "20=256,21=4,19=4"; do
  t="${v:-default}"; t="${t//=/_}"; t="${t//,/-}"
  GRM_BENCH_OPTS="$v" timeout -k 10 200 python -u tools/pass_phases.py 8 1e6 > gpurun_out/s3g_warm_$t.log 2>&1 || { tail -5 gpurun_out/s3g_warm_$t.log; exit 1; }
  echo "== $t"; grep -v admissions gpurun_out/s3g_warm_$t.log | sed -E 's/, pool drained.*recorded/ recorded/'
done
rm -f gpurun_out/*.dump
