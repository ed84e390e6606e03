#!/bin/bash
# default bench run (+ optional rocprof kernel-trace/stats of a short bench)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-x}
timeout -k 10 900 python -u bench.py $BARGS > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rc=$?; python3 -c "
import json,sys; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1])
print('value',d['value'],'ms/pass',d['ms_per_step']); print('passes',d['detail']['pass_s']['all']); print('roofline',{k:d['roofline'][k] for k in ('achieved','frac','traffic')}); print('longest life',d['detail']['longest_photon_life_steps'], 'overlapped', d['detail'].get('overlapped'))
" ; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_bench.err; exit $rc; }
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  ( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_prof" -o run -- python3 $R/bench.py --steps 10 --warmup 1 --cpu-seconds 0 --overlap 0 ) > gpurun_out/${T}_prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; cat gpurun_out/${T}_prof/run_kernel_stats.csv | cut -c1-150
fi
exit $rc
