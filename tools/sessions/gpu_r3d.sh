#!/bin/bash
# bench A/B: new lone interaction wave vs HEAD
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out




for round in 1 2; do for v in new base; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" timeout -k 10 300 python bench.py --cpu-seconds 0 --overlap 0 > gpurun_out/benchab_${v}_$round.json 2> gpurun_out/benchab_${v}_$round.err || { tail -3 gpurun_out/benchab_${v}_$round.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/benchab_${v}_$round.json').read().strip().splitlines()[-1])
print('$v', round(d['value']/1e6,2), 'M/s passes', d['detail']['pass_s']['all'], 'longest', d['detail']['longest_photon_life_steps'])"
done; done
rm -f gpurun_out/*.dump
