#!/bin/bash
# A/B of named engine builds (cuda-grmonty_amd/variants/libgrmonty_amd_v<name>.so) on one box:
# device emission + transport of photon_n=1e6 on the 192^2 synthetic dump, DIAG_REPS passes each.
# Bulk speed = median wave exit (the straggler tail is excluded).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R"; mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  DEV_EMIT=1 DIAG_REPS=${DIAG_REPS:-3} GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/variants/libgrmonty_amd_v$v.so" \
    timeout -k 10 ${T_AB:-240} python tools/gpu_diag.py ${DIAG:-192 1e6} > gpurun_out/ab_v$v.log 2>&1
  rc=$?; echo "== $v rc=$rc"
  grep -E "^rep|waves|timing|stuck|^ *\[|^\[\[" gpurun_out/ab_v$v.log | sed -E 's/children.*rate/... rate/; s/\| longest launch[^|]*steps\) /| /'
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
done
