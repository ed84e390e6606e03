#!/bin/bash
# split_kernel configurations on the 192^2, photon_n = 1e6 diag pass (timing build): CFGS = "mode:gthr:thr:spin ..."
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-sw}
for c in $CFGS; do
  IFS=: read -r m g t s b <<< "$c"
  b=${b:-1}
  f=gpurun_out/${T}_${m}_${g}_${t}_${s}_$b.log
  GRMONTY_AMD_LIB=$R/cuda-grmonty_amd/ab/libgrmonty_amd_timing.so SPLIT=$m SPLIT_GTHR=$g SPLIT_THR=$t SPLIT_SPIN=$s SPLIT_BATCH=$b DIAG_REPS=2 DEV_EMIT=1 \
    timeout -k 10 200 python tools/gpu_diag.py 192 1e6 > $f 2>&1 || { echo "$c failed"; tail -3 $f; exit 1; }
  echo "== mode $m gthr $g thr $t spin $s batch $b: $(grep -E '^rep 1' $f | sed -E 's/.*\(([0-9.e+]+) Msteps.*/\1 Msteps\/s/')"
  grep -E "split " $f | tail -2
done
