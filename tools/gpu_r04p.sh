#!/bin/bash
# round-4: the N-rank counter offset -- ranks run one after another (seq), early worker off (15=0);
# then a GRM_TIMING diagnostic of the bulk (per-region wave cycles) on the product configuration
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 700 python -u tools/emu_sweep.py gpurun_out/r04p_emu.jsonl "w8_ne:8:48:shared:15=0" "w1_ne:1:48:15=0" "w8_seq:8:24:shared:seq" > gpurun_out/r04p_emu.log 2>&1
rc=$?; cat gpurun_out/r04p_emu.log; [ $rc -eq 0 ] || exit $rc
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_timing.so" DEV_EMIT=1 DIAG_REPS=2 timeout -k 10 200 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/r04p_timing_diag.log 2>&1
rc=$?; tail -8 gpurun_out/r04p_timing_diag.log | cut -c1-600; exit $rc
