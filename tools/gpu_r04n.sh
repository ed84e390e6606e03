#!/bin/bash
# round-4: which part of the emulated N-rank job moves the live-bias counters (tools/emu_sweep.py)
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -u tools/emu_sweep.py gpurun_out/r04n_emu_sweep.jsonl \
  "w1:1:48" "w8:8:48:shared" "w8_r192:8:48:shared:20=192" "w8_wu0:8:48:shared:8=0" "w2:2:48:shared" "w1_r192:1:48:20=192" \
  > gpurun_out/r04n_emu_sweep.log 2>&1
rc=$?; cat gpurun_out/r04n_emu_sweep.log | tail -12; exit $rc
