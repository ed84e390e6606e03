#!/bin/bash
# round-4: N-rank offset -- the warm-up: larger, stricter, unspread
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 800 python -u tools/emu_sweep.py gpurun_out/r04r_emu.jsonl "w8_wu16k:8:48:shared:8=16384" "w8_sl4:8:48:shared:12=4" "w8_sp0:8:48:shared:19=0" "w1_wu0:1:48:8=0" > gpurun_out/r04r_emu.log 2>&1
rc=$?; cat gpurun_out/r04r_emu.log; exit $rc
