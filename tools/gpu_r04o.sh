#!/bin/bash
# round-4: the N-rank counter offset -- all ranks counting into ONE block (sb), bias refresh every 8
# trips instead of 64 (rf8), against the product build
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
A="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v"
GRMONTY_AMD_LIB=${A}sb.so timeout -k 10 400 python -u tools/emu_sweep.py gpurun_out/r04o_emu.jsonl "w8_sb:8:48:shared" "w2_sb:2:48:shared" > gpurun_out/r04o_emu.log 2>&1 || { tail -5 gpurun_out/r04o_emu.log; exit 1; }
GRMONTY_AMD_LIB=${A}rf8.so timeout -k 10 400 python -u tools/emu_sweep.py gpurun_out/r04o_emu.jsonl "w8_rf8:8:48:shared" "w1_rf8:1:48" >> gpurun_out/r04o_emu.log 2>&1 || { tail -5 gpurun_out/r04o_emu.log; exit 1; }
timeout -k 10 400 python -u tools/emu_sweep.py gpurun_out/r04o_emu.jsonl "w8:8:48:shared" "w4:4:48:shared" >> gpurun_out/r04o_emu.log 2>&1
rc=$?; cat gpurun_out/r04o_emu.log; exit $rc
