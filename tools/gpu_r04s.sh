#!/bin/bash
# round-4: N-rank offset -- batches sized from the job's history, the job's warm-up ends together
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
timeout -k 10 800 python -u tools/emu_sweep.py gpurun_out/r04s_emu.jsonl "w8:8:48:shared" "w4:4:48:shared" "w2:2:48:shared" "w1:1:48" > gpurun_out/r04s_emu.log 2>&1
rc=$?; cat gpurun_out/r04s_emu.log; exit $rc
