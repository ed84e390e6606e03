#!/bin/bash
# round-4 combined session: the N-rank warm-up test (emulated ranks), then the full GPU suite, smoke
# and the measurement session (gpu_final4.sh, TAG r04t)
export TMPDIR=/tmp
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
bash tools/gpu_r04s.sh || exit 1
TAG=r04t bash tools/gpu_final4.sh
