#!/bin/bash
# round-end measurement set on the final tree (r02s): GPU tests, smoke, PMC traffic, bench, rocprof, PMC mix
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
TAG=r02s bash tools/gpu_final2.sh
