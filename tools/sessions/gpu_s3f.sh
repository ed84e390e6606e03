#!/bin/bash
# Round-3 session s3f: bulk -- transport steps counted per wave by ballot (no per-step LDS RMW of a
# lane counter): interleaved bench A/B against the previous build (vprev)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
cp cuda-grmonty_amd/libgrmonty_amd.so cuda-grmonty_amd/ab/libgrmonty_amd_vcur.so
VARIANTS="prev cur" ROUNDS=3 STEPS=6 TAG=s3f bash tools/ab_bench.sh
