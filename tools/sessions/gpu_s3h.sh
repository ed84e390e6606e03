#!/bin/bash
# Round-3 session s3h: long-photon chain, connection rows to the quad lanes: selected from four (vq1,
# current) vs two blocks of two rows + one select level (vq2)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for round in 1 2 3; do for v in q1 q2; do echo "== v$v ($round)"
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
done; done
