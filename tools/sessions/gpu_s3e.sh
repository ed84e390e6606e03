#!/bin/bash
# Round-3 session s3e: long-photon chain with machine LICM on: quad push with selected rows (current),
# divergent-block rows (vq0), plain push (vnq)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for round in 1 2; do
  echo "== current ($round)"; timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
  for v in q0 nq; do echo "== v$v ($round)"
    GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
  done
done
