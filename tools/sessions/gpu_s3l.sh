#!/bin/bash
# Round-3 session s3l: exp polynomial through the three-operand VGPR fma in the lone unit (vnew) vs
# plain fma (vold): long-photon chain
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
for round in 1 2 3; do for v in old new; do echo "== v$v ($round)"
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
done; done
