#!/bin/bash
# PC sampling of the bulk transport (rocprofv3, beta): which instructions the waves of track_kernel
# sit at.  Lists the box's PC-sampling configurations first, then samples one photon_n = 1e6 pass of
# tools/gpu_diag.py with the first method the device offers (stochastic preferred: it also records the
# stall reason).  TAG names gpurun_out/<TAG>_pcs*.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-pcs}
( cd /tmp && timeout -s KILL 60 rocprofv3 -L ) > gpurun_out/${T}_list.txt 2>&1
if grep -qi stochastic gpurun_out/${T}_list.txt; then M="--pc-sampling-method stochastic --pc-sampling-unit cycles --pc-sampling-interval ${CYC:-1048576}"
elif grep -qi host_trap gpurun_out/${T}_list.txt; then M="--pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval ${US:-100}"
else echo "no PC sampling on this device"; grep -i -m5 sampl gpurun_out/${T}_list.txt; exit 0; fi
echo "pc sampling: $M"
( cd /tmp && DIAG_REPS=1 DEV_EMIT=1 timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled $M --output-format csv \
    -d "$R/gpurun_out/${T}_pcs" -o run -- python3 "$R/tools/gpu_diag.py" 192 1e6 ) > gpurun_out/${T}_pcs.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pcs.log; ls -la gpurun_out/${T}_pcs 2>/dev/null | head
exit $rc
