#!/bin/bash
# Round-3 session s3c: quad push in the lone geometry wave (default now) -- photon-by-photon tests of
# every device path; the geometry wave alone (geom_only); trip-time attribution of the bulk kernel
# (GRM_TIMING build) at the bench's configuration.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=s3c
: timeout -k 10 600 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_probes.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
# pytest ran in the first s3c call: 18 passed
M="$R/tools/microbench"; FL="--offload-arch=gfx950 -O3 -std=c++17 -mllvm -disable-machine-licm -Wno-unused-value -Wno-unused-result -I$R/cuda-grmonty_amd/csrc"
LK="-L/opt/rocm/lib -lrccl -L$R/cuda-grmonty_amd -lgrmonty_amd -Wl,-rpath,$R/cuda-grmonty_amd"
/opt/rocm/bin/hipcc $FL $M/geom_only.hip -o /tmp/geo_q $LK && /opt/rocm/bin/hipcc $FL -DGRM_X_NO_GEO_QUAD $M/geom_only.hip -o /tmp/geo_vg $LK || exit 1
for v in vg q; do echo "== geom_only $v"; timeout -k 10 60 /tmp/geo_$v || exit 1; done
echo "== bulk trip attribution (GRM_TIMING build), 192^2 photon_n=1e6"
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_timing.so" timeout -k 10 300 python -u tools/gpu_diag.py 192 1e6 > gpurun_out/${T}_timing.log 2>&1 || { tail -5 gpurun_out/${T}_timing.log; exit 1; }
cat gpurun_out/${T}_timing.log | tail -12
echo "== long photon, current tree (quad push and quad halving walk)"
timeout -k 10 200 python -u tools/long_photon_bench.py 2 || exit 1
echo "== long photon, GRM_TIMING build"
GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_timing.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
