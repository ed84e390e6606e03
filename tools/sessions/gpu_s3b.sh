#!/bin/bash
# Round-3 session s3b: where the lone geometry wave's time goes.
#  1 geom_only: the engine's lone_geometry with a trivial consumer / a busy neighbour (current tree,
#    and with -DGRM_X_NO_GEO_VGPR: push parameters spilled to VGPR lanes, v_readlane per use)
#  2 long-photon chain A/B (631 k-step photon, frozen bias): base / vg (parameters in VGPRs) / vgq (+ quad push)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
M="$R/tools/microbench"; FL="--offload-arch=gfx950 -O3 -std=c++17 -mllvm -disable-machine-licm -Wno-unused-value -Wno-unused-result -I$R/cuda-grmonty_amd/csrc"
LK="-L/opt/rocm/lib -lrccl -L$R/cuda-grmonty_amd -lgrmonty_amd -Wl,-rpath,$R/cuda-grmonty_amd"
/opt/rocm/bin/hipcc $FL $M/geom_only.hip -DGRM_X_NO_GEO_QUAD -o /tmp/geo_vg $LK && /opt/rocm/bin/hipcc $FL -DGRM_X_NO_GEO_VGPR -DGRM_X_NO_GEO_QUAD $M/geom_only.hip -o /tmp/geo_base $LK || exit 1
/opt/rocm/bin/hipcc $FL $M/geom_only.hip -o /tmp/geo_vgq $LK || exit 1
for v in base vg vgq; do echo "== geom_only $v"; timeout -k 10 60 /tmp/geo_$v || exit 1; done
for round in 1 2; do for v in base vg vgq; do
  echo "== long photon $v ($round)"
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 1 || exit 1
done; done
