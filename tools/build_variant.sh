#!/bin/bash
# Build the working tree's kernels with extra engine flags as an A/B variant:
#   [SCHED=none|max-ilp|...] VFLAGS="-DX=1" tools/build_variant.sh <name>  ->  cuda-grmonty_amd/ab/libgrmonty_amd_v<name>.so
#   (VFLAGS containing -DGRM_WITH_SPLIT also builds csrc/grm_split.hip, the role-split bulk kernel)
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
name=$1
D="$R/cuda-grmonty_amd/build/var_$name"; mkdir -p "$D" "$R/cuda-grmonty_amd/ab"
make -s -C "$R/cuda-grmonty_amd" build/grm_host.o build/grm_probe.o build/grm_emit.o build/grm_tables.o
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -mllvm -disable-machine-licm"
SCHED=${SCHED:-none}; SF=""; [ "$SCHED" = none ] || SF="-mllvm -amdgpu-sched-strategy=$SCHED"
/opt/rocm/bin/hipcc $FL $SF $VFLAGS -c "$R/cuda-grmonty_amd/csrc/grm_engine.hip" -o "$D/grm_engine.o"
/opt/rocm/bin/hipcc ${FL/-mllvm -disable-machine-licm/} -mllvm -amdgpu-sched-strategy=max-ilp $VFLAGS -c "$R/cuda-grmonty_amd/csrc/grm_lone.hip" -o "$D/grm_lone.o"
SPLIT_O=""
case "$VFLAGS" in *GRM_WITH_SPLIT*)  # the role-split bulk kernel (not in the product)
  /opt/rocm/bin/hipcc $FL $VFLAGS -c "$R/cuda-grmonty_amd/csrc/grm_split.hip" -o "$D/grm_split.o"; SPLIT_O="$D/grm_split.o";;
esac
B="$R/cuda-grmonty_amd/build"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$name.so" \
  "$D/grm_engine.o" "$D/grm_lone.o" $SPLIT_O $B/grm_probe.o $B/grm_emit.o $B/grm_tables.o $B/grm_host.o -L/opt/rocm/lib -lrccl -lpthread
echo "built ab/libgrmonty_amd_v$name.so ($VFLAGS)"
