#!/bin/bash
# Build the transport kernel of an earlier git revision as an A/B variant:
#   tools/build_rev.sh <rev> <name>  ->  cuda-grmonty_amd/ab/libgrmonty_amd_v<name>.so
# (kernel sources of <rev>, current host objects; only for revisions with the same C ABI)
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
rev=$1; name=$2
D="$R/cuda-grmonty_amd/build/rev_$name"
rm -rf "$D"; mkdir -p "$D/csrc" "$D/include"
for f in grm_engine.hip grm_lone.hip grm_split.hip grm_probe.hip grm_emit.hip grm_tables.hip grm_device.h grm_emit.h; do
  git -C "$R" show "$rev:cuda-grmonty_amd/csrc/$f" > "$D/csrc/$f" 2>/dev/null || rm -f "$D/csrc/$f"
done
git -C "$R" show "$rev:include/grmonty_amd.h" > "$D/include/grmonty_amd.h"
git -C "$R" show "$rev:include/grmonty_amd_debug.h" > "$D/include/grmonty_amd_debug.h" 2>/dev/null || rm -f "$D/include/grmonty_amd_debug.h"
sed -i 's|"../../include/grmonty_amd|"../include/grmonty_amd|' "$D/csrc/"*.h "$D/csrc/"*.hip
make -s -C "$R/cuda-grmonty_amd" build/grm_host.o
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value -mllvm -disable-machine-licm"
SF=""; [ -n "$SCHED" ] && SF="-mllvm -amdgpu-sched-strategy=$SCHED"  # revisions before 58fc566 were built with SCHED=iterative-ilp
/opt/rocm/bin/hipcc $FL $SF $VFLAGS -c "$D/csrc/grm_engine.hip" -o "$D/grm_engine.o" &
objs="$D/grm_engine.o"
if [ -f "$D/csrc/grm_lone.hip" ]; then
  /opt/rocm/bin/hipcc ${FL/-mllvm -disable-machine-licm/} -mllvm -amdgpu-sched-strategy=max-ilp $VFLAGS -c "$D/csrc/grm_lone.hip" -o "$D/grm_lone.o" &
  objs="$objs $D/grm_lone.o"
fi
if [ -f "$D/csrc/grm_split.hip" ]; then
  /opt/rocm/bin/hipcc $FL $VFLAGS -c "$D/csrc/grm_split.hip" -o "$D/grm_split.o" &
  objs="$objs $D/grm_split.o"
fi
for f in grm_probe grm_emit grm_tables; do
  [ -f "$D/csrc/$f.hip" ] || continue
  /opt/rocm/bin/hipcc $FL -c "$D/csrc/$f.hip" -o "$D/$f.o" &
  objs="$objs $D/$f.o"
done
wait
mkdir -p "$R/cuda-grmonty_amd/ab"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$name.so" \
  $objs "$R/cuda-grmonty_amd/build/grm_host.o" -L/opt/rocm/lib -lrccl -lpthread
echo "built ab/libgrmonty_amd_v$name.so from $rev"
