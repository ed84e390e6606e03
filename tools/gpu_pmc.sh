#!/bin/bash
# Hardware-counter passes over one diag run (each pass its own process; counters only, no tracing).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd /tmp; export TMPDIR=/tmp
TAG=${PROF_TAG:-x}
SETS=(
  "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM"
  "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32"
  "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH"
  "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
)
if [ -n "$PMC_SETS" ]; then IFS=';' read -r -a SETS <<< "$PMC_SETS"; fi
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  DIAG_REPS=1 timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$i" -o run -- python3 "$R/tools/gpu_diag.py" ${DIAG:-192 1e5} > "$R/gpurun_out/pmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "pmc pass $i [$set] rc=$rc"
  if [ $rc -ne 0 ] && ! grep -qiE "invalid|not found|unsupported|unknown" "$R/gpurun_out/pmc_${TAG}_$i.log"; then exit $rc; fi
done
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out" "$TAG" > "$R/gpurun_out/pmc_${TAG}_summary.txt" 2>&1
cat "$R/gpurun_out/pmc_${TAG}_summary.txt"
exit 0
