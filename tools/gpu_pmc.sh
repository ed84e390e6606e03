#!/bin/bash
# hardware-counter passes over one diag run (each pass its own process; counters only, no tracing)
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd /tmp; export TMPDIR=/tmp
TAG=${PROF_TAG:-x}
timeout -k 10 120 rocprofv3 -L > "$R/gpurun_out/counters_list.txt" 2>&1; echo "list rc=$?"
i=0
for set in "${PMC_SETS[@]:-SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES}"; do :; done
for set in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU" "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_LDS"; do
  i=$((i+1))
  DIAG_REPS=1 timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d "$R/gpurun_out/pmc_${TAG}_$i" -o run -- python3 "$R/tools/gpu_diag.py" ${DIAG:-192 1e5} > "$R/gpurun_out/pmc_${TAG}_$i.log" 2>&1
  rc=$?; echo "pmc pass $i [$set] rc=$rc"; tail -2 "$R/gpurun_out/pmc_${TAG}_$i.log"
  if [ $rc -ne 0 ] && ! grep -qiE "invalid|not found|unsupported|unknown" "$R/gpurun_out/pmc_${TAG}_$i.log"; then exit $rc; fi
done
exit 0
