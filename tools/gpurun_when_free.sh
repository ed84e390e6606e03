#!/bin/bash
# Run one gpurun command, waiting for a free box: retries ONLY while gpurun reports that no box or
# slot was free (status=transient: nothing ran, nothing was charged); any other outcome -- the
# command ran, failed, timed out or was refused -- is returned as is.
#   tools/gpurun_when_free.sh TIMEOUT_S LOG 'command'
T=$1; LOG=$2; CMD=$3
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -q "status=transient" "$LOG"; then sleep 60; continue; fi
  exit $rc
done
exit 3
