#!/bin/bash
# One GPU session. Each GPU step has its own time limit; a crash-type exit status
# (anything but 0, or 1/5 from pytest = test failures / none collected) stops the session.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || { echo "stopping after rc=$1"; exit "$1"; }; }
if [ -n "$TESTS" ]; then
  timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -q ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -6 gpurun_out/pytest_gpu.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 5 ] || { echo "stopping after rc=$rc"; exit $rc; }
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; ok $rc
fi
if [ -n "$DIAG" ]; then
  timeout -k 10 ${T_DIAG:-300} python tools/gpu_diag.py $DIAG > gpurun_out/diag.log 2>&1
  rc=$?; echo "diag rc=$rc"; tail -8 gpurun_out/diag.log; ok $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 ${T_BENCH:-600} python bench.py $BENCH > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log; ok $rc
fi
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  ( cd /tmp && timeout -k 10 ${T_PROF:-600} rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/prof_${PROF_TAG:-x}" -o run -- python3 "$R/bench.py" $PROF ) > gpurun_out/prof_${PROF_TAG:-x}.log 2>&1
  rc=$?; echo "prof rc=$rc"; tail -3 gpurun_out/prof_${PROF_TAG:-x}.log; ok $rc
fi
if [ -n "$PMC" ]; then
  export TMPDIR=/tmp
  ( cd /tmp && timeout -k 10 ${T_PROF:-600} rocprofv3 --pmc $PMC_COUNTERS --output-format csv \
      -d "$R/gpurun_out/pmc_${PROF_TAG:-x}" -o run -- python3 "$R/bench.py" $PMC ) > gpurun_out/pmc_${PROF_TAG:-x}.log 2>&1
  rc=$?; echo "pmc rc=$rc"; tail -3 gpurun_out/pmc_${PROF_TAG:-x}.log; ok $rc
fi
exit 0
