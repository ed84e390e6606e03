#!/bin/bash
# one GPU session: tests then diagnostics; stops at the first crash-type exit status
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -q -x ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then echo "stopping after rc=$rc"; exit $rc; fi
if [ -n "$DIAG" ]; then
  timeout -k 10 ${T_DIAG:-300} python tools/gpu_diag.py $DIAG > gpurun_out/diag.log 2>&1
  rc=$?; echo "diag rc=$rc"; tail -8 gpurun_out/diag.log
fi
exit $rc
