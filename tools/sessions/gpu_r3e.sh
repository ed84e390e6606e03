#!/bin/bash
# Round-3 session e: job-wide bias counters (linked / IPC peer counter blocks): emulated-rank parity,
# IPC test, stash test; the headline parity; smoke; a default bench line.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3e
timeout -k 10 900 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_parity_192.py -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop rc=$rc"; exit $rc; }
grep -E "ranks (recorded|scattered|steps|luminosity)|^(recorded|scattered|steps|luminosity) " gpurun_out/${T}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
for v in timing vrecbuf vcur; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_$v.so" timeout -k 10 200 python -u tools/long_photon_bench.py 2 > gpurun_out/${T}_long_$v.log 2>&1 || { tail -5 gpurun_out/${T}_long_$v.log; exit 1; }
  echo "== $v"; grep -E "rep|wave" gpurun_out/${T}_long_$v.log
done
rm -f gpurun_out/*.dump
exit $rc
