#!/bin/bash
# Round-3 session d: GPU tests of the record buffer + row-parallel lone push; lone latency A/B;
# bulk A/B base vs record buffer; the warm-up / rank sweep of the counter systematic.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=r3d
timeout -k 10 600 python -u -m pytest tests/test_gpu_transport.py tests/test_gpu_probes.py tests/test_gpu_multirank.py::test_gloo_reduction_of_engine_stash tests/test_gpu_safety.py tests/test_gpu_configs.py::test_grid512_photon_by_photon -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop rc=$rc"; exit $rc; }
for v in recbuf cur recbuf cur; do
  GRMONTY_AMD_LIB="$R/cuda-grmonty_amd/ab/libgrmonty_amd_v$v.so" timeout -k 10 200 python -u tools/lone_bench.py 2000 3 > gpurun_out/${T}_lone_$v.log 2>&1 || { tail -5 gpurun_out/${T}_lone_$v.log; exit 1; }
  echo "$v $(grep rep gpurun_out/${T}_lone_$v.log | tail -2 | tr '\n' ' ')"
done
VARIANTS="base recbuf" ROUNDS=2 STEPS=6 TAG=${T}ab bash tools/ab_bench.sh || exit 1
timeout -k 10 500 python -u tools/warmup_sweep2.py --photon-n 1e5 --seeds 16 --warmups 4096,16384,65536,-1 --worlds 1,8 > gpurun_out/${T}_sweep_1e5.log 2>&1 || { tail -5 gpurun_out/${T}_sweep_1e5.log; exit 1; }
cat gpurun_out/${T}_sweep_1e5.log
rm -f gpurun_out/*.dump
exit $rc
