#!/bin/bash
# The early worker's own children (GRM_OPT_EARLY_CHILDREN): photon-by-photon parity of the early paths,
# the long-photon chain (us/step) of the product against HEAD's build and the inlined set-up variant,
# and frozen-bias replays of the tail passes (seeds 125, 126) with the option on and off.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-kids}
PYTHONPATH=cuda-grmonty_amd python -c "from grmonty_amd.synth_dump import ensure_dump; ensure_dump('gpurun_out/synth192.dump', 192, 192)" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_transport.py -x -v -s --timeout 150 --timeout-method thread \
  -k "photon_by_photon" > gpurun_out/${T}_pbp.log 2>&1 || { echo "pbp failed"; tail -30 gpurun_out/${T}_pbp.log; rm -f gpurun_out/*.dump; exit 1; }
grep -E "PASSED|FAILED|early worker:|matching" gpurun_out/${T}_pbp.log
for lib in product vhead vinl product; do
  L=""; [ $lib = product ] || L="cuda-grmonty_amd/ab/libgrmonty_amd_$lib.so"
  GRMONTY_AMD_LIB=$L EARLY=1 timeout -k 10 120 python -u tools/long_photon_bench.py 3 > gpurun_out/${T}_chain_$lib.log 2>&1 || { echo "chain $lib failed"; tail -5 gpurun_out/${T}_chain_$lib.log; rm -f gpurun_out/*.dump; exit 1; }
  echo "== $lib"; tail -3 gpurun_out/${T}_chain_$lib.log
done
cp profiles/r05_tail_snapshots.json gpurun_out/tail_snap.json
for r in 1 2; do
  for k in 1 0; do
    timeout -k 10 200 python -u tools/tail_replay.py --seeds 125 126 --snap gpurun_out/tail_snap.json --opt 29=$k > gpurun_out/${T}_tail_k${k}_$r.log 2>&1 || { echo "tail $k failed"; tail -5 gpurun_out/${T}_tail_k${k}_$r.log; rm -f gpurun_out/*.dump; exit 1; }
    echo "== kids=$k rep $r"; cat gpurun_out/${T}_tail_k${k}_$r.log | grep -v "^\s*$" | tail -4
  done
done
rm -f gpurun_out/*.dump
