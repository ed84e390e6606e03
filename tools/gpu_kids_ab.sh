#!/bin/bash
# Children tracked by the two-wave pairs themselves (GRM_OPT_EARLY_CHILDREN): photon-by-photon parity
# of the pair paths, the long-photon chain (us/step) of the product against HEAD's build (vhead) on the
# early worker and in the lone kernel, emulated 4-rank jobs (96 each) with the option on and off, and
# frozen-bias replays of the tail passes (seeds 125, 126) on and off.  STEPS selects (default all).
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-kids}
S=" ${STEPS:-pbp chain mr tail} "
has() { [[ "$S" == *" $1 "* ]]; }
fail() { echo "$1 failed"; tail -30 "$2"; rm -f gpurun_out/*.dump; exit 1; }
export GPU_MAX_HW_QUEUES=18
PYTHONPATH=cuda-grmonty_amd python -c "from grmonty_amd.synth_dump import ensure_dump; ensure_dump('gpurun_out/synth192.dump', 192, 192)" || exit 1
if has pbp; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_transport.py -x -v -s --timeout 150 --timeout-method thread \
    -k "photon_by_photon" > gpurun_out/${T}_pbp.log 2>&1 || fail pbp gpurun_out/${T}_pbp.log
  grep -E "PASSED|FAILED|early worker:|lone kernel:|matching" gpurun_out/${T}_pbp.log
fi
if has chain; then
  for lib in product vhead; do
    for mode in 1 0; do
      L=""; [ $lib = product ] || L="cuda-grmonty_amd/ab/libgrmonty_amd_$lib.so"
      GRMONTY_AMD_LIB=$L EARLY=$mode timeout -k 10 120 python -u tools/long_photon_bench.py 3 > gpurun_out/${T}_chain_${lib}_e$mode.log 2>&1 || fail "chain $lib" gpurun_out/${T}_chain_${lib}_e$mode.log
      echo "== $lib early=$mode"; tail -3 gpurun_out/${T}_chain_${lib}_e$mode.log
    done
  done
fi
if has mr; then
  for k in 1 0; do
    timeout -k 10 400 python -u tests/multirank_emu.py gpurun_out/synth192.dump 4 96 gpurun_out/${T}_mr4_k$k.json --shared --seed0 300 --opt 29=$k \
      > gpurun_out/${T}_mr4_k$k.log 2>&1 || fail "mr $k" gpurun_out/${T}_mr4_k$k.log
    python tools/emu_vs_oracle.py gpurun_out/${T}_mr4_k$k.json --photon-n 1e5 --pool > gpurun_out/${T}_mr4_k${k}_summary.txt 2>&1 || exit 1
    echo "== 4 ranks, children on pairs $k"; cat gpurun_out/${T}_mr4_k${k}_summary.txt
  done
fi
if has tail; then
  cp profiles/r05_tail_snapshots.json gpurun_out/tail_snap.json
  for r in 1 2; do
    for k in 1 0; do
      timeout -k 10 200 python -u tools/tail_replay.py --seeds 125 126 --snap gpurun_out/tail_snap.json --opt 29=$k > gpurun_out/${T}_tail_k${k}_$r.log 2>&1 || fail "tail $k" gpurun_out/${T}_tail_k${k}_$r.log
      echo "== kids=$k rep $r"; grep -v "^\s*$" gpurun_out/${T}_tail_k${k}_$r.log | tail -2 | cut -c1-400
    done
  done
fi
rm -f gpurun_out/*.dump
