#!/bin/bash
# Multi-rank warm-up barrier where it will run (verdict r04 item 5): emulated 8-rank jobs of the job
# photon_n = 1e6 (strong: 1/8 of the photons per rank, each rank on 1/8 of the CUs, counter blocks
# linked) at the automatic multi-rank barrier (1/16 of the job's history) and at 1/2
# (GRM_OPT_WARMUP_SLACK = 1), interleaved; then each against the six photon_n = 1e6 oracle runs.
R="${GRAFT_REPO_ROOT:-/root/repo}"; cd "$R" && mkdir -p gpurun_out
T=${TAG:-bar}; J=${JOBS:-12}
export GPU_MAX_HW_QUEUES=18
PYTHONPATH=cuda-grmonty_amd python -c "from grmonty_amd.synth_dump import ensure_dump; ensure_dump('gpurun_out/synth192.dump', 192, 192)" || exit 1
for r in 1 2; do
  for s in auto 1; do
    o=""; [ $s = 1 ] && o="--opt 12=1"
    timeout -k 10 300 python -u tests/multirank_emu.py gpurun_out/synth192.dump 8 $J gpurun_out/${T}_slack${s}_$r.json --shared \
      --photon-n 1e6 --seed0 $((1000 + 100 * r)) $o > gpurun_out/${T}_slack${s}_$r.log 2>&1 || { echo "emu $s $r failed"; tail -3 gpurun_out/${T}_slack${s}_$r.log; exit 1; }
  done
done
for s in auto 1; do
  python tools/emu_vs_oracle.py gpurun_out/${T}_slack${s}_1.json gpurun_out/${T}_slack${s}_2.json --photon-n 1e6 --pool
done
