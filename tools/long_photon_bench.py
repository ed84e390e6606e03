"""Deterministic long-photon latency probe of the lone / early pipelines: primary 13,288,390 of the
seed-126 pass (192^2, photon_n = 1e6) with the bias frozen at that pass's live counters has a
grandchild that lives ~634 k steps (profiles/r02u_long_photon_replay.txt, a bound orbit at r ~ 9 M;
the CPU oracle replays the same family).  Tracking that primary alone puts the grandchild on the
serial chain of a two-wave pair; prints its steps and the pair's time per step.  With a GRM_TIMING
build (GRMONTY_AMD_LIB=.../ab/libgrmonty_amd_timing.so) also the geometry / interaction wave split.
Usage: python tools/long_photon_bench.py [reps]
EARLY=1: the chain on the early worker instead (lone hand-over off, a two-workgroup grid so that the
worker is launched, which takes the grandchild at its 5,000th step)."""
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

SEED, ROOT = 126, 13288390
SNAP = dict(scatt=26712171, rec=18308001, maxtau=0.002517)
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=1e6).init(0)
ph = m.emit(seed=SEED)
e = G.Engine(m, 0)
e.set_option(G.OPT_BIAS_MODE, 1)
e.set_option(G.OPT_FROZEN_SCATT, SNAP["scatt"])
e.set_option(G.OPT_FROZEN_REC, SNAP["rec"])
e.set_option(G.OPT_FROZEN_MAXTAU, struct.unpack("<q", struct.pack("<d", SNAP["maxtau"]))[0])
EARLY = os.environ.get("EARLY") == "1"
for kv in os.environ.get("OPTS", "").split():  # engine options K=V (experiments)
    e.set_option(int(kv.split("=")[0]), int(kv.split("=")[1]))
if EARLY:
    e.set_option(G.OPT_LONE, 0)
    e.set_option(G.OPT_GRID_BLOCKS, 2)
for r in range(reps):
    e.reset()
    e.set_option(G.OPT_SEED, SEED)
    e.set_option(G.OPT_ID_BASE, ROOT)
    e.debug_timing(reset=True)
    e.track(ph[ROOT:ROOT + 1])
    e.finish()
    st = e.stats()
    inst, tm = e.debug_timing(reset=True)
    if EARLY:
        print(f"rep {r} (early worker): longest life {st['max_photon_steps']} steps, tracked {st['n_tracked']}, early "
              f"photons {st['n_early']}, early worker {st['early_ms']:.1f} ms, all kernels {st['last_kernel_ms']:.1f} ms -> "
              f"{st['early_ms'] * 1e3 / max(st['max_photon_steps'], 1):.3f} us/step of the longest life", flush=True)
    else:
        print(f"rep {r}: longest life {st['max_photon_steps']} steps, tracked {st['n_tracked']}, lone photons "
              f"{st['n_lone']} lone kernel {st['lone_ms']:.1f} ms, all kernels {st['last_kernel_ms']:.1f} ms -> "
              f"{st['last_kernel_ms'] * 1e3 / max(st['max_photon_steps'], 1):.3f} us/step of the longest life", flush=True)
    if inst:
        g, i = tm[16:22], tm[36:40]
        if g[0]:
            print(f"  geometry wave (> 1e5-step photons): {g[0]} steps, walk rounds/step {g[1] / g[0]:.3f}, "
                  f"halved {g[5] / g[0]:.3f}; cycles/step walk {g[2] / g[0]:.0f} step_size {g[3] / g[0]:.0f} "
                  f"loop-rest {g[4] / g[0]:.0f}", flush=True)
        if i[0]:
            print(f"  interaction wave (> 1e5-step photons): {i[0]} batches of {i[1] / i[0]:.2f} steps; cycles: batch "
                  f"evaluation {i[2] / i[0]:.0f} per batch, serial {i[3] / max(i[1], 1):.0f} per step, total "
                  f"{(i[2] + i[3]) / max(i[1], 1):.0f} per step; waits: interaction {tm[30] / 2.4e6:.1f} ms geometry "
                  f"{tm[31] / 2.4e6:.1f} ms", flush=True)
