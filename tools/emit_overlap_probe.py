"""Would the emission slow the live-bias warm-up if it ran beside it?  (the emission
could overlap the warm-up only on the CUs the warm-up leaves free; round 5's in-launch variant saw the
warm-up's families slow about twofold.)  Engine A tracks a photon_n = 1e6 pass on the warm-up's 64
workgroups only (GRM_OPT_GRID_BLOCKS = 64, so 192 CUs stay free); engine B, from a second thread,
emits passes back to back into its own buffer on the free CUs while A's warm-up runs.  Prints A's
warm-up end (and admission log) with and without B.

    python tools/emit_overlap_probe.py [reps]
"""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=1e6).init(0, device=0)
a = G.Engine(m, 0)
a.emit_setup(m)
a.set_option(G.OPT_GRID_BLOCKS, 64)
b = G.Engine(m, 0)
b.emit_setup(m)
b.emit(seed=999)  # allocate B's buffer outside the measurement
for r in range(reps):
    for concurrent in (False, True):
        seed = 123 + r
        a.reset()
        a.set_option(G.OPT_SEED, seed)
        p, n = a.emit(seed=seed)
        stop = threading.Event()
        emitted = [0]

        def emitter():
            while not stop.is_set():
                b.emit(seed=500 + emitted[0])
                emitted[0] += 1

        th = threading.Thread(target=emitter) if concurrent else None
        if th:
            th.start()
            time.sleep(0.002)
        t0 = time.time()
        a.track_device(p, n)
        wall = time.time() - t0
        stop.set()
        if th:
            th.join()
        ph = a.debug_phases()
        st = a.stats()
        print(f"seed {seed} concurrent emission {'on ' if concurrent else 'off'}: warm-up ends "
              f"{ph['warmup_end_ms']:.1f} ms, emissions beside it {emitted[0]}, dominant {st['max_launch_ms']:.0f} ms "
              f"(64 workgroups), admissions " + " ".join(f"{t:.1f}" for t, _ in ph["admissions"]), flush=True)
        a.finish()
