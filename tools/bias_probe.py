"""Adaptive-bias dynamics probe (192^2, photon_n=1e5, device emission seed 123): counters of the
device under (a) live bias, (b) live bias with the whole batch in warm-up admission, (c) bias frozen
at given counters.  Compare with the oracle (tests/golden/oracle_synth192_pn1e5.json)."""
import os
import struct
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=100000).init(0)
e = G.Engine(m, 0)
e.emit_setup(m)
e.set_option(G.OPT_WATCHDOG_MS, 120000)
modes = sys.argv[1:] or ["live", "warmall", "frozen:3634679:2218559:0.0023690051872363254"]
seeds = [int(x) for x in os.environ.get("SEEDS", "123").split(",")]
for mode, seed in [(md, sd) for md in modes for sd in seeds]:
    e.reset()
    e.set_option(G.OPT_SEED, seed)
    e.set_option(G.OPT_BIAS_MODE, 0)
    e.set_option(G.OPT_WARMUP, 32768)
    e.set_option(G.OPT_WARMUP_SLACK, 4)
    e.set_option(G.OPT_WARMUP_BATCH, 64)
    if mode == "warmall":
        e.set_option(G.OPT_WARMUP, 10**9)
    elif mode.startswith("frozen"):
        _, s, r, mt = mode.split(":")
        e.set_option(G.OPT_BIAS_MODE, 1)
        e.set_option(G.OPT_FROZEN_SCATT, int(s))
        e.set_option(G.OPT_FROZEN_REC, int(r))
        e.set_option(G.OPT_FROZEN_MAXTAU, struct.unpack("<q", struct.pack("<d", float(mt)))[0])
    elif mode.startswith("warm:"):
        f = mode.split(":")
        e.set_option(G.OPT_WARMUP, int(f[1]))
        if len(f) > 2:
            e.set_option(G.OPT_WARMUP_SLACK, int(f[2]))
        if len(f) > 3:
            e.set_option(G.OPT_WARMUP_BATCH, int(f[3]))
    t = time.time()
    p, n = e.emit(seed=seed)
    e.track_device(p, n)
    spec, n_rec, n_scatt, mt = e.finish()
    st = e.stats()
    lum = m.write_spectrum(spec, None)["luminosity"]
    print(f"{mode} seed {seed}: {time.time() - t:.2f}s created {n} recorded {n_rec} scattered {n_scatt} steps {st['n_steps']} "
          f"max_tau {mt:.4g} L {lum:.4f} launches {st['n_launches']}", flush=True)
