"""Device adaptive-bias dynamics by chunk: the emitted batch (192^2, photon_n=1e5, seed 123) tracked in
successive slices on one engine (counters carry over), printing recorded/created per slice -- compare
with the oracle's serial run sliced the same way."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=100000).init(0)
e = G.Engine(m, 0)
e.emit_setup(m)
for spec in (sys.argv[1:] or ["0"]):
    grid = int(spec.rstrip("zs"))
    zone_order, single = "z" in spec, "s" in spec
    e.reset()
    e.set_option(G.OPT_SEED, 123)
    e.set_option(G.OPT_GRID_BLOCKS, grid)
    p, n = e.emit(seed=123)
    ph = e.download(p, n)
    import numpy as np
    if not zone_order:
        ph = ph[np.random.default_rng(1).permutation(n)]
    d = e.upload(ph)
    edges = [0, n] if single else [0, 1000, 5000, 20000, 50000, 100000, 200000, 400000, 700000, 1000000, n]
    prev = e.debug_counters()
    print(f"grid {grid or 'all CUs'} {'zone order' if zone_order else 'random order'}"
          f"{' one call' if single else ''}", flush=True)
    for a, b in zip(edges[:-1], edges[1:]):
        e.track_device(d + a * 128, b - a)
        c = e.debug_counters()
        dr, ds = c["n_recorded"] - prev["n_recorded"], c["n_scatt"] - prev["n_scatt"]
        print(f"photons {a:8d}-{b:8d}: rec/created {dr / (b - a):.3f} scatt/created {ds / (b - a):.3f} "
              f"max_tau {c['max_tau_scatt']:.3e} avg_nscatt {c['n_scatt'] / (c['n_recorded'] + 1):.3f}"
              , flush=True)
        prev = c
