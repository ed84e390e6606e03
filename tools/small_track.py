"""Track calls of a few photons (1, 2, 7, 64): every primary must be tracked."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth64.dump"), 64, 64)
m = G.Model.load(path, photon_n=2e3).init(0)
ph = m.emit(seed=123)
e = G.Engine(m, 0)
for lone in (1, 2):
    e.set_option(G.OPT_LONE, lone)
    for n in (1, 2, 7, 64):
        for base in (0, 5):
            e.reset()
            e.set_option(G.OPT_ID_BASE, base)
            e.track(ph[base:base + n])
            e.finish()
            st = e.stats()
            print(f"lone {lone} n {n} id_base {base}: primaries {st['n_primaries']} tracked {st['n_tracked']} "
                  f"steps {st['n_steps']} lone {st['n_lone']}", flush=True)
