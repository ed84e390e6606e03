"""Diagnostic: fate of hand-made pathological photons (trace end records)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import numpy as np  # noqa: E402

import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth64.dump"), 64, 64)
m = G.Model.load(path, photon_n=20000).init(0)
ph = m.emit(seed=123)
eng = G.Engine(m, 0)
eng.set_option(G.OPT_WATCHDOG_MS, 20000)
cases = {"x2=0": ("x", 2, 0.0), "x2=1": ("x", 2, 1.0), "k1=inf": ("k", 1, np.inf), "k3=inf": ("k", 3, np.inf),
         "k2=inf": ("k", 2, np.inf), "k0=inf": ("k", 0, np.inf)}
for name, (f, i, v) in cases.items():
    b = ph[np.flatnonzero((ph["x"][:, 1] > 1.0) & (ph["x"][:, 1] < 2.5))[:1]].copy()
    b[f][0, i] = v
    b["w"] = 1e40
    eng.reset()
    eng.set_option(G.OPT_TRACE_CAP, 1000)
    try:
        eng.track(b)
    except RuntimeError as exc:
        print(name, "FAILED", exc, eng.debug_stuck()[:2], flush=True)
        continue
    tr = eng.trace(1000)
    st = eng.stats()
    print(name, "nan-ended", st["n_nan_photons"], "steps", st["n_steps"],
          [(int(t["end_reason"]), int(t["n_step"]), float(t["x1"]), float(t["w"])) for t in tr[:4]], flush=True)
