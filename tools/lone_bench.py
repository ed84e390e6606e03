"""Deterministic latency probe of the lone-photon pipeline: a fixed set of emitted photons, bias
frozen at a fixed snapshot, every photon handed to lone_kernel at its first step (GRM_OPT_LONE = 2),
so the lone launch time is the longest photon's serial chain.  Prints per-step time of that chain.
Usage: python tools/lone_bench.py [n_photons] [reps]   (GRMONTY_AMD_LIB selects a variant)"""
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import numpy as np  # noqa: E402

import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=1e5).init(0)
ph = m.emit(seed=123)
sel = ph[np.random.default_rng(7).permutation(len(ph))[:n]]
e = G.Engine(m, 0)
e.set_option(G.OPT_LONE, 2)
e.set_option(G.OPT_EARLY_STEPS, 0)
e.set_option(G.OPT_BIAS_MODE, 1)
e.set_option(5, 1_000_000)
e.set_option(6, 800_000)
e.set_option(7, struct.unpack("<q", struct.pack("<d", 2.0))[0])
# pass 1: find the longest-lived primary of the set (frozen bias: deterministic given its id)
e.set_option(G.OPT_TRACE_CAP, 4_000_000)
e.reset()
e.set_option(G.OPT_SEED, 123)
e.set_option(G.OPT_ID_BASE, 0)
e.track(sel)
tr = e.trace(4_000_000)
e.finish()
e.set_option(G.OPT_TRACE_CAP, 0)
prim = tr[(tr["id"] < n) & (tr["end_reason"] != 4)]
i = int(prim["id"][np.argmax(prim["n_step"])])
print(f"{n} photons: longest primary id {i}, {int(prim['n_step'].max())} steps", flush=True)

# pass 2: that photon alone (same id, so the same stream), its chain is the lone launch
for r in range(reps):
    e.reset()
    e.set_option(G.OPT_SEED, 123)
    e.set_option(G.OPT_ID_BASE, i)
    e.track(sel[i:i + 1])
    e.finish()
    st = e.stats()
    if r == 0:
        print({k: v for k, v in st.items()}, flush=True)
    print(f"rep {r}: lone photons {st['n_lone']} lone kernel {st['lone_ms']:.2f} ms, longest life "
          f"{st['max_photon_steps']} steps -> {st['lone_ms'] * 1e3 / max(st['max_photon_steps'], 1):.3f} us/step, "
          f"steps {st['n_steps']}", flush=True)
