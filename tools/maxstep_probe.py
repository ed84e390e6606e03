"""Which photons of a pass run to max_n_step (1.28 M steps), and is that the reference's behaviour?
Runs the seed-126 pass at 192^2, photon_n = 1e6 on the device with the bias FROZEN at a snapshot
(deterministic, so the oracle can replay it photon by photon), traces every photon's end, and saves
the root primaries of any photon that lived > 1e5 steps (with the snapshot) to
gpurun_out/maxstep_<seed>.npz for a CPU replay through the oracle.
Usage: python tools/maxstep_probe.py [seed] [reps]"""
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import numpy as np  # noqa: E402

import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 126
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=1e6).init(0)
ph = m.emit(seed=seed)
n = len(ph)
e = G.Engine(m, 0)
# snapshot: the live counters of one live pass of this seed
e.reset()
e.set_option(G.OPT_SEED, seed)
e.set_option(G.OPT_ID_BASE, 0)
e.track(ph)
st = e.stats()
_, n_rec, n_scatt, max_tau = e.finish()
print(f"live pass: {n} photons, recorded {n_rec} scattered {n_scatt} max_tau {max_tau:.4g} longest life "
      f"{st['max_photon_steps']} steps, lives > 1e5: {st.get('n_long_photons', st.get('n_long'))}", flush=True)
snap = dict(scatt=int(n_scatt), rec=int(n_rec), maxtau=float(max_tau))
e.set_option(G.OPT_BIAS_MODE, 1)
e.set_option(5, snap["scatt"])
e.set_option(6, snap["rec"])
e.set_option(7, struct.unpack("<q", struct.pack("<d", snap["maxtau"]))[0])
cap = 48_000_000
e.set_option(G.OPT_TRACE_CAP, cap)
e.reset()
e.set_option(G.OPT_SEED, seed)
e.set_option(G.OPT_ID_BASE, 0)
e.track(ph)
st = e.stats()
tr = e.trace(cap)
e.finish()
print(f"frozen pass: trace {len(tr)} records, longest life {st['max_photon_steps']} steps", flush=True)
long_ = tr[tr["n_step"] > 100000]
print("photons > 1e5 steps:", len(long_), flush=True)
par = dict(zip(tr["id"].tolist(), tr["parent_id"].tolist()))
roots = []
for r in long_:
    i, hops = int(r["id"]), 0
    while i >= n and hops < 1000:  # children carry hashed ids; primaries are batch indices < n
        i = int(par.get(i, -1))
        hops += 1
        if i < 0:
            break
    print(f"  id {int(r['id'])} n_step {int(r['n_step'])} end {int(r['end_reason'])} x1 {r['x1']:.6g} x2 {r['x2']:.17g} "
          f"x3 {r['x3']:.6g} w {r['w']:.4g} n_scatt {int(r['n_scatt'])} root {i} hops {hops}", flush=True)
    if 0 <= i < n:
        roots.append(i)
roots = sorted(set(roots))
np.savez(os.path.join(REPO, "gpurun_out", f"maxstep_{seed}.npz"), roots=np.array(roots, dtype=np.int64),
         photons=ph[roots] if roots else ph[:0], long=long_, snap=np.array([snap["scatt"], snap["rec"], snap["maxtau"]]))
