"""CPU oracle replay (mt19937 off: the device Philox streams, bias frozen at the probe snapshot) of the
root primaries saved by tools/maxstep_probe.py: does the reference algorithm give the same long-lived
photon?  Usage: python tools/maxstep_replay.py [seed]   (test infrastructure: runs the oracle)"""
import os, sys, time
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd")); sys.path.insert(0, os.path.join(REPO, "oracle"))
SEED = int(sys.argv[1]) if len(sys.argv) > 1 else 126
import oracle_py as O
from grmonty_amd.synth_dump import ensure_dump
d = np.load(os.path.join(REPO, "gpurun_out", f"maxstep_{SEED}.npz"))
roots, ph, snap = d["roots"], d["photons"], d["snap"]
print("roots", roots, "long", d["long"][["id", "n_step", "end_reason", "x1", "x2", "x3", "n_scatt"]])
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
orc = O.OracleModel(path, photon_n=1000000)
orc.init(8)
for r, p in zip(roots, ph):
    t = time.time()
    tr = orc.track(p[None], rng_mode=1, seed=SEED, id_base=int(r), frozen=True, scatt0=int(snap[0]), rec0=int(snap[1]),
                   max_tau0=float(snap[2]), trace_cap=100000)
    print(f"root {r}: {len(tr)} family ends in {time.time()-t:.1f}s; longest {tr['n_step'].max()} steps")
    for x in tr[np.argsort(-tr['n_step'])][:3]:
        print("  ", int(x['id']), int(x['parent_id']), int(x['n_step']), int(x['end_reason']), x['x1'], x['x2'], x['x3'], x['w'], int(x['n_scatt']))
