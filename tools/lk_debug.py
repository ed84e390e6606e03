"""Debug: children tracked in the lone kernel (GRM_OPT_EARLY_CHILDREN) against the oracle and the relaunch path."""
import os, sys, struct
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(R, "tests")); sys.path.insert(0, os.path.join(R, "cuda-grmonty_amd")); sys.path.insert(0, os.path.join(R, "oracle"))
import grmonty_amd as G
import oracle_py as O
from grmonty_amd.synth_dump import write_dump
d = write_dump(os.path.join(R, "gpurun_out", "synth64.dump"), 64, 64)
om = O.OracleModel(d, photon_n=2000); om.init(8)
m = G.Model.load(d, photon_n=2000).init(8)
ph = m.emit(seed=123)
rng = np.random.default_rng(42)
sel = ph[rng.permutation(len(ph))[:1500]]
warm = ph[rng.permutation(len(ph))[:1000]]
om.reset(); om.L.grmo_model_set_max_tau_scatt(om.h, m.scalars()["max_tau_scatt"])
om.track(warm, rng_mode=O.GRMO_RNG_MT19937 if hasattr(O, "GRMO_RNG_MT19937") else 0, seed=5, frozen=False)
c = om.counters(); snap = dict(scatt=c["scattered"], rec=c["recorded"], maxtau=om.scalars()["max_tau_scatt"])
om.reset()
tr_o = om.track(sel, rng_mode=1, seed=123, id_base=0, frozen=True, scatt0=snap["scatt"], rec0=snap["rec"], max_tau0=snap["maxtau"], trace_cap=4_000_000)
go = {int(r["id"]): r for r in tr_o}
eng = G.Engine(m, device=0)
f2i = lambda v: struct.unpack("<q", struct.pack("<d", v))[0]
out = {}
for kids in (1, 0):
    eng.set_option(G.OPT_LONE, 2)
    eng.set_option(G.OPT_EARLY_CHILDREN, kids)
    eng.reset()
    eng.set_option(G.OPT_SEED, 123); eng.set_option(G.OPT_ID_BASE, 0); eng.set_option(G.OPT_BIAS_MODE, 1)
    eng.set_option(5, snap["scatt"]); eng.set_option(6, snap["rec"]); eng.set_option(7, f2i(snap["maxtau"]))
    eng.set_option(G.OPT_TRACE_CAP, 4_000_000)
    eng.track(sel)
    tr = eng.trace(4_000_000)
    eng.finish()
    st = eng.stats()
    out[kids] = {int(r["id"]): r for r in tr}
    print(f"kids={kids}: ends {len(tr)} lone {st['n_lone']} lone_children {st['n_lone_children']} overflow {st['n_overflow']} launches {st['n_launches']}")
keys = ("end_reason", "n_step", "n_scatt", "w", "e", "x1", "ix2", "i_e", "parent_id")
n = 0
for i, a in out[1].items():
    if i < 1500: continue
    o = go.get(i); b = out[0].get(i)
    print("child", i, "\n  dev-lk ", {k: a[k].item() for k in keys}, "\n  dev-ovf", {k: b[k].item() for k in keys} if b is not None else None,
          "\n  oracle ", {k: o[k].item() for k in keys} if o is not None else None)
    n += 1
    if n >= 8: break
