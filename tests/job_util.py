"""One run_simulation job on the device as bench.py runs it (harm_model.cpp:340-414): device emission
of a seed, transport with the live adaptive bias, spectrum and counters read back -- either on one
engine, or as an N-rank job emulated on one GPU: the zones split into shards (grmonty_amd.zone_shards:
(z0, z1, stride) zone sets), each shard a pass of its own after grm_engine_reset (so that each
emulated rank's adaptive bias runs on its own counters, as on N GPUs), photon ids global (rank r's
id base = the photons of the shards before it), the ranks' spectra and counters summed (max for
max tau_scatt) as grm_engine_allreduce_stash reduces them."""
import numpy as np

from spectrum_stats import cell_sums_from_trace

KEYS = ("recorded", "scattered", "steps", "luminosity")


def run_job(eng, model, seed, shards=None, trace_cap=0):
    """returns dict(created, recorded, scattered, steps, luminosity, spectrum, cells (if traced),
    per_rank: list of per-rank counters)"""
    import grmonty_amd as G
    if shards is None:
        shards = [(0, -1, 1)]
    spec = None
    out = dict(created=0, recorded=0, scattered=0, steps=0, max_tau=0.0, per_rank=[])
    cells = np.zeros((1200, 5)) if trace_cap else None
    base = 0
    for sh in shards:
        z0, z1, stride = (tuple(sh) + (1,))[:3]
        eng.reset()
        eng.set_option(G.OPT_SEED, seed)
        eng.set_option(G.OPT_ID_BASE, base)
        if trace_cap:
            eng.set_option(G.OPT_TRACE_CAP, trace_cap)
        p, n = eng.emit(seed=seed, z0=z0, z1=z1, stride=stride)
        eng.track_device(p, n)
        st = eng.stats()
        assert st["n_dropped"] == 0 and st["n_abandoned"] == 0
        s, n_rec, n_scatt, mt = eng.finish()
        if trace_cap:
            tr = eng.trace(trace_cap)
            assert len(tr) == st["n_tracked"], "trace overflow"
            cells += cell_sums_from_trace(tr)
        spec = s.copy() if spec is None else _add_cells(spec, s)
        out["created"] += n
        out["recorded"] += n_rec
        out["scattered"] += n_scatt
        out["steps"] += st["n_steps"]
        out["max_tau"] = max(out["max_tau"], mt)
        out["per_rank"].append(dict(created=n, recorded=n_rec, scattered=n_scatt, steps=st["n_steps"]))
        base += n
    if trace_cap:
        eng.set_option(G.OPT_TRACE_CAP, 0)
        out["cells"] = cells
    out["spectrum"] = spec
    out["luminosity"] = model.write_spectrum(spec, None)["luminosity"]
    return out


def _add_cells(a, b):
    r = a.copy()
    for f in a.dtype.names:
        r[f] = a[f] + b[f]
    return r
