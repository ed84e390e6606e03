"""A whole run_simulation pass with the adaptive bias FROZEN at one snapshot, on the device or on the
oracle: with the bias frozen every photon's trajectory is fixed by its Philox stream alone, so the
device and the oracle must agree photon by photon on the whole pass -- including the rare paths a
2,000-photon test never reaches (lone / early hand-overs, overflow relaunches, 10^5-step photons),
which decide extreme-value counters such as max tau_scatt.

    python tools/frozen_pass_probe.py --side oracle --out gpurun_out/frozen_oracle.json   (CPU, ~6 min)
    python tools/frozen_pass_probe.py --side device --out gpurun_out/frozen_device.json   (GPU)
    python tools/frozen_pass_probe.py --compare a.json b.json

Summary per side: counters, end reasons, the recorded photons with the largest tau_scatt, every
photon of more than --long steps, and a 1/--every sample of all end records keyed by photon id.
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))

FIELDS = ("id", "parent_id", "w", "e", "x1", "x2", "x3", "tau_abs", "tau_scatt", "n_scatt", "n_step", "end_reason")


def rows(tr):
    return [{f: (int(r[f]) if f in ("id", "parent_id", "n_scatt", "n_step", "end_reason") else float(r[f]))
             for f in FIELDS} for r in tr]


def roots_of(tr, ids):
    """the primary each photon descends from (walking parent ids through the trace)"""
    order = np.argsort(tr["id"])
    sid, spar = tr["id"][order], tr["parent_id"][order]
    out = []
    for i in ids:
        cur = np.uint64(i)
        for _ in range(10000):
            k = np.searchsorted(sid, cur)
            if k >= len(sid) or sid[k] != cur or spar[k] == np.uint64(~np.uint64(0)):
                break
            cur = spar[k]
        out.append(int(cur))
    return out


def summarise(tr, counters, args):
    rec = tr[tr["end_reason"] == 0]
    top = rec[np.argsort(rec["tau_scatt"])[::-1][:args.top]]
    long_ = tr[tr["n_step"] > args.long]
    samp = tr[(tr["id"] % np.uint64(args.every)) == 0]
    return dict(counters=counters, n_trace=int(len(tr)),
                end_reasons={int(k): int(v) for k, v in zip(*np.unique(tr["end_reason"], return_counts=True))},
                max_tau_recorded=float(rec["tau_scatt"].max()) if len(rec) else 0.0,
                max_tau_any=float(tr["tau_scatt"].max()), max_n_step=int(tr["n_step"].max()),
                top_tau=rows(top), top_roots=roots_of(tr, top["id"][:args.top]), long=rows(long_),
                long_roots=roots_of(tr, long_["id"]), sample=rows(samp))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--side", choices=("device", "oracle"))
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--seed", type=int, default=123)
    ap.add_argument("--photon-n", type=float, default=1e5)
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--scatt0", type=int, default=3_700_000)
    ap.add_argument("--rec0", type=int, default=2_250_000)
    ap.add_argument("--maxtau0", type=float, default=6.0e-4)
    ap.add_argument("--top", type=int, default=200)
    ap.add_argument("--long", type=int, default=20000)
    ap.add_argument("--every", type=int, default=499)
    ap.add_argument("--cap", type=int, default=40_000_000)
    ap.add_argument("--roots", default="", help="oracle: track only these primaries (a JSON file's top_roots)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    if a.compare:
        return compare(*a.compare)
    from grmonty_amd.synth_dump import ensure_dump
    d = os.path.join(REPO, "gpurun_out") if os.path.isdir(os.path.join(REPO, "gpurun_out")) else "/tmp"
    path = ensure_dump(os.path.join(d, f"synth{a.grid}.dump"), a.grid, a.grid)
    if a.side == "oracle":
        import oracle_py as O
        m = O.OracleModel(path, photon_n=int(a.photon_n))
        m.init(8)
        ph = m.emit_philox(seed=a.seed)
        if a.roots:
            js = json.load(open(a.roots))
            sel = sorted(set(js["top_roots"]) | set(js["long_roots"]))
            tr = np.concatenate([m.track(ph[i:i + 1], rng_mode=1, seed=a.seed, id_base=i, frozen=True,
                                         scatt0=a.scatt0, rec0=a.rec0, max_tau0=a.maxtau0, trace_cap=a.cap)
                                 for i in sel])
            ph = ph[sel]
        else:
            tr = m.track(ph, rng_mode=1, seed=a.seed, id_base=0, frozen=True, scatt0=a.scatt0, rec0=a.rec0,
                         max_tau0=a.maxtau0, trace_cap=a.cap)
        c = m.counters()
        counters = dict(created=len(ph), recorded=c["recorded"], scattered=c["scattered"], steps=c["steps"])
    else:
        import struct
        import grmonty_amd as G
        model = G.Model.load(path, photon_n=int(a.photon_n)).init(8)
        eng = G.Engine(model, device=0)
        eng.emit_setup(model)
        eng.reset()
        eng.set_option(G.OPT_SEED, a.seed)
        eng.set_option(G.OPT_ID_BASE, 0)
        eng.set_option(G.OPT_BIAS_MODE, 1)
        eng.set_option(G.OPT_FROZEN_SCATT, a.scatt0)
        eng.set_option(G.OPT_FROZEN_REC, a.rec0)
        eng.set_option(G.OPT_FROZEN_MAXTAU, struct.unpack("<q", struct.pack("<d", a.maxtau0))[0])
        eng.set_option(G.OPT_TRACE_CAP, a.cap)
        p, n = eng.emit(seed=a.seed)
        eng.track_device(p, n)
        st = eng.stats()
        tr = eng.trace(a.cap)
        _, n_rec, n_scatt, mt = eng.finish()
        counters = dict(created=int(n), recorded=int(n_rec), scattered=int(n_scatt), steps=int(st["n_steps"]),
                        max_tau_engine=float(mt), stats={k: (v if isinstance(v, (int, float)) else str(v))
                                                         for k, v in st.items()})
        eng.close()
    out = summarise(tr, counters, a)
    print(json.dumps({k: v for k, v in out.items() if k not in ("top_tau", "long", "sample", "top_roots",
                                                                  "long_roots")}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f)


def compare(pa, pb):
    A, B = json.load(open(pa)), json.load(open(pb))
    for k in ("counters", "end_reasons", "max_tau_recorded", "max_tau_any", "max_n_step", "n_trace"):
        print(f"{k}:\n  {pa}: {A[k]}\n  {pb}: {B[k]}")
    for part in ("sample", "long", "top_tau"):
        da = {r["id"]: r for r in A[part]}
        db = {r["id"]: r for r in B[part]}
        common = set(da) & set(db)
        same = [i for i in common if da[i]["end_reason"] == db[i]["end_reason"] and da[i]["n_step"] == db[i]["n_step"]
                and abs(da[i]["tau_scatt"] - db[i]["tau_scatt"]) <= 1e-9 * max(1e-300, abs(da[i]["tau_scatt"]))]
        print(f"{part}: {len(da)} vs {len(db)} records, {len(common)} common ids, {len(same)} equal "
              f"(end, n_step, tau_scatt)")
        bad = sorted(common - set(same))[:10]
        for i in bad:
            print("  A", {k: da[i][k] for k in ("n_step", "end_reason", "tau_scatt", "n_scatt", "w")})
            print("  B", {k: db[i][k] for k in ("n_step", "end_reason", "tau_scatt", "n_scatt", "w")})
        only = sorted(set(da) - set(db))[:5]
        for i in only:
            print("  only A", {k: da[i][k] for k in ("id", "n_step", "end_reason", "tau_scatt", "n_scatt")})
        only = sorted(set(db) - set(da))[:5]
        for i in only:
            print("  only B", {k: db[i][k] for k in ("id", "n_step", "end_reason", "tau_scatt", "n_scatt")})


if __name__ == "__main__":
    main()
