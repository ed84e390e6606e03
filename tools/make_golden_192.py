"""Statistical parity fixtures at the headline scale (BASELINE configs[0]: photon_n = 1e5 on the
dump019-class 192x192 synthetic dump, mass_unit = 4e19).

Runs the oracle's run_simulation (reference CPU semantics: serial, one mt19937 stream for emission
and transport, live adaptive bias; harm_model.cpp:340-414) for several seeds in parallel processes
and commits, per seed:
  - counters (created, scattered, recorded, steps), luminosity and max tau_scatt (report_spectrum,
    harm_model.cpp:416-471);
  - per (theta, energy) cell sums over the recorded superphotons: count, sum w, sum w^2, sum w E,
    sum (w E)^2 -- enough for a binned KS test on nu L_nu with Kish effective N;
and the full 6x200x13 spectrum of seed 123 (writer fixtures).
Output: tests/golden/oracle_synth192_pn1e5.npz (+ .json summary).  Takes ~5 min on 6 cores.

    python tools/make_golden_192.py [--seeds 123,124,125,126,127,128] [--photon-n 1e5] [--merge]

--merge adds the new seeds' runs to the committed fixtures (seeds already there are skipped).
Each run is a process of its own (a run that dies is reported by seed, not waited for); --from-dir
merges runs saved one per file by `tools/make_golden_192.py --one SEED --save-dir DIR` instead of
running them (photon_n = 1e6 runs take ~1 h each).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
OUT = os.path.join(REPO, "tests", "golden", "oracle_synth192_pn1e5")
N_CELL = 6 * 200


def cell_sums(tr):
    """count, sum w, sum w^2, sum wE, sum (wE)^2 per (ix2, i_e) cell over recorded photons"""
    r = tr[tr["end_reason"] == 0]
    c = r["ix2"].astype(np.int64) * 200 + r["i_e"].astype(np.int64)
    w, we = r["w"], r["w"] * r["e"]
    out = np.zeros((N_CELL, 5))
    for k, v in enumerate((np.ones_like(w), w, w * w, we, we * we)):
        out[:, k] = np.bincount(c, weights=v, minlength=N_CELL)
    return out


def run(args):
    path, photon_n, seed, cap = args
    import oracle_py as O
    m = O.OracleModel(path, photon_n=photon_n)
    m.init(1)
    t, tr, n_tr = m.run_simulation_traced(seed=seed, trace_cap=cap)
    assert n_tr <= cap, "trace overflow"
    c = m.counters()
    rep = m.report(None)
    return dict(seed=seed, wall_s=t, counters=c, luminosity=rep["luminosity"], max_tau_scatt=rep["max_tau_scatt"],
                cells=cell_sums(tr), spectrum=m.spectrum().view(np.float64).reshape(6, 200, 13) if seed == 123 else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="123,124,125,126,127,128")
    ap.add_argument("--photon-n", type=float, default=1e5)
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--merge", action="store_true", help="append to the committed fixtures")
    ap.add_argument("--out", default=OUT, help="fixture path prefix (.npz / .json)")
    ap.add_argument("--trace-cap", type=int, default=1 << 24, help="photon ends traced per run")
    ap.add_argument("--procs", type=int, default=0, help="parallel runs (default: one per seed)")
    ap.add_argument("--one", type=int, default=None, help="run this one seed and save it (--save-dir)")
    ap.add_argument("--save-dir", default="", help="directory of per-seed result files")
    ap.add_argument("--from-dir", default="", help="merge the per-seed result files of this directory")
    args = ap.parse_args()
    out = args.out
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump(os.path.join("/tmp", f"synth{args.grid}.dump"), args.grid, args.grid)
    seeds = [int(s) for s in args.seeds.split(",")]
    old = []
    if args.merge:
        g = np.load(out + ".npz")
        js = json.load(open(out + ".json"))
        for i, r in enumerate(js["runs"]):
            old.append(dict(seed=r["seed"], wall_s=r["wall_s"], luminosity=r["luminosity"],
                            max_tau_scatt=r["max_tau_scatt"], cells=g["cells"][i],
                            counters={k: r[k] for k in ("created", "scattered", "recorded", "steps")},
                            spectrum=g["spectrum123"] if r["seed"] == 123 else None))
        seeds = [s for s in seeds if s not in {r["seed"] for r in old}]
    if args.one is not None:
        r = run((path, int(args.photon_n), args.one, args.trace_cap))
        np.savez(os.path.join(args.save_dir, f"seed{args.one}.npz"), cells=r["cells"],
                 counters=np.array([r["counters"][k] for k in ("created", "scattered", "recorded", "steps")],
                                   dtype=np.int64),
                 luminosity=r["luminosity"], max_tau_scatt=r["max_tau_scatt"], wall_s=r["wall_s"])
        print(f"seed {args.one}: {r['wall_s']:.0f} s, {r['counters']}")
        return
    t = time.time()
    if args.from_dir:
        res = []
        for sd in seeds:
            f = np.load(os.path.join(args.from_dir, f"seed{sd}.npz"))
            c = f["counters"]
            res.append(dict(seed=sd, wall_s=float(f["wall_s"]), luminosity=float(f["luminosity"]),
                            max_tau_scatt=float(f["max_tau_scatt"]), cells=f["cells"], spectrum=None,
                            counters=dict(zip(("created", "scattered", "recorded", "steps"), (int(x) for x in c)))))
    else:
        from concurrent.futures import ProcessPoolExecutor
        with ProcessPoolExecutor(args.procs or max(1, len(seeds))) as pool:
            res = list(pool.map(run, [(path, int(args.photon_n), s, args.trace_cap) for s in seeds]))
    print(f"{len(seeds)} oracle runs in {time.time() - t:.0f} s")
    res = old + res
    res.sort(key=lambda r: r["seed"])
    spec = next(r["spectrum"] for r in res if r["spectrum"] is not None)
    np.savez_compressed(out + ".npz", seeds=np.array([r["seed"] for r in res]), cells=np.stack([r["cells"] for r in res]),
                        spectrum123=spec,
                        counters=np.array([[r["counters"][k] for k in ("created", "scattered", "recorded", "steps")]
                                           for r in res], dtype=np.int64),
                        luminosity=np.array([r["luminosity"] for r in res]),
                        max_tau_scatt=np.array([r["max_tau_scatt"] for r in res]))
    summ = {"dump": f"synth_dump.write_dump(path, {args.grid}, {args.grid})", "photon_n": int(args.photon_n),
            "mass_unit": 4e19, "oracle": "grmo_run_simulation_traced (mt19937, live bias, reference order)",
            "runs": [dict(seed=r["seed"], wall_s=round(r["wall_s"], 1), luminosity=r["luminosity"],
                          max_tau_scatt=r["max_tau_scatt"], **r["counters"]) for r in res]}
    for key in ("created", "scattered", "recorded", "steps", "luminosity"):
        v = np.array([x[key] for x in summ["runs"]], dtype=np.float64)
        summ.setdefault("mean", {})[key] = float(v.mean())
        summ.setdefault("std", {})[key] = float(v.std(ddof=1))
    with open(out + ".json", "w") as fh:
        json.dump(summ, fh, indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
