"""Does the ORDER in which superphotons are tracked move the reference's counters?

The adaptive bias (bias_func, harm_model.cpp:1391-1404) runs on counters of the photons recorded so
far, so the expected recorded / scattered / step counts of a run depend on the processing order.
The reference tracks photons serially in zone-walk order (make_super_photon, :673-811); the device
claims them interleaved over 4096 evenly spaced runs of the zone-ordered batch (grm_engine.hip,
run_transport) and many at once.  This probe runs the oracle SERIALLY (reference semantics: mt19937
transport, live bias) over the same Philox-emitted photons in both orders, per seed, so that the
order effect is separated from the concurrency effect.

    python tools/order_probe.py [--seeds 123,124,125,126] [--photon-n 1e5] [--orders zone,interleaved]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "cuda-grmonty_amd")]


def claim_order(n, sh=12):
    """grm_engine.hip run_transport: claim position q -> photon (q mod 2^sh) * m + q / 2^sh"""
    if n < (2 << sh):
        return np.arange(n)
    m = (n + (1 << sh) - 1) >> sh
    q = np.arange(m << sh, dtype=np.int64)
    idx = (q & ((1 << sh) - 1)) * m + (q >> sh)
    return idx[idx < n]


def run(args):
    path, photon_n, seed, order = args
    import oracle_py as O
    m = O.OracleModel(path, photon_n=photon_n)
    m.init(1)
    ph = m.emit_philox(seed=seed)
    if order == "interleaved":
        ph = ph[claim_order(len(ph))]
    elif order == "reversed":
        ph = ph[::-1]
    t = time.time()
    m.track(ph, rng_mode=0, seed=seed, frozen=False)
    c = m.counters()
    rep = m.report(None)
    return dict(seed=seed, order=order, wall_s=round(time.time() - t, 1), luminosity=rep["luminosity"],
                max_tau_scatt=rep["max_tau_scatt"], **c)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="123,124,125,126")
    ap.add_argument("--photon-n", type=float, default=1e5)
    ap.add_argument("--orders", default="zone,interleaved")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03_order_probe.json"))
    args = ap.parse_args()
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump("/tmp/synth192.dump", 192, 192)
    jobs = [(path, int(args.photon_n), int(s), o) for s in args.seeds.split(",") for o in args.orders.split(",")]
    with mp.Pool(min(8, len(jobs))) as pool:
        res = pool.map(run, jobs)
    summ = {}
    for o in args.orders.split(","):
        rs = [r for r in res if r["order"] == o]
        summ[o] = {k: (float(np.mean([r[k] for r in rs])), float(np.std([r[k] for r in rs], ddof=1)))
                   for k in ("recorded", "scattered", "steps", "luminosity")}
    out = {"photon_n": args.photon_n, "runs": res, "mean_sd": summ}
    json.dump(out, open(args.out, "w"), indent=1)
    print(json.dumps(summ, indent=1))


if __name__ == "__main__":
    main()
