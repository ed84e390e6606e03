"""Concurrency emulator runs (oracle grmo_track_concurrent): the reference's transport scheduled the
way a concurrent engine schedules it, to pin where the device's live-bias counter offset comes from
(VERDICT r03, next-round item 1a).

Each job: the 192^2 synthetic dump at photon_n (default 1e5), the device emission of a seed
(grmo_emit_philox: the same photon list the engine tracks), tracked by grmo_track_concurrent under a
named scheduling configuration; prints one JSON line per job (counters, max tau_scatt, rounds) and
appends it to --out.  The serial oracle fixtures (tests/golden/oracle_synth192_pn1e5.json) are the
bar.

    python tools/lag_emulator.py --configs serial,device --seeds 123-130 [--photon-n 1e5] [--procs 8]

Configurations (oracle_py.OracleModel.EMU_DEVICE / EMU_SERIAL plus overrides, see CONFIGS).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))

DEV = dict(slots=131072, group=64, refresh=64, child_min=8, depth_first=0, claim_sh=-1, warm_n=-1, warm_slack=4,
           warm_b0=64, flight_cap=0)
SER = dict(slots=1, group=1, refresh=1, child_min=1, depth_first=1, claim_sh=0, warm_n=0, warm_slack=4, warm_b0=64,
           flight_cap=0)
CONFIGS = {
    "serial": SER,                                   # = the serial reference (Philox streams)
    "serial_claim": dict(SER, claim_sh=-1),          # serial, the device's interleaved claim order
    "device": DEV,                                   # the engine at photon_n = 1e5 (ramp to a grid of lanes)
    "device_w4096": dict(DEV, warm_n=4096, warm_slack=1),  # the engine's large-pass warm-up
    "device_df": dict(DEV, depth_first=1),           # device, children depth-first in their parent's lane
    "device_r1": dict(DEV, refresh=1),               # device, counters fresh every round
    "device_cm1": dict(DEV, child_min=1),            # device, children before primaries
}


def parse_seeds(s):
    out = []
    for part in s.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def tables_cache(path, photon_n):
    import oracle_py as O
    cache = path + f".tables_pn{int(photon_n)}.npz"
    if not os.path.exists(cache):
        m = O.OracleModel(path, photon_n=int(photon_n))
        m.init(8)
        np.savez(cache, **{str(i): m.table(i) for i in range(6)})
    return cache


def job(args):
    path, cache, photon_n, name, cfg, seed = args
    import oracle_py as O
    m = O.OracleModel(path, photon_n=int(photon_n))
    O.lib().grmo_init_geometry(m.h)
    t = np.load(cache)
    for i in range(6):
        m.set_table(i, t[str(i)])
    ph = m.emit_philox(seed=seed)
    t0 = time.time()
    rounds, _, _ = m.track_concurrent(ph, seed=seed, **cfg)
    c = m.counters()
    rep = m.report(None)
    return dict(config=name, seed=seed, photon_n=photon_n, rounds=int(rounds), wall_s=time.time() - t0,
                luminosity=rep["luminosity"], max_tau_scatt=rep["max_tau_scatt"], **c, cfg=cfg)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="serial,device")
    ap.add_argument("--seeds", default="123-130")
    ap.add_argument("--photon-n", type=float, default=1e5)
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--set", action="append", default=[], help="name:key=v,key=v -- an extra configuration")
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r04_lag_emulator.jsonl"))
    a = ap.parse_args()
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump(os.path.join("/tmp", f"synth{a.grid}.dump"), a.grid, a.grid)
    cache = tables_cache(path, a.photon_n)
    cfgs = dict(CONFIGS)
    for s in a.set:
        name, kv = s.split(":", 1)
        base = dict(DEV)
        for item in kv.split(","):
            k, v = item.split("=")
            if k == "base":
                base = dict(CONFIGS[v])
            else:
                base[k] = int(float(v))
        cfgs[name] = base
    jobs = [(path, cache, a.photon_n, c, cfgs[c], s) for c in a.configs.split(",") for s in parse_seeds(a.seeds)]
    with mp.Pool(a.procs) as pool, open(a.out, "a") as f:
        for r in pool.imap_unordered(job, jobs):
            line = json.dumps(r)
            print(line, flush=True)
            f.write(line + "\n")
            f.flush()


if __name__ == "__main__":
    main()
