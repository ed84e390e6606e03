"""How often does a photon's hotcross / K2 lookup hit the table cell of its previous lookup?
(verdict r05, next-round item 1a: sizes the speculative table loads of track_kernel before any GPU
work.)  Runs the oracle's serial run_simulation (mt19937, live bias -- the reference's semantics) on
the 192^2 synthetic dump with the GRMO_IDXSTAT build (oracle/Makefile count/liboracle_idxstat.so) and
prints per-lookup reuse rates, plus the probability that every one of n lanes hits (the wave-level
rate that decides whether a speculative load removes the dependent round trip: a wave waits for the
reload if ANY of its lanes misses).

    make -C oracle count/liboracle_idxstat.so && python tools/table_reuse.py --photon-n 2e4 --seeds 123,124
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "oracle", "count", "liboracle_idxstat.so")
os.environ["GRMO_ORACLE_LIB"] = LIB
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--photon-n", type=float, default=2e4)
    ap.add_argument("--seeds", default="123")
    ap.add_argument("--lanes", default="1,8,16,41,64")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import oracle_py as O
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump("/tmp/synth192.dump", 192, 192)
    L = O.lib()
    L.grmo_idxstat.argtypes = [C.POINTER(C.c_uint64), C.c_int]
    L.grmo_idxstat.restype = None
    m = O.OracleModel(path, photon_n=int(a.photon_n))
    m.init(8)
    buf = (C.c_uint64 * 16)()
    L.grmo_idxstat(buf, 1)
    tot = np.zeros(16, dtype=np.float64)
    for s in [int(x) for x in a.seeds.split(",")]:
        m.reset()
        wall = m.run_simulation(seed=s)
        L.grmo_idxstat(buf, 1)
        tot += np.array(list(buf), dtype=np.float64)
        print(f"seed {s}: {wall:.1f} s, counters {m.counters()}", flush=True)
    hc_prev, k2_prev = tot[1], tot[9]
    r = {
        "hc_lookups": tot[7], "hc_table_frac": tot[0] / tot[7], "hc_with_prev": hc_prev / tot[7],
        "hc_same_cell": tot[2] / hc_prev, "hc_within_1": tot[3] / hc_prev, "hc_same_w_row": tot[4] / hc_prev,
        "hc_same_theta_col": tot[5] / hc_prev, "hc_w_pm1_theta_same": tot[6] / hc_prev,
        "k2_lookups": tot[12], "k2_table_frac": tot[8] / tot[12], "k2_same": tot[10] / k2_prev,
        "k2_within_1": tot[11] / k2_prev,
    }
    # a lookup hits when the photon had a table cell before and the cell is the same (both tables)
    p_exact = (tot[2] / tot[7]) * (r["k2_same"])
    p_nbhd = (tot[3] / tot[7]) * (r["k2_within_1"])
    r["p_lane_hit_exact"] = p_exact
    r["p_lane_hit_3x3"] = p_nbhd
    for n in [int(x) for x in a.lanes.split(",")]:
        r[f"p_wave_all_hit_exact_{n}"] = p_exact ** n
        r[f"p_wave_all_hit_3x3_{n}"] = p_nbhd ** n
    for k, v in r.items():
        print(f"{k:28s} {v:.6g}")
    if a.out:
        json.dump(dict(photon_n=a.photon_n, seeds=a.seeds, raw=tot.tolist(), **r), open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
