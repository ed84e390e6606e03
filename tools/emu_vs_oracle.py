"""Counter means of emulated N-rank jobs (tests/multirank_emu.py output) against the oracle's runs of
the same photon_n (tests/golden/oracle_synth192_pn1e{5,6}.json): recorded / scattered / steps /
luminosity, Welch z per counter, and the jobs' wall times if recorded.

    python tools/emu_vs_oracle.py JOBS.json [JOBS2.json ...] --photon-n 1e6
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from spectrum_stats import welch_z  # noqa: E402

KEYS = ("recorded", "scattered", "steps", "luminosity")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("jobs", nargs="+")
    ap.add_argument("--photon-n", type=float, default=1e6)
    ap.add_argument("--pool", action="store_true", help="the files' jobs as one sample")
    a = ap.parse_args()
    tag = "pn1e6" if a.photon_n >= 1e6 else "pn1e5"
    o = json.load(open(os.path.join(REPO, "tests", "golden", f"oracle_synth192_{tag}.json")))["runs"]
    sets = [(p, json.load(open(p))) for p in a.jobs]
    if a.pool:
        sets = [(" + ".join(a.jobs), [j for _, js in sets for j in js])]
    for path, jobs in sets:
        print(f"{path}: {len(jobs)} jobs vs {len(o)} oracle runs")
        for k in KEYS:
            dev = np.array([j[k] for j in jobs], dtype=np.float64)
            ref = np.array([r[k] for r in o], dtype=np.float64)
            diff, se, z = welch_z(dev, ref)
            print(f"  {k:10s} {dev.mean():.6g} +- {dev.std(ddof=1):.3g}  oracle {ref.mean():.6g} +- "
                  f"{ref.std(ddof=1):.3g}  diff {diff / ref.mean():+.2%} = {z:+.2f} SE")
        wall = [j.get("wall_s") for j in jobs if j.get("wall_s")]
        if wall:
            created = np.mean([j["created"] for j in jobs])
            print(f"  job wall {np.mean(wall):.3f} s (median {np.median(wall):.3f}) -> "
                  f"{created / np.mean(wall) / 1e6:.2f} M superphotons/s")


if __name__ == "__main__":
    main()
