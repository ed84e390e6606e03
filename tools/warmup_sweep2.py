"""Counter systematic of the live adaptive bias vs the warm-up admission size (GRM_OPT_WARMUP) and
the emulated rank count, on the 192^2 dump: N jobs of distinct seeds per setting, means printed with
the oracle fixtures' means beside them, plus the pass time.

    python tools/warmup_sweep2.py [--photon-n 1e5] [--seeds 16] [--warmups 4096,16384,65536,-1] [--worlds 1]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "cuda-grmonty_amd"), os.path.join(REPO, "tests")]
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402
from job_util import KEYS, run_job  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--photon-n", type=float, default=1e5)
    ap.add_argument("--seeds", type=int, default=16)
    ap.add_argument("--warmups", default="4096,16384,65536,-1")
    ap.add_argument("--worlds", default="1")
    ap.add_argument("--golden", default="oracle_synth192_pn1e5")
    args = ap.parse_args()
    path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
    model = G.Model.load(path, photon_n=int(args.photon_n)).init(8, device=0)
    eng = G.Engine(model, device=0)
    eng.emit_setup(model)
    gp = os.path.join(REPO, "tests", "golden", args.golden + ".json")
    if os.path.exists(gp):
        runs = json.load(open(gp))["runs"]
        print("oracle  " + "  ".join(f"{k} {np.mean([r[k] for r in runs]):.5g}+-{np.std([r[k] for r in runs], ddof=1):.3g}"
                                    for k in KEYS) + f"  ({len(runs)} runs)", flush=True)
    for world in [int(w) for w in args.worlds.split(",")]:
        shards = G.zone_shards(model.zone_weights(), world)
        for wu in [int(w) for w in args.warmups.split(",")]:
            eng.set_option(G.OPT_WARMUP, wu)
            vals = {k: [] for k in KEYS}
            ts = []
            for s in range(args.seeds):
                t = time.time()
                job = run_job(eng, model, 123 + s, shards=shards)
                ts.append(time.time() - t)
                for k in KEYS:
                    vals[k].append(job[k])
            print(f"world {world} warmup {wu:6d}  " + "  ".join(
                f"{k} {np.mean(vals[k]):.5g}+-{np.std(vals[k], ddof=1) / np.sqrt(len(vals[k])):.2g}" for k in KEYS) +
                f"  job s median {np.median(ts):.3f} mean {np.mean(ts):.3f}", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
