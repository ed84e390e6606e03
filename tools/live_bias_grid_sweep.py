"""Live-bias run_simulation passes on the device at several grid sizes (photons in flight): if the
counter offset against the oracle is the concurrency lag it must shrink with the grid; if it stays,
it is not the lag.  192^2 dump, photon_n 1e5, device emission, host tables.

    python tools/live_bias_grid_sweep.py --grids 8,64,256 --seeds 123-138 --out gpurun_out/x.jsonl
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def seeds_of(s):
    out = []
    for part in s.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="8,64,256")
    ap.add_argument("--seeds", default="123-138")
    ap.add_argument("--photon-n", type=float, default=1e5)
    ap.add_argument("--grid-n", type=int, default=192)
    ap.add_argument("--opts", default="", help="engine options k=v,k=v (grmonty_amd.OPT_*)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import grmonty_amd as G
    from grmonty_amd.synth_dump import ensure_dump
    from job_util import run_job
    d = os.path.join(REPO, "gpurun_out") if os.path.isdir(os.path.join(REPO, "gpurun_out")) else "/tmp"
    path = ensure_dump(os.path.join(d, f"synth{a.grid_n}.dump"), a.grid_n, a.grid_n)
    model = G.Model.load(path, photon_n=int(a.photon_n)).init(8)
    f = open(a.out, "a") if a.out else None
    for g in [int(x) for x in a.grids.split(",")]:
        eng = G.Engine(model, device=0)
        eng.emit_setup(model)
        eng.set_option(G.OPT_GRID_BLOCKS, g)
        for kv in filter(None, a.opts.split(",")):
            k, v = kv.split("=")
            eng.set_option(int(k), int(v))
        for s in seeds_of(a.seeds):
            t = time.time()
            j = run_job(eng, model, s)
            r = dict(grid=g, seed=s, opts=a.opts, wall_s=round(time.time() - t, 3),
                     **{k: j[k] for k in ("created", "recorded", "scattered", "steps", "luminosity", "max_tau")})
            print(json.dumps(r), flush=True)
            if f:
                f.write(json.dumps(r) + "\n")
                f.flush()
        eng.close()


if __name__ == "__main__":
    main()
