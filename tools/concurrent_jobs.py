"""W independent single-GPU jobs (full photon_n = 1e5 run_simulation passes, distinct seeds, own
counters) running CONCURRENTLY on one GPU, each engine on 256 / W workgroups (then the live-bias
flight cap): does sharing the GPU with other engines move a job's live-bias counters?  Compared with
the 1e5 oracle fixture.

    python tools/concurrent_jobs.py W ROUNDS [K=V ...]
"""
import json
import os
import sys
import threading

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "cuda-grmonty_amd")]
from job_util import KEYS, run_job  # noqa: E402
from spectrum_stats import welch_z  # noqa: E402


def main():
    import grmonty_amd as G
    from grmonty_amd.synth_dump import ensure_dump
    world, rounds = int(sys.argv[1]), int(sys.argv[2])
    opts = [kv.split("=") for kv in sys.argv[3:]]
    path = ensure_dump(os.path.join(R, "gpurun_out", "synth192.dump"), 192, 192)
    model = G.Model.load(path, photon_n=100000).init(8, device=0)
    engines = []
    for r in range(world):
        e = G.Engine(model, device=0)
        e.set_option(G.OPT_GRID_BLOCKS, max(1, 256 // world))
        for k, v in opts:
            e.set_option(int(k), int(v))
        e.emit_setup(model)
        engines.append(e)
    jobs = []
    for s in range(rounds):
        out = [None] * world
        go = threading.Barrier(world)

        def one(r):
            go.wait()
            out[r] = run_job(engines[r], model, 123 + s * world + r)

        th = [threading.Thread(target=one, args=(r,)) for r in range(world)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        jobs += out
    for e in engines:
        e.close()
    summ = json.load(open(os.path.join(R, "tests", "golden", "oracle_synth192_pn1e5.json")))
    o = {k: np.array([x[k] for x in summ["runs"]], dtype=np.float64) for k in KEYS}
    line = f"{world} concurrent independent jobs x {rounds} rounds {sys.argv[3:]}:"
    for k in KEYS:
        diff, se, z = welch_z([j[k] for j in jobs], o[k])
        line += f"  {k} {diff / o[k].mean():+.2%} ({z:+.1f} SE)"
    print(line, flush=True)


if __name__ == "__main__":
    main()
