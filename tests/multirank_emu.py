"""N-rank job emulated on ONE GPU, ranks running concurrently (run as its own process, so that the
HIP runtime starts with enough hardware queues for N concurrent engines: GPU_MAX_HW_QUEUES).

Each emulated rank is an engine with 1/N of the CUs (GRM_OPT_GRID_BLOCKS), the zone shard bench.py
gives rank r (grmonty_amd.zone_shards: every N-th zone from r), its global photon id base, and its
own counter block per pass; with --shared the blocks are linked (grm_engine_link_peers), so every
rank's adaptive bias runs on the job's counters as on N GPUs with grm_engine_set_peers.  The N
passes of a seed start together from N host threads (each rank's emission, a barrier, then the
transport launches, which also wait for each other at the job's device-side start barrier); the job's
results are the ranks' sums.

    python tests/multirank_emu.py DUMP WORLD SEEDS OUT.json [--shared] [--photon-n 1e5]
"""
import argparse
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(os.path.dirname(HERE), "cuda-grmonty_amd"), HERE]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dump")
    ap.add_argument("world", type=int)
    ap.add_argument("seeds", type=int)
    ap.add_argument("out")
    ap.add_argument("--shared", action="store_true")
    ap.add_argument("--photon-n", type=float, default=1e5)
    ap.add_argument("--seed0", type=int, default=123)
    ap.add_argument("--sequential", action="store_true", help="ranks one after another (experiments)")
    ap.add_argument("--phases", action="store_true", help="per-rank launch phases (diagnostics)")
    ap.add_argument("--opt", action="append", default=[], help="engine option K=V (grmonty_amd.OPT_*), experiments")
    args = ap.parse_args()
    import numpy as np
    import grmonty_amd as G
    world = args.world
    model = G.Model.load(args.dump, photon_n=int(args.photon_n)).init(8, device=0)
    shards = G.zone_shards(model.zone_weights(), world)
    engines = []
    for r in range(world):
        e = G.Engine(model, device=0)
        e.set_option(G.OPT_GRID_BLOCKS, max(1, 256 // world))
        # the ranks' launches queue behind each other on the one GPU: the job's device-side start
        # barrier keeps every rank in the job's warm-up (on N GPUs launched together it is not needed)
        if not args.sequential:  # ranks run one after another there: nothing to wait for
            e.set_option(G.OPT_JOB_START_WAIT_MS, 500)
        for kv in args.opt:
            k, v = kv.split("=")
            e.set_option(int(k), int(v))
        e.emit_setup(model)
        e.stash_reserve(args.seeds)
        engines.append(e)
    if args.shared:
        G.link_peers(engines)
    res = []
    for s in range(args.seeds):
        seed = args.seed0 + s
        counts = [model.count(seed=seed, z0=a, z1=b, stride=st) for a, b, st in shards]
        out = [None] * world
        err = []
        go = threading.Barrier(world)

        def rank(r):
            try:
                e = engines[r]
                e.begin_pass(s)
                e.set_option(G.OPT_SEED, seed)
                e.set_option(G.OPT_ID_BASE, int(sum(counts[:r])))
                a, b, st = shards[r]
                # every rank's emission first, then the transport launches together: on one GPU a
                # rank's emission queued behind the others' transport launches started its warm-up
                # after the job's had ended (8 ranks, photon_n = 1e8: two ranks, round 5).  The
                # launches also meet at the job's device-side start barrier (job_started).
                p, n = e.emit(seed=seed, z0=a, z1=b, stride=st)
                go.wait()
                e.track_device(p, n)
                stt = e.stats()
                if stt["n_dropped"] or stt["n_abandoned"]:
                    raise RuntimeError("photons lost")
                spec, nr, ns, mt = e.finish()
                out[r] = dict(spec=spec, created=n, recorded=nr, scattered=ns, steps=stt["n_steps"], max_tau=mt,
                              rec_spec=float(spec["nph"].sum()), scatt_spec=float(spec["nscatt"].sum()),
                              n_early=stt["n_early"],
                              phases=e.debug_phases() if args.phases else None)
            except Exception as ex:  # reported below
                err.append(repr(ex))
                go.abort()

        wall = None
        if args.sequential:  # each rank's pass alone, in rank order (no barrier)
            go = threading.Barrier(1)
            for r in range(world):
                rank(r)
        else:
            th = [threading.Thread(target=rank, args=(r,)) for r in range(world)]
            t0 = time.time()
            for t in th:
                t.start()
            for t in th:
                t.join()
            wall = time.time() - t0
        if err:
            raise RuntimeError(err[0])
        spec = out[0]["spec"].copy()
        for o in out[1:]:
            for f in spec.dtype.names:
                spec[f] += o["spec"][f]
        job = {k: int(sum(o[k] for o in out)) for k in ("created", "recorded", "scattered", "steps")}
        job["luminosity"] = model.write_spectrum(spec, None)["luminosity"]
        job["wall_s"] = wall  # the ranks' passes, emission to read-back (concurrent runs only)
        # every rank's view of the job's counters once all passes ended (the kernels' bias_den path):
        # must be the sums of the ranks' own counters and the max of their max tau_scatt
        job["max_tau"] = max(o["max_tau"] for o in out)
        job["job_view"] = [e.job_counters() for e in engines] if args.shared else None
        job["per_rank_recorded"] = [o["recorded"] for o in out]
        job["per_rank_created"] = [o["created"] for o in out]
        job["per_rank_scattered"] = [o["scattered"] for o in out]
        job["per_rank_n_early"] = [o["n_early"] for o in out]
        if args.phases:
            job["per_rank_phases"] = [o["phases"] for o in out]
        # the spectrum's own sums (independent of the counter blocks)
        job["rec_spec"] = sum(o["rec_spec"] for o in out)
        job["scatt_spec"] = sum(o["scatt_spec"] for o in out)
        res.append(job)
        print(json.dumps({k: v for k, v in job.items() if k != "job_view"}), flush=True)
    for e in engines:
        e.close()
    json.dump(res, open(args.out, "w"))


if __name__ == "__main__":
    main()
