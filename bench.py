"""bench.py -- superphotons/s of the MI355X transport engine on the dump019-class config.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--photon-n 1e6] [--grid 192]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): dump019 at photon_n = 1e6, mass_unit = 4e19.  dump019 is not
available offline, so a deterministic synthetic HARM dump of dump019's class (192x192 MKS torus,
a = 0.9375; cuda-grmonty_amd/grmonty_amd/synth_dump.py) is used -- "data": "synthetic".
A step = one run_simulation pass (harm_model.cpp:340-414) on the GPU: the superphotons are emitted on
the device from the zone table already resident in HBM (grm_engine_emit: zone counts, scan,
sample_zone_photon), every one of them is tracked to completion (scattered children included), then
spectrum + counters are reduced.  `--host-emit` instead times transport only, over photons emitted
on the host and uploaded before the timed region (the previous definition of a step).

Passes in flight (--jobs, default 4): each pass runs on its own engine (stream, buffers, spectrum,
counters, bias state) from its own host thread.  A pass ends with a few long-lived superphotons
(polar Zeno-stepping or full-depth step halving, up to ~1e6 serial push attempts, one lane on one
CU); the next passes' photons fill the other CUs meanwhile.  Every pass is complete; value is the
sustained rate of back-to-back passes, and detail.single_pass_rate / pass_latency_s report one pass
alone.

Multi-GPU (weak scaling): N ranks run ONE job of photon_n x N whose zones are split into N
contiguous ranges of equal expected photon count; zone emission streams and photon stream ids are
global, so the union of the shards is exactly the single-GPU job's photon list.  The only exchange
is the RCCL all-reduce (xGMI) of the 6x200x13 fp64 spectrum + counters, issued by the engine's C
library on its own HIP stream.  torch.distributed is used with the gloo backend only (rendezvous,
RCCL unique-id broadcast, barriers, max-over-ranks timing): torch's bundled HIP runtime is never
initialised, because a second HIP runtime in the process cannot open the GPU.  Every engine call
returns after its stream has synchronised, so the barriers bracket finished device work.

value = superphotons emitted by all ranks (the reference's "created", harm_model.cpp:407-409) per
second of max-over-ranks wall time of the K timed steps -- the reference's "Final rate" window
(emission + transport, tables already built).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402  (load the engine's HIP runtime before anything else)
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

ALG_BYTES_PER_STEP = 304  # per transport step: HARM gather 8x4x8 + hotcross 4x8 + K2 2x8
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--photon-n", type=float, default=1e6, help="photon_n per GPU")
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--dump", default="", help="HARM dump to use (default: synthetic dump019-class)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--jobs", type=int, default=16,
                    help="run_simulation passes in flight per GPU (engines with their own streams and buffers)")
    ap.add_argument("--host-emit", action="store_true",
                    help="emit on the host, upload before timing, time transport only")
    ap.add_argument("--pmc-summary", default=os.environ.get("GRM_PMC_SUMMARY", ""),
                    help="rocprofv3 --pmc counter CSVs, comma-separated (FETCH_SIZE pass, WRITE_SIZE pass) "
                         "of this same command, to fill roofline.traffic")
    return ap.parse_args()


def host_threads(world: int) -> int:
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if n <= 0:
        n = min(16, os.cpu_count() or 1)
    return max(1, n // world) if world > 1 else n


def cpu_baseline(path: str, photon_n: int, photons: np.ndarray, seconds: float):
    """The oracle (single-thread C++ restatement of the reference CPU path; reference semantics:
    serial, mt19937, live adaptive bias) on a bounded random sample of the same photons, plus the
    oracle's emission (zone walk + sample_zone_photon) timed on a random sample of zones: the CPU
    cost of one superphoton = emission + transport, as in the reference's run_simulation."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O
    m = O.OracleModel(path, photon_n=photon_n)
    m.init(host_threads(1))
    rng = np.random.default_rng(0)
    order = rng.permutation(len(photons))
    done, t0, chunk = 0, time.time(), 256
    while time.time() - t0 < seconds and done < len(order):
        sel = np.ascontiguousarray(photons[order[done:done + chunk]]).view(O.INIT_PHOTON)
        m.track(sel, rng_mode=0, seed=123, frozen=False)
        done += len(sel)
    t_track = time.time() - t0
    h = m.header
    zones = rng.permutation(h.n[0] * h.n[1])
    n_em, t0 = 0, time.time()
    for z in zones:
        n_em += len(m.emit_philox(seed=123, z0=int(z), z1=int(z) + 1))
        if time.time() - t0 > max(1.0, 0.1 * seconds):
            break
    t_emit = time.time() - t0
    per = t_track / max(done, 1) + t_emit / max(n_em, 1)
    return {"value": 1.0 / per, "unit": "superphotons/s", "cores": 1, "kind": "port",
            "sample": f"{done} of the {len(photons)} emitted superphotons (random subset) tracked in {t_track:.1f} s "
                      f"+ {n_em} superphotons emitted from random zones in {t_emit:.1f} s by the oracle "
                      f"(oracle/grmonty_oracle.cpp: serial reference CPU semantics, mt19937, live bias) on 1 "
                      f"host core"}


def pmc_traffic(path: str, k: int):
    """HBM bytes per dominant track_kernel dispatch from rocprofv3 --pmc counter CSVs (FETCH_SIZE and
    WRITE_SIZE in KB, from separate passes; gfx950 FETCH_SIZE reports half of wide streaming reads ->
    doubled, MI355X_MICROARCH.md §HBM).  `path` = comma-separated CSVs; mean over the dominant
    dispatches (one per pass)."""
    if not path:
        return None
    import csv
    per = {"FETCH_SIZE": {}, "WRITE_SIZE": {}}
    for f in path.split(","):
        if not os.path.exists(f):
            return None
        with open(f) as fh:
            for row in csv.DictReader(fh):
                c = row.get("Counter_Name")
                if "track_kernel" in row.get("Kernel_Name", "") and c in per:
                    d = row.get("Dispatch_Id", "0")
                    per[c][d] = per[c].get(d, 0.0) + float(row.get("Counter_Value", 0))
    if not per["FETCH_SIZE"] or not per["WRITE_SIZE"]:
        return None
    # the dominant launches of the profiled run (the warm-up launches are a thousand times smaller)
    ids = [d for d in per["FETCH_SIZE"] if d in per["WRITE_SIZE"]]
    tot = {d: 2.0 * per["FETCH_SIZE"][d] + per["WRITE_SIZE"][d] for d in ids}
    big = [v for v in tot.values() if v >= 0.1 * max(tot.values())]
    return float(np.mean(big)) * 1024.0


def main():
    args = parse()
    # one hardware queue per engine (+1): a pass's long-lived last photons keep its kernel running on
    # a CU or two, and a kernel queued behind it on a shared hardware queue would wait for it.  HIP
    # reads this when its runtime starts (the first engine call below); 4 is the box default.
    os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(4, args.jobs + 1)))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
    threads = args.threads or host_threads(world)
    photon_n_job = int(args.photon_n) * world
    path = args.dump or os.path.join(REPO, "gpurun_out" if os.path.isdir(os.path.join(REPO, "gpurun_out")) else ".",
                                     f"synth{args.grid}_r{rank}.dump")
    if not args.dump:
        ensure_dump(path, args.grid, args.grid)
    t = time.time()
    model = G.Model.load(path, photon_n=photon_n_job).init(threads)
    t_init = time.time() - t
    shards = G.shard_zones(model.zone_weights(), world)
    z0, z1 = shards[rank]
    counts = [model.count(seed=123, z0=a, z1=b, threads=threads) for a, b in shards]
    t = time.time()
    photons = model.emit(seed=123, z0=z0, z1=z1, threads=threads)
    t_emit = time.time() - t
    n = len(photons)
    assert n == counts[rank]
    id_base = int(sum(counts[:rank]))
    # HBM per engine: the emitted batch (128 B per superphoton) + two overflow pools (2 x n/4 x 208 B)
    # + lane stacks; keep the engines of one GPU within ~200 GB of its 288 GB
    per_engine = n * (128 + 104) + 0.5e9
    jobs = max(1, min(args.jobs, int(200e9 // per_engine)))
    engines = [G.Engine(model, device=local) for _ in range(jobs)]
    for engine in engines:
        engine.set_option(G.OPT_SEED, 123)
    if world > 1:  # one RCCL communicator per concurrent pass; pass s uses engine s % jobs on every rank
        uid = [[G.rccl_unique_id() for _ in range(jobs)] if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        for engine, u in zip(engines, uid[0]):
            engine.comm_init(u, world, rank)
    # inputs resident in HBM before the timed region: the zone table (device emission) or the
    # host-emitted photons (--host-emit)
    for engine in engines:
        engine.emit_setup(model)
    d_ph = [engine.upload(photons) for engine in engines] if args.host_emit else None

    import threading
    ar_turn = [0]
    ar_cv = threading.Condition()
    AR_ABORT = 1 << 60

    def allreduce_in_order(engine, s_):
        """every rank issues pass s_'s collective after passes < s_ (one global order for RCCL)"""
        with ar_cv:
            ar_cv.wait_for(lambda: ar_turn[0] == s_ or ar_turn[0] >= AR_ABORT)
            if ar_turn[0] >= AR_ABORT:
                raise RuntimeError("another pass failed")
        try:
            engine.allreduce()
        finally:
            with ar_cv:
                ar_turn[0] += 1
                ar_cv.notify_all()

    def step(j, s_):
        """one run_simulation pass on engine j (its own stream, buffers, spectrum and counters)"""
        engine = engines[j]
        t = time.time()
        engine.reset()
        engine.set_option(G.OPT_ID_BASE, id_base)
        if args.host_emit:
            engine.track_device(d_ph[j], n)
        else:
            ptr, n_dev = engine.emit(seed=123, z0=z0, z1=z1)
            if n_dev != n:
                raise RuntimeError(f"device emission made {n_dev} superphotons, host count {n}")
            engine.track_device(ptr, n_dev)
        st = engine.stats()
        if world > 1:
            allreduce_in_order(engine, s_)
        spec, n_rec, n_scatt, max_tau = engine.finish()
        return st, n_rec, n_scatt, time.time() - t

    def run(n_steps):
        """n_steps passes, pass s on engine s % jobs; the engines' host threads run concurrently, so a
        pass's last long-lived superphoton (one lane on one CU) overlaps the next passes' work"""
        res = [None] * n_steps
        err = []
        ar_turn[0] = 0

        def worker(j):
            try:
                for s_ in range(j, n_steps, jobs):
                    res[s_] = step(j, s_)
            except Exception as ex:  # surfaced below
                err.append(ex)
                with ar_cv:  # do not leave the other threads waiting for this pass's collective
                    ar_turn[0] = AR_ABORT
                    ar_cv.notify_all()

        th = [threading.Thread(target=worker, args=(j,)) for j in range(min(jobs, n_steps))]
        for t_ in th:
            t_.start()
        for t_ in th:
            t_.join()
        if err:
            raise err[0]
        return res

    run(max(args.warmup, jobs))  # every engine warmed (buffers sized, code loaded)
    if dist is not None:
        dist.barrier()
    t0 = time.time()
    res = run(args.steps)
    if dist is not None:
        dist.barrier()
    elapsed = time.time() - t0
    kern_ms = sum(r[0]["last_kernel_ms"] for r in res)
    steps_tot = sum(r[0]["last_steps"] for r in res)
    tracked = sum(r[0]["n_tracked"] for r in res)
    children = sum(r[0]["n_children"] for r in res)
    emit_ms = 0.0 if args.host_emit else sum(r[0]["last_emit_ms"] for r in res)
    big_ms = sum(r[0]["max_launch_ms"] for r in res)
    big_steps = sum(r[0]["max_launch_steps"] for r in res)
    pass_s = sorted(r[3] for r in res)
    longest_life = max(r[0]["max_photon_steps"] for r in res)
    launches = sum(e_.stats()["n_launches"] for e_ in engines)
    tmax, total = elapsed, n * args.steps
    if dist is not None:
        tm = torch.tensor([elapsed], dtype=torch.float64)
        tt = torch.tensor([float(total)], dtype=torch.float64)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        tmax, total = float(tm[0]), int(tt[0])
    if rank == 0:
        k_ms = kern_ms / args.steps
        # per launch, for the dominant track_kernel launch of each step (rocprof's longest dispatches)
        achieved = big_steps * ALG_BYTES_PER_STEP / (big_ms * 1e-3) / 1e9
        traffic = pmc_traffic(args.pmc_summary, args.steps + max(args.warmup, jobs))
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            try:
                cpu = cpu_baseline(path, photon_n_job, photons, args.cpu_seconds)
            except Exception as ex:  # the baseline is reported beside the product, never part of it
                cpu = {"value": None, "error": repr(ex)}
        out = {
            "metric": "superphotons/sec on dump019-class HARM dump (photon_n=1e6 per GPU)"
                      + (" [transport only]" if args.host_emit else ""),
            "value": total / tmax,
            "unit": "superphotons/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": tmax / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"synthetic dump019-class {args.grid}x{args.grid} MKS HARM dump, photon_n="
                                   f"{int(args.photon_n):g} per GPU (one photon_n x {world} job zone-sharded), "
                                   f"mass_unit=4e19, {n} emitted superphotons on rank 0",
                       "photon_n_per_gpu": int(args.photon_n), "grid": f"{args.grid}x{args.grid}",
                       "superphotons_rank0": n, "parallelism": f"zone shards x{world}, RCCL spectrum all-reduce"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "achieved_sustained": steps_tot * ALG_BYTES_PER_STEP / tmax / 1e9,
                         "frac_sustained": steps_tot * ALG_BYTES_PER_STEP / tmax / 1e9 / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "note": f"dominant track_kernel launch: {ALG_BYTES_PER_STEP} algorithmic B per transport step x "
                                 f"{big_steps // args.steps} steps / {big_ms / args.steps:.1f} ms (HIP events on the "
                                 f"engine stream, {jobs} passes in flight); all launches of a step: "
                                 f"{steps_tot // args.steps} steps in {k_ms:.1f} ms; sustained over the timed window "
                                 f"{steps_tot * ALG_BYTES_PER_STEP / tmax / 1e9:.0f} GB/s; the kernel is "
                                 f"fp64-VALU/latency bound -- DESIGN.md"},
            "cpu_baseline": cpu,
            "detail": {"transport_steps_per_s": steps_tot / (kern_ms * 1e-3), "kernel_ms_per_step": k_ms,
                       "passes_in_flight": jobs,
                       "pass_latency_s": {"min": pass_s[0], "median": pass_s[len(pass_s) // 2], "max": pass_s[-1]},
                       "single_pass_rate": n / pass_s[len(pass_s) // 2],
                       "longest_photon_life_steps": longest_life,
                       "emit_ms_per_step": emit_ms / args.steps,
                       "emission": "host (untimed)" if args.host_emit else "device (timed)",
                       "tracked_per_step": tracked // args.steps, "children_per_step": children // args.steps,
                       "launches_total": launches, "init_s": t_init, "emit_s": t_emit},
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
