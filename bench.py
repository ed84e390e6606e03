"""bench.py -- superphotons/s of the MI355X transport engine on the dump019-class config.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--photon-n 1e6] [--grid 192]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): dump019 at photon_n = 1e6, mass_unit = 4e19.  dump019 is not
available offline, so a deterministic synthetic HARM dump of dump019's class (192x192 MKS torus,
a = 0.9375; cuda-grmonty_amd/grmonty_amd/synth_dump.py) is used -- "data": "synthetic".
A step = one run_simulation pass: every emitted superphoton (already resident in HBM) is tracked to
completion (scattered children included), then spectrum + counters are reduced.

Multi-GPU (weak scaling): N ranks run ONE job of photon_n x N whose zones are split into N
contiguous ranges of equal expected photon count; zone emission streams and photon stream ids are
global, so the union of the shards is exactly the single-GPU job's photon list.  The only exchange
is the RCCL all-reduce (xGMI) of the 6x200x13 fp64 spectrum + counters, issued by the engine's C
library on its own HIP stream.  torch.distributed is used with the gloo backend only (rendezvous,
RCCL unique-id broadcast, barriers, max-over-ranks timing): torch's bundled HIP runtime is never
initialised, because a second HIP runtime in the process cannot open the GPU.  Every engine call
returns after its stream has synchronised, so the barriers bracket finished device work.

value = superphotons emitted by all ranks (the reference's "created", harm_model.cpp:407-409) per
second of max-over-ranks wall time of the K timed steps.
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
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--photon-n", type=float, default=1e6, help="photon_n per GPU")
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--dump", default="", help="HARM dump to use (default: synthetic dump019-class)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--pmc-summary", default=os.environ.get("GRM_PMC_SUMMARY", ""),
                    help="rocprofv3 --pmc counter CSV (FETCH_SIZE/WRITE_SIZE) to fill roofline.traffic")
    return ap.parse_args()


def host_threads(world: int) -> int:
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if n <= 0:
        n = min(16, os.cpu_count() or 1)
    return max(1, n // world) if world > 1 else n


def cpu_baseline(path: str, photon_n: int, photons: np.ndarray, seconds: float):
    """The oracle (single-thread C++ restatement of the reference CPU path; reference semantics:
    serial, mt19937, live adaptive bias) on a bounded random sample of the same photons."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O
    m = O.OracleModel(path, photon_n=photon_n)
    m.init(host_threads(1))
    order = np.random.default_rng(0).permutation(len(photons))
    done, t0, chunk = 0, time.time(), 256
    while time.time() - t0 < seconds and done < len(order):
        sel = np.ascontiguousarray(photons[order[done:done + chunk]]).view(O.INIT_PHOTON)
        m.track(sel, rng_mode=0, seed=123, frozen=False)
        done += len(sel)
    dt = time.time() - t0
    return {"value": done / dt, "unit": "superphotons/s", "cores": 1, "kind": "port",
            "sample": f"{done} of the {len(photons)} emitted superphotons (random subset) tracked by the oracle "
                      f"(oracle/grmonty_oracle.cpp: serial reference CPU semantics, mt19937, live bias) in "
                      f"{dt:.1f} s on 1 host core"}


def pmc_traffic(path: str):
    """HBM bytes of all track_kernel dispatches in a rocprofv3 --pmc CSV (FETCH_SIZE/WRITE_SIZE in KB;
    gfx950 FETCH_SIZE reports half of wide streaming reads -> doubled, MI355X_MICROARCH.md §HBM)."""
    if not path or not os.path.exists(path):
        return None
    import csv
    tot = {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0}
    seen = False
    with open(path) as f:
        for row in csv.DictReader(f):
            if "track_kernel" in row.get("Kernel_Name", "") and row.get("Counter_Name") in tot:
                tot[row["Counter_Name"]] += float(row.get("Counter_Value", 0))
                seen = True
    return (2.0 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024.0 if seen else None


def main():
    args = parse()
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
    engine = G.Engine(model, device=local)
    engine.set_option(G.OPT_SEED, 123)
    if world > 1:
        uid = [G.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        engine.comm_init(uid[0], world, rank)
    d_ph = engine.upload(photons)  # inputs resident in HBM before the timed region

    def step():
        engine.reset()
        engine.set_option(G.OPT_ID_BASE, id_base)
        engine.track_device(d_ph, n)
        st = engine.stats()
        if world > 1:
            engine.allreduce()
        spec, n_rec, n_scatt, max_tau = engine.finish()
        return st, n_rec, n_scatt

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    t0 = time.time()
    kern_ms, steps_tot, tracked, children = 0.0, 0, 0, 0
    for _ in range(args.steps):
        st, n_rec, n_scatt = step()
        kern_ms += st["last_kernel_ms"]
        steps_tot += st["last_steps"]
        tracked += st["n_tracked"]
        children += st["n_children"]
    if dist is not None:
        dist.barrier()
    elapsed = time.time() - t0
    launches = engine.stats()["n_launches"]
    tmax, total = elapsed, n * args.steps
    if dist is not None:
        tm = torch.tensor([elapsed], dtype=torch.float64)
        tt = torch.tensor([float(total)], dtype=torch.float64)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        tmax, total = float(tm[0]), int(tt[0])
    if rank == 0:
        k_ms = kern_ms / args.steps
        achieved = steps_tot / args.steps * ALG_BYTES_PER_STEP / (k_ms * 1e-3) / 1e9
        traffic = pmc_traffic(args.pmc_summary)
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            try:
                cpu = cpu_baseline(path, photon_n_job, photons, args.cpu_seconds)
            except Exception as ex:  # the baseline is reported beside the product, never part of it
                cpu = {"value": None, "error": repr(ex)}
        out = {
            "metric": "superphotons/sec on dump019-class HARM dump (photon_n=1e6 per GPU)",
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
                         "traffic": traffic / max(1, args.steps + args.warmup) if traffic else None,
                         "note": f"{ALG_BYTES_PER_STEP} algorithmic B per transport step x {steps_tot // args.steps} "
                                 f"steps per pass / {k_ms:.1f} ms of track_kernel (HIP events on the engine stream); "
                                 f"the kernel is fp64-VALU/latency bound -- DESIGN.md"},
            "cpu_baseline": cpu,
            "detail": {"transport_steps_per_s": steps_tot / (kern_ms * 1e-3), "kernel_ms_per_step": k_ms,
                       "tracked_per_step": tracked // args.steps, "children_per_step": children // args.steps,
                       "launches_total": launches, "init_s": t_init, "emit_s": t_emit},
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
