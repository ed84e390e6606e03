"""bench.py -- superphotons/s of the MI355X transport engine on the dump019-sized config.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--photon-n 1e6] [--grid 192]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): dump019 at photon_n = 1e6, mass_unit = 4e19.  dump019 is not
available offline, so a deterministic synthetic HARM dump of dump019's class (192x192 MKS torus,
a = 0.9375) is generated (cuda-grmonty_amd/grmonty_amd/synth_dump.py) -- "data": "synthetic".
One step = one run_simulation pass: the emitted superphotons (already resident in HBM) are tracked
to completion (children included), spectrum and counters reduced.  Multi-GPU: one process per GPU,
each rank tracks its own photon_n = 1e6 shard (emission seed 123 + rank, disjoint Philox keys) --
weak scaling; the only collective is the RCCL all-reduce of the 6x200x13 fp64 spectrum + counters.

value = superphotons (the reference's "created", harm_model.cpp:407-409) processed by all ranks /
max-over-ranks wall time of the timed steps.
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

ALG_BYTES_PER_STEP = 304  # HARM gather 8x4x8 + hotcross 4x8 + K2 2x8
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
FP64_VECTOR_PEAK_TFLOPS = 78.6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--photon-n", type=float, default=1e6)
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--dump", default="", help="HARM dump to use (default: synthetic dump019-class)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--pmc-summary", default=os.environ.get("GRM_PMC_SUMMARY", ""),
                    help="rocprofv3 counter CSV to fill roofline.traffic")
    return ap.parse_args()


def host_threads(world: int) -> int:
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if n <= 0:
        n = min(16, os.cpu_count() or 1)
    return max(1, n // max(1, world) if world > 1 else n)


def cpu_baseline(model_path: str, photon_n: int, photons: np.ndarray, seconds: float):
    """Oracle (single-thread C++ restatement of the reference CPU path) on a bounded sample of the
    same emitted photons, reference semantics (mt19937, live adaptive bias)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle_py as O
    m = O.OracleModel(model_path, photon_n=photon_n)
    m.init(host_threads(1))
    rng = np.random.default_rng(0)
    order = rng.permutation(len(photons))
    done, t0, chunk = 0, time.time(), 256
    while time.time() - t0 < seconds and done < len(order):
        sel = photons[order[done:done + chunk]]
        m.track(sel.view(O.INIT_PHOTON), rng_mode=0, seed=123, frozen=False)
        done += len(sel)
    dt = time.time() - t0
    return {"value": done / dt, "unit": "superphotons/s", "cores": 1, "kind": "port",
            "sample": f"{done} of the {len(photons)} emitted superphotons (random subset), tracked by the "
                      f"oracle (oracle/grmonty_oracle.cpp, reference CPU semantics: serial, mt19937, live bias) "
                      f"in {dt:.1f}s on 1 host core"}


def pmc_traffic(path: str, launches_per_step: float):
    """HBM bytes per step from a rocprofv3 --pmc FETCH_SIZE/WRITE_SIZE counter CSV (KB units;
    gfx950 FETCH_SIZE counts half of wide streaming reads -> doubled, MI355X_MICROARCH.md §HBM)."""
    if not path or not os.path.exists(path):
        return None
    import csv
    tot = {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0}
    n = 0
    with open(path) as f:
        for row in csv.DictReader(f):
            if "track_kernel" not in row.get("Kernel_Name", ""):
                continue
            name = row.get("Counter_Name", "")
            if name in tot:
                tot[name] += float(row.get("Counter_Value", 0))
                n += 1
    if n == 0:
        return None
    return (2.0 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024.0


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import grmonty_amd as G
    from grmonty_amd.synth_dump import ensure_dump

    photon_n = int(args.photon_n)
    threads = args.threads or host_threads(world)
    if args.dump:
        path = args.dump
    else:
        path = os.path.join(REPO, "gpurun_out" if os.path.isdir(os.path.join(REPO, "gpurun_out")) else ".",
                            f"synth{args.grid}_r{rank}.dump")
        ensure_dump(path, args.grid, args.grid)
    t = time.time()
    model = G.Model.load(path, photon_n=photon_n).init(threads)
    t_init = time.time() - t
    t = time.time()
    photons = model.emit(seed=123 + rank, threads=threads)
    t_emit = time.time() - t
    engine = G.Engine(model, device=local)
    engine.set_option(G.OPT_SEED, 0x5EED0000 + rank)
    # inputs resident in HBM before the timed region
    import torch
    dev = torch.device("cuda", local)
    d_ph = torch.from_numpy(photons.view(np.uint8)).to(dev)
    torch.cuda.synchronize(dev)
    n = len(photons)

    def step():
        engine.reset()
        engine.track_device(d_ph.data_ptr(), n)
        spec, n_rec, n_scatt, max_tau = engine.finish()
        st = engine.stats()
        if dist is not None:
            s = torch.from_numpy(spec.view(np.float64).reshape(-1).copy()).to(dev)
            c = torch.tensor([float(n), float(n_rec), float(n_scatt), float(st["n_steps"])], dtype=torch.float64,
                             device=dev)
            m = torch.tensor([max_tau], dtype=torch.float64, device=dev)
            dist.all_reduce(s)
            dist.all_reduce(c)
            dist.all_reduce(m, op=dist.ReduceOp.MAX)
        return st

    for _ in range(args.warmup):
        step()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.time()
    kern_ms, steps_tot, tracked, children, launches = 0.0, 0, 0, 0, 0
    for _ in range(args.steps):
        st = step()
        kern_ms += st["last_kernel_ms"]
        steps_tot += st["last_steps"]
        tracked += st["n_tracked"]
        children += st["n_children"]
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    elapsed = time.time() - t0
    launches = engine.stats()["n_launches"]
    tmax = elapsed
    total_photons = n * args.steps
    if dist is not None:
        tt = torch.tensor([elapsed, float(total_photons)], dtype=torch.float64, device=dev)
        tm = tt.clone()
        dist.all_reduce(tm[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        tmax = float(tm[0])
        total_photons = int(tt[1])
    if rank == 0:
        ms_per_launch_step = kern_ms / args.steps
        alg_bytes = steps_tot / args.steps * ALG_BYTES_PER_STEP
        achieved = alg_bytes / (ms_per_launch_step * 1e-3) / 1e9
        traffic = pmc_traffic(args.pmc_summary, launches / max(1, args.steps + args.warmup))
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            try:
                cpu = cpu_baseline(path, photon_n, photons, args.cpu_seconds)
            except Exception as ex:  # the baseline is reported, never the product path
                cpu = {"value": None, "error": str(ex)}
        out = {
            "metric": "superphotons/sec on dump019-class HARM dump (photon_n=1e6)",
            "value": total_photons / tmax,
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
                                   f"{photon_n:g} per GPU ({n} emitted superphotons/GPU/step), mass_unit=4e19",
                       "photon_n": photon_n, "grid": f"{args.grid}x{args.grid}", "superphotons_per_gpu": n,
                       "parallelism": f"photon shards x{world} (weak), RCCL all-reduce of the spectrum"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": (traffic / max(1, args.steps + args.warmup)) if traffic else None,
                         "note": f"algorithmic {ALG_BYTES_PER_STEP} B per transport step x {steps_tot // args.steps} "
                                 f"steps per step-pass / track_kernel time {ms_per_launch_step:.1f} ms (HIP events); "
                                 f"the kernel is fp64-VALU/latency bound, see DESIGN.md"},
            "cpu_baseline": cpu,
            "detail": {"transport_steps_per_s": steps_tot / (kern_ms * 1e-3), "kernel_ms_per_step": ms_per_launch_step,
                       "tracked_per_step": tracked // args.steps, "children_per_step": children // args.steps,
                       "launches": launches, "init_s": t_init, "emit_s": t_emit},
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
