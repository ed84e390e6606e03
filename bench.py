"""bench.py -- superphotons/s of the MI355X transport engine on the dump019-class config.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--photon-n 1e6] [--grid 192] [--scaling weak|strong]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): dump019 at photon_n = 1e6, mass_unit = 4e19.  dump019 is not
available offline, so a deterministic synthetic HARM dump of dump019's class (192x192 MKS torus,
a = 0.9375; cuda-grmonty_amd/grmonty_amd/synth_dump.py) is used -- "data": "synthetic".

A step = ONE complete run_simulation pass (harm_model.cpp:340-414), run alone on the GPU: the
superphotons are emitted on the device from the zone table already resident in HBM (grm_engine_emit:
zone counts, scan, sample_zone_photon), every one of them is tracked to completion (scattered
children included), spectrum + counters are reduced (RCCL all-reduce across ranks) and read back.
Pass s of the timed region runs seed 123 + s for emission and transport (pass 0 is the reference's
own seed, consts.hpp:14); warm-up passes use other seeds, so every pass is an independent Monte Carlo
run.  value = superphotons created by all ranks in the K passes / max-over-ranks wall time of the K
passes -- the reference's "Final rate" (created / elapsed of run_simulation, harm_model.cpp:407-409)
averaged over K runs.

detail.overlapped (1 GPU only, --overlap J, default 16): J such passes in flight at once (J engines,
own streams and buffers, distinct seeds) -- device throughput when independent runs share the GPU;
it is NOT value.

Multi-GPU: one process per GPU.  --scaling weak (default): the job is photon_n x N, zone-sharded
over the N ranks, rank r taking every N-th zone from zone r (grmonty_amd.zone_shards "strided": each
rank's adaptive bias then sees a history of the whole disk; contiguous ranges moved the counters by
+17..+43 %); --scaling strong: the job is photon_n, zone-sharded the same way.  Zone
emission streams are keyed by zone and photon ids are global (rank r's id base = the photons of the
ranks before it), so the union of the shards' emitted photons is exactly the single-GPU job's set
(the same initial states; a photon's transport stream is keyed by its id, which under strided shards
is its rank-major position, not its single-GPU zone-order index -- so the N-rank job is an equally
valid run with other transport draws, not a bit-replay of the single-GPU one).  The only exchange is the end-of-pass RCCL
all-reduce (xGMI) of the 6x200x13 fp64 spectrum + counters, one communicator per rank, issued by the
engine's C library on its stream.  torch.distributed runs with the gloo backend only (rendezvous,
RCCL unique-id broadcast, barriers, max-over-ranks timing): torch's own HIP runtime is never
initialised, since a second HIP runtime in the process cannot open the GPU.

roofline: the dominant kernel is track_kernel; it is fp64-VALU bound.  achieved =
exact FP64 flops per transport step (counted on the oracle restatement by an instrumented build,
tests/golden/fp64_ops_per_step.json, tools/count_fp64.py) x transport steps of each pass's dominant
track_kernel launch / that launch's duration (HIP events on the engine stream; passes run alone, so
the launch is not overlapped), against the MI355X FP64 vector peak.  The HBM view (304 algorithmic
bytes per step) is reported beside it.
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
FP64_PEAK_TFS = 78.6      # MI355X FP64 vector peak (spec: 256 CU x 4 SIMD x 16 lanes x FMA x 2.4 GHz)
FP64_COUNT = os.path.join(REPO, "tests", "golden", "fp64_ops_per_step.json")
SEED0 = 123               # consts.hpp:14
WARM_SEED0 = 1_000_000    # warm-up passes: seeds disjoint from the timed ones
OVERLAP_SEED0 = 2_000_000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--photon-n", type=float, default=1e6,
                    help="photon_n per GPU (--scaling weak) or of the whole job (--scaling strong)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak")
    ap.add_argument("--shard-of", default="",
                    help="R/N: run only rank R's zone shard of an N-rank job on this one GPU (a rehearsal of one "
                         "rank of BASELINE configs[3] -- photon_n 1e8 over 8 GPUs -- without the other ranks)")
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--dump", default="", help="HARM dump to use (default: synthetic dump019-class)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--overlap", type=int, default=16,
                    help="detail only: passes in flight for the overlapped-throughput figure (0 = skip; 1 GPU)")
    ap.add_argument("--pmc-summary", default=os.environ.get("GRM_PMC_SUMMARY", ""),
                    help="rocprofv3 --pmc counter CSVs, comma-separated (FETCH_SIZE pass, WRITE_SIZE pass) "
                         "of this same command, to fill roofline.traffic")
    return ap.parse_args()


def host_threads(world: int) -> int:
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if n <= 0:
        n = min(16, os.cpu_count() or 1)
    return max(1, n // world) if world > 1 else n


def fp64_count():
    """exact FP64 operation counts per transport step of the oracle restatement (tools/count_fp64.py)"""
    try:
        with open(FP64_COUNT) as fh:
            return json.load(fh)
    except (OSError, ValueError):
        return None


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
            "sample": f"{done} of the {len(photons)} superphotons of pass 0 (random subset) tracked in {t_track:.1f} s "
                      f"+ {n_em} superphotons emitted from random zones in {t_emit:.1f} s by the oracle "
                      f"(oracle/grmonty_oracle.cpp: serial reference CPU semantics, mt19937, live bias) on 1 "
                      f"host core; the reference's own CPU build is not buildable here (DESIGN.md §3)",
            "ratio_R": None,
            "ratio_R_note": "R = reference CPU build rate / this oracle's rate on the same dump is not measurable here: "
                            "the reference CPU build needs spdlog/<format> stand-ins, which this pipeline does not allow; "
                            "the survey measured that build at ~3.2 k superphotons/s on its own synthetic 192^2 dump "
                            "(BASELINE.md section 2, a dump scattering ~3x more per photon than this one)"}


PMC_TRAFFIC = os.path.join(REPO, "profiles", "pmc_traffic.json")


def committed_traffic():
    """(HBM bytes per dominant track_kernel launch, the PMC file's provenance, whether the file was
    measured on the kernel sources this run executes) from rocprofv3 PMC passes over this same bench
    command (tools/traffic_summary.py -> profiles/pmc_traffic.json), or (None, None, False).  The file
    records the content hash of the kernel sources it was measured on (grmonty_amd.srchash); only a
    matching hash lets bench.py call traffic / this run's launch time a measured HBM rate."""
    from grmonty_amd.srchash import kernel_source_hash
    try:
        with open(PMC_TRAFFIC) as fh:
            d = json.load(fh)
        same = d.get("kernel_src_hash") == kernel_source_hash()
        return d["bytes_per_dominant_launch"], d.get("source", PMC_TRAFFIC.replace(REPO + "/", "")), same
    except (OSError, ValueError, KeyError):
        return None, None, False


def pmc_traffic(path: str):
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
    fetch = [v for v in per["FETCH_SIZE"].values()]
    write = [v for v in per["WRITE_SIZE"].values()]
    fb = [v for v in fetch if v >= 0.1 * max(fetch)]
    wb = [v for v in write if v >= 0.1 * max(write)]
    return (2.0 * float(np.mean(fb)) + float(np.mean(wb))) * 1024.0


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    overlap = args.overlap if world == 1 else 0
    if overlap > 1:
        # one hardware queue per engine of the overlapped figure (+1); HIP reads it at runtime start
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(4, overlap + 1)))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        # one GPU per rank; with more ranks than GPUs (a rehearsal on a smaller box) ranks share them
        # round-robin (counting devices does not initialise the GPU on this image)
        n_dev = torch.cuda.device_count()
        if n_dev and local >= n_dev:
            local = local % n_dev
    # ranks sharing a GPU (a rehearsal with more ranks than GPUs): RCCL refuses two ranks on one
    # device, so the job's one reduction of the stashed passes goes over gloo instead, with the same
    # sum / max split of the engine's packing (tests/test_gpu_multirank.py reduces it the same way)
    shared_gpu = False
    reduce_note = ""
    devs = [local]
    threads = args.threads or host_threads(world)
    # the partition: the job's ranks, and this process's place in it (--shard-of R/N: one rank of an
    # N-rank job alone on this GPU)
    part_rank, part_world = rank, world
    if args.shard_of:
        if world != 1:
            raise SystemExit("--shard-of runs one rank's shard in a single process")
        part_rank, part_world = (int(v) for v in args.shard_of.split("/"))
        assert 0 <= part_rank < part_world
    photon_n_job = int(args.photon_n) * (part_world if args.scaling == "weak" else 1)
    path = args.dump or os.path.join(REPO, "gpurun_out" if os.path.isdir(os.path.join(REPO, "gpurun_out")) else ".",
                                     f"synth{args.grid}_r{rank}.dump")
    if not args.dump:
        ensure_dump(path, args.grid, args.grid)
    t = time.time()
    model = G.Model.load(path, photon_n=photon_n_job).init(threads, device=local)
    t_init = time.time() - t
    shards = G.zone_shards(model.zone_weights(), part_world, "strided")
    z0, z1, zst = shards[part_rank]
    timed_seeds = [SEED0 + s for s in range(args.steps)]
    warm_seeds = [WARM_SEED0 + s for s in range(args.warmup)]
    # per-seed photon counts of every shard (host, outside the timing): the rank's id base
    t = time.time()
    id_base = {}
    for sd in warm_seeds + timed_seeds:
        id_base[sd] = sum(model.count(seed=sd, z0=a, z1=b, threads=threads, stride=st) for a, b, st in shards[:part_rank])
    t_count = time.time() - t
    engine = G.Engine(model, device=local)
    # A/B hook: GRM_BENCH_OPTS="15=2000,9=2" sets engine options (grmonty_amd.OPT_*) before the passes
    for kv in filter(None, os.environ.get("GRM_BENCH_OPTS", "").split(",")):
        k, v = kv.split("=")
        engine.set_option(int(k), int(v))
    if world > 1:  # one RCCL communicator per rank
        devs = [None] * world
        dist.all_gather_object(devs, local)
        shared_gpu = len(set(devs)) < world
        reduce_note = ""
        if not shared_gpu and os.environ.get("GRM_BENCH_REDUCE", "") != "gloo":
            # RCCL over xGMI; a rank whose communicator cannot be created makes the whole job reduce
            # over gloo instead (the same packing and sum / max split), and the line says so
            uid = [G.rccl_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            err = ""
            try:
                engine.comm_init(uid[0], world, rank)
            except RuntimeError as ex:
                err = repr(ex)
            errs = [None] * world
            dist.all_gather_object(errs, err)
            if any(errs):
                shared_gpu = True
                reduce_note = f" (RCCL unavailable: {next(e for e in errs if e)[:120]}; reduced over gloo)"
                if rank == 0:
                    print(f"WARNING: RCCL communicator failed{reduce_note}", file=sys.stderr, flush=True)
        elif not shared_gpu:
            shared_gpu = True
            reduce_note = " (GRM_BENCH_REDUCE=gloo)"
    engine.emit_setup(model)  # the zone table is resident in HBM before the timed region
    bias_counters = "single GPU"
    valid_for_parity = True
    if args.shard_of and part_world > 1:
        # one rank's shard alone: its adaptive bias runs on its own history, 1/N of the job's (DESIGN.md
        # §7: +35 % recorded at 8 ranks with per-rank counters), so its work per photon -- and this
        # line's rate -- are not the reference's counters
        bias_counters = "per shard (this rank's own history, 1/N of the job's)"
        valid_for_parity = False
    # pre-flight: which of the job's GPUs this rank can read over xGMI (hipDeviceCanAccessPeer)
    peer_row = [int(d == local or G.lib().grm_device_peer_ok(local, d) == 1) for d in sorted(set(devs))]
    peer_matrix = [peer_row]
    if world > 1:
        rows = [None] * world
        dist.all_gather_object(rows, (local, peer_row))
        peer_matrix = [r for _, r in sorted(dict(rows).items())]
    if world > 1:
        # pass slots: warm-up passes 0..W-1, timed passes W..W+K-1 (each pass its own counter block)
        engine.stash_reserve(len(warm_seeds) + len(timed_seeds))
        # the job's adaptive bias: every rank's kernels read every rank's counter block of the pass
        # (IPC over xGMI, grm_engine_set_peers); without it each rank's bias would run on a history N
        # times shorter
        handles = [None] * world
        dist.all_gather_object(handles, engine.counters_ipc_handle())
        devices = [None] * world
        dist.all_gather_object(devices, local)
        # every rank's GPU must be readable from this one (xGMI peer access) before its blocks are mapped
        ok = all(d == local or G.lib().grm_device_peer_ok(local, d) == 1 for d in devices)
        if ok:
            try:
                engine.set_peers(handles, rank)
            except RuntimeError as ex:
                ok = False
                print(f"rank {rank}: peer counters unavailable ({ex}); per-rank bias counters", file=sys.stderr)
        else:
            print(f"rank {rank}: no peer access to every rank's GPU; per-rank bias counters", file=sys.stderr)
        flags = [None] * world
        dist.all_gather_object(flags, ok)
        if not all(flags):
            engine.set_peers([], rank)
        bias_counters = "job-wide (peer counter blocks over xGMI)" if all(flags) else "per rank (IPC unavailable)"
        if not all(flags):
            # not silent: per-rank counters run each rank's adaptive bias on a history N times shorter
            # (recorded +18/+30/+35 % at 2/4/8 ranks) -- the line says so
            valid_for_parity = False
            if rank == 0:
                print("WARNING: job-wide bias counters unavailable (no peer access / IPC); the counters of this "
                      "job are NOT the reference's (valid_for_parity=false)", file=sys.stderr, flush=True)

    def one_pass(eng, seed, base, slot):
        """one run_simulation pass on this rank's shard: emission + transport + readback; with
        several ranks its results are stashed on the device (slot) for the job's one all-reduce"""
        if slot is None:
            eng.reset()
        else:
            eng.begin_pass(slot)
        eng.set_option(G.OPT_SEED, seed)
        eng.set_option(G.OPT_ID_BASE, base)
        ptr, n_dev = eng.emit(seed=seed, z0=z0, z1=z1, stride=zst)
        eng.track_device(ptr, n_dev)
        st = eng.stats()
        if slot is not None:
            eng.stash(slot)
        spec, n_rec, n_scatt, max_tau = eng.finish()
        if st["n_dropped"] or st["n_abandoned"]:
            raise RuntimeError(f"pass seed {seed}: {st['n_dropped']} children dropped, {st['n_abandoned']} abandoned")
        return n_dev, st, n_rec, n_scatt

    def reduce_job(eng, first, n):
        """the job's one exchange: a grouped RCCL all-reduce of every pass's stashed results, then
        each pass's reduced spectrum and counters read back (the ranks' pass timelines stay
        uncoupled: a rank held up by a long-lived photon does not stall the others pass by pass)"""
        if shared_gpu:
            spec, sums, maxs = eng.stash_raw(n, first)
            ts, tu = torch.from_numpy(spec), torch.from_numpy(sums.view(np.int64))
            tm = torch.from_numpy(maxs.view(np.int64))
            dist.all_reduce(ts, op=dist.ReduceOp.SUM)
            dist.all_reduce(tu, op=dist.ReduceOp.SUM)
            dist.all_reduce(tm, op=dist.ReduceOp.MAX)  # every word < 2^63: int64 order = u64 order
            eng.stash_raw_write(ts.numpy(), tu.numpy().view(np.uint64), tm.numpy().view(np.uint64), first)
        else:
            eng.allreduce_stash(n, first)
        return [eng.stash_read(first + s) for s in range(n)]

    for i, sd in enumerate(warm_seeds):
        one_pass(engine, sd, id_base[sd], i if world > 1 else None)
    if world > 1 and warm_seeds:
        reduce_job(engine, 0, len(warm_seeds))
    launches0 = engine.stats()["n_launches"]
    if dist is not None:
        dist.barrier()
    res, pass_s = [], []
    t0 = time.time()
    for i, sd in enumerate(timed_seeds):
        tp = time.time()
        res.append(one_pass(engine, sd, id_base[sd], len(warm_seeds) + i if world > 1 else None))
        pass_s.append(time.time() - tp)
    job = reduce_job(engine, len(warm_seeds), len(timed_seeds)) if world > 1 else None
    if dist is not None:
        dist.barrier()
    elapsed = time.time() - t0
    if job is not None:  # the job-level results: the reduced counters of every pass
        res = [(r[0], r[1], j[1], j[2]) for r, j in zip(res, job)]
    n_rank = sum(r[0] for r in res)
    tmax, total = elapsed, n_rank
    if dist is not None:
        tm = torch.tensor([elapsed], dtype=torch.float64)
        tt = torch.tensor([float(n_rank)], dtype=torch.float64)
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        tmax, total = float(tm[0]), int(tt[0])

    # cold run (detail, outside the timed region): the reference's own window alloc_memory ...
    # free_memory (harm_model.cpp:341-409) -- a fresh engine (device buffers, stream, events), the
    # zone table built on the host and uploaded, one pass of seed 123, destroy; every rank, one pass
    cold = None
    tc = time.time()
    eng_c = G.Engine(model, device=local)
    t_create = time.time() - tc
    eng_c.emit_setup(model)
    t_setup = time.time() - tc - t_create
    tp = time.time()
    n_c = one_pass(eng_c, SEED0, id_base[SEED0], None)[0] if SEED0 in id_base else None
    t_pass = time.time() - tp
    eng_c.close()
    t_cold = time.time() - tc
    cold = {"wall_s": t_cold, "engine_create_s": t_create, "emit_setup_s": t_setup, "pass_s": t_pass,
            "destroy_s": t_cold - t_create - t_setup - t_pass, "superphotons": n_c,
            "superphotons_per_s": (n_c / t_cold) if n_c else None,
            "amortised_setup_s": t_create + t_setup,
            "note": "one run_simulation pass in the reference's timing window alloc_memory..free_memory "
                    "(harm_model.cpp:341-409): engine creation + zone-table upload + pass + destroy, rank 0; "
                    "value amortises creation and setup over the job's passes"}

    overlapped = None
    if rank == 0 and overlap > 1:
        overlapped = overlapped_throughput(model, overlap, z0, z1, zst)
    if rank == 0:
        sts = [r[1] for r in res]
        launches = res[-1][1]["n_launches"] - launches0
        kern_ms = sum(s["last_kernel_ms"] for s in sts)
        steps_tot = sum(s["last_steps"] for s in sts)
        big_ms = sum(s["max_launch_ms"] for s in sts)
        big_steps = sum(s["max_launch_steps"] for s in sts)
        emit_ms = sum(s["last_emit_ms"] for s in sts)
        cnt = fp64_count()
        flops_step = cnt["flops_per_step"] if cnt else None
        traffic, traffic_src, traffic_same = ((pmc_traffic(args.pmc_summary), "--pmc-summary CSVs of this run", True)
                                              if args.pmc_summary else committed_traffic())
        # measured HBM rate of the dominant launch: PMC bytes per launch / this run's launch time --
        # only when the bytes were measured on these kernels (this run's CSVs, or a committed file whose
        # kernel-source hash matches); otherwise the traffic is reported as borrowed and no rate is formed
        hbm_gbs = traffic / (big_ms / args.steps * 1e-3) / 1e9 if (traffic and traffic_same) else None
        if traffic and not traffic_same:
            traffic_src = f"BORROWED (other kernel sources): {traffic_src}"
        achieved_tf = big_steps * flops_step / (big_ms * 1e-3) / 1e12 if flops_step else None
        alg_gbs = big_steps * ALG_BYTES_PER_STEP / (big_ms * 1e-3) / 1e9
        cpu = None
        if world == 1 and args.cpu_seconds > 0:
            try:
                ph = model.emit(seed=SEED0, z0=z0, z1=z1, threads=threads, stride=zst)
                cpu = cpu_baseline(path, photon_n_job, ph, args.cpu_seconds)
            except Exception as ex:  # the baseline is reported beside the product, never part of it
                cpu = {"value": None, "error": repr(ex)}
        srt = sorted(pass_s)
        out = {
            "metric": "superphotons/sec on dump019-class HARM dump (photon_n=1e6 per run_simulation)",
            "value": total / tmax,
            "unit": "superphotons/s",
            "n_gpus": len(set(devs)),
            "ranks": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": tmax / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"synthetic dump019-class {args.grid}x{args.grid} MKS HARM dump, photon_n="
                                   f"{photon_n_job:g} run_simulation passes (seeds {SEED0}..{SEED0 + args.steps - 1}), "
                                   f"mass_unit=4e19, zone-sharded over {world} GPU(s)" + (
                                       f"; this line: rank {part_rank}'s strided shard of a {part_world}-rank job "
                                       f"alone on one GPU (value = that rank's rate)" if args.shard_of else ""),
                       "photon_n_job": photon_n_job, "grid": f"{args.grid}x{args.grid}",
                       "superphotons_per_pass_rank0": n_rank // max(1, args.steps),
                       "bias_counters": bias_counters,
                       "valid_for_parity": valid_for_parity,
                       "peer_access": peer_matrix,
                       "parallelism": f"strided zone shards x{world}" + (
                           ((", ranks sharing GPUs (rehearsal)" if len(set(devs)) < world else "") +
                            ", passes stashed on the device, one gloo reduction per job" + reduce_note
                            if shared_gpu else ", passes stashed on the device, one RCCL all-reduce per job")
                           if world > 1 else "")},
            "roofline": {"bound": "fp64-valu", "achieved": achieved_tf, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                         "frac": achieved_tf / FP64_PEAK_TFS if achieved_tf else None,
                         "traffic": traffic if traffic_same else None,
                         "traffic_borrowed": None if traffic_same else traffic,
                         "flops_per_step": flops_step,
                         "transcendentals_per_step": cnt.get("transcendentals_per_step") if cnt else None,
                         "traffic_source": traffic_src,
                         "hbm_gbs": hbm_gbs, "hbm_measured_frac": hbm_gbs / HBM_PEAK_GBS if hbm_gbs else None,
                         "hbm_algorithmic_gbs": alg_gbs, "hbm_frac": alg_gbs / HBM_PEAK_GBS,
                         "note": f"dominant track_kernel launch per pass (alone on the GPU): "
                                 f"{big_steps // args.steps} transport steps in {big_ms / args.steps:.1f} ms "
                                 f"(HIP events on the engine stream) x {flops_step} counted FP64 flops/step "
                                 f"({FP64_COUNT.replace(REPO + '/', '')}); HBM view: {ALG_BYTES_PER_STEP} algorithmic "
                                 f"B/step -> {alg_gbs:.0f} GB/s (mostly L2 hits); traffic = PMC FETCH(x2)+WRITE bytes per dominant "
                                 f"launch (--pmc-summary CSVs of this run, else profiles/pmc_traffic.json: the PMC passes of this bench "
                                 f"command, tools/traffic_summary.py); hbm_gbs = traffic / this run's dominant launch time"},
            "cpu_baseline": cpu,
            "detail": {"pass_s": {"min": srt[0], "median": srt[len(srt) // 2], "max": srt[-1],
                                  "all": [round(v, 4) for v in pass_s]},
                       # the rate of the median pass (value is the whole job's: the long-photon tail passes
                       # weigh in there)
                       "median_pass_rate": (total / args.steps) / srt[len(srt) // 2],
                       "transport_steps_per_s": steps_tot / (kern_ms * 1e-3), "kernel_ms_per_pass": kern_ms / args.steps,
                       "dominant_launch_ms_per_pass": big_ms / args.steps,
                       "emit_ms_per_pass": emit_ms / args.steps,
                       "longest_photon_life_steps": max(s["max_photon_steps"] for s in sts),
                       # where each pass's time went beyond its bulk launch: the early worker's launch (beside
                       # the bulk), the lone-photon kernels after it, the photons they took (and the children
                       # those pairs tracked themselves, GRM_OPT_EARLY_CHILDREN), the longest life
                       "tail_per_pass": [{"bulk_ms": round(s["max_launch_ms"], 1), "early_ms": round(s["early_ms"], 1),
                                          "n_early": s["n_early"], "n_early_children": s.get("n_early_children", 0),
                                          "lone_ms": round(s["lone_ms"], 1), "n_lone": s["n_lone"],
                                          "n_lone_children": s.get("n_lone_children", 0),
                                          "kernels_ms": round(s["last_kernel_ms"], 1),
                                          "longest_life": s["max_photon_steps"], "lives_gt_1e5": s["n_long_photons"]}
                                         for s in sts],
                       "tracked_per_pass": sum(s["n_tracked"] for s in sts) // args.steps,
                       "children_per_pass": sum(s["n_children"] for s in sts) // args.steps,
                       "recorded_per_pass": sum(r[2] for r in res) // args.steps,
                       "launches_per_pass": launches / args.steps,
                       "overlapped": overlapped,
                       "cold_run": cold,
                       "init_s": t_init, "count_s": t_count},
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def overlapped_throughput(model, jobs: int, z0: int, z1: int, zst: int = 1):
    """detail only: `jobs` independent passes (distinct seeds) in flight at once, one engine + host
    thread each, on this rank's zones -- what the device sustains when runs share it"""
    import threading
    engines = [G.Engine(model, device=int(os.environ.get("LOCAL_RANK", "0"))) for _ in range(jobs)]
    for e in engines:
        e.emit_setup(model)
    err, counts = [], [0] * jobs

    def run(j, seed):
        try:
            e = engines[j]
            e.reset()
            e.set_option(G.OPT_SEED, seed)
            e.set_option(G.OPT_ID_BASE, 0)
            ptr, n = e.emit(seed=seed, z0=z0, z1=z1, stride=zst)
            e.track_device(ptr, n)
            st = e.stats()
            if st["n_dropped"] or st["n_abandoned"]:
                raise RuntimeError("overlapped pass lost photons")
            e.finish()
            counts[j] += n
        except Exception as ex:
            err.append(ex)

    def phase(seed0):
        th = [threading.Thread(target=run, args=(j, seed0 + j)) for j in range(jobs)]
        for t_ in th:
            t_.start()
        for t_ in th:
            t_.join()

    phase(OVERLAP_SEED0)  # warm every engine
    counts[:] = [0] * jobs
    t = time.time()
    phase(OVERLAP_SEED0 + jobs)
    el = time.time() - t
    for e in engines:
        e.close()
    if err:
        return {"error": repr(err[0])}
    return {"passes_in_flight": jobs, "passes": jobs, "superphotons_per_s": sum(counts) / el, "wall_s": el,
            "note": "independent passes (distinct seeds) sharing the GPU; not the reference's per-run rate"}


if __name__ == "__main__":
    main()
