"""The multi-GPU job on one MI355X.

1. N-rank jobs emulated on one GPU (N = 2, 4, 8), live adaptive bias, against the oracle's
   run_simulation at the headline scale (192x192, photon_n = 1e5; tests/golden/oracle_synth192_pn1e5.*).
   tests/multirank_emu.py runs N engines concurrently, each with 1/N of the CUs, bench.py's zone
   shard (grmonty_amd.zone_shards: every N-th zone from r), its global id base and its per-pass
   counter block, the blocks linked (grm_engine_link_peers: the kernels run bias_func on the job's
   counters, harm_model.cpp:1391-1404, as grm_engine_set_peers makes them do across GPUs).  The job's
   counters are tested against the oracle's mean over N_DEV seeds: the luminosity (the estimator is
   unbiased whatever the bias) and the counters the live bias drives (recorded, scattered, steps)
   within Z_MAX combined standard errors (no allowance: the sharding faults this test exists for
   are +17 to +43 %, below, and the job's warm-up now ramps job-wide -- each rank admits 1/N of a
   single GPU's batches behind a barrier at 1/16 of the job's history, grm_engine.hip run_passes,
   DESIGN.md §7: 8 ranks +5 % at 1/2, +1.2 to +3.7 % at 1/16; and a multi-rank job's small calls run
   at twice the in-flight ratio since round 6: 96-job 8-rank sessions +2.97 % at ratio 96, +1.42 % at
   192); and every rank's view of the job counters (the kernels' own summation path) must equal the
   sums of the ranks'.
   Without the link each rank's bias runs on its own history, N times shorter: +18 / +30 / +35 %
   recorded at 2 / 4 / 8 ranks with strided shards (profiles/r03b_pytest_multirank_unshared.log),
   +17 / +30 / +43 % with contiguous ones (profiles/r03a_multirank_contiguous.log).

2. The multi-rank reduction on the engine's own stash buffers: two processes on the GPU, one engine
   each, run the two shards of a frozen-bias job (so the result is exact), stash their passes
   (grm_engine_stash: the engine's packing), read the raw slots (grm_engine_stash_raw), reduce them
   over gloo -- the spectrum and the "sum" words summed, the "max" words maxed, which is what
   grm_engine_allreduce_stash asks RCCL for -- write them back and decode them with
   grm_engine_stash_read.  Must equal one engine tracking the ranks' photons concatenated (the
   same photon ids): this checks the stash
   word order, the split of the counters between sum and max and the slot indexing, which RCCL
   with N > 1 would reduce the same way (RCCL itself with N > 1 needs N GPUs: not run here).
"""
import json
import os
import socket

import numpy as np
import pytest

from job_util import KEYS
from spectrum_stats import welch_z

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "oracle_synth192_pn1e5")
N_DEV = 40
Z_MAX = 4.5


@pytest.mark.parametrize("world", [2, 4, 8])
def test_emulated_ranks_vs_oracle(dump_dir, tmp_path, world):
    import subprocess
    import sys
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump(os.path.join(dump_dir, "synth192.dump"), 192, 192)
    out = tmp_path / "emu.json"
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(min(32, 2 * world + 2)))
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "multirank_emu.py"), path, str(world), str(N_DEV),
                        str(out), "--shared"], env=env, capture_output=True, text=True, timeout=280)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stderr[-3000:]
    jobs = json.load(open(out))
    summ = json.load(open(GOLD + ".json"))
    o = {k: np.array([x[k] for x in summ["runs"]], dtype=np.float64) for k in KEYS}
    bad = []
    for k in KEYS:
        dev = [j[k] for j in jobs]
        diff, se, z = welch_z(dev, o[k])
        print(f"{world} ranks {k:10s} device {np.mean(dev):.6g} +- {np.std(dev, ddof=1):.3g} ({len(dev)} jobs)  "
              f"oracle {o[k].mean():.6g} +- {o[k].std(ddof=1):.3g} ({len(o[k])} runs)  diff {diff / o[k].mean():+.2%} "
              f"= {z:+.2f} SE (bar {Z_MAX} SE)")
        if abs(z) > Z_MAX:
            bad.append((k, z))
    for j in jobs:
        for v in j["job_view"]:
            assert v["n_recorded"] == j["recorded"] and v["n_scatt"] == j["scattered"]
            assert v["max_tau_scatt"] == j["max_tau"]
    assert not bad, bad


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SEEDS = (123, 124)
SNAP = dict(scatt=3000, rec=2000)


def _configure(G, eng, model, seed, base):
    eng.reset()
    eng.set_option(G.OPT_SEED, seed)
    eng.set_option(G.OPT_ID_BASE, base)
    eng.set_option(G.OPT_BIAS_MODE, 1)
    eng.set_option(G.OPT_FROZEN_SCATT, SNAP["scatt"])
    eng.set_option(G.OPT_FROZEN_REC, SNAP["rec"])
    eng.set_option(G.OPT_FROZEN_MAXTAU, int(np.float64(model.scalars()["max_tau_scatt"]).view(np.int64)))


def _rank(rank, world, dump, out_dir, port):
    import sys
    sys.path[:0] = [os.path.join(os.path.dirname(HERE), "cuda-grmonty_amd"), HERE]
    import torch
    import torch.distributed as dist
    import grmonty_amd as G
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = G.Model.load(dump, photon_n=3000).init(4)
    shards = G.zone_shards(model.zone_weights(), world)
    eng = G.Engine(model, device=0)
    eng.stash_reserve(len(SEEDS))
    for slot, seed in enumerate(SEEDS):
        base = sum(model.count(seed=seed, z0=a, z1=b, stride=st) for a, b, st in shards[:rank])
        _configure(G, eng, model, seed, base)
        a, b, st = shards[rank]
        eng.track(model.emit(seed=seed, z0=a, z1=b, stride=st))  # host emission, as the reference below
        eng.stash(slot)
    spec, sums, maxs = eng.stash_raw(len(SEEDS))
    ts, tu, tm = torch.from_numpy(spec), torch.from_numpy(sums.view(np.int64)), torch.from_numpy(maxs.view(np.int64))
    dist.all_reduce(ts, op=dist.ReduceOp.SUM)
    dist.all_reduce(tu, op=dist.ReduceOp.SUM)
    dist.all_reduce(tm, op=dist.ReduceOp.MAX)  # every word < 2^63: int64 order = u64 order
    eng.stash_raw_write(ts.numpy(), tu.numpy().view(np.uint64), tm.numpy().view(np.uint64))
    if rank == 0:
        res = []
        for slot in range(len(SEEDS)):
            sp, nr, ns, mt, st = eng.stash_read(slot)
            res.append((sp.view(np.float64).reshape(-1), nr, ns, mt, st))
        np.save(os.path.join(out_dir, "spec.npy"), np.stack([r[0] for r in res]))
        np.save(os.path.join(out_dir, "ctr.npy"), np.array([[r[1], r[2], r[4]] for r in res], dtype=np.uint64))
        np.save(os.path.join(out_dir, "maxtau.npy"), np.array([r[3] for r in res]))
        np.save(os.path.join(out_dir, "raw_sums.npy"), tu.numpy().view(np.uint64))
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


def test_gloo_reduction_of_engine_stash(dump64, tmp_path):
    import torch.multiprocessing as mp
    import grmonty_amd as G
    world = 2
    mp.spawn(_rank, args=(world, dump64, str(tmp_path), _free_port()), nprocs=world, join=True)
    spec_d = np.load(tmp_path / "spec.npy")
    ctr_d = np.load(tmp_path / "ctr.npy")
    mt_d = np.load(tmp_path / "maxtau.npy")
    raw = np.load(tmp_path / "raw_sums.npy")
    model = G.Model.load(dump64, photon_n=3000).init(4)
    shards = G.zone_shards(model.zone_weights(), world)
    eng = G.Engine(model, device=0)
    for slot, seed in enumerate(SEEDS):
        _configure(G, eng, model, seed, 0)
        ph = np.concatenate([model.emit(seed=seed, z0=a, z1=b, stride=st) for a, b, st in shards])
        n = len(ph)
        eng.track(ph)
        spec1, nr, ns, mt = eng.finish()
        st = eng.stats()
        print(f"seed {seed}: one engine recorded {nr} scattered {ns} steps {st['n_steps']}; two ranks "
              f"{ctr_d[slot].tolist()}")
        assert st["n_steps"] > 0 and nr > 0
        np.testing.assert_array_equal(ctr_d[slot], np.array([nr, ns, st["n_steps"]], dtype=np.uint64))
        assert np.float64(mt_d[slot]).view(np.uint64) == np.float64(mt).view(np.uint64)
        # the stash's other summed words: tracked, children, primaries
        assert raw[slot][3] == st["n_tracked"] and raw[slot][4] == st["n_children"] and raw[slot][7] == n
        np.testing.assert_allclose(spec_d[slot], spec1.view(np.float64).reshape(-1), rtol=1e-12, atol=0)
    eng.close()


def _ipc_rank(rank, world, dump, out_dir, port):
    """grm_engine_set_peers across processes: IPC handles of the pass counter blocks exchanged over
    gloo, a live-bias pass on each rank, then every rank's kernel-side view of the job counters"""
    import sys
    sys.path[:0] = [os.path.join(os.path.dirname(HERE), "cuda-grmonty_amd"), HERE]
    import torch
    import torch.distributed as dist
    import grmonty_amd as G
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = G.Model.load(dump, photon_n=3000).init(4)
    shards = G.zone_shards(model.zone_weights(), world)
    eng = G.Engine(model, device=0)
    eng.emit_setup(model)
    eng.stash_reserve(1)
    handles = [None] * world
    dist.all_gather_object(handles, eng.counters_ipc_handle())
    eng.set_peers(handles, rank)
    eng.begin_pass(0)
    dist.barrier()
    eng.set_option(G.OPT_SEED, 123)
    eng.set_option(G.OPT_ID_BASE, sum(model.count(seed=123, z0=a, z1=b, stride=st) for a, b, st in shards[:rank]))
    a, b, st = shards[rank]
    p, n = eng.emit(seed=123, z0=a, z1=b, stride=st)
    eng.track_device(p, n)
    _, nr, ns, mt = eng.finish()
    dist.barrier()  # both passes done
    view = eng.job_counters()
    own = torch.tensor([float(nr), float(ns)], dtype=torch.float64)
    mx = torch.tensor([mt], dtype=torch.float64)
    dist.all_reduce(own, op=dist.ReduceOp.SUM)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    json.dump(dict(view=view, rec=float(own[0]), scatt=float(own[1]), max_tau=float(mx[0]), own_rec=nr),
              open(os.path.join(out_dir, f"ipc_{rank}.json"), "w"))
    dist.barrier()
    eng.set_peers([], 0)  # close the mapped blocks before the owners free them
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


def test_ipc_peer_counters(dump64, tmp_path):
    """two processes on the GPU: each maps the other's per-pass counter blocks by IPC
    (grm_engine_counters_ipc_handle / grm_engine_set_peers), and the transport kernels' view of the
    job counters equals the sums of both ranks' counters (max for max tau_scatt)"""
    import torch.multiprocessing as mp
    world = 2
    mp.spawn(_ipc_rank, args=(world, dump64, str(tmp_path), _free_port()), nprocs=world, join=True)
    for r in range(world):
        d = json.load(open(tmp_path / f"ipc_{r}.json"))
        print(r, d)
        assert d["view"]["n_recorded"] == d["rec"] and d["view"]["n_scatt"] == d["scatt"]
        assert d["view"]["max_tau_scatt"] == d["max_tau"]
        assert 0 < d["own_rec"] < d["rec"]
