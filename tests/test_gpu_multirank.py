"""The multi-GPU job on one MI355X.

1. N-rank jobs emulated on one GPU (N = 2, 4, 8), live adaptive bias, against the oracle's
   run_simulation at the headline scale (192x192, photon_n = 1e5; tests/golden/oracle_synth192_pn1e5.*):
   each emulated rank runs bench.py's zone shard (grmonty_amd.zone_shards, strided: every N-th
   zone) as a pass of its own after a reset, so its bias_func (harm_model.cpp:1391-1404) sees only
   its own counters, as on N GPUs; the ranks' results are summed.  The job's counters are tested
   the way the single-GPU job's are (tests/test_gpu_parity_192.py): the mean over N_DEV seeds
   against the oracle's mean, and the KS test of one traced job.  (Contiguous zone ranges failed
   this: +17 / +30 / +43 % recorded at 2 / 4 / 8 ranks, profiles/r03a_multirank_contiguous.log.)

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

from job_util import KEYS, run_job
from spectrum_stats import binned_ks, ks_crit, welch_z

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden", "oracle_synth192_pn1e5")
N_DEV = 16
Z_MAX = 4.5


@pytest.fixture(scope="module")
def setup192(dump_dir):
    import grmonty_amd as GA
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump(os.path.join(dump_dir, "synth192.dump"), 192, 192)
    model = GA.Model.load(path, photon_n=100000).init(8, device=0)  # the tables bench.py uses
    eng = GA.Engine(model, device=0)
    eng.emit_setup(model)
    yield model, eng
    eng.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_emulated_ranks_vs_oracle(setup192, world):
    import grmonty_amd as GA
    model, eng = setup192
    shards = GA.zone_shards(model.zone_weights(), world)
    summ = json.load(open(GOLD + ".json"))
    o = {k: np.array([r[k] for r in summ["runs"]], dtype=np.float64) for k in KEYS}
    dev = {k: [] for k in KEYS}
    per_rank = []
    for s in range(N_DEV):
        job = run_job(eng, model, 123 + s, shards=shards)
        for k in KEYS:
            dev[k].append(job[k])
        per_rank.append([r["recorded"] / max(1, r["created"]) for r in job["per_rank"]])
    print(f"{world} ranks, shards {shards}; recorded per created by rank (mean over seeds): "
          f"{np.round(np.mean(per_rank, axis=0), 3).tolist()}")
    bad = []
    for k in KEYS:
        diff, se, z = welch_z(dev[k], o[k])
        print(f"{k:10s} device {np.mean(dev[k]):.6g} +- {np.std(dev[k], ddof=1):.3g} ({N_DEV} jobs)  oracle "
              f"{o[k].mean():.6g} +- {o[k].std(ddof=1):.3g} ({len(o[k])} runs)  diff {diff / o[k].mean():+.2%} "
              f"= {z:+.2f} SE")
        if abs(z) > Z_MAX:
            bad.append((k, z))
    # the spectrum's shape: one traced job against the pooled oracle runs
    job = run_job(eng, model, 123, shards=shards, trace_cap=12_000_000)
    pooled = np.load(GOLD + ".npz")["cells"].sum(axis=0)
    for th in [None, 0, 1, 2, 3, 4, 5]:
        d, n1, n2 = binned_ks(job["cells"], pooled, th)
        crit = ks_crit(n1, n2, 1e-4)
        print(f"theta bin {th}: KS D={d:.4f} crit={crit:.4f}")
        if not d < crit:
            bad.append(("ks", th, d, crit))
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
