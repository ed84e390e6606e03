"""Multi-rank path on CPU (gloo, world_size 2): zone-range shards of one job (the partition bench.py
uses), per-rank transport of each shard (oracle stands in for the device kernel: same Philox stream
ids), and the engine's end-of-run exchange on the engine's own packed buffers.  The reduced result
must equal one process tracking the whole job: the partition, the global photon ids and the
reduction are exact.

The exchange mirrors grm_engine_allreduce (cuda-grmonty_amd/csrc/grm_engine.hip) collective for
collective, on the same buffers: the device spectrum, 6 x 200 cells x 13 fp64 = 15,600 doubles,
SUM; the device counter block (DevCounters, 16 u64): words 0-1 (n_recorded, n_scatt) SUM, word 2
(max tau_scatt as its IEEE-754 bit pattern: tau >= 0 orders as an integer) MAX, words 3-8 (steps,
tracked, children, overflow, dropped, primaries) SUM -- here over gloo instead of RCCL."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SNAP = dict(scatt=300, rec=150, maxtau=2e-3)


def pack_counters(orc) -> np.ndarray:
    """the engine's DevCounters block (16 words) from an oracle run: n_recorded, n_scatt, max
    tau_scatt bits, n_steps, n_tracked, n_children, n_overflow, n_dropped, n_primaries (gloo has no
    u64: int64, every value < 2^63)"""
    c = orc.counters()
    v = np.zeros(16, dtype=np.int64)
    v[0], v[1], v[3] = c["recorded"], c["scattered"], c["steps"]
    v[2] = np.array([orc.scalars()["max_tau_scatt"]], dtype=np.float64).view(np.int64)[0]
    v[8] = c["created"]
    return v


def job_photon_n(world, scaling):
    """bench.py's job size: photon_n per GPU (weak) or for the whole job (strong)"""
    return 150 * world if scaling == "weak" else 300


def _shard_job(rank, world, dump, out_dir, port, photon_n):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "cuda-grmonty_amd"), os.path.join(os.path.dirname(here), "oracle")]
    import grmonty_amd as G
    import oracle_py as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = G.Model.load(dump, photon_n=photon_n).init(2)
    shards = G.zone_shards(model.zone_weights(), world)
    counts = [model.count(seed=123, z0=a, z1=b, stride=st) for a, b, st in shards]
    a, b, st = shards[rank]
    ph = model.emit(seed=123, z0=a, z1=b, stride=st)
    orc = O.OracleModel(dump, photon_n=photon_n)
    orc.init(2)
    orc.track(ph.view(O.INIT_PHOTON), rng_mode=1, seed=123, id_base=int(sum(counts[:rank])), frozen=True,
              scatt0=SNAP["scatt"], rec0=SNAP["rec"], max_tau0=SNAP["maxtau"])
    spec = torch.from_numpy(orc.spectrum().view(np.float64).reshape(-1).copy())
    assert spec.numel() == 15600
    ctr = torch.from_numpy(pack_counters(orc))
    # grm_engine_allreduce: spectrum SUM; counters [0:2] SUM, [2] MAX (bit pattern), [3:9] SUM
    dist.all_reduce(spec, op=dist.ReduceOp.SUM)
    dist.all_reduce(ctr[0:2], op=dist.ReduceOp.SUM)
    dist.all_reduce(ctr[2:3], op=dist.ReduceOp.MAX)
    dist.all_reduce(ctr[3:9], op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(os.path.join(out_dir, "spec.npy"), spec.numpy())
        np.save(os.path.join(out_dir, "ctr.npy"), ctr.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("scaling", ["weak", "strong"])
def test_two_rank_shards_equal_single_job(dump32, tmp_path, scaling):
    """bench.py --scaling weak (photon_n per GPU) and strong (photon_n for the job): the ranks'
    strided shards reduce to exactly the single-process job"""
    import grmonty_amd as G
    import oracle_py as O
    world = 2
    pn = job_photon_n(world, scaling)
    mp.spawn(_shard_job, args=(world, dump32, str(tmp_path), _free_port(), pn), nprocs=world, join=True)
    spec_d = np.load(tmp_path / "spec.npy")
    ctr_d = np.load(tmp_path / "ctr.npy")
    model = G.Model.load(dump32, photon_n=pn).init(2)
    # the ranks' photons in rank order: the ids they were tracked under
    ph = np.concatenate([model.emit(seed=123, z0=a, z1=b, stride=st)
                         for a, b, st in G.zone_shards(model.zone_weights(), world)])
    assert len(ph) == model.count(seed=123)  # the shards' union is the single-GPU photon set
    orc = O.OracleModel(dump32, photon_n=pn)
    orc.init(2)
    orc.track(ph.view(O.INIT_PHOTON), rng_mode=1, seed=123, id_base=0, frozen=True, scatt0=SNAP["scatt"],
              rec0=SNAP["rec"], max_tau0=SNAP["maxtau"])
    spec_1 = orc.spectrum().view(np.float64).reshape(-1)
    ctr_1 = pack_counters(orc)
    np.testing.assert_array_equal(ctr_d, ctr_1)  # counts exact, max tau_scatt bit-exact
    np.testing.assert_allclose(spec_d, spec_1, rtol=1e-12, atol=0)


STASH_SEEDS = (123, 124)


def stash_counters(orc):
    """one pass's counters as grm_engine_stash lays them out: 9 summed words (recorded, scattered,
    steps, tracked, children, overflow, dropped, primaries, lives > 1e5) and 2 maxed (max tau_scatt
    bits, longest life); the oracle fills the words it has"""
    c = orc.counters()
    s = np.zeros(9, dtype=np.int64)
    s[0], s[1], s[2], s[7] = c["recorded"], c["scattered"], c["steps"], c["created"]
    m = np.zeros(2, dtype=np.int64)
    m[0] = np.array([orc.scalars()["max_tau_scatt"]], dtype=np.float64).view(np.int64)[0]
    return s, m


def _stash_job(rank, world, dump, out_dir, port):
    """several passes per rank, each stashed, then ONE grouped reduction of all of them
    (grm_engine_allreduce_stash: spectra SUM, 9 counters SUM, 2 counters MAX -- over gloo here)"""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "cuda-grmonty_amd"), os.path.join(os.path.dirname(here), "oracle")]
    import grmonty_amd as G
    import oracle_py as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = G.Model.load(dump, photon_n=150 * world).init(2)
    shards = G.zone_shards(model.zone_weights(), world)
    k = len(STASH_SEEDS)
    st_spec = np.zeros((k, 15600))
    st_sum = np.zeros((k, 9), dtype=np.int64)
    st_max = np.zeros((k, 2), dtype=np.int64)
    for slot, seed in enumerate(STASH_SEEDS):
        counts = [model.count(seed=seed, z0=a, z1=b, stride=st) for a, b, st in shards]
        a, b, st = shards[rank]
        ph = model.emit(seed=seed, z0=a, z1=b, stride=st)
        orc = O.OracleModel(dump, photon_n=150 * world)
        orc.init(2)
        orc.track(ph.view(O.INIT_PHOTON), rng_mode=1, seed=seed, id_base=int(sum(counts[:rank])), frozen=True,
                  scatt0=SNAP["scatt"], rec0=SNAP["rec"], max_tau0=SNAP["maxtau"])
        st_spec[slot] = orc.spectrum().view(np.float64).reshape(-1)
        st_sum[slot], st_max[slot] = stash_counters(orc)
    spec, ssum, smax = torch.from_numpy(st_spec), torch.from_numpy(st_sum), torch.from_numpy(st_max)
    dist.all_reduce(spec, op=dist.ReduceOp.SUM)
    dist.all_reduce(ssum, op=dist.ReduceOp.SUM)
    dist.all_reduce(smax, op=dist.ReduceOp.MAX)
    if rank == 0:
        np.save(os.path.join(out_dir, "st_spec.npy"), spec.numpy())
        np.save(os.path.join(out_dir, "st_sum.npy"), ssum.numpy())
        np.save(os.path.join(out_dir, "st_max.npy"), smax.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_stashed_passes_equal_single_jobs(dump32, tmp_path):
    """bench.py's multi-GPU exchange: every pass stashed, one reduction for the job; each reduced slot
    must equal one process running that pass's whole job"""
    import grmonty_amd as G
    import oracle_py as O
    world = 2
    mp.spawn(_stash_job, args=(world, dump32, str(tmp_path), _free_port()), nprocs=world, join=True)
    st_spec = np.load(tmp_path / "st_spec.npy")
    st_sum = np.load(tmp_path / "st_sum.npy")
    st_max = np.load(tmp_path / "st_max.npy")
    model = G.Model.load(dump32, photon_n=150 * world).init(2)
    for slot, seed in enumerate(STASH_SEEDS):
        ph = np.concatenate([model.emit(seed=seed, z0=a, z1=b, stride=st)
                             for a, b, st in G.zone_shards(model.zone_weights(), world)])
        orc = O.OracleModel(dump32, photon_n=150 * world)
        orc.init(2)
        orc.track(ph.view(O.INIT_PHOTON), rng_mode=1, seed=seed, id_base=0, frozen=True, scatt0=SNAP["scatt"],
                  rec0=SNAP["rec"], max_tau0=SNAP["maxtau"])
        s1, m1 = stash_counters(orc)
        np.testing.assert_array_equal(st_sum[slot], s1)
        np.testing.assert_array_equal(st_max[slot], m1)
        np.testing.assert_allclose(st_spec[slot], orc.spectrum().view(np.float64).reshape(-1), rtol=1e-12, atol=0)
