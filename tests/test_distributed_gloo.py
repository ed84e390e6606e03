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


def _shard_job(rank, world, dump, out_dir, port):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.join(os.path.dirname(here), "cuda-grmonty_amd"), os.path.join(os.path.dirname(here), "oracle")]
    import grmonty_amd as G
    import oracle_py as O
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    model = G.Model.load(dump, photon_n=150 * world).init(2)
    shards = G.shard_zones(model.zone_weights(), world)
    counts = [model.count(seed=123, z0=a, z1=b) for a, b in shards]
    ph = model.emit(seed=123, z0=shards[rank][0], z1=shards[rank][1])
    orc = O.OracleModel(dump, photon_n=150 * world)
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


def test_two_rank_shards_equal_single_job(dump32, tmp_path):
    import grmonty_amd as G
    import oracle_py as O
    world = 2
    mp.spawn(_shard_job, args=(world, dump32, str(tmp_path), _free_port()), nprocs=world, join=True)
    spec_d = np.load(tmp_path / "spec.npy")
    ctr_d = np.load(tmp_path / "ctr.npy")
    model = G.Model.load(dump32, photon_n=150 * world).init(2)
    ph = model.emit(seed=123)
    orc = O.OracleModel(dump32, photon_n=150 * world)
    orc.init(2)
    orc.track(ph.view(O.INIT_PHOTON), rng_mode=1, seed=123, id_base=0, frozen=True, scatt0=SNAP["scatt"],
              rec0=SNAP["rec"], max_tau0=SNAP["maxtau"])
    spec_1 = orc.spectrum().view(np.float64).reshape(-1)
    ctr_1 = pack_counters(orc)
    np.testing.assert_array_equal(ctr_d, ctr_1)  # counts exact, max tau_scatt bit-exact
    np.testing.assert_allclose(spec_d, spec_1, rtol=1e-12, atol=0)
