"""Multi-rank path on CPU (gloo, world_size 2): zone-range shards of one job (the partition bench.py
uses), per-rank transport of each shard (oracle stands in for the device kernel: same Philox stream
ids), and an all-reduce of the spectrum + counters.  The reduced result must equal one process
tracking the whole job: the partition, the global photon ids and the reduction are exact."""
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
    c = orc.counters()
    cnt = torch.tensor([c["created"], c["recorded"], c["scattered"]], dtype=torch.float64)
    dist.all_reduce(spec)
    dist.all_reduce(cnt)
    if rank == 0:
        np.save(os.path.join(out_dir, "spec.npy"), spec.numpy())
        np.save(os.path.join(out_dir, "cnt.npy"), cnt.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_equal_single_job(dump32, tmp_path):
    import grmonty_amd as G
    import oracle_py as O
    world = 2
    mp.spawn(_shard_job, args=(world, dump32, str(tmp_path), _free_port()), nprocs=world, join=True)
    spec_d = np.load(tmp_path / "spec.npy")
    cnt_d = np.load(tmp_path / "cnt.npy")
    model = G.Model.load(dump32, photon_n=150 * world).init(2)
    ph = model.emit(seed=123)
    orc = O.OracleModel(dump32, photon_n=150 * world)
    orc.init(2)
    orc.track(ph.view(O.INIT_PHOTON), rng_mode=1, seed=123, id_base=0, frozen=True, scatt0=SNAP["scatt"],
              rec0=SNAP["rec"], max_tau0=SNAP["maxtau"])
    spec_1 = orc.spectrum().view(np.float64).reshape(-1)
    c = orc.counters()
    assert list(cnt_d) == [c["created"], c["recorded"], c["scattered"]]
    np.testing.assert_allclose(spec_d, spec_1, rtol=1e-12, atol=0)
