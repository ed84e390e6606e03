"""RCCL all-reduce of the spectrum/counters from the engine's C library (the multi-GPU exchange
step).  On a 1-GPU box a single-rank communicator is exercised: the all-reduce must leave the
spectrum and counters unchanged."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_single_rank_allreduce_is_identity(model64):
    import grmonty_amd as G
    e = G.Engine(model64, device=0)
    ph = model64.emit(seed=3)[:3000]
    d = e.upload(ph)
    e.set_option(G.OPT_SEED, 11)
    e.track_device(d, len(ph))
    s0, r0, c0, m0 = e.finish()
    e.comm_init(G.rccl_unique_id(), 1, 0)
    e.allreduce()
    s1, r1, c1, m1 = e.finish()
    assert (r0, c0, m0) == (r1, c1, m1)
    np.testing.assert_array_equal(s0.view(np.float64), s1.view(np.float64))
    e.close()


def test_single_rank_stash_reduce_is_identity(model64):
    """grm_engine_stash / _allreduce_stash / _stash_read (bench.py's one exchange per job): with one
    rank, every stashed pass reads back exactly as grm_engine_finish returned it"""
    import grmonty_amd as G
    e = G.Engine(model64, device=0)
    ph = model64.emit(seed=3)[:3000]
    d = e.upload(ph)
    e.comm_init(G.rccl_unique_id(), 1, 0)
    e.stash_reserve(3)
    ref = []
    for slot, seed in enumerate((11, 12, 13)):
        e.reset()
        e.set_option(G.OPT_SEED, seed)
        e.track_device(d, len(ph))
        e.stash(slot)
        ref.append(e.finish())
    e.allreduce_stash(2, 1)  # slots [1, 3), then slot 0: each slot reduced once
    e.allreduce_stash(1, 0)
    for slot, (s0, r0, c0, m0) in enumerate(ref):
        s1, r1, c1, m1, _ = e.stash_read(slot)
        assert (r0, c0, m0) == (r1, c1, m1)
        np.testing.assert_array_equal(s0.view(np.float64), s1.view(np.float64))
    e.close()
