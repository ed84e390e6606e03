"""The C-ABI library loads and exports every symbol that include/grmonty_amd.h declares; POD
struct sizes agree between the header, the library and the oracle (no compute, no GPU)."""
import ctypes as C

import grmonty_amd as G
import oracle_py as O


def test_all_header_symbols_exported():
    L = G.lib()
    names = G.header_symbols()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert set(names) == set(G.SIGNATURES), set(names) ^ set(G.SIGNATURES)


def test_struct_sizes():
    L = G.lib()
    assert L.grm_sizeof(0) == C.sizeof(G.Header) == O.lib().grmo_sizeof(0)
    assert L.grm_sizeof(1) == C.sizeof(G.Units) == 64
    assert L.grm_sizeof(2) == G.INIT_PHOTON.itemsize == 128
    assert L.grm_sizeof(3) == G.SPECTRUM_CELL.itemsize == 104
    assert L.grm_sizeof(4) == G.TRACE.itemsize == O.TRACE.itemsize
    assert L.grm_sizeof(5) == C.sizeof(G.Stats)
    assert L.grm_version().decode().startswith("grmonty_amd")


def test_engine_creation_fails_loudly_without_gpu(model64):
    """No CPU fallback: without a HIP device the engine reports an error instead of running."""
    import pytest
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError):
        G.Engine(model64, device=0)
