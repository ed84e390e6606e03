"""pytest configuration: `gpu` marker, shared fixtures (synthetic dumps, oracle and product models)."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "cuda-grmonty_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


# The statistical parity tests (counter means and KS of live-bias jobs against the oracle's runs)
# run after every deterministic test: under `-x` a statistical failure then still leaves the
# photon-by-photon, probe, table and safety results of the run recorded.
STATISTICAL = ("test_gpu_parity_192.py", "test_gpu_multirank.py::test_emulated_ranks_vs_oracle")


def pytest_collection_modifyitems(config, items):
    items.sort(key=lambda it: any(k in it.nodeid for k in STATISTICAL))  # stable: order kept otherwise


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dump_dir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("dumps"))


@pytest.fixture(scope="session")
def dump64(dump_dir):
    from grmonty_amd.synth_dump import write_dump
    return write_dump(os.path.join(dump_dir, "synth64.dump"), 64, 64)


@pytest.fixture(scope="session")
def dump32(dump_dir):
    from grmonty_amd.synth_dump import write_dump
    return write_dump(os.path.join(dump_dir, "synth32.dump"), 32, 48)


@pytest.fixture(scope="session")
def oracle64(dump64):
    import oracle_py as O
    m = O.OracleModel(dump64, photon_n=2000)
    m.init(8)
    return m


@pytest.fixture(scope="session")
def model64(dump64):
    import grmonty_amd as G
    return G.Model.load(dump64, photon_n=2000).init(8)
