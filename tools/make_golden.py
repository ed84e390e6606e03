"""Regenerate the committed fixtures under tests/golden/ (run in the dev container).

  oracle_spread_synth64.json  seed-to-seed spread of the oracle's counters (reference CPU semantics:
                              mt19937, live bias) on synth64 at photon_n=2000 -- the yardstick for
                              comparing device counters (cascades make them over-dispersed vs sqrt(N)).
  ref_samplers.npz            outputs of the REFERENCE's own proba/tetrads code (oracle/_ref partial
                              build, seed 123) for fixed inputs: lets the GPU box (no /root/reference)
                              still check the oracle against real reference outputs.
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import ctypes as C  # noqa: E402

import oracle_py as O  # noqa: E402
from grmonty_amd.synth_dump import write_dump  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")
DP = C.POINTER(C.c_double)


def spread():
    path = write_dump("/tmp/golden_synth64.dump", 64, 64)
    rows = []
    for seed in (123, 7, 99, 1000, 31337, 2):
        m = O.OracleModel(path, photon_n=2000)
        m.init(8)
        ph = m.emit(seed)
        m.track(ph, rng_mode=0, seed=seed, frozen=False)
        c = m.counters()
        rows.append(dict(seed=seed, created=len(ph), recorded=c["recorded"], scattered=c["scattered"],
                         steps=c["steps"], max_tau_scatt=m.scalars()["max_tau_scatt"]))
        print(rows[-1], flush=True)
    r = {k: [row[k] for row in rows] for k in rows[0]}
    out = dict(dump="synth64 (write_dump(path, 64, 64))", photon_n=2000, runs=rows,
               mean={k: float(np.mean(v)) for k, v in r.items() if k != "seed"},
               std={k: float(np.std(v, ddof=1)) for k, v in r.items() if k != "seed"})
    json.dump(out, open(os.path.join(GOLD, "oracle_spread_synth64.json"), "w"), indent=1)


def ref_samplers():
    R = O.ref()
    assert R is not None, "needs the partial reference build (make -C oracle)"
    rng = np.random.default_rng(2025)
    n = 300
    k = rng.normal(size=(n, 4))
    k[:, 0] = np.linalg.norm(k[:, 1:], axis=1)
    k *= 10 ** rng.uniform(-5, 1, n)[:, None]
    te = 10 ** rng.uniform(-1.5, 2.5, n)
    R.ref_rng_init(123)
    p = np.zeros((n, 4))
    for i in range(n):
        kk = np.ascontiguousarray(k[i])
        out = np.zeros(4)
        R.ref_sample_electron(kk.ctypes.data_as(DP), out.ctypes.data_as(DP), te[i])
        p[i] = out
    k0 = 10 ** rng.uniform(-4, 3, n)
    kn = np.array([R.ref_sample_klein_nishina(v) for v in k0])
    th = np.array([R.ref_sample_thomson() for _ in range(n)])
    np.savez(os.path.join(GOLD, "ref_samplers.npz"), k=k, theta_e=te, p=p, k0=k0, kn=kn, thomson=th)


if __name__ == "__main__":
    os.makedirs(GOLD, exist_ok=True)
    ref_samplers()
    spread()
