"""Statistical parity at the headline scale: the device vs the reference CPU semantics on the
192x192 dump019-class synthetic dump at photon_n = 1e5 (BASELINE configs[0]; SURVEY.md §8(d)
parity check: KS on nu L_nu, counters within the seed spread).

Reference side: six oracle run_simulation runs (serial, mt19937, live adaptive bias;
tests/golden/oracle_synth192_pn1e5.*, tools/make_golden_192.py), pooled for the KS test.
Device side: one run_simulation pass as bench.py runs it -- device emission (seed 123), transport
with the live adaptive bias -- with every photon end traced for the per-cell sums.

Asserted:
  - binned KS on the nu L_nu cumulative (Kish effective N), per theta bin and summed, alpha = 1e-4
    per statistic (the oracle seeds pass the same statistic against each other at 1e-3,
    tests/test_golden_192.py);
  - created within 6 sigma of the oracle mean (stochastic rounding of the zone counts);
  - recorded, scattered and transport steps within 5 sigma of the oracle seed-to-seed spread;
  - luminosity (report_spectrum, harm_model.cpp:461) within 5 sigma of the oracle spread.
"""
import json
import os

import numpy as np
import pytest

from spectrum_stats import binned_ks, cell_sums_from_trace, ks_crit

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden", "oracle_synth192_pn1e5")


def test_headline_scale_statistics_vs_oracle(dump_dir):
    import grmonty_amd as GA
    from grmonty_amd.synth_dump import write_dump
    gold = np.load(G + ".npz")
    summ = json.load(open(G + ".json"))
    path = write_dump(os.path.join(dump_dir, "synth192.dump"), 192, 192)
    model = GA.Model.load(path, photon_n=100000).init(8)
    eng = GA.Engine(model, device=0)
    eng.emit_setup(model)
    eng.reset()
    eng.set_option(GA.OPT_SEED, 123)
    eng.set_option(GA.OPT_TRACE_CAP, 12_000_000)
    p, n = eng.emit(seed=123)
    eng.track_device(p, n)
    tr = eng.trace(12_000_000)
    spec, n_rec, n_scatt, _ = eng.finish()
    st = eng.stats()
    eng.close()
    assert st["n_dropped"] == 0 and st["n_abandoned"] == 0
    assert len(tr) == st["n_tracked"], "trace overflow"
    lum = model.write_spectrum(spec, None)["luminosity"]
    mean, sd = summ["mean"], summ["std"]
    print(f"device: created {n} recorded {n_rec} scattered {n_scatt} steps {st['n_steps']} L {lum:.4f}")
    print(f"oracle: created {mean['created']:.0f}+-{sd['created']:.0f} recorded {mean['recorded']:.0f}+-"
          f"{sd['recorded']:.0f} scattered {mean['scattered']:.0f}+-{sd['scattered']:.0f} steps "
          f"{mean['steps']:.3g}+-{sd['steps']:.2g} L {mean['luminosity']:.4f}+-{sd['luminosity']:.4f}")
    assert abs(n - mean["created"]) <= 6 * max(sd["created"], np.sqrt(mean["created"]) * 0.05)
    for key, dev in (("recorded", n_rec), ("scattered", n_scatt), ("steps", st["n_steps"]), ("luminosity", lum)):
        assert abs(dev - mean[key]) <= 5 * sd[key], (key, dev, mean[key], sd[key])
    # per-cell sums on the device; the spectrum's own sums cross-check the trace
    cd = cell_sums_from_trace(tr)
    np.testing.assert_allclose(cd[:, 0], spec["nph"].reshape(-1), rtol=0, atol=0.5)
    np.testing.assert_allclose(cd[:, 3], spec["de_dle"].reshape(-1), rtol=1e-9, atol=0)
    pooled = gold["cells"].sum(axis=0)
    for th in [None, 0, 1, 2, 3, 4, 5]:
        d, n1, n2 = binned_ks(cd, pooled, th)
        crit = ks_crit(n1, n2, 1e-4)
        print(f"theta bin {th}: KS D={d:.4f} crit={crit:.4f} n_eff device {n1:.0f} oracle (6 runs) {n2:.0f}")
        assert d < crit, th
