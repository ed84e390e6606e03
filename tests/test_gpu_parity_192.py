"""Statistical parity at the headline scale: the device vs the reference CPU semantics on the
192x192 dump019-class synthetic dump at photon_n = 1e5 (BASELINE configs[0]; SURVEY.md §8(d)
parity check: KS on nu L_nu, counters within the seed spread).

Reference side: the oracle's run_simulation (serial, mt19937, live adaptive bias) for every seed in
tests/golden/oracle_synth192_pn1e5.* (tools/make_golden_192.py), pooled for the KS test.
Device side: run_simulation jobs as bench.py runs them -- device emission, transport with the live
adaptive bias -- with the init tables built on the host (grm_model_init) or on the GPU
(grm_model_init_device, the path bench.py times), both under test.

Asserted:
  - one traced job (seed 123): binned KS on the nu L_nu cumulative (Kish effective N), per theta bin
    and summed, alpha = 1e-4 per statistic (the oracle seeds pass the same statistic against each
    other at 1e-3, tests/test_golden_192.py); the spectrum's own sums cross-check the trace;
  - N_DEV jobs of distinct seeds: the MEAN of recorded, scattered, transport steps and luminosity
    against the oracle runs' mean, |difference| <= Z_MAX combined standard errors (Welch: each side's
    own sample variance over its own run count).  The live adaptive bias makes the counters of one
    run scatter by 4-6 % (sd) on either side, so the means need many runs: 96 device jobs (0.25 s
    each) against 60 oracle runs give a combined standard error of ~0.8 % of recorded, and a
    systematic offset of the scattering or adaptive-bias machinery above ~3.5 % fails.  Measured
    (round 4, 24-run means): the device +0.0 to +4.3 %, the oracle's concurrency emulator scheduling
    the reference like the device +2.9 % and serially +1.2 % (tools/lag_emulator.py,
    tests/golden/lag_emulator_synth192_pn1e5.json) -- concurrency moves the counters by ~1-2 %.
"""
import json
import os

import numpy as np
import pytest

from job_util import KEYS, run_job
from spectrum_stats import binned_ks, ks_crit, welch_z

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
G = os.path.join(HERE, "golden", "oracle_synth192_pn1e5")
N_DEV = 96
Z_MAX = 4.5


def oracle_runs():
    summ = json.load(open(G + ".json"))
    return {k: np.array([r[k] for r in summ["runs"]], dtype=np.float64) for k in KEYS + ("created",)}


@pytest.fixture(scope="module", params=["host-tables", "device-tables"])
def setup192(request, dump_dir):
    import grmonty_amd as GA
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump(os.path.join(dump_dir, "synth192.dump"), 192, 192)
    model = GA.Model.load(path, photon_n=100000)
    model.init(8) if request.param == "host-tables" else model.init(8, device=0)
    eng = GA.Engine(model, device=0)
    eng.emit_setup(model)
    yield model, eng
    eng.close()


def test_headline_ks_vs_oracle(setup192):
    model, eng = setup192
    gold = np.load(G + ".npz")
    o = oracle_runs()
    job = run_job(eng, model, 123, trace_cap=12_000_000)
    print(f"device seed 123: created {job['created']} recorded {job['recorded']} scattered {job['scattered']} "
          f"steps {job['steps']} L {job['luminosity']:.4f}")
    assert abs(job["created"] - o["created"].mean()) <= 6 * max(o["created"].std(ddof=1),
                                                                 np.sqrt(o["created"].mean()) * 0.05)
    cd = job["cells"]
    spec = job["spectrum"]
    np.testing.assert_allclose(cd[:, 0], spec["nph"].reshape(-1), rtol=0, atol=0.5)
    np.testing.assert_allclose(cd[:, 3], spec["de_dle"].reshape(-1), rtol=1e-9, atol=0)
    pooled = gold["cells"].sum(axis=0)
    for th in [None, 0, 1, 2, 3, 4, 5]:
        d, n1, n2 = binned_ks(cd, pooled, th)
        crit = ks_crit(n1, n2, 1e-4)
        print(f"theta bin {th}: KS D={d:.4f} crit={crit:.4f} n_eff device {n1:.0f} oracle "
              f"({len(gold['cells'])} runs) {n2:.0f}")
        assert d < crit, th


EMU = os.path.join(HERE, "golden", "lag_emulator_synth192_pn1e5.json")


def emulator_runs(config):
    """the oracle's concurrency emulator runs of one scheduling configuration (tools/lag_emulator.py)"""
    runs = [r for r in json.load(open(EMU))["runs"] if r["config"] == config]
    return {k: np.array([r[k] for r in runs], dtype=np.float64) for k in KEYS}


def test_headline_counter_means_vs_oracle(setup192):
    """The device's counter means against (1) the reference (the oracle's serial runs, mt19937) and
    (2) the reference SCHEDULED AS THE DEVICE SCHEDULES IT: the oracle's concurrency emulator
    (grmo_track_concurrent) with the device's lanes in flight at this size (14,848: the in-flight cap's
    29 workgroups), wave stacks, deferred children, counter snapshots every 64 trips and interleaved
    claims (config "device_cap", tests/golden/lag_emulator_synth192_pn1e5.json).  Both within Z_MAX
    combined standard errors: (2) tests that what separates the device from the serial reference is
    the concurrency of its live bias (bias_func's counters trail the photons in flight,
    harm_model.cpp:1391-1404), not the scattering or the counter machinery.  The emulator's serial
    configuration (the reference's own scheduling on the device's Philox streams) is printed beside."""
    model, eng = setup192
    o = oracle_runs()
    emu, ser = emulator_runs("device_cap"), emulator_runs("serial")
    dev = {k: [] for k in KEYS}
    for s in range(N_DEV):
        job = run_job(eng, model, 123 + s)
        for k in KEYS:
            dev[k].append(job[k])
    bad = []
    for k in KEYS:
        diff, se, z = welch_z(dev[k], o[k])
        de, _, ze = welch_z(dev[k], emu[k])
        print(f"{k:10s} device {np.mean(dev[k]):.6g} +- {np.std(dev[k], ddof=1):.3g} ({N_DEV} runs)  oracle "
              f"{o[k].mean():.6g} +- {o[k].std(ddof=1):.3g} ({len(o[k])} runs)  diff {diff / o[k].mean():+.2%} "
              f"= {z:+.2f} SE | device-scheduled emulator {emu[k].mean():.6g} ({len(emu[k])} runs): diff "
              f"{de / emu[k].mean():+.2%} = {ze:+.2f} SE | serial emulator vs oracle "
              f"{ser[k].mean() / o[k].mean() - 1:+.2%} ({len(ser[k])} runs)")
        if abs(z) > Z_MAX:
            bad.append((k, "oracle", z))
        if abs(ze) > Z_MAX:
            bad.append((k, "emulator", ze))
    assert not bad, bad


G6 = os.path.join(HERE, "golden", "oracle_synth192_pn1e6")
N_DEV6 = 8


def test_bench_config_vs_oracle(dump_dir):
    """The bench's own configuration (BASELINE configs[1]): photon_n = 1e6 on the 192^2 dump, tables
    built on the GPU, as bench.py runs it, against 42 oracle run_simulation runs at photon_n = 1e6
    (tests/golden/oracle_synth192_pn1e6.*, ~1 h of CPU each; seeds 123-164): the binned KS test of one traced pass
    and the counter means of N_DEV6 passes (Welch, |diff| <= Z_MAX standard errors)."""
    import grmonty_amd as GA
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump(os.path.join(dump_dir, "synth192.dump"), 192, 192)
    model = GA.Model.load(path, photon_n=1_000_000).init(8, device=0)
    eng = GA.Engine(model, device=0)
    eng.emit_setup(model)
    summ = json.load(open(G6 + ".json"))
    o = {k: np.array([r[k] for r in summ["runs"]], dtype=np.float64) for k in KEYS}
    dev = {k: [] for k in KEYS}
    job = None
    for s in range(N_DEV6):
        j = run_job(eng, model, 123 + s, trace_cap=40_000_000 if s == 0 else 0)
        job = j if s == 0 else job
        for k in KEYS:
            dev[k].append(j[k])
    eng.close()
    bad = []
    for k in KEYS:
        diff, se, z = welch_z(dev[k], o[k])
        print(f"1e6 {k:10s} device {np.mean(dev[k]):.6g} +- {np.std(dev[k], ddof=1):.3g} ({N_DEV6} passes)  oracle "
              f"{o[k].mean():.6g} +- {o[k].std(ddof=1):.3g} ({len(o[k])} runs)  diff {diff / o[k].mean():+.2%} = {z:+.2f} SE")
        if abs(z) > Z_MAX:
            bad.append((k, z))
    pooled = np.load(G6 + ".npz")["cells"].sum(axis=0)
    for th in [None, 0, 1, 2, 3, 4, 5]:
        d, n1, n2 = binned_ks(job["cells"], pooled, th)
        crit = ks_crit(n1, n2, 1e-4)
        print(f"1e6 theta bin {th}: KS D={d:.4f} crit={crit:.4f} n_eff device {n1:.0f} oracle {n2:.0f}")
        if not d < crit:
            bad.append(("ks", th, d, crit))
    assert not bad, bad
