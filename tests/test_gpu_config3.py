"""BASELINE configs[3] -- 8 x MI355X, photon_n = 1e8 sharded -- the WHOLE job run on one GPU.

tests/multirank_emu.py runs the eight ranks of the job concurrently, each an engine on 1/8 of the
CUs with the zone shard bench.py gives rank r of 8 (grmonty_amd.zone_shards: every 8th zone from r,
~1.8e8 superphotons each, 1.46e9 in the job), its global photon id base and its pass counter block;
the eight blocks are linked (grm_engine_link_peers), so every rank's kernels run bias_func on the
job's counters and every rank takes part in the job's warm-up (1/8 shares of one GPU's batches behind
the job barrier), as grm_engine_set_peers makes them do over xGMI on the 8-GPU node.  The eight
ranks' results are then reduced as the job's one all-reduce does (spectrum and counters summed,
max tau_scatt maxed).

Asserted (the reference keeps int32 device counters, super_photon.cu:41-46, 978-979 -- SURVEY Q7;
here every counter is u64):
  - no child dropped and no photon abandoned on any rank (multirank_emu fails the job otherwise);
  - every rank's transport-step counter past 2^32 would be needed for the job (job steps > 2^34);
  - the job's u64 counters = the sums of the ranks' spectra's independent fp64 sums (nph = recorded,
    nscatt = scattered; integers below 2^53 add exactly in fp64), and every rank's kernel-side view
    of the job counters = the sums of the ranks' own counters and the max of their max tau_scatt;
  - the job's warm-up ended on every rank, within WARMUP_MS of its launch start (a job barrier that
    never opened would hold it to the 1 s stall guard -- ADVICE r04), and EVERY rank admitted in
    batches: the ranks emit first and launch together, and the launches meet at the job's
    device-side start barrier (job_started, grm_engine.hip), so no rank's warm-up begins after the
    job's has ended (round 5 saw two of eight ranks log only the closing entry);
  - no rank's early-worker queue filled (at 1,500 steps a 1.8e8-photon shard handed over
    888-1,024 photons to a 1,024-slot queue);
  - the JOB's luminosity within LUM_BAR of the photon_n = 1e6 oracle runs' mean
    (tests/golden/oracle_synth192_pn1e6.json, 42 runs, spread 0.11 %): the estimator is unbiased
    whatever the adaptive bias, and at 1.46e9 superphotons its Monte Carlo error is ~0.01 %.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WORLD = 8
PHOTON_N = 100_000_000
LUM_BAR = 0.002
WARMUP_MS = 500.0
EARLY_CAP = 1024


def test_whole_photon_n_1e8_job_on_one_gpu(dump_dir, tmp_path):
    from grmonty_amd.synth_dump import ensure_dump
    path = ensure_dump(os.path.join(dump_dir, "synth192.dump"), 192, 192)
    out = tmp_path / "job.json"
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(2 * WORLD + 2))
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "multirank_emu.py"), path, str(WORLD), "1", str(out),
                        "--shared", "--phases", "--photon-n", str(PHOTON_N)],
                       env=env, capture_output=True, text=True, timeout=400)
    print(r.stdout[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    job = json.load(open(out))[0]
    per = job["per_rank_created"]
    print(f"job: {job['created']} superphotons over {WORLD} ranks ({min(per)}..{max(per)} per rank), "
          f"{job['recorded']} recorded, {job['scattered']} scattered, {job['steps']} steps, "
          f"max tau_scatt {job['max_tau']:.4g}")
    assert 1.3e9 < job["created"] < 1.6e9 and all(1.5e8 < n < 2.2e8 for n in per)
    assert job["steps"] > 2 ** 34
    assert float(job["rec_spec"]) == float(job["recorded"])
    assert float(job["scatt_spec"]) == float(job["scattered"])
    for v in job["job_view"]:
        assert v["n_recorded"] == job["recorded"] and v["n_scatt"] == job["scattered"]
        assert v["max_tau_scatt"] == job["max_tau"]
    for rk, ph in enumerate(job["per_rank_phases"]):
        print(f"rank {rk}: warm-up end {ph['warmup_end_ms']} ms, {len(ph['admissions'])} admission batches, "
              f"pool drained {ph['pool_drained_ms']} ms, last exit {ph['last_exit_ms']} ms")
        assert ph["warmup_end_ms"] is not None and 0 <= ph["warmup_end_ms"] < WARMUP_MS, ph
        assert len(ph["admissions"]) >= 2, (rk, ph)
    # the early worker's queue (EARLY_CAP = 1024 slots per launch) must not fill: its hand-over
    # threshold grows with the call's photons (grm_engine::early_steps_for, ~2,000 steps here)
    print(f"early-worker hand-overs per rank: {job['per_rank_n_early']} (queue 1024)")
    assert all(n < EARLY_CAP for n in job["per_rank_n_early"])
    o = json.load(open(os.path.join(HERE, "golden", "oracle_synth192_pn1e6.json")))["runs"]
    l_o = np.array([x["luminosity"] for x in o])
    rel = job["luminosity"] / l_o.mean() - 1
    print(f"job luminosity {job['luminosity']:.5f}, oracle photon_n=1e6 {l_o.mean():.5f} +- "
          f"{l_o.std(ddof=1) / l_o.mean():.3%} ({len(l_o)} runs): {rel:+.3%} (bar {LUM_BAR:.1%})")
    assert abs(rel) < LUM_BAR
