"""The command-line driver (host/grm_main.cpp; reference main.cpp:20-53 + run_simulation
harm_model.cpp:340-414 + report_spectrum :416-471) end to end on the GPU: reference flags, device
emission + transport, the reference's end-of-run log lines, a 200 x 37 spectrum file, and recorded /
scattered counts within the seed-to-seed spread of the oracle's reference-semantics runs on the same
dump (tests/golden/oracle_spread_synth64.json)."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "cuda-grmonty_amd", "bin", "grmonty_amd")


@pytest.mark.parametrize("host_emit", [False, True])
def test_cli_run(dump64, tmp_path, host_emit):
    out = tmp_path / "spectrum"
    cmd = [CLI, f"--harm_dump_path={dump64}", f"--spectrum_path={out}", "--photon_n=2000", "--mass_unit=4e19"]
    if host_emit:
        cmd.append("--host_emit")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    log = r.stderr
    for key in ("Final rate", "created:", "scattered:", "recorded:", "lumosity:", "max_tau_scatt:"):
        assert key in log, key
    created = int(re.search(r"created: (\d+)", log).group(1))
    rows = [ln.split() for ln in out.read_text().splitlines()]
    assert len(rows) == 200 and all(len(x) == 37 for x in rows)
    spec = np.array(rows, dtype=float)
    np.testing.assert_allclose(spec[:, 0], (np.arange(200) * 0.25 + np.log(1e-12)) / np.log(10), rtol=1e-4)
    assert created > 20000
    lum = float(re.search(r"lumosity: ([0-9.eE+-]+)", log).group(1))
    assert np.isfinite(lum) and lum > 0
    g = json.load(open(os.path.join(REPO, "tests", "golden", "oracle_spread_synth64.json")))
    for key in ("recorded", "scattered"):
        dev = int(re.search(key + r": (\d+)", log).group(1))
        mu, sd = g["mean"][key], g["std"][key]
        assert abs(dev - mu) <= 4 * sd, (key, dev, mu, sd)
