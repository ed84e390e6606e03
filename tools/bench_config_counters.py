"""Counter means of many bench-configuration passes (192^2, photon_n = 1e6, tables built on the GPU,
device emission, live bias -- BASELINE configs[1] as bench.py runs it) against the photon_n = 1e6
oracle fixture (tests/golden/oracle_synth192_pn1e6.json).  tests/test_gpu_parity_192.py checks 8 passes
in the suite; this tool runs more (seeds 123.., one engine, each pass after grm_engine_reset) and
writes their counters to a JSON list, for a tighter comparison (tools/emu_vs_oracle.py reads it).

    python tools/bench_config_counters.py OUT.json [passes]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "cuda-grmonty_amd"), os.path.join(REPO, "tests")]
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402
from job_util import run_job  # noqa: E402

out = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 48
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
model = G.Model.load(path, photon_n=1_000_000).init(8, device=0)
eng = G.Engine(model, device=0)
eng.emit_setup(model)
res = []
for s in range(n):
    j = run_job(eng, model, 123 + s)
    res.append({k: (float(j[k]) if k == "luminosity" else int(j[k])) for k in
                ("created", "recorded", "scattered", "steps", "luminosity")})
    res[-1]["seed"] = 123 + s
    print(json.dumps(res[-1]), flush=True)
eng.close()
json.dump(res, open(out, "w"))
