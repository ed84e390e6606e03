"""Per pass of the bench's configuration (192^2, photon_n = 1e6, device tables, seeds 123...): wall
time, the dominant bulk launch, the early worker's launch (it runs beside the bulk on a second stream
and takes every photon that reaches GRM_OPT_EARLY_STEPS steps), the photons handed to it, the lone
kernel's time and the longest life -- where a long-photon pass spends its excess.
Usage: python tools/early_probe.py [passes]   (GRM_BENCH_OPTS as in bench.py)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=1e6).init(0, device=0)
e = G.Engine(m, 0)
e.emit_setup(m)
for kv in filter(None, os.environ.get("GRM_BENCH_OPTS", "").split(",")):
    k, v = kv.split("=")
    e.set_option(int(k), int(v))
for s in range(-2, n):  # two warm-up passes of other seeds, as bench.py
    seed = 123 + s if s >= 0 else 9000 + s
    t = time.time()
    e.reset()
    e.set_option(G.OPT_SEED, seed)
    p, cnt = e.emit(seed=seed)
    e.track_device(p, cnt)
    e.finish()
    wall = time.time() - t
    st = e.stats()
    if s < 0:
        continue
    print(f"seed {seed}: wall {wall * 1e3:.1f} ms; bulk {st['max_launch_ms']:.1f} ms, early worker {st['early_ms']:.1f} ms "
          f"({st['n_early']} photons), lone {st['lone_ms']:.1f} ms ({st['n_lone']}), launches {st['n_launches']}, "
          f"longest life {st['max_photon_steps']} steps, lives > 1e5 {st['n_long_photons']}", flush=True)
