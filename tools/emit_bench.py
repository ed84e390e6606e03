"""Device emission time (zone_count_scan + emit_kernel, wall clock around Engine.emit, which
synchronises) at 192^2, photon_n = 1e6, and a checksum of the emitted photons (identical across
builds that emit the same streams).  Usage: python tools/emit_bench.py [reps]"""
import hashlib
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=1e6).init(0, device=0)
e = G.Engine(m, 0)
e.emit_setup(m)
ts = []
for r in range(reps):
    t = time.time()
    p, n = e.emit(seed=123 + r)
    ts.append((time.time() - t) * 1e3)
dev = e.download(*e.emit(seed=123))
print(f"lib {os.environ.get('GRMONTY_AMD_LIB', 'in-tree')}: {n} photons, emit ms {[round(x, 2) for x in ts]}, "
      f"median {sorted(ts)[len(ts) // 2]:.2f} ms; seed-123 sha1 {hashlib.sha1(dev.tobytes()).hexdigest()[:16]}", flush=True)
