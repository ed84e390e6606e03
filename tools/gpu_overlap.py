"""Diagnostic: how concurrent run_simulation passes (one engine each) overlap on the GPU.
For every pass: host start/end and, from the per-wave launch records (s_memrealtime, 100 MHz, one
clock for the whole GPU), first wave start, 50/99 % wave exit and last wave exit of its longest
launch, all in ms from the first pass's start."""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import numpy as np  # noqa: E402

import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

jobs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
passes = int(sys.argv[2]) if len(sys.argv) > 2 else 8
os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(4, jobs + 1)))
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=1_000_000).init(0)
engines = [G.Engine(m, 0) for _ in range(jobs)]
for e in engines:
    e.emit_setup(m)
    e.set_option(G.OPT_SEED, 123)
rows = [None] * passes
t_host0 = time.time()


def one(j, s):
    e = engines[j]
    t0 = time.time()
    e.reset()
    e.set_option(G.OPT_ID_BASE, 0)
    p, n = e.emit(seed=123)
    e.track_device(p, n)
    st = e.stats()
    w = e.debug_waves().astype(np.float64)
    rows[s] = (j, t0 - t_host0, time.time() - t_host0, w, st)


def worker(j):
    for s in range(j, passes, jobs):
        one(j, s)


# warm each engine once (sizes buffers)
ths = [threading.Thread(target=one, args=(j, 0)) for j in range(jobs)]
for t in ths:
    t.start()
for t in ths:
    t.join()
rows = [None] * passes
t_host0 = time.time()
ths = [threading.Thread(target=worker, args=(j,)) for j in range(jobs)]
for t in ths:
    t.start()
for t in ths:
    t.join()
wall = time.time() - t_host0
rt0 = min(r[3][:, 0].min() for r in rows)
print(f"jobs {jobs} passes {passes} wall {wall:.2f}s", flush=True)
for s, (j, h0, h1, w, st) in enumerate(rows):
    ws = (w[:, 0] - rt0) / 1e5
    we = (w[:, 1] - rt0) / 1e5
    q = np.percentile(we, [50, 99])
    print(f"pass {s} eng {j}: host {h0 * 1e3:.0f}-{h1 * 1e3:.0f} ms | waves start {ws.min():.0f}-{ws.max():.0f} "
          f"exit p50 {q[0]:.0f} p99 {q[1]:.0f} last {we.max():.0f} | kernel {st['last_kernel_ms']:.0f} ms "
          f"longest life {st['max_photon_steps']}", flush=True)
