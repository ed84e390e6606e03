"""Timeline of a pass's main transport launch (grm_engine_debug_phases): when the live-bias warm-up
admission ended, when the pool's last claim chunk was taken, when the last wave left -- over a few
bench-like passes (192^2, photon_n = 1e6, device tables).
Usage: python tools/pass_phases.py [passes] [photon_n]   (GRM_BENCH_OPTS as in bench.py)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
pn = float(sys.argv[2]) if len(sys.argv) > 2 else 1e6
path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
m = G.Model.load(path, photon_n=pn).init(0, device=0)
e = G.Engine(m, 0)
e.emit_setup(m)
for kv in filter(None, os.environ.get("GRM_BENCH_OPTS", "").split(",")):
    k, v = kv.split("=")
    e.set_option(int(k), int(v))
for s in range(n):
    e.reset()
    e.set_option(G.OPT_SEED, 123 + s)
    p, cnt = e.emit(seed=123 + s)
    e.track_device(p, cnt)
    st = e.stats()
    ph = e.debug_phases()
    w = e.debug_waves()
    ex = sorted(((w[:, 1] - w[:, 0].min()) * 1e-5).tolist())
    print(f"seed {123 + s}: dominant {st['max_launch_ms']:.1f} ms, steps {st['max_launch_steps']:.4g}; warm-up ends "
          f"{ph['warmup_end_ms']:.1f} ms, pool drained {ph['pool_drained_ms']:.1f} ms, wave exits p10/50/90/100 "
          f"{ex[len(ex) // 10]:.1f}/{ex[len(ex) // 2]:.1f}/{ex[9 * len(ex) // 10]:.1f}/{ex[-1]:.1f} ms; lone "
          f"{st['n_lone']} photons {st['lone_ms']:.1f} ms, launches {st['n_launches']}; recorded {e.debug_counters()['n_recorded']} "
          f"dropped {st['n_dropped']} abandoned {st['n_abandoned']}", flush=True)
    print("   admissions (ms, in flight): " + " ".join(f"{t:.1f}/{f}" for t, f in ph["admissions"]), flush=True)
