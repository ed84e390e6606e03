"""Quick GPU performance snapshot: transport of an emitted batch, kernel time, steps/s."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import numpy as np  # noqa: E402

import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 192
photon_n = int(float(sys.argv[2])) if len(sys.argv) > 2 else 100000
grid = int(sys.argv[3]) if len(sys.argv) > 3 else 0
path = ensure_dump(os.path.join(REPO, "gpurun_out", f"synth{n}.dump"), n, n)
t = time.time()
m = G.Model.load(path, photon_n=photon_n).init(0)
print(f"init {time.time() - t:.2f}s", flush=True)
t = time.time()
ph = m.emit(seed=123)
print(f"emit {len(ph)} photons {time.time() - t:.2f}s", flush=True)
e = G.Engine(m, 0)
if grid:
    e.set_option(G.OPT_GRID_BLOCKS, grid)
if os.environ.get("SPLIT"):
    e.set_option(G.OPT_SPLIT, int(os.environ["SPLIT"]))
    print(f"split {os.environ['SPLIT']}", flush=True)
for key, opt in (("SPLIT_THR", 24), ("SPLIT_SPIN", 25), ("SPLIT_GTHR", 26), ("SPLIT_BATCH", 27)):
    if os.environ.get(key):
        e.set_option(opt, int(os.environ[key]))
        print(f"{key} {os.environ[key]}", flush=True)
if os.environ.get("WARMUP"):
    e.set_option(G.OPT_WARMUP, int(os.environ["WARMUP"]))
    print(f"warmup {os.environ['WARMUP']}", flush=True)
e.set_option(G.OPT_WATCHDOG_MS, int(os.environ.get("WATCHDOG_MS", "60000")))
if os.environ.get("EARLY_STEPS"):
    e.set_option(G.OPT_EARLY_STEPS, int(os.environ["EARLY_STEPS"]))
    print(f"early steps {os.environ['EARLY_STEPS']}", flush=True)
if os.environ.get("SLACK"):
    e.set_option(G.OPT_WARMUP_SLACK, int(os.environ["SLACK"]))
    print(f"warmup slack {os.environ['SLACK']}", flush=True)
if os.environ.get("WARMUP_BATCH"):
    e.set_option(G.OPT_WARMUP_BATCH, int(os.environ["WARMUP_BATCH"]))
    print(f"warmup batch {os.environ['WARMUP_BATCH']}", flush=True)
if os.environ.get("CHILD_MIN"):
    e.set_option(G.OPT_CHILD_MIN, int(os.environ["CHILD_MIN"]))
    print(f"child_min {os.environ['CHILD_MIN']}", flush=True)
if os.environ.get("REFILL_MIN"):
    e.set_option(G.OPT_REFILL_MIN, int(os.environ["REFILL_MIN"]))
    print(f"refill_min {os.environ['REFILL_MIN']}", flush=True)
dev_emit = os.environ.get("DEV_EMIT")
if dev_emit:
    e.emit_setup(m)
for rep in range(int(os.environ.get('DIAG_REPS', '3'))):
    e.reset()
    if os.environ.get("IDB"):
        e.set_option(G.OPT_ID_BASE, int(os.environ["IDB"].split(",")[rep]))
    seed = int(os.environ.get("SEED", "123")) + rep  # distinct Monte Carlo pass per rep
    e.set_option(G.OPT_SEED, seed)
    t = time.time()
    try:
        if dev_emit:
            p, n_dev = e.emit(seed=seed)
            e.track_device(p, n_dev)
        else:
            e.track(ph)
    except RuntimeError as exc:
        print(f"rep {rep}: FAILED after {time.time() - t:.1f}s: {exc}", flush=True)
        np.set_printoptions(linewidth=200, precision=6)
        print("stuck: id n_step phase depth pend w e_0_s dl x0..3 k0..3", flush=True)
        print(e.debug_stuck()[:16], flush=True)
        sys.exit(3)
    wall = time.time() - t
    spec, nr, ns, mt = e.finish()
    st = e.stats()
    n_em = n_dev if dev_emit else len(ph)
    print(f"rep {rep} seed {seed}: wall {wall:.3f}s kernel {st['last_kernel_ms']:.1f}ms steps {st['last_steps']} "
          f"({st['last_steps'] / st['last_kernel_ms'] / 1e3:.3g} Msteps/s) tracked {st['n_tracked']} "
          f"children {st['n_children']} overflow {st['n_overflow']} launches {st['n_launches']} "
          f"rate {n_em / wall:.4g} ph/s rec {nr} scatt {ns} | longest launch "
          f"{st['max_launch_ms']:.1f}ms ({st['max_launch_steps']} steps) longest life {st['max_photon_steps']} steps, "
          f"{st['n_long_photons']} lives > 1e5 steps, {st['n_nan_photons']} NaN-ended", flush=True)
    wv = e.debug_waves().astype(np.float64)
    t0w = wv[:, 0].min()
    ex = (wv[:, 1] - t0w) / 1e5  # ms
    st_ = (wv[:, 0] - t0w) / 1e5
    q = np.percentile(ex, [0, 10, 50, 90, 99, 100])
    print(f"  waves {len(wv)}: start max {st_.max():.2f}ms, exit ms p0/10/50/90/99/100 "
          + "/".join(f"{v:.0f}" for v in q) + f", trips max/median {wv[:, 2].max():.0f}/{np.median(wv[:, 2]):.0f}, "
          f"photons max/median {wv[:, 3].max():.0f}/{np.median(wv[:, 3]):.0f}, "
          f"bulk {st['last_steps'] / max(q[2], 1e-9) / 1e3:.4g} Msteps/s (steps / median wave exit)", flush=True)
    inst, tm = e.debug_timing(reset=True)
    if inst:
        if os.environ.get("SPLIT"):
            it, gt = tm[0:8], tm[8:16]
            print(f"  split interaction waves: trips {it[0]}, rounds {it[1]} ({it[1] / max(it[0], 1):.3f} of trips), "
                  f"ready lanes/round {it[2] / max(it[1], 1):.1f} of active {it[3] / max(it[1], 1):.1f}, cycles: "
                  f"evaluation {it[4] / max(it[1], 1):.0f}/round = {it[4] / max(it[5], 1):.3f} of the loop, waiting trips "
                  f"{it[6]}, refill trips {it[7]}; per round: to the fluid {tm[44] / max(it[1], 1):.0f}, gather+fluid "
                  f"{tm[45] / max(it[1], 1):.0f}, radiation+bias {tm[46] / max(it[1], 1):.0f} cycles; per trip: loop top + "
                  f"refill {tm[32] / max(it[0], 1):.0f}, hand-overs {tm[33] / max(it[0], 1):.0f}, readiness "
                  f"{tm[34] / max(it[0], 1):.0f} cycles", flush=True)
            print(f"  split geometry waves: trips {gt[0]}, push trips {gt[1]}, pushing lanes/push trip "
                  f"{gt[2] / max(gt[1], 1):.1f}, ring-full lanes/trip {gt[3] / max(gt[0], 1):.1f}, idle lanes/trip "
                  f"{gt[4] / max(gt[0], 1):.1f}, push cycles/push trip {gt[6] / max(gt[1], 1):.0f} = "
                  f"{gt[6] / max(gt[5], 1):.3f} of the loop, idle trips {gt[7]}", flush=True)
        tot = max(tm[3], 1)
        names = {0: "child", 1: "init", 2: "trip-tail", 7: "bias", 8: "phase0", 9: "attempt", 10: "restore",
                 11: "fluid", 12: "radiation", 13: "interact", 14: "refill-decision"}
        print("  timing: " + " ".join(f"{v}={tm[k] / tot:.3f}" for k, v in names.items()) +
              f" | trips/wave {tm[4]} child-refills {tm[5] / max(tm[4], 1):.4f} pool-refills "
              f"{tm[6] / max(tm[4], 1):.4f} cycles/trip {tot / max(tm[4], 1):.0f} | lone kernel: {st['n_lone']} photons "
          f"{st['lone_ms']:.1f} ms, interaction-wave wait {tm[30] / 2.4e6:.1f} ms geometry-wave wait "
          f"{tm[31] / 2.4e6:.1f} ms (s_memtime at 2.4 GHz)", flush=True)
        if tm[34]:
            print(f"  lane occupancy (track_kernel): push attempt {tm[35] / tm[34]:.1f} lanes in {tm[34]} executions, "
                  f"fluid/radiation/interaction block {tm[33] / max(tm[32], 1):.1f} lanes in {tm[32]} executions", flush=True)
        for lo, what in ((36, "photons > 1e5 steps"), (40, "other photons")):
            if tm[lo]:
                print(f"  lone interaction wave, {what}: {tm[lo]} batches of {tm[lo + 1] / tm[lo]:.2f} steps; cycles: "
                      f"batch evaluation {tm[lo + 2] / tm[lo]:.0f} per batch, serial {tm[lo + 3] / tm[lo + 1]:.0f} per "
                      f"step, total {(tm[lo + 2] + tm[lo + 3]) / tm[lo + 1]:.0f} per step", flush=True)
        for lo, what in ((16, "photons > 1e5 steps"), (22, "other photons")):
            if tm[lo]:
                n_, r_ = tm[lo], tm[lo + 1]
                print(f"  lone geometry wave, {what}: {n_} steps, walk rounds/step {r_ / n_:.3f}, halved "
                      f"{tm[lo + 5] / n_:.3f}; cycles/step: walk {tm[lo + 2] / n_:.0f} (per round "
                      f"{tm[lo + 2] / max(r_, 1):.0f}) step_size+pack {tm[lo + 3] / n_:.0f} loop-rest "
                      f"{tm[lo + 4] / n_:.0f}", flush=True)
