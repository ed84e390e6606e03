"""Multi-GPU scaling model of bench.py from measured single-GPU pass times.

A measured pass (192^2, photon_n = 1e6, 14.5 M superphotons) is t = c + b + e:
  c  fixed per pass, independent of the photon count: the live-bias warm-up admission (~20 ms of
     batch barriers), launches, counter readback -- C_FIXED below;
  b  proportional to the rank's photons: emission + the bulk transport (median pass - c);
  e  the long-photon excess, t - median when positive: a photon of 1e5-1e6 steps whose serial chain
     (two-wave pair, ~1.6 us/step) outlives the bulk.
Weak scaling (bench.py default, photon_n per GPU): every rank runs full passes with independent draws
from the measured distribution; with the job's one reduction (grm_engine_allreduce_stash) the job
takes max over ranks of the rank's summed pass times.
Strong scaling (photon_n for the job): a rank's pass is c + b / N; a pass's long photon (if any) is on
one rank: its chain L = e + b - s started at s ~ U(0, b) in the single-GPU pass, at s / N on its
rank, so that rank's pass is c + max(b / N, s / N + L).
Efficiency = single-GPU job time x N / (N-rank job time x N) for weak (same work per GPU), and
single-GPU job time / (N x N-rank job time) for strong.
    python tools/scaling_model.py [bench json ...]
"""
import glob
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C_FIXED = 0.025  # s: warm-up admission batches (~20 ms) + launches + readback


def passes(paths):
    out = []
    for f in paths:
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except (OSError, ValueError):
            continue
        if "run" in d and "stdout_tail" in d.get("run", {}):
            d = json.loads(d["run"]["stdout_tail"].strip().splitlines()[-1])
        p = d.get("detail", {}).get("pass_s", {}).get("all")
        if p and d.get("config", {}).get("grid", "192x192") == "192x192" and d.get("n_gpus", 1) == 1:
            out += p
    return np.array(out)


def main():
    paths = sys.argv[1:] or (sorted(glob.glob(os.path.join(REPO, "profiles", "r02[p-z]*bench*.json"))) +
                             sorted(glob.glob(os.path.join(REPO, "profiles", "r03*bench*.json"))) +
                             sorted(glob.glob(os.path.join(REPO, "profiles", "r03_ab", "*.json"))) +
                             [os.path.join(REPO, "BENCH_r02.json")])
    t = passes(paths)
    med = float(np.median(t))
    b = med - C_FIXED
    e = np.maximum(t - med, 0.0)
    rng = np.random.default_rng(1)
    K, trials = 20, 4000
    print(f"{len(t)} measured passes: median {med:.3f} s, mean {t.mean():.3f} s; passes with a long-photon excess "
          f"> 50 ms: {np.mean(e > 0.05):.2f}; fixed c = {C_FIXED} s, photon part b = {b:.3f} s")
    single = np.array([rng.choice(t, K).sum() for _ in range(trials)])
    print(f"{'N':>3} {'weak eff':>9} {'strong eff':>11} {'strong speedup':>15}")
    for n in (1, 2, 4, 8):
        weak = np.array([rng.choice(t, (n, K)).sum(axis=1).max() for _ in range(trials)])
        strong = np.empty(trials)
        for i in range(trials):
            tot = np.full(n, 0.0)
            for k in range(K):
                ek = e[rng.integers(len(e))]
                tr = np.full(n, C_FIXED + b / n)
                if ek > 0.0:
                    s = rng.uniform(0.0, b)
                    L = ek + b - s
                    r = rng.integers(n)
                    tr[r] = C_FIXED + max(b / n, s / n + L)
                tot += tr
            strong[i] = tot.max()
        print(f"{n:>3} {single.mean() / weak.mean():>9.2f} {single.mean() / (n * strong.mean()):>11.2f} "
              f"{single.mean() / strong.mean():>15.2f}")


if __name__ == "__main__":
    main()
