"""Exact FP64 operation count per transport step of the oracle restatement.

The oracle (oracle/grmonty_oracle.cpp, reference CPU semantics) is built a second time with every
double-precision arithmetic instruction and libm call followed by a counter increment
(oracle/count/instrument_ir.py on clang -O1 IR; `make -C oracle count/liboracle_count.so`).  This
script tracks a random sample of the superphotons of the bench workload (synthetic 192x192
dump019-class dump, photon_n = 1e6, seed 123, mt19937, live adaptive bias) with that build and
divides the counts by the transport steps taken (sum of n_step over every tracked photon, children
included -- the reference's n_step, harm_model.cpp:1058).  The result is the numerator of bench.py's
FP64 roofline: flops/step = add + sub + mul + div + sqrt (+ 2 per fma, none in this ISO build);
transcendental calls (exp, log, pow, sin, cos, acos, ...) are counted one per call and reported
separately, not folded into the flops.

    python tools/count_fp64.py [--photons 50000] [--grid 192] [--out tests/golden/fp64_ops_per_step.json]
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COUNT_LIB = os.path.join(REPO, "oracle", "count", "liboracle_count.so")
SLOTS = ["fadd", "fsub", "fmul", "fdiv", "sqrt", "fma", "fcmp", "cvt", "exp", "log", "log10", "pow", "sin", "cos",
         "acos", "cbrt", "tgamma", "other_libm", "exp10", "sincos"]
TRANS = ["exp", "log", "log10", "pow", "sin", "cos", "acos", "cbrt", "tgamma", "exp10", "sincos"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--photons", type=int, default=50000)
    ap.add_argument("--grid", type=int, default=192)
    ap.add_argument("--photon-n", type=float, default=1e6)
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden", "fp64_ops_per_step.json"))
    args = ap.parse_args()
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "count/liboracle_count.so"], check=True)
    os.environ["GRMO_ORACLE_LIB"] = COUNT_LIB
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
    import ctypes as C
    import oracle_py as O
    from grmonty_amd.synth_dump import ensure_dump

    path = ensure_dump(os.path.join("/tmp", f"synth{args.grid}.dump"), args.grid, args.grid)
    m = O.OracleModel(path, photon_n=int(args.photon_n))
    m.init(min(8, os.cpu_count() or 1))
    L = O.lib()
    L.grmo_fpcount_get.argtypes = [C.POINTER(C.c_uint64)]
    L.grmo_fpcount_reset.argtypes = []
    # a random sample of the workload's superphotons: every photon of randomly chosen zones
    h = m.header
    rng = np.random.default_rng(7)
    zones = rng.permutation(h.n[0] * h.n[1])
    chunks, n = [], 0
    for z in zones:
        ph = m.emit_philox(seed=123, z0=int(z), z1=int(z) + 1)
        if len(ph):
            chunks.append(ph)
            n += len(ph)
        if n >= args.photons:
            break
    sel = np.concatenate(chunks)
    L.grmo_fpcount_reset()
    t = time.time()
    tr = m.track(sel, rng_mode=0, seed=123, frozen=False, trace_cap=50 * len(sel))
    el = time.time() - t
    cnt = (C.c_uint64 * 32)()
    L.grmo_fpcount_get(cnt)
    c = {s: int(cnt[i]) for i, s in enumerate(SLOTS)}
    steps = int(tr["n_step"].astype(np.int64).sum())
    flops = c["fadd"] + c["fsub"] + c["fmul"] + c["fdiv"] + c["sqrt"] + 2 * c["fma"]
    trans = sum(c[s] for s in TRANS)
    out = {
        "flops_per_step": flops / steps,
        "transcendentals_per_step": trans / steps,
        "per_step": {s: c[s] / steps for s in SLOTS if c[s]},
        "steps": steps, "superphotons": int(len(sel)), "tracked_incl_children": int(len(tr)),
        "steps_per_superphoton": steps / len(sel),
        "workload": f"synthetic {args.grid}x{args.grid} dump019-class dump, photon_n={args.photon_n:g}, all superphotons "
                    f"of {len(chunks)} random zones (seed 123 emission), tracked by the oracle restatement with "
                    f"mt19937 seed 123 and the live adaptive bias",
        "method": "oracle/count/instrument_ir.py: clang -O1 IR of oracle/grmonty_oracle.cpp (no vectorisation, no FP "
                  "contraction) with a counter increment after every double fadd/fsub/fmul/fdiv/fcmp/conversion and "
                  "every libm call; flops = add+sub+mul+div+sqrt (+2 per fma); transcendental calls counted 1 each, "
                  "separately",
        "count_seconds": el,
    }
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "per_step"}, indent=1))
    print("per step:", {k: round(v, 2) for k, v in out["per_step"].items()})


if __name__ == "__main__":
    main()
