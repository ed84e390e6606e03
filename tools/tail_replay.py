"""Frozen-bias replay of bench passes (192^2, photon_n = 1e6, device emission, one GPU), for comparing
the tail of a pass between builds.  A pass's tail (the long photons of DESIGN §8.4) depends on the
live bias, so a live pass draws a different tail every run; with the bias frozen at one snapshot of
the counters every photon's life is fixed by its Philox stream, and the same pass replays with the
same photons on any build that is photon-by-photon exact.  Snapshots come from one live pass per seed
and are kept in --snap (JSON): a second build run with the same file replays the same passes.

    python tools/tail_replay.py --seeds 124 125 126 --snap gpurun_out/tail_snap.json [--reps 1]
    GRMONTY_AMD_LIB=cuda-grmonty_amd/ab/libgrmonty_amd_vr04.so python tools/tail_replay.py ...   (an older build)

Per pass: wall time of emission + transport, the dominant launch, the early worker and lone kernels,
the photons they took and the longest life."""
import argparse
import json
import os
import struct
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-grmonty_amd"))
import grmonty_amd as G  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[124, 125, 126])
    ap.add_argument("--snap", default=os.path.join(REPO, "gpurun_out", "tail_snap.json"))
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--photon-n", type=float, default=1e6)
    ap.add_argument("--opt", action="append", default=[], help="engine option K=V (grmonty_amd.OPT_*)")
    a = ap.parse_args()
    path = ensure_dump(os.path.join(REPO, "gpurun_out", "synth192.dump"), 192, 192)
    m = G.Model.load(path, photon_n=a.photon_n).init(0, device=0)
    e = G.Engine(m, 0)
    e.emit_setup(m)
    for kv in a.opt:
        k, v = kv.split("=")
        e.set_option(int(k), int(v))
    snap = json.load(open(a.snap)) if os.path.exists(a.snap) else {}
    lib = os.environ.get("GRMONTY_AMD_LIB", "in-tree")

    def run(seed):
        e.reset()
        e.set_option(G.OPT_SEED, seed)
        e.set_option(G.OPT_ID_BASE, 0)
        t = time.time()
        p, cnt = e.emit(seed=seed)
        e.track_device(p, cnt)
        st = e.stats()
        c = e.debug_counters()
        e.finish()
        return time.time() - t, cnt, st, c

    for seed in a.seeds:
        key = str(seed)
        if key not in snap:
            e.set_option(G.OPT_BIAS_MODE, 0)
            _, _, _, c = run(seed)
            snap[key] = {"scatt": c["n_scatt"], "rec": c["n_recorded"], "maxtau": c["max_tau_scatt"]}
            json.dump(snap, open(a.snap, "w"), indent=1)
        s = snap[key]
        e.set_option(G.OPT_BIAS_MODE, 1)
        e.set_option(G.OPT_FROZEN_SCATT, s["scatt"])
        e.set_option(G.OPT_FROZEN_REC, s["rec"])
        e.set_option(G.OPT_FROZEN_MAXTAU, struct.unpack("<q", struct.pack("<d", s["maxtau"]))[0])
        for r in range(a.reps):
            wall, cnt, st, c = run(seed)
            print(json.dumps({"lib": lib, "opts": a.opt, "seed": seed, "rep": r, "snapshot": s, "pass_s": round(wall, 4),
                              "photons": cnt, "bulk_ms": round(st["max_launch_ms"], 1),
                              "early_ms": round(st["early_ms"], 1), "n_early": st["n_early"],
                              "lone_ms": round(st["lone_ms"], 1), "n_lone": st["n_lone"],
                              "kernels_ms": round(st["last_kernel_ms"], 1), "longest_life": st["max_photon_steps"],
                              "lives_gt_1e5": st["n_long_photons"], "recorded": c["n_recorded"],
                              "steps": c["n_steps"]}), flush=True)
        e.set_option(G.OPT_BIAS_MODE, 0)


if __name__ == "__main__":
    main()
