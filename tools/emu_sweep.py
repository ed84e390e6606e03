"""Multi-rank emulation variants (tests/multirank_emu.py) against the 1e5 oracle fixture: which
part of the N-rank job moves the live-bias counters.

    python tools/emu_sweep.py OUT.jsonl "name:world:seeds[:shared][:K=V,...]" ...
"""
import json
import os
import subprocess
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "cuda-grmonty_amd")]
from spectrum_stats import welch_z  # noqa: E402
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402

KEYS = ("recorded", "scattered", "steps", "luminosity")


def main():
    out = sys.argv[1]
    dump = ensure_dump(os.path.join(R, "gpurun_out", "synth192.dump"), 192, 192)
    summ = json.load(open(os.path.join(R, "tests", "golden", "oracle_synth192_pn1e5.json")))
    o = {k: np.array([x[k] for x in summ["runs"]], dtype=np.float64) for k in KEYS}
    for spec in sys.argv[2:]:
        f = spec.split(":")
        name, world, seeds = f[0], int(f[1]), int(f[2])
        shared = "shared" in f[3:]
        seq = "seq" in f[3:]
        opts = [kv for x in f[3:] if x not in ("shared", "seq") for kv in x.split(",") if kv]
        tmp = os.path.join(R, "gpurun_out", f"emu_{name}.json")
        cmd = [sys.executable, "-u", os.path.join(R, "tests", "multirank_emu.py"), dump, str(world), str(seeds), tmp]
        cmd += ["--shared"] if shared else []
        cmd += ["--sequential"] if seq else []
        for kv in opts:
            cmd += ["--opt", kv]
        env = dict(os.environ, GPU_MAX_HW_QUEUES=str(min(32, 2 * world + 2)))
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        if r.returncode:
            print(name, "failed", r.stderr[-2000:], flush=True)
            sys.exit(1)
        jobs = json.load(open(tmp))
        row = {"name": name, "world": world, "seeds": seeds, "shared": shared, "opts": opts}
        for k in KEYS:
            # with the counters in rank 0's block (variant library "sb") the per-rank counter reads
            # are incomplete: recorded / scattered from the spectra's own sums
            src = {"recorded": "rec_spec", "scattered": "scatt_spec"}.get(k, k) if "sb" in name else k
            dev = [j[src] for j in jobs]
            diff, se, z = welch_z(dev, o[k])
            row[k] = {"mean": float(np.mean(dev)), "diff": float(diff / o[k].mean()), "z": float(z)}
        print(f"{name:14s} world {world} {'shared' if shared else 'own'} {opts}: " +
              "  ".join(f"{k} {row[k]['diff']:+.2%} ({row[k]['z']:+.1f} SE)" for k in KEYS), flush=True)
        with open(out, "a") as fh:
            fh.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
