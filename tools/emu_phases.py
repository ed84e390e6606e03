"""Per-rank launch timelines of an emulated N-rank job (tests/multirank_emu.py --phases): when each
rank's main launch started (s_memrealtime, one clock for the whole GPU), when its warm-up admission
ended, its admission batches (time, photons in flight), when its pool drained and its last wave left,
and its recorded / scattered per created photon -- to see whether the N-rank live-bias offset
 sits in some ranks or in some phase.

    python tools/emu_phases.py OUT.jsonl WORLD SEEDS [K=V ...]
"""
import json
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "cuda-grmonty_amd")]
from grmonty_amd.synth_dump import ensure_dump  # noqa: E402


def main():
    out, world, seeds = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    opts = sys.argv[4:]
    dump = ensure_dump(os.path.join(R, "gpurun_out", "synth192.dump"), 192, 192)
    tmp = os.path.join(R, "gpurun_out", f"emu_phases_w{world}.json")
    cmd = [sys.executable, "-u", os.path.join(R, "tests", "multirank_emu.py"), dump, str(world), str(seeds), tmp,
           "--phases"] + (["--shared"] if world > 1 else [])
    for kv in opts:
        cmd += ["--opt", kv]
    env = dict(os.environ, GPU_MAX_HW_QUEUES=str(min(32, 2 * world + 2)))
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=900)
    if r.returncode:
        print(r.stderr[-3000:])
        sys.exit(1)
    jobs = json.load(open(tmp))
    with open(out, "a") as f:
        for s, j in enumerate(jobs):
            ph = j["per_rank_phases"]
            t00 = min(p["t0_ticks"] for p in ph)
            print(f"world {world} seed {s}: job recorded {j['recorded']} / created {j['created']} = "
                  f"{j['recorded'] / j['created']:.4f}", flush=True)
            for r_, p in enumerate(ph):
                off = (p["t0_ticks"] - t00) * 1e-5
                adm = p["admissions"]
                rr = j["per_rank_recorded"][r_] / j["per_rank_created"][r_]
                print(f"  rank {r_}: start +{off:7.2f} ms  warm-up end {p['warmup_end_ms']}  batches {len(adm)} "
                      f"(last {adm[-1] if adm else None})  drained {p['pool_drained_ms']}  exit {p['last_exit_ms']}  "
                      f"rec/created {rr:.4f}", flush=True)
                if s == 0:
                    print("     admissions (ms, in flight):", [(round(t, 2) if t else t, fl) for t, fl in adm], flush=True)
            f.write(json.dumps({k: v for k, v in j.items() if k != "job_view"}) + "\n")


if __name__ == "__main__":
    main()
