"""One-line summary of a bench.py JSON output (development helper)."""
import json
import sys

for path in sys.argv[1:]:
    with open(path) as f:
        lines = [ln for ln in f if ln.startswith("{")]
    d = json.loads(lines[-1])
    det = d["detail"]
    print(f"{path}: value {d['value']:.4g} {d['unit']} jobs {det.get('passes_in_flight')} "
          f"pass latency {det.get('pass_latency_s')} longest life {det.get('longest_photon_life_steps')} "
          f"tracked/pass {det['tracked_per_step']} launches {det['launches_total']} "
          f"roofline {d['roofline']['achieved']:.0f} GB/s")
