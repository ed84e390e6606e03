"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py for profiles/: per-kernel stats,
and for track_kernel the dominant dispatch of each pass (the longest ones, one per pass) against
the bench line's own per-launch figure (HIP events), which must agree."""
import csv
import json
import os
import sys

d, bench_json = sys.argv[1], sys.argv[2]
stats = os.path.join(d, "run_kernel_stats.csv")
trace = os.path.join(d, "run_kernel_trace.csv")
print("== rocprofv3 --stats (run_kernel_stats.csv)")
for r in csv.DictReader(open(stats)):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} total {float(r['TotalDurationNs']) / 1e6:10.1f} ms "
          f"avg {float(r['AverageNs']) / 1e6:9.3f} ms max {float(r['MaxNs']) / 1e6:9.1f} ms")
print("   (early_kernel runs on a second stream beside each pass's main track_kernel launch and mostly sleeps\n"
      "    until a photon of >= 1500 steps (GRM_OPT_EARLY_STEPS) is handed to it: its time overlaps the bulk, it is not added to it)")
dur = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
             for r in csv.DictReader(open(trace)) if "track_kernel" in r["Kernel_Name"])
b = json.loads(open(bench_json).read())
k = b["steps"] + max(b["warmup"], b["detail"].get("passes_in_flight", 1))
top = dur[-k:]
print(f"== track_kernel dispatches: {len(dur)}; the {k} longest (one dominant launch per pass): "
      f"mean {sum(top) / len(top):.1f} ms, min {top[0]:.1f} ms, max {top[-1]:.1f} ms")
note = b["roofline"]["note"]
rf = b["roofline"]
print(f"== bench line under rocprof: value {b['value']:.4g} {b['unit']}, roofline ({rf['bound']}) achieved "
      f"{rf['achieved']:.2f} {rf['unit']} of {rf['peak']} (frac {rf['frac']:.3f})")
print(f"   {note}")
