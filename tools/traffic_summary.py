"""HBM traffic of the dominant track_kernel launch per pass, from two rocprofv3 --pmc runs of the
same bench command (FETCH_SIZE pass, WRITE_SIZE pass; separate runs, MI355X_MICROARCH.md §HBM:
FETCH_SIZE reports half the bytes of wide streaming reads on gfx950 -> doubled).  Writes
profiles/pmc_traffic.json, which bench.py reports as roofline.traffic.

    python tools/traffic_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <bench.json> <out.json>
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cuda-grmonty_amd"))
from grmonty_amd.srchash import kernel_source_hash  # noqa: E402


def per_dispatch(path, counter):
    v = {}
    for r in csv.DictReader(open(path)):
        if "track_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            d = int(r["Dispatch_Id"])
            v[d] = v.get(d, 0.0) + float(r["Counter_Value"])
    return [v[d] for d in sorted(v)]


fetch = per_dispatch(sys.argv[1], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], "WRITE_SIZE")
bench = json.loads([ln for ln in open(sys.argv[3]).read().splitlines() if ln.startswith('{"metric"')][-1])
k = bench["steps"] + bench["warmup"]
fb = sorted(fetch)[-k:]
wb = sorted(write)[-k:]
f_kb, w_kb = sum(fb) / len(fb), sum(wb) / len(wb)
steps = bench["roofline"]["note"]
out = {"bytes_per_dominant_launch": (2.0 * f_kb + w_kb) * 1024.0,
       "fetch_kb_per_dominant_launch_raw": f_kb, "write_kb_per_dominant_launch": w_kb,
       "dominant_launches": k, "all_fetch_kb": fetch, "all_write_kb": write,
       "command": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) -- python3 bench.py --steps %d "
                  "--warmup %d --cpu-seconds 0 --overlap 0" % (bench["steps"], bench["warmup"]),
       "source": "%s (tree %s)" % (sys.argv[4], os.environ.get("TREE_REV", "?")),
       "kernel_src_hash": kernel_source_hash(),
       "note": "the K+W largest track_kernel dispatches = one dominant launch per pass; bytes = 2 x FETCH_SIZE + "
               "WRITE_SIZE (KB -> B); the bench line of the FETCH run: " + steps}
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps({k_: v for k_, v in out.items() if not k_.startswith("all_")}, indent=1))
