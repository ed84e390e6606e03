"""Sum rocprofv3 --pmc CSVs (gpurun_out/pmc_<tag>_<i>/run_counter_collection.csv) over track_kernel (or split_kernel)
dispatches and print the derived ratios used in DESIGN.md §8."""
import collections
import csv
import glob
import os
import re
import sys

root, tag = sys.argv[1], sys.argv[2]
tot = collections.defaultdict(float)
for f in sorted(glob.glob(os.path.join(root, f"pmc_{tag}_*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "track_kernel" in r["Kernel_Name"] or "split_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
steps = None
for f in sorted(glob.glob(os.path.join(root, f"pmc_{tag}_*.log"))):
    m = re.search(r"steps (\d+)", open(f).read())
    if m:
        steps = int(m.group(1))
for k in sorted(tot):
    print(f"{k:32s} {tot[k]:.6g}")
g = tot.get
if g("SQ_THREAD_CYCLES_VALU") and g("SQ_ACTIVE_INST_VALU"):
    print(f"VALU lane utilisation       {g('SQ_THREAD_CYCLES_VALU') / (64 * g('SQ_ACTIVE_INST_VALU')):.3f}")
if g("SQ_ACTIVE_INST_VALU") and g("SQ_WAVE_CYCLES"):
    print(f"VALU-active / wave cycles   {g('SQ_ACTIVE_INST_VALU') / g('SQ_WAVE_CYCLES'):.3f}")
if g("SQ_WAIT_ANY") and g("SQ_WAVE_CYCLES"):
    print(f"wait-any / wave cycles      {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}  (from a different run)")
if g("TCC_HIT_sum") is not None and g("TCC_REQ_sum"):
    print(f"L2 hit rate                 {g('TCC_HIT_sum') / max(1.0, g('TCC_HIT_sum') + g('TCC_MISS_sum')):.3f}")
if steps:
    print(f"transport steps (pass)      {steps}")
    for k in sorted(k for k in tot if k.startswith("SQ_INSTS")):
        if g(k):
            print(f"{k + ' / step (wave instr)':44s} {g(k) / steps:.2f}")
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        hbm = (2.0 * g("FETCH_SIZE") + g("WRITE_SIZE")) * 1024.0
        print(f"HBM bytes / step (FETCH x2 + WRITE)   {hbm / steps:.2f}")
