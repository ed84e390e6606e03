"""Summarise tools/sessions/ab_libs.sh output: per variant, the single-pass transport rate (G steps/s) of
every rep after the first (rep 0 carries the live-bias warm-up)."""
import re
import sys
from collections import defaultdict

rates = defaultdict(list)
cur = None
for line in open(sys.argv[1]):
    m = re.match(r"== (\S+) rc=", line)
    if m:
        cur = m.group(1)
        continue
    m = re.match(r"rep (\d+):.*\(([\d.e+]+) Msteps/s\)", line)
    if m and cur and int(m.group(1)) > 0:
        rates[cur].append(float(m.group(2)) / 1e3)
for v, r in rates.items():
    print(f"{v:8s} n={len(r)} mean {sum(r) / len(r):.3f} G steps/s  [{', '.join(f'{x:.2f}' for x in r)}]")
