"""Content hash of the transport kernels' sources (cuda-grmonty_amd/csrc/*.hip, *.h and include/*.h).

A PMC traffic file (profiles/pmc_traffic.json, tools/traffic_summary.py) records the hash of the
sources it was measured on; bench.py reports that traffic as this run's measured HBM rate only when
the hash of the sources it runs is the same (the kernels are then the measured ones), and marks it
borrowed otherwise.  Hashing file contents rather than a git revision works on the GPU box, which
gets the tree without .git."""
import hashlib
import os

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)


def kernel_source_hash() -> str:
    h = hashlib.sha256()
    files = []
    for d, exts in ((os.path.join(PKG_DIR, "csrc"), (".hip", ".h")), (os.path.join(REPO_DIR, "include"), (".h",))):
        if os.path.isdir(d):
            files += sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts))
    for f in files:
        h.update(os.path.relpath(f, REPO_DIR).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
