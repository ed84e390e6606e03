"""bench.py's host-side measurement helpers (no GPU): the PMC traffic of the dominant launch from the
rocprofv3 counter CSVs (FETCH_SIZE doubled on gfx950, plus WRITE_SIZE, KB -> B, the small
dispatches of the control kernels' passes excluded) and the committed traffic file with its
provenance, which the bench line reports as roofline.traffic / traffic_source."""
import csv
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _csv(path, counter, values):
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, v in enumerate(values):
            w.writerow({"Dispatch_Id": i, "Kernel_Name": "(anonymous namespace)::track_kernel(grm::Params, Ctl)",
                        "Counter_Name": counter, "Counter_Value": v})
        w.writerow({"Dispatch_Id": 99, "Kernel_Name": "ctl_kernel", "Counter_Name": counter, "Counter_Value": 1e9})


def test_pmc_traffic_from_counter_csvs(tmp_path):
    bench = pytest.importorskip("bench")
    f, w = tmp_path / "fetch.csv", tmp_path / "write.csv"
    # two dominant launches and two small relaunches per pass
    _csv(f, "FETCH_SIZE", [2.0e6, 1.0e4, 3.0e6, 1.2e4])
    _csv(w, "WRITE_SIZE", [8.0e6, 4.0e2, 6.0e6, 3.0e2])
    got = bench.pmc_traffic(f"{f},{w}")
    assert got == pytest.approx((2.0 * 2.5e6 + 7.0e6) * 1024.0)
    assert bench.pmc_traffic(f"{f},{tmp_path / 'missing.csv'}") is None


def test_committed_traffic_has_provenance():
    """the committed file's bytes and provenance; it counts as measured on the running kernels only
    when its kernel-source hash equals the hash of the sources in this tree"""
    bench = pytest.importorskip("bench")
    from grmonty_amd.srchash import kernel_source_hash
    traffic, src, same = bench.committed_traffic()
    d = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))
    assert traffic == d["bytes_per_dominant_launch"] and traffic > 0
    assert src and "tree" in src
    assert same == (d.get("kernel_src_hash") == kernel_source_hash())


def test_borrowed_traffic_gives_no_hbm_rate(tmp_path, monkeypatch):
    """a traffic file measured on other kernel sources is reported as borrowed: committed_traffic
    says so, and bench.py then forms no measured HBM rate from it"""
    bench = pytest.importorskip("bench")
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps({"bytes_per_dominant_launch": 1.0e10, "source": "x (tree y)",
                             "kernel_src_hash": "0000000000000000"}))
    monkeypatch.setattr(bench, "PMC_TRAFFIC", str(p))
    traffic, src, same = bench.committed_traffic()
    assert traffic == 1.0e10 and not same
