"""The device table builders' log / log10 (cuda-grmonty_amd/csrc/grm_crlog.h), compiled on the host
(tests/native/crlog_check.cpp) with glibc's log as the starting point: cr_log agrees with glibc's log
except where glibc misrounds (each such argument is checked here against a 60-digit log: cr_log is the
correctly rounded one, glibc's is off by just over half an ulp), and grm_log10 -- fdlibm's e_log10
construction, which is glibc's -- agrees with glibc's log10 wherever cr_log agrees with glibc's log, and
on zero, subnormal, negative, infinite and NaN arguments returns what glibc's log10 does."""
import math
import os
import shutil
import subprocess
from decimal import Decimal, getcontext

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "cuda-grmonty_amd", "csrc")


def test_crlog_vs_glibc(tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "crlog")
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", f"-I{CSRC}",
                    os.path.join(HERE, "native", "crlog_check.cpp"), "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.splitlines()
    n, d_log, d_l10, d_special = (int(v) for v in out[-1].split()[1::2])
    print(f"{n} arguments: cr_log != glibc log {d_log}, grm_log10 != glibc log10 {d_l10}; "
          f"special arguments (0, subnormal, negative, inf, NaN) differing {d_special}")
    assert n == 400000 and d_log < n * 5e-4 and d_l10 <= d_log + n * 1e-4
    assert d_special == 0, [l for l in out if l.startswith("special")]
    getcontext().prec = 60
    for line in out[:-1]:
        if not line.startswith("log "):
            continue
        _, x, a, b = line.split()
        x, a, b = float.fromhex(x), float.fromhex(a), float.fromhex(b)
        t = Decimal(x).ln()
        err_cr = abs((Decimal(a) - t) / Decimal(math.ulp(a)))
        err_gl = abs((Decimal(b) - t) / Decimal(math.ulp(b)))
        assert err_cr <= Decimal("0.5") < err_gl < Decimal("0.52"), (x, err_cr, err_gl)
