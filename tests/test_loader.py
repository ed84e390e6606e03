"""HARM dump loader (harm_model.cpp:81-232): the reference's own parser fixture
(tests/harm_model_test.cpp: a 2x3 dump with sentinel values) and agreement of the product
loader (C++ host) with the oracle loader on a synthetic dump."""
import os

import numpy as np
import pytest

import grmonty_amd as G
import oracle_py as O

# tests/harm_model_test.cpp:16-93 -- fixture data (values only)
HDR = dict(t=1.0, n=(2, 3), x_start=(0.0, 4.0, 5.0, 0.0), dx=(0.0, 8.0, 9.0, 0.0), t_final=10.0, n_step=11, a=12.0,
           gamma=13.0, courant=14.0, dt_dump=15.0, dt_log=16.0, dt_img=17.0, dt_rdump=18, cnt_dump=19, cnt_img=20,
           cnt_rdump=21, dt=22.0, lim=23, failed=24, r_in=25.0, r_out=26.0, h_slope=27.0, r_0=28.0)
FIELDS = {name: np.array([[b + 11, b + 12, b + 13], [b + 21, b + 22, b + 23]], dtype=float)
          for name, b in zip(["rho", "u", "u1", "u2", "u3", "b1", "b2", "b3"], range(100, 900, 100))}


def fmt(v):
    return repr(float(v)).rstrip("0").rstrip(".") if isinstance(v, float) else str(v)


def write_fixture(path):
    h = HDR
    head = " ".join(fmt(v) for v in [h["t"], h["n"][0], h["n"][1], h["x_start"][1], h["x_start"][2], h["dx"][1],
                                     h["dx"][2], h["t_final"], h["n_step"], h["a"], h["gamma"], h["courant"],
                                     h["dt_dump"], h["dt_log"], h["dt_img"], h["dt_rdump"], h["cnt_dump"],
                                     h["cnt_img"], h["cnt_rdump"], h["dt"], h["lim"], h["failed"], h["r_in"],
                                     h["r_out"], h["h_slope"], h["r_0"]])
    with open(path, "w") as f:
        f.write(head + "\n")
        for i in range(2):
            for j in range(3):
                vals = ["0 0 0 0"] + [fmt(FIELDS[n][i, j]) for n in FIELDS] + ["0", "0 0 0 0 0 0 0 0",
                                                                               "0 0 0 0 0 0 0 0", "0 0 0 0", "0"]
                f.write(" ".join(vals) + "\n")


@pytest.mark.parametrize("which", ["product", "oracle"])
def test_reference_parser_fixture(tmp_path, which):
    p = str(tmp_path / "harm_dump")
    write_fixture(p)
    if which == "product":
        m = G.Model.load(p, photon_n=10)
        h = m.header
        fields = [m.field(i) for i in range(8)]
    else:
        m = O.OracleModel(p, photon_n=10)
        h = m.header
        fields = [m.field(i) for i in range(8)]
    assert h.t == 1.0 and tuple(h.n) == (2, 3)
    assert list(h.x_start) == [0.0, 4.0, 5.0, 0.0]
    assert list(h.x_stop) == [1.0, 20.0, 32.0, 2 * np.pi]  # harm_model.cpp:114-117
    assert list(h.dx) == [1.0, 8.0, 9.0, 2 * np.pi]
    for k in ("t_final", "n_step", "a", "gamma", "courant", "dt_dump", "dt_log", "dt_img", "dt_rdump", "cnt_dump",
              "cnt_img", "cnt_rdump", "dt", "lim", "failed", "r_in", "r_out", "h_slope", "r_0"):
        assert getattr(h, k) == HDR[k], k
    for arr, name in zip(fields, FIELDS):
        np.testing.assert_array_equal(arr, FIELDS[name])


def test_missing_and_truncated_files(tmp_path):
    with pytest.raises(IOError):
        G.Model.load(str(tmp_path / "nope"))
    p = tmp_path / "trunc"
    p.write_text("0 4 4 0.1 0 0.1 0.25 1 0 0.5 1.4 0.8 1 1 1 1 0 0 0 0.1 0 0 1 10 0.3 0\n1 2 3\n")
    with pytest.raises(IOError):
        G.Model.load(str(p))


def test_product_loader_matches_oracle(dump64):
    m = G.Model.load(dump64, photon_n=2000)
    o = O.OracleModel(dump64, photon_n=2000)
    hm, ho = m.header, o.header
    for k, _ in hm._fields_:
        a, b = getattr(hm, k), getattr(ho, k)
        assert (list(a) if hasattr(a, "__len__") else a) == (list(b) if hasattr(b, "__len__") else b), k
    for i in range(8):
        np.testing.assert_array_equal(m.field(i), o.field(i))
    um, uo = m.units, o.units
    for k, _ in um._fields_:
        assert getattr(um, k) == getattr(uo, k), k
    sm, so = m.scalars(), o.scalars()
    for k in ("bias_norm", "x1_min", "max_tau_scatt", "d_tau_k", "rh"):
        assert sm[k] == so[k], k
