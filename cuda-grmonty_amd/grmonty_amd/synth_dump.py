"""Deterministic synthetic HARM dump generator (exact text format of the reference loader).

dump019 (the reference README's benchmark input, README.md:63, a remote URL) is not available
offline, so every test and benchmark runs on dumps written by this generator.  The format is the
one HARMModel::read_file parses (reference harm_model.cpp:81-232):

  header: 26 tokens  t N1 N2 x1_start x2_start dx1 dx2 t_final n_step a gamma courant
                     dt_dump dt_log dt_img dt_rdump cnt_dump cnt_img cnt_rdump dt lim failed
                     r_in r_out h_slope r_0
  zones:  N1*N2 lines (x2 fastest) of 34 tokens
                     x1 x2 r h rho u U1 U2 U3 B1 B2 B3 divb ucon[4] ucov[4] bcon[4] bcov[4]
                     vmin1 vmax1 vmin2 vmax2 gdet

Physics of the synthetic flow (a hot, magnetised torus around a spinning hole in modified
Kerr-Schild coordinates; parameters typical of HARM, NOT calibrated to dump019):
  rho   torus Gaussian in r around r_c plus a tenuous r^-1.5 atmosphere
  u     u/rho = uor0 (1 + uor_r/r) -> Theta_e ~ 2.2 (1 + 2/r) (theta_e_unit ~ 224, gamma = 13/9);
        a mild profile keeps Theta_e^2 / <Theta_e^2> (the scattering bias, harm_model.cpp:1394) O(1)
  U^i   Keplerian-ish rotation U3 ~ 1/(r^1.5 + a), slow radial inflow U1
  B^i   poloidal + toroidal field at plasma beta ~ 10
A seeded, smooth multiplicative perturbation breaks the axisymmetry of the bins.
"""
from __future__ import annotations

import math
import os

import numpy as np


def mks_theta(x2: np.ndarray, h_slope: float) -> np.ndarray:
    return np.pi * x2 + 0.5 * (1.0 - h_slope) * np.sin(2.0 * np.pi * x2)


def make_fields(n1: int, n2: int, a: float = 0.9375, gamma: float = 13.0 / 9.0, h_slope: float = 0.3,
                r_in: float = 1.3, r_out: float = 40.0, seed: int = 19, rho_max: float = 1.0,
                uor0: float = 0.01, uor_r: float = 2.0):
    """Return (header dict, dict of 2-D field arrays, x1, x2, r, th, gdet)."""
    x1s = math.log(r_in)
    dx1 = (math.log(r_out) - math.log(r_in)) / n1
    x2s = 0.0
    dx2 = 1.0 / n2
    i = np.arange(n1)[:, None]
    j = np.arange(n2)[None, :]
    x1 = x1s + (i + 0.5) * dx1 + 0.0 * j
    x2 = x2s + (j + 0.5) * dx2 + 0.0 * i
    r = np.exp(x1)
    th = mks_theta(x2, h_slope)
    cth, sth = np.cos(th), np.sin(th)
    rng = np.random.default_rng(seed)
    ph = rng.uniform(0, 2 * np.pi, size=4)
    pert = (1.0 + 0.15 * np.sin(3.0 * x1 * 2 * np.pi / (x1.max() - x1s + 1e-12) + ph[0])
            * np.sin(4.0 * np.pi * x2 + ph[1])
            + 0.08 * np.cos(7.0 * x1 + ph[2]) * np.cos(10.0 * np.pi * x2 + ph[3]))
    r_c, sig_r, sig_th = 8.0, 3.0, 0.35
    rho = rho_max * np.exp(-0.5 * ((r - r_c) / sig_r) ** 2) * np.exp(-0.5 * (cth / sig_th) ** 2)
    rho = rho * pert + 1.0e-3 * rho_max * (r / 2.0) ** -1.5
    u = rho * uor0 * (1.0 + uor_r / r)
    u1 = -0.05 / r
    u2 = 0.0 * r
    u3 = 1.0 / (r ** 1.5 + a)
    beta = 10.0
    pgas = (gamma - 1.0) * u
    bt = np.sqrt(2.0 * pgas / beta)
    b1 = bt * cth / r
    b2 = 0.5 * bt * sth / (np.pi * r)
    b3 = 0.3 * bt / r
    dthdx2 = np.pi * (1.0 + (1.0 - h_slope) * np.cos(2.0 * np.pi * x2))
    gdet = (r * r + a * a * cth * cth) * np.abs(sth) * r * dthdx2
    hdr = dict(t=0.0, n1=n1, n2=n2, x1s=x1s, x2s=x2s, dx1=dx1, dx2=dx2, t_final=2000.0, n_step=0, a=a,
               gamma=gamma, courant=0.8, dt_dump=50.0, dt_log=10.0, dt_img=1.0, dt_rdump=100, cnt_dump=19,
               cnt_img=0, cnt_rdump=0, dt=0.01, lim=0, failed=0, r_in=r_in, r_out=r_out, h_slope=h_slope,
               r_0=0.0)
    fields = dict(rho=rho, u=u, u1=u1 + 0 * r, u2=u2, u3=u3, b1=b1, b2=b2, b3=b3)
    return hdr, fields, x1, x2, r, th, gdet


def write_dump(path: str, n1: int = 64, n2: int = 64, **kw) -> str:
    """Write a synthetic HARM dump; returns path.  Deterministic for given arguments."""
    hdr, f, x1, x2, r, th, gdet = make_fields(n1, n2, **kw)
    head = ("{t:.17g} {n1:d} {n2:d} {x1s:.17g} {x2s:.17g} {dx1:.17g} {dx2:.17g} {t_final:.17g} {n_step:d} "
            "{a:.17g} {gamma:.17g} {courant:.17g} {dt_dump:.17g} {dt_log:.17g} {dt_img:.17g} {dt_rdump:d} "
            "{cnt_dump:d} {cnt_img:d} {cnt_rdump:d} {dt:.17g} {lim:d} {failed:d} {r_in:.17g} {r_out:.17g} "
            "{h_slope:.17g} {r_0:.17g}").format(**hdr)
    nz = n1 * n2
    cols = np.zeros((nz, 34))
    cols[:, 0] = x1.ravel()
    cols[:, 1] = x2.ravel()
    cols[:, 2] = r.ravel()
    cols[:, 3] = th.ravel()
    for c, name in enumerate(["rho", "u", "u1", "u2", "u3", "b1", "b2", "b3"]):
        cols[:, 4 + c] = np.broadcast_to(f[name], x1.shape).ravel()
    cols[:, 13] = 1.0  # ucon0 (only logged by the reference loader)
    cols[:, 33] = gdet.ravel()
    tmp = path + ".tmp"
    with open(tmp, "w") as fh:
        fh.write(head + "\n")
        np.savetxt(fh, cols, fmt="%.17g", delimiter=" ")
    os.replace(tmp, path)
    return path


def ensure_dump(path: str, n1: int, n2: int, **kw) -> str:
    """Write the dump only if it does not exist yet (cache for tests/bench)."""
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        write_dump(path, n1, n2, **kw)
    return path


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("path")
    ap.add_argument("--n1", type=int, default=192)
    ap.add_argument("--n2", type=int, default=192)
    ap.add_argument("--seed", type=int, default=19)
    args = ap.parse_args()
    write_dump(args.path, args.n1, args.n2, seed=args.seed)
