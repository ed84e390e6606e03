"""Photon-by-photon parity helpers shared by the GPU parity tests (device vs oracle, same emitted
photons, same Philox streams, bias frozen at the same snapshot).

A photon matches when its end reason, theta/energy bin, scattering count and step count agree (the
step count exactly: round 5 measured no photon off by one step on any path, r05m) and
its weight and energy agree to rounding (device FMA / OCML vs glibc).  A photon whose rejection or
sub-stepping decision flips on a last-bit difference diverges, and so do its children; such
photons are counted (MIN_MATCH bounds them) and the spectrum cells they reach on either side are
excluded from the per-cell comparison of all twelve accumulated fields (record_super_photon,
harm_model.cpp:1291-1335), which must agree to SPEC_RTOL everywhere else.
"""
import numpy as np

MIN_MATCH = 0.998      # observed: 1.0000 in every driver run (r01-r04); a flip is a last-bit event
# weight / energy of matching photons: the largest relative differences observed over the four
# transport variants and 512^2 are printed by every test (match_residuals); round 5 (r05a): w 2.04e-11
# (lone kernel), e 8.9e-10 (512^2: a child's energy from the tetrad and the electron sample).  Bars:
# 10x the weight's, ~5x the energy's
W_RTOL, E_RTOL = 2e-10, 5e-9
SPEC_RTOL = 1e-6       # per-cell sums of matching photons: the weight tolerance
SPEC_ATOL = 1e-12      # x the field's total: underflow-level terms (e.g. an absorption optical depth of
                       # 1e-263 that one side's exp rounds to 0) are not a disagreement
SPEC_FIELDS = ["dn_dle", "de_dle", "nph", "nscatt", "x1i_av", "x2i_sq", "x3f_sq", "tau_abs", "tau_scatt",
               "ne_0", "theta_e_0", "b_0"]


def trace_match(tr_o, tr_g):
    """(n_oracle_ends, n_device_ends, n_matching, ids of non-matching photons on either side)"""
    go = {int(r["id"]): r for r in tr_o}
    gg = {int(r["id"]): r for r in tr_g}
    match, bad = 0, set()
    for i in set(go) | set(gg):
        a, b = go.get(i), gg.get(i)
        if (a is not None and b is not None and a["end_reason"] == b["end_reason"] and a["ix2"] == b["ix2"]
                and a["i_e"] == b["i_e"] and a["n_scatt"] == b["n_scatt"] and int(a["n_step"]) == int(b["n_step"])
                and np.isclose(a["w"], b["w"], rtol=W_RTOL, atol=0) and np.isclose(a["e"], b["e"], rtol=E_RTOL)):
            match += 1
        else:
            bad.add(i)
    return len(go), len(gg), match, bad


def match_residuals(tr_o, tr_g, steps=None):
    """largest relative |w| and |e| differences over the photons whose discrete outcome (end reason,
    bins, n_scatt, n_step within 1) agrees on both sides -- what W_RTOL / E_RTOL must cover; with
    `steps` (a dict) also the count of those photons whose n_step differs (the +-1 allowance)"""
    go = {int(r["id"]): r for r in tr_o}
    mw = me = 0.0
    n_step_off = 0
    for r in tr_g:
        a = go.get(int(r["id"]))
        if (a is None or a["end_reason"] != r["end_reason"] or a["ix2"] != r["ix2"] or a["i_e"] != r["i_e"]
                or a["n_scatt"] != r["n_scatt"] or abs(int(a["n_step"]) - int(r["n_step"])) > 1):
            continue
        n_step_off += int(a["n_step"]) != int(r["n_step"])
        rel = []
        for key in ("w", "e"):
            x, y = float(a[key]), float(r[key])
            rel.append(abs(x - y) / max(abs(x), abs(y)) if max(abs(x), abs(y)) > 0 else 0.0)
        mw, me = max(mw, rel[0]), max(me, rel[1])
    if steps is not None:
        steps["n_step_off_by_one"] = n_step_off
    return mw, me


def check_spectrum_cells(spec_o, spec_g, tr_o, tr_g, bad):
    """all 12 fields, every (theta, energy) cell not reached by a non-matching photon; returns the
    number of cells compared and of cells excluded"""
    excl = set()
    for tr in (tr_o, tr_g):
        for r in tr:
            if int(r["id"]) in bad and r["end_reason"] == 0:
                excl.add((int(r["ix2"]), int(r["i_e"])))
    so = np.asarray(spec_o).reshape(6, 200)
    sg = np.asarray(spec_g).reshape(6, 200)
    n_cmp = 0
    floor = {f: SPEC_ATOL * max(np.abs(so[f]).sum(), np.abs(sg[f]).sum()) for f in SPEC_FIELDS}
    for j in range(6):
        for i in range(200):
            if (j, i) in excl:
                continue
            n_cmp += 1
            for f in SPEC_FIELDS:
                a, b = float(so[f][j, i]), float(sg[f][j, i])
                assert abs(a - b) <= SPEC_RTOL * max(abs(a), abs(b)) + floor[f], (f, j, i, a, b)
    return n_cmp, len(excl)
