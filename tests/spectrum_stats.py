"""Statistical comparison of two spectra from per-cell sums over recorded superphotons
(count, sum w, sum w^2, sum wE, sum (wE)^2 per (theta, energy) cell; tools/make_golden_192.py).

binned_ks: KS statistic on the normalised cumulative nu L_nu (weights w E) over the 200 energy bins
of one theta bin (or of all of them summed), with the Kish effective sample sizes
(sum wE)^2 / sum (wE)^2.  Binning can only lower D, so the test is conservative in D; the
threshold is c(alpha) sqrt((n1 + n2) / (n1 n2)).
"""
import numpy as np

C_ALPHA = {1e-2: 1.628, 1e-3: 1.949, 1e-4: 2.228}


def cell_sums_from_trace(tr):
    r = tr[tr["end_reason"] == 0]
    c = r["ix2"].astype(np.int64) * 200 + r["i_e"].astype(np.int64)
    w, we = r["w"], r["w"] * r["e"]
    out = np.zeros((1200, 5))
    for k, v in enumerate((np.ones_like(w), w, w * w, we, we * we)):
        out[:, k] = np.bincount(c, weights=v, minlength=1200)
    return out


def binned_ks(c1, c2, theta=None):
    """c1, c2: [1200, 5] cell sums; theta = 0..5 or None (all bins summed over theta)"""
    a = c1.reshape(6, 200, 5)
    b = c2.reshape(6, 200, 5)
    if theta is None:
        a, b = a.sum(axis=0), b.sum(axis=0)
    else:
        a, b = a[theta], b[theta]
    f1 = np.cumsum(a[:, 3]) / a[:, 3].sum()
    f2 = np.cumsum(b[:, 3]) / b[:, 3].sum()
    d = float(np.max(np.abs(f1 - f2)))
    n1 = a[:, 3].sum() ** 2 / a[:, 4].sum()
    n2 = b[:, 3].sum() ** 2 / b[:, 4].sum()
    return d, n1, n2


def ks_crit(n1, n2, alpha=1e-3):
    return C_ALPHA[alpha] * np.sqrt((n1 + n2) / (n1 * n2))


def welch_z(dev, ref):
    """(difference of the means, its combined standard error, z): the device runs' mean against the
    oracle runs' mean, each with its own sample variance (Welch)"""
    dev = np.asarray(dev, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    se = np.sqrt(dev.var(ddof=1) / len(dev) + ref.var(ddof=1) / len(ref))
    diff = dev.mean() - ref.mean()
    return diff, se, diff / se
