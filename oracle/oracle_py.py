"""ctypes binding of the CPU oracle (oracle/liboracle.so) and of the partial reference build
(oracle/_ref/libref_partial.so).  TEST INFRASTRUCTURE ONLY: imported by tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg -- never by the product.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GRMO_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref_partial.so")

DP = C.POINTER(C.c_double)
U64P = C.POINTER(C.c_uint64)

# numpy views of the POD structs (same layout as include/grmonty_amd.h)
INIT_PHOTON = np.dtype([("x", "<f8", 4), ("k", "<f8", 4), ("w", "<f8"), ("e", "<f8"), ("l", "<f8"),
                        ("n_e_0", "<f8"), ("theta_e_0", "<f8"), ("b_0", "<f8"), ("e_0", "<f8"),
                        ("n_scatt", "<i4"), ("pad_", "<i4")])
SPEC_FIELDS = ["dn_dle", "de_dle", "nph", "nscatt", "x1i_av", "x2i_sq", "x3f_sq", "tau_abs", "tau_scatt",
               "ne_0", "theta_e_0", "b_0", "e_0"]
SPECTRUM_CELL = np.dtype([(f, "<f8") for f in SPEC_FIELDS])
TRACE = np.dtype([("id", "<u8"), ("parent_id", "<u8"), ("w", "<f8"), ("e", "<f8"), ("x1", "<f8"), ("x2", "<f8"),
                  ("x3", "<f8"), ("tau_abs", "<f8"), ("tau_scatt", "<f8"), ("n_scatt", "<i4"),
                  ("n_step", "<i4"), ("end_reason", "<i4"), ("ix2", "<i4"), ("i_e", "<i4"), ("pad_", "<i4")])
FLUID = np.dtype([("n_e", "<f8"), ("theta_e", "<f8"), ("b", "<f8"), ("u_con", "<f8", 4), ("u_cov", "<f8", 4),
                  ("b_con", "<f8", 4), ("b_cov", "<f8", 4)])


class Header(C.Structure):
    _fields_ = [("t", C.c_double), ("n", C.c_int * 2), ("x_start", C.c_double * 4), ("x_stop", C.c_double * 4),
                ("dx", C.c_double * 4), ("t_final", C.c_double), ("n_step", C.c_int), ("a", C.c_double),
                ("gamma", C.c_double), ("courant", C.c_double), ("dt_dump", C.c_double), ("dt_log", C.c_double),
                ("dt_img", C.c_double), ("dt_rdump", C.c_int), ("cnt_dump", C.c_int), ("cnt_img", C.c_int),
                ("cnt_rdump", C.c_int), ("dt", C.c_double), ("lim", C.c_int), ("failed", C.c_int),
                ("r_in", C.c_double), ("r_out", C.c_double), ("h_slope", C.c_double), ("r_0", C.c_double)]


class Units(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("mass_unit", "l_unit", "t_unit", "rho_unit", "u_unit", "b_unit",
                                          "theta_e_unit", "n_e_unit")]


def ptr(a: np.ndarray, t=DP):
    return a.ctypes.data_as(t)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        vp = C.c_void_p
        sig = {
            "grmo_model_new": (vp, [C.c_int, C.c_double]),
            "grmo_model_free": (None, [vp]),
            "grmo_model_read_file": (C.c_int, [vp, C.c_char_p]),
            "grmo_model_set": (C.c_int, [vp, C.POINTER(Header), C.POINTER(DP)]),
            "grmo_model_get_header": (None, [vp, C.POINTER(Header)]),
            "grmo_model_get_units": (None, [vp, C.POINTER(Units)]),
            "grmo_model_get_scalars": (None, [vp, DP]),
            "grmo_model_set_max_tau_scatt": (None, [vp, C.c_double]),
            "grmo_model_field": (DP, [vp, C.c_int]),
            "grmo_init_geometry": (None, [vp]),
            "grmo_init_hotcross": (None, [vp, C.c_int]),
            "grmo_init_emiss_tables": (None, [vp]),
            "grmo_init_weight_table": (None, [vp]),
            "grmo_init_nint_table": (None, [vp]),
            "grmo_init_all": (None, [vp, C.c_int]),
            "grmo_table": (DP, [vp, C.c_int]),
            "grmo_set_table": (None, [vp, C.c_int, DP]),
            "grmo_gcov": (None, [vp, DP, DP]),
            "grmo_gcon": (None, [vp, DP, DP]),
            "grmo_connection": (None, [vp, DP, DP]),
            "grmo_init_dkdlam": (None, [vp, DP, DP, DP]),
            "grmo_step_size": (C.c_double, [vp, DP, DP]),
            "grmo_push_photon": (None, [vp, DP, C.c_double]),
            "grmo_fluid_params": (None, [vp, DP, vp]),
            "grmo_bk_angle": (C.c_double, [DP, vp, C.c_double]),
            "grmo_fluid_nu": (C.c_double, [DP, DP]),
            "grmo_alpha_inv_scatt": (C.c_double, [vp, C.c_double, C.c_double, C.c_double]),
            "grmo_alpha_inv_abs": (C.c_double, [vp] + [C.c_double] * 5),
            "grmo_hotcross_lookup": (C.c_double, [vp, C.c_double, C.c_double]),
            "grmo_hotcross_num": (C.c_double, [C.c_double, C.c_double]),
            "grmo_synch": (C.c_double, [vp] + [C.c_double] * 5),
            "grmo_k2_eval": (C.c_double, [vp, C.c_double]),
            "grmo_f_eval": (C.c_double, [vp, C.c_double, C.c_double, C.c_double]),
            "grmo_make_tetrad": (None, [DP, DP, DP, DP, DP]),
            "grmo_boost": (None, [DP, DP, DP]),
            "grmo_gk61": (C.c_double, [C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                                       C.c_int]),
            "grmo_rng_new": (vp, [C.c_int, C.c_uint64, C.c_uint64]),
            "grmo_rng_free": (None, [vp]),
            "grmo_rng_uniform": (C.c_double, [vp]),
            "grmo_rng_chi_sq": (C.c_double, [vp, C.c_int]),
            "grmo_rng_counter": (C.c_uint64, [vp]),
            "grmo_sample_electron": (None, [vp, DP, DP, C.c_double]),
            "grmo_sample_klein_nishina": (C.c_double, [vp, C.c_double]),
            "grmo_sample_thomson": (C.c_double, [vp]),
            "grmo_sample_rand_dir": (None, [vp, DP]),
            "grmo_sample_scattered": (None, [vp, DP, DP, DP]),
            "grmo_philox4x32": (None, [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
            "grmo_child_id": (C.c_uint64, [C.c_uint64, C.c_uint64]),
            "grmo_track_batch": (C.c_int64, [vp, vp, C.c_size_t, C.c_int, C.c_uint64, C.c_uint64, C.c_int,
                                             C.c_uint64, C.c_uint64, C.c_double, vp, C.c_size_t]),
            "grmo_track_concurrent": (C.c_int64, [vp, vp, C.c_size_t, C.c_uint64, C.c_uint64,
                                                  C.POINTER(C.c_int64), C.c_size_t, vp, C.c_size_t, DP,
                                                  C.c_size_t, C.POINTER(C.c_int64)]),
            "grmo_last_trace_count": (C.c_int64, [vp]),
            "grmo_reset_spectrum": (None, [vp]),
            "grmo_get_spectrum": (None, [vp, vp]),
            "grmo_set_spectrum": (None, [vp, vp]),
            "grmo_get_counters": (None, [vp, U64P]),
            "grmo_emit": (C.c_int64, [vp, C.c_uint64, vp, C.c_size_t, C.POINTER(C.c_int)]),
            "grmo_init_zone": (None, [vp, C.c_int, C.c_int, DP]),
            "grmo_emit_philox": (C.c_int64, [vp, C.c_uint64, C.c_int64, C.c_int64, vp, C.c_size_t]),
            "grmo_run_simulation": (C.c_double, [vp, C.c_uint64]),
            "grmo_run_simulation_traced": (C.c_double, [vp, C.c_uint64, vp, C.c_size_t, C.POINTER(C.c_int64)]),
            "grmo_report_spectrum": (C.c_int, [vp, C.c_char_p, DP]),
            "grmo_sizeof": (C.c_size_t, [C.c_int]),
            "grmo_dbg_push_stats": (None, [U64P]),
            "grmo_dbg_hotcross_stats": (None, [U64P]),
            "grmo_dbg_sampler_stats": (None, [U64P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def ref():
    """The reference's own tetrads/proba/monty_rand/integration sources (partial build), or None."""
    global _ref
    if _ref is None:
        if not os.path.exists(REF_PATH):
            return None
        R = C.CDLL(REF_PATH)
        for name, (res, args) in {
            "ref_rng_init": (None, [C.c_int]),
            "ref_uniform": (C.c_double, []),
            "ref_chi_sq": (C.c_double, [C.c_int]),
            "ref_sample_electron": (None, [DP, DP, C.c_double]),
            "ref_sample_klein_nishina": (C.c_double, [C.c_double]),
            "ref_sample_thomson": (C.c_double, []),
            "ref_sample_rand_dir": (None, [DP]),
            "ref_sample_y": (C.c_double, [C.c_double]),
            "ref_sample_mu": (C.c_double, [C.c_double]),
            "ref_make_tetrad": (None, [DP, DP, DP, DP, DP]),
            "ref_coordinate_to_tetrad": (None, [DP, DP, DP]),
            "ref_tetrad_to_coordinate": (None, [DP, DP, DP]),
            "ref_gk61": (C.c_double, [C.c_int, C.c_double, C.c_double, C.c_double, C.c_double, C.c_int]),
        }.items():
            f = getattr(R, name)
            f.restype = res
            f.argtypes = args
        _ref = R
    return _ref


class OracleModel:
    """HARMModel restatement: load dump, init tables, emit, track, report."""

    def __init__(self, path: str | None = None, photon_n: int = 5000, mass_unit: float = 4e19):
        self.L = lib()
        self.h = self.L.grmo_model_new(photon_n, mass_unit)
        if path is not None:
            rc = self.L.grmo_model_read_file(self.h, path.encode())
            if rc != 0:
                raise IOError(f"oracle could not read {path}: {rc}")

    def close(self):
        if self.h:
            self.L.grmo_model_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def header(self) -> Header:
        h = Header()
        self.L.grmo_model_get_header(self.h, C.byref(h))
        return h

    @property
    def units(self) -> Units:
        u = Units()
        self.L.grmo_model_get_units(self.h, C.byref(u))
        return u

    def scalars(self):
        out = np.zeros(5)
        self.L.grmo_model_get_scalars(self.h, ptr(out))
        return dict(bias_norm=out[0], rh=out[1], x1_min=out[2], max_tau_scatt=out[3], d_tau_k=out[4])

    def field(self, which: int) -> np.ndarray:
        h = self.header
        n = h.n[0] * h.n[1]
        p = self.L.grmo_model_field(self.h, which)
        return np.ctypeslib.as_array(p, shape=(n,)).copy().reshape(h.n[0], h.n[1])

    def init(self, n_threads: int = 8):
        self.L.grmo_init_all(self.h, n_threads)

    TABLE_SIZES = {0: 221 * 81, 1: 201, 2: 201, 3: 201, 4: 20001, 5: 20001}

    def table(self, which: int) -> np.ndarray:
        if which == 6:
            h = self.header
            n = h.n[0] * h.n[1]
        else:
            n = self.TABLE_SIZES[which]
        p = self.L.grmo_table(self.h, which)
        return np.ctypeslib.as_array(p, shape=(n,)).copy()

    def set_table(self, which: int, arr: np.ndarray):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        self.L.grmo_set_table(self.h, which, ptr(a))

    def emit(self, seed: int = 123, cap: int = 1 << 22) -> np.ndarray:
        out = np.zeros(cap, dtype=INIT_PHOTON)
        done = C.c_int(0)
        n = self.L.grmo_emit(self.h, seed, out.ctypes.data_as(C.c_void_p), cap, C.byref(done))
        return out[:n]

    def emit_philox(self, seed: int = 123, z0: int = 0, z1: int = -1) -> np.ndarray:
        """Emission with the product's per-photon Philox streams (zones [z0, z1))."""
        n = self.L.grmo_emit_philox(self.h, seed, z0, z1, None, 0)
        out = np.zeros(n, dtype=INIT_PHOTON)
        got = self.L.grmo_emit_philox(self.h, seed, z0, z1, out.ctypes.data_as(C.c_void_p), n)
        assert got == n
        return out

    def init_zone(self, i: int, j: int):
        out = np.zeros(2)
        self.L.grmo_init_zone(self.h, i, j, ptr(out))
        return out[0], out[1]

    def track(self, photons: np.ndarray, rng_mode: int = 1, seed: int = 123, id_base: int = 0, frozen: bool = True,
              scatt0: int = 0, rec0: int = 0, max_tau0: float | None = None, trace_cap: int = 0):
        ph = np.ascontiguousarray(photons, dtype=INIT_PHOTON)
        if max_tau0 is None:
            max_tau0 = self.scalars()["max_tau_scatt"]
        tr = np.zeros(max(trace_cap, 1), dtype=TRACE)
        n = self.L.grmo_track_batch(self.h, ph.ctypes.data_as(C.c_void_p), len(ph), rng_mode, seed, id_base,
                                    1 if frozen else 0, scatt0, rec0, max_tau0,
                                    tr.ctypes.data_as(C.c_void_p) if trace_cap else None, trace_cap)
        return tr[:min(n, trace_cap)] if trace_cap else None

    EMU_KEYS = ("slots", "group", "refresh", "child_min", "depth_first", "claim_sh", "warm_n", "warm_slack",
                "warm_b0", "flight_cap", "timeline")
    EMU_DEVICE = dict(slots=131072, group=64, refresh=64, child_min=8, depth_first=0, claim_sh=-1, warm_n=-1,
                      warm_slack=4, warm_b0=64, flight_cap=0, timeline=0)
    EMU_SERIAL = dict(slots=1, group=1, refresh=1, child_min=1, depth_first=1, claim_sh=0, warm_n=0,
                      warm_slack=4, warm_b0=64, flight_cap=0, timeline=0)

    def track_concurrent(self, photons: np.ndarray, seed: int = 123, id_base: int = 0, trace_cap: int = 0,
                         timeline_cap: int = 0, **cfg):
        """grmo_track_concurrent: the batch scheduled as a concurrent engine would (EMU_KEYS; defaults
        EMU_SERIAL, i.e. the serial reference).  Returns (rounds, trace or None, timeline rows)."""
        c = dict(self.EMU_SERIAL)
        for k, v in cfg.items():
            if k not in c:
                raise KeyError(k)
            c[k] = v
        arr = (C.c_int64 * len(self.EMU_KEYS))(*[int(c[k]) for k in self.EMU_KEYS])
        ph = np.ascontiguousarray(photons, dtype=INIT_PHOTON)
        tr = np.zeros(max(trace_cap, 1), dtype=TRACE)
        tl = np.zeros(max(timeline_cap, 1) * 6)
        ntl = C.c_int64(0)
        rounds = self.L.grmo_track_concurrent(self.h, ph.ctypes.data_as(C.c_void_p), len(ph), seed, id_base, arr,
                                              len(self.EMU_KEYS), tr.ctypes.data_as(C.c_void_p) if trace_cap else None,
                                              trace_cap, ptr(tl), len(tl), C.byref(ntl))
        nt = min(self.L.grmo_last_trace_count(self.h), trace_cap)
        return rounds, (tr[:nt] if trace_cap else None), tl[:6 * ntl.value].reshape(-1, 6)

    def spectrum(self) -> np.ndarray:
        s = np.zeros(6 * 200, dtype=SPECTRUM_CELL)
        self.L.grmo_get_spectrum(self.h, s.ctypes.data_as(C.c_void_p))
        return s.reshape(6, 200)

    def set_spectrum(self, spec: np.ndarray):
        s = np.ascontiguousarray(spec, dtype=SPECTRUM_CELL).reshape(-1)
        assert len(s) == 6 * 200
        self.L.grmo_set_spectrum(self.h, s.ctypes.data_as(C.c_void_p))

    def counters(self):
        c = np.zeros(4, dtype=np.uint64)
        self.L.grmo_get_counters(self.h, ptr(c, U64P))
        return dict(created=int(c[0]), scattered=int(c[1]), recorded=int(c[2]), steps=int(c[3]))

    def reset(self):
        self.L.grmo_reset_spectrum(self.h)

    def run_simulation(self, seed: int = 123) -> float:
        return self.L.grmo_run_simulation(self.h, seed)

    def run_simulation_traced(self, seed: int = 123, trace_cap: int = 1 << 23):
        """run_simulation (reference stream and order) with every photon end recorded"""
        tr = np.zeros(trace_cap, dtype=TRACE)
        n = C.c_int64(0)
        t = self.L.grmo_run_simulation_traced(self.h, seed, tr.ctypes.data_as(C.c_void_p), trace_cap, C.byref(n))
        return t, tr[:min(n.value, trace_cap)], n.value

    def report(self, path: str | None):
        out = np.zeros(2)
        self.L.grmo_report_spectrum(self.h, path.encode() if path else None, ptr(out))
        return dict(luminosity=out[0], max_tau_scatt=out[1])


def push_stats():
    out = np.zeros(3, dtype=np.uint64)
    lib().grmo_dbg_push_stats(ptr(out, U64P))
    return dict(attempts=int(out[0]), iter2=int(out[1]), halvings=int(out[2]))
