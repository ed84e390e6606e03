"""grmonty_amd -- Python binding of the MI355X superphoton transport engine (C-ABI in
include/grmonty_amd.h, implemented in cuda-grmonty_amd/libgrmonty_amd.so).

The library is loaded from the source tree; if it is missing the import raises (there is no CPU
fallback: the transport path is the HIP kernel or nothing).

    m = Model.load(dump_path, photon_n=1_000_000)     # HARMModel(photon_n, mass_unit).read_file
    m.init(threads)                                     # init(): geometry + tables
    e = Engine(m, device=0)                             # cuda_super_photon::alloc_memory
    e.emit_setup(m)                                     # zone table -> HBM
    ptr, n = e.emit(seed=123)                           # make_super_photon on the GPU
    e.track_device(ptr, n)                              # track_super_photons
    (host emission, m.emit(seed) -> InitPhoton records, + e.track(ph) is the same list of photons)
    spec, n_rec, n_scatt, max_tau = e.finish()
    m.write_spectrum(spec, "spectrum.txt")              # report_spectrum
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("GRMONTY_AMD_LIB") or os.path.join(PKG_DIR, "libgrmonty_amd.so")
REPO_DIR = os.path.dirname(PKG_DIR)
HEADER_PATH = os.path.join(REPO_DIR, "include", "grmonty_amd.h")
DEBUG_HEADER_PATH = os.path.join(REPO_DIR, "include", "grmonty_amd_debug.h")

DP = C.POINTER(C.c_double)
VP = C.c_void_p

INIT_PHOTON = np.dtype([("x", "<f8", 4), ("k", "<f8", 4), ("w", "<f8"), ("e", "<f8"), ("l", "<f8"),
                        ("n_e_0", "<f8"), ("theta_e_0", "<f8"), ("b_0", "<f8"), ("e_0", "<f8"),
                        ("n_scatt", "<i4"), ("pad_", "<i4")])
SPEC_FIELDS = ["dn_dle", "de_dle", "nph", "nscatt", "x1i_av", "x2i_sq", "x3f_sq", "tau_abs", "tau_scatt",
               "ne_0", "theta_e_0", "b_0", "e_0"]
SPECTRUM_CELL = np.dtype([(f, "<f8") for f in SPEC_FIELDS])
TRACE = np.dtype([("id", "<u8"), ("parent_id", "<u8"), ("w", "<f8"), ("e", "<f8"), ("x1", "<f8"), ("x2", "<f8"),
                  ("x3", "<f8"), ("tau_abs", "<f8"), ("tau_scatt", "<f8"), ("n_scatt", "<i4"),
                  ("n_step", "<i4"), ("end_reason", "<i4"), ("ix2", "<i4"), ("i_e", "<i4"), ("pad_", "<i4")])

EMIT_ZONE = np.dtype([("nz", "<f8"), ("dn_max", "<f8"), ("x", "<f8", 4), ("n_e", "<f8"), ("theta_e", "<f8"),
                      ("b", "<f8"), ("e_con", "<f8", (4, 4)), ("e_cov_t", "<f8", 4), ("e_cov_z", "<f8", 4),
                      ("pad_", "<f8")])

OPT_SEED, OPT_BIAS_MODE, OPT_TRACE_CAP, OPT_GRID_BLOCKS, OPT_ID_BASE = 0, 1, 2, 3, 4
OPT_FROZEN_SCATT, OPT_FROZEN_REC, OPT_FROZEN_MAXTAU, OPT_WARMUP, OPT_REFILL_MIN = 5, 6, 7, 8, 9
OPT_WATCHDOG_MS = 10
OPT_CHILD_MIN = 11
OPT_WARMUP_SLACK = 12
OPT_LONE = 13
OPT_WARMUP_BATCH = 14
OPT_EARLY_STEPS = 15
OPT_EARLY_SERIAL = 16
OPT_KARG_TEST = 17
OPT_WARMUP_SPREAD = 19
OPT_FLIGHT_RATIO = 22
OPT_JOB_START_WAIT_MS = 28
OPT_EARLY_CHILDREN = 29
OPT_SPLIT, OPT_SPLIT_THR, OPT_SPLIT_SPIN, OPT_SPLIT_GTHR, OPT_SPLIT_BATCH = 23, 24, 25, 26, 27
N_TH_BINS, N_E_BINS = 6, 200


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


class Stats(C.Structure):
    _fields_ = [("n_tracked", C.c_uint64), ("n_primaries", C.c_uint64), ("n_children", C.c_uint64),
                ("n_steps", C.c_uint64), ("n_overflow", C.c_uint64), ("n_dropped", C.c_uint64),
                ("n_launches", C.c_uint64), ("kernel_ms", C.c_double), ("last_kernel_ms", C.c_double),
                ("last_steps", C.c_uint64), ("last_emit_ms", C.c_double),
                ("max_launch_ms", C.c_double), ("max_launch_steps", C.c_uint64),
                ("max_photon_steps", C.c_uint64), ("n_long_photons", C.c_uint64), ("n_abandoned", C.c_uint64),
                ("n_nan_photons", C.c_uint64), ("n_lone", C.c_uint64), ("lone_ms", C.c_double),
                ("n_early", C.c_uint64), ("early_ms", C.c_double), ("last_grid", C.c_uint64),
                ("n_early_children", C.c_uint64), ("n_lone_children", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# every entry point of include/grmonty_amd.h with its ctypes signature
SIGNATURES = {
    "grm_engine_create": (C.c_int, [C.POINTER(Header), C.POINTER(DP), C.POINTER(Units), DP, DP, DP, C.c_int,
                                    C.POINTER(VP)]),
    "grm_engine_destroy": (None, [VP]),
    "grm_engine_last_error": (C.c_char_p, [VP]),
    "grm_engine_set_option": (C.c_int, [VP, C.c_int, C.c_int64]),
    "grm_engine_track": (C.c_int, [VP, VP, C.c_size_t]),
    "grm_engine_track_device": (C.c_int, [VP, VP, C.c_size_t]),
    "grm_engine_finish": (C.c_int, [VP, VP, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), DP]),
    "grm_engine_reset": (C.c_int, [VP]),
    "grm_engine_stats": (C.c_int, [VP, C.POINTER(Stats)]),
    "grm_engine_spectrum_device_ptr": (VP, [VP]),
    "grm_engine_trace": (C.c_int64, [VP, VP, C.c_size_t]),
    "grm_model_load": (C.c_int, [C.c_char_p, C.c_int, C.c_double, C.POINTER(VP)]),
    "grm_model_free": (None, [VP]),
    "grm_model_last_error": (C.c_char_p, []),
    "grm_model_init": (C.c_int, [VP, C.c_int]),
    "grm_model_init_device": (C.c_int, [VP, C.c_int, C.c_int]),
    "grm_model_table_ms": (C.c_double, [VP]),
    "grm_model_header": (None, [VP, C.POINTER(Header)]),
    "grm_model_units": (None, [VP, C.POINTER(Units)]),
    "grm_model_scalars": (None, [VP, DP]),
    "grm_model_field": (DP, [VP, C.c_int]),
    "grm_model_table": (DP, [VP, C.c_int]),
    "grm_engine_create_from_model": (C.c_int, [VP, C.c_int, C.POINTER(VP)]),
    "grm_model_emit": (C.c_int64, [VP, C.c_uint64, C.c_int64, C.c_int64, VP, C.c_size_t, C.c_int]),
    "grm_model_emit_strided": (C.c_int64, [VP, C.c_uint64, C.c_int64, C.c_int64, C.c_int64, VP, C.c_size_t, C.c_int]),
    "grm_model_zone_weights": (C.c_int, [VP, DP]),
    "grm_write_spectrum": (C.c_int, [VP, VP, C.c_char_p, DP]),
    "grm_write_spectrum_stats": (C.c_int, [VP, VP, C.c_char_p]),
    "grm_model_zone_table": (C.c_int, [VP, C.c_int64, C.c_int64, VP, C.c_int]),
    "grm_engine_emit_setup": (C.c_int, [VP, VP, C.c_int64, DP, DP]),
    "grm_engine_emit_setup_from_model": (C.c_int, [VP, VP]),
    "grm_engine_emit": (C.c_int, [VP, C.c_uint64, C.c_int64, C.c_int64, C.POINTER(VP), C.POINTER(C.c_uint64)]),
    "grm_engine_emit_strided": (C.c_int, [VP, C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.POINTER(VP),
                                          C.POINTER(C.c_uint64)]),
    "grm_engine_download": (C.c_int, [VP, VP, C.c_size_t, VP]),
    "grm_probe": (C.c_int, [VP, C.c_int, DP, C.c_int, DP, C.c_int, C.c_size_t]),
    "grm_engine_upload": (C.c_int, [VP, VP, C.c_size_t, C.POINTER(VP)]),
    "grm_rccl_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "grm_engine_comm_init": (C.c_int, [VP, C.POINTER(C.c_uint8), C.c_int, C.c_int]),
    "grm_engine_allreduce": (C.c_int, [VP]),
    "grm_engine_stash_reserve": (C.c_int, [VP, C.c_int]),
    "grm_engine_stash": (C.c_int, [VP, C.c_int]),
    "grm_engine_allreduce_stash": (C.c_int, [VP, C.c_int, C.c_int]),
    "grm_engine_stash_read": (C.c_int, [VP, C.c_int, VP, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "grm_engine_stash_raw": (C.c_int, [VP, C.c_int, C.c_int, VP, VP, VP, C.c_int]),
    "grm_stash_words": (C.c_int, [C.c_int]),
    "grm_engine_begin_pass": (C.c_int, [VP, C.c_int]),
    "grm_engine_counters_ipc_handle": (C.c_int, [VP, C.POINTER(C.c_uint8)]),
    "grm_engine_set_peers": (C.c_int, [VP, C.POINTER(C.c_uint8), C.c_int, C.c_int]),
    "grm_engine_link_peers": (C.c_int, [C.POINTER(VP), C.c_int]),
    "grm_engine_job_counters": (C.c_int, [VP, DP]),
    "grm_device_peer_ok": (C.c_int, [C.c_int, C.c_int]),
    "grm_engine_debug_timing": (C.c_int, [VP, C.POINTER(C.c_uint64), C.c_int]),
    "grm_engine_debug_waves": (C.c_int64, [VP, VP, C.c_size_t]),
    "grm_engine_debug_stuck": (C.c_int64, [VP, VP, C.c_size_t]),
    "grm_engine_debug_counters": (C.c_int, [VP, C.POINTER(C.c_uint64)]),
    "grm_engine_debug_phases": (C.c_int, [VP, C.POINTER(C.c_uint64)]),
    "grm_engine_debug_admissions": (C.c_int64, [VP, C.POINTER(C.c_uint64), C.c_size_t]),
    "grm_sizeof": (C.c_size_t, [C.c_int]),
    "grm_version": (C.c_char_p, []),
}

_lib = None


def lib() -> C.CDLL:
    """Load the in-tree C-ABI library; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C cuda-grmonty_amd` or __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


class Model:
    """HARMModel host side (loader, tables, emission, writer) -- C++ in libgrmonty_amd.so."""

    TABLE_SIZES = {0: 221 * 81, 1: 201, 2: 201, 3: 201, 4: 20001, 5: 20001}

    def __init__(self, handle):
        self.L = lib()
        self.h = handle

    @classmethod
    def load(cls, path: str, photon_n: int = 5_000_000, mass_unit: float = 4e19) -> "Model":
        L = lib()
        h = VP()
        if L.grm_model_load(path.encode(), int(photon_n), float(mass_unit), C.byref(h)) != 0:
            raise IOError(L.grm_model_last_error().decode())
        return cls(h)

    def close(self):
        if getattr(self, "h", None):
            self.L.grm_model_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def init(self, n_threads: int = 0, device=None) -> "Model":
        """init() of the model (harm_model.cpp:234-240); device = a GPU index: the hotcross, K2 and
        nint tables are built there (csrc/grm_tables.hip), the rest on the host."""
        if device is None:
            rc = self.L.grm_model_init(self.h, int(n_threads))
        else:
            rc = self.L.grm_model_init_device(self.h, int(n_threads), int(device))
        if rc != 0:
            raise RuntimeError(self.L.grm_model_last_error().decode())
        return self

    @property
    def table_ms(self) -> float:
        """GPU time (ms) of the device table builders of the last init(device=...)"""
        return float(self.L.grm_model_table_ms(self.h))

    @property
    def header(self) -> Header:
        h = Header()
        self.L.grm_model_header(self.h, C.byref(h))
        return h

    @property
    def units(self) -> Units:
        u = Units()
        self.L.grm_model_units(self.h, C.byref(u))
        return u

    def scalars(self) -> dict:
        o = np.zeros(5)
        self.L.grm_model_scalars(self.h, o.ctypes.data_as(DP))
        return dict(bias_norm=o[0], x1_min=o[1], max_tau_scatt=o[2], d_tau_k=o[3], rh=o[4])

    def field(self, which: int) -> np.ndarray:
        h = self.header
        n = h.n[0] * h.n[1]
        return np.ctypeslib.as_array(self.L.grm_model_field(self.h, which), shape=(n,)).copy().reshape(h.n[0], h.n[1])

    def table(self, which: int) -> np.ndarray:
        if which == 6:
            h = self.header
            n = h.n[0] * h.n[1]
        else:
            n = self.TABLE_SIZES[which]
        return np.ctypeslib.as_array(self.L.grm_model_table(self.h, which), shape=(n,)).copy()

    def count(self, seed: int = 123, z0: int = 0, z1: int = -1, threads: int = 0, stride: int = 1) -> int:
        n = self.L.grm_model_emit_strided(self.h, seed, z0, z1, stride, None, 0, threads)
        if n < 0:
            raise RuntimeError(self.L.grm_model_last_error().decode())
        return int(n)

    def emit(self, seed: int = 123, z0: int = 0, z1: int = -1, threads: int = 0, stride: int = 1) -> np.ndarray:
        """the superphotons of zones z0, z0 + stride, ... < z1 (make_super_photon's zone walk)"""
        n = self.count(seed, z0, z1, threads, stride)
        out = np.zeros(n, dtype=INIT_PHOTON)
        got = self.L.grm_model_emit_strided(self.h, seed, z0, z1, stride, _ptr(out), n, threads)
        if got != n:
            raise RuntimeError(self.L.grm_model_last_error().decode())
        return out

    def zone_table(self, z0: int = 0, z1: int = -1, threads: int = 0) -> np.ndarray:
        """Per-zone emission records (init_zone nz / dn_max, zone centre, fluid, tetrad)."""
        h = self.header
        nz = h.n[0] * h.n[1]
        z1 = nz if z1 < 0 or z1 > nz else z1
        out = np.zeros(max(z1 - z0, 0), dtype=EMIT_ZONE)
        if self.L.grm_model_zone_table(self.h, z0, z1, _ptr(out), threads) != 0:
            raise RuntimeError(self.L.grm_model_last_error().decode())
        return out

    def zone_weights(self) -> np.ndarray:
        h = self.header
        out = np.zeros(h.n[0] * h.n[1])
        if self.L.grm_model_zone_weights(self.h, out.ctypes.data_as(DP)) != 0:
            raise RuntimeError(self.L.grm_model_last_error().decode())
        return out

    def write_spectrum(self, spectrum: np.ndarray, path: str | None):
        s = np.ascontiguousarray(spectrum, dtype=SPECTRUM_CELL).reshape(-1)
        o = np.zeros(2)
        if self.L.grm_write_spectrum(self.h, _ptr(s), path.encode() if path else None, o.ctypes.data_as(DP)) != 0:
            raise IOError(self.L.grm_model_last_error().decode())
        return dict(luminosity=o[0], max_tau_scatt=o[1])

    def write_spectrum_stats(self, spectrum: np.ndarray, path: str):
        s = np.ascontiguousarray(spectrum, dtype=SPECTRUM_CELL).reshape(-1)
        if self.L.grm_write_spectrum_stats(self.h, _ptr(s), path.encode()) != 0:
            raise IOError(self.L.grm_model_last_error().decode())


class Engine:
    """cuda_super_photon replacement: device buffers + persistent transport kernel on one GPU."""

    def __init__(self, model: Model, device: int = 0):
        self.L = lib()
        h = VP()
        rc = self.L.grm_engine_create_from_model(model.h, int(device), C.byref(h))
        if rc != 0:
            msg = self.L.grm_engine_last_error(h).decode() if h else self.L.grm_model_last_error().decode()
            if h:
                self.L.grm_engine_destroy(h)
            raise RuntimeError(f"engine creation failed: {msg}")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.grm_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(self.L.grm_engine_last_error(self.h).decode())

    def set_option(self, opt: int, value: int):
        self._check(self.L.grm_engine_set_option(self.h, opt, int(value)))

    def emit_setup(self, model: "Model"):
        """Upload the model's zone table and emission tables (once per model)."""
        rc = self.L.grm_engine_emit_setup_from_model(self.h, model.h)
        if rc != 0:
            msg = self.L.grm_engine_last_error(self.h).decode() or self.L.grm_model_last_error().decode()
            raise RuntimeError(msg)

    def emit(self, seed: int = 123, z0: int = 0, z1: int = -1, stride: int = 1) -> tuple[int, int]:
        """Emit the superphotons of zones z0, z0 + stride, ... < z1 on the GPU; returns (device
        address, count).  The buffer is engine-owned and valid until the next emit."""
        p, n = VP(), C.c_uint64()
        self._check(self.L.grm_engine_emit_strided(self.h, int(seed), int(z0), int(z1), int(stride), C.byref(p),
                                                   C.byref(n)))
        return int(p.value or 0), int(n.value)

    def download(self, dev_ptr: int, n: int) -> np.ndarray:
        out = np.zeros(n, dtype=INIT_PHOTON)
        self._check(self.L.grm_engine_download(self.h, C.c_void_p(dev_ptr), int(n), _ptr(out)))
        return out

    def track(self, photons: np.ndarray):
        ph = np.ascontiguousarray(photons, dtype=INIT_PHOTON)
        self._check(self.L.grm_engine_track(self.h, _ptr(ph), len(ph)))

    def track_device(self, dev_ptr: int, n: int):
        self._check(self.L.grm_engine_track_device(self.h, C.c_void_p(dev_ptr), int(n)))

    def finish(self):
        spec = np.zeros(N_TH_BINS * N_E_BINS, dtype=SPECTRUM_CELL)
        nr, ns, mt = C.c_uint64(), C.c_uint64(), C.c_double()
        self._check(self.L.grm_engine_finish(self.h, _ptr(spec), C.byref(nr), C.byref(ns), C.byref(mt)))
        return spec.reshape(N_TH_BINS, N_E_BINS), nr.value, ns.value, mt.value

    def reset(self):
        self._check(self.L.grm_engine_reset(self.h))

    def stats(self) -> dict:
        s = Stats()
        self._check(self.L.grm_engine_stats(self.h, C.byref(s)))
        return s.as_dict()

    def spectrum_device_ptr(self) -> int:
        return int(self.L.grm_engine_spectrum_device_ptr(self.h))

    def trace(self, cap: int) -> np.ndarray:
        out = np.zeros(max(cap, 1), dtype=TRACE)
        n = self.L.grm_engine_trace(self.h, _ptr(out), cap)
        if n < 0:
            raise RuntimeError("trace not enabled")
        return out[:min(n, cap)]

    def upload(self, photons: np.ndarray) -> int:
        """Copy photons into an engine-owned device buffer; returns its device address."""
        ph = np.ascontiguousarray(photons, dtype=INIT_PHOTON)
        out = VP()
        self._check(self.L.grm_engine_upload(self.h, _ptr(ph), len(ph), C.byref(out)))
        return int(out.value or 0)

    def comm_init(self, uid: bytes, nranks: int, rank: int):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._check(self.L.grm_engine_comm_init(self.h, buf, nranks, rank))

    def debug_timing(self, reset: bool = True):
        out = (C.c_uint64 * 48)()
        instrumented = self.L.grm_engine_debug_timing(self.h, out, 1 if reset else 0)
        return instrumented, list(out)

    def debug_waves(self) -> np.ndarray:
        """Per-wave record of the last transport launch: (start, exit) s_memrealtime ticks (100 MHz),
        loop trips, superphotons tracked."""
        n = self.L.grm_engine_debug_waves(self.h, None, 0)
        if n < 0:
            raise RuntimeError("no transport launch yet")
        out = np.zeros((n, 4), dtype=np.uint64)
        self.L.grm_engine_debug_waves(self.h, _ptr(out), n)
        return out

    def debug_stuck(self) -> np.ndarray:
        """Photons the launch watchdog abandoned: id, n_step, phase, depth, pend, w, e_0_s, dl, x[4], k[4]."""
        out = np.zeros((256, 16), dtype=np.float64)
        n = self.L.grm_engine_debug_stuck(self.h, _ptr(out), 256)
        if n < 0:
            raise RuntimeError(self.L.grm_engine_last_error(self.h).decode())
        return out[:n]

    def debug_phases(self) -> dict:
        """ms from the first wave's start of the last call's main launch to the end of the warm-up
        admission, to the pool's last claim chunk, and to the last wave's exit"""
        out = (C.c_uint64 * 4)()
        self._check(self.L.grm_engine_debug_phases(self.h, out))
        t0 = out[0]
        ms = lambda t: (t - t0) * 1e-5 if t else None  # noqa: E731  (100 MHz ticks)
        adm = (C.c_uint64 * 64)()
        k = self.L.grm_engine_debug_admissions(self.h, adm, 32)
        batches = [(ms(adm[2 * i]), int(adm[2 * i + 1])) for i in range(max(0, min(k, 32)))]
        return {"t0_ticks": int(t0), "warmup_end_ms": ms(out[1]), "pool_drained_ms": ms(out[2]),
                "last_exit_ms": ms(out[3]), "admissions": batches}

    def debug_counters(self) -> dict:
        """raw device counters (grm_engine_debug_counters)"""
        out = (C.c_uint64 * 16)()
        self._check(self.L.grm_engine_debug_counters(self.h, out))
        v = list(out)
        f = lambda b: float(np.array([b], dtype=np.uint64).view(np.float64)[0])  # noqa: E731
        return {"n_recorded": v[0], "n_scatt": v[1], "max_tau_scatt": f(v[2]), "n_steps": v[3],
                "n_tracked": v[4], "n_children": v[5], "n_overflow": v[6], "n_dropped": v[7], "n_primaries": v[8],
                "max_photon_steps": v[9], "n_long": v[10], "n_abandoned": v[11], "n_nan": v[13],
                "karg_bad": v[14]}

    def allreduce(self):
        self._check(self.L.grm_engine_allreduce(self.h))

    # deferred reduction: stash each pass's results on the device, one all-reduce for the job
    def stash_reserve(self, n_slots: int):
        self._check(self.L.grm_engine_stash_reserve(self.h, int(n_slots)))

    def stash(self, slot: int):
        self._check(self.L.grm_engine_stash(self.h, int(slot)))

    def allreduce_stash(self, n_slots: int, first: int = 0):
        """one grouped RCCL all-reduce of stash slots [first, first + n_slots)"""
        self._check(self.L.grm_engine_allreduce_stash(self.h, int(first), int(n_slots)))

    def stash_read(self, slot: int):
        """(spectrum, n_recorded, n_scatt, max_tau_scatt, n_steps) of a stashed pass"""
        spec = np.zeros(N_TH_BINS * N_E_BINS, dtype=SPECTRUM_CELL)
        nr, ns, mt, st = C.c_uint64(), C.c_uint64(), C.c_double(), C.c_uint64()
        self._check(self.L.grm_engine_stash_read(self.h, int(slot), _ptr(spec), C.byref(nr), C.byref(ns), C.byref(mt),
                                                 C.byref(st)))
        return spec.reshape(N_TH_BINS, N_E_BINS), nr.value, ns.value, mt.value, st.value

    def begin_pass(self, slot: int):
        """count the next pass into counter block `slot` (shared with the peers; reset first); -1 = the
        engine's private block"""
        self._check(self.L.grm_engine_begin_pass(self.h, int(slot)))

    def counters_ipc_handle(self) -> bytes:
        buf = (C.c_uint8 * 64)()
        self._check(self.L.grm_engine_counters_ipc_handle(self.h, buf))
        return bytes(buf)

    def set_peers(self, handles: list, rank: int):
        """the other ranks' counter blocks (their counters_ipc_handle(), rank order)"""
        n = len(handles)
        buf = (C.c_uint8 * (64 * max(n, 1))).from_buffer_copy(b"".join(handles) if n else bytes(64))
        self._check(self.L.grm_engine_set_peers(self.h, buf, n, int(rank)))

    def job_counters(self) -> dict:
        o = np.zeros(4)
        self._check(self.L.grm_engine_job_counters(self.h, o.ctypes.data_as(DP)))
        return dict(bias_den=o[0], n_scatt=o[1], n_recorded=o[2], max_tau_scatt=o[3])

    def stash_raw(self, n_slots: int, first: int = 0):
        """(spectra [n, words0] f64, sums [n, words1] u64, maxs [n, words2] u64): the stash's raw
        words in the engine's packing (grm_engine_stash_raw)"""
        w = [self.L.grm_stash_words(i) for i in range(3)]
        spec = np.zeros((n_slots, w[0]))
        sums = np.zeros((n_slots, w[1]), dtype=np.uint64)
        maxs = np.zeros((n_slots, w[2]), dtype=np.uint64)
        self._check(self.L.grm_engine_stash_raw(self.h, int(first), int(n_slots), _ptr(spec), _ptr(sums), _ptr(maxs), 0))
        return spec, sums, maxs

    def stash_raw_write(self, spec: np.ndarray, sums: np.ndarray, maxs: np.ndarray, first: int = 0):
        spec = np.ascontiguousarray(spec, dtype=np.float64)
        sums = np.ascontiguousarray(sums, dtype=np.uint64)
        maxs = np.ascontiguousarray(maxs, dtype=np.uint64)
        self._check(self.L.grm_engine_stash_raw(self.h, int(first), int(spec.shape[0]), _ptr(spec), _ptr(sums),
                                                _ptr(maxs), 1))

    def probe(self, which: int, inputs: np.ndarray, out_width: int) -> np.ndarray:
        a = np.ascontiguousarray(inputs, dtype=np.float64)
        if a.ndim == 1:
            a = a[:, None]
        out = np.zeros((a.shape[0], out_width))
        self._check(self.L.grm_probe(self.h, which, a.ctypes.data_as(DP), a.shape[1], out.ctypes.data_as(DP),
                                     out_width, a.shape[0]))
        return out


def shard_zones(zone_weights: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous zone ranges [z0, z1) with ~equal expected photon counts (init_zone's nz,
    harm_model.cpp:1337-1389) -- the multi-GPU partition of one run.  Zone streams are keyed by
    zone index, so the union over ranks emits exactly the single-GPU photon list."""
    w = np.asarray(zone_weights, dtype=np.float64)
    c = np.cumsum(w)
    tot = c[-1] if len(c) else 0.0
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(c, tot * r / world, side="right")))
    cuts.append(len(w))
    for r in range(1, len(cuts)):
        cuts[r] = max(cuts[r], cuts[r - 1])
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def zone_shards(zone_weights: np.ndarray, world: int, mode: str = "strided") -> list[tuple[int, int, int]]:
    """The multi-GPU partition of one run as (z0, z1, stride) zone sets, rank r's zones being
    z0, z0 + stride, ... < z1.

    "strided" (the default, bench.py's): rank r takes every world-th zone from zone r.  Each rank's
    photons then sample the whole disk, so its adaptive bias (bias_func, harm_model.cpp:1391-1404,
    driven by the counters of the photons IT recorded) sees the same mix of histories as one GPU
    does.  "contiguous": shard_zones' ranges of equal expected count -- a rank of inner zones alone
    records nothing and one of the escape region records 2-3x the average, which moved the job's
    recorded / scattered counts +17 / +30 / +43 % at 2 / 4 / 8 ranks (tests/test_gpu_multirank.py,
    DESIGN.md §7).  Either way zone streams are keyed by zone, so the union of the shards is exactly
    the single-GPU photon set -- the same initial states.  Transport streams are keyed by photon id,
    and rank r's ids start after the photons of ranks < r (rank-major), so with strided shards a
    photon's id, and its transport draws, differ from the single-GPU job's (zone order): the N-rank
    job is another valid run of the same photons, not a bit-replay."""
    n = len(zone_weights)
    if mode == "strided":
        return [(r, n, world) for r in range(world)]
    if mode == "contiguous":
        return [(a, b, 1) for a, b in shard_zones(zone_weights, world)]
    raise ValueError(mode)


def link_peers(engines: list):
    """share the pass counter blocks of engines on one device in one process (N-rank emulation)"""
    arr = (VP * len(engines))(*[e.h for e in engines])
    if lib().grm_engine_link_peers(arr, len(engines)) != 0:
        raise RuntimeError("grm_engine_link_peers failed")


def rccl_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    if lib().grm_rccl_unique_id(buf) != 0:
        raise RuntimeError("ncclGetUniqueId failed")
    return bytes(buf)


def header_symbols(paths=(HEADER_PATH, DEBUG_HEADER_PATH)) -> list[str]:
    """Names of the functions declared in the C headers -- the boundary (include/grmonty_amd.h) and
    the diagnostic / probe entry points (include/grmonty_amd_debug.h) -- for the ABI test."""
    import re
    if isinstance(paths, str):
        paths = (paths,)
    txt = "\n".join(open(p).read() for p in paths)
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(grm_[a-z0-9_]+)\s*\(", txt)))
