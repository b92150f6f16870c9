"""Python binding of libalvrl.so (the C ABI in include/alvrl.h).

This is the host-side mirror used by tests and bench.py.  It is a thin ctypes
layer: device buffers are torch tensors (plumbing only), every computation runs
in the HIP kernels of libalvrl.so.  There is no CPU fallback: importing this
module on a box without the built library raises, and every call that fails
inside the library raises AlvrlError with the library's message (the reference
raises std::runtime_error from Log(EError), src/libcore/logger.cpp:147).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "libalvrl.so")

REC_WORDS = 16
REC_HIT, REC_SMOOTH, REC_MEDIUM = 1, 2, 4
UINT32_MAX = 0xFFFFFFFF

ALVRL_OK = 0
ERRORS = {1: "INVALID", 2: "STATE", 3: "HIP", 4: "NOMEM", 5: "NUMERIC"}


class AlvrlError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"alvrl error {ERRORS.get(code, code)}: {msg}")
        self.code = code


def build(jobs: int = 8) -> str:
    """Compile libalvrl.so in-tree (hipcc --offload-arch=gfx950)."""
    subprocess.check_call(["make", "-s", f"-j{jobs}", "-C", PKG_DIR])
    return LIB_PATH


class Config(C.Structure):
    _fields_ = [("device", C.c_int), ("vol_vol_samples", C.c_int), ("vol_surf_samples", C.c_int),
                ("short_vrls", C.c_int), ("seed", C.c_uint32)]


class MediumDesc(C.Structure):
    _fields_ = [("sigma_s", C.c_float * 3), ("sigma_a", C.c_float * 3),
                ("sampling_weight", C.c_float), ("phase_type", C.c_int), ("phase_g", C.c_float)]


class ClusterJob(C.Structure):
    _fields_ = [("rows", C.POINTER(C.c_uint32)), ("locw", C.POINTER(C.c_double)),
                ("nrows", C.c_uint32), ("pixel_undersampling", C.c_float),
                ("undersampling", C.c_float), ("depth_correction", C.c_float),
                ("do_refine", C.c_int), ("stage_refine", C.c_uint32), ("stage_sample", C.c_uint32)]


_lib: Optional[C.CDLL] = None


def lib() -> C.CDLL:
    """Load the in-tree libalvrl.so; raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libalvrl.so not found at {LIB_PATH}: run __graft_entry__.build() "
                          "(there is no CPU fallback)")
    L = C.CDLL(LIB_PATH)
    u32, u64, i32, f32, vp = C.c_uint32, C.c_uint64, C.c_int, C.c_float, C.c_void_p
    P = C.POINTER
    L.alvrl_abi_version.restype = i32
    L.alvrl_last_error.argtypes = [vp]; L.alvrl_last_error.restype = C.c_char_p
    L.alvrl_ctx_create.argtypes = [P(Config), P(vp)]
    L.alvrl_ctx_destroy.argtypes = [vp]; L.alvrl_ctx_destroy.restype = None
    L.alvrl_set_medium.argtypes = [vp, P(MediumDesc)]
    L.alvrl_set_pass.argtypes = [vp, u32]
    L.alvrl_upload_vrls.argtypes = [vp, vp, u32, u64, i32]
    L.alvrl_num_vrls.argtypes = [vp]; L.alvrl_num_vrls.restype = u32
    L.alvrl_set_clusters.argtypes = [vp, u32, P(u32), P(u32), P(f32), P(u32), P(f32), u32]
    L.alvrl_gather_brute.argtypes = [vp, vp, vp, u32, vp, vp]
    L.alvrl_gather_clustered.argtypes = [vp, vp, vp, vp, u32, vp, vp]
    L.alvrl_make_work_items.argtypes = [P(u32), u32, vp, u32]; L.alvrl_make_work_items.restype = u32
    L.alvrl_build_R.argtypes = [vp, vp, vp, u32, vp, u64, u64, vp]
    L.alvrl_refine.argtypes = [vp, vp, u64, u32, P(ClusterJob), P(u32), P(u32), u32, P(u32),
                               P(u32), P(f32), P(i32), vp]
    L.alvrl_last_refine_ms.argtypes = [vp, P(f32)]
    L.alvrl_get_stats.argtypes = [vp, P(u64), P(u64)]
    L.alvrl_reset_stats.argtypes = [vp]
    L.alvrl_gather_brute_host.argtypes = [vp, vp, vp, u32, vp]
    L.alvrl_gather_clustered_host.argtypes = [vp, vp, vp, vp, u32, vp]
    L.alvrl_last_kernel_ms.argtypes = [vp, P(f32)]
    _lib = L
    return L


def _check(rc: int):
    if rc != ALVRL_OK:
        raise AlvrlError(rc, lib().alvrl_last_error(None).decode())


def _ptr(t) -> C.c_void_p:
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return C.c_void_p(t.ctypes.data)
    return C.c_void_p(t.data_ptr())


def _np(a, dt):
    return np.ascontiguousarray(a, dt)


def _arr(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


@dataclass
class Medium:
    sigma_s: Sequence[float] = (0.8, 0.6, 0.4)
    sigma_a: Sequence[float] = (0.05, 0.05, 0.05)
    sampling_weight: float = -1.0
    phase_type: int = 0
    phase_g: float = 0.0


class Context:
    """One device context = the device half of a vrlIntegrator (m_vrls, m_ci)."""

    def __init__(self, device: int = 0, vol_vol_samples: int = 2, vol_surf_samples: int = 2,
                 short_vrls: bool = True, seed: int = 0xA1B2C3D4):
        L = lib()
        self.L = L
        cfg = Config(device, vol_vol_samples, vol_surf_samples, int(short_vrls), seed & 0xFFFFFFFF)
        h = C.c_void_p()
        _check(L.alvrl_ctx_create(C.byref(cfg), C.byref(h)))
        self.h = h
        self.device = device
        self.nvrl = 0
        self.particle_count = 0

    def close(self):
        if getattr(self, "h", None):
            self.L.alvrl_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- state ----
    def set_medium(self, m: Medium):
        d = MediumDesc((C.c_float * 3)(*m.sigma_s), (C.c_float * 3)(*m.sigma_a),
                       m.sampling_weight, m.phase_type, m.phase_g)
        _check(self.L.alvrl_set_medium(self.h, C.byref(d)))

    def set_pass(self, p: int):
        _check(self.L.alvrl_set_pass(self.h, p))

    def upload_vrls(self, soa, particle_count: int):
        """soa: (9, n) float32 numpy array or CUDA tensor (start xyz, end xyz, power rgb)."""
        if isinstance(soa, np.ndarray):
            soa = _np(soa, np.float32)
            n = soa.shape[1]
            _check(self.L.alvrl_upload_vrls(self.h, _ptr(soa), n, particle_count, 0))
        else:
            soa = soa.contiguous()
            n = soa.shape[1]
            _check(self.L.alvrl_upload_vrls(self.h, _ptr(soa), n, particle_count, 1))
        self.nvrl = n
        self.particle_count = particle_count

    def set_clusters(self, slice_off, reps, weights, fb_reps, fb_weights):
        so = _np(slice_off, np.uint32); r = _np(reps, np.uint32); w = _np(weights, np.float32)
        fr = _np(fb_reps, np.uint32); fw = _np(fb_weights, np.float32)
        _check(self.L.alvrl_set_clusters(self.h, len(so) - 1, _arr(so, C.c_uint32),
                                         _arr(r, C.c_uint32), _arr(w, C.c_float),
                                         _arr(fr, C.c_uint32), _arr(fw, C.c_float), len(fr)))

    # ---- hot path ----
    def gather_brute(self, d_recs, d_out, d_ids=None, stream=None):
        n = d_recs.shape[0]
        _check(self.L.alvrl_gather_brute(self.h, _ptr(d_recs), _ptr(d_ids), n, _ptr(d_out),
                                         C.c_void_p(stream) if stream else None))

    def gather_clustered(self, d_recs, d_items, nitems, d_out, d_ids=None, stream=None):
        _check(self.L.alvrl_gather_clustered(self.h, _ptr(d_recs), _ptr(d_ids), _ptr(d_items),
                                             nitems, _ptr(d_out),
                                             C.c_void_p(stream) if stream else None))

    @staticmethod
    def make_work_items(slice_sorted: np.ndarray) -> np.ndarray:
        s = _np(slice_sorted, np.uint32)
        items = np.zeros((len(s) + 1, 4), np.uint32)
        n = lib().alvrl_make_work_items(_arr(s, C.c_uint32), len(s), C.c_void_p(items.ctypes.data),
                                        len(items))
        return items[:n].copy()

    def build_R(self, d_recs, d_Rt, ld: int, row0: int = 0, d_ids=None, stream=None):
        n = d_recs.shape[0]
        _check(self.L.alvrl_build_R(self.h, _ptr(d_recs), _ptr(d_ids), n, _ptr(d_Rt), ld, row0,
                                    C.c_void_p(stream) if stream else None))

    def refine(self, d_Rt, ld: int, jobs: list, init_vrls, init_off, stream=None):
        """jobs: list of dicts(rows, locw, pixel_undersampling, undersampling,
        depth_correction, do_refine, stage_refine, stage_sample)."""
        keep = []
        cj = (ClusterJob * max(1, len(jobs)))()
        for i, j in enumerate(jobs):
            rows = _np(j["rows"], np.uint32); lw = _np(j["locw"], np.float64)
            keep += [rows, lw]
            cj[i] = ClusterJob(_arr(rows, C.c_uint32), _arr(lw, C.c_double), len(rows),
                               j["pixel_undersampling"], j["undersampling"],
                               j.get("depth_correction", 1.0), int(j.get("do_refine", True)),
                               j["stage_refine"], j["stage_sample"])
        iv = _np(init_vrls, np.uint32); io = _np(init_off, np.uint32)
        nj = len(jobs)
        off = np.zeros(nj + 1, np.uint32)
        reps = np.zeros(max(1, nj * self.nvrl), np.uint32)
        w = np.zeros(max(1, nj * self.nvrl), np.float32)
        refined = np.zeros(max(1, nj), np.int32)
        _check(self.L.alvrl_refine(self.h, _ptr(d_Rt), ld, nj, cj, _arr(iv, C.c_uint32),
                                   _arr(io, C.c_uint32), len(io) - 1, _arr(off, C.c_uint32),
                                   _arr(reps, C.c_uint32), _arr(w, C.c_float),
                                   _arr(refined, C.c_int), C.c_void_p(stream) if stream else None))
        return off, reps[:off[-1]].copy(), w[:off[-1]].copy(), refined[:nj].astype(bool)

    def last_refine_ms(self) -> float:
        ms = C.c_float()
        _check(self.L.alvrl_last_refine_ms(self.h, C.byref(ms)))
        return ms.value

    # ---- host-pointer conveniences ----
    def gather_brute_host(self, recs: np.ndarray, ids=None) -> np.ndarray:
        recs = _np(recs, np.float32)
        out = np.zeros((recs.shape[0], 3), np.float32)
        idn = None if ids is None else _np(ids, np.uint32)
        _check(self.L.alvrl_gather_brute_host(self.h, _ptr(recs), _ptr(idn), recs.shape[0],
                                              _ptr(out)))
        return out

    def gather_clustered_host(self, recs: np.ndarray, slice_of_rec, ids=None) -> np.ndarray:
        recs = _np(recs, np.float32)
        out = np.zeros((recs.shape[0], 3), np.float32)
        sl = _np(slice_of_rec, np.uint32)
        idn = None if ids is None else _np(ids, np.uint32)
        _check(self.L.alvrl_gather_clustered_host(self.h, _ptr(recs), _ptr(idn), _ptr(sl),
                                                  recs.shape[0], _ptr(out)))
        return out

    # ---- stats / timing ----
    def stats(self):
        a, b = C.c_uint64(), C.c_uint64()
        _check(self.L.alvrl_get_stats(self.h, C.byref(a), C.byref(b)))
        return int(a.value), int(b.value)

    def reset_stats(self):
        _check(self.L.alvrl_reset_stats(self.h))

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        _check(self.L.alvrl_last_kernel_ms(self.h, C.byref(ms)))
        return ms.value
