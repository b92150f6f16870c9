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
LIB_PATH = os.environ.get("ALVRL_LIB") or os.path.join(PKG_DIR, "libalvrl.so")   # ALVRL_LIB: developer variant builds

REC_WORDS = 20
REC_HIT, REC_SMOOTH, REC_MEDIUM, REC_DELTA, REC_ACCUM = 1, 2, 4, 8, 16   # alvrl_gather_rec.flags
UINT32_MAX = 0xFFFFFFFF

ALVRL_OK = 0
ALVRL_ERR_INVALID, ALVRL_ERR_STATE, ALVRL_ERR_HIP, ALVRL_ERR_NOMEM, ALVRL_ERR_NUMERIC, ALVRL_ERR_COMM = 1, 2, 3, 4, 5, 6
ERRORS = {1: "INVALID", 2: "STATE", 3: "HIP", 4: "NOMEM", 5: "NUMERIC", 6: "COMM"}


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
                ("sampling_weight", C.c_float), ("phase_type", C.c_int), ("phase_g", C.c_float),
                ("strategy", C.c_int), ("channel", C.c_int), ("sampling_density", C.c_float)]


# HomogeneousMedium "strategy" (alvrl_medium_desc.strategy)
STRATEGIES = {"balance": 0, "single": 1, "manual": 2, "maximum": 3}


class ClusterJob(C.Structure):
    _fields_ = [("rows", C.POINTER(C.c_uint32)), ("locw", C.POINTER(C.c_double)),
                ("nrows", C.c_uint32), ("pixel_undersampling", C.c_float),
                ("undersampling", C.c_float), ("depth_correction", C.c_float),
                ("do_refine", C.c_int), ("stage_refine", C.c_uint32), ("stage_sample", C.c_uint32),
                ("row_off", C.POINTER(C.c_uint64)), ("row_stride", C.POINTER(C.c_uint32))]


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
    L.alvrl_set_occluders.argtypes = [vp, vp, u32]
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
    L.alvrl_last_refine_entries.argtypes = [vp, P(u64)]
    L.alvrl_last_refine_split_entries.argtypes = [vp, P(u64)]
    L.alvrl_set_rsamples.argtypes = [vp, i32]
    L.alvrl_build_R_blocks.argtypes = [vp, vp, vp, u32, vp, vp, vp, vp, vp]
    L.alvrl_refine_members.argtypes = [vp, vp, u64, P(ClusterJob), P(u32), P(u32), u32, P(u32), P(u32),
                                       P(u32), P(i32), vp]
    L.alvrl_get_stats.argtypes = [vp, P(u64), P(u64)]
    L.alvrl_reset_stats.argtypes = [vp]
    L.alvrl_gather_brute_host.argtypes = [vp, vp, vp, u32, vp]
    L.alvrl_gather_clustered_host.argtypes = [vp, vp, vp, vp, u32, vp]
    L.alvrl_last_kernel_ms.argtypes = [vp, P(f32)]
    L.alvrl_nonzero_columns.argtypes = [vp, vp, u64, u32, vp, vp]
    L.alvrl_accumulate_rgb.argtypes = [vp, vp, vp, u32, vp, vp]
    L.alvrl_set_strict_rbuild.argtypes = [vp, i32]
    L.alvrl_host_batch_stats.argtypes = [vp, P(u64), P(u64)]
    L.alvrl_detmath_eval.argtypes = [i32, vp, vp, u32, vp]
    L.alvrl_detmath_exhaustive.argtypes = [i32, u64, u64, P(u64), P(u32), u32]
    L.alvrl_detmath_div_check.argtypes = [u64, u64, P(u64), P(u32), u32]
    _lib = L
    return L


def build_info() -> dict:
    """The loaded library's build id and whether its source hash matches the
    sources in this tree (Makefile SRC_HASH): {"library", "build_id",
    "src_hash_tree", "matches_tree"}."""
    import glob
    import hashlib
    L = lib()
    if hasattr(L, "alvrl_build_id"):
        L.alvrl_build_id.restype = C.c_char_p
        bid = L.alvrl_build_id().decode()
    else:                                   # a developer variant built before the id existed
        bid = "unknown"
    os_ = os.path
    rel = []
    for pat in ("csrc/*.hip", "csrc/*.hpp", "csrc/*.h", "csrc/host/*.cpp", "csrc/host/*.hpp", "../include/*.h"):
        rel += [os_.relpath(p, PKG_DIR) for p in glob.glob(os_.join(PKG_DIR, pat))]
    h = hashlib.sha1()
    for r in sorted(rel):
        with open(os_.join(PKG_DIR, r), "rb") as f:
            h.update(f.read())
    tree = h.hexdigest()[:16]
    return {"library": os_.relpath(LIB_PATH, REPO), "build_id": bid, "src_hash_tree": tree,
            "matches_tree": bid.split()[1] == tree if bid.startswith("src ") else False}


DETMATH_FNS = ("exp", "log", "atan", "tan", "asinh", "sinh")


def detmath_eval(fn: str, d_in, d_out, stream=None):
    """csrc/detmath.h's float function `fn` on the device, elementwise over
    float32 CUDA tensors (alvrl_detmath_eval)."""
    _check(lib().alvrl_detmath_eval(DETMATH_FNS.index(fn), _ptr(d_in), _ptr(d_out), int(d_in.numel()),
                                    C.c_void_p(stream) if stream else None))


def detmath_fast_eval(fn: str, d_in, d_out, stream=None):
    """The strict kernels' fast form of detmath.h's `fn` (csrc/detmath_fast.h,
    fn in exp/atan/tan/asinh/sinh) on the device, elementwise."""
    _check(lib().alvrl_detmath_eval(8 + DETMATH_FNS.index(fn), _ptr(d_in), _ptr(d_out), int(d_in.numel()),
                                    C.c_void_p(stream) if stream else None))


def detmath_exhaustive(fn: str, begin: int = 0, end: int = 1 << 32):
    """detmath_fast.h against detmath.h on every float bit pattern in
    [begin, end) (alvrl_detmath_exhaustive): (number of inputs whose results
    differ, some of those inputs as uint32 bit patterns)."""
    mism = C.c_uint64(0)
    first = (C.c_uint32 * 16)()
    _check(lib().alvrl_detmath_exhaustive({"sqrt": 6, "rcp": 7}[fn] if fn in ("sqrt", "rcp") else DETMATH_FNS.index(fn), int(begin), int(end), C.byref(mism), first, 16))
    return int(mism.value), [int(x) for x in first if x != 0xFFFFFFFF]


def detmath_div_check(n: int, seed: int = 1):
    """The strict kernels' fast division against IEEE division on n random
    operand pairs (alvrl_detmath_div_check): (mismatches, [(a_bits, b_bits)])."""
    mism = C.c_uint64(0)
    first = (C.c_uint32 * 16)()
    _check(lib().alvrl_detmath_div_check(int(n), int(seed), C.byref(mism), first, 16))
    pairs = [(int(first[2 * k]), int(first[2 * k + 1])) for k in range(8) if first[2 * k] != 0xFFFFFFFF]
    return int(mism.value), pairs


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
    strategy: str = "balance"      # "balance" | "single" | "manual" | "maximum"
    channel: int = -1              # 'single': the channel (-1: the smallest sigma_t)
    sampling_density: float = 0.0  # 'manual': samplingDensity

    def desc(self) -> "MediumDesc":
        return MediumDesc((C.c_float * 3)(*self.sigma_s), (C.c_float * 3)(*self.sigma_a),
                          self.sampling_weight, self.phase_type, self.phase_g,
                          STRATEGIES[self.strategy], self.channel + 1, self.sampling_density)


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

    @classmethod
    def borrow(cls, handle, device: int = 0) -> "Context":
        """A non-owning view of a context another object owns (alvrl_integrator_ctx)."""
        c = cls.__new__(cls)
        c.L, c.h, c.device, c.nvrl, c.particle_count, c._borrowed = lib(), handle, device, 0, 0, True
        return c

    def close(self):
        if getattr(self, "_borrowed", False):
            self.h = None
            return
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
        d = m.desc()
        _check(self.L.alvrl_set_medium(self.h, C.byref(d)))

    def set_pass(self, p: int):
        _check(self.L.alvrl_set_pass(self.h, p))

    def set_occluders(self, tris, material=None):
        """Occluder triangles ((n, 9) float32) blocking the gathers' connections;
        material: None or one MAT_* per triangle (MAT_NULL ones let them pass)."""
        arr = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
        mat = None if material is None else np.ascontiguousarray(
            np.broadcast_to(np.asarray(material, np.uint32), (len(arr),)))
        _check(self.L.alvrl_set_occluders(self.h, _ptr(arr) if len(arr) else None, len(arr), _ptr(mat)))

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

    def set_rsamples(self, n: int):
        _check(self.L.alvrl_set_rsamples(self.h, n))

    def host_batch_stats(self) -> dict:
        """Launches of the host-pointer gathers and the requests they carried
        (concurrent calls are merged, alvrl_host_batch_stats)."""
        b = (C.c_uint64 * 2)(); r = (C.c_uint64 * 2)()
        _check(self.L.alvrl_host_batch_stats(self.h, b, r))
        return {"brute": (int(b[0]), int(r[0])), "clustered": (int(b[1]), int(r[1]))}

    def set_strict_rbuild(self, on: bool = True):
        """The R build in the oracle's arithmetic (alvrl_set_strict_rbuild): R
        entries equal the CPU restatement's bit for bit."""
        _check(self.L.alvrl_set_strict_rbuild(self.h, int(bool(on))))

    def build_R_blocks(self, d_recs, d_Rt, d_row_off, d_row_stride, d_nonzero=None, d_ids=None,
                       stream=None):
        """Rows scattered over per-slice blocks: row r's pair for VRL v at float2
        index row_off[r] + v * row_stride[r] (alvrl_build_R_blocks)."""
        n = int(d_recs.shape[0])
        _check(self.L.alvrl_build_R_blocks(self.h, _ptr(d_recs), _ptr(d_ids), n, _ptr(d_Rt),
                                           _ptr(d_row_off), _ptr(d_row_stride), _ptr(d_nonzero),
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

    def refine_members(self, d_Rt, ld: int, job: dict, init_vrls, init_off, stream=None):
        """clusterRefinement + getVrlsPerCluster (alvrl_refine_members):
        (member ids, cluster offsets, refined)."""
        rows = _np(job["rows"], np.uint32); lw = _np(job["locw"], np.float64)
        cj = ClusterJob(_arr(rows, C.c_uint32), _arr(lw, C.c_double), len(rows),
                        job["pixel_undersampling"], job["undersampling"], 1.0, 1,
                        job.get("stage_refine", 0xFFFFFFFE), job.get("stage_refine", 0xFFFFFFFE))
        iv = _np(init_vrls, np.uint32); io = _np(init_off, np.uint32)
        nv = int(io[-1])
        mem = np.zeros(max(1, nv), np.uint32); off = np.zeros(nv + 2, np.uint32)
        nc = C.c_uint32(); ok = C.c_int()
        _check(self.L.alvrl_refine_members(self.h, _ptr(d_Rt), ld, C.byref(cj), _arr(iv, C.c_uint32),
                                           _arr(io, C.c_uint32), len(io) - 1, _arr(mem, C.c_uint32),
                                           _arr(off, C.c_uint32), C.byref(nc), C.byref(ok),
                                           C.c_void_p(stream) if stream else None))
        return mem[:nv].copy(), off[:nc.value + 1].copy(), bool(ok.value)

    def last_refine_ms(self) -> float:
        ms = C.c_float()
        _check(self.L.alvrl_last_refine_ms(self.h, C.byref(ms)))
        return ms.value

    def last_refine_entries(self) -> int:
        n = C.c_uint64()
        _check(self.L.alvrl_last_refine_entries(self.h, C.byref(n)))
        return int(n.value)

    def last_refine_split_entries(self) -> int:
        """The splits' share of last_refine_entries (each split reads it three times)."""
        n = C.c_uint64()
        _check(self.L.alvrl_last_refine_split_entries(self.h, C.byref(n)))
        return int(n.value)

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

    def nonzero_columns(self, d_Rt, ld: int, nrows: int) -> np.ndarray:
        mask = np.zeros(max(1, self.nvrl), np.uint8)
        _check(self.L.alvrl_nonzero_columns(self.h, _ptr(d_Rt), ld, nrows, _ptr(mask), None))
        return mask[:self.nvrl].astype(bool)

    def accumulate_rgb(self, d_rgb, d_pixel, d_fb, stream=None):
        _check(self.L.alvrl_accumulate_rgb(self.h, _ptr(d_rgb), _ptr(d_pixel), d_pixel.shape[0],
                                           _ptr(d_fb), C.c_void_p(stream) if stream else None))

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


# ---------------------------------------------------------------------------
# host harness (include/alvrl_host.h)
# ---------------------------------------------------------------------------
class SceneDesc(C.Structure):
    _fields_ = [("cam_origin", C.c_float * 3), ("cam_target", C.c_float * 3), ("cam_up", C.c_float * 3),
                ("fov_x_deg", C.c_float), ("width", C.c_int), ("height", C.c_int),
                ("box_min", C.c_float * 3), ("box_max", C.c_float * 3), ("albedo", C.c_float * 3),
                ("light_pos", C.c_float * 3), ("light_intensity", C.c_float * 3),
                ("medium", MediumDesc), ("occluders", C.POINTER(C.c_float)), ("n_occluders", C.c_uint32),
                ("occluder_albedo", C.c_float * 3), ("occluder_material", C.POINTER(C.c_uint32)),
                ("occluder_specular", C.c_float * 3), ("occluder_eta", C.c_float),
                ("emitter_tris", C.POINTER(C.c_float)), ("n_emitter_tris", C.c_uint32),
                ("emitter_radiance", C.c_float * 3), ("occluder_albedos", C.POINTER(C.c_float))]


MAT_DIFFUSE, MAT_MIRROR, MAT_NULL, MAT_DIELECTRIC = 0, 1, 2, 3


class SceneExt(C.Structure):
    """alvrl_scene_ext: a host-cast scene (the Mitsuba plugin's records mode)."""
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("scene_min", C.c_float * 3),
                ("scene_max", C.c_float * 3), ("medium", MediumDesc), ("slice_recs", C.c_void_p),
                ("triangles", C.c_void_p), ("n_triangles", C.c_uint32), ("triangle_material", C.c_void_p),
                ("tracer", C.POINTER(SceneDesc))]


class IntegratorStats(C.Structure):
    _fields_ = [("vrls", C.c_uint64), ("particles", C.c_uint64), ("slices", C.c_uint64),
                ("rep_rows", C.c_uint64), ("clusters_total", C.c_uint64),
                ("contrib_preprocess", C.c_uint64), ("contrib_render", C.c_uint64),
                ("ms_trace", C.c_double), ("ms_slices", C.c_double), ("ms_rbuild", C.c_double),
                ("ms_refine", C.c_double), ("ms_render_kernel", C.c_double),
                ("ms_prepass_wall", C.c_double), ("slices_failed", C.c_uint32),
                ("fallback_built", C.c_int), ("slices_local", C.c_uint64), ("rows_built", C.c_uint64),
                ("ms_exchange", C.c_double), ("ms_refine_kernel", C.c_double),
                ("refine_entries", C.c_uint64), ("global_clusters", C.c_uint64),
                ("refine_split_entries", C.c_uint64), ("ms_alloc", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p)


class ExchangeDesc(C.Structure):
    _fields_ = [("user", C.c_void_p), ("allgather", ALLGATHER_FN)]


class LocalExchange:
    """alvrl_local_exchange: ranks that are threads of this process (one
    Integrator per device, each driven by its own thread).  `rank(r)` is the
    exchange to pass to rank r's Integrator.prepass."""

    class _Rank:
        def __init__(self, owner, desc):
            self.owner, self.desc, self.error, self.world = owner, desc, None, owner.world

        def _check(self, rc: int):
            if rc != ALVRL_OK:
                raise AlvrlError(rc, _host().alvrl_host_last_error().decode())

        def allgatherv(self, data):
            return Exchange.allgatherv(self, data)

        def or_(self, mask):
            return Exchange.or_(self, mask)

    def __init__(self, world: int):
        L = _host()
        h = C.c_void_p()
        rc = L.alvrl_local_exchange_create(world, C.byref(h))
        if rc != ALVRL_OK:
            raise AlvrlError(rc, L.alvrl_host_last_error().decode())
        self.h, self.world = h, world
        self._ranks = [self._Rank(self, C.cast(L.alvrl_local_exchange_rank(h, r), C.POINTER(ExchangeDesc)).contents)
                       for r in range(world)]

    def rank(self, r: int) -> "LocalExchange._Rank":
        return self._ranks[r]

    def close(self):
        if getattr(self, "h", None):
            _host().alvrl_local_exchange_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceExchange(LocalExchange):
    """alvrl_device_exchange: ranks that are the GPUs of this process over
    RCCL (one communicator per device, ncclCommInitAll; distinct devices).
    `rank(r)` is rank r's exchange; `reduce_frame(r, d_fb)` sums every rank's
    framebuffer into rank 0's (one ncclReduce, each rank calls it)."""

    def __init__(self, devices):
        L = _host()
        h = C.c_void_p()
        devs = np.asarray(list(devices), np.int32)
        rc = L.alvrl_device_exchange_create(_ptr(devs), len(devs), C.byref(h))
        if rc != ALVRL_OK:
            raise AlvrlError(rc, L.alvrl_host_last_error().decode())
        self.h, self.world, self.devices = h, len(devs), [int(d) for d in devs]
        self._ranks = [self._Rank(self, C.cast(L.alvrl_device_exchange_rank(h, r), C.POINTER(ExchangeDesc)).contents)
                       for r in range(self.world)]

    def reduce_frame(self, rank: int, d_fb, stream=None):
        _hcheck(_host().alvrl_device_exchange_reduce_frame(self.h, rank, _ptr(d_fb), d_fb.numel(),
                                                           C.c_void_p(stream) if stream else None))

    def close(self):
        if getattr(self, "h", None):
            _host().alvrl_device_exchange_destroy(self.h)
            self.h = None


class Exchange:
    """alvrl_exchange over a torch.distributed process group.

    The library asks for one collective: a fixed-size all-gather of bytes.  With
    the "nccl" backend (RCCL on ROCm) the bytes travel as a device tensor over
    xGMI; with gloo (CPU tests) as a host tensor.  A failing collective is kept
    in `error` and reported to the library as a non-zero status, which aborts the
    prepass with ALVRL_ERR_COMM."""

    def __init__(self, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        if device is None:
            device = (torch.device("cuda", torch.cuda.current_device())
                      if dist.get_backend(group) == "nccl" else torch.device("cpu"))
        self.device = device
        self.error = None
        self.calls = 0

        def allgather(user, send, nbytes, recv):
            try:
                n = int(nbytes)
                src = np.frombuffer((C.c_uint8 * n).from_address(send), np.uint8).copy()
                t = torch.from_numpy(src).to(self.device)
                out = torch.empty(n * self.world, dtype=torch.uint8, device=self.device)
                dist.all_gather_into_tensor(out, t, group=self.group)
                host = out.cpu().numpy()
                C.memmove(recv, host.ctypes.data, host.nbytes)
                self.calls += 1
                return 0
            except Exception as e:   # reported to the library as ALVRL_ERR_COMM
                self.error = e
                return 1

        self._fn = ALLGATHER_FN(allgather)   # keep the thunk alive
        self.desc = ExchangeDesc(None, self._fn)

    def _check(self, rc: int):
        if rc != ALVRL_OK:
            raise AlvrlError(rc, _host().alvrl_host_last_error().decode()
                             + (f" ({self.error!r})" if self.error else ""))

    def allgatherv(self, data: np.ndarray) -> list:
        """Variable-size all-gather of a uint8 array: one array per rank."""
        L = _host()
        data = _np(data, np.uint8)
        counts = np.zeros(self.world, np.uint64)
        self._check(L.alvrl_exchange_allgatherv(C.byref(self.desc), self.world, _ptr(data), data.size,
                                                None, 0, _arr(counts, C.c_uint64)))
        out = np.zeros(max(1, int(counts.sum())), np.uint8)
        self._check(L.alvrl_exchange_allgatherv(C.byref(self.desc), self.world, _ptr(data), data.size,
                                                _ptr(out), out.size, _arr(counts, C.c_uint64)))
        ends = np.cumsum(counts.astype(np.int64))
        return [out[e - int(c):e].copy() for e, c in zip(ends, counts)]

    def or_(self, mask: np.ndarray) -> np.ndarray:
        m = _np(mask, np.uint8).copy()
        self._check(_host().alvrl_exchange_or(C.byref(self.desc), self.world, _ptr(m), m.size))
        return m

    def clusters(self, nslices: int, local: dict):
        """Merge {slice: (refined, reps, weights)} of every rank into the CSR
        over all slices: (refined[nslices], slice_off, reps, weights)."""
        L = _host()
        ids = np.array(sorted(local), np.uint32)
        ref = np.array([int(bool(local[s][0])) for s in ids], np.int32)
        off = np.zeros(len(ids) + 1, np.uint32)
        for k, s in enumerate(ids):
            off[k + 1] = off[k] + len(local[s][1])
        reps = np.concatenate([np.asarray(local[s][1], np.uint32) for s in ids] or [np.zeros(0, np.uint32)])
        w = np.concatenate([np.asarray(local[s][2], np.float32) for s in ids] or [np.zeros(0, np.float32)])
        refined = np.zeros(max(1, nslices), np.int32)
        soff = np.zeros(nslices + 1, np.uint32)
        total = C.c_uint64()
        cap = 0
        while True:
            out_r = np.zeros(max(1, cap), np.uint32); out_w = np.zeros(max(1, cap), np.float32)
            rc = L.alvrl_exchange_clusters(C.byref(self.desc), self.world, nslices, len(ids), _ptr(ids),
                                           _ptr(ref), _ptr(off), _ptr(reps), _ptr(w), _ptr(refined),
                                           _ptr(soff), _ptr(out_r), _ptr(out_w), cap, C.byref(total))
            if rc == ALVRL_OK:
                return refined[:nslices], soff, out_r[:total.value], out_w[:total.value]
            if total.value <= cap:
                self._check(rc)
            cap = int(total.value)


_host_bound = False


def _host():
    global _host_bound
    L = lib()
    if _host_bound:
        return L
    u32, u64, i32, f32, vp = C.c_uint32, C.c_uint64, C.c_int, C.c_float, C.c_void_p
    P = C.POINTER
    L.alvrl_scene_default.argtypes = [P(SceneDesc), i32, i32]; L.alvrl_scene_default.restype = None
    L.alvrl_scene_records.argtypes = [P(SceneDesc), i32, vp, u32, vp]
    L.alvrl_scene_chain.argtypes = [P(SceneDesc), i32, u32, u32, i32, f32, i32, i32, vp, u32, P(u32)]
    L.alvrl_scene_slice_record.argtypes = [P(SceneDesc), i32, i32, vp]
    L.alvrl_trace_vrls.argtypes = [P(SceneDesc), u32, u32, u32, i32, i32, i32, vp, u32, P(u32), P(u64)]
    L.alvrl_trace_vrls_gpu.argtypes = [P(SceneDesc), u32, u32, u32, i32, i32, i32, vp, u32, P(u32), P(u64)]
    L.alvrl_scene_records_gpu.argtypes = [P(SceneDesc), i32, vp, u32, vp, vp]
    L.alvrl_scene_records_spp.argtypes = [P(SceneDesc), i32, u32, u32, u32, vp, u32, vp]
    L.alvrl_scene_records_spp_gpu.argtypes = [P(SceneDesc), i32, u32, u32, u32, vp, u32, vp, vp]
    L.alvrl_scene_chain_spp.argtypes = [P(SceneDesc), i32, u32, u32, i32, f32, i32, i32, u32, u32, vp, u32, P(u32)]
    L.alvrl_volpath_default.argtypes = [P(VolpathParams)]; L.alvrl_volpath_default.restype = None
    L.alvrl_volpath_render.argtypes = [P(SceneDesc), P(VolpathParams), u32, u32, u32, vp, u32, vp, vp]
    L.alvrl_read_vrl_file.argtypes = [C.c_char_p, P(MediumDesc), vp, u32, P(u32), P(u64)]
    L.alvrl_write_vrl_file.argtypes = [C.c_char_p, vp, u32]
    L.alvrl_tile_pixels.argtypes = [i32, i32, u32, u32, vp, u32, P(u32)]
    L.alvrl_host_last_error.restype = C.c_char_p
    L.alvrl_integrator_create.argtypes = [C.c_char_p, i32, P(vp)]
    L.alvrl_integrator_destroy.argtypes = [vp]; L.alvrl_integrator_destroy.restype = None
    L.alvrl_integrator_preprocess.argtypes = [vp, P(SceneDesc)]
    L.alvrl_integrator_prepass.argtypes = [vp, u32]
    L.alvrl_integrator_render.argtypes = [vp, u32, u32, vp, vp]
    L.alvrl_integrator_set_vrls.argtypes = [vp, vp, u32, u64]
    L.alvrl_integrator_get_stats.argtypes = [vp, P(IntegratorStats)]
    L.alvrl_integrator_ctx.argtypes = [vp]; L.alvrl_integrator_ctx.restype = vp
    L.alvrl_integrator_slices.argtypes = [vp, P(u32), u32]
    L.alvrl_integrator_num_slices.argtypes = [vp]; L.alvrl_integrator_num_slices.restype = u32
    L.alvrl_integrator_reps.argtypes = [vp, P(u32), P(u32), u32]
    L.alvrl_integrator_clusters.argtypes = [vp, P(u32), P(u32), P(f32), u32, P(u32), P(f32), u32, P(u32)]
    L.alvrl_integrator_vrls.argtypes = [vp, vp, u32, P(u32), P(u64)]
    L.alvrl_integrator_R.argtypes = [vp, vp, u64]
    L.alvrl_integrator_slice_job.argtypes = [vp, u32, vp, vp, u32, P(u32), P(f32), vp, vp, P(u32)]
    L.alvrl_integrator_prepass_dist.argtypes = [vp, u32, u32, u32, P(ExchangeDesc)]
    L.alvrl_exchange_allgatherv.argtypes = [P(ExchangeDesc), u32, vp, u64, vp, u64, P(u64)]
    L.alvrl_exchange_or.argtypes = [P(ExchangeDesc), u32, vp, u64]
    L.alvrl_local_exchange_create.argtypes = [u32, P(vp)]
    L.alvrl_local_exchange_rank.argtypes = [vp, u32]; L.alvrl_local_exchange_rank.restype = vp
    L.alvrl_local_exchange_destroy.argtypes = [vp]; L.alvrl_local_exchange_destroy.restype = None
    L.alvrl_integrator_local_slices.argtypes = [vp, vp, u32, P(u32)]
    L.alvrl_device_exchange_create.argtypes = [vp, u32, P(vp)]
    L.alvrl_device_exchange_rank.argtypes = [vp, u32]; L.alvrl_device_exchange_rank.restype = vp
    L.alvrl_device_exchange_reduce_frame.argtypes = [vp, u32, vp, u64, vp]
    L.alvrl_device_exchange_destroy.argtypes = [vp]; L.alvrl_device_exchange_destroy.restype = None
    L.alvrl_exchange_clusters.argtypes = [P(ExchangeDesc), u32, u32, u32, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                          u64, P(u64)]
    L.alvrl_cluster_info_write.argtypes = [C.c_char_p, u32, vp, u32, vp, vp, vp, u32, vp, vp, u32, vp, vp]
    L.alvrl_cluster_info_read.argtypes = [C.c_char_p, P(vp)]
    L.alvrl_cluster_info_free.argtypes = [vp]; L.alvrl_cluster_info_free.restype = None
    L.alvrl_cluster_info_sizes.argtypes = [vp, P(u32), P(u32), P(u32), P(u32), P(u32)]
    L.alvrl_cluster_info_get.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.alvrl_integrator_save_cluster_info.argtypes = [vp, C.c_char_p]
    L.alvrl_integrator_load_cluster_info.argtypes = [vp, C.c_char_p, u32]
    L.alvrl_write_exr.argtypes = [C.c_char_p, vp, i32, i32, i32]
    L.alvrl_read_exr.argtypes = [C.c_char_p, vp, u64, P(i32), P(i32)]
    L.alvrl_image_rms.argtypes = [vp, vp, u64, C.c_double, C.c_double, i32, P(C.c_double)]
    L.alvrl_pass_file_name.argtypes = [C.c_char_p, u64, C.c_char_p, i32] + [C.c_double] * 6
    L.alvrl_integrator_preprocess_ext.argtypes = [vp, P(SceneExt)]
    L.alvrl_integrator_rep_pixels.argtypes = [vp, u32, vp, u32, P(u32)]
    L.alvrl_integrator_prepass_records.argtypes = [vp, u32, vp, vp, u32, u32, u32, P(ExchangeDesc)]
    L.alvrl_integrator_set_cluster_info.argtypes = [vp, u32, u32, vp, u32, vp, vp, vp, u32, vp, vp]
    _host_bound = True
    return L


def _hcheck(rc: int):
    if rc != ALVRL_OK:
        raise AlvrlError(rc, _host().alvrl_host_last_error().decode())


def scene_default(width: int, height: int) -> SceneDesc:
    s = SceneDesc()
    _host().alvrl_scene_default(C.byref(s), width, height)
    return s


def scene_set_area_emitter(scene: SceneDesc, tris, radiance) -> SceneDesc:
    """An area emitter replacing the point light (alvrl_scene_desc.emitter_tris):
    (n, 9) triangles emitting `radiance` on the side of cross(p1 - p0, p2 - p0).
    The array is kept alive on the descriptor."""
    arr = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
    scene._emit_keep = arr
    scene.emitter_tris = arr.ctypes.data_as(C.POINTER(C.c_float)) if len(arr) else None
    scene.n_emitter_tris = len(arr)
    for i in range(3):
        scene.emitter_radiance[i] = float(radiance[i])
    return scene


def scene_set_occluders(scene: SceneDesc, tris, albedo=(0.5, 0.5, 0.5), material=None,
                        specular=(1.0, 1.0, 1.0), eta=None, albedos=None) -> SceneDesc:
    """Occluder triangles inside the box (alvrl_scene_desc.occluders): an
    (n, 9) float array of (p0, p1, p2), face normal cross(p1 - p0, p2 - p0);
    material: None (all diffuse) or one MAT_* per triangle; specular: the
    mirrors' reflectance; eta: the dielectrics' intIOR / extIOR (None: the
    default bk7 / air); albedos: (n, 3) per-triangle diffuse reflectances
    (occluder_albedos, replacing albedo).  The arrays are kept alive on the
    descriptor."""
    if eta is not None:
        scene.occluder_eta = float(eta)
    arr = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
    scene._occ_keep = arr
    scene.occluders = arr.ctypes.data_as(C.POINTER(C.c_float)) if len(arr) else None
    scene.n_occluders = len(arr)
    for i in range(3):
        scene.occluder_albedo[i] = float(albedo[i])
        scene.occluder_specular[i] = float(specular[i])
    if material is None:
        scene.occluder_material = None
    else:
        mat = np.ascontiguousarray(np.broadcast_to(np.asarray(material, np.uint32), (len(arr),)))
        scene._mat_keep = mat
        scene.occluder_material = mat.ctypes.data_as(C.POINTER(C.c_uint32))
    if albedos is None:
        scene.occluder_albedos = None
    else:
        alb = np.ascontiguousarray(np.asarray(albedos, np.float32).reshape(len(arr), 3))
        scene._alb_keep = alb
        scene.occluder_albedos = alb.ctypes.data_as(C.POINTER(C.c_float))
    return scene


def box_mesh(lo, hi) -> np.ndarray:
    """12 triangles of an axis-aligned box [lo, hi] with outward face normals."""
    lo = np.asarray(lo, np.float32)
    hi = np.asarray(hi, np.float32)
    c = np.array([[lo[0] if i & 1 == 0 else hi[0], lo[1] if i & 2 == 0 else hi[1],
                   lo[2] if i & 4 == 0 else hi[2]] for i in range(8)], np.float32)
    quads = [(0, 2, 6, 4), (1, 5, 7, 3), (0, 4, 5, 1), (2, 3, 7, 6), (0, 1, 3, 2), (4, 6, 7, 5)]
    tris = []
    for a, b, cc, d in quads:   # outward: x-, x+, y-, y+, z-, z+
        tris.append(np.concatenate([c[a], c[cc], c[b]]))
        tris.append(np.concatenate([c[a], c[d], c[cc]]))
    return np.asarray(tris, np.float32)


def scene_records(scene: SceneDesc, pixel_ids=None, medium_scatters: bool = True) -> np.ndarray:
    L = _host()
    n = scene.width * scene.height if pixel_ids is None else len(pixel_ids)
    out = np.zeros((n, REC_WORDS), np.float32)
    ids = None if pixel_ids is None else _np(pixel_ids, np.uint32)
    _hcheck(L.alvrl_scene_records(C.byref(scene), int(medium_scatters), _ptr(ids), n, _ptr(out)))
    return out


def scene_chain(scene: SceneDesc, x: int, y: int, medium_scatters: bool = True, seed: int = 0xA1B2C3D4,
                pass_: int = 0, spec_rr_depth: int = 100, init_throughput: float = 20.0) -> np.ndarray:
    """alvrl_scene_chain: LiInternal's eye path of pixel (x, y), (k, REC_WORDS)."""
    L = _host()
    out = np.zeros((256, REC_WORDS), np.float32)
    n = C.c_uint32()
    _hcheck(L.alvrl_scene_chain(C.byref(scene), int(medium_scatters), seed, pass_, spec_rr_depth,
                                float(init_throughput), x, y, _ptr(out), 256, C.byref(n)))
    return out[:n.value].copy()


def scene_records_spp(scene: SceneDesc, spp: int, pixel_ids=None, medium_scatters: bool = True,
                      seed: int = 0xA1B2C3D4, pass_: int = 0) -> np.ndarray:
    """alvrl_scene_records_spp: the records of spp sensor samples per pixel,
    sample major ((spp * n, REC_WORDS); record j * n + i = pixel i, sample j)."""
    L = _host()
    n = scene.width * scene.height if pixel_ids is None else len(pixel_ids)
    out = np.zeros((spp * n, REC_WORDS), np.float32)
    ids = None if pixel_ids is None else _np(pixel_ids, np.uint32)
    _hcheck(L.alvrl_scene_records_spp(C.byref(scene), int(medium_scatters), seed, pass_, spp, _ptr(ids), n,
                                      _ptr(out)))
    return out


def scene_chain_spp(scene: SceneDesc, x: int, y: int, sample: int, spp: int, medium_scatters: bool = True,
                    seed: int = 0xA1B2C3D4, pass_: int = 0, spec_rr_depth: int = 100,
                    init_throughput: float = 20.0) -> np.ndarray:
    """alvrl_scene_chain_spp: the eye path of sensor sample `sample` of `spp`."""
    L = _host()
    out = np.zeros((256, REC_WORDS), np.float32)
    n = C.c_uint32()
    _hcheck(L.alvrl_scene_chain_spp(C.byref(scene), int(medium_scatters), seed, pass_, spec_rr_depth,
                                    float(init_throughput), x, y, sample, spp, _ptr(out), 256, C.byref(n)))
    return out[:n.value].copy()


def scene_slice_record(scene: SceneDesc, x: int, y: int) -> np.ndarray:
    L = _host()
    out = np.zeros(REC_WORDS, np.float32)
    _hcheck(L.alvrl_scene_slice_record(C.byref(scene), x, y, _ptr(out)))
    return out


def trace_vrls(scene: SceneDesc, target: int, seed: int = 0x5EED0001, pass_: int = 0,
               short_vrls: bool = True, max_depth: int = -1, rr_depth: int = 5):
    L = _host()
    cap = target + 8192
    soa = np.zeros((9, cap), np.float32)
    n = C.c_uint32(); pc = C.c_uint64()
    _hcheck(L.alvrl_trace_vrls(C.byref(scene), seed, pass_, target, int(short_vrls), max_depth,
                               rr_depth, _ptr(soa), cap, C.byref(n), C.byref(pc)))
    return np.ascontiguousarray(soa[:, :n.value]), int(pc.value)


def scene_records_gpu(scene: SceneDesc, pixel_ids=None, medium_scatters: bool = True, device: int = 0):
    """alvrl_scene_records_gpu: the records on the HIP device (a CUDA tensor)."""
    import torch
    L = _host()
    dev = torch.device("cuda", device)
    n = scene.width * scene.height if pixel_ids is None else len(pixel_ids)
    out = torch.empty((n, REC_WORDS), dtype=torch.float32, device=dev)
    ids = None if pixel_ids is None else torch.as_tensor(np.asarray(pixel_ids, np.uint32).astype(np.int32)).to(dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _hcheck(L.alvrl_scene_records_gpu(C.byref(scene), int(medium_scatters),
                                          None if ids is None else ids.data_ptr(), n, out.data_ptr(), stream))
    return out


def scene_records_spp_gpu(scene: SceneDesc, spp: int, pixel_ids=None, medium_scatters: bool = True,
                          seed: int = 0xA1B2C3D4, pass_: int = 0, device: int = 0):
    """alvrl_scene_records_spp_gpu: scene_records_spp on the HIP device (a CUDA tensor)."""
    import torch
    L = _host()
    dev = torch.device("cuda", device)
    n = scene.width * scene.height if pixel_ids is None else len(pixel_ids)
    out = torch.empty((spp * n, REC_WORDS), dtype=torch.float32, device=dev)
    ids = None if pixel_ids is None else torch.as_tensor(np.asarray(pixel_ids, np.uint32).astype(np.int32)).to(dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _hcheck(L.alvrl_scene_records_spp_gpu(C.byref(scene), int(medium_scatters), seed, pass_, spp,
                                              None if ids is None else ids.data_ptr(), n, out.data_ptr(), stream))
    return out


class VolpathParams(C.Structure):
    _fields_ = [("max_depth", C.c_int), ("rr_depth", C.c_int), ("only_vrl_paths", C.c_int),
                ("vrl_vol_to_vol", C.c_int), ("vrl_vol_to_surf", C.c_int)]


def volpath_render(scene: SceneDesc, spp: int, seed: int = 0xA1B2C3D4, pass_: int = 0, pixel_ids=None,
                   device: int = 0, **params):
    """alvrl_volpath_render: the volpath onlyVRLpaths reference image (a CUDA
    tensor (n, 3), means over spp); params: max_depth, rr_depth,
    only_vrl_paths, vrl_vol_to_vol, vrl_vol_to_surf."""
    import torch
    L = _host()
    vp = VolpathParams()
    L.alvrl_volpath_default(C.byref(vp))
    for k, v in params.items():
        setattr(vp, k, int(v))
    dev = torch.device("cuda", device)
    n = scene.width * scene.height if pixel_ids is None else len(pixel_ids)
    out = torch.empty((n, 3), dtype=torch.float32, device=dev)
    ids = None if pixel_ids is None else torch.as_tensor(np.asarray(pixel_ids, np.uint32).astype(np.int32)).to(dev)
    with torch.cuda.device(dev):
        stream = torch.cuda.current_stream(dev).cuda_stream
        _hcheck(L.alvrl_volpath_render(C.byref(scene), C.byref(vp), seed, pass_, spp,
                                       None if ids is None else ids.data_ptr(), n, out.data_ptr(), stream))
    return out


def trace_vrls_gpu(scene: SceneDesc, target: int, seed: int = 0x5EED0001, pass_: int = 0,
                   short_vrls: bool = True, max_depth: int = -1, rr_depth: int = 5):
    """vrlTracer::randomWalk on the current HIP device (same result as trace_vrls)."""
    L = _host()
    n = C.c_uint32(); pc = C.c_uint64()
    _hcheck(L.alvrl_trace_vrls_gpu(C.byref(scene), seed, pass_, target, int(short_vrls), max_depth, rr_depth,
                                   None, 0, C.byref(n), C.byref(pc)))
    cap = max(1, n.value)
    soa = np.zeros((9, cap), np.float32)
    _hcheck(L.alvrl_trace_vrls_gpu(C.byref(scene), seed, pass_, target, int(short_vrls), max_depth, rr_depth,
                                   _ptr(soa), cap, C.byref(n), C.byref(pc)))
    return np.ascontiguousarray(soa[:, :n.value]), int(pc.value)


def tile_pixels(width: int, height: int, rank: int = 0, world: int = 1) -> np.ndarray:
    """Pixel ids (row-major) rendered by `rank` of `world` (64x64 tiles,
    round-robin): the partition alvrl_integrator_render uses."""
    L = _host()
    n = C.c_uint32()
    _hcheck(L.alvrl_tile_pixels(width, height, rank, world, None, 0, C.byref(n)))
    out = np.zeros(max(1, n.value), np.uint32)
    _hcheck(L.alvrl_tile_pixels(width, height, rank, world, _ptr(out), n.value, C.byref(n)))
    return out[:n.value].copy()


def read_vrl_file(path: str, medium: Medium = Medium()):
    L = _host()
    md = medium.desc()
    n = C.c_uint32(); pc = C.c_uint64()
    _hcheck(L.alvrl_read_vrl_file(path.encode(), C.byref(md), None, 0, C.byref(n), C.byref(pc)))
    soa = np.zeros((9, max(1, n.value)), np.float32)
    _hcheck(L.alvrl_read_vrl_file(path.encode(), C.byref(md), _ptr(soa), n.value, C.byref(n),
                                  C.byref(pc)))
    return soa[:, :n.value].copy(), int(pc.value)


def write_vrl_file(path: str, soa: np.ndarray):
    soa = _np(soa, np.float32)
    _hcheck(_host().alvrl_write_vrl_file(path.encode(), _ptr(soa), soa.shape[1]))


def write_cluster_info(path: str, info: dict):
    """vrlClusterInfo stream (vrlIntegrator.cpp:66-101).  info: slices
    (m_slices, y + H*x), slice_off / reps / weights (CSR), optional
    global_reps / global_weights and fb_reps / fb_weights."""
    u = lambda k: _np(info.get(k, np.zeros(0)), np.uint32)
    f = lambda k: _np(info.get(k, np.zeros(0)), np.float32)
    sl, so, rp, w = u("slices"), u("slice_off"), u("reps"), f("weights")
    gr, gw, fr, fw = u("global_reps"), f("global_weights"), u("fb_reps"), f("fb_weights")
    _hcheck(_host().alvrl_cluster_info_write(path.encode(), len(sl), _ptr(sl), max(0, len(so) - 1), _ptr(so),
                                             _ptr(rp), _ptr(w), len(gr), _ptr(gr), _ptr(gw), len(fr),
                                             _ptr(fr), _ptr(fw)))


def read_cluster_info(path: str) -> dict:
    """vrlClusterInfo(Stream*, InstanceManager*) (:29-64, fall-back ids fixed)."""
    L = _host()
    h = C.c_void_p()
    _hcheck(L.alvrl_cluster_info_read(path.encode(), C.byref(h)))
    try:
        n = [C.c_uint32() for _ in range(5)]
        _hcheck(L.alvrl_cluster_info_sizes(h, *[C.byref(x) for x in n]))
        npix, ns, nr, ng, nfb = (x.value for x in n)
        out = {"slices": np.zeros(npix, np.uint32), "slice_off": np.zeros(ns + 1, np.uint32),
               "reps": np.zeros(nr, np.uint32), "weights": np.zeros(nr, np.float32),
               "global_reps": np.zeros(ng, np.uint32), "global_weights": np.zeros(ng, np.float32),
               "fb_reps": np.zeros(nfb, np.uint32), "fb_weights": np.zeros(nfb, np.float32)}
        keys = ("slices", "slice_off", "reps", "weights", "global_reps", "global_weights", "fb_reps", "fb_weights")
        _hcheck(L.alvrl_cluster_info_get(h, *[_ptr(out[k]) if out[k].size else None for k in keys]))
        return out
    finally:
        L.alvrl_cluster_info_free(h)


def write_exr(path: str, rgb: np.ndarray, half: bool = False):
    """Uncompressed scanline OpenEXR, rgb of shape (H, W, 3)."""
    rgb = _np(rgb, np.float32)
    _hcheck(_host().alvrl_write_exr(path.encode(), _ptr(rgb), rgb.shape[1], rgb.shape[0], int(half)))


def read_exr(path: str) -> np.ndarray:
    L = _host()
    w, h = C.c_int(), C.c_int()
    _hcheck(L.alvrl_read_exr(path.encode(), None, 0, C.byref(w), C.byref(h)))
    out = np.zeros((h.value, w.value, 3), np.float32)
    _hcheck(L.alvrl_read_exr(path.encode(), _ptr(out), out.size, C.byref(w), C.byref(h)))
    return out


def image_rms(sample, reference, gamma: float = 1.0, robust_fraction: float = 0.0,
              relative: bool = False) -> float:
    """mtsutil rms (src/utils/rms.cpp)."""
    a, b = _np(sample, np.float32).ravel(), _np(reference, np.float32).ravel()
    if a.size != b.size:
        raise ValueError("images differ in size")
    r = C.c_double()
    _hcheck(_host().alvrl_image_rms(_ptr(a), _ptr(b), a.size, gamma, robust_fraction, int(relative),
                                    C.byref(r)))
    return r.value


def pass_file_name(dest: str, pass_: int, prepass_cpu: float, prepass_wall: float, render_cpu: float,
                   render_wall: float, vrls_preprocess: float, vrls_render: float) -> str:
    """dumpPass file name (integrator.cpp:361-378 + passFileSuffix)."""
    buf = C.create_string_buffer(len(dest) + 256)
    _hcheck(_host().alvrl_pass_file_name(buf, len(buf), dest.encode(), pass_, prepass_cpu, prepass_wall,
                                         render_cpu, render_wall, vrls_preprocess, vrls_render))
    return buf.value.decode()


class Integrator:
    """vrlIntegrator pipeline (preprocess / prepass / render) on one device."""

    def __init__(self, props: str = "", device: int = 0):
        L = _host()
        self.L = L
        h = C.c_void_p()
        _hcheck(L.alvrl_integrator_create(props.encode(), device, C.byref(h)))
        self.h = h
        self.device = device
        self.scene = None

    def close(self):
        if getattr(self, "h", None):
            self.L.alvrl_integrator_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def preprocess(self, scene: SceneDesc):
        self.scene = scene
        _hcheck(self.L.alvrl_integrator_preprocess(self.h, C.byref(scene)))

    def set_vrls(self, soa: np.ndarray, particle_count: int):
        soa = _np(soa, np.float32)
        _hcheck(self.L.alvrl_integrator_set_vrls(self.h, _ptr(soa), soa.shape[1], particle_count))

    def prepass(self, pass_: int = 0, rank: int = 0, world: int = 1, exchange: "Exchange" = None):
        """vrlIntegrator::prepass; with world > 1 the LightSlice work is sharded
        by slice over the ranks of `exchange` (alvrl_integrator_prepass_dist)."""
        if world == 1:
            _hcheck(self.L.alvrl_integrator_prepass(self.h, pass_))
            return
        if exchange is None:
            raise ValueError("a sharded prepass needs an Exchange")
        rc = self.L.alvrl_integrator_prepass_dist(self.h, pass_, rank, world, C.byref(exchange.desc))
        if rc != ALVRL_OK:
            exchange._check(rc)

    def render(self, d_fb, rank: int = 0, world: int = 1, stream=None):
        _hcheck(self.L.alvrl_integrator_render(self.h, rank, world, _ptr(d_fb),
                                               C.c_void_p(stream) if stream else None))

    def preprocess_ext(self, width: int, height: int, slice_recs: np.ndarray, scene_min, scene_max,
                       medium: "Medium" = None, triangles=None, material=None, tracer: "SceneDesc" = None):
        """alvrl_integrator_preprocess_ext: buildSlices over the caller's gather
        points (slice_recs: W*H records, row-major).  tracer: the VRL tracer's
        scene (a SceneDesc; its arrays must stay alive for this call): each
        prepass then traces the pass's VRLs over it (no set_vrls needed)."""
        sr = _np(slice_recs, np.float32)
        if sr.shape != (width * height, REC_WORDS):
            raise ValueError("slice_recs must be (W*H, REC_WORDS)")
        tri = None if triangles is None else _np(triangles, np.float32).reshape(-1, 9)
        mat = None if material is None else _np(material, np.uint32)
        e = SceneExt(width, height, (C.c_float * 3)(*scene_min), (C.c_float * 3)(*scene_max),
                     (medium or Medium()).desc(), sr.ctypes.data, None if tri is None else tri.ctypes.data,
                     0 if tri is None else tri.shape[0], None if mat is None else mat.ctypes.data,
                     None if tracer is None else C.pointer(tracer))
        self.scene = e
        self._ext_keep = (sr, tri, mat)
        _hcheck(self.L.alvrl_integrator_preprocess_ext(self.h, C.byref(e)))

    def rep_pixels(self, pass_: int = 0) -> np.ndarray:
        """sampleSliceMapping of the pass: representative pixels (row-major ids) in R-row order."""
        n = C.c_uint32()
        _hcheck(self.L.alvrl_integrator_rep_pixels(self.h, pass_, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value), np.uint32)
        _hcheck(self.L.alvrl_integrator_rep_pixels(self.h, pass_, _ptr(out), out.size, C.byref(n)))
        return out[:n.value].copy()

    def prepass_records(self, pass_: int, recs: np.ndarray, rows, rank: int = 0, world: int = 1,
                        exchange: "Exchange" = None):
        """The prepass over the caller's R-row records (recs[i] adds into row rows[i])."""
        r = _np(recs, np.float32).reshape(-1, REC_WORDS)
        rw = _np(rows, np.uint32)
        if rw.size != r.shape[0]:
            raise ValueError("one row per record")
        if world > 1 and exchange is None:
            raise ValueError("a sharded prepass needs an Exchange")
        rc = self.L.alvrl_integrator_prepass_records(self.h, pass_, _ptr(r), _ptr(rw), r.shape[0], rank, world,
                                                     C.byref(exchange.desc) if exchange is not None else None)
        if rc != ALVRL_OK:
            if exchange is not None:
                exchange._check(rc)
            _hcheck(rc)

    def set_cluster_info(self, info: dict, pass_: int = 0):
        """alvrl_integrator_set_cluster_info: install a vrlClusterInfo (dict as
        read_cluster_info returns) for the pass."""
        u = lambda k: _np(info.get(k, np.zeros(0)), np.uint32)
        f = lambda k: _np(info.get(k, np.zeros(0)), np.float32)
        sl, so, rp, w, fr, fw = u("slices"), u("slice_off"), u("reps"), f("weights"), u("fb_reps"), f("fb_weights")
        _hcheck(self.L.alvrl_integrator_set_cluster_info(self.h, pass_, sl.size, _ptr(sl), so.size - 1, _ptr(so),
                                                         _ptr(rp), _ptr(w), fr.size, _ptr(fr), _ptr(fw)))

    def context(self) -> "Context":
        """The device context this integrator drives (a non-owning view)."""
        return Context.borrow(self.L.alvrl_integrator_ctx(self.h), self.device)

    def save_cluster_info(self, path: str):
        """The vrlClusterInfo of the last prepass, to a file (vrlIntegrator.cpp:66-101)."""
        _hcheck(self.L.alvrl_integrator_save_cluster_info(self.h, path.encode()))

    def load_cluster_info(self, path: str, pass_: int = 0):
        """Install a saved vrlClusterInfo for `pass_` instead of running the
        prepass's R build and refinement (a remote worker's wakeup)."""
        _hcheck(self.L.alvrl_integrator_load_cluster_info(self.h, path.encode(), pass_))

    def stats(self) -> dict:
        st = IntegratorStats()
        _hcheck(self.L.alvrl_integrator_get_stats(self.h, C.byref(st)))
        return st.as_dict()

    def local_slices(self) -> np.ndarray:
        """The slices the last prepass refined here (alvrl_integrator_local_slices)."""
        n = C.c_uint32()
        _hcheck(self.L.alvrl_integrator_local_slices(self.h, None, 0, C.byref(n)))
        out = np.zeros(max(1, n.value), np.uint32)
        _hcheck(self.L.alvrl_integrator_local_slices(self.h, _ptr(out), n.value, C.byref(n)))
        return out[:n.value].copy()

    def num_slices(self) -> int:
        return int(self.L.alvrl_integrator_num_slices(self.h))

    def slices(self) -> np.ndarray:
        n = self.scene.width * self.scene.height
        out = np.zeros(n, np.uint32)
        _hcheck(self.L.alvrl_integrator_slices(self.h, _arr(out, C.c_uint32), n))
        return out

    def reps(self):
        ns = self.num_slices()
        cap = self.scene.width * self.scene.height
        off = np.zeros(ns + 1, np.uint32); pix = np.zeros(cap, np.uint32)
        _hcheck(self.L.alvrl_integrator_reps(self.h, _arr(off, C.c_uint32), _arr(pix, C.c_uint32), cap))
        return off, pix[:off[-1]].copy()

    def vrls(self):
        n = C.c_uint32(); pc = C.c_uint64()
        _hcheck(self.L.alvrl_integrator_vrls(self.h, None, 0, C.byref(n), C.byref(pc)))
        soa = np.zeros((9, max(1, n.value)), np.float32)
        _hcheck(self.L.alvrl_integrator_vrls(self.h, _ptr(soa), n.value, C.byref(n), C.byref(pc)))
        return soa[:, :n.value].copy(), int(pc.value)

    def R(self) -> np.ndarray:
        """R of the last prepass as [nvrl, rep_rows, 2] (mean, var)."""
        st = self.stats()
        nv, rows = int(st["vrls"]), int(st["rep_rows"])
        out = np.zeros((nv, rows, 2), np.float32)
        _hcheck(self.L.alvrl_integrator_R(self.h, _ptr(out), out.size))
        return out

    def slice_job(self, s: int, with_R: bool = True) -> dict:
        """Slice s's clustering job of the last prepass (refineSlice's
        inputs, Preprocessor.cpp:254-283): R [nvrl, nrows, 2], rows' locality
        weights, pixel undersampling, initial clusters."""
        nr = C.c_uint32(); ni = C.c_uint32(); pu = C.c_float()
        _hcheck(self.L.alvrl_integrator_slice_job(self.h, s, None, None, 0, C.byref(nr), C.byref(pu), None, None,
                                                  C.byref(ni)))
        nv = int(self.stats()["vrls"])
        R = np.zeros((nv, nr.value, 2), np.float32) if with_R else None
        locw = np.zeros(max(1, nr.value), np.float64)
        iv = np.zeros(max(1, nv), np.uint32); io = np.zeros(ni.value + 1, np.uint32)
        _hcheck(self.L.alvrl_integrator_slice_job(self.h, s, _ptr(R) if with_R else None, _ptr(locw), nr.value,
                                                  C.byref(nr), C.byref(pu), _ptr(iv), _ptr(io), C.byref(ni)))
        return dict(R=R, locw=locw[:nr.value].copy(), pixel_undersampling=pu.value, init_vrls=iv[:nv].copy(),
                    init_off=io)

    def clusters(self):
        ns = self.num_slices()
        nv = self.vrls()[0].shape[1]
        cap = max(1, ns * nv)
        off = np.zeros(ns + 1, np.uint32); reps = np.zeros(cap, np.uint32)
        w = np.zeros(cap, np.float32)
        fr = np.zeros(nv + 1, np.uint32); fw = np.zeros(nv + 1, np.float32); nf = C.c_uint32()
        _hcheck(self.L.alvrl_integrator_clusters(self.h, _arr(off, C.c_uint32), _arr(reps, C.c_uint32),
                                                 _arr(w, C.c_float), cap, _arr(fr, C.c_uint32),
                                                 _arr(fw, C.c_float), nv + 1, C.byref(nf)))
        return dict(slice_off=off, reps=reps[:off[-1]].copy(), weights=w[:off[-1]].copy(),
                    fb_reps=fr[:nf.value].copy(), fb_weights=fw[:nf.value].copy())
