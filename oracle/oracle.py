"""ctypes binding of the CPU restatement (oracle/liboracle*.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  See
oracle/alvrl_oracle.h for what is restated (with reference file:line) and for
the parity status ("parity unpinned" except the Philox RNG).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REC_WORDS = 20
FLAG_HIT, FLAG_SMOOTH, FLAG_MEDIUM = 1, 2, 4
DOM_GATHER, DOM_RBUILD, DOM_TRACER, DOM_REPS, DOM_CLUSTER = 1, 2, 3, 4, 5
UINT32_MAX = 0xFFFFFFFF


def build(force: bool = False) -> None:
    """Compile liboracle.so / liboracle_fast.so with oracle/Makefile."""
    need = force or not all(
        os.path.exists(os.path.join(HERE, n)) for n in ("liboracle.so", "liboracle_fast.so"))
    if need:
        subprocess.check_call(["make", "-s", "-C", HERE] + (["-B"] if force else []))


class Medium(C.Structure):
    _fields_ = [("sigma_s", C.c_float * 3), ("sigma_a", C.c_float * 3), ("sigma_t", C.c_float * 3),
                ("sampling_weight", C.c_float), ("phase_type", C.c_int), ("phase_g", C.c_float),
                ("strategy", C.c_int), ("density", C.c_float), ("mx_sigma", C.c_float * 3),
                ("mx_cdf", C.c_float * 4), ("mx_start", C.c_float * 3), ("mx_lower", C.c_float * 3),
                ("mx_norm", C.c_float), ("mx_inv_norm", C.c_float)]


STRATEGIES = {"balance": 0, "single": 1, "manual": 2, "maximum": 3}


class Params(C.Structure):
    _fields_ = [("medium", Medium), ("vol_vol_samples", C.c_int), ("vol_surf_samples", C.c_int),
                ("short_vrls", C.c_int), ("seed", C.c_uint32), ("pass_", C.c_uint32),
                ("r_samples", C.c_int), ("occ", C.POINTER(C.c_float)), ("nocc", C.c_uint32),
                ("occ_mat", C.POINTER(C.c_uint32))]


class Scene(C.Structure):
    _fields_ = [("cam_origin", C.c_float * 3), ("cam_target", C.c_float * 3), ("cam_up", C.c_float * 3),
                ("fov_x_deg", C.c_float), ("width", C.c_int), ("height", C.c_int),
                ("box_min", C.c_float * 3), ("box_max", C.c_float * 3), ("albedo", C.c_float * 3),
                ("light_pos", C.c_float * 3), ("light_intensity", C.c_float * 3),
                ("occ", C.POINTER(C.c_float)), ("nocc", C.c_uint32), ("occ_albedo", C.c_float * 3),
                ("occ_mat", C.POINTER(C.c_uint32)), ("occ_spec", C.c_float * 3), ("occ_eta", C.c_float),
                ("emit", C.POINTER(C.c_float)), ("nemit", C.c_uint32), ("emit_radiance", C.c_float * 3),
                ("occ_albedos", C.POINTER(C.c_float))]


MAT_DIFFUSE, MAT_MIRROR, MAT_NULL, MAT_DIELECTRIC = 0, 1, 2, 3


def set_area_emitter(scene, tris, radiance):
    """An area emitter replacing the point light ((n, 9) float32 triangles,
    radiance on the side of cross(p1 - p0, p2 - p0)); kept alive on the Scene."""
    arr = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
    scene._emit_keep = arr
    scene.emit = arr.ctypes.data_as(C.POINTER(C.c_float)) if len(arr) else None
    scene.nemit = len(arr)
    for i in range(3):
        scene.emit_radiance[i] = float(radiance[i])
    return scene


def set_occluders(obj, tris, albedo=None, material=None, specular=None, eta=None, albedos=None):
    """Occluder triangles ((n, 9) float32) on a Scene (hit by eye rays and
    particles, occ_albedo) or a Params (blocking the gather's connections);
    material: None (all diffuse) or one MAT_* per triangle; specular: the
    mirrors' reflectance (Scene); albedos: (n, 3) per-triangle reflectances
    (Scene; replaces occ_albedo).  The arrays are kept alive on the object."""
    arr = np.ascontiguousarray(np.asarray(tris, np.float32).reshape(-1, 9))
    obj._occ_keep = arr
    obj.occ = arr.ctypes.data_as(C.POINTER(C.c_float)) if len(arr) else None
    obj.nocc = len(arr)
    if albedo is not None:
        for i in range(3):
            obj.occ_albedo[i] = float(albedo[i])
    if albedos is not None:
        alb = np.ascontiguousarray(np.asarray(albedos, np.float32).reshape(len(arr), 3))
        obj._alb_keep = alb
        obj.occ_albedos = alb.ctypes.data_as(C.POINTER(C.c_float))
    if material is not None:
        mat = np.ascontiguousarray(np.broadcast_to(np.asarray(material, np.uint32), (len(arr),)))
        obj._mat_keep = mat
        obj.occ_mat = mat.ctypes.data_as(C.POINTER(C.c_uint32))
    if specular is not None:
        for i in range(3):
            obj.occ_spec[i] = float(specular[i])
    if eta is not None:
        obj.occ_eta = float(eta)
    return obj


class PrepParams(C.Structure):
    _fields_ = [("target_num_slices", C.c_uint32), ("neighbour_count", C.c_uint32),
                ("neighbour_weight", C.c_float), ("global_cluster", C.c_int),
                ("local_refinement", C.c_int), ("global_undersampling", C.c_float),
                ("local_undersampling", C.c_float), ("fallback_undersampling", C.c_float),
                ("depth_correction", C.c_float), ("slice_curvature_factor", C.c_float),
                ("seed", C.c_uint32), ("pass_", C.c_uint32)]


def _p(a, t=C.c_float):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


class Oracle:
    """Thin wrapper; `fast=True` loads the reference-flags build (timing only)."""

    def __init__(self, fast: bool = False):
        build()
        # ALVRL_ORACLE_LIB: the sanitizer build of the checker (tools/sanitize_cpu.sh)
        path = os.environ.get("ALVRL_ORACLE_LIB") if not fast else None
        self.lib = C.CDLL(path or os.path.join(HERE, "liboracle_fast.so" if fast else "liboracle.so"))
        L = self.lib
        u32, f32, i32, u64 = C.c_uint32, C.c_float, C.c_int, C.c_uint64
        P = C.POINTER
        L.alvrl_o_philox4x32_10.argtypes = [P(u32), P(u32), P(u32)]
        L.alvrl_o_u01.argtypes = [u32]; L.alvrl_o_u01.restype = f32
        L.alvrl_o_medium_init.argtypes = [P(Medium), P(f32), P(f32), f32, i32, f32]
        L.alvrl_o_medium_eval.argtypes = [P(Medium), f32, P(f32), P(f32)]
        L.alvrl_o_detmath.argtypes = [i32, P(f32), P(f32), u32]
        L.alvrl_o_medium_strategy.argtypes = [P(Medium), i32, i32, f32]
        L.alvrl_o_closest_points.argtypes = [P(f32)] * 6
        L.alvrl_o_closest_points.restype = f32
        L.alvrl_o_kulla.argtypes = [P(f32), P(f32), P(f32), f32, P(f32)]
        L.alvrl_o_kulla.restype = f32
        L.alvrl_o_sample_v_to_distance.argtypes = [P(f32)] * 5 + [f32, P(f32)]
        L.alvrl_o_sample_v_to_distance.restype = f32
        L.alvrl_o_integrate_vrl.argtypes = [P(Params), P(f32), u32, P(f32), u32, u32, u32,
                                            P(f32), P(f32), P(f32)]
        L.alvrl_o_gather_brute.argtypes = [P(Params), P(f32), u32, P(u32), P(f32), u32, u64, u32,
                                           P(f32), P(f32), i32]
        L.alvrl_o_gather_brute.restype = u64
        L.alvrl_o_gather_clustered.argtypes = [P(Params), P(f32), u32, P(u32), P(u32), P(f32), u32,
                                               u64, P(u32), P(u32), P(f32), P(u32), P(f32), u32,
                                               P(f32), i32]
        L.alvrl_o_gather_clustered.restype = u64
        L.alvrl_o_scene_default.argtypes = [P(Scene), i32, i32]
        L.alvrl_o_camera_ray.argtypes = [P(Scene), f32, f32, P(f32), P(f32)]
        L.alvrl_o_make_records.argtypes = [P(Scene), i32, P(f32)]
        L.alvrl_o_make_record.argtypes = [P(Scene), i32, i32, i32, P(f32)]
        L.alvrl_o_make_slice_record.argtypes = [P(Scene), i32, i32, P(f32)]
        L.alvrl_o_make_chain.argtypes = [P(Scene), P(Medium), i32, i32, i32, u32, u32, i32, f32, P(f32), u32]
        L.alvrl_o_make_chain.restype = u32
        L.alvrl_o_make_record_s.argtypes = [P(Scene), i32, i32, i32, u32, u32, u32, u32, P(f32)]
        L.alvrl_o_make_chain_s.argtypes = [P(Scene), P(Medium), i32, i32, i32, u32, u32, i32, f32, u32, u32,
                                           P(f32), u32]
        L.alvrl_o_make_chain_s.restype = u32
        L.alvrl_o_trace_vrls.argtypes = [P(Scene), P(Medium), u32, u32, u32, i32, i32, i32,
                                         P(f32), u32, P(u64)]
        L.alvrl_o_trace_vrls.restype = u32
        L.alvrl_o_prep_create.argtypes = [P(PrepParams)]; L.alvrl_o_prep_create.restype = C.c_void_p
        L.alvrl_o_prep_destroy.argtypes = [C.c_void_p]
        L.alvrl_o_prep_build_slices.argtypes = [C.c_void_p, P(Scene), P(u32)]
        L.alvrl_o_prep_num_slices.argtypes = [C.c_void_p]; L.alvrl_o_prep_num_slices.restype = u32
        L.alvrl_o_prep_sample_slice_mapping.argtypes = [C.c_void_p, f32, P(u32), P(u32), u32,
                                                        P(f32), P(f32)]
        L.alvrl_o_prep_local_rows.argtypes = [C.c_void_p, u32, P(u32), P(C.c_double)]
        L.alvrl_o_prep_local_rows.restype = u32
        L.alvrl_o_prep_build_clusters.argtypes = [C.c_void_p, P(f32), u32, P(u32), P(u32), P(f32),
                                                  u32, P(u32), P(f32), P(u32), P(u32), P(f32), P(u32)]
        L.alvrl_o_cluster_members.argtypes = [P(f32), u64, P(u32), u32, P(C.c_double), u32, P(u32),
                                              P(u32), u32, f32, f32, u32, u32, u32, P(u32), P(u32),
                                              P(u32), P(C.c_int)]
        L.alvrl_o_cluster_refine.argtypes = [P(f32), u64, P(u32), u32, P(C.c_double), u32, P(u32),
                                             P(u32), u32, f32, f32, f32, i32, u32, u32, u32, u32,
                                             P(u32), P(f32), P(u32), P(i32)]

    # ---- RNG ----
    def philox(self, ctr, key):
        c = (C.c_uint32 * 4)(*ctr); k = (C.c_uint32 * 2)(*key); o = (C.c_uint32 * 4)()
        self.lib.alvrl_o_philox4x32_10(c, k, o)
        return list(o)

    # ---- single functions (known-answer fixtures) ----
    def closest_points(self, s1p0, s1p1, s2p0, s2p1):
        f3 = C.c_float * 3
        a, b = f3(), f3()
        h = self.lib.alvrl_o_closest_points(f3(*s1p0), f3(*s1p1), f3(*s2p0), f3(*s2p1), a, b)
        return h, list(a), list(b)

    def kulla(self, A, B, D, u):
        f3 = C.c_float * 3
        r = f3()
        pdf = self.lib.alvrl_o_kulla(f3(*A), f3(*B), f3(*D), u, r)
        return pdf, list(r)

    def sample_v_to_distance(self, E, d, hitp, S, End, u):
        f3 = C.c_float * 3
        r = f3()
        pdf = self.lib.alvrl_o_sample_v_to_distance(f3(*E), f3(*d), f3(*hitp), f3(*S), f3(*End), u, r)
        return pdf, list(r)

    DETMATH_FNS = ("exp", "log", "atan", "tan", "asinh", "sinh")

    def detmath(self, fn: str, x):
        """detmath.h's float function `fn` elementwise (float32 in and out)."""
        x = np.ascontiguousarray(x, np.float32)
        out = np.empty_like(x)
        self.lib.alvrl_o_detmath(self.DETMATH_FNS.index(fn), _p(x), _p(out), x.size)
        return out

    def medium_eval(self, medium: Medium, distance: float):
        tr = (C.c_float * 3)(); pf = C.c_float()
        self.lib.alvrl_o_medium_eval(C.byref(medium), distance, tr, C.byref(pf))
        return list(tr), pf.value

    # ---- scene / medium ----
    def scene(self, width: int, height: int) -> Scene:
        s = Scene()
        self.lib.alvrl_o_scene_default(C.byref(s), width, height)
        return s

    def medium(self, sigma_s=(0.8, 0.6, 0.4), sigma_a=(0.05, 0.05, 0.05), weight=-1.0,
               phase_type=0, g=0.0, strategy="balance", channel=-1, density=0.0) -> Medium:
        """HomogeneousMedium: strategy 'balance' | 'single' (channel, -1 = the
        smallest sigma_t) | 'manual' (samplingDensity) | 'maximum'."""
        m = Medium()
        ss = (C.c_float * 3)(*sigma_s); sa = (C.c_float * 3)(*sigma_a)
        self.lib.alvrl_o_medium_init(C.byref(m), ss, sa, weight, phase_type, g)
        if self.lib.alvrl_o_medium_strategy(C.byref(m), STRATEGIES[strategy], channel, density) != 0:
            raise ValueError(f"medium strategy {strategy!r} not possible for sigma_t {list(m.sigma_t)}")
        return m

    def params(self, medium: Medium, nvv=2, nvs=2, short_vrls=1, seed=0xA1B2C3D4, pass_=0,
               r_samples=1) -> Params:
        return Params(medium, nvv, nvs, short_vrls, seed, pass_, r_samples)

    def records(self, scene: Scene, medium_scatters: bool = True) -> np.ndarray:
        out = np.zeros((scene.width * scene.height, REC_WORDS), np.float32)
        self.lib.alvrl_o_make_records(C.byref(scene), int(medium_scatters), _p(out))
        return out

    def record(self, scene: Scene, x: int, y: int, medium_scatters: bool = True) -> np.ndarray:
        out = np.zeros(REC_WORDS, np.float32)
        self.lib.alvrl_o_make_record(C.byref(scene), int(medium_scatters), x, y, _p(out))
        return out

    def chain(self, scene: Scene, medium: Medium, x: int, y: int, medium_scatters: bool = True,
              seed=0xA1B2C3D4, pass_=0, spec_rr_depth=100, init_throughput=20.0, cap=256) -> np.ndarray:
        """LiInternal's eye path of pixel (x, y): (k, REC_WORDS) records."""
        out = np.zeros((cap, REC_WORDS), np.float32)
        n = self.lib.alvrl_o_make_chain(C.byref(scene), C.byref(medium), int(medium_scatters), x, y, seed,
                                        pass_, spec_rr_depth, init_throughput, _p(out), cap)
        return out[:n].copy()

    def record_s(self, scene: Scene, x: int, y: int, sample: int, spp: int, medium_scatters: bool = True,
                 seed=0xA1B2C3D4, pass_=0) -> np.ndarray:
        """Record of sensor sample `sample` of `spp` of pixel (x, y) (jittered
        unless spp == 1; the depth word carries the sample in bits 16-31)."""
        out = np.zeros(REC_WORDS, np.float32)
        self.lib.alvrl_o_make_record_s(C.byref(scene), int(medium_scatters), x, y, seed, pass_, sample, spp, _p(out))
        return out

    def records_spp(self, scene: Scene, pixel_ids, spp: int, medium_scatters: bool = True, seed=0xA1B2C3D4,
                    pass_=0):
        """Records of every sensor sample of the row-major pixel ids, sample
        major (record s * n + i: pixel_ids[i], sample s): (records, pixels)."""
        ids = np.asarray(pixel_ids, np.uint32)
        out = np.zeros((spp * len(ids), REC_WORDS), np.float32)
        for sm in range(spp):
            for i, p in enumerate(ids):
                self.lib.alvrl_o_make_record_s(C.byref(scene), int(medium_scatters), int(p % scene.width),
                                               int(p // scene.width), seed, pass_, sm, spp,
                                               _p(out[sm * len(ids) + i]))
        return out, np.tile(ids, spp)

    def chain_s(self, scene: Scene, medium: Medium, x: int, y: int, sample: int, spp: int,
                medium_scatters: bool = True, seed=0xA1B2C3D4, pass_=0, spec_rr_depth=100, init_throughput=20.0,
                cap=256) -> np.ndarray:
        """The eye path of sensor sample `sample` of `spp` of pixel (x, y)."""
        out = np.zeros((cap, REC_WORDS), np.float32)
        n = self.lib.alvrl_o_make_chain_s(C.byref(scene), C.byref(medium), int(medium_scatters), x, y, seed, pass_,
                                          spec_rr_depth, init_throughput, sample, spp, _p(out), cap)
        return out[:n].copy()

    def chains(self, scene: Scene, medium: Medium, pixel_ids, **kw):
        """Eye paths of row-major pixel ids: (records, pixel of each record)."""
        recs, pix = [], []
        for p in np.asarray(pixel_ids, np.uint32):
            c = self.chain(scene, medium, int(p % scene.width), int(p // scene.width), **kw)
            recs.append(c)
            pix.append(np.full(len(c), p, np.uint32))
        return np.concatenate(recs), np.concatenate(pix)

    def slice_record(self, scene: Scene, x: int, y: int) -> np.ndarray:
        out = np.zeros(REC_WORDS, np.float32)
        self.lib.alvrl_o_make_slice_record(C.byref(scene), x, y, _p(out))
        return out

    def volpath(self, scene: Scene, medium: Medium, spp: int, seed=0xA1B2C3D4, pass_=0, pixel_ids=None,
                max_depth=-1, rr_depth=5, only_vrl_paths=True, vol_to_vol=True, vol_to_surf=True):
        """volpath onlyVRLpaths reference (alvrl_o_volpath): (n, 3) means over spp."""
        class VP(C.Structure):
            _fields_ = [("max_depth", C.c_int), ("rr_depth", C.c_int), ("only_vrl_paths", C.c_int),
                        ("vrl_vol_to_vol", C.c_int), ("vrl_vol_to_surf", C.c_int)]
        vp = VP(max_depth, rr_depth, int(only_vrl_paths), int(vol_to_vol), int(vol_to_surf))
        n = scene.width * scene.height if pixel_ids is None else len(pixel_ids)
        ids = None if pixel_ids is None else np.ascontiguousarray(pixel_ids, np.uint32)
        out = np.zeros((n, 3), np.float32)
        self.lib.alvrl_o_volpath(C.byref(scene), C.byref(medium), C.byref(vp), seed, pass_, spp,
                                 _p(ids, C.c_uint32), n, _p(out))
        return out

    def trace(self, scene: Scene, medium: Medium, target: int, seed=0x5EED0001, pass_=0,
              short_vrls=True, max_depth=-1, rr_depth=5):
        cap = target + 4096
        soa = np.zeros((9, cap), np.float32)
        pc = C.c_uint64()
        n = self.lib.alvrl_o_trace_vrls(C.byref(scene), C.byref(medium), seed, pass_, target,
                                        int(short_vrls), max_depth, rr_depth, _p(soa), cap,
                                        C.byref(pc))
        return np.ascontiguousarray(soa[:, :n]), int(pc.value)

    # ---- gathers ----
    def integrate(self, P: Params, rec, rec_id, vrls, vrl_id, domain=DOM_GATHER):
        rgb = np.zeros(3, np.float32); c = C.c_float(); v = C.c_float()
        vrls = np.ascontiguousarray(vrls, np.float32)
        self.lib.alvrl_o_integrate_vrl(C.byref(P), _p(np.ascontiguousarray(rec, np.float32)),
                                       rec_id, _p(vrls), vrls.shape[1], vrl_id, domain, _p(rgb),
                                       C.byref(c), C.byref(v))
        return rgb, c.value, v.value

    def gather_brute(self, P: Params, recs, vrls, particle_count, rec_ids=None,
                     domain=DOM_GATHER, want_R=False, nthreads=None):
        recs = np.ascontiguousarray(recs, np.float32)
        vrls = np.ascontiguousarray(vrls, np.float32)
        n, nv = recs.shape[0], vrls.shape[1]
        out = np.zeros((n, 3), np.float32)
        R = np.zeros((n, nv, 2), np.float32) if want_R else None
        ids = None if rec_ids is None else np.ascontiguousarray(rec_ids, np.uint32)
        cnt = self.lib.alvrl_o_gather_brute(C.byref(P), _p(recs), n, _p(ids, C.c_uint32), _p(vrls),
                                            nv, particle_count, domain, _p(out), _p(R),
                                            nthreads or min(16, os.cpu_count() or 1))
        return (out, R, int(cnt)) if want_R else (out, int(cnt))

    def gather_clustered(self, P: Params, recs, slice_of_rec, vrls, particle_count, slice_off,
                         reps, weights, fb_reps, fb_weights, rec_ids=None, nthreads=None):
        recs = np.ascontiguousarray(recs, np.float32)
        vrls = np.ascontiguousarray(vrls, np.float32)
        n, nv = recs.shape[0], vrls.shape[1]
        out = np.zeros((n, 3), np.float32)
        ids = None if rec_ids is None else np.ascontiguousarray(rec_ids, np.uint32)
        a = [np.ascontiguousarray(x, dt) for x, dt in (
            (slice_of_rec, np.uint32), (slice_off, np.uint32), (reps, np.uint32),
            (weights, np.float32), (fb_reps, np.uint32), (fb_weights, np.float32))]
        cnt = self.lib.alvrl_o_gather_clustered(
            C.byref(P), _p(recs), n, _p(ids, C.c_uint32), _p(a[0], C.c_uint32), _p(vrls), nv,
            particle_count, _p(a[1], C.c_uint32), _p(a[2], C.c_uint32), _p(a[3]),
            _p(a[4], C.c_uint32), _p(a[5]), len(a[4]), _p(out), nthreads or min(16, os.cpu_count() or 1))
        return out, int(cnt)

    # ---- LightSlice preprocessing ----
    def prep_params(self, target_num_slices=100, neighbour_count=0, neighbour_weight=0.0,
                    global_cluster=False, local_refinement=True, global_undersampling=-1.0,
                    local_undersampling=-1.0, fallback_undersampling=5.0, depth_correction=1.0,
                    slice_curvature_factor=0.5, seed=0xA1B2C3D4, pass_=0) -> PrepParams:
        return PrepParams(target_num_slices, neighbour_count, neighbour_weight, int(global_cluster),
                          int(local_refinement), global_undersampling, local_undersampling,
                          fallback_undersampling, depth_correction, slice_curvature_factor, seed,
                          pass_)

    def cluster_refine(self, Rt, rows, locw, init_vrls, init_off, pixel_undersampling,
                       undersampling, depth_correction=1.0, do_refine=True, seed=0xA1B2C3D4,
                       pass_=0, stage_refine=3, stage_sample=4):
        """One Clustering (ctor + refine + sampleRepresentatives) on Rt[v][row] pairs."""
        Rt = np.ascontiguousarray(Rt, np.float32)
        nv, ld = Rt.shape[0], Rt.shape[1]
        rows = np.ascontiguousarray(rows, np.uint32)
        locw = np.ascontiguousarray(locw, np.float64)
        iv = np.ascontiguousarray(init_vrls, np.uint32)
        io = np.ascontiguousarray(init_off, np.uint32)
        reps = np.zeros(nv + 1, np.uint32); w = np.zeros(nv + 1, np.float32)
        nr = C.c_uint32(); refined = C.c_int()
        rc = self.lib.alvrl_o_cluster_refine(
            _p(Rt), ld, _p(rows, C.c_uint32), len(rows), _p(locw, C.c_double), nv,
            _p(iv, C.c_uint32), _p(io, C.c_uint32), len(io) - 1, pixel_undersampling,
            undersampling, depth_correction, int(do_refine), seed, pass_, stage_refine,
            stage_sample, _p(reps, C.c_uint32), _p(w), C.byref(nr), C.byref(refined))
        if rc != 0:
            raise RuntimeError(f"oracle cluster_refine failed rc={rc}")
        return reps[:nr.value].copy(), w[:nr.value].copy(), bool(refined.value)

    def cluster_members(self, Rt, rows, locw, init_vrls, init_off, pixel_undersampling,
                        undersampling, seed=0xA1B2C3D4, pass_=0, stage_refine=0xFFFFFFFE):
        """ctor + refine + getVrlsPerCluster (Preprocessor.cpp:526-543):
        (vrls, offsets, refined)."""
        Rt = np.ascontiguousarray(Rt, np.float32)
        nv, ld = Rt.shape[0], Rt.shape[1]
        rows = np.ascontiguousarray(rows, np.uint32)
        locw = np.ascontiguousarray(locw, np.float64)
        iv = np.ascontiguousarray(init_vrls, np.uint32)
        io = np.ascontiguousarray(init_off, np.uint32)
        out = np.zeros(len(iv) + 1, np.uint32); off = np.zeros(len(iv) + 2, np.uint32)
        nc = C.c_uint32(); refined = C.c_int()
        rc = self.lib.alvrl_o_cluster_members(
            _p(Rt), ld, _p(rows, C.c_uint32), len(rows), _p(locw, C.c_double), nv,
            _p(iv, C.c_uint32), _p(io, C.c_uint32), len(io) - 1, pixel_undersampling,
            undersampling, seed, pass_, stage_refine, _p(out, C.c_uint32), _p(off, C.c_uint32),
            C.byref(nc), C.byref(refined))
        if rc != 0:
            raise RuntimeError(f"oracle cluster_members failed rc={rc}")
        return out[:len(iv)].copy(), off[:nc.value + 1].copy(), bool(refined.value)


class Prep:
    """Oracle Preprocessor (slices, representatives, localities, clusters)."""

    def __init__(self, o: Oracle, params: PrepParams):
        self.o = o
        self.h = o.lib.alvrl_o_prep_create(C.byref(params))
        self.params = params

    def __del__(self):
        if getattr(self, "h", None):
            self.o.lib.alvrl_o_prep_destroy(self.h)
            self.h = None

    def build_slices(self, scene: Scene) -> np.ndarray:
        out = np.zeros(scene.width * scene.height, np.uint32)
        rc = self.o.lib.alvrl_o_prep_build_slices(self.h, C.byref(scene), _p(out, C.c_uint32))
        if rc:
            raise RuntimeError("buildSlices failed")
        return out

    @property
    def num_slices(self) -> int:
        return int(self.o.lib.alvrl_o_prep_num_slices(self.h))

    def sample_slice_mapping(self, target_pixel_undersampling: float, cap: int):
        ns = self.num_slices
        off = np.zeros(ns + 1, np.uint32); pix = np.zeros(cap, np.uint32)
        su = np.zeros(ns, np.float32); gu = C.c_float()
        rc = self.o.lib.alvrl_o_prep_sample_slice_mapping(self.h, target_pixel_undersampling,
                                                          _p(off, C.c_uint32), _p(pix, C.c_uint32),
                                                          cap, _p(su), C.byref(gu))
        if rc:
            raise RuntimeError(f"sampleSliceMapping failed rc={rc}")
        return off, pix[:off[-1]].copy(), su, gu.value

    def local_rows(self, s: int, cap: int):
        rows = np.zeros(cap, np.uint32); w = np.zeros(cap, np.float64)
        n = self.o.lib.alvrl_o_prep_local_rows(self.h, s, _p(rows, C.c_uint32), _p(w, C.c_double))
        return rows[:n].copy(), w[:n].copy()

    def build_clusters(self, Rt: np.ndarray):
        Rt = np.ascontiguousarray(Rt, np.float32)
        nv = Rt.shape[0]
        ns = self.num_slices
        cap = ns * nv + 1
        off = np.zeros(ns + 1, np.uint32); reps = np.zeros(cap, np.uint32)
        w = np.zeros(cap, np.float32)
        gr = np.zeros(nv + 1, np.uint32); gw = np.zeros(nv + 1, np.float32); ng = C.c_uint32()
        fr = np.zeros(nv + 1, np.uint32); fw = np.zeros(nv + 1, np.float32); nf = C.c_uint32()
        rc = self.o.lib.alvrl_o_prep_build_clusters(
            self.h, _p(Rt), nv, _p(off, C.c_uint32), _p(reps, C.c_uint32), _p(w), cap,
            _p(gr, C.c_uint32), _p(gw), C.byref(ng), _p(fr, C.c_uint32), _p(fw), C.byref(nf))
        if rc:
            raise RuntimeError(f"buildClusters failed rc={rc}")
        n = int(off[-1])
        return dict(slice_off=off, reps=reps[:n].copy(), weights=w[:n].copy(),
                    gc_reps=gr[:ng.value].copy(), gc_weights=gw[:ng.value].copy(),
                    fb_reps=fr[:nf.value].copy(), fb_weights=fw[:nf.value].copy())
