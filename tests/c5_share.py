"""BASELINE.json configs[4] (C5: 2048^2, 1M VRLs, adaptive LightSlice, 8 GPUs)
on ONE GPU, rank by rank, through the real slice-sharded prepass
(alvrl_integrator_prepass_dist).  Rank r builds R for, and
refines, slices s % 8 == r -- its 1/8 of C5's R, about 61 GB -- so the eight
shares run one after the other on one card, each freed before the next.

The exchange (`SimExchange`, an in-process alvrl_exchange) plays the other
seven ranks with the data they would really send:

  phase 1  every rank builds its R rows; its non-zero VRL mask (the OR round of
           Preprocessor::cluster, :843-855) is captured and the prepass is
           stopped there (the callback fails -> ALVRL_ERR_COMM);
  phase 2  every rank's prepass runs to the end with the TRUE OR of all eight
           masks; the cluster all-gather hands it one-entry placeholder lists
           for the other ranks' slices (they are not read: the rank's own
           slices are taken from its result);
  phase 3  the eight ranks' own slices are merged into one vrlClusterInfo (the
           resource the reference ships to render workers, vrlIntegrator.cpp:
           29-101), installed with alvrl_integrator_load_cluster_info, and the
           2048^2 frame is rendered as the eight ranks' 64x64 tiles, summed
           (the framebuffer reduce of vrlIntegrator's render over ranks).

`run_share` keeps round 3's rank-0-only form for the timing tool.
Used by tests/test_gpu_scale.py and tools/c5_share.py."""
from __future__ import annotations

import ctypes as C
import os
import struct
import time

import numpy as np

SEED_VRL = 0x5EED0001
SEED_RNG = 0xA1B2C3D4
C5_W = C5_H = 2048
C5_VRLS = 1_000_000
C5_WORLD = 8


class SimExchange:
    """alvrl_exchange for rank `rank` of `world`, the other ranks simulated.

    masks: None -> capture mode: the OR round records this rank's mask and
    fails the call (the prepass stops before refining).  Otherwise a list of
    `world` byte strings: the OR round receives them in rank order (this
    rank's own bytes in its slot), so the library ORs the true masks.
    "zero": the others send zero masks (round 3's rank-0 timing form)."""

    def __init__(self, rank: int, world: int, nslices: int, masks=None, owners=None):
        import alvrl
        self.rank, self.world, self.nslices = rank, world, nslices
        self.masks = masks
        self.mask = None            # captured own mask (capture mode)
        self.error = None
        self.calls = []
        self._pending = None        # a counts round was seen: the next call is the data round
        self.others = {}
        # the other ranks' slices (owners[r]; default s % world)
        for r in range(world):
            if r != rank:
                mine = owners[r] if owners is not None else range(r, nslices, world)
                self.others[r] = b"".join(struct.pack("<IIIIf", s, 1, 1, 0, 1.0) for s in mine)

        def allgather(user, send, nbytes, recv):
            try:
                n = int(nbytes)
                src = C.string_at(send, n) if n else b""
                if self._pending is None and n == 8:             # allgather_counts
                    own = struct.unpack("<Q", src)[0]
                    counts = [own if r == rank else len(self.others[r]) for r in range(world)]
                    out = struct.pack(f"<{world}Q", *counts)
                    self._pending = True
                    self.calls.append(("counts", counts))
                elif self._pending:                               # allgatherv data, padded to n
                    out = b"".join(src if r == rank else self.others[r].ljust(n, b"\0") for r in range(world))
                    self._pending = None
                    self.calls.append(("data", n))
                else:                                             # or_reduce of the mask
                    self.calls.append(("or", n))
                    if self.masks is None:
                        self.mask = src
                        return 7                                  # stop the prepass here
                    if isinstance(self.masks, str):               # "zero": OR-neutral others
                        out = src + b"\0" * (n * (world - 1))
                        C.memmove(recv, out, len(out))
                        return 0
                    if any(len(m) != n for m in self.masks):
                        raise ValueError("mask sizes differ between ranks")
                    out = b"".join(src if r == rank else self.masks[r] for r in range(world))
                C.memmove(recv, out, len(out))
                return 0
            except Exception as e:     # reported as ALVRL_ERR_COMM
                self.error = e
                return 1

        self._fn = alvrl.ALLGATHER_FN(allgather)
        self.desc = alvrl.ExchangeDesc(None, self._fn)

    def _check(self, rc: int):
        import alvrl
        if rc != alvrl.ALVRL_OK:
            raise alvrl.AlvrlError(rc, alvrl._host().alvrl_host_last_error().decode()
                                   + (f" ({self.error!r})" if self.error else ""))


def lpt_owners(rows, world: int):
    """The integrator's default slice assignment (integrator.hip
    slices_of_rank) for slices whose local matrix is their own rows
    (neighbourCount = 0): slices by row count, largest first (ties: lower
    index), each to the least-loaded rank (ties: lower rank)."""
    order = sorted(range(len(rows)), key=lambda s: (-int(rows[s]), s))
    load = [0] * world
    owners = [[] for _ in range(world)]
    for s in order:
        r = min(range(world), key=lambda q: (load[q], q))
        load[r] += int(rows[s])
        owners[r].append(s)
    return [sorted(o) for o in owners]


def _props(nvrl: int, gpu_tracer: bool, props: str) -> str:
    return (f"vrlTargetNum={nvrl};gpuTracer={'true' if gpu_tracer else 'false'};"
            f"seed={SEED_RNG};vrlSeed={SEED_VRL}" + (";" + props if props else ""))


def run_full(props: str = "", nvrl: int = C5_VRLS, width: int = C5_W, height: int = C5_H,
             world: int = C5_WORLD, pass_: int = 0, check=None, workdir: str = "/tmp", log=print):
    """C5's eight ranks on one GPU (phases 1-3 above).

    check(rank, it, info, mine): called after rank `rank`'s full prepass while
    its R is still resident (for oracle checks of its slices).
    Returns (integrator with the merged cluster info installed, info dict);
    the caller renders and closes it."""
    import alvrl
    scene = alvrl.scene_default(width, height)
    P = _props(nvrl, True, props)
    t_start = time.time()
    # phase 1: the masks (and the slice assignment every rank derives)
    masks, ns, phase1_owners = [], None, None
    for r in range(world):
        it = alvrl.Integrator(P, device=0)
        try:
            it.preprocess(scene)
            ns = it.num_slices()
            if phase1_owners is None:
                it.rep_pixels(pass_)
                off, _ = it.reps()
                phase1_owners = lpt_owners(np.diff(off), world)
            ex = SimExchange(r, world, ns, masks=None, owners=phase1_owners)
            try:
                it.prepass(pass_, rank=r, world=world, exchange=ex)
                raise AssertionError("capture exchange did not stop the prepass")
            except alvrl.AlvrlError as e:
                if ex.mask is None:
                    raise
                assert e.code == alvrl.ALVRL_ERR_COMM, e
            masks.append(ex.mask)
        finally:
            it.close()
    nz = np.zeros(len(masks[0]), np.uint8)
    for m in masks:
        nz |= np.frombuffer(m, np.uint8)
    owners = phase1_owners
    t1 = time.time()
    log(f"C5 phase 1: {world} masks in {t1 - t_start:.1f} s, {int(nz.sum())} of {nz.size} VRLs non-zero "
        f"(per rank {[int(np.frombuffer(m, np.uint8).sum()) for m in masks]})")
    # phase 2: every rank's prepass with the true OR
    per_rank, own = [], {}
    p2s = vrls = None
    for r in range(world):
        it = alvrl.Integrator(P, device=0)
        try:
            it.preprocess(scene)
            ex = SimExchange(r, world, ns, masks=masks, owners=owners)
            t0 = time.time()
            it.prepass(pass_, rank=r, world=world, exchange=ex)
            dt_first = time.time() - t0
            assert [int(x) for x in it.local_slices()] == owners[r], "the integrator's slice assignment" 
            st_first = it.stats()
            # the same pass again: the steady state of a rank that keeps its
            # integrator across passes (R and the refinement's arenas already
            # allocated, as in the bench); the first pass of a fresh
            # integrator also pays their hipMalloc
            ex = SimExchange(r, world, ns, masks=masks, owners=owners)
            t0 = time.time()
            it.prepass(pass_, rank=r, world=world, exchange=ex)
            dt = time.time() - t0
            st = it.stats()
            off, _ = it.reps()
            mine = owners[r]
            rows = np.diff(off)[mine]
            cl = it.clusters()
            for s in mine:
                b, e = cl["slice_off"][s], cl["slice_off"][s + 1]
                own[s] = (cl["reps"][b:e].copy(), cl["weights"][b:e].copy())
            info = dict(rank=r, slices_local=int(st["slices_local"]), rows_local=[int(x) for x in rows],
                        rows_built=int(st["rows_built"]), vrls=int(st["vrls"]),
                        R_bytes=int(st["rows_built"]) * int(st["vrls"]) * 8, ms_rbuild=st["ms_rbuild"],
                        ms_refine_kernel=st["ms_refine_kernel"], refine_entries=int(st["refine_entries"]),
                        refine_split_entries=int(st["refine_split_entries"]),
                        contrib_preprocess=int(st["contrib_preprocess"] - st_first["contrib_preprocess"]), slices_failed=int(st["slices_failed"]),
                        fallback_built=int(st["fallback_built"]), s_prepass=dt, s_prepass_first=dt_first,
                        ms_refine_wall_first=st_first["ms_refine"],
                        ms_alloc=st["ms_alloc"], ms_trace=st["ms_trace"], ms_refine_wall=st["ms_refine"],
                        ms_exchange=st["ms_exchange"], ms_prepass_wall=st["ms_prepass_wall"],
                        clusters_local=[int(len(own[s][0])) for s in mine],
                        exchange_calls=[c[0] for c in ex.calls])
            per_rank.append(info)
            log(f"C5 rank {r}: {len(mine)} slices, rows {rows.min()}..{rows.max()} (sum {rows.sum()}), "
                f"R {info['R_bytes'] / 1e9:.1f} GB, R build {info['ms_rbuild']:.0f} ms, "
                f"refine {info['ms_refine_kernel']:.0f} ms ({info['refine_entries'] / 1e9:.1f}e9 entries), "
                f"prepass {dt:.1f} s (first pass {dt_first:.1f} s, refine wall {st_first['ms_refine']:.0f} ms; "
                f"steady: alloc {info['ms_alloc']:.0f} ms, trace {info['ms_trace']:.0f} ms, "
                f"refine wall {info['ms_refine_wall']:.0f} ms, exchange {info['ms_exchange']:.0f} ms)")
            if r == 0:
                p2s = it.slices()
                vrls = it.vrls()
            if check is not None:
                check(r, it, info, mine)
        finally:
            it.close()
    t2 = time.time()
    # phase 3: merge and install
    slice_off = np.zeros(ns + 1, np.uint32)
    for s in range(ns):
        slice_off[s + 1] = slice_off[s] + len(own[s][0])
    reps = np.concatenate([own[s][0] for s in range(ns)]).astype(np.uint32)
    weights = np.concatenate([own[s][1] for s in range(ns)]).astype(np.float32)
    path = os.path.join(workdir, f"c5_cluster_info_{os.getpid()}.bin")
    alvrl.write_cluster_info(path, dict(slices=p2s, slice_off=slice_off, reps=reps, weights=weights))
    it = alvrl.Integrator(P, device=0)
    try:
        it.preprocess(scene)
        it.load_cluster_info(path, pass_)
    except Exception:
        it.close()
        raise
    finally:
        os.unlink(path)
    info = dict(slices=ns, per_rank=per_rank, p2s=p2s, vrls=vrls, slice_off=slice_off, reps=reps,
                weights=weights, s_phase1=t1 - t_start, s_phase2=t2 - t1,
                refine_ms_per_rank=[x["ms_refine_kernel"] for x in per_rank],
                rbuild_ms_per_rank=[x["ms_rbuild"] for x in per_rank])
    return it, info


def run_share(props: str = "", nvrl: int = C5_VRLS, width: int = C5_W, height: int = C5_H,
              world: int = C5_WORLD, pass_: int = 0, gpu_tracer: bool = True, log=print):
    """Rank 0's prepass of the C5 pass alone, the other ranks' masks zero (round
    3's timing form): returns (integrator, info dict, rank 0's slices)."""
    import alvrl
    t0 = time.time()
    scene = alvrl.scene_default(width, height)
    it = alvrl.Integrator(_props(nvrl, gpu_tracer, props), device=0)
    it.preprocess(scene)
    t1 = time.time()
    ns = it.num_slices()
    it.rep_pixels(pass_)
    off, _ = it.reps()
    owners = lpt_owners(np.diff(off), world)
    t1 = time.time()
    ex = SimExchange(0, world, ns, masks="zero", owners=owners)
    it.prepass(pass_, rank=0, world=world, exchange=ex)
    t2 = time.time()
    st = it.stats()
    off, _ = it.reps()
    mine = owners[0]
    assert [int(x) for x in it.local_slices()] == mine, "the integrator's slice assignment"
    rows = np.diff(off)[mine]
    info = dict(slices=ns, slices_local=st["slices_local"], vrls=st["vrls"], particles=st["particles"],
                rep_rows=st["rep_rows"], rows_built=st["rows_built"], rows_local=[int(x) for x in rows],
                R_bytes=int(st["rows_built"]) * int(st["vrls"]) * 8, ms_rbuild=st["ms_rbuild"],
                ms_refine=st["ms_refine"], ms_refine_kernel=st["ms_refine_kernel"],
                refine_entries=st["refine_entries"], contrib_preprocess=st["contrib_preprocess"],
                slices_failed=st["slices_failed"], s_preprocess=t1 - t0, s_prepass=t2 - t1,
                exchange_calls=[c[0] for c in ex.calls])
    log(f"{width}^2 x {nvrl} VRLs, rank 0 of {world}: {info['slices_local']} of {ns} slices, rows {rows.min()}..{rows.max()} "
        f"(sum {rows.sum()}), R {info['R_bytes'] / 1e9:.1f} GB, R build {info['ms_rbuild']:.0f} ms, "
        f"refine {info['ms_refine_kernel']:.0f} ms ({info['refine_entries'] / 1e9:.1f}e9 entries), "
        f"preprocess {info['s_preprocess']:.1f} s, prepass {info['s_prepass']:.1f} s")
    return it, info, mine
