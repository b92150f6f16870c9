"""Rank 0's share of BASELINE.json configs[4] (C5: 2048^2, 1M VRLs, adaptive
LightSlice, 8 GPUs) on ONE GPU, through the real slice-sharded prepass
(alvrl_integrator_prepass_dist): this rank builds R for, and
refines, slices s % 8 == 0 only -- its 1/8 of C5's R, about 65 GB.

The seven other ranks are stood in for by `StubExchange`, an in-process
alvrl_exchange: the non-zero VRL mask gets zeros from them (OR-neutral), and
the cluster all-gather gets, for every slice s % 8 != 0, a one-entry list
(VRL 0, weight 1) in the wire format of csrc/host/exchange.cpp.  Rank 0's
own slices go through the library's exchange code unchanged.

Used by tests/test_gpu_scale.py and tools/c5_share.py (timings)."""
from __future__ import annotations

import ctypes as C
import struct
import time

import numpy as np

SEED_VRL = 0x5EED0001
SEED_RNG = 0xA1B2C3D4
C5_W = C5_H = 2048
C5_VRLS = 1_000_000
C5_WORLD = 8


class StubExchange:
    """alvrl_exchange for rank 0 of `world`, the other ranks simulated."""

    def __init__(self, world: int, nslices: int, nvrl: int):
        import alvrl
        self.world, self.nslices, self.nvrl = world, nslices, nvrl
        self.error = None
        self.calls = []
        self._pending = None        # per-rank messages after a count round
        self.others = []
        for r in range(1, world):
            msg = b"".join(struct.pack("<IIIIf", s, 1, 1, 0, 1.0) for s in range(r, nslices, world))
            self.others.append(msg)

        def allgather(user, send, nbytes, recv):
            try:
                n = int(nbytes)
                src = C.string_at(send, n) if n else b""
                if self._pending is None and n == 8:             # allgather_counts
                    own = struct.unpack("<Q", src)[0]
                    counts = [own] + [len(m) for m in self.others]
                    out = struct.pack(f"<{world}Q", *counts)
                    self._pending = True
                    self.calls.append(("counts", counts))
                elif self._pending:                               # allgatherv data, padded to n
                    out = src + b"".join(m.ljust(n, b"\0") for m in self.others)
                    self._pending = None
                    self.calls.append(("data", n))
                else:                                             # or_reduce of the mask
                    out = src + b"\0" * (n * (world - 1))
                    self.calls.append(("or", n))
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


def run_share(props: str = "", nvrl: int = C5_VRLS, width: int = C5_W, height: int = C5_H,
              world: int = C5_WORLD, pass_: int = 0, gpu_tracer: bool = True, log=print):
    """Rank 0's prepass of the C5 pass: returns (integrator, info dict)."""
    import alvrl
    t0 = time.time()
    scene = alvrl.scene_default(width, height)
    it = alvrl.Integrator(f"vrlTargetNum={nvrl};gpuTracer={'true' if gpu_tracer else 'false'};"
                          f"seed={SEED_RNG};vrlSeed={SEED_VRL}" + (";" + props if props else ""), device=0)
    it.preprocess(scene)
    t1 = time.time()
    ns = it.num_slices()
    # the VRL count of the pass is known only after tracing; the mask stub
    # only needs the byte count it is handed, so nvrl is informational
    ex = StubExchange(world, ns, nvrl)
    it.prepass(pass_, rank=0, world=world, exchange=ex)
    t2 = time.time()
    st = it.stats()
    off, _ = it.reps()
    mine = list(range(0, ns, world))
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
