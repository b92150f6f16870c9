#!/usr/bin/env python3
"""Timing of the refinement's split engine in isolation (GPU).

J identical clustering jobs over one synthetic local matrix (R rows x N VRL
columns, positive means and variances), each refined with a fixed depth of
two clusters: every job is the column weights, the initial cluster's
variance and ONE split of all N columns (projections, sort, both variance
passes, argmin).  Team mode is off, so each job is one workgroup.  J = 1
gives the latency of one big split (the leader's critical path); J = 256
fills the GPU (throughput).  With ALVRL_REFINE_PROFILE=1 the library prints
the per-phase cycles.  Compare builds with ALVRL_LIB=<variant libalvrl.so>.

    python tools/refine_engine_bench.py --rows 164 --vrls 100000 --jobs 1 256
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "mitsuba-alvrl_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=164)
    ap.add_argument("--vrls", type=int, default=100000)
    ap.add_argument("--jobs", type=int, nargs="+", default=[1, 256])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--tag", default="")
    ap.add_argument("--shuffle", action="store_true",
                    help="the root cluster's columns in a random order (not memory order)")
    a = ap.parse_args()
    os.environ.setdefault("ALVRL_REFINE_TEAM", "1")
    import torch
    import alvrl
    R, N = a.rows, a.vrls
    g = torch.Generator(device="cuda").manual_seed(1234)
    # entries: (mean, var) pairs, [vrl][row] with ld = R; a smooth low-rank
    # mean plus noise, so projections and splits are not degenerate
    base = torch.rand((N, 1), device="cuda", generator=g) * torch.rand((1, R), device="cuda", generator=g)
    mean = (base + 0.05 * torch.rand((N, R), device="cuda", generator=g)).float()
    var = (0.01 * torch.rand((N, R), device="cuda", generator=g) * mean).float()
    Rt = torch.stack([mean, var], dim=-1).contiguous()           # [N][R][2]
    ctx = alvrl.Context(device=0, seed=0xA1B2C3D4)
    ctx.set_medium(alvrl.Medium())
    ctx.upload_vrls(np.zeros((9, N), np.float32) + 0.5, 1000)
    rows = np.arange(R, dtype=np.uint32)
    locw = np.full(R, 1.0 / R, np.float64)
    init_vrls = np.arange(N, dtype=np.uint32)
    if a.shuffle:
        init_vrls = np.random.default_rng(7).permutation(N).astype(np.uint32)
    init_off = np.array([0, N], np.uint32)
    out = {"rows": R, "vrls": N, "lib": os.environ.get("ALVRL_LIB", "default"), "tag": a.tag,
           "shuffle": a.shuffle, "runs": []}
    for J in a.jobs:
        jobs = [dict(rows=rows, locw=locw, pixel_undersampling=1.0 / 64.0, undersampling=N / 2.0,
                     depth_correction=1.0, do_refine=True, stage_refine=3 + 2 * j, stage_sample=4 + 2 * j)
                for j in range(J)]
        ms = []
        for r in range(a.reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            off, reps, w, ok = ctx.refine(Rt, R, jobs, init_vrls, init_off)
            torch.cuda.synchronize()
            if r:
                ms.append(ctx.last_refine_ms())
        ent = ctx.last_refine_entries()
        rec = {"jobs": J, "kernel_ms": min(ms), "kernel_ms_all": ms, "entries": ent,
               "cycles_per_column_est": min(ms) * 1e-3 * 2.4e9 / N}
        out["runs"].append(rec)
        print(json.dumps(rec), flush=True)
        # timing-only variants (tools/build_variant.sh with ALVRL_EXP_* macros) give no valid clusters
        if os.environ.get("ALVRL_ENGINE_NOCHECK") != "1":
            assert ok.all() and (np.diff(off) == 2).all(), (off[:4], ok[:4])
    print(json.dumps(out))


if __name__ == "__main__":
    main()
