#!/usr/bin/env python3
"""Time the R build alone (dense alvrl_build_R) at C4 size: 100k VRLs of the
benchmark scene x N representative rows (pixel-centre records of random
pixels).  No refinement, so developer timing variants whose results are
invalid (ALVRL_LIB=variants/libalvrl_*.so) can be timed safely.

    python tools/rbuild_only.py [--rows 15000] [--reps 3] [--mode strict|fast]

Session tool, not part of the bench contract."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mitsuba-alvrl_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=15000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--mode", default="strict")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    import alvrl
    scene = alvrl.scene_default(1024, 1024)
    vrls, pc = alvrl.trace_vrls(scene, 100000, seed=bench.SEED_VRL)
    rng = np.random.default_rng(7)
    pix = np.sort(rng.choice(1024 * 1024, a.rows, replace=False)).astype(np.uint32)
    recs = alvrl.scene_records(scene, pix)
    ctx = alvrl.Context(0, seed=bench.SEED_RNG)
    ctx.set_medium(alvrl.Medium())
    ctx.set_pass(1)
    ctx.upload_vrls(vrls, pc)
    ctx.set_strict_rbuild(a.mode == "strict")
    d_recs = torch.from_numpy(recs.view(np.float32).reshape(len(recs), -1).copy()).cuda()
    d_ids = torch.from_numpy(pix.astype(np.int32)).cuda()
    nv = vrls.shape[1]
    d_Rt = torch.empty((nv, a.rows, 2), dtype=torch.float32, device="cuda")
    ms = []
    for r in range(a.reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        ctx.build_R(d_recs, d_Rt, a.rows, 0, d_ids=d_ids)
        e1.record()
        torch.cuda.synchronize()
        if r:
            ms.append(e0.elapsed_time(e1))
    chk = float(d_Rt[:, :, 0].double().sum().item())
    print(json.dumps({"mode": a.mode, "lib": os.environ.get("ALVRL_LIB", "default"), "rows": a.rows, "vrls": nv,
                      "ms": ms, "ms_min": min(ms), "pairs_per_s": a.rows * nv / (min(ms) * 1e-3),
                      "checksum": chk}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
