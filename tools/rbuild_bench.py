#!/usr/bin/env python3
"""Time the R build of a C4 pass (1024^2, 100k VRLs, 100 slices) with the
strict (oracle-arithmetic) and the fast kernels, prepass only.

    python tools/rbuild_bench.py [--passes 3] [--mode strict|fast|both] [--config C4]

Prints one JSON line per mode: R build ms (HIP events, alvrl stats), refine ms
and the pair count.  Session tool, not part of the bench contract."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mitsuba-alvrl_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--mode", default="both")
    ap.add_argument("--config", default="C4")
    a = ap.parse_args()
    import bench
    import alvrl
    cfg = bench.CONFIGS[a.config]
    W, H = cfg["w"], cfg["h"]
    scene = alvrl.scene_default(W, H)
    vrls, pc = alvrl.trace_vrls(scene, cfg["nvrl"], seed=bench.SEED_VRL)
    modes = ["strict", "fast"] if a.mode == "both" else [a.mode]
    for m in modes:
        props = cfg["props"] + f";seed={bench.SEED_RNG};strictRbuild={'true' if m == 'strict' else 'false'}"
        it = alvrl.Integrator(props, device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        it.prepass(0)
        rb, rf, wall = [], [], []
        for p in range(1, a.passes + 1):
            t0 = time.perf_counter()
            it.prepass(p)
            st = it.stats()
            wall.append((time.perf_counter() - t0) * 1e3)
            rb.append(st["ms_rbuild"])
            rf.append(st["ms_refine"])
            print(json.dumps({"mode": m, "pass": p, "rbuild_ms": rb[-1], "refine_ms": rf[-1],
                              "wall_ms": wall[-1], "contrib_preprocess": st["contrib_preprocess"],
                              "contrib_render": st["contrib_render"]}), flush=True)
        print(json.dumps({"mode": m, "config": a.config, "rbuild_ms_mean": sum(rb) / len(rb),
                          "refine_ms_mean": sum(rf) / len(rf), "prepass_wall_ms_mean": sum(wall) / len(wall),
                          "build_id": alvrl.build_info()["build_id"]}), flush=True)
        it.close()


if __name__ == "__main__":
    main()
