"""C5 rank-0 share on one GPU (tests/c5_share.py): timings, and with
--oracle the strict oracle's refinement of the smallest local slice compared
bit for bit with the device's lists (a heartbeat line every 20 s while the
oracle runs, so a long check is not taken for a hang).

  python tools/c5_share.py [--oracle] [--json out.json] [--props "..."]
  python tools/c5_share.py --res 1024 --vrls 100000 --world 8   # C4's rank-0 share at N = 8
  python tools/c5_share.py --full [--res 256 --vrls 10000]        # every rank in turn + the tile render
"""
import argparse
import json
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "mitsuba-alvrl_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np   # noqa: E402

import c5_share      # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--oracle", action="store_true")
    ap.add_argument("--oracle-rows", type=int, default=0,
                    help="compare the local slice whose row count is nearest this (default: the smallest)")
    ap.add_argument("--props", default="")
    ap.add_argument("--json", default="")
    ap.add_argument("--vrls", type=int, default=c5_share.C5_VRLS)
    ap.add_argument("--res", type=int, default=c5_share.C5_W, help="image width = height")
    ap.add_argument("--world", type=int, default=c5_share.C5_WORLD)
    ap.add_argument("--passes", type=int, default=1, help="prepasses run (timings of the last)")
    ap.add_argument("--full", action="store_true", help="all ranks, true mask OR, merged lists, tile render")
    a = ap.parse_args()
    if a.full:
        return full(a)
    for p in range(a.passes):
        it, info, mine = c5_share.run_share(a.props, nvrl=a.vrls, width=a.res, height=a.res, world=a.world,
                                            pass_=p, log=lambda s: print(s, flush=True))
        if p + 1 < a.passes:
            it.close()
    cl = it.clusters()
    ncl = np.diff(cl["slice_off"])
    info["clusters_local"] = [int(ncl[s]) for s in mine]
    print("clusters per local slice:", info["clusters_local"], flush=True)
    if a.oracle:
        from oracle import Oracle
        o = Oracle()
        rl = np.array(info["rows_local"])
        k = int(np.argmin(np.abs(rl - a.oracle_rows))) if a.oracle_rows else int(np.argmin(rl))
        s = mine[k]
        t0 = time.time()
        job = it.slice_job(s)
        n = job["R"].shape[1]
        print(f"slice {s}: {n} rows x {job['R'].shape[0]} VRLs copied in {time.time() - t0:.1f} s", flush=True)
        res = {}

        def work():
            res["out"] = o.cluster_refine(job["R"], np.arange(n, dtype=np.uint32), job["locw"], job["init_vrls"],
                                          job["init_off"], job["pixel_undersampling"], -1.0,
                                          seed=c5_share.SEED_RNG, pass_=0, stage_refine=3 + 2 * s,
                                          stage_sample=4 + 2 * s)

        th = threading.Thread(target=work)
        t1 = time.time()
        th.start()
        while th.is_alive():
            th.join(20)
            if th.is_alive():
                print(f"  oracle refining slice {s}: {time.time() - t1:.0f} s", flush=True)
        reps, w, refined = res["out"]
        b, e = cl["slice_off"][s], cl["slice_off"][s + 1]
        same = bool(refined and np.array_equal(reps, cl["reps"][b:e]) and
                    np.array_equal(w.view(np.uint32), cl["weights"][b:e].view(np.uint32)))
        info["oracle"] = dict(slice=s, rows=n, clusters_oracle=len(reps), clusters_device=int(e - b),
                              identical=same, oracle_s=time.time() - t1)
        print(f"oracle slice {s}: {len(reps)} clusters (device {e - b}), identical: {same}, "
              f"{time.time() - t1:.1f} s", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(info, f, indent=1)
    it.close()


def full(a):
    import torch
    t0 = time.time()
    it, info = c5_share.run_full(a.props, nvrl=a.vrls, width=a.res, height=a.res, world=a.world,
                                 log=lambda s: print(s, flush=True))
    W = H = a.res
    total = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    for r in range(a.world):
        fb = torch.zeros_like(total)
        it.render(fb, rank=r, world=a.world)
        torch.cuda.synchronize()   # the render ran on the integrator's stream
        total += fb
    one = torch.zeros_like(total)
    it.render(one)
    torch.cuda.synchronize()
    same = bool(torch.equal(total, one))
    if not same:
        two = torch.zeros_like(total)
        it.render(two)
        torch.cuda.synchronize()
        d = (total - one).abs()
        bad = (total != one).view(-1, 3).any(1)
        print(f"tiles != world 1: {int(bad.sum())} of {bad.numel()} pixels differ, max |diff| {float(d.max()):.3e}, "
              f"nan total {int(torch.isnan(total).sum())} one {int(torch.isnan(one).sum())}, "
              f"world-1 repeat equal {bool(torch.equal(one, two))}, zero pixels total {int((total.view(-1, 3) == 0).all(1).sum())} "
              f"one {int((one.view(-1, 3) == 0).all(1).sum())}", flush=True)
        idx = torch.nonzero(bad).view(-1)[:8].tolist()
        for i in idx:
            print(f"  pixel {i} (x {i % W}, y {i // W}): tiles {total.view(-1, 3)[i].tolist()} one {one.view(-1, 3)[i].tolist()}",
                  flush=True)
    st = it.stats()
    out = {k: v for k, v in info.items() if k not in ("p2s", "vrls", "slice_off", "reps", "weights")}
    out.update(tiles_equal_world1=same, render_kernel_ms=st["ms_render_kernel"], s_total=time.time() - t0,
               clusters_total=int(info["slice_off"][-1]))
    print(json.dumps(dict(refine_ms_per_rank=out["refine_ms_per_rank"], tiles_equal_world1=same,
                          render_kernel_ms=out["render_kernel_ms"], s_total=out["s_total"])), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    it.close()
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
