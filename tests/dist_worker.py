"""One rank of tests/test_distributed.py, launched by torch.distributed.run
with the gloo backend on CPU: renders this rank's share of the image tiles
(alvrl_tile_pixels, the partition alvrl_integrator_render uses) with the
oracle, reduces the framebuffer to rank 0 (the bench's one collective per
step) and checks bench.aggregate_over_ranks.  Rank 0 writes a JSON verdict."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "mitsuba-alvrl_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np          # noqa: E402
import torch                # noqa: E402
import torch.distributed as dist  # noqa: E402

import alvrl                # noqa: E402
import bench                # noqa: E402
from oracle import Oracle   # noqa: E402


def _slice_lists(s, nv=50):
    """Deterministic stand-in for slice s's refined cluster list (ragged,
    some empty, every fifth slice failed)."""
    rng = np.random.default_rng(1000 + s)
    k = int(rng.integers(0, 12)) if s % 7 else 0
    return (s % 5 != 3, rng.choice(nv, k, replace=False).astype(np.uint32),
            rng.random(k, dtype=np.float32))


def check_exchange(rank, world):
    """alvrl_exchange's building blocks (the collectives of the slice-sharded
    prepass, alvrl_integrator_prepass_dist) over gloo."""
    ex = alvrl.Exchange()
    ok = {}
    # variable-size all-gather, rank 0 contributing nothing
    mine = np.arange(3 * rank, dtype=np.uint8) + rank
    got = ex.allgatherv(mine)
    ok["allgatherv"] = all(np.array_equal(g, np.arange(3 * r, dtype=np.uint8) + r) for r, g in enumerate(got))
    # OR of the ranks' non-zero masks
    nv = 77
    mask = np.zeros(nv, np.uint8)
    mask[rank::world + 1] = 1
    ref = np.zeros(nv, np.uint8)
    for r in range(world):
        ref[r::world + 1] = 1
    ok["or"] = bool(np.array_equal(ex.or_(mask), ref))
    # cluster lists of slices dealt round robin, merged into the global CSR
    ns = 23
    local = {s: _slice_lists(s) for s in range(rank, ns, world)}
    refined, off, reps, w = ex.clusters(ns, local)
    good = len(off) == ns + 1 and off[0] == 0
    for s in range(ns):
        r_ok, rr, ww = _slice_lists(s)
        good &= bool(refined[s]) == r_ok
        good &= np.array_equal(reps[off[s]:off[s + 1]], rr) and np.array_equal(ww, w[off[s]:off[s + 1]])
    ok["clusters"] = bool(good)
    # a slice reported twice is rejected
    try:
        ex.clusters(ns, {0: _slice_lists(0)})
        ok["duplicate_rejected"] = world == 1
    except alvrl.AlvrlError as e:
        ok["duplicate_rejected"] = e.code == 6
    return ok


def main():
    out_path = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    o = Oracle()
    W, H = 150, 70                        # 3 x 2 tiles, ragged edges
    sc = o.scene(W, H)
    m = o.medium()
    vrls, pc = o.trace(sc, m, 64, seed=0x5EED0001)
    P = o.params(m, seed=0xA1B2C3D4)
    recs = o.records(sc)
    pix = alvrl.tile_pixels(W, H, rank, world)
    rgb, cnt = o.gather_brute(P, recs[pix], vrls, pc, rec_ids=pix, nthreads=2)
    fb = torch.zeros((W * H, 3), dtype=torch.float32)
    fb[torch.from_numpy(pix.astype(np.int64))] = torch.from_numpy(rgb)
    dist.reduce(fb, dst=0)
    elapsed, counts = bench.aggregate_over_ranks(1.0 + rank, [cnt, 1], world, torch.device("cpu"))
    sizes = torch.tensor([len(pix)], dtype=torch.int64)
    dist.all_reduce(sizes)
    exchange = check_exchange(rank, world)
    if rank == 0:
        full, fcnt = o.gather_brute(P, recs, vrls, pc, nthreads=2)
        verdict = {
            "world": world,
            "frame_bit_exact": bool(np.array_equal(fb.numpy().view(np.uint32), full.view(np.uint32))),
            "pixels_total": int(sizes.item()),
            "elapsed_max": elapsed,
            "count_sum": counts[0], "count_full": int(fcnt), "ranks": counts[1],
            "exchange": exchange,
        }
        with open(out_path, "w") as f:
            json.dump(verdict, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
