"""One rank of test_gpu_pipeline.test_sharded_prepass: torch.distributed.run
with the gloo backend, every rank on cuda:0 of the one-GPU box.  Each rank
runs the slice-sharded prepass (alvrl_integrator_prepass_dist: R and
refinement for slices s % world == rank, mask OR and cluster all-gather
through alvrl.Exchange) and renders its tiles; the frames are summed to rank
0.  Every rank also runs the one-GPU prepass and compares: the cluster lists
must be identical bit for bit, the summed frame too, and the ranks' R-build
pair counts must add up to the one-GPU count (no slice built twice when
neighbourCount = 0).  Rank 0 writes a JSON verdict."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "mitsuba-alvrl_amd")):
    sys.path.insert(0, p)

import numpy as np                 # noqa: E402
import torch                       # noqa: E402
import torch.distributed as dist   # noqa: E402

import alvrl                       # noqa: E402

SEED_VRL = 0x5EED0001
SEED_RNG = 0xA1B2C3D4
CASES = [
    ("adaptive", "targetNumSlices=40", 256, 192, 1500, 2),
    ("neighbours", "targetNumSlices=30;neighbourCount=3;neighbourWeight=0.5", 192, 128, 900, 1),
    ("fixed", "targetNumSlices=25;localUndersampling=20", 160, 160, 1200, 5),
    ("global", "targetNumSlices=20;globalCluster=true;globalUndersampling=8", 128, 128, 800, 0),
    ("samples", "targetNumSlices=30;sampleCount=3", 160, 128, 900, 3),
]


def run_case(name, props, w, h, nvrl, pass_, rank, world, ex):
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, nvrl, seed=SEED_VRL)

    def make():
        it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        return it

    it = make()
    it.prepass(pass_, rank=rank, world=world, exchange=ex)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb, rank=rank, world=world)
    torch.cuda.synchronize()
    st = it.stats()
    frame = fb.cpu()
    dist.reduce(frame, dst=0)
    counts = torch.tensor([st["contrib_preprocess"], st["slices_local"], st["rows_built"]], dtype=torch.int64)
    dist.all_reduce(counts)
    cl = it.clusters()
    it.close()

    one = make()
    one.prepass(pass_)
    full = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    one.render(full)
    torch.cuda.synchronize()
    st1 = one.stats()
    cl1 = one.clusters()
    one.close()
    same = all(np.array_equal(cl[k].view(np.uint32), cl1[k].view(np.uint32)) for k in cl1)
    flags = torch.tensor([int(same)], dtype=torch.int64)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    return {
        "clusters_identical_all_ranks": bool(flags.item()),
        "frame_bit_exact": bool(torch.equal(frame, full.cpu())) if rank == 0 else None,
        "pairs_sum": int(counts[0]), "pairs_one": int(st1["contrib_preprocess"]),
        "slices_sum": int(counts[1]), "slices": int(st1["slices"]),
        "rows_sum": int(counts[2]), "rows": int(st1["rep_rows"]),
        "clusters": len(cl1["reps"]), "fallback": int(st1["fallback_built"]),
        "exchange_ms": st["ms_exchange"],
    }


def main():
    out_path = sys.argv[1]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(0)
    ex = alvrl.Exchange()
    verdict = {"world": world}
    for case in CASES:
        verdict[case[0]] = run_case(*case, rank=rank, world=world, ex=ex)
    if rank == 0:
        with open(out_path, "w") as f:
            json.dump(verdict, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
