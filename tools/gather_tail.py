"""Gather launch-shape timing at C4: the clustered gather over every pixel's
record with the integrator's cluster lists, its work items (<= 64 pixels of
one slice, one wave each) in slice order, sorted by their slice's list length
(longest first), and truncated to whole rounds of resident waves.  Prints
per-variant kernel ms (HIP events on the context's stream)."""
import sys
import numpy as np
import torch

sys.path.insert(0, "mitsuba-alvrl_amd")
import alvrl  # noqa: E402

W = H = 1024
scene = alvrl.scene_default(W, H)
vrls, pc = alvrl.trace_vrls(scene, 100000, seed=0x5EED0001)
it = alvrl.Integrator("targetNumSlices=100;seed=2712847316", device=0)
it.set_vrls(vrls, pc)
it.preprocess(scene)
it.prepass(0)
p2s = it.slices()                       # column-major y + H*x
cl = it.clusters()
ctx = alvrl.Context(device=0, seed=0xA1B2C3D4)
ctx.set_medium(alvrl.Medium())
ctx.upload_vrls(vrls, pc)
ctx.set_clusters(cl["slice_off"], cl["reps"], cl["weights"], cl["fb_reps"], cl["fb_weights"])
pid = np.arange(W * H, dtype=np.uint32)
sl = p2s[(pid % W) * H + pid // W]
order = np.argsort(sl, kind="stable")
pix = pid[order]
items = alvrl.Context.make_work_items(sl[order])
recs = alvrl.scene_records_gpu(scene, pixel_ids=pix)
d_ids = torch.from_numpy(pix.view(np.int32)).cuda()
d_out = torch.zeros((len(pix), 3), dtype=torch.float32, device="cuda")
k = np.diff(cl["slice_off"].astype(np.int64))
nfb = len(cl["fb_reps"])
kk = np.array([k[s] if s != 0xFFFFFFFF else nfb for s in items[:, 0]])
print(f"items {len(items)}, reps per item: min {kk.min()} median {int(np.median(kk))} max {kk.max()}", flush=True)
variants = {
    "slice order": items,
    "longest first": items[np.argsort(-kk, kind="stable")],
    "shortest first": items[np.argsort(kk, kind="stable")],
    "first 16384": items[:16384],
    "first 12288": items[:12288],
}
keep = []
for name, its in variants.items():
    d_items = torch.from_numpy(np.ascontiguousarray(its).view(np.int32)).cuda()
    keep.append(d_items)
    ms = []
    for r in range(6):
        ctx.gather_clustered(recs, d_items, len(its), d_out, d_ids)
        torch.cuda.synchronize()
        ms.append(ctx.last_kernel_ms())
    print(f"{name:16s} items {len(its):6d}  ms {np.round(ms[1:], 2)}  per item us {1e3 * np.median(ms[1:]) / len(its):.3f}",
          flush=True)
