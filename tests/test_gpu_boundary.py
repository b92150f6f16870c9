"""The C ABI under the reference's threading model.

Mitsuba calls renderBlock -> Li from every LocalWorker thread at once on one
shared integrator (src/librender/renderproc.cpp:52-86), one 32x32 image block
per call (the default blockSize, src/librender/renderjob.cpp).  The gathers of
include/alvrl.h must therefore be reentrant on one context: each calling
thread gets its own stream and device scratch (csrc/capi.hip ThreadSlot).

  * 8 host threads render a frame block by block through
    alvrl_gather_clustered_host / alvrl_gather_brute_host; the assembled frame
    equals the one-call frame bit for bit (every pixel's sum depends only on
    its record, id and slice list), and the concurrent calls were merged into
    fewer launches (the library's host-gather batching), also for calls
    without record ids;
  * alvrl_set_clusters right after a gather launched on a caller's stream:
    the gather still sees the lists it was launched with (set_clusters waits
    for it, alvrl.h).
"""
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_VRL = 0x5EED0001
SEED_RNG = 0xA1B2C3D4


def _setup(w, h, nvrl, props):
    import alvrl
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, nvrl, seed=SEED_VRL)
    it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(scene)
    it.prepass(0)
    cl = it.clusters()
    p2s = it.slices()
    it.close()
    ctx = alvrl.Context(device=0, seed=SEED_RNG)
    ctx.set_medium(alvrl.Medium())
    ctx.upload_vrls(vrls, pc)
    ctx.set_clusters(cl["slice_off"], cl["reps"], cl["weights"], cl["fb_reps"], cl["fb_weights"])
    recs = alvrl.scene_records(scene)                      # row-major pixel ids
    pid = np.arange(w * h, dtype=np.uint32)
    sl = p2s[(pid % w) * h + pid // w]                     # m_slices[y + H*x]
    return ctx, recs, sl, cl


def _blocks(w, h, b=32):
    out = []
    for y0 in range(0, h, b):
        for x0 in range(0, w, b):
            ys, xs = np.mgrid[y0:min(y0 + b, h), x0:min(x0 + b, w)]
            out.append((ys * w + xs).ravel().astype(np.uint32))
    return out


@pytest.mark.parametrize("mode", ["clustered", "brute"])
def test_concurrent_block_gathers(gpu_ok, mode):
    w, h = 320, 256
    ctx, recs, sl, _ = _setup(w, h, 3000, "targetNumSlices=40")
    pid = np.arange(w * h, dtype=np.uint32)

    def gather(ids):
        if mode == "clustered":
            return ctx.gather_clustered_host(recs[ids], sl[ids], ids=ids)
        return ctx.gather_brute_host(recs[ids], ids=ids)

    t0 = time.perf_counter()
    whole = gather(pid)
    t_whole = time.perf_counter() - t0
    blocks = _blocks(w, h)
    frame = np.zeros((w * h, 3), np.float32)
    for rep in range(2):   # the second round re-uses every thread's stream and scratch
        frame[:] = 0
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=8) as ex:
            for ids, out in zip(blocks, ex.map(gather, blocks)):
                frame[ids] = out
        t_blocks = time.perf_counter() - t0
        assert np.array_equal(frame.view(np.uint32), whole.view(np.uint32)), rep
    assert whole.any()
    # concurrent calls were merged into fewer launches (csrc/capi.hip host_gather)
    nb, nr = ctx.host_batch_stats()[mode]
    assert nr == 1 + 2 * len(blocks) and nb < nr, (nb, nr)
    print(f"{mode}: {nr} requests in {nb} launches")
    # without ids a record's streams are keyed by its index in its own call,
    # also when its call is merged with others
    sub = [b[:300] for b in blocks[:24]]

    def gather_noid(ids):
        if mode == "clustered":
            return ctx.gather_clustered_host(recs[ids], sl[ids])
        return ctx.gather_brute_host(recs[ids])

    alone = [gather_noid(ids) for ids in sub]
    with ThreadPoolExecutor(max_workers=8) as ex:
        merged = list(ex.map(gather_noid, sub))
    for a, m in zip(alone, merged):
        assert np.array_equal(a.view(np.uint32), m.view(np.uint32))
    print(f"{mode}: {len(blocks)} blocks of 32x32 on 8 threads {t_blocks * 1e3:.1f} ms, "
          f"one call {t_whole * 1e3:.1f} ms")


def test_set_clusters_waits_for_running_gather(gpu_ok):
    """alvrl_set_clusters overwrites the lists in place; a gather
    launched on a caller's stream just before must finish with the old lists."""
    import torch
    import alvrl
    w, h = 512, 384
    ctx, recs, sl, cl = _setup(w, h, 6000, "targetNumSlices=30;localUndersampling=4")
    order = np.argsort(sl, kind="stable").astype(np.uint32)
    items = alvrl.Context.make_work_items(sl[order])
    d_recs = torch.from_numpy(recs[order]).cuda()
    d_ids = torch.from_numpy(order.view(np.int32)).cuda()
    d_items = torch.from_numpy(items.view(np.int32)).cuda()
    ref = torch.zeros((w * h, 3), dtype=torch.float32, device="cuda")
    ctx.gather_clustered(d_recs, d_items, len(items), ref, d_ids=d_ids)
    torch.cuda.synchronize()
    # other lists: every slice's list replaced by its first entry at weight 1
    so = cl["slice_off"]
    reps2 = cl["reps"][so[:-1]]
    w2 = np.ones(len(reps2), np.float32)
    so2 = np.arange(len(so), dtype=np.uint32)
    s = torch.cuda.Stream()
    out = torch.zeros_like(ref)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        ctx.gather_clustered(d_recs, d_items, len(items), out, d_ids=d_ids, stream=s.cuda_stream)
    ctx.set_clusters(so2, reps2, w2, cl["fb_reps"], cl["fb_weights"])   # right after the launch
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    after = torch.zeros_like(ref)
    ctx.gather_clustered(d_recs, d_items, len(items), after, d_ids=d_ids)
    torch.cuda.synchronize()
    assert not torch.equal(after, ref)


@pytest.mark.parametrize("samples", [2, 3])
def test_split_gather_same_bits(gpu_ok, samples, monkeypatch):
    """Host batches too small to fill the chip (renderBlock-sized calls) take
    the split gather (csrc/gather.hip k_gather_split_pairs / _sum: a wave per
    chunk of a representative list, the pairs added in list order afterwards).
    Its frame equals the one-wave-per-item kernel's (the device-pointer
    alvrl_gather_clustered) bit for bit: forced on, forced off, and in 32x32
    blocks from 8 threads; samples = 3 takes the generic (not unrolled) form."""
    import torch
    import alvrl
    w, h = 320, 256
    ctx, recs, sl, cl = _setup(w, h, 3000, "targetNumSlices=40")
    if samples != 2:
        scene = alvrl.scene_default(w, h)
        vrls, pc = alvrl.trace_vrls(scene, 3000, seed=SEED_VRL)
        ctx = alvrl.Context(device=0, vol_vol_samples=samples, vol_surf_samples=samples, seed=SEED_RNG)
        ctx.set_medium(alvrl.Medium())
        ctx.upload_vrls(vrls, pc)
        ctx.set_clusters(cl["slice_off"], cl["reps"], cl["weights"], cl["fb_reps"], cl["fb_weights"])
    pid = np.arange(w * h, dtype=np.uint32)
    order = np.argsort(sl, kind="stable").astype(np.uint32)
    items = alvrl.Context.make_work_items(sl[order])
    ref = torch.zeros((w * h, 3), dtype=torch.float32, device="cuda")
    ctx.gather_clustered(torch.from_numpy(recs[order]).cuda(), torch.from_numpy(items.view(np.int32)).cuda(),
                         len(items), ref, d_ids=torch.from_numpy(order.view(np.int32)).cuda())
    torch.cuda.synchronize()
    # the device-pointer gather writes record order[i]'s result at row i
    ref_px = np.zeros((w * h, 3), np.float32)
    ref_px[order] = ref.cpu().numpy()
    assert ref_px.any()
    for mode in ("0", "1"):
        monkeypatch.setenv("ALVRL_HOST_SPLIT", mode)
        whole = ctx.gather_clustered_host(recs, sl, ids=pid)
        same = whole.view(np.uint32) == ref_px.view(np.uint32)
        rel = np.abs(whole.astype(np.float64) - ref_px) / np.maximum(np.abs(ref_px), 1e-30)
        print(f"ALVRL_HOST_SPLIT={mode}: {same.mean():.6f} of the values equal, max rel {rel.max():.3e}")
        assert same.all(), f"ALVRL_HOST_SPLIT={mode}"
    monkeypatch.delenv("ALVRL_HOST_SPLIT")
    frame = np.zeros((w * h, 3), np.float32)
    blocks = _blocks(w, h)
    with ThreadPoolExecutor(max_workers=8) as ex:
        for ids, out in zip(blocks, ex.map(lambda ids: ctx.gather_clustered_host(recs[ids], sl[ids], ids=ids),
                                           blocks)):
            frame[ids] = out
    assert np.array_equal(frame.view(np.uint32), ref_px.view(np.uint32)), "32x32 blocks"
