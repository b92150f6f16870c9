"""The in-process multi-GPU path of the Mitsuba plugin (amdDevices): one
library integrator per device, each driven by its own host thread, the
slice-sharded prepass over alvrl_local_exchange (threads instead of
processes) and each integrator rendering its 64x64 tiles; the framebuffers'
sum is the frame.  Rehearsed here with two and three integrators on device 0:
cluster lists and frame bit-identical to one integrator."""
import threading

import numpy as np
import pytest

from test_gpu_parity import SEED_RNG, SEED_VRL

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,props", [(2, "targetNumSlices=40"),
                                         (3, "targetNumSlices=30;neighbourCount=2;neighbourWeight=0.5"),
                                         (3, "targetNumSlices=30;sliceSharding=roundrobin"),
                                         (2, "localRefinement=false;globalCluster=false")])
def test_local_exchange_integrators(gpu_ok, world, props):
    import torch
    import alvrl
    w, h = 256, 192
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, 3000, seed=SEED_VRL)

    def integrator():
        it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        return it

    one = integrator()
    one.prepass(4)
    ref = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    one.render(ref)
    torch.cuda.synchronize()
    ref_cl = one.clusters() if "localRefinement=false" not in props else None
    ref_st = one.stats()
    one.close()

    its = [integrator() for _ in range(world)]
    fbs = [torch.zeros(w * h * 3, dtype=torch.float32, device="cuda") for _ in range(world)]
    g = alvrl.LocalExchange(world)
    errs = []

    def run(r):
        try:
            its[r].prepass(4, r, world, g.rank(r))
            its[r].render(fbs[r], r, world)
            torch.cuda.synchronize()
        except Exception as e:   # reported below
            errs.append((r, e))

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join(300) for t in th]
    assert not errs, errs
    frame = sum(fbs)
    torch.cuda.synchronize()
    assert torch.equal(frame, ref)
    if ref_cl is not None:
        for r in range(world):
            cl = its[r].clusters()
            for k in ref_cl:
                assert np.array_equal(cl[k].view(np.uint32), ref_cl[k].view(np.uint32)), (r, k)
        # every slice refined once over the integrators: the ranks' shares
        # (longest processing time first by default, s mod N with
        # sliceSharding=roundrobin) partition the slices
        assert sum(it.stats()["slices_local"] for it in its) == ref_st["slices"]
        shares = [list(it.local_slices()) for it in its]
        assert sorted(s_ for sh in shares for s_ in sh) == list(range(ref_st["slices"])), shares
        if "roundrobin" in props:
            assert all(s_ % world == r for r, sh in enumerate(shares) for s_ in sh), shares
    for it in its:
        it.close()
    g.close()


def test_device_exchange_rccl(gpu_ok):
    """alvrl_device_exchange (the plugin's amdDevices over RCCL): a repeated
    device is refused; on every visible device (one on the test box) the
    exchange's all-gather, OR and cluster merge give what the host exchange
    gives, the framebuffer reduce is the sum, and the sharded prepass through
    it equals the one-GPU prepass."""
    import torch
    import alvrl
    with pytest.raises(alvrl.AlvrlError):
        alvrl.DeviceExchange([0, 0])
    n = torch.cuda.device_count()
    devs = list(range(n))
    g = alvrl.DeviceExchange(devs)
    try:
        out = [None] * n
        errs = []

        def run(r):
            try:
                torch.cuda.set_device(devs[r])
                rk = g.rank(r)
                data = np.arange(5 + r, dtype=np.uint8) * (r + 1)
                parts = rk.allgatherv(data)
                mask = np.zeros(64, np.uint8)
                mask[r::n + 1] = 1
                ored = rk.or_(mask)
                fb = torch.full((1000,), float(r + 1), device=f"cuda:{devs[r]}")
                g.reduce_frame(r, fb)
                torch.cuda.synchronize(devs[r])
                out[r] = (parts, ored, fb.cpu().numpy())
            except Exception as e:   # reported below
                errs.append((r, e))

        th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
        [t.start() for t in th]
        [t.join(120) for t in th]
        assert not errs, errs
        for r in range(n):
            parts, ored, fb = out[r]
            assert [p.tolist() for p in parts] == [(np.arange(5 + q, dtype=np.uint8) * (q + 1)).tolist()
                                                   for q in range(n)]
            ref = np.zeros(64, np.uint8)
            for q in range(n):
                ref[q::n + 1] = 1
            assert np.array_equal(ored, ref)
        assert np.all(out[0][2] == sum(range(1, n + 1)))   # rank 0 holds the sum
        if n == 1:
            # the sharded prepass over it (world 1) equals the plain prepass
            w, h = 128, 96
            scene = alvrl.scene_default(w, h)
            vrls, pc = alvrl.trace_vrls(scene, 1500, seed=SEED_VRL)
            res = []
            for sharded in (False, True):
                it = alvrl.Integrator(f"targetNumSlices=16;seed={SEED_RNG}", device=0)
                it.set_vrls(vrls, pc)
                it.preprocess(scene)
                if sharded:
                    import ctypes as C
                    assert it.L.alvrl_integrator_prepass_dist(it.h, 3, 0, 1, C.byref(g.rank(0).desc)) == 0
                else:
                    it.prepass(3)
                res.append(it.clusters())
                it.close()
            for k in res[0]:
                assert np.array_equal(res[0][k].view(np.uint32), res[1][k].view(np.uint32)), k
    finally:
        g.close()
