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
        # every slice refined once over the integrators
        assert sum(it.stats()["slices_local"] for it in its) == ref_st["slices"]
    for it in its:
        it.close()
    g.close()
