"""GPU parity of multi-sample renders (the sampler's sampleCount,
renderBlock's sample loop, integrator.cpp:240-264; test_spp.py has the host
side).  Bars: the device's jittered eye records equal the host's bit for
bit; the integrator's frame with sampleCount = 4 equals the oracle's gather
over the oracle's sensor-sample records (clustered with the device's lists,
or brute force), averaged per pixel, on test_gpu_parity's tolerance; the
samples are not all the same (the jittered frame differs from the
single-sample one)."""
import numpy as np
import pytest

from oracle import set_occluders
from test_chains import ALB, SPEC, chain_mesh
from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close

pytestmark = pytest.mark.gpu

SPP = 4


def test_records_spp_gpu_matches_host(gpu_ok):
    import alvrl
    w, h = 64, 48
    s = alvrl.scene_default(w, h)
    ids = np.arange(3, w * h, 7, dtype=np.uint32)
    for spp, pass_ in ((1, 0), (SPP, 0), (SPP, 5)):
        host = alvrl.scene_records_spp(s, spp, pixel_ids=ids, seed=SEED_RNG, pass_=pass_)
        dev = alvrl.scene_records_spp_gpu(s, spp, pixel_ids=ids, seed=SEED_RNG, pass_=pass_).cpu().numpy()
        assert np.array_equal(dev.view(np.uint32), host.view(np.uint32)), (spp, pass_)


def _frame(it, w, h):
    import torch
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    return fb.view(h * w, 3).cpu().numpy()


def _mean_per_pixel(vals, pix, npix, spp):
    out = np.zeros((npix, 3), np.float64)
    np.add.at(out, pix, vals.astype(np.float64))
    return (out / spp).astype(np.float32)


@pytest.mark.parametrize("props,mirrors", [("targetNumSlices=12", False),
                                           ("localRefinement=false;globalCluster=false", False),
                                           ("targetNumSlices=12", True)])
def test_integrator_sample_count_matches_oracle(oracle, gpu_ok, props, mirrors):
    import alvrl
    w, h, pass_ = 48, 32, 1
    s = alvrl.scene_default(w, h)
    o = oracle.scene(w, h)
    m = oracle.medium()
    P = oracle.params(m, seed=SEED_RNG, pass_=pass_)
    if mirrors:
        tris, mat = chain_mesh()
        s = alvrl.scene_set_occluders(s, tris, ALB, material=mat, specular=SPEC)
        o = set_occluders(o, tris, ALB, material=mat, specular=SPEC)
        P = set_occluders(P, tris, material=mat)
    vrls, pc = oracle.trace(o, m, 800, seed=SEED_VRL)
    pid = np.arange(w * h, dtype=np.uint32)
    if mirrors:
        recs, pix = [], []
        for j in range(SPP):
            for p in pid:
                c = oracle.chain_s(o, m, int(p % w), int(p // w), j, SPP, seed=SEED_RNG, pass_=pass_)
                recs.append(c)
                pix.append(np.full(len(c), p, np.uint32))
        recs, pix = np.concatenate(recs), np.concatenate(pix)
        assert (recs[:, 19].view(np.uint32) & 0xFFFF).max() >= 1
    else:
        recs, pix = oracle.records_spp(o, pid, SPP, seed=SEED_RNG, pass_=pass_)
    imgs = {}
    for spp in (1, SPP):
        it = alvrl.Integrator(props + f";seed={SEED_RNG};sampleCount={spp}", device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(s)
        it.prepass(pass_)
        imgs[spp] = _frame(it, w, h)
        if spp == SPP:
            if "localRefinement=false" in props:
                cpu, _ = oracle.gather_brute(P, recs, vrls, pc, rec_ids=pix)
            else:
                p2s = it.slices()
                icl = it.clusters()
                sl_pix = p2s[(pid % w) * h + pid // w]
                cpu, _ = oracle.gather_clustered(P, recs, sl_pix[pix], vrls, pc, icl["slice_off"], icl["reps"],
                                                 icl["weights"], icl["fb_reps"], icl["fb_weights"], rec_ids=pix)
            _assert_close(imgs[spp], _mean_per_pixel(cpu, pix, w * h, SPP), f"sampleCount={SPP} frame ({props})")
        it.close()
    # the sensor samples are jittered: the frames differ, their totals agree
    assert not np.array_equal(imgs[1], imgs[SPP])
    t1, t4 = float(imgs[1].sum()), float(imgs[SPP].sum())
    assert abs(t4 - t1) < 0.1 * abs(t1)
