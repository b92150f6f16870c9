"""GPU parity of the medium's distance-sampling strategies (see
test_medium_strategies.py): the gathers' pdfFailure (brute, clustered and R
rows, on test_gpu_parity's tolerance), and the GPU tracer and volpath
reference (bit for bit) under 'single', 'manual' and 'maximum'."""
import numpy as np
import pytest

from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close, _assert_close_pairs, _ctx
from test_medium_strategies import STRATS, scene_with

pytestmark = pytest.mark.gpu

OTHER = [s for s in STRATS if s[0] != "balance"]


def _medium(alvrl, strategy, channel, density):
    return alvrl.Medium(strategy=strategy, channel=channel, sampling_density=density)


@pytest.mark.parametrize("strategy,channel,density", OTHER)
def test_gather_strategies(oracle, gpu_ok, strategy, channel, density):
    """Brute gather and R rows of a 48x32 frame under the strategy (VRLs
    traced under it too) against the oracle; short and long VRLs (short
    VRLs divide by the strategy's pdfFailure, vrlIntegrator.cpp:675-676, 750-751)."""
    import torch
    import alvrl
    w, h = 48, 32
    for short in (True, False):
        m = oracle.medium(strategy=strategy, channel=channel, density=density)
        sc = oracle.scene(w, h)
        vrls, pc = oracle.trace(sc, m, 1500, seed=SEED_VRL, short_vrls=short)
        recs = oracle.records(sc)
        P = oracle.params(m, seed=SEED_RNG, short_vrls=int(short))
        cpu, _ = oracle.gather_brute(P, recs, vrls, pc)
        ctx = _ctx(_medium(alvrl, strategy, channel, density), short_vrls=short)
        ctx.upload_vrls(vrls, pc)
        d_out = torch.zeros((len(recs), 3), dtype=torch.float32, device="cuda")
        d_recs = torch.from_numpy(recs).cuda()   # referenced until the kernel is done
        ctx.gather_brute(d_recs, d_out)
        torch.cuda.synchronize()
        _assert_close(d_out.cpu().numpy(), cpu, f"brute {strategy} short={short}")
        # with short VRLs the balance gather of the same records differs (the
        # strategy is not ignored); long VRLs do not divide by pdfFailure
        Pb = oracle.params(oracle.medium(), seed=SEED_RNG, short_vrls=int(short))
        base, _ = oracle.gather_brute(Pb, recs, vrls, pc)
        if short:
            assert np.abs(base - cpu).max() > 1e-3 * np.abs(cpu).max()
        ids = np.arange(0, w * h, 11, dtype=np.uint32)
        _, R, _ = oracle.gather_brute(P, recs[ids], vrls, pc, rec_ids=ids, want_R=True, domain=2)
        nr, nv = len(ids), vrls.shape[1]
        d_Rt = torch.zeros((nv, nr, 2), dtype=torch.float32, device="cuda")
        d_rr, d_ids = torch.from_numpy(recs[ids]).cuda(), torch.from_numpy(ids.view(np.int32)).cuda()
        ctx.build_R(d_rr, d_Rt, ld=nr, d_ids=d_ids)
        torch.cuda.synchronize()
        Rg = d_Rt.cpu().numpy().transpose(1, 0, 2)
        # one ill-conditioned pair in 10^5 (rel 1e-2, the tail of test_gpu_parity)
        # can dominate a column of 140 rows: column sums to 5e-3 here
        _assert_close_pairs(Rg[..., 0], R[..., 0], f"R mean {strategy}", csum=5e-3)
        ctx.close()


@pytest.mark.parametrize("strategy,channel,density", OTHER)
def test_gpu_tracer_and_volpath_strategies(oracle, gpu_ok, strategy, channel, density):
    """The GPU tracer == the host tracer, and the GPU volpath == the oracle's,
    bit for bit, under the strategy."""
    import alvrl
    s = scene_with(alvrl, 20, 14, strategy, channel, density)
    for target, short in ((20000, True), (5000, False)):
        dev, pcd = alvrl.trace_vrls_gpu(s, target, seed=SEED_VRL, short_vrls=short)
        host, pch = alvrl.trace_vrls(s, target, seed=SEED_VRL, short_vrls=short)
        assert pcd == pch
        assert np.array_equal(dev.view(np.uint32), host.view(np.uint32)), (strategy, target, short)
    m = oracle.medium(strategy=strategy, channel=channel, density=density)
    dev = alvrl.volpath_render(s, 16, seed=SEED_RNG, pass_=2).cpu().numpy()
    ref = oracle.volpath(oracle.scene(20, 14), m, 16, seed=SEED_RNG, pass_=2)
    assert np.array_equal(dev.view(np.uint32), ref.view(np.uint32)), np.abs(dev - ref).max()
    assert (dev > 0).any()


def test_integrator_strategy(oracle, gpu_ok):
    """A clustered prepass + render with the 'maximum' strategy through the
    integrator: the cluster lists equal the oracle's clustering of the
    device's R, and the frame the oracle's clustered gather with them."""
    import torch
    import alvrl
    from oracle import Prep
    w, h = 48, 32
    s = scene_with(alvrl, w, h, "maximum", -1, 0.0)
    m = oracle.medium(strategy="maximum")
    o = oracle.scene(w, h)
    vrls, pc = oracle.trace(o, m, 800, seed=SEED_VRL)
    it = alvrl.Integrator(f"targetNumSlices=12;seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(s)
    it.prepass(0)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    prep = Prep(oracle, oracle.prep_params(seed=SEED_RNG, pass_=0, target_num_slices=12))
    p2s = prep.build_slices(o)
    assert np.array_equal(p2s, it.slices())
    prep.sample_slice_mapping(64.0, w * h)
    icl = it.clusters()
    ocl = prep.build_clusters(it.R())
    assert np.array_equal(ocl["reps"], icl["reps"])
    assert np.array_equal(ocl["weights"].view(np.uint32), icl["weights"].view(np.uint32))
    pid = np.arange(w * h, dtype=np.uint32)
    sl = p2s[(pid % w) * h + pid // w]
    P = oracle.params(m, seed=SEED_RNG, pass_=0)
    cpu, _ = oracle.gather_clustered(P, oracle.records(o), sl, vrls, pc, icl["slice_off"], icl["reps"],
                                     icl["weights"], icl["fb_reps"], icl["fb_weights"], rec_ids=pid)
    _assert_close(fb.view(-1, 3).cpu().numpy(), cpu, "maximum-strategy frame")
    it.close()
