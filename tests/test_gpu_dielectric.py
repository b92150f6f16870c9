"""GPU parity for dielectric occluders (test_dielectric.py): the integrator
over a scene whose eye paths branch into reflection and refraction at glass
(LiInternal's component loop, vrlIntegrator.cpp:464-511), and the same scene
through the host-cast ABI (alvrl_integrator_prepass_records with the
branching records the host forms).

Bars as in test_gpu_chains.py: slices and representatives bit-exact against
the oracle; R rows (every record of a row's tree added into it) and frames on
test_gpu_parity's tolerance; cluster lists bit-exact against the oracle's
clustering of the device's R; the host-cast pipeline bit-identical to the
descriptor pipeline."""
import numpy as np
import pytest

from oracle import set_occluders
from test_chains import ALB, SPEC
from test_dielectric import ETA, glass_mesh
from test_gpu_chains import _per_pixel
from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close, _assert_close_pairs

pytestmark = pytest.mark.gpu


def _setup(oracle, w, h, nvrl, pass_):
    import alvrl
    tris, mat = glass_mesh()
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, material=mat, specular=SPEC, eta=ETA)
    o = set_occluders(oracle.scene(w, h), tris, ALB, material=mat, specular=SPEC, eta=ETA)
    m = oracle.medium()
    vrls, pc = oracle.trace(o, m, nvrl, seed=SEED_VRL)
    P = set_occluders(oracle.params(m, seed=SEED_RNG, pass_=pass_), tris, material=mat)
    return s, o, m, tris, mat, vrls, pc, P


@pytest.mark.parametrize("props", ["targetNumSlices=12", "localRefinement=false;globalCluster=false"])
def test_integrator_dielectric_matches_oracle(oracle, gpu_ok, props):
    import torch
    import alvrl
    from oracle import Prep
    w, h, pass_ = 48, 32, 1
    s, o, m, tris, mat, vrls, pc, P = _setup(oracle, w, h, 800, pass_)
    it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
    try:
        it.set_vrls(vrls, pc)
        it.preprocess(s)
        it.prepass(pass_)
        fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        it.render(fb)
        torch.cuda.synchronize()
        img = fb.view(h * w, 3).cpu().numpy()
        pid = np.arange(w * h, dtype=np.uint32)
        recs, pix = oracle.chains(o, m, pid, seed=SEED_RNG, pass_=pass_)
        # the trees branch: more records than the longest chain per pixel would give
        assert len(recs) > 1.5 * w * h
        if "localRefinement=false" in props:
            cpu, _ = oracle.gather_brute(P, recs, vrls, pc, rec_ids=pix)
            _assert_close(img, _per_pixel(cpu, pix, w * h), "brute dielectric frame")
            return
        prep = Prep(oracle, oracle.prep_params(seed=SEED_RNG, pass_=pass_, target_num_slices=12))
        p2s = prep.build_slices(o)
        assert np.array_equal(p2s, it.slices())
        off, rpix, _, _ = prep.sample_slice_mapping(64.0, w * h)
        ioff, ipix = it.reps()
        assert np.array_equal(off, ioff) and np.array_equal(rpix, ipix)
        rid = ((ipix % h) * w + ipix // h).astype(np.uint32)
        rrecs, rr = oracle.chains(o, m, rid, seed=SEED_RNG, pass_=pass_)
        _, Rr, _ = oracle.gather_brute(P, rrecs, vrls, pc, rec_ids=rr, want_R=True, domain=2)
        row_of = {int(p): j for j, p in enumerate(rid)}
        row = np.array([row_of[int(p)] for p in rr], np.int64)
        Rc = _per_pixel(Rr, row, len(rid))
        Rg = it.R()
        _assert_close_pairs(Rg[..., 0].T, Rc[..., 0], "dielectric R mean")
        icl = it.clusters()
        ocl = prep.build_clusters(Rg)
        assert np.array_equal(ocl["reps"], icl["reps"])
        assert np.array_equal(ocl["weights"].view(np.uint32), icl["weights"].view(np.uint32))
        sl_pix = p2s[(pid % w) * h + pid // w]
        cpu, _ = oracle.gather_clustered(P, recs, sl_pix[pix], vrls, pc, icl["slice_off"], icl["reps"],
                                         icl["weights"], icl["fb_reps"], icl["fb_weights"], rec_ids=pix)
        _assert_close(img, _per_pixel(cpu, pix, w * h), "clustered dielectric frame")
    finally:
        it.close()


def test_ext_scene_dielectric_matches_descriptor(gpu_ok):
    """The host-cast pipeline over branching records: the host's eye-path
    trees for R (alvrl_scene_chain, the plugin's appendPath) through
    alvrl_integrator_prepass_records give the descriptor pipeline's R and
    cluster lists bit for bit."""
    import alvrl
    from test_gpu_ext_scene import _paths, _slice_recs
    w, h, pass_ = 48, 32, 2
    tris, mat = glass_mesh()
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, material=mat, specular=SPEC, eta=ETA)
    vrls, pc = alvrl.trace_vrls(s, 2500, seed=SEED_VRL)
    props = f"targetNumSlices=10;seed={SEED_RNG}"
    a = alvrl.Integrator(props, device=0)
    b = alvrl.Integrator(props, device=0)
    try:
        a.set_vrls(vrls, pc)
        a.preprocess(s)
        a.prepass(pass_)
        b.set_vrls(vrls, pc)
        b.preprocess_ext(w, h, _slice_recs(s, w, h), list(s.box_min), list(s.box_max), alvrl.Medium(), tris, mat)
        pix = b.rep_pixels(pass_)
        recs, rows = _paths(s, pix, w, pass_)
        b.prepass_records(pass_, recs, rows)
        ca, cb = a.clusters(), b.clusters()
        for k in ca:
            assert np.array_equal(ca[k].view(np.uint32), cb[k].view(np.uint32)), k
        assert np.array_equal(a.R().view(np.uint32), b.R().view(np.uint32))
    finally:
        a.close()
        b.close()
