"""Host-cast scenes (alvrl_integrator_preprocess_ext / _rep_pixels /
_prepass_records / _set_cluster_info, include/alvrl_host.h): the entry points
the Mitsuba plugin's records mode drives when Mitsuba casts every ray itself
(mitsuba_plugin/vrlAmdIntegrator.cpp).

The host here plays Mitsuba with the library's own smoke-box scene (occluders
with diffuse, mirror and null BSDFs, so the eye paths branch into delta
chains): its gather points for buildSlices (Preprocessor.cpp:1140-1170), its
representative pixels' eye paths for R (vrlIntegrator.cpp:322-330 ->
LiInternal :445-511) and its render records.  Fed the same rays, the
record-driven pipeline must give the descriptor-driven pipeline's slices,
representatives, R, cluster lists and frame bit for bit."""
import numpy as np
import pytest

from test_chains import ALB, SPEC, chain_mesh
from test_gpu_parity import SEED_RNG, SEED_VRL

pytestmark = pytest.mark.gpu


def _scene(w, h):
    import alvrl
    tris, mat = chain_mesh()
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, material=mat, specular=SPEC)
    return s, tris, mat


def _slice_recs(s, w, h):
    import alvrl
    return np.stack([alvrl.scene_slice_record(s, x, y) for y in range(h) for x in range(w)])


def _paths(s, pix, w, pass_):
    """LiInternal's eye path of each pixel (alvrl_scene_chain): records and
    the index into pix of each."""
    import alvrl
    recs, own = [], []
    for i, p in enumerate(pix):
        ch = alvrl.scene_chain(s, int(p) % w, int(p) // w, seed=SEED_RNG, pass_=pass_)
        recs.append(ch)
        own += [i] * len(ch)
    return np.concatenate(recs), np.array(own, np.uint32)


def _ext_integrator(props, s, w, h, tris, mat, vrls, pc):
    import alvrl
    it = alvrl.Integrator(props, device=0)
    it.set_vrls(vrls, pc)
    it.preprocess_ext(w, h, _slice_recs(s, w, h), list(s.box_min), list(s.box_max), alvrl.Medium(), tris, mat)
    return it


def test_ext_scene_matches_descriptor(gpu_ok):
    import torch
    import alvrl
    w, h, pass_ = 48, 32, 1
    s, tris, mat = _scene(w, h)
    vrls, pc = alvrl.trace_vrls(s, 3000, seed=SEED_VRL)
    props = f"targetNumSlices=12;seed={SEED_RNG}"
    a = alvrl.Integrator(props, device=0)
    a.set_vrls(vrls, pc)
    a.preprocess(s)
    a.prepass(pass_)
    fa = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    a.render(fa)
    torch.cuda.synchronize()
    img_a = fa.view(-1, 3).cpu().numpy()
    cl_a, R_a, p2s_a = a.clusters(), a.R(), a.slices()
    off_a, rep_a = a.reps()

    b = _ext_integrator(props, s, w, h, tris, mat, vrls, pc)
    try:
        assert np.array_equal(b.slices(), p2s_a)
        pix = b.rep_pixels(pass_)
        assert np.array_equal(pix, (rep_a % h) * w + rep_a // h)         # x*H + y -> y*W + x
        recs, rows = _paths(s, pix, w, pass_)
        assert len(recs) > len(pix)                                       # chains: rows with several segments
        b.prepass_records(pass_, recs, rows)
        cl_b = b.clusters()
        for k in cl_a:
            assert np.array_equal(cl_a[k].view(np.uint32), cl_b[k].view(np.uint32)), k
        assert np.array_equal(R_a.view(np.uint32), b.R().view(np.uint32))
        st_a, st_b = a.stats(), b.stats()
        assert st_a["contrib_preprocess"] == st_b["contrib_preprocess"] > 0
        # render: the host's eye paths of every pixel through the context's gather
        allpix = np.arange(w * h, dtype=np.uint32)
        recs, own = _paths(s, allpix, w, pass_)
        pid = allpix[own]
        sl = p2s_a[(pid % w) * h + pid // w]                               # m_slices[y + H*x]
        rgb = b.context().gather_clustered_host(recs, sl, ids=pid)
        img_b = np.zeros((w * h, 3), np.float32)
        for k in range(len(recs)):                                         # depth order within a pixel
            img_b[pid[k]] += rgb[k]
        assert img_a.any()
        assert np.array_equal(img_a.view(np.uint32), img_b.view(np.uint32))
        with pytest.raises(alvrl.AlvrlError):                              # no camera of its own
            b.render(torch.zeros(w * h * 3, dtype=torch.float32, device="cuda"))
    finally:
        a.close()
        b.close()


def test_ext_scene_misses_and_empty_rows(gpu_ok):
    """Pixels whose centre ray leaves the scene (no HIT in the slicing record)
    get no slice, which makes the fall-back clustering necessary (:564-571);
    a representative row whose eye path has no record is a zero row of R."""
    import alvrl
    w, h, pass_ = 40, 30, 0
    s, tris, mat = _scene(w, h)
    vrls, pc = alvrl.trace_vrls(s, 2000, seed=SEED_VRL)
    sr = _slice_recs(s, w, h)
    flags = sr[:, 15].view(np.uint32)
    flags[: 3 * w] &= ~np.uint32(alvrl.REC_HIT)                            # the top three image rows miss
    b = alvrl.Integrator(f"targetNumSlices=10;seed={SEED_RNG}", device=0)
    try:
        b.set_vrls(vrls, pc)
        b.preprocess_ext(w, h, sr, list(s.box_min), list(s.box_max), alvrl.Medium(), tris, mat)
        p2s = b.slices()
        y = np.arange(w * h) % h                                           # column-major: index x*H + y
        assert (p2s[y < 3] == 0xFFFFFFFF).all() and (p2s[y >= 3] != 0xFFFFFFFF).all()
        pix = b.rep_pixels(pass_)
        assert (pix // w >= 3).all()
        recs, rows = _paths(s, pix, w, pass_)
        drop = np.isin(rows, [0, 5])                                       # rows 0 and 5 get no records
        b.prepass_records(pass_, recs[~drop], rows[~drop])
        R = b.R()
        assert not R[:, [0, 5], :].any() and R[:, 1, 0].any()
        st = b.stats()
        assert st["fallback_built"] == 1 and st["slices_failed"] == 0
        cl = b.clusters()
        assert len(cl["fb_reps"]) > 0
        # a second prepass without records is refused, as is one without VRLs
        with pytest.raises(alvrl.AlvrlError):
            b.prepass(pass_)
    finally:
        b.close()


def test_set_cluster_info_in_memory(gpu_ok):
    """wakeup (vrlIntegrator.cpp:378-384): a render worker installs the
    vrlClusterInfo it receives instead of running the prepass; its frame is
    the prepass integrator's bit for bit."""
    import torch
    import alvrl
    w, h, pass_ = 48, 32, 2
    s, tris, mat = _scene(w, h)
    vrls, pc = alvrl.trace_vrls(s, 2500, seed=SEED_VRL)
    props = f"targetNumSlices=8;seed={SEED_RNG}"
    a = alvrl.Integrator(props, device=0)
    c = alvrl.Integrator(props, device=0)
    try:
        for it in (a, c):
            it.set_vrls(vrls, pc)
            it.preprocess(s)
        a.prepass(pass_)
        cl = a.clusters()
        cl["slices"] = a.slices()
        c.set_cluster_info(cl, pass_)
        fa = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        fc = torch.zeros_like(fa)
        a.render(fa)
        c.render(fc)
        torch.cuda.synchronize()
        assert fa.abs().sum() > 0 and torch.equal(fa, fc)
        bad = dict(cl)
        bad["slice_off"] = cl["slice_off"][:-1].copy()                   # inconsistent sizes
        with pytest.raises(alvrl.AlvrlError):
            c.set_cluster_info(bad, pass_)
    finally:
        a.close()
        c.close()
