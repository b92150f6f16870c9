"""GPU parity for scenes with occluders: the device BVH
(csrc/bvh_device.hpp over host/bvh.cpp) behind the GPU tracer, the GPU
eye-ray first hit (alvrl_scene_records_gpu) and the gathers' shadow tests
(Scene::evalTransmittance's occluder test, scene.cpp:619-679).

Bars: the tracer and the eye records are BIT-IDENTICAL to the host (and so to
the oracle, test_occluders.py): the same triangle arithmetic, the closest hit
with ties to the lowest triangle index.  Gathers and R entries: the
tolerance of test_gpu_parity.py (the gather's fast maths can flip the
visibility of a sample that grazes an edge; none of the pixel-level bounds
needs loosening).  Slicing and the cluster lists of a prepass over the
occluded scene: identical to the oracle on the device's R."""
import numpy as np
import pytest

from oracle import set_occluders
from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close, _assert_close_pairs, _ctx

pytestmark = pytest.mark.gpu

ALB = (0.7, 0.4, 0.25)


def sphere_mesh(c, r, n_lat=24, n_lon=48):
    """UV sphere with outward normals (n_lat * n_lon * 2 - 2 n_lon triangles)."""
    c = np.asarray(c, np.float64)
    th = np.linspace(0.0, np.pi, n_lat + 1)
    ph = np.linspace(0.0, 2 * np.pi, n_lon + 1)
    P = np.stack([np.sin(th)[:, None] * np.cos(ph)[None], np.cos(th)[:, None] * np.ones_like(ph)[None],
                  np.sin(th)[:, None] * np.sin(ph)[None]], -1) * r + c
    tris = []
    for i in range(n_lat):
        for j in range(n_lon):
            a, b, d, e = P[i, j], P[i + 1, j], P[i + 1, j + 1], P[i, j + 1]
            if i > 0:
                tris.append(np.concatenate([a, e, b]))
            if i < n_lat - 1:
                tris.append(np.concatenate([b, e, d]))
    t = np.asarray(tris, np.float32)
    # orient outward
    v = t.reshape(-1, 3, 3).astype(np.float64)
    n = np.cross(v[:, 1] - v[:, 0], v[:, 2] - v[:, 0])
    flip = (n * (v.mean(1) - c)).sum(1) < 0
    t3 = t.reshape(-1, 3, 3)
    t3[flip] = t3[flip][:, [0, 2, 1]]
    return t3.reshape(-1, 9)


def scene_mesh(alvrl, big=False):
    from test_occluders import occluder_mesh
    m = occluder_mesh(alvrl)
    if big:
        m = np.concatenate([m, sphere_mesh([-0.45, 0.25, 0.45], 0.28), sphere_mesh([0.5, -0.55, 0.1], 0.2, 16, 32)])
    return m


def test_gpu_records_occluders(gpu_ok):
    """alvrl_scene_records_gpu == alvrl_scene_records bit for bit: all pixels
    of a 256x192 frame over ~4k triangles (BVH depth ~10), and a pixel
    subset; without occluders it equals the convex records."""
    import alvrl
    for big in (False, True):
        tris = scene_mesh(alvrl, big)
        s = alvrl.scene_set_occluders(alvrl.scene_default(256, 192), tris, ALB)
        host = alvrl.scene_records(s)
        dev = alvrl.scene_records_gpu(s).cpu().numpy()
        assert np.array_equal(dev.view(np.uint32), host.view(np.uint32)), f"big={big}: {np.argwhere(dev != host)[:5]}"
        ids = np.arange(7, 256 * 192, 97, dtype=np.uint32)
        sub = alvrl.scene_records_gpu(s, pixel_ids=ids).cpu().numpy()
        assert np.array_equal(sub.view(np.uint32), host[ids].view(np.uint32))
    plain = alvrl.scene_default(64, 48)
    assert np.array_equal(alvrl.scene_records_gpu(plain).cpu().numpy().view(np.uint32),
                          alvrl.scene_records(plain).view(np.uint32))


def test_gpu_tracer_occluders(gpu_ok):
    """The GPU tracer over the BVH == the host tracer's brute-force loop, bit
    for bit (short and long VRLs, HG-free default medium, 20k and 100k VRLs)."""
    import alvrl
    tris = scene_mesh(alvrl, big=True)
    s = alvrl.scene_set_occluders(alvrl.scene_default(16, 16), tris, ALB)
    for target, short in ((20000, True), (6000, False), (100003, True)):
        dev, pcd = alvrl.trace_vrls_gpu(s, target, seed=SEED_VRL, short_vrls=short)
        host, pch = alvrl.trace_vrls(s, target, seed=SEED_VRL, short_vrls=short)
        assert pcd == pch
        assert np.array_equal(dev.view(np.uint32), host.view(np.uint32)), (target, short)


def test_gpu_occluder_albedos(gpu_ok):
    """Per-triangle reflectances (alvrl_scene_desc.occluder_albedos) on the
    device: the eye-record kernel and the GPU tracer equal the host (and so
    the oracle, test_occluders.py) bit for bit, with the BVH's triangle order
    mapped back to each triangle's own reflectance."""
    import alvrl
    from test_occluders import per_triangle_albedos
    tris = scene_mesh(alvrl, big=True)
    alb = per_triangle_albedos(len(tris))
    alb[30:] = np.random.default_rng(5).uniform(0.0, 1.0, (len(tris) - 30, 3)).astype(np.float32)
    s = alvrl.scene_set_occluders(alvrl.scene_default(256, 192), tris, ALB, albedos=alb)
    host = alvrl.scene_records(s)
    dev = alvrl.scene_records_gpu(s).cpu().numpy()
    assert np.array_equal(dev.view(np.uint32), host.view(np.uint32))
    s16 = alvrl.scene_set_occluders(alvrl.scene_default(16, 16), tris, ALB, albedos=alb)
    for target, short in ((20000, True), (6000, False)):
        d, pcd = alvrl.trace_vrls_gpu(s16, target, seed=SEED_VRL, short_vrls=short)
        h, pch = alvrl.trace_vrls(s16, target, seed=SEED_VRL, short_vrls=short)
        assert pcd == pch and np.array_equal(d.view(np.uint32), h.view(np.uint32)), (target, short)


def test_gather_brute_occluders(oracle, gpu_ok):
    """Brute gather with shadow tests vs the oracle's (evalTransmittance with
    the occluders), 64x48 records x 2000 VRLs traced in the occluded scene;
    the occluders change the image (shadows), so the test is not vacuous."""
    import torch
    import alvrl
    tris = scene_mesh(alvrl, big=True)
    o = set_occluders(oracle.scene(64, 48), tris, ALB)
    m = oracle.medium()
    vrls, pc = oracle.trace(o, m, 2000, seed=SEED_VRL)
    recs = oracle.records(o)
    P = set_occluders(oracle.params(m, seed=SEED_RNG), tris)
    cpu, ccnt = oracle.gather_brute(P, recs, vrls, pc)
    P0 = oracle.params(m, seed=SEED_RNG)
    cpu_open, _ = oracle.gather_brute(P0, recs, vrls, pc)
    assert np.abs(cpu - cpu_open).max() > 0.05 * np.abs(cpu_open).max()
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    ctx.set_occluders(tris)
    d_out = torch.zeros((recs.shape[0], 3), dtype=torch.float32, device="cuda")
    ctx.gather_brute(torch.from_numpy(recs).cuda(), d_out)
    torch.cuda.synchronize()
    _assert_close(d_out.cpu().numpy(), cpu, "brute occluded 64x48x2k")
    ctx.set_occluders(np.zeros((0, 9), np.float32))   # back to the convex container
    d_out.zero_()
    ctx.gather_brute(torch.from_numpy(recs).cuda(), d_out)
    torch.cuda.synchronize()
    _assert_close(d_out.cpu().numpy(), cpu_open, "brute occluders removed")


def test_rbuild_occluders(oracle, gpu_ok):
    """R rows with shadow tests vs the oracle's (float pairs)."""
    import torch
    import alvrl
    tris = scene_mesh(alvrl, big=True)
    o = set_occluders(oracle.scene(40, 30), tris, ALB)
    m = oracle.medium()
    vrls, pc = oracle.trace(o, m, 1500, seed=SEED_VRL)
    recs = oracle.records(o)
    ids = np.arange(0, 40 * 30, 7, dtype=np.uint32)
    P = set_occluders(oracle.params(m, seed=SEED_RNG), tris)
    _, R, _ = oracle.gather_brute(P, recs[ids], vrls, pc, rec_ids=ids, want_R=True, domain=2)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    ctx.set_occluders(tris)
    nr, nv = len(ids), vrls.shape[1]
    d_Rt = torch.zeros((nv, nr, 2), dtype=torch.float32, device="cuda")
    ctx.build_R(torch.from_numpy(recs[ids]).cuda(), d_Rt, ld=nr, d_ids=torch.from_numpy(ids.view(np.int32)).cuda())
    torch.cuda.synchronize()
    Rg = d_Rt.cpu().numpy().transpose(1, 0, 2)
    _assert_close_pairs(Rg[..., 0], R[..., 0], "R mean occluded")
    # a sample whose shadow ray grazes an edge can flip between the device's
    # reduced-form U and the oracle's point construction; in the variance
    # (M2 of 4 samples) one flip moves a column sum by a few 1e-3
    _assert_close_pairs(Rg[..., 1], R[..., 1], "R var occluded", q50=1e-5, csum=1e-2)


def test_integrator_occluders_matches_oracle(oracle, gpu_ok):
    """A clustered prepass over the occluded scene: GPU records and tracer,
    slicing, the R build with shadow tests and the refinement; the slices
    equal the oracle's and the cluster lists equal the oracle's clustering
    of the device's R, bit for bit; the rendered frame is finite."""
    import torch
    import alvrl
    from oracle import Prep
    w, h = 48, 32
    tris = scene_mesh(alvrl, big=True)
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB)
    o = set_occluders(oracle.scene(w, h), tris, ALB)
    vrls, pc = oracle.trace(o, oracle.medium(), 600, seed=SEED_VRL)
    it = alvrl.Integrator(f"targetNumSlices=12;seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(s)
    it.prepass(0)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    prep = Prep(oracle, oracle.prep_params(seed=SEED_RNG, pass_=0, target_num_slices=12))
    assert np.array_equal(prep.build_slices(o), it.slices())
    prep.sample_slice_mapping(64.0, w * h)
    ocl, icl = prep.build_clusters(it.R()), it.clusters()
    assert np.array_equal(ocl["reps"], icl["reps"])
    assert np.array_equal(ocl["weights"].view(np.uint32), icl["weights"].view(np.uint32))
    assert np.isfinite(fb.cpu().numpy()).all()
    it.close()


def test_default_pipeline_occluder_albedos_vs_oracle_pipeline(oracle, gpu_ok):
    """The default pipeline (strict R build) over an occluded scene whose
    triangles each carry their own reflectance, against the oracle's own
    pipeline on the same scene: VRLs traced by the GPU tracer equal the
    oracle's, then slices, representatives, R of the representative records
    (shadow tests through the BVH, each record's own reflectance in vol->surf)
    and the cluster lists, bit for bit; the frame within the gather tolerance."""
    import torch
    import alvrl
    from oracle import Prep
    from test_gpu_strict import _assert_bits
    from test_occluders import per_triangle_albedos
    w, h = 64, 48
    tris = scene_mesh(alvrl, big=True)
    alb = per_triangle_albedos(len(tris))
    alb[30:] = np.random.default_rng(7).uniform(0.05, 0.95, (len(tris) - 30, 3)).astype(np.float32)
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, albedos=alb)
    o = set_occluders(oracle.scene(w, h), tris, ALB, albedos=alb)
    m = oracle.medium()
    vrls, pc = oracle.trace(o, m, 1500, seed=SEED_VRL)
    gv, gpc = alvrl.trace_vrls_gpu(s, 1500, seed=SEED_VRL)
    assert gpc == pc and np.array_equal(gv.view(np.uint32), vrls.view(np.uint32)), "GPU tracer vs oracle"
    it = alvrl.Integrator(f"targetNumSlices=12;seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(s)
    it.prepass(0)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    prep = Prep(oracle, oracle.prep_params(seed=SEED_RNG, pass_=0, target_num_slices=12))
    p2s = prep.build_slices(o)
    assert np.array_equal(p2s, it.slices()), "slices"
    off, pix, _, _ = prep.sample_slice_mapping(64.0, w * h)
    ioff, ipix = it.reps()
    assert np.array_equal(off, ioff) and np.array_equal(pix, ipix), "representatives"
    rep_ids = ((pix % h) * w + pix // h).astype(np.uint32)
    recs = oracle.records(o)
    P = set_occluders(oracle.params(m, seed=SEED_RNG, pass_=0), tris)
    _, R, _ = oracle.gather_brute(P, recs[rep_ids], vrls, pc, rec_ids=rep_ids, domain=2, want_R=True)
    _assert_bits(it.R().transpose(1, 0, 2), R, "occluded R with per-triangle reflectances (strict)")
    ocl, icl = prep.build_clusters(np.ascontiguousarray(R.transpose(1, 0, 2))), it.clusters()
    for k in ("slice_off", "reps", "weights"):
        a, b = ocl[k], icl[k]
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), k
    pid = np.arange(w * h, dtype=np.uint32)
    sl = p2s[(pid % w) * h + pid // w]
    img, _ = oracle.gather_clustered(P, recs, sl, vrls, pc, ocl["slice_off"], ocl["reps"], ocl["weights"],
                                     ocl["fb_reps"], ocl["fb_weights"], rec_ids=pid)
    _assert_close(fb.view(h * w, 3).cpu().numpy(), img, "occluded frame, per-triangle reflectances")
    it.close()
