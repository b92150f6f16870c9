"""The strict R build (integrator property strictRbuild,
csrc/rbuild_strict.hip) against the oracle, BIT FOR BIT.

The default R build trades the last ulps for speed (test_gpu_parity.py's
tolerance), so its cluster lists can only be compared with the oracle's
clustering of the DEVICE's R.  The strict build evaluates integrateVRL
(vrlIntegrator.cpp:603-785) in the oracle's statement order with IEEE
division and sqrt, no contraction and detmath.h's transcendentals, which the
oracle shares.  Bars, all exact:

  * detmath.h on the device = on the host, every input;
  * R entries (mean and variance) = oracle.gather_brute(want_R=True) for the
    smoke box, HG phase, long VRLs, every medium sampling strategy, Rsamples
    > 1, other sample counts and occluder meshes; the fused non-zero mask;
  * the whole pipeline at C1 (256^2, 1k VRLs, ALVRL defaults): slices,
    representatives, R, and then the cluster lists of the ORACLE's OWN
    buildClusters on the ORACLE's OWN R (not the device's); the frame on
    test_gpu_parity's gather tolerance against the oracle's clustered gather
    with the oracle's lists.  This closes the conditional comparison of
    test_c1_pipeline_adaptive.
"""
import numpy as np
import pytest

from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close, _ctx

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _assert_bits(dev, cpu, what):
    dev, cpu = np.asarray(dev, np.float32), np.asarray(cpu, np.float32)
    assert dev.shape == cpu.shape, what
    bad = np.nonzero(_bits(dev).ravel() != _bits(cpu).ravel())[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} of {dev.size} entries differ, first at {i}: "
                             f"{dev.ravel()[i]!r} vs {cpu.ravel()[i]!r}")
    print(f"[{what}] {dev.size} entries bit-identical ({int((cpu != 0).sum())} non-zero)")


def test_detmath_device_matches_host(oracle, gpu_ok):
    import torch
    import alvrl
    rng = np.random.default_rng(7)
    n = 1 << 20
    doms = {"exp": rng.uniform(-110, 95, n), "log": np.exp(rng.uniform(-100, 88, n)),
            "atan": np.exp(rng.uniform(-30, 30, n)) * rng.choice([-1, 1], n),
            "tan": rng.uniform(-1.5707963, 1.5707963, n),
            "asinh": np.exp(rng.uniform(-40, 40, n)) * rng.choice([-1, 1], n),
            "sinh": rng.uniform(-95, 95, n)}
    for fn, x in doms.items():
        x = x.astype(np.float32)
        x[:6] = [0.0, -0.0, 1.0, -1.0, np.inf, np.nan]
        d_in = torch.from_numpy(x).cuda()
        d_out = torch.empty_like(d_in)
        alvrl.detmath_eval(fn, d_in, d_out)
        torch.cuda.synchronize()
        host = oracle.detmath(fn, x)
        dev = d_out.cpu().numpy()
        same = (_bits(dev) == _bits(host)) | (np.isnan(dev) & np.isnan(host))
        assert same.all(), (fn, x[~same][:4], dev[~same][:4], host[~same][:4])


@pytest.mark.parametrize("fn", ["exp", "atan", "tan", "asinh", "sinh", "sqrt", "rcp"])
def test_detmath_fast_exhaustive(fn, gpu_ok):
    """csrc/detmath_fast.h (the strict R build's transcendentals: a short f64
    evaluation and Ziv's rounding test, detmath.h when the rounding is in
    doubt; its square root: v_sqrt_f32 and the one-ulp correction; its reciprocal:
    v_rcp_f32 and two Markstein corrections; IEEE sqrtf / 1.0f / x outside the
    ranges where those are exact) returns detmath.h's float -- IEEE sqrtf's
    and 1.0f / x's for sqrt and rcp -- for EVERY one of the 2^32 float inputs."""
    import time
    import alvrl
    t0 = time.perf_counter()
    bad, first = alvrl.detmath_exhaustive(fn)
    print(f"[{fn}] 2^32 inputs in {time.perf_counter() - t0:.1f} s, {bad} differ")
    assert bad == 0, (fn, bad, [hex(b) for b in first])


def test_fast_division_matches_ieee(gpu_ok):
    """The strict kernels' division (the IEEE expansion's core without its
    scaling, IEEE division outside [2^-40, 2^40]) equals IEEE a / b bit for
    bit on 2^34 random operand pairs: half over all bit patterns, half
    log-uniform around the fast range's edges."""
    import time
    import alvrl
    t0 = time.perf_counter()
    bad, first = alvrl.detmath_div_check(1 << 34, seed=20261018)
    print(f"2^34 pairs in {time.perf_counter() - t0:.1f} s, {bad} differ")
    assert bad == 0, [(hex(a), hex(b)) for a, b in first]


def _strict_R(oracle, w, h, nvrl, step, medium=("balance", -1, 0.0), phase=(0, 0.0), short=True,
              nvv=2, nvs=2, rsamples=1, tris=None):
    import torch
    import alvrl
    from oracle import set_occluders
    strategy, channel, density = medium
    sc = oracle.scene(w, h)
    if tris is not None:
        sc = set_occluders(sc, tris, (0.7, 0.4, 0.25))
    m = oracle.medium(strategy=strategy, channel=channel, density=density, phase_type=phase[0], g=phase[1])
    vrls, pc = oracle.trace(sc, m, nvrl, seed=SEED_VRL, short_vrls=short)
    recs = oracle.records(sc)
    ids = np.arange(0, w * h, step, dtype=np.uint32)
    P = oracle.params(m, nvv=nvv, nvs=nvs, short_vrls=int(short), seed=SEED_RNG, r_samples=rsamples)
    if tris is not None:
        P = set_occluders(P, tris)
    _, R, cnt = oracle.gather_brute(P, recs[ids], vrls, pc, rec_ids=ids, want_R=True, domain=2)
    ctx = _ctx(alvrl.Medium(strategy=strategy, channel=channel, sampling_density=density,
                            phase_type=phase[0], phase_g=phase[1]),
               short_vrls=short, vol_vol_samples=nvv, vol_surf_samples=nvs)
    ctx.set_strict_rbuild(True)
    if rsamples > 1:
        ctx.set_rsamples(rsamples)
    ctx.upload_vrls(vrls, pc)
    if tris is not None:
        ctx.set_occluders(tris)
    nr, nv = len(ids), vrls.shape[1]
    d_Rt = torch.zeros((nv, nr, 2), dtype=torch.float32, device="cuda")
    d_recs, d_ids = torch.from_numpy(recs[ids]).cuda(), torch.from_numpy(ids.view(np.int32)).cuda()
    ctx.build_R(d_recs, d_Rt, ld=nr, d_ids=d_ids)
    torch.cuda.synchronize()
    pre, _ = ctx.stats()
    assert pre == cnt, (pre, cnt)
    Rg = d_Rt.cpu().numpy().transpose(1, 0, 2)
    ctx.close()
    return Rg, R


@pytest.mark.parametrize("case", ["default", "hg", "long", "single", "manual", "maximum", "rsamples",
                                  "samples"])
def test_strict_R_bit_exact(oracle, gpu_ok, case):
    kw = dict(default={}, hg=dict(phase=(1, 0.6)), long=dict(short=False),
              single=dict(medium=("single", -1, 0.0)), manual=dict(medium=("manual", -1, 0.7)),
              maximum=dict(medium=("maximum", -1, 0.0)), rsamples=dict(rsamples=3),
              samples=dict(nvv=3, nvs=5))[case]
    Rg, R = _strict_R(oracle, 64, 48, 1500, 3, **kw)
    assert (R[..., 0] != 0).mean() > 0.5
    _assert_bits(Rg, R, f"strict R {case}")


def test_strict_R_occluders(oracle, gpu_ok):
    """Shadow tests through the device BVH (any hit) against the oracle's
    loop over every triangle: the same booleans, so the same bits."""
    import alvrl
    from test_gpu_occluders import scene_mesh
    tris = scene_mesh(alvrl, big=True)
    Rg, R = _strict_R(oracle, 40, 30, 1500, 7, tris=tris)
    _assert_bits(Rg, R, "strict R occluders")


def test_strict_R_blocks_nonzero(oracle, gpu_ok):
    """alvrl_build_R_blocks in strict mode: rows scattered over two blocks,
    the fused non-zero mask equal to the oracle's non-zero columns."""
    import torch
    w, h = 64, 48
    sc = oracle.scene(w, h)
    m = oracle.medium()
    vrls, pc = oracle.trace(sc, m, 2000, seed=SEED_VRL)
    recs = oracle.records(sc)
    ids = np.arange(0, w * h, 5, dtype=np.uint32)
    P = oracle.params(m, seed=SEED_RNG)
    _, R, _ = oracle.gather_brute(P, recs[ids], vrls, pc, rec_ids=ids, want_R=True, domain=2)
    nr, nv = len(ids), vrls.shape[1]
    a = nr // 3                                     # block 0: rows [0, a), block 1: [a, nr)
    off = np.where(np.arange(nr) < a, np.arange(nr), nv * a + (np.arange(nr) - a)).astype(np.uint64)
    stride = np.where(np.arange(nr) < a, a, nr - a).astype(np.uint32)
    ctx = _ctx()
    ctx.set_strict_rbuild(True)
    ctx.upload_vrls(vrls, pc)
    d_Rt = torch.zeros(nv * nr * 2, dtype=torch.float32, device="cuda")
    d_nz = torch.zeros(nv, dtype=torch.uint8, device="cuda")
    t = (torch.from_numpy(recs[ids]).cuda(), torch.from_numpy(off.view(np.int64)).cuda(),
         torch.from_numpy(stride.view(np.int32)).cuda(), torch.from_numpy(ids.view(np.int32)).cuda())
    ctx.build_R_blocks(t[0], d_Rt, t[1], t[2], d_nz, t[3])
    torch.cuda.synchronize()
    flat = d_Rt.cpu().numpy().reshape(-1, 2)
    Rg = np.empty_like(R)
    for r in range(nr):
        Rg[r] = flat[off[r] + np.arange(nv, dtype=np.uint64) * stride[r]]
    _assert_bits(Rg, R, "strict R blocks")
    assert np.array_equal(d_nz.cpu().numpy().astype(bool), (R[..., 0] != 0).any(axis=0))
    ctx.close()


def _oracle_pipeline(oracle, w, h, vrls, pc, pass_, prep_kw=None, **pkw):
    """The oracle's own prepass and render: slices, representatives, R of the
    representative pixels, buildClusters on that R, clustered gather."""
    from oracle import Prep
    prep = Prep(oracle, oracle.prep_params(seed=SEED_RNG, pass_=pass_, **(prep_kw or {})))
    osc = oracle.scene(w, h)
    p2s = prep.build_slices(osc)
    off, pix, _, _ = prep.sample_slice_mapping(64.0, w * h)
    rep_ids = ((pix % h) * w + pix // h).astype(np.uint32)     # column-major ids -> row-major
    recs = oracle.records(osc)
    P = oracle.params(oracle.medium(), seed=SEED_RNG, pass_=pass_, **pkw)
    _, R, rcnt = oracle.gather_brute(P, recs[rep_ids], vrls, pc, rec_ids=rep_ids, domain=2, want_R=True)
    cl = prep.build_clusters(np.ascontiguousarray(R.transpose(1, 0, 2)))
    pid = np.arange(w * h, dtype=np.uint32)
    sl = p2s[(pid % w) * h + pid // w]
    img, gcnt = oracle.gather_clustered(P, recs, sl, vrls, pc, cl["slice_off"], cl["reps"], cl["weights"],
                                        cl["fb_reps"], cl["fb_weights"], rec_ids=pid)
    return dict(slices=p2s, rep_off=off, rep_pix=pix, R=R, clusters=cl, img=img, rcnt=rcnt, gcnt=gcnt)


def _device_pipeline(props, w, h, vrls, pc, pass_):
    import torch
    import alvrl
    it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(alvrl.scene_default(w, h))
    it.prepass(pass_)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    return it, fb.view(h * w, 3).cpu().numpy()


@pytest.mark.parametrize("props,prep_kw,pass_", [
    ("", {}, 0),
    ("localUndersampling=20", {"local_undersampling": 20.0}, 1),
    ("neighbourCount=3;neighbourWeight=0.5", {"neighbour_count": 3, "neighbour_weight": 0.5}, 2),
])
def test_strict_pipeline_c1(oracle, gpu_ok, props, prep_kw, pass_):
    """C1 end to end with strictRbuild against the oracle's own pipeline."""
    import alvrl
    w = h = 256
    vrls, pc = alvrl.trace_vrls(alvrl.scene_default(w, h), 1000, seed=SEED_VRL)
    it, img = _device_pipeline(props + (";" if props else "") + "strictRbuild=true", w, h, vrls, pc, pass_)
    o = _oracle_pipeline(oracle, w, h, vrls, pc, pass_, prep_kw)
    assert np.array_equal(it.slices(), o["slices"]), "slices"
    off, pix = it.reps()
    assert np.array_equal(off, o["rep_off"]) and np.array_equal(pix, o["rep_pix"]), "representatives"
    _assert_bits(it.R().transpose(1, 0, 2), o["R"], "C1 R")
    cl, ocl = it.clusters(), o["clusters"]
    st = it.stats()
    keys = ("slice_off", "reps", "weights") + (("fb_reps", "fb_weights") if st["fallback_built"] else ())
    for k in keys:   # the fall-back list is built lazily (deviation 4)
        assert np.array_equal(_bits(cl[k]) if cl[k].dtype == np.float32 else cl[k],
                              _bits(ocl[k]) if ocl[k].dtype == np.float32 else ocl[k]), k
    assert st["contrib_preprocess"] == o["rcnt"] and st["contrib_render"] == o["gcnt"]
    print(f"C1 strict ({props or 'defaults'}): {len(cl['reps'])} representatives identical to the "
          f"oracle's own pipeline, R build {st['ms_rbuild']:.2f} ms")
    _assert_close(img, o["img"], f"C1 strict frame {props}")
    it.close()
