"""Parity of the HIP hot path (libalvrl.so, through the C ABI) with the CPU
restatement (oracle/), on identical inputs and identical counter-RNG streams.

Tolerances (floating point, stated here):
  * gather / R entries: the device uses hardware exp2/log2/rcp/rsq based
    expf/asinh/sinh/cosh and reduced-range tan/atan (<= 4 ulp, tools/mathcheck.hip),
    contracts a*b+c into FMA and evaluates integrateVRL in the algebraically
    reduced form documented in vrl_device.hpp; the oracle follows the
    reference's statement order with glibc maths and no contraction.  Almost
    every pair agrees to ~1e-7 relative.  A few pairs are ill-conditioned in
    float itself: when a VRL point V lies very close to the eye ray, Kulla's
    equi-angular sampler evaluates tan(atan(x)) with x ~ 1e6 (angle within
    ~1e-6 of pi/2), so one ulp in the angle moves that single sample by up to
    ~10% -- in the reference as much as here (tests/diag_pairs.py isolates
    such pairs).  Hence the bound is on the error distribution over pixels:
        median rel <= 1e-6, q99 <= 1e-4, q99.9 <= 2e-3, max <= 5e-2,
        RMSE (rms.cpp: gamma 1, absolute, all pixels x RGB) <= 2e-4 * mean.
    R entries are single pairs (no averaging over VRLs), so their tail is
    heavier: median <= 1e-6 (mean) / 1e-5 (variance: Welford's M2 is a
    difference of nearby values), at most 0.5% of entries above 1e-3, and every
    VRL column sum (what clustering consumes first) within 1e-3.
  * refinement: cluster representatives and weights must be BIT-IDENTICAL
    (integer/index work; the kernel is compiled without FMA contraction and
    uses the oracle's reduction order).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_VRL = 0x5EED0001
SEED_RNG = 0xA1B2C3D4


def _torch():
    import torch
    return torch


def _ctx(medium=None, **kw):
    import alvrl
    ctx = alvrl.Context(device=0, seed=SEED_RNG, **kw)
    ctx.set_medium(medium or alvrl.Medium())
    return ctx


def _scene_inputs(oracle, w, h, nvrl):
    sc = oracle.scene(w, h)
    m = oracle.medium()
    vrls, pc = oracle.trace(sc, m, nvrl, seed=SEED_VRL)
    recs = oracle.records(sc)
    return sc, m, vrls, pc, recs


def _rel(gpu, cpu):
    gpu = np.asarray(gpu, np.float64)
    cpu = np.asarray(cpu, np.float64)
    assert gpu.shape == cpu.shape
    assert np.isfinite(gpu).all(), "non-finite device values"
    err = np.abs(gpu - cpu)
    rel = np.where(err == 0, 0.0, err / np.maximum(np.abs(cpu), 1e-30))
    return gpu, cpu, err, rel


def _assert_close(gpu, cpu, what, q50=1e-6, q99=1e-4, q999=2e-3, qmax=5e-2, rmse_rel=2e-4):
    gpu, cpu, err, rel = _rel(gpu, cpu)
    qs = np.quantile(rel, [0.5, 0.99, 0.999]) if rel.size else np.zeros(3)
    rmse = float(np.sqrt(np.mean((gpu - cpu) ** 2)))
    mean = float(np.abs(cpu).mean())
    print(f"[{what}] rel q50={qs[0]:.2e} q99={qs[1]:.2e} q999={qs[2]:.2e} max={rel.max():.2e} "
          f"rmse={rmse:.2e} (mean {mean:.3e}, n={rel.size})")
    assert qs[0] <= q50 and qs[1] <= q99 and qs[2] <= q999, f"{what}: quantiles {qs}"
    assert rel.max() <= qmax, f"{what}: max rel {rel.max()}"
    assert rmse <= rmse_rel * max(mean, 1e-30), f"{what}: RMSE {rmse}"


def _assert_close_pairs(gpu, cpu, what, q50=1e-6, csum=1e-3):
    gpu, cpu, err, rel = _rel(gpu, cpu)
    frac = float((rel > 1e-3).mean())
    print(f"[{what}] rel q50={np.median(rel):.2e} frac>1e-3={frac:.2e} max={rel.max():.2e}")
    assert np.median(rel) <= q50 and frac <= 5e-3, what
    cs_g, cs_c = gpu.sum(axis=0), cpu.sum(axis=0)
    crel = np.abs(cs_g - cs_c) / np.maximum(np.abs(cs_c), 1e-30)
    assert ((cs_c == 0) == (cs_g == 0)).all(), f"{what}: zero-column pattern differs"
    assert crel.max() <= csum, f"{what}: column sums max rel {crel.max()}"


def test_gather_brute_small(oracle, gpu_ok):
    """C1-shaped: 64x64 records x 1000 VRLs, every pixel."""
    torch = _torch()
    sc, m, vrls, pc, recs = _scene_inputs(oracle, 64, 64, 1000)
    P = oracle.params(m, seed=SEED_RNG)
    cpu, ccnt = oracle.gather_brute(P, recs, vrls, pc)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    d_recs = torch.from_numpy(recs).cuda()
    d_out = torch.zeros((recs.shape[0], 3), dtype=torch.float32, device="cuda")
    ctx.reset_stats()
    ctx.gather_brute(d_recs, d_out)
    torch.cuda.synchronize()
    gpu = d_out.cpu().numpy()
    _, ren = ctx.stats()
    assert ren == ccnt == recs.shape[0] * vrls.shape[1]
    _assert_close(gpu, cpu, "brute 64x64x1k")


def test_gather_brute_c2_subset(oracle, gpu_ok):
    """C2 shape (1024^2, 10k VRLs): a strided subset of pixels, ids = pixel ids."""
    torch = _torch()
    sc, m, vrls, pc, recs = _scene_inputs(oracle, 1024, 1024, 10000)
    ids = np.arange(0, 1024 * 1024, 2053, dtype=np.uint32)
    sub = recs[ids]
    P = oracle.params(m, seed=SEED_RNG)
    cpu, _ = oracle.gather_brute(P, sub, vrls, pc, rec_ids=ids)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    d_out = torch.zeros((len(ids), 3), dtype=torch.float32, device="cuda")
    ctx.gather_brute(torch.from_numpy(sub).cuda(), d_out, d_ids=torch.from_numpy(ids.view(np.int32)).cuda())
    torch.cuda.synchronize()
    _assert_close(d_out.cpu().numpy(), cpu, "brute c2-subset")


def test_gather_host_pointer_variant(oracle, gpu_ok):
    sc, m, vrls, pc, recs = _scene_inputs(oracle, 32, 32, 500)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    a = ctx.gather_brute_host(recs)
    P = oracle.params(m, seed=SEED_RNG)
    cpu, _ = oracle.gather_brute(P, recs, vrls, pc)
    _assert_close(a, cpu, "brute host-pointer")


def test_gather_deterministic(oracle, gpu_ok):
    torch = _torch()
    sc, m, vrls, pc, recs = _scene_inputs(oracle, 64, 64, 2000)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    d_recs = torch.from_numpy(recs).cuda()
    outs = []
    for _ in range(2):
        d = torch.zeros((recs.shape[0], 3), dtype=torch.float32, device="cuda")
        ctx.gather_brute(d_recs, d)
        torch.cuda.synchronize()
        outs.append(d.cpu().numpy())
    assert np.array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


def test_gather_nondefault_samples_and_hg(oracle, gpu_ok):
    """Generic (runtime sample count) kernel path + HG phase + long VRL flag."""
    import alvrl
    torch = _torch()
    sc = oracle.scene(32, 32)
    m = oracle.medium(phase_type=1, g=0.4)
    vrls, pc = oracle.trace(sc, oracle.medium(), 300, seed=SEED_VRL)
    recs = oracle.records(sc)
    P = oracle.params(m, nvv=3, nvs=4, short_vrls=0, seed=SEED_RNG)
    cpu, _ = oracle.gather_brute(P, recs, vrls, pc)
    ctx = _ctx(alvrl.Medium(phase_type=1, phase_g=0.4), vol_vol_samples=3, vol_surf_samples=4,
               short_vrls=False)
    ctx.upload_vrls(vrls, pc)
    d = torch.zeros((recs.shape[0], 3), dtype=torch.float32, device="cuda")
    ctx.gather_brute(torch.from_numpy(recs).cuda(), d)
    torch.cuda.synchronize()
    _assert_close(d.cpu().numpy(), cpu, "brute nvv3 nvs4 hg")


def test_build_R_parity(oracle, gpu_ok):
    """Rbuilder::run rows (mean, var) against the oracle's R rows."""
    torch = _torch()
    sc, m, vrls, pc, recs = _scene_inputs(oracle, 128, 128, 1500)
    rows = np.arange(0, 128 * 128, 61, dtype=np.uint32)
    sub = recs[rows]
    P = oracle.params(m, seed=SEED_RNG)
    _, Rcpu, cnt = oracle.gather_brute(P, sub, vrls, pc, rec_ids=rows, domain=2, want_R=True)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    nr, nv = len(rows), vrls.shape[1]
    d_Rt = torch.zeros((nv, nr, 2), dtype=torch.float32, device="cuda")
    ctx.reset_stats()
    ctx.build_R(torch.from_numpy(sub).cuda(), d_Rt, ld=nr, d_ids=torch.from_numpy(rows.view(np.int32)).cuda())
    torch.cuda.synchronize()
    Rg = d_Rt.cpu().numpy().transpose(1, 0, 2)
    pre, _ = ctx.stats()
    assert pre == cnt
    _assert_close_pairs(Rg[..., 0], Rcpu[..., 0], "R mean")
    _assert_close_pairs(Rg[..., 1], Rcpu[..., 1], "R var", q50=1e-5)   # M2: a difference, cancels


def test_build_R_rsamples(oracle, gpu_ok):
    """Rsamples = 3 (vrlIntegrator.cpp:194): R entries are sums over three
    independent samples (LiInternal's samples loop, :427-443 / :812-813);
    blocked build (alvrl_build_R_blocks) with its fused non-zero mask."""
    torch = _torch()
    sc, m, vrls, pc, recs = _scene_inputs(oracle, 96, 96, 700)
    rows = np.arange(0, 96 * 96, 97, dtype=np.uint32)
    sub = recs[rows]
    P = oracle.params(m, seed=SEED_RNG, r_samples=3)
    _, Rcpu, cnt = oracle.gather_brute(P, sub, vrls, pc, rec_ids=rows, domain=2, want_R=True)
    P1 = oracle.params(m, seed=SEED_RNG)
    _, R1, _ = oracle.gather_brute(P1, sub, vrls, pc, rec_ids=rows, domain=2, want_R=True)
    assert not np.array_equal(Rcpu, R1)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    ctx.set_rsamples(3)
    nr, nv = len(rows), vrls.shape[1]
    d_Rt = torch.zeros((nv, nr, 2), dtype=torch.float32, device="cuda")
    ctx.reset_stats()
    ctx.build_R(torch.from_numpy(sub).cuda(), d_Rt, ld=nr, d_ids=torch.from_numpy(rows.view(np.int32)).cuda())
    # the same rows through the blocked build: two blocks of different strides
    h = nr // 2
    boff = np.concatenate([np.arange(h), nv * h + np.arange(nr - h)]).astype(np.uint64)
    bstr = np.concatenate([np.full(h, h), np.full(nr - h, nr - h)]).astype(np.uint32)
    d_B = torch.zeros(nv * nr * 2, dtype=torch.float32, device="cuda")
    d_nz = torch.zeros(nv, dtype=torch.uint8, device="cuda")
    ctx.build_R_blocks(torch.from_numpy(sub).cuda(), d_B, torch.from_numpy(boff.view(np.int64)).cuda(),
                       torch.from_numpy(bstr.view(np.int32)).cuda(), d_nz,
                       d_ids=torch.from_numpy(rows.view(np.int32)).cuda())
    torch.cuda.synchronize()
    Rg = d_Rt.cpu().numpy().transpose(1, 0, 2)
    pre, _ = ctx.stats()
    assert pre == 2 * cnt
    _assert_close_pairs(Rg[..., 0], Rcpu[..., 0], "R mean (Rsamples=3)")
    _assert_close_pairs(Rg[..., 1], Rcpu[..., 1], "R var (Rsamples=3)", q50=1e-5)
    B = d_B.cpu().numpy().reshape(-1, 2)
    Bt = np.concatenate([B[:nv * h].reshape(nv, h, 2), B[nv * h:].reshape(nv, nr - h, 2)], axis=1)
    assert np.array_equal(Bt.view(np.uint32), d_Rt.cpu().numpy().view(np.uint32))
    assert np.array_equal(d_nz.cpu().numpy().astype(bool), (Rg[..., 0] != 0).any(axis=0))


def _degenerate_inputs(oracle):
    """Eye rays exactly along +z (so sinTheta is exactly 0 against z-aligned
    VRLs on both sides), VRLs parallel to them (sampleVtoDistance's uniform
    branch, vrlIntegrator.cpp:929-933), zero-length VRLs (:920-924) and
    ordinary traced VRLs."""
    sc, m, vrls, pc, recs = _scene_inputs(oracle, 64, 64, 300)
    rng = np.random.default_rng(11)
    nrec = 96
    xy = rng.uniform(-0.8, 0.8, size=(nrec, 2)).astype(np.float32)
    base = recs[32 * 64 + 32].copy()
    R = np.repeat(base[None], nrec, axis=0)
    R[:, 0:2] = xy; R[:, 2] = -0.9                      # o
    R[:, 3:6] = (0.0, 0.0, 1.0)                         # d
    R[:, 6:8] = xy; R[:, 8] = 1.0                       # p on the back wall z = 1
    R[:, 9:12] = (0.0, 0.0, -1.0)                       # inward normal
    V = vrls.copy()
    nz, npar = 24, 48
    V[3:6, :nz] = V[0:3, :nz]                           # zero length: end = start
    for j in range(nz, nz + npar):                      # parallel to +-z, off the eye rays
        L = np.float32(rng.uniform(0.05, 1.2)) * (1 if j % 2 else -1)
        V[0:2, j] = rng.uniform(-0.9, 0.9, 2)
        V[2, j] = np.float32(rng.uniform(-0.7, 0.7))
        V[3:5, j] = V[0:2, j]
        V[5, j] = V[2, j] + L
    return m, np.ascontiguousarray(V), pc, np.ascontiguousarray(R), nz, npar


def test_degenerate_vrls(oracle, gpu_ok):
    torch = _torch()
    m, V, pc, R, nz, npar = _degenerate_inputs(oracle)
    ids = np.arange(R.shape[0], dtype=np.uint32) * 37
    P = oracle.params(m, seed=SEED_RNG)
    _, Rc, _ = oracle.gather_brute(P, R, V, pc, rec_ids=ids, domain=2, want_R=True)
    cpu, _ = oracle.gather_brute(P, R, V, pc, rec_ids=ids)
    ctx = _ctx()
    ctx.upload_vrls(V, pc)
    d_R = torch.from_numpy(R).cuda()
    d_ids = torch.from_numpy(ids.view(np.int32)).cuda()
    d_Rt = torch.zeros((V.shape[1], R.shape[0], 2), dtype=torch.float32, device="cuda")
    ctx.build_R(d_R, d_Rt, ld=R.shape[0], d_ids=d_ids)
    d_out = torch.zeros((R.shape[0], 3), dtype=torch.float32, device="cuda")
    ctx.gather_brute(d_R, d_out, d_ids=d_ids)
    torch.cuda.synchronize()
    Rg = d_Rt.cpu().numpy().transpose(1, 0, 2)
    # the special columns carry real contributions on both sides
    for lo, hi, what in ((0, nz, "zero-length"), (nz, nz + npar, "parallel")):
        cg, cc = Rg[:, lo:hi, 0].sum(axis=0), Rc[:, lo:hi, 0].sum(axis=0)
        assert (cc > 0).all() and (cg > 0).all(), f"{what} VRLs contribute nothing"
        rel = np.abs(cg - cc) / cc
        print(f"[{what}] column rel max {rel.max():.2e}")
        assert rel.max() <= 1e-4, f"{what} columns differ: {rel.max()}"
    _assert_close_pairs(Rg[..., 0], Rc[..., 0], "degenerate R mean")
    _assert_close(d_out.cpu().numpy(), cpu, "degenerate brute")


def _refine_case(oracle, w, h, nvrl, nslice_rows, undersampling, torch):
    sc, m, vrls, pc, recs = _scene_inputs(oracle, w, h, nvrl)
    rng = np.random.default_rng(7)
    nrows = sum(nslice_rows)
    rows_pix = rng.choice(w * h, size=nrows, replace=False).astype(np.uint32)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    d_Rt = torch.zeros((vrls.shape[1], nrows, 2), dtype=torch.float32, device="cuda")
    ctx.build_R(torch.from_numpy(recs[rows_pix]).cuda(), d_Rt, ld=nrows,
                d_ids=torch.from_numpy(rows_pix.view(np.int32)).cuda())
    torch.cuda.synchronize()
    Rt = d_Rt.cpu().numpy()
    nv = vrls.shape[1]
    colsum = Rt[:, :, 0].sum(axis=1)
    nz = np.nonzero(colsum != 0)[0].astype(np.uint32)
    z = np.nonzero(colsum == 0)[0].astype(np.uint32)
    init = np.concatenate([nz, z])
    init_off = [0] + ([len(nz)] if len(nz) else []) + ([nv] if len(z) else [])
    init_off = np.array(init_off, np.uint32)
    off = np.cumsum([0] + list(nslice_rows))
    jobs = []
    for s in range(len(nslice_rows)):
        r = np.arange(off[s], off[s + 1], dtype=np.uint32)
        jobs.append(dict(rows=r, locw=np.full(len(r), 1.0 / len(r)), pixel_undersampling=0.25,
                         undersampling=undersampling, depth_correction=1.0, do_refine=True,
                         stage_refine=3 + 2 * s, stage_sample=4 + 2 * s))
    return ctx, d_Rt, Rt, jobs, init, init_off


@pytest.mark.parametrize("undersampling", [-1.0, 10.0])
def test_refine_bit_exact(oracle, gpu_ok, undersampling):
    """Per-slice Clustering refine + sampleRepresentatives: device == oracle, bit for bit."""
    torch = _torch()
    ctx, d_Rt, Rt, jobs, init, init_off = _refine_case(oracle, 96, 96, 1200, [40, 23, 64, 70, 5],
                                                       undersampling, torch)
    off, reps, w, refined = ctx.refine(d_Rt, Rt.shape[1], jobs, init, init_off)
    # roofline counters: 3 setup passes over every job's rows, and the splits' columns
    ent, sent = ctx.last_refine_entries(), ctx.last_refine_split_entries()
    assert ent - sent == 3 * Rt.shape[0] * sum(len(j["rows"]) for j in jobs) and sent > 0, (ent, sent)
    for s, j in enumerate(jobs):
        cr, cw, cref = oracle.cluster_refine(Rt, j["rows"], j["locw"], init, init_off,
                                             j["pixel_undersampling"], undersampling,
                                             stage_refine=j["stage_refine"],
                                             stage_sample=j["stage_sample"], seed=SEED_RNG)
        gr, gw = reps[off[s]:off[s + 1]], w[off[s]:off[s + 1]]
        print(f"slice {s}: {len(cr)} clusters (cpu) {len(gr)} (gpu) refined={cref}/{refined[s]}")
        assert bool(refined[s]) == cref
        assert np.array_equal(gr, cr)
        assert np.array_equal(gw.view(np.uint32), cw.view(np.uint32))


def test_refine_large_cluster_radix_path(oracle, gpu_ok):
    """Cluster sizes above the LDS bitonic limit exercise the radix-sort path."""
    torch = _torch()
    ctx, d_Rt, Rt, jobs, init, init_off = _refine_case(oracle, 96, 96, 6000, [48], 200.0, torch)
    off, reps, w, refined = ctx.refine(d_Rt, Rt.shape[1], jobs, init, init_off)
    j = jobs[0]
    cr, cw, cref = oracle.cluster_refine(Rt, j["rows"], j["locw"], init, init_off,
                                         j["pixel_undersampling"], 200.0, stage_refine=3,
                                         stage_sample=4, seed=SEED_RNG)
    assert np.array_equal(reps, cr)
    assert np.array_equal(w.view(np.uint32), cw.view(np.uint32))


def test_gather_clustered_parity(oracle, gpu_ok):
    torch = _torch()
    import alvrl
    sc, m, vrls, pc, recs = _scene_inputs(oracle, 64, 64, 800)
    rng = np.random.default_rng(3)
    ns = 7
    slice_of = rng.integers(0, ns, size=recs.shape[0]).astype(np.uint32)
    slice_of[::97] = 0xFFFFFFFF
    sizes = rng.integers(1, 60, size=ns)
    slice_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    reps = rng.integers(0, vrls.shape[1], size=slice_off[-1]).astype(np.uint32)
    wts = rng.uniform(0.5, 20, size=slice_off[-1]).astype(np.float32)
    fb = rng.choice(vrls.shape[1], 40, replace=False).astype(np.uint32)
    fbw = rng.uniform(1, 5, size=40).astype(np.float32)
    P = oracle.params(m, seed=SEED_RNG)
    cpu, ccnt = oracle.gather_clustered(P, recs, slice_of, vrls, pc, slice_off, reps, wts, fb, fbw)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    ctx.set_clusters(slice_off, reps, wts, fb, fbw)
    ctx.reset_stats()
    gpu = ctx.gather_clustered_host(recs, slice_of)
    _, ren = ctx.stats()
    assert ren == ccnt
    _assert_close(gpu, cpu, "clustered")


def test_c2_full_frame_properties(gpu_ok):
    """Full BASELINE configs[1] frame (1024^2 x 10k): size-independent checks."""
    torch = _torch()
    import alvrl
    from oracle import Oracle
    o = Oracle()
    sc = o.scene(1024, 1024)
    vrls, pc = o.trace(sc, o.medium(), 10000, seed=SEED_VRL)
    recs = o.records(sc)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    d_recs = torch.from_numpy(recs).cuda()
    d = torch.zeros((recs.shape[0], 3), dtype=torch.float32, device="cuda")
    ctx.reset_stats()
    ctx.gather_brute(d_recs, d)
    torch.cuda.synchronize()
    img = d.cpu().numpy()
    assert np.isfinite(img).all() and (img >= 0).all()
    _, ren = ctx.stats()
    assert ren == recs.shape[0] * vrls.shape[1]
    print(f"C2 frame: {ctx.last_kernel_ms():.1f} ms, mean {img.mean(0)}")


def test_refine_bit_exact_row_blocks(oracle, gpu_ok):
    """Local matrices of 3, 4 and 5 row blocks (up to 192 rows, 193-256 and
    beyond: the split variance engine's row-block layouts and the older
    engine above 256 rows): device == oracle, bit for bit."""
    torch = _torch()
    sizes = [129, 192, 193, 214, 256, 260]
    ctx, d_Rt, Rt, jobs, init, init_off = _refine_case(oracle, 64, 64, 700, sizes, -1.0, torch)
    off, reps, w, refined = ctx.refine(d_Rt, Rt.shape[1], jobs, init, init_off)
    for s, j in enumerate(jobs):
        cr, cw, cref = oracle.cluster_refine(Rt, j["rows"], j["locw"], init, init_off,
                                             j["pixel_undersampling"], -1.0,
                                             stage_refine=j["stage_refine"],
                                             stage_sample=j["stage_sample"], seed=SEED_RNG)
        gr, gw = reps[off[s]:off[s + 1]], w[off[s]:off[s + 1]]
        assert bool(refined[s]) == cref, sizes[s]
        assert np.array_equal(gr, cr), sizes[s]
        assert np.array_equal(gw.view(np.uint32), cw.view(np.uint32)), sizes[s]


@pytest.mark.parametrize("undersampling", [-1.0, 20.0])
def test_refine_bit_exact_c5_rows(oracle, gpu_ok, undersampling):
    """Local matrices of C5's size (2048^2 / 100 slices: ~655 representative
    rows, 11 row blocks) and around it -- 320, 512, 655 and 700 rows -- on
    the >256-row variance engine: device == oracle, bit for bit."""
    torch = _torch()
    sizes = [320, 512, 655, 700]
    ctx, d_Rt, Rt, jobs, init, init_off = _refine_case(oracle, 64, 64, 900, sizes, undersampling, torch)
    off, reps, w, refined = ctx.refine(d_Rt, Rt.shape[1], jobs, init, init_off)
    for s, j in enumerate(jobs):
        cr, cw, cref = oracle.cluster_refine(Rt, j["rows"], j["locw"], init, init_off,
                                             j["pixel_undersampling"], undersampling,
                                             stage_refine=j["stage_refine"],
                                             stage_sample=j["stage_sample"], seed=SEED_RNG)
        gr, gw = reps[off[s]:off[s + 1]], w[off[s]:off[s + 1]]
        print(f"{sizes[s]} rows: {len(cr)} clusters")
        assert bool(refined[s]) == cref, sizes[s]
        assert np.array_equal(gr, cr), sizes[s]
        assert np.array_equal(gw.view(np.uint32), cw.view(np.uint32)), sizes[s]


@pytest.mark.parametrize("blk,proj", [(1, 0), (3, 300), (4, 300)])
def test_refine_bit_exact_split_parts(oracle, gpu_ok, monkeypatch, capfd, blk, proj):
    """Every split of more than 256 columns divided into parts (split_parts:
    one part per variance pass and group of `blk` row blocks, run by idle
    workgroups, the block totals added in block order by the split's owner),
    the initial clusters' variances of the jobs above 256 rows by row groups
    (init_parts), and with proj > 0 the projections of every split of >= proj
    columns and the column weights in 64-column ranges (proj_parts,
    colw_parts): device == oracle, bit for bit, and some parts ran on other
    workgroups."""
    import re
    torch = _torch()
    monkeypatch.setenv("ALVRL_PART_MIN", "64")
    monkeypatch.setenv("ALVRL_PART_IDLE", "0")
    monkeypatch.setenv("ALVRL_PART_IDLE_SHORT", "0")
    monkeypatch.setenv("ALVRL_PART_BLK", str(blk))
    monkeypatch.setenv("ALVRL_PART_BLK_SHORT", str(blk))
    monkeypatch.setenv("ALVRL_PROJ_MIN", str(proj))
    monkeypatch.setenv("ALVRL_PROJ_CPP", "64")
    monkeypatch.setenv("ALVRL_REFINE_TEAM_STATS", "1")
    sizes = [40, 129, 214, 260, 455]
    ctx, d_Rt, Rt, jobs, init, init_off = _refine_case(oracle, 64, 64, 1500, sizes, -1.0, torch)
    capfd.readouterr()
    off, reps, w, refined = ctx.refine(d_Rt, Rt.shape[1], jobs, init, init_off)
    err = capfd.readouterr().err
    m = re.search(r"divided splits (\d+) \(no free slot (\d+)\), parts by owner (\d+), by others (\d+)", err)
    assert m, err
    print(m.group(0))
    assert int(m.group(1)) > 0 and int(m.group(3)) + int(m.group(4)) >= 2 * int(m.group(1))
    for s, j in enumerate(jobs):
        cr, cw, cref = oracle.cluster_refine(Rt, j["rows"], j["locw"], init, init_off,
                                             j["pixel_undersampling"], -1.0,
                                             stage_refine=j["stage_refine"],
                                             stage_sample=j["stage_sample"], seed=SEED_RNG)
        gr, gw = reps[off[s]:off[s + 1]], w[off[s]:off[s + 1]]
        assert bool(refined[s]) == cref, sizes[s]
        assert np.array_equal(gr, cr), sizes[s]
        assert np.array_equal(gw.view(np.uint32), cw.view(np.uint32)), sizes[s]


@pytest.mark.parametrize("depth_correction", [0.8, 1.3])
def test_refine_depth_correction(oracle, gpu_ok, depth_correction):
    """refineAdaptively with depthCorrection != 1 (Preprocessor.cpp:456-469:
    after the convergence stop the snapshot is restored and the splits are
    replayed with the replayable sampler, src/libbidir/rsampler.cpp:68-91, up
    to the corrected cluster count): device == oracle, bit for bit, on
    slices of 1-5 row blocks."""
    torch = _torch()
    ctx, d_Rt, Rt, jobs, init, init_off = _refine_case(oracle, 96, 96, 1500, [40, 64, 150, 230, 300], -1.0,
                                                       torch)
    for j in jobs:
        j["depth_correction"] = depth_correction
    off, reps, w, refined = ctx.refine(d_Rt, Rt.shape[1], jobs, init, init_off)
    for s, j in enumerate(jobs):
        cr, cw, cref = oracle.cluster_refine(Rt, j["rows"], j["locw"], init, init_off,
                                             j["pixel_undersampling"], -1.0,
                                             depth_correction=depth_correction,
                                             stage_refine=j["stage_refine"],
                                             stage_sample=j["stage_sample"], seed=SEED_RNG)
        c1, _, _ = oracle.cluster_refine(Rt, j["rows"], j["locw"], init, init_off,
                                         j["pixel_undersampling"], -1.0, stage_refine=j["stage_refine"],
                                         stage_sample=j["stage_sample"], seed=SEED_RNG)
        gr, gw = reps[off[s]:off[s + 1]], w[off[s]:off[s + 1]]
        print(f"slice {s} ({len(j['rows'])} rows): {len(cr)} clusters at depthCorrection "
              f"{depth_correction}, {len(c1)} at 1")
        assert bool(refined[s]) == cref
        assert np.array_equal(gr, cr), s
        assert np.array_equal(gw.view(np.uint32), cw.view(np.uint32)), s
