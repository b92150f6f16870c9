"""GPU parity for delta-BSDF occluders (mirrors and null panes, see
test_chains.py): the gathers over LiInternal's weighted chain records, the R
build adding a chain's levels into its row (ALVRL_REC_ACCUM), and the
integrator's clustered pipeline over such a scene.

Bars: the oracle's restatement of the same records (oracle.chains, bit-equal
to the host's, test_chains.py) gathered on the CPU -- per record and per
pixel on test_gpu_parity's tolerance; slices bit-exact; cluster lists
bit-exact against the oracle's clustering of the device's R."""
import numpy as np
import pytest

from oracle import set_occluders
from test_chains import ALB, SPEC, chain_mesh
from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close, _assert_close_pairs, _ctx

pytestmark = pytest.mark.gpu


def _setup(oracle, w, h, nvrl, pass_):
    import alvrl
    tris, mat = chain_mesh()
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, material=mat, specular=SPEC)
    o = set_occluders(oracle.scene(w, h), tris, ALB, material=mat, specular=SPEC)
    m = oracle.medium()
    vrls, pc = oracle.trace(o, m, nvrl, seed=SEED_VRL)
    P = set_occluders(oracle.params(m, seed=SEED_RNG, pass_=pass_), tris, material=mat)
    return s, o, m, tris, mat, vrls, pc, P


def _per_pixel(vals, pix, npix):
    """Add per-record values into pixels level by level (records are in pixel
    order, depth ascending within a pixel): float32, depth order."""
    out = np.zeros((npix,) + vals.shape[1:], np.float32)
    for k in range(len(pix)):
        out[pix[k]] += vals[k]
    return out


def test_gather_brute_chains(oracle, gpu_ok):
    """Brute gather over every chain record of a 48x32 frame (the records'
    path weights, the delta surfaces' missing surface term, the null pane's
    pass-through visibility): device vs oracle per record; the chains change
    the frame (mirror images), so the test is not vacuous."""
    import torch
    w, h = 48, 32
    s, o, m, tris, mat, vrls, pc, P = _setup(oracle, w, h, 2000, 0)
    recs, pix = oracle.chains(o, m, np.arange(w * h, dtype=np.uint32), seed=SEED_RNG)
    assert len(recs) > w * h // 2 and (recs[:, 19].view(np.uint32) > 0).sum() > 100
    cpu, _ = oracle.gather_brute(P, recs, vrls, pc, rec_ids=pix)
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    ctx.set_occluders(tris, mat)
    d_out = torch.zeros((len(recs), 3), dtype=torch.float32, device="cuda")
    # the inputs stay referenced until the device is done: the context's
    # stream is not torch's, so a freed block could be reused under the kernel
    d_recs, d_pix = torch.from_numpy(recs).cuda(), torch.from_numpy(pix.view(np.int32)).cuda()
    ctx.gather_brute(d_recs, d_out, d_pix)
    torch.cuda.synchronize()
    dev = d_out.cpu().numpy()
    _assert_close(dev, cpu, "brute chain records")
    deep = recs[:, 19].view(np.uint32) > 0
    assert np.abs(cpu[deep]).max() > 0.05 * np.abs(cpu).max()
    _assert_close(_per_pixel(dev, pix, w * h), _per_pixel(cpu, pix, w * h), "brute chain pixels")


def test_rbuild_chain_rows(oracle, gpu_ok):
    """R rows of chained pixels: the depth-0 launch writes the row, each
    deeper level's launch (records flagged ALVRL_REC_ACCUM) adds into it;
    against the oracle's per-record R entries summed in depth order."""
    import torch
    import alvrl
    w, h = 40, 30
    s, o, m, tris, mat, vrls, pc, P = _setup(oracle, w, h, 1500, 0)
    ids = np.arange(0, w * h, 5, dtype=np.uint32)
    recs, pix = oracle.chains(o, m, ids, seed=SEED_RNG)
    row = np.searchsorted(ids, pix).astype(np.uint32)
    depth = recs[:, 19].view(np.uint32)
    assert depth.max() >= 2
    _, Rr, _ = oracle.gather_brute(P, recs, vrls, pc, rec_ids=pix, want_R=True, domain=2)
    Rc = _per_pixel(Rr, row, len(ids))
    ctx = _ctx()
    ctx.upload_vrls(vrls, pc)
    ctx.set_occluders(tris, mat)
    nr, nv = len(ids), vrls.shape[1]
    d_Rt = torch.zeros((nv, nr, 2), dtype=torch.float32, device="cuda")
    d_nz = torch.zeros(nv, dtype=torch.uint8, device="cuda")
    keep = []   # every level's inputs stay referenced until the launches are done
    for d in range(int(depth.max()) + 1):
        sel = np.nonzero(depth == d)[0]
        r = recs[sel].copy()
        if d:
            r[:, 15] = (r[:, 15].view(np.uint32) | alvrl.REC_ACCUM).view(np.float32)
        off = row[sel].astype(np.uint64)
        stride = np.full(len(sel), nr, np.uint32)
        keep.append((torch.from_numpy(r).cuda(), torch.from_numpy(off.view(np.int64)).cuda(),
                     torch.from_numpy(stride.view(np.int32)).cuda(), torch.from_numpy(pix[sel].view(np.int32)).cuda()))
        t_r, t_off, t_str, t_ids = keep[-1]
        ctx.build_R_blocks(t_r, d_Rt, t_off, t_str, d_nz, t_ids)
    torch.cuda.synchronize()
    Rg = d_Rt.cpu().numpy().transpose(1, 0, 2)
    _assert_close_pairs(Rg[..., 0], Rc[..., 0], "R mean chains")
    _assert_close_pairs(Rg[..., 1], Rc[..., 1], "R var chains", q50=1e-5, csum=1e-2)
    assert np.array_equal(d_nz.cpu().numpy().astype(bool), (Rc[..., 0] != 0).any(0))


@pytest.mark.parametrize("props", ["targetNumSlices=12", "localRefinement=false;globalCluster=false"])
def test_integrator_chains_matches_oracle(oracle, gpu_ok, props):
    """The integrator over the mirror/null scene: slices (buildSlices through
    the null pane) equal the oracle's; the device's R equals the oracle's
    chained rows; the cluster lists equal the oracle's clustering of the
    device's R bit for bit; the frame equals the oracle's gather over the
    chain records with those lists, per pixel."""
    import torch
    import alvrl
    from oracle import Prep
    w, h = 48, 32
    pass_ = 1
    s, o, m, tris, mat, vrls, pc, P = _setup(oracle, w, h, 600, pass_)
    it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(s)
    it.prepass(pass_)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    img = fb.view(h * w, 3).cpu().numpy()
    pid = np.arange(w * h, dtype=np.uint32)
    recs, pix = oracle.chains(o, m, pid, seed=SEED_RNG, pass_=pass_)
    if "localRefinement=false" in props:
        cpu, _ = oracle.gather_brute(P, recs, vrls, pc, rec_ids=pix)
        _assert_close(img, _per_pixel(cpu, pix, w * h), "brute chain frame")
        it.close()
        return
    # buildSlices draws nothing; sampleSliceMapping and the clustering use the pass's streams
    prep = Prep(oracle, oracle.prep_params(seed=SEED_RNG, pass_=pass_, target_num_slices=12))
    p2s = prep.build_slices(o)
    assert np.array_equal(p2s, it.slices())
    off, rpix, _, _ = prep.sample_slice_mapping(64.0, w * h)
    ioff, ipix = it.reps()
    assert np.array_equal(off, ioff) and np.array_equal(rpix, ipix)
    # R: the representatives' chains
    rid = ((ipix % h) * w + ipix // h).astype(np.uint32)          # column-major ids -> row-major
    rrecs, rr = oracle.chains(o, m, rid, seed=SEED_RNG, pass_=pass_)
    _, Rr, _ = oracle.gather_brute(P, rrecs, vrls, pc, rec_ids=rr, want_R=True, domain=2)
    row_of = {int(p): j for j, p in enumerate(rid)}
    row = np.array([row_of[int(p)] for p in rr], np.int64)
    Rc = _per_pixel(Rr, row, len(rid))
    Rg = it.R()
    _assert_close_pairs(Rg[..., 0].T, Rc[..., 0], "chained R mean")
    icl = it.clusters()
    ocl = prep.build_clusters(Rg)
    assert np.array_equal(ocl["reps"], icl["reps"])
    assert np.array_equal(ocl["weights"].view(np.uint32), icl["weights"].view(np.uint32))
    sl_pix = p2s[(pid % w) * h + pid // w]
    cpu, _ = oracle.gather_clustered(P, recs, sl_pix[pix], vrls, pc, icl["slice_off"], icl["reps"],
                                     icl["weights"], icl["fb_reps"], icl["fb_weights"], rec_ids=pix)
    deep = recs[:, 19].view(np.uint32) > 0
    assert np.abs(cpu[deep]).max() > 0
    _assert_close(img, _per_pixel(cpu, pix, w * h), "clustered chain frame")
    it.close()

