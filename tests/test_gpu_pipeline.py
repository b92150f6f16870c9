"""End-to-end parity of the vrl integrator pipeline (libalvrl.so host side +
HIP kernels) with the oracle's restatement of vrlIntegrator + Preprocessor, on
BASELINE.json configs[0]-shaped inputs (C1: 256^2 smoke box, 1k VRLs, ALVRL
defaults) and variants.

  * slicing and representative pixels: bit-exact (host code, same streams);
  * R: within the tolerance of test_gpu_parity (device maths);
  * clusters: the oracle's buildClusters run on the DEVICE's R must give
    bit-identical per-slice representatives and weights;
  * frame: the oracle's clustered gather with those clusters vs the device
    frame, within test_gpu_parity's tolerance.
"""
import os
import numpy as np
import pytest

from test_gpu_parity import _assert_close, _assert_close_pairs

pytestmark = pytest.mark.gpu

SEED_VRL = 0x5EED0001
SEED_RNG = 0xA1B2C3D4


def _run(props, w, h, nvrl, oracle, pass_=0, prep_kw=None):
    import torch
    import alvrl
    from oracle import Prep
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, nvrl, seed=SEED_VRL)
    it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(scene)
    it.prepass(pass_)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    img = fb.view(h * w, 3).cpu().numpy()

    pp = oracle.prep_params(seed=SEED_RNG, pass_=0, **(prep_kw or {}))
    prep = Prep(oracle, pp)
    osc = oracle.scene(w, h)
    p2s = prep.build_slices(osc)
    assert np.array_equal(p2s, it.slices()), "slices differ"
    off, pix, su, gu = prep.sample_slice_mapping(64.0, w * h)
    ioff, ipix = it.reps()
    assert np.array_equal(off, ioff) and np.array_equal(pix, ipix), "representatives differ"
    return it, img, prep, vrls, pc, p2s


def test_c1_pipeline_adaptive(oracle, gpu_ok):
    w = h = 256
    it, img, prep, vrls, pc, p2s = _run("", w, h, 1000, oracle)
    st = it.stats()
    assert st["slices"] == 100 and st["slices_failed"] == 0
    # R of the device against the oracle's R rows
    Rg = it.R()                                        # [nv, rows, 2]
    ioff, ipix = it.reps()
    xs, ys = ipix // h, ipix % h                       # column-major ids -> (x, y)
    rec_ids = (ys * w + xs).astype(np.uint32)
    recs = oracle.records(oracle.scene(w, h))[rec_ids]
    P = oracle.params(oracle.medium(), seed=SEED_RNG, pass_=0)
    _, Rc, cnt = oracle.gather_brute(P, recs, vrls, pc, rec_ids=rec_ids, domain=2, want_R=True)
    assert st["contrib_preprocess"] == cnt
    _assert_close_pairs(Rg[..., 0].T, Rc[..., 0], "C1 R mean")
    # buildClusters on the device's R: bit-exact per-slice lists
    ocl = prep.build_clusters(Rg)
    icl = it.clusters()
    assert np.array_equal(ocl["slice_off"], icl["slice_off"])
    assert np.array_equal(ocl["reps"], icl["reps"])
    assert np.array_equal(ocl["weights"].view(np.uint32), icl["weights"].view(np.uint32))
    print(f"C1: {len(icl['reps'])} representatives over {st['slices']} slices, "
          f"refine {st['ms_refine']:.1f} ms, R {st['ms_rbuild']:.2f} ms")
    # the frame
    pid = np.arange(w * h, dtype=np.uint32)
    sl = p2s[(pid % w) * h + pid // w]
    cpu, ccnt = oracle.gather_clustered(P, oracle.records(oracle.scene(w, h)), sl, vrls, pc,
                                        icl["slice_off"], icl["reps"], icl["weights"],
                                        icl["fb_reps"], icl["fb_weights"], rec_ids=pid)
    assert st["contrib_render"] == ccnt
    _assert_close(img, cpu, "C1 frame")


@pytest.mark.parametrize("props,prep_kw", [
    ("localUndersampling=20", {}),
    ("neighbourCount=3;neighbourWeight=0.5", {"neighbour_count": 3, "neighbour_weight": 0.5}),
    ("localRefinement=false;globalCluster=false", None),
    ("globalCluster=true;globalUndersampling=20", {"global_cluster": True, "global_undersampling": 20.0}),
    ("globalCluster=true;targetNumSlices=40", {"global_cluster": True, "target_num_slices": 40}),
    ("Rsamples=2", {}),
    # depthCorrection (Preprocessor.cpp:456-469): the adaptive refinement
    # replays its splits past the best snapshot with the scaled bound
    ("depthCorrection=0.8", {"depth_correction": 0.8}),
    ("depthCorrection=1.3;targetNumSlices=60", {"depth_correction": 1.3, "target_num_slices": 60}),
])
def test_pipeline_variants(oracle, gpu_ok, props, prep_kw):
    import alvrl
    w, h = 128, 96
    if prep_kw is None:   # brute force: no slices
        import torch
        scene = alvrl.scene_default(w, h)
        vrls, pc = alvrl.trace_vrls(scene, 600, seed=SEED_VRL)
        it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        it.prepass(3)
        fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        it.render(fb)
        torch.cuda.synchronize()
        P = oracle.params(oracle.medium(), seed=SEED_RNG, pass_=3)
        cpu, _ = oracle.gather_brute(P, oracle.records(oracle.scene(w, h)), vrls, pc)
        _assert_close(fb.view(-1, 3).cpu().numpy(), cpu, "brute pipeline")
        return
    pk = dict(target_num_slices=100)
    pk.update(prep_kw)
    under = float(props.split("localUndersampling=")[1]) if "localUndersampling=" in props else -1.0
    pk["local_undersampling"] = under
    it, img, prep, vrls, pc, p2s = _run(props, w, h, 600, oracle, prep_kw=pk)
    ocl = prep.build_clusters(it.R())
    icl = it.clusters()
    if pk.get("global_cluster"):
        assert it.stats()["global_clusters"] > 1
    assert np.array_equal(ocl["reps"], icl["reps"])
    assert np.array_equal(ocl["weights"].view(np.uint32), icl["weights"].view(np.uint32))


def test_tile_sharding_covers_frame(gpu_ok):
    """Ranks' tile sets partition the frame: the sum of 3 'rank' renders equals
    the 1-rank render bit for bit (each pixel is written by exactly one rank)."""
    import torch
    import alvrl
    w, h = 200, 130
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, 300, seed=SEED_VRL)
    it = alvrl.Integrator(f"localRefinement=false;seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(scene)
    it.prepass(0)
    full = torch.zeros(w * h * 3, device="cuda")
    it.render(full)
    parts = torch.zeros(w * h * 3, device="cuda")
    for r in range(3):
        it.render(parts, rank=r, world=3)
    torch.cuda.synchronize()
    assert torch.equal(full, parts)


def test_golden_c1_small_device(oracle, gpu_ok):
    """The committed fixtures (tests/golden/c1_small.npz, vrls_c1.txt) against
    the device.  Fast paths: brute frame and R rows within test_gpu_parity's
    tolerance.  Strict R build (strictRbuild): the fixture's R rows bit for
    bit, and the integrator pipeline (host slicing + strict device R + device
    refinement) gives the fixture's slice map, representatives and cluster
    lists bit for bit -- the oracle's own clustering of its own R -- and its
    clustered frame matches the fixture's on the gather tolerance."""
    import os
    import torch
    import alvrl
    from test_gpu_strict import _assert_bits
    gdir = os.path.join(os.path.dirname(__file__), "golden")
    g = np.load(os.path.join(gdir, "c1_small.npz"))
    w, h = 48, 32
    vrls, pc = alvrl.read_vrl_file(os.path.join(gdir, "vrls_c1.txt"))
    assert pc == vrls.shape[1] == 256
    recs = alvrl.scene_records(alvrl.scene_default(w, h))
    ctx = alvrl.Context(device=0, seed=SEED_RNG)
    ctx.set_medium(alvrl.Medium())
    ctx.upload_vrls(vrls, pc)
    d_out = torch.zeros((w * h, 3), dtype=torch.float32, device="cuda")
    ctx.gather_brute(torch.from_numpy(recs).cuda(), d_out)
    rows = g["R_rows"]
    d_rows, d_ids = torch.from_numpy(recs[rows]).cuda(), torch.from_numpy(rows.view(np.int32)).cuda()
    d_Rt = torch.zeros((vrls.shape[1], len(rows), 2), dtype=torch.float32, device="cuda")
    ctx.build_R(d_rows, d_Rt, ld=len(rows), d_ids=d_ids)
    d_Rs = torch.zeros_like(d_Rt)
    ctx.set_strict_rbuild(True)
    ctx.build_R(d_rows, d_Rs, ld=len(rows), d_ids=d_ids)
    torch.cuda.synchronize()
    _assert_close(d_out.cpu().numpy(), g["brute"], "golden brute")
    _assert_close_pairs(d_Rt.cpu().numpy()[..., 0].T, g["R"][..., 0], "golden R mean")
    _assert_bits(d_Rs.cpu().numpy().transpose(1, 0, 2), g["R"], "golden R, strict build")

    it = alvrl.Integrator(f"targetNumSlices=12;strictRbuild=true;seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(alvrl.scene_default(w, h))
    it.prepass(0)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    assert np.array_equal(it.slices(), g["slices"])
    off, pix = it.reps()
    assert np.array_equal(off, g["rep_off"]) and np.array_equal(pix, g["rep_pix"])
    cl = it.clusters()
    assert np.array_equal(cl["slice_off"], g["cl_slice_off"]) and np.array_equal(cl["reps"], g["cl_reps"])
    assert np.array_equal(cl["weights"].view(np.uint32), g["cl_weights"].view(np.uint32))
    if it.stats()["fallback_built"]:   # built lazily (deviation 4)
        assert np.array_equal(cl["fb_reps"], g["cl_fb_reps"])
        assert np.array_equal(cl["fb_weights"].view(np.uint32), g["cl_fb_weights"].view(np.uint32))
    _assert_close(fb.view(-1, 3).cpu().numpy(), g["clustered"], "golden clustered")


def test_sharded_prepass(gpu_ok, tmp_path):
    """The slice-sharded prepass (alvrl_integrator_prepass_dist):
    2 gloo ranks on the one GPU, see tests/gpu_dist_worker.py.  Cluster lists
    and the frame are identical to the one-GPU prepass bit for bit; without
    neighbours every slice and R row is built exactly once over the ranks.
    The 'samples' case renders three jittered sensor samples per pixel
    (sampleCount) on each rank's tiles."""
    import json
    import os
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "verdict.json"
    here = os.path.dirname(os.path.abspath(__file__))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(here, "gpu_dist_worker.py"), str(out)]
    r = subprocess.run(cmd, env=dict(os.environ, OMP_NUM_THREADS="4"), capture_output=True, text=True,
                       timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    v = json.loads(out.read_text())
    print(v)
    assert v["world"] == 2
    for name in ("adaptive", "neighbours", "fixed", "global", "samples"):
        c = v[name]
        assert c["clusters_identical_all_ranks"] and c["frame_bit_exact"], name
        assert c["slices_sum"] == c["slices"], name
        if name == "neighbours":
            assert c["rows_sum"] >= c["rows"], name
        elif name == "global":     # the global refinement needs every row on every rank
            assert c["rows_sum"] == 2 * c["rows"], name
        else:
            assert c["pairs_sum"] == c["pairs_one"] and c["rows_sum"] == c["rows"], name


@pytest.mark.parametrize("gu", [15.0, -1.0])
def test_refine_members(oracle, gpu_ok, gu):
    """alvrl_refine_members (clusterRefinement + getVrlsPerCluster) against the
    oracle on the same R: identical member order and cluster offsets."""
    import torch
    import alvrl
    w, h = 96, 64
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, 500, seed=SEED_VRL)
    rows = np.arange(0, w * h, 37, dtype=np.uint32)
    recs = alvrl.scene_records(scene, rows)
    ctx = alvrl.Context(device=0, seed=SEED_RNG)
    ctx.set_medium(alvrl.Medium())
    ctx.upload_vrls(vrls, pc)
    nv = vrls.shape[1]
    d_Rt = torch.zeros((nv, len(rows), 2), dtype=torch.float32, device="cuda")
    ctx.build_R(torch.from_numpy(recs).cuda(), d_Rt, ld=len(rows),
                d_ids=torch.from_numpy(rows.view(np.int32)).cuda())
    torch.cuda.synchronize()
    Rt = d_Rt.cpu().numpy()
    nz = np.nonzero((Rt[..., 0] != 0).any(axis=1))[0].astype(np.uint32)
    lrows = np.arange(len(rows), dtype=np.uint32)
    locw = np.full(len(rows), 1.0 / len(rows))
    job = dict(rows=lrows, locw=locw, pixel_undersampling=0.25, undersampling=gu)
    mem, off, ok = ctx.refine_members(d_Rt, len(rows), job, nz, [0, len(nz)])
    omem, ooff, ook = oracle.cluster_members(Rt, lrows, locw, nz, [0, len(nz)], 0.25, gu)
    assert ok and ook
    print(f"global clusters: {len(off) - 1} (device) {len(ooff) - 1} (oracle)")
    assert np.array_equal(off, ooff) and np.array_equal(mem, omem)


def test_false_color_modes(gpu_ok):
    """numVrlFalseColor / slicesFalseColor (vrlIntegrator.cpp:545-599, 794-806)
    against their closed forms from the integrator's own slice map and
    cluster lists; slicesFalseColor without clustering is an error, and
    convergenceFalseColor leaves a diffuse-only frame unchanged (:514-521)."""
    import torch
    import alvrl
    w, h = 128, 96
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, 400, seed=SEED_VRL)
    nv = vrls.shape[1]

    def frame(props):
        it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        it.prepass(0)
        fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        it.render(fb)
        torch.cuda.synchronize()
        return it, fb.view(h, w, 3).cpu().numpy()

    it, img = frame("targetNumSlices=20;numVrlFalseColor=true")
    cl, p2s = it.clusters(), it.slices()
    sizes = np.diff(cl["slice_off"]).astype(np.float32)
    ys, xs = np.mgrid[0:h, 0:w]
    sl = p2s[ys + h * xs]                                        # m_slices[y + H*x]
    k = np.where(sl == 0xFFFFFFFF, np.float32(len(cl["fb_reps"])), sizes[np.minimum(sl, len(sizes) - 1)])
    assert np.array_equal(img[..., 0], (k / np.float32(nv)).astype(np.float32))
    assert it.stats()["contrib_render"] == int(k.sum())

    it, img = frame("targetNumSlices=20;slicesFalseColor=true")
    s = sl.astype(np.uint32)
    col = np.stack([((s + s * s) % 43) / 43.0, ((7 * s + 2 * s * s + 7) % 41) / 41.0,
                    ((23 * s + 5 * s * s + s * s * s + 17) % 53) / 53.0], axis=-1).astype(np.float32)
    col[sl == 0xFFFFFFFF] = 0.5
    assert np.array_equal(img, col)

    _, img = frame("localRefinement=false;numVrlFalseColor=true")
    assert (img == 1.0).all()
    with pytest.raises(alvrl.AlvrlError):
        frame("localRefinement=false;slicesFalseColor=true")
    _, a = frame("targetNumSlices=20;convergenceFalseColor=true")
    _, b = frame("targetNumSlices=20")
    assert np.array_equal(a, b)


# every environment knob of the refine kernel's team mode (refine.hip host
# side): saved, cleared and restored by the team tests so no value leaks in
TEAM_ENV_KEYS = ("ALVRL_REFINE_TEAM", "ALVRL_REFINE_ROAM", "ALVRL_SPEC_WIDTH", "ALVRL_SPEC_MIN",
                 "ALVRL_REFINE_SPIN_MS", "ALVRL_ENQ_START", "ALVRL_LEADER_SIDE",
                 "ALVRL_LEADER_WAIT_TICKS", "ALVRL_REFINE_TEAM_STATS", "ALVRL_ROAM_ORDER",
                 "ALVRL_TEAM_SETUP", "ALVRL_EARLY_SPEC", "ALVRL_VAR_SMALL", "ALVRL_REFINE_NROAM",
                 "ALVRL_FINISHED_ROAM", "ALVRL_SPLIT_FUSED")


def test_team_mode_settings(gpu_ok):
    """Speculative split teams (refine.hip team mode) under every knob: team
    size, roaming helpers, speculation width and threshold, and a 1 ms bound
    on every wait (leaders give up on running helpers and split themselves,
    idle helpers leave).  The cluster lists must equal those of one workgroup
    per slice bit for bit in every case."""
    import os
    import torch
    import alvrl
    w, h = 256, 192
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, 3000, seed=SEED_VRL)
    keys = TEAM_ENV_KEYS
    saved = {k: os.environ.get(k) for k in keys}

    def run(props, **env):
        for k in keys:
            os.environ.pop(k, None)
        os.environ.update({k: str(v) for k, v in env.items()})
        it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        it.prepass(1)
        cl = it.clusters()
        it.close()
        return cl

    settings = [dict(ALVRL_REFINE_TEAM=2), dict(ALVRL_REFINE_TEAM=4, ALVRL_REFINE_ROAM=0),
                dict(ALVRL_REFINE_TEAM=8), dict(ALVRL_SPEC_WIDTH=1, ALVRL_SPEC_MIN=2),
                dict(ALVRL_SPEC_WIDTH=32, ALVRL_SPEC_MIN=2), dict(ALVRL_REFINE_SPIN_MS=1),
                dict(ALVRL_REFINE_TEAM=3, ALVRL_REFINE_SPIN_MS=1, ALVRL_SPEC_MIN=2),
                dict(ALVRL_ENQ_START=1), dict(ALVRL_LEADER_SIDE=0, ALVRL_REFINE_SPIN_MS=1),
                dict(ALVRL_LEADER_WAIT_TICKS=0), dict(ALVRL_TEAM_SETUP=0),
                dict(ALVRL_TEAM_SETUP=1, ALVRL_REFINE_ROAM=0), dict(ALVRL_EARLY_SPEC=0),
                dict(ALVRL_EARLY_SPEC=1, ALVRL_REFINE_ROAM=0, ALVRL_LEADER_WAIT_TICKS=0), dict(ALVRL_VAR_SMALL=0),
                dict(ALVRL_REFINE_NROAM=3, ALVRL_FINISHED_ROAM=0), dict(ALVRL_SPLIT_FUSED=0),
                dict(ALVRL_SPLIT_FUSED=1), {}]
    try:
        for props in ("targetNumSlices=40", "targetNumSlices=30;localUndersampling=10",
                      "targetNumSlices=25;depthCorrection=0.8"):
            ref = run(props, ALVRL_REFINE_TEAM=1)
            for st in settings:
                cl = run(props, **st)
                for k in ref:
                    assert np.array_equal(ref[k].view(np.uint32), cl[k].view(np.uint32)), (props, st, k)
        torch.cuda.synchronize()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_team_wait_timeout(gpu_ok, capfd):
    """A leader that gives up waiting on a running helper (refine.hip
    split_team, wait bound 0 ticks here) retires its job's team and splits
    that cluster and every later one itself; the helper's late result in
    team.spec / team.res / state is never committed.  Large clusters (few
    slices, 20k VRLs) keep helpers mid-split when their leader pops the
    cluster.  The cluster lists equal one workgroup per slice bit for bit,
    and the team counters show that timeouts happened."""
    import os
    import re
    import alvrl
    w, h = 256, 192
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, 20000, seed=SEED_VRL)
    saved = {k: os.environ.get(k) for k in TEAM_ENV_KEYS}

    def run(props, **env):
        for k in TEAM_ENV_KEYS:
            os.environ.pop(k, None)
        os.environ.update({k: str(v) for k, v in env.items()})
        it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        it.prepass(1)
        cl = it.clusters()
        it.close()
        return cl

    timeouts = 0
    try:
        for props in ("targetNumSlices=6", "targetNumSlices=4;localUndersampling=4"):
            ref = run(props, ALVRL_REFINE_TEAM=1)
            capfd.readouterr()
            for st in (dict(ALVRL_LEADER_WAIT_TICKS=0), dict(ALVRL_LEADER_WAIT_TICKS=0, ALVRL_REFINE_TEAM=8),
                       dict(ALVRL_LEADER_WAIT_TICKS=2000, ALVRL_REFINE_ROAM=0)):
                cl = run(props, ALVRL_REFINE_TEAM_STATS=1, **st)
                err = capfd.readouterr().err
                m = re.search(r"wait-timeout (\d+)", err)
                assert m, err
                timeouts += int(m.group(1))
                for k in ref:
                    assert np.array_equal(ref[k].view(np.uint32), cl[k].view(np.uint32)), (props, st, k)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert timeouts > 0


@pytest.mark.parametrize("props", ["targetNumSlices=100;localUndersampling=-1",
                                   "targetNumSlices=100;localUndersampling=100"])
def test_refine_c4_scale(oracle, gpu_ok, props):
    """The benchmark's own configs (C4 / C3: 1024^2, 100k VRLs, 100 slices,
    team mode with speculation and roaming helpers as by default).

      * refinement: the oracle's Clustering (Preprocessor.cpp:254-283, strict
        build) on the device's job for three slices -- the most rows, the
        most clusters and a median one -- gives the device's cluster lists
        bit for bit (representatives and weights);
      * frame: every 64th image row of the device's full-frame render
        (getClusteredVrlContributions, vrlIntegrator.cpp:542-599, through
        alvrl_integrator_render) against the oracle's clustered gather with
        the device's cluster lists, on test_gpu_parity's tolerance."""
    import torch
    import alvrl
    W = H = 1024
    scene = alvrl.scene_default(W, H)
    vrls, pc = alvrl.trace_vrls(scene, 100000, seed=SEED_VRL)
    it = alvrl.Integrator(props + f";seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(scene)
    it.prepass(2)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    img = fb.view(H * W, 3).cpu().numpy()
    cl = it.clusters()
    p2s = it.slices()
    pid = (np.arange(0, H, 64, dtype=np.uint32)[:, None] * W + np.arange(W, dtype=np.uint32)[None, :]).ravel()
    sl = p2s[(pid % W) * H + pid // W]                 # m_slices[y + H*x]
    recs = oracle.records(oracle.scene(W, H))[pid]
    P = oracle.params(oracle.medium(), seed=SEED_RNG, pass_=2)
    cpu, _ = oracle.gather_clustered(P, recs, sl, vrls, pc, cl["slice_off"], cl["reps"], cl["weights"],
                                     cl["fb_reps"], cl["fb_weights"], rec_ids=pid)
    assert (sl != 0xFFFFFFFF).all() and img.any()
    _assert_close(img[pid], cpu, f"{props} frame, every 64th row")
    off, _ = it.reps()
    nrows, ncl = np.diff(off), np.diff(cl["slice_off"])
    kv = dict(x.split("=", 1) for x in props.split(";"))
    under = float(kv["localUndersampling"])
    picks = sorted({int(np.argmax(nrows)), int(np.argmax(ncl)), int(np.argsort(ncl)[len(ncl) // 2])})
    for s in picks:
        job = it.slice_job(s)
        n = job["R"].shape[1]
        reps, w, refined = oracle.cluster_refine(job["R"], np.arange(n, dtype=np.uint32), job["locw"],
                                                 job["init_vrls"], job["init_off"], job["pixel_undersampling"],
                                                 under, seed=SEED_RNG, pass_=2, stage_refine=3 + 2 * s,
                                                 stage_sample=4 + 2 * s)
        assert refined
        b, e = cl["slice_off"][s], cl["slice_off"][s + 1]
        assert np.array_equal(reps, cl["reps"][b:e]), (s, n, len(reps), e - b)
        assert np.array_equal(w.view(np.uint32), cl["weights"][b:e].view(np.uint32)), s
    it.close()


def test_context_reuse_across_passes(gpu_ok):
    """One integrator re-used over passes whose sizes grow and shrink (VRL
    counts 3000 -> 9000 -> 3000, slice counts 40 -> 25): alvrl_refine's device
    scratch and the cluster lists' device buffers are kept by the context
    between passes (grow-only), so every pass must give the cluster lists and
    the frame of a fresh integrator bit for bit."""
    import torch
    import alvrl
    w, h = 256, 192
    scene = alvrl.scene_default(w, h)
    sets = [alvrl.trace_vrls(scene, n, seed=SEED_VRL + n) for n in (3000, 9000, 3000)]
    props = [f"targetNumSlices=40;seed={SEED_RNG}", f"targetNumSlices=40;seed={SEED_RNG}",
             f"targetNumSlices=25;seed={SEED_RNG}"]

    def run(it, k, pass_):
        it.prepass(pass_)
        fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        it.render(fb)
        torch.cuda.synchronize()
        return it.clusters(), fb.cpu().numpy()

    fresh = []
    for k, (vrls, pc) in enumerate(sets):
        it = alvrl.Integrator(props[k], device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        fresh.append(run(it, k, k + 1))
        it.close()
    it = alvrl.Integrator(props[0], device=0)
    it.preprocess(scene)
    for k, (vrls, pc) in enumerate(sets):
        if k == 2:   # fewer slices: a new integrator state, the same context scratch is not shared
            it.close()
            it = alvrl.Integrator(props[k], device=0)
            it.preprocess(scene)
        it.set_vrls(vrls, pc)
        cl, fb = run(it, k, k + 1)
        for key in cl:
            assert np.array_equal(cl[key].view(np.uint32), fresh[k][0][key].view(np.uint32)), (k, key)
        assert np.array_equal(fb.view(np.uint32), fresh[k][1].view(np.uint32)), k
    it.close()


def test_cluster_info_checkpoint(gpu_ok, tmp_path):
    """vrlClusterInfo out of one integrator and into another (the resource the
    reference ships to remote workers, vrlIntegrator.cpp:29-101, :353-354):
    the second renders the same frame bit for bit without R build or
    refinement; the frame goes through the EXR writer unchanged."""
    import torch
    import alvrl
    w, h = 48, 32
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, 600, seed=SEED_VRL)
    frames = []
    for load in (False, True):
        it = alvrl.Integrator(f"targetNumSlices=12;seed={SEED_RNG}", device=0)
        it.set_vrls(vrls, pc)
        it.preprocess(scene)
        if load:
            it.load_cluster_info(str(tmp_path / "ci.bin"), 0)
            assert it.stats()["refine_entries"] == 0
        else:
            it.prepass(0)
            it.save_cluster_info(str(tmp_path / "ci.bin"))
        fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        it.render(fb)
        torch.cuda.synchronize()
        frames.append(fb.cpu().numpy())
        it.close()
    assert frames[0].any()
    assert np.array_equal(frames[0].view(np.uint32), frames[1].view(np.uint32))
    ci = alvrl.read_cluster_info(str(tmp_path / "ci.bin"))
    assert len(ci["slices"]) == w * h and len(ci["slice_off"]) == 13
    p = str(tmp_path / alvrl.pass_file_name("smoke", 0, 0, 0, 0, 0, 0, 0).split("/")[-1])
    alvrl.write_exr(p, frames[0].reshape(h, w, 3))
    assert np.array_equal(alvrl.read_exr(p).ravel(), frames[0])
    assert alvrl.image_rms(frames[1], frames[0]) == 0.0


@pytest.mark.parametrize("target,short,max_depth,rr_depth,pass_", [
    (700, True, -1, 5, 0), (300, False, -1, 5, 0), (500, True, 3, 5, 2), (400, True, -1, 1, 1),
    (100003, True, -1, 5, 0)])
def test_gpu_tracer_matches_host(oracle, gpu_ok, target, short, max_depth, rr_depth, pass_):
    """vrlTracer::randomWalk on the device (csrc/tracer.hip)
    gives the host tracer's VRL set and particle count bit for bit (the host
    tracer is itself bit-exact with the oracle, tests/test_host.py)."""
    import alvrl
    s = alvrl.scene_default(16, 16)
    host, hpc = alvrl.trace_vrls(s, target, seed=SEED_VRL, pass_=pass_, short_vrls=short,
                                 max_depth=max_depth, rr_depth=rr_depth)
    dev, dpc = alvrl.trace_vrls_gpu(s, target, seed=SEED_VRL, pass_=pass_, short_vrls=short,
                                    max_depth=max_depth, rr_depth=rr_depth)
    assert dpc == hpc and dev.shape == host.shape
    assert np.array_equal(dev.view(np.uint32), host.view(np.uint32))
    if target <= 1000:
        ref, rpc = oracle.trace(oracle.scene(16, 16), oracle.medium(), target, seed=SEED_VRL, pass_=pass_,
                                short_vrls=short, max_depth=max_depth, rr_depth=rr_depth)
        assert rpc == dpc and np.array_equal(ref.view(np.uint32), dev.view(np.uint32))


def test_integrator_gpu_tracer(gpu_ok):
    """prepass with gpuTracer=true traces on the device; the pass (VRLs,
    clusters, frame) is the host-traced one bit for bit."""
    import torch
    import alvrl
    w, h = 32, 24
    scene = alvrl.scene_default(w, h)
    out = []
    for gt in ("false", "true"):
        it = alvrl.Integrator(f"targetNumSlices=8;vrlTargetNum=800;gpuTracer={gt};seed={SEED_RNG}", device=0)
        it.preprocess(scene)
        it.prepass(1)
        fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        it.render(fb)
        torch.cuda.synchronize()
        out.append((it.vrls(), it.clusters(), fb.cpu().numpy()))
        it.close()
    (v0, p0), c0, f0 = out[0]
    (v1, p1), c1, f1 = out[1]
    assert p0 == p1 and np.array_equal(v0.view(np.uint32), v1.view(np.uint32))
    assert np.array_equal(c0["reps"], c1["reps"])
    assert np.array_equal(f0.view(np.uint32), f1.view(np.uint32))
