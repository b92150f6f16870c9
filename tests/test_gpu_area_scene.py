"""A scene the point-light smoke box cannot express -- an area emitter and a
medium bounded by a closed, rotated triangle mesh (tests/test_area_emitter.py)
-- on the device, against the oracle:

  * the GPU tracer (csrc/tracer.hip) = the host tracer = the oracle, bit for
    bit;
  * the host-cast pipeline (the Mitsuba plugin's records mode: the host casts
    the slicing rays and the representative pixels' eye paths,
    alvrl_integrator_preprocess_ext / _prepass_records) with the strict R
    build against the ORACLE's OWN pipeline on the same scene: slices,
    representatives, R and cluster lists bit for bit, the frame on the gather
    tolerance of test_gpu_parity.py;
  * the descriptor pipeline (frame mode) with the device tracer: the same
    pass as with the host tracer, bit for bit.
"""
import numpy as np
import pytest

from test_area_emitter import area_scene
from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close
from test_gpu_strict import _assert_bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


@pytest.mark.parametrize("target,short", [(1500, True), (600, False), (100003, True)])
def test_area_gpu_tracer(alvrl, oracle, gpu_ok, target, short):
    s, o, _ = area_scene(alvrl, oracle, 16, 16)
    host, hpc = alvrl.trace_vrls(s, target, seed=SEED_VRL, short_vrls=short)
    dev, dpc = alvrl.trace_vrls_gpu(s, target, seed=SEED_VRL, short_vrls=short)
    assert dpc == hpc and dev.shape == host.shape
    assert np.array_equal(dev.view(np.uint32), host.view(np.uint32))
    if target <= 2000:
        ref, rpc = oracle.trace(o, oracle.medium(), target, seed=SEED_VRL, short_vrls=short)
        assert rpc == dpc and np.array_equal(ref.view(np.uint32), dev.view(np.uint32))


@pytest.mark.parametrize("vrl_source", ["set_vrls", "library_gpu_tracer"])
def test_area_scene_records_mode_vs_oracle(alvrl, oracle, gpu_ok, vrl_source):
    """vrl_source "library_gpu_tracer" is the Mitsuba plugin's records mode:
    the scene's transport descriptor goes in as alvrl_scene_ext::tracer and
    the prepass traces the pass's VRLs on the device (gpuTracer=true); they
    must be the oracle's vrlTracer output bit for bit."""
    import torch
    from oracle import Prep
    w, h, pass_ = 96, 64, 1
    s, o, tris = area_scene(alvrl, oracle, w, h)
    lib_tracer = vrl_source == "library_gpu_tracer"
    props = f"targetNumSlices=24;seed={SEED_RNG}"      # the default pipeline: strict R build
    if lib_tracer:
        props += f";vrlTargetNum=3000;vrlSeed={SEED_VRL}"      # gpuTracer: the default
        vrls, pc = oracle.trace(o, oracle.medium(), 3000, seed=SEED_VRL, pass_=pass_)
    else:
        vrls, pc = alvrl.trace_vrls(s, 3000, seed=SEED_VRL)
    it = alvrl.Integrator(props, device=0)
    try:
        if not lib_tracer:
            it.set_vrls(vrls, pc)
        # the host plays Mitsuba: buildSlices' gather points, then each
        # representative pixel's eye record (no delta BSDF: one segment each)
        sr = np.stack([alvrl.scene_slice_record(s, x, y) for y in range(h) for x in range(w)])
        it.preprocess_ext(w, h, sr, list(s.box_min), list(s.box_max), alvrl.Medium(), tris,
                          tracer=s if lib_tracer else None)
        pix = it.rep_pixels(pass_)
        recs = alvrl.scene_records(s, pix)
        it.prepass_records(pass_, recs, np.arange(len(pix), dtype=np.uint32))
        if lib_tracer:
            dv, dpc = it.vrls()
            assert dpc == pc and dv.shape == vrls.shape, (dpc, pc, dv.shape, vrls.shape)
            assert np.array_equal(dv.view(np.uint32), vrls.view(np.uint32)), "device-traced VRLs vs oracle"
        # the oracle's own pipeline on its own scene
        prep = Prep(oracle, oracle.prep_params(seed=SEED_RNG, pass_=pass_, target_num_slices=24))
        p2s = prep.build_slices(o)
        off, opix, _, _ = prep.sample_slice_mapping(64.0, w * h)
        assert np.array_equal(it.slices(), p2s), "slices"
        assert np.array_equal(pix, ((opix % h) * w + opix // h).astype(np.uint32)), "representatives"
        orecs = oracle.records(o)
        assert np.array_equal(recs.view(np.uint32), orecs[pix].view(np.uint32)), "eye records"
        P = oracle.params(oracle.medium(), seed=SEED_RNG, pass_=pass_)
        from oracle import set_occluders
        P = set_occluders(P, tris)
        _, R, _ = oracle.gather_brute(P, orecs[pix], vrls, pc, rec_ids=pix, domain=2, want_R=True)
        _assert_bits(it.R().transpose(1, 0, 2), R, "area scene R (records mode, strict)")
        ocl = prep.build_clusters(np.ascontiguousarray(R.transpose(1, 0, 2)))
        cl = it.clusters()
        for k in ("slice_off", "reps", "weights"):
            assert np.array_equal(cl[k].view(np.uint32), ocl[k].view(np.uint32)), k
        # render: the host's records of every pixel through the context's gather
        allpix = np.arange(w * h, dtype=np.uint32)
        arecs = alvrl.scene_records(s)
        sl = p2s[(allpix % w) * h + allpix // w]
        rgb = it.context().gather_clustered_host(arecs, sl, ids=allpix)
        cpu, _ = oracle.gather_clustered(P, orecs, sl, vrls, pc, ocl["slice_off"], ocl["reps"], ocl["weights"],
                                         ocl["fb_reps"], ocl["fb_weights"], rec_ids=allpix)
        assert cpu.any()
        _assert_close(rgb, cpu, "area scene frame (records mode)")
    finally:
        it.close()


def test_area_scene_descriptor_gpu_tracer(alvrl, oracle, gpu_ok):
    import torch
    w, h = 64, 48
    s, _, _ = area_scene(alvrl, oracle, w, h)
    out = []
    for gt in ("false", "true"):
        it = alvrl.Integrator(f"targetNumSlices=16;vrlTargetNum=2000;gpuTracer={gt};seed={SEED_RNG}", device=0)
        it.preprocess(s)
        it.prepass(2)
        fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        it.render(fb)
        torch.cuda.synchronize()
        out.append((it.vrls(), it.clusters(), fb.cpu().numpy()))
        it.close()
    (v0, p0), c0, f0 = out[0]
    (v1, p1), c1, f1 = out[1]
    assert p0 == p1 and np.array_equal(v0.view(np.uint32), v1.view(np.uint32))
    for k in c0:
        assert np.array_equal(c0[k].view(np.uint32), c1[k].view(np.uint32)), k
    assert f0.any() and np.array_equal(f0.view(np.uint32), f1.view(np.uint32))
