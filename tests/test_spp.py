"""Multi-sample renders (the sampler's sampleCount; renderBlock's sample loop,
integrator.cpp:240-264): sensor sample j of spp is the pixel centre for one
sample per pixel, else the pixel corner plus rRec.nextSample2D(), drawn here
from the counter stream (seed, pass, dom 8, pixel, j).  The product's host
records and chains must equal the oracle's bit for bit; sample 0 of a
single-sample render is the old pixel-centre record."""
import numpy as np
import pytest

from oracle import set_occluders
from test_chains import ALB, SPEC, chain_mesh


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


def test_records_spp_match_oracle(alvrl, oracle):
    w, h, spp = 24, 16, 4
    s = alvrl.scene_default(w, h)
    o = oracle.scene(w, h)
    ids = np.array([0, 7, 100, w * h - 1, 55], np.uint32)
    for seed, pass_ in ((0xA1B2C3D4, 0), (0x1234, 3)):
        mine = alvrl.scene_records_spp(s, spp, pixel_ids=ids, seed=seed, pass_=pass_)
        ref, pix = oracle.records_spp(o, ids, spp, seed=seed, pass_=pass_)
        assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
        assert np.array_equal(pix, np.tile(ids, spp))
        # the depth word carries the sample; the eye rays differ per sample
        assert np.array_equal(mine[:, 19].view(np.uint32), np.repeat(np.arange(spp, dtype=np.uint32), len(ids)) << 16)
        d = mine[:, 3:6].reshape(spp, len(ids), 3)
        assert all(not np.array_equal(d[0], d[j]) for j in range(1, spp))
    # one sample per pixel: the pixel centres, as the single-sample records
    one = alvrl.scene_records_spp(s, 1, pixel_ids=ids)
    assert np.array_equal(one.view(np.uint32), alvrl.scene_records(s, pixel_ids=ids).view(np.uint32))


def test_records_spp_jitter_stays_in_pixel(alvrl, oracle):
    """The sample positions cover the pixel square: the eye directions of a
    pixel's samples lie between those of its corners' neighbours (the camera
    maps x to a monotone direction), and their mean is near the centre ray."""
    w, h, spp = 8, 8, 64
    s = alvrl.scene_default(w, h)
    ids = np.array([27], np.uint32)
    r = alvrl.scene_records_spp(s, spp, pixel_ids=ids)
    c = alvrl.scene_records(s, pixel_ids=ids)[0]
    left = alvrl.scene_records(s, pixel_ids=np.array([26], np.uint32))[0]
    right = alvrl.scene_records(s, pixel_ids=np.array([28], np.uint32))[0]
    lo, hi = sorted((left[3], right[3]))
    assert ((r[:, 3] > lo) & (r[:, 3] < hi)).all()
    assert abs(r[:, 3].mean() - c[3]) < 0.25 * (hi - lo)


@pytest.mark.parametrize("pass_", [0, 2])
def test_chains_spp_match_oracle(alvrl, oracle, pass_):
    w, h, spp = 40, 30, 3
    tris, mat = chain_mesh()
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, material=mat, specular=SPEC)
    o = set_occluders(oracle.scene(w, h), tris, ALB, material=mat, specular=SPEC)
    m = oracle.medium()
    deep = 0
    for p in range(0, w * h, 37):
        x, y = p % w, p // w
        for j in range(spp):
            mine = alvrl.scene_chain_spp(s, x, y, j, spp, pass_=pass_, spec_rr_depth=2)
            ref = oracle.chain_s(o, m, x, y, j, spp, pass_=pass_, spec_rr_depth=2)
            assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
            k = mine[:, 19].view(np.uint32)
            assert np.array_equal(k >> 16, np.full(len(k), j, np.uint32))
            assert np.array_equal(k & 0xFFFF, np.arange(len(k), dtype=np.uint32))
            deep += len(k) > 1
        assert np.array_equal(alvrl.scene_chain_spp(s, x, y, 0, 1, pass_=pass_).view(np.uint32),
                              alvrl.scene_chain(s, x, y, pass_=pass_).view(np.uint32))
    assert deep > 0


def test_integrator_sample_count_validation(alvrl):
    for bad in ("sampleCount=0", "sampleCount=70000"):
        with pytest.raises(alvrl.AlvrlError, match="sampleCount"):
            alvrl.Integrator(bad)
