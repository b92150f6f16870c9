"""Delta-BSDF occluders ("specular chains"): mirrors (smooth
conductor, material "none": conductor.cpp:254-268) and null surfaces
(null.cpp:38-76) inside the smoke box.

LiInternal (vrlIntegrator.cpp:398-524) follows a delta BSDF's sampled
direction and gathers again at the next hit, with the path weight
transmittance * bsdfWeight / rrProb (:505) and Russian roulette on
throughputWithEtaSq (initialSpecularThroughput, :480-492; maxRR 0.98 from
specularForcedRRdepth on).  Null surfaces pass Scene::evalTransmittance
(scene.cpp:633-676) and the slicing ray (Preprocessor.cpp:1157-1169), and cut
VRLs in the tracer (vrlTracer.h:173-213).

CPU part: the product's host harness (eye chains, slicing records, the VRL
tracer) against the oracle, BIT FOR BIT.  The device gathers and the
integrator over such scenes are in test_gpu_chains.py."""
import numpy as np
import pytest

from oracle import MAT_DIFFUSE, MAT_MIRROR, MAT_NULL, set_occluders

REC_DELTA = 8
SEED = 0xA1B2C3D4


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


def quad(p0, p1, p2, p3, facing):
    """Two triangles (p0 p1 p2), (p0 p2 p3), wound so the face normal points
    along 'facing'."""
    p = [np.asarray(x, np.float32) for x in (p0, p1, p2, p3)]
    n = np.cross(p[1] - p[0], p[2] - p[0])
    if np.dot(n, facing) < 0:
        p = [p[0], p[3], p[2], p[1]]
    return np.stack([np.concatenate([p[0], p[1], p[2]]), np.concatenate([p[0], p[2], p[3]])]).astype(np.float32)


def chain_mesh():
    """Two facing mirrors on the side walls (long chains, Russian roulette),
    a tilted mirror at the back, a null pane in the middle of the box and a
    diffuse plate; returns (triangles, materials)."""
    parts = [
        (quad([-0.95, -0.45, 0.1], [-0.95, -0.45, 0.9], [-0.95, 0.45, 0.9], [-0.95, 0.45, 0.1], [1, 0, 0]), MAT_MIRROR),
        (quad([0.95, -0.45, 0.1], [0.95, -0.45, 0.9], [0.95, 0.45, 0.9], [0.95, 0.45, 0.1], [-1, 0, 0]), MAT_MIRROR),
        (quad([-0.5, -0.9, 0.95], [0.3, -0.9, 0.8], [0.3, -0.2, 0.8], [-0.5, -0.2, 0.95], [0.15, 0.1, -1]), MAT_MIRROR),
        (quad([0.05, -0.7, 0.2], [0.65, -0.7, 0.2], [0.65, 0.1, 0.35], [0.05, 0.1, 0.35], [0, 0, -1]), MAT_NULL),
        (quad([-0.6, 0.35, 0.3], [-0.2, 0.35, 0.3], [-0.2, 0.35, 0.7], [-0.6, 0.35, 0.7], [0, -1, 0]), MAT_DIFFUSE),
    ]
    tris = np.concatenate([p[0] for p in parts])
    mat = np.concatenate([np.full(len(p[0]), p[1], np.uint32) for p in parts])
    return tris, mat


ALB = (0.7, 0.4, 0.25)
SPEC = (0.9, 0.8, 0.95)


def chain_scenes(alvrl, oracle, w, h):
    tris, mat = chain_mesh()
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, material=mat, specular=SPEC)
    o = set_occluders(oracle.scene(w, h), tris, ALB, material=mat, specular=SPEC)
    return s, o, tris, mat


@pytest.mark.parametrize("rr_depth,pass_", [(100, 0), (2, 3)])
def test_chains_match_oracle(alvrl, oracle, rr_depth, pass_):
    """Every pixel's eye chain, host == oracle bit for bit; the chains are
    not vacuous: mirrors continue them (some are >= 4 records long), weights
    fall below 1, and with specularForcedRRdepth 2 the roulette ends some."""
    w, h = 48, 32
    s, o, _, _ = chain_scenes(alvrl, oracle, w, h)
    m = oracle.medium()
    lens = []
    min_w = 1.0
    for y in range(h):
        for x in range(w):
            mine = alvrl.scene_chain(s, x, y, seed=SEED, pass_=pass_, spec_rr_depth=rr_depth)
            ref = oracle.chain(o, m, x, y, seed=SEED, pass_=pass_, spec_rr_depth=rr_depth)
            assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32)), (x, y)
            lens.append(len(mine))
            if len(mine):
                min_w = min(min_w, float(mine[:, 16:19].min()))
                assert np.array_equal(mine[:, 19].view(np.uint32), np.arange(len(mine), dtype=np.uint32))
                # every record but the last is a delta surface
                assert np.all(mine[:-1, 15].view(np.uint32) & REC_DELTA)
    lens = np.asarray(lens)
    assert (lens >= 2).sum() > 50 and lens.max() >= 4, np.bincount(lens)
    assert min_w < 0.8


def test_chain_depth0_is_primary_record(alvrl, oracle):
    """The first record of a chain is the primary record the device forms."""
    w, h = 40, 30
    s, _, _, _ = chain_scenes(alvrl, oracle, w, h)
    prim = alvrl.scene_records(s)
    for p in range(0, w * h, 7):
        c = alvrl.scene_chain(s, p % w, p // w)
        if len(c):
            assert np.array_equal(c[0].view(np.uint32), prim[p].view(np.uint32)), p


def test_chain_roulette_is_unbiased(alvrl, oracle):
    """A chain over several mirrors: with specularForcedRRdepth 1
    every bounce plays roulette with probability <= 0.98 and the survivors'
    weights are divided by it, so the mean weight of depth k over passes is
    the deterministic product transmittance * reflectance (within sampling
    error), while single chains end early."""
    w, h = 48, 32
    s, _, _, _ = chain_scenes(alvrl, oracle, w, h)
    # the pixel with the longest chain without roulette
    best = max(((len(alvrl.scene_chain(s, x, y, spec_rr_depth=1000, init_throughput=1e9)), x, y)
                for y in range(0, h, 2) for x in range(0, w, 2)))
    assert best[0] >= 4
    x, y = best[1], best[2]
    ref = alvrl.scene_chain(s, x, y, spec_rr_depth=1000, init_throughput=1e9)
    k = 3
    acc, ends = np.zeros(3), 0
    n = 3000
    for p in range(n):
        c = alvrl.scene_chain(s, x, y, pass_=p, spec_rr_depth=1)
        if len(c) > k:
            acc += c[k, 16:19]
        else:
            ends += 1
    assert ends > 0
    np.testing.assert_allclose(acc / n, ref[k, 16:19], rtol=0.05)


def test_slice_records_match_oracle(alvrl, oracle):
    """buildSlices' gather point passes null surfaces: host == oracle bit for
    bit, and it differs from the primary record exactly where a null pane is
    the first hit."""
    w, h = 48, 32
    s, o, _, _ = chain_scenes(alvrl, oracle, w, h)
    prim = alvrl.scene_records(s)
    passed = 0
    for p in range(w * h):
        mine = alvrl.scene_slice_record(s, p % w, p // w)
        ref = oracle.slice_record(o, p % w, p // w)
        assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32)), p
        if not np.array_equal(mine[6:12], prim[p, 6:12]):
            passed += 1
            assert prim[p, 15].view(np.uint32) & REC_DELTA
    assert passed > 20


@pytest.mark.parametrize("short", [True, False])
def test_tracer_mirrors_null_match_oracle(alvrl, oracle, short):
    """Particles reflect off the mirrors and pass the null pane (cutting
    their VRLs there): host tracer == oracle bit for bit, and the VRL set
    differs from the all-diffuse scene's."""
    s, o, tris, mat = chain_scenes(alvrl, oracle, 16, 16)
    mine, pc = alvrl.trace_vrls(s, 3000, seed=0x5EED0001, short_vrls=short)
    ref, rpc = oracle.trace(o, oracle.medium(), 3000, seed=0x5EED0001, short_vrls=short)
    assert pc == rpc
    assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
    diffuse = alvrl.scene_set_occluders(alvrl.scene_default(16, 16), tris, ALB)
    plain, _ = alvrl.trace_vrls(diffuse, 3000, seed=0x5EED0001, short_vrls=short)
    assert plain.shape != mine.shape or not np.array_equal(plain, mine)
