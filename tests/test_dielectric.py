"""Smooth dielectric occluders (dielectric.cpp: m_eta = intIOR / extIOR,
specular reflectance and transmittance 1) inside the smoke box.

LiInternal (vrlIntegrator.cpp:464-511) follows EVERY delta component of a
hit's BSDF (bRec.component = i): at a dielectric the eye path branches into
the reflected (weight F) and the refracted direction (weight (1 - F) / eta^2
in radiance mode), each with its own throughput, roulette and recursion, so a
pixel's records form a tree.  The VRL tracer samples one component, reflection
with probability F (dielectric.cpp:335-364, importance mode), and its Russian
roulette scales by the accumulated eta^2 (vrlTracer.h:203-222).

CPU part: the product's host harness (eye-path trees, slicing records, the
VRL tracer) against the oracle, BIT FOR BIT; the device side over such scenes
is test_gpu_dielectric.py."""
import numpy as np
import pytest

from oracle import MAT_DIELECTRIC, MAT_DIFFUSE, MAT_MIRROR, set_occluders
from test_chains import ALB, SPEC, quad

REC_DELTA, REC_SMOOTH = 8, 2
SEED = 0xA1B2C3D4
ETA = 1.5


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


def glass_mesh():
    """A glass pane across the view, a closed glass block (rays enter, reflect
    totally inside, leave), a mirror behind them and a diffuse plate."""
    import alvrl
    block = alvrl.box_mesh([0.2, -0.6, 0.35], [0.6, -0.1, 0.65])
    parts = [
        (quad([-0.8, -0.2, 0.25], [-0.1, -0.2, 0.25], [-0.1, 0.6, 0.45], [-0.8, 0.6, 0.45], [0.1, 0, -1]), MAT_DIELECTRIC),
        (block, MAT_DIELECTRIC),
        (quad([-0.6, -0.9, 0.95], [0.6, -0.9, 0.9], [0.6, 0.5, 0.9], [-0.6, 0.5, 0.95], [0, 0.05, -1]), MAT_MIRROR),
        (quad([-0.3, 0.5, 0.6], [0.3, 0.5, 0.6], [0.3, 0.5, 0.9], [-0.3, 0.5, 0.9], [0, -1, 0]), MAT_DIFFUSE),
    ]
    tris = np.concatenate([p[0] for p in parts]).astype(np.float32)
    mat = np.concatenate([np.full(len(p[0]), p[1], np.uint32) for p in parts])
    return tris, mat


def glass_scenes(alvrl, oracle, w, h, eta=ETA):
    tris, mat = glass_mesh()
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, material=mat, specular=SPEC, eta=eta)
    o = set_occluders(oracle.scene(w, h), tris, ALB, material=mat, specular=SPEC, eta=eta)
    return s, o, tris, mat


def _branches(chain):
    """Records whose predecessor in pre-order is not their parent: a record
    that follows a diffuse (terminal) record starts a sibling branch."""
    flags = chain[:, 15].view(np.uint32)
    return int(np.sum((flags[:-1] & REC_SMOOTH) != 0))


@pytest.mark.parametrize("rr_depth,pass_,eta", [(100, 0, ETA), (2, 3, ETA), (100, 1, 1.3333)])
def test_dielectric_trees_match_oracle(alvrl, oracle, rr_depth, pass_, eta):
    """Every pixel's eye-path tree, host == oracle bit for bit.  The trees are
    not chains: many pixels branch at the glass (two children of one
    dielectric record), the reflected branch carries weight F < 0.2 at these
    angles while the refracted one carries most of the rest, and depth words
    are the pre-order record index."""
    w, h = 48, 32
    s, o, _, _ = glass_scenes(alvrl, oracle, w, h, eta)
    m = oracle.medium()
    branched = 0
    lens = []
    for y in range(h):
        for x in range(w):
            mine = alvrl.scene_chain(s, x, y, seed=SEED, pass_=pass_, spec_rr_depth=rr_depth)
            ref = oracle.chain(o, m, x, y, seed=SEED, pass_=pass_, spec_rr_depth=rr_depth)
            assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32)), (x, y)
            lens.append(len(mine))
            if len(mine):
                assert np.array_equal(mine[:, 19].view(np.uint32), np.arange(len(mine), dtype=np.uint32))
                branched += _branches(mine) > 0
    lens = np.asarray(lens)
    assert branched > 100, branched
    assert lens.max() >= 5


def test_dielectric_branch_weights(alvrl):
    """The two children of a pane hit at normal-ish incidence: reflection
    weight F = Fresnel reflectance, refraction weight (1 - F) / eta^2 (entering
    glass, radiance scaling, dielectric.cpp:376-385) times the segment's
    transmittance; both with rrProb 1 (initial throughput 1e6, no roulette)."""
    w, h = 48, 32
    tris = quad([-1, -1, 0.0], [1, -1, 0.0], [1, 1, 0.0], [-1, 1, 0.0], [0, 0, -1])
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB, material=[MAT_DIELECTRIC] * 2, eta=ETA)
    c = alvrl.scene_chain(s, w // 2, h // 2, seed=SEED, init_throughput=1e6)
    assert len(c) == 3                                             # pane, back wall, far wall
    t = np.linalg.norm(c[0, 6:9] - c[0, 0:3])
    sigma_t = np.array([0.85, 0.65, 0.45])
    tr = np.exp(-sigma_t * t)
    d = c[0, 3:6] / np.linalg.norm(c[0, 3:6])
    ci = abs(d[2])
    ct = np.sqrt(1 - (1 - ci * ci) / ETA ** 2)
    rs = (ci - ETA * ct) / (ci + ETA * ct)
    rp = (ETA * ci - ct) / (ETA * ci + ct)
    F = 0.5 * (rs * rs + rp * rp)
    refl, refr = c[1], c[[i for i in range(2, len(c)) if c[i, 5] > 0][0]]
    assert refl[5] < 0 < refr[5]                                   # back towards the camera / onwards
    np.testing.assert_allclose(refl[16:19], tr * F, rtol=2e-5)
    np.testing.assert_allclose(refr[16:19], tr * (1 - F) / ETA ** 2, rtol=2e-5)


def test_dielectric_slice_records(alvrl, oracle):
    """buildSlices stops at a dielectric (not a null surface): host == oracle
    bit for bit, equal to the primary record's hit."""
    w, h = 48, 32
    s, o, _, _ = glass_scenes(alvrl, oracle, w, h)
    prim = alvrl.scene_records(s)
    for p in range(0, w * h, 3):
        mine = alvrl.scene_slice_record(s, p % w, p // w)
        ref = oracle.slice_record(o, p % w, p // w)
        assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32)), p
        assert np.array_equal(mine[6:12], prim[p, 6:12])


@pytest.mark.parametrize("short", [True, False])
def test_tracer_dielectric_matches_oracle(alvrl, oracle, short):
    """Particles reflect off or refract through the glass (cutting their VRLs
    there; eta enters the roulette): host tracer == oracle bit for bit, and
    the VRL set differs from the all-diffuse scene's."""
    s, o, tris, mat = glass_scenes(alvrl, oracle, 16, 16)
    mine, pc = alvrl.trace_vrls(s, 4000, seed=0x5EED0001, short_vrls=short, rr_depth=2)
    ref, rpc = oracle.trace(o, oracle.medium(), 4000, seed=0x5EED0001, short_vrls=short, rr_depth=2)
    assert pc == rpc
    assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
    diffuse = alvrl.scene_set_occluders(alvrl.scene_default(16, 16), tris, ALB)
    plain, _ = alvrl.trace_vrls(diffuse, 4000, seed=0x5EED0001, short_vrls=short, rr_depth=2)
    assert plain.shape != mine.shape or not np.array_equal(plain, mine)

