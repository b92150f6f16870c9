"""Scenes with occluders inside the smoke box (general
visibility instead of the convex container).  Occluders are triangles with a
one-sided diffuse BSDF: eye rays and particles hit them (TriangleT::rayIntersect,
include/mitsuba/core/triangle.h:109-145; hit record skdtree.h:350-396) and they
block the gather's U-V and surface-V connections (Scene::evalTransmittance,
src/librender/scene.cpp:619-679).

CPU part: the product's host harness (records, the VRL tracer, LightSlice
slicing) against the oracle, BIT FOR BIT.  The GPU part (BVH traversal in
the tracer, the eye-record kernel and the gathers) is in test_gpu_occluders.py."""
import numpy as np
import pytest

from oracle import set_occluders


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


def occluder_mesh(alvrl):
    """A box standing on the floor under the light, a thin tilted plate and
    a triangle facing away from the camera (back faces are hit, and their
    one-sided BSDF is black)."""
    tris = [alvrl.box_mesh([-0.35, -1.0, 0.05], [0.15, -0.2, 0.55]),
            alvrl.box_mesh([0.2, 0.1, -0.3], [0.7, 0.14, 0.2])]
    t = np.array([[-0.8, 0.3, 0.6, -0.2, 0.3, 0.6, -0.5, 0.7, 0.6]], np.float32)
    tris.append(t[:, [0, 1, 2, 6, 7, 8, 3, 4, 5]])   # reversed winding: normal +z
    return np.concatenate(tris).astype(np.float32)


ALB = (0.7, 0.4, 0.25)


def scenes(alvrl, oracle, w, h):
    tris = occluder_mesh(alvrl)
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, ALB)
    o = set_occluders(oracle.scene(w, h), tris, ALB)
    return s, o, tris


def test_occluder_records_match_oracle(alvrl, oracle):
    s, o, tris = scenes(alvrl, oracle, 96, 64)
    mine = alvrl.scene_records(s)
    ref = oracle.records(o)
    assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
    # the occluders are visible: some records carry their albedo and a
    # non-axis normal, and the scene without them differs exactly there
    occ_hit = np.all(mine[:, 12:15] == np.float32(ALB), axis=1)
    assert 200 < occ_hit.sum() < len(mine) - 200
    plain = alvrl.scene_records(alvrl.scene_default(96, 64))
    same = np.all(plain == mine, axis=1)
    assert not same[occ_hit].any()


def test_occluder_tracer_matches_oracle(alvrl, oracle):
    s, o, tris = scenes(alvrl, oracle, 16, 16)
    for target, short in ((900, True), (400, False)):
        mine, pc = alvrl.trace_vrls(s, target, seed=0x5EED0001, short_vrls=short)
        ref, rpc = oracle.trace(o, oracle.medium(), target, seed=0x5EED0001, short_vrls=short)
        assert pc == rpc
        assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
        # particles end on / start from the occluders: some VRL endpoints lie
        # on their faces (inside the occluder boxes' closed bounds)
        ends = mine[3:6].T
        on_box = np.all((ends >= np.array([-0.35, -1.0, 0.05]) - 1e-5) &
                        (ends <= np.array([0.15, -0.2, 0.55]) + 1e-5), axis=1)
        assert on_box.sum() > 0
        plain, _ = alvrl.trace_vrls(alvrl.scene_default(16, 16), target, seed=0x5EED0001, short_vrls=short)
        assert plain.shape != mine.shape or not np.array_equal(plain, mine)


def per_triangle_albedos(n):
    """Each occluder its own reflectance: the first box black (an emitter's
    all-absorbing mesh, shape.cpp:49-56), the plate and the last triangle
    coloured."""
    alb = np.zeros((n, 3), np.float32)
    alb[12:24] = (0.2, 0.6, 0.3)
    alb[24:] = (0.9, 0.1, 0.5)
    return alb


def test_occluder_albedos_match_oracle(alvrl, oracle):
    """alvrl_scene_desc.occluder_albedos (per-triangle reflectances): the
    records and the tracer equal the oracle's bit for bit, a black occluder
    ends the particles that reach it, and the records carry each triangle's
    own reflectance."""
    tris = occluder_mesh(alvrl)
    alb = per_triangle_albedos(len(tris))
    s = alvrl.scene_set_occluders(alvrl.scene_default(96, 64), tris, ALB, albedos=alb)
    o = set_occluders(oracle.scene(96, 64), tris, ALB, albedos=alb)
    mine = alvrl.scene_records(s)
    ref = oracle.records(o)
    assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
    for a in (alb[0], alb[12], alb[24]):
        assert np.all(mine[:, 12:15] == a, axis=1).sum() > 50
    s16 = alvrl.scene_set_occluders(alvrl.scene_default(16, 16), tris, ALB, albedos=alb)
    o16 = set_occluders(oracle.scene(16, 16), tris, ALB, albedos=alb)
    v, pc = alvrl.trace_vrls(s16, 900, seed=0x5EED0001)
    rv, rpc = oracle.trace(o16, oracle.medium(), 900, seed=0x5EED0001)
    assert pc == rpc and np.array_equal(v.view(np.uint32), rv.view(np.uint32))
    shared, _ = alvrl.trace_vrls(alvrl.scene_set_occluders(alvrl.scene_default(16, 16), tris, ALB), 900,
                                 seed=0x5EED0001)
    assert shared.shape != v.shape or not np.array_equal(shared, v)
