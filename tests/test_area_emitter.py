"""Scenes beyond the point-light smoke box: an area
emitter (src/emitters/area.cpp on a triangle mesh) and a medium bounded by a
closed, rotated triangle mesh instead of the axis-aligned box.

The vrlTracer's emission (vrlTracer.h:98-120): Scene::sampleEmitterPosition
(scene.cpp:958-974) -> AreaEmitter::samplePosition (area.cpp:94-98) ->
TriMesh::samplePosition (trimesh.cpp:388-423: a triangle by area through
DiscreteDistribution::sampleReuse, pmf.h:101-169; Triangle::sample,
triangle.cpp:24-59) with power radiance * pi * area (area.cpp:198), then a
cosine-weighted direction (area.cpp:115-123).

CPU part: the host tracer against the oracle, BIT FOR BIT, plus the emission's
closed forms; the GPU tracer and the pipeline are in test_gpu_area_scene.py."""
import numpy as np
import pytest

from oracle import set_area_emitter, set_occluders

RADIANCE = (3.0, 2.5, 2.0)


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


def emitter_tris():
    """A quad under the ceiling facing down (-y) and a smaller triangle facing
    down-left: unequal areas for the area CDF."""
    q = np.array([[-0.3, 0.9, -0.3], [0.3, 0.9, -0.3], [0.3, 0.9, 0.3], [-0.3, 0.9, 0.3]], np.float32)
    tris = [np.concatenate([q[0], q[1], q[2]]), np.concatenate([q[0], q[2], q[3]]),
            np.array([0.5, 0.85, 0.1, 0.7, 0.6, 0.1, 0.5, 0.85, 0.3], np.float32)]
    t = np.asarray(tris, np.float32)
    # face the medium below: flip any triangle whose normal points up
    n = np.cross(t[:, 3:6] - t[:, 0:3], t[:, 6:9] - t[:, 0:3])
    up = n[:, 1] > 0
    t[up] = t[up][:, [0, 1, 2, 6, 7, 8, 3, 4, 5]]
    return t


def container_mesh(alvrl, half=0.95, angle_deg=20.0):
    """A closed cube rotated about y, inward normals: the medium's boundary
    (its diffuse walls face the camera)."""
    b = alvrl.box_mesh([-half] * 3, [half] * 3)
    b = b[:, [0, 1, 2, 6, 7, 8, 3, 4, 5]]                  # reversed winding: inward normals
    a = np.deg2rad(angle_deg)
    R = np.array([[np.cos(a), 0, np.sin(a)], [0, 1, 0], [-np.sin(a), 0, np.cos(a)]], np.float32)
    return (b.reshape(-1, 3, 3) @ R.T).reshape(-1, 9).astype(np.float32)


def area_scene(alvrl, oracle, w, h, container=True):
    tris = [container_mesh(alvrl)] if container else []
    tris.append(alvrl.box_mesh([-0.3, -0.95, 0.1], [0.2, -0.4, 0.5]))
    tris = np.concatenate(tris).astype(np.float32)
    alb = (0.6, 0.5, 0.4)
    s = alvrl.scene_set_occluders(alvrl.scene_default(w, h), tris, alb)
    s = alvrl.scene_set_area_emitter(s, emitter_tris(), RADIANCE)
    o = set_area_emitter(set_occluders(oracle.scene(w, h), tris, alb), emitter_tris(), RADIANCE)
    return s, o, tris


@pytest.mark.parametrize("container", [False, True])
def test_area_tracer_matches_oracle(alvrl, oracle, container):
    s, o, _ = area_scene(alvrl, oracle, 16, 16, container)
    for target, short, rr in ((1200, True, 5), (500, False, 5), (800, True, 1)):
        mine, pc = alvrl.trace_vrls(s, target, seed=0x5EED0001, short_vrls=short, rr_depth=rr)
        ref, rpc = oracle.trace(o, oracle.medium(), target, seed=0x5EED0001, short_vrls=short, rr_depth=rr)
        assert pc == rpc and mine.shape == ref.shape
        assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))


def test_area_emission_closed_forms(alvrl, oracle):
    """First VRLs start on the emitter with power radiance * pi * area, in a
    cosine-weighted direction (E[cos] = 2/3) away from the emitting side,
    and the quad (area 0.36) is picked in proportion to its area."""
    s, o, _ = area_scene(alvrl, oracle, 16, 16, container=False)
    t = emitter_tris()
    area = float(sum(0.5 * np.linalg.norm(np.cross(x[3:6] - x[0:3], x[6:9] - x[0:3])) for x in t))
    power = np.float32(RADIANCE) * np.float32(np.pi) * np.float32(area)
    v, pc = alvrl.trace_vrls(s, 20000, seed=0x5EED0002, short_vrls=True)
    st = v[0:3].T
    first = np.all(np.isclose(v[6:9].T, power, rtol=1e-5), axis=1)    # no throughput yet
    assert first.sum() > 0.2 * pc
    on_quad = np.abs(st[first, 1] - 0.9) < 1e-6
    frac_quad = on_quad.mean()
    assert abs(frac_quad - 0.36 / area) < 0.02, (frac_quad, 0.36 / area)
    d = v[3:6].T[first] - st[first]
    d /= np.linalg.norm(d, axis=1)[:, None]
    cosq = -d[on_quad, 1]                                                # the quad emits along -y
    assert (cosq > 0).all()
    assert abs(cosq.mean() - 2.0 / 3.0) < 0.02, cosq.mean()


def test_area_emitter_validation(alvrl):
    s = alvrl.scene_set_area_emitter(alvrl.scene_default(8, 8), np.zeros((1, 9), np.float32), RADIANCE)
    with pytest.raises(alvrl.AlvrlError):                               # zero area
        alvrl.trace_vrls(s, 10)
    bad = emitter_tris().copy()
    bad[0, 0] = np.nan
    s = alvrl.scene_set_area_emitter(alvrl.scene_default(8, 8), bad, RADIANCE)
    with pytest.raises(alvrl.AlvrlError):
        alvrl.trace_vrls(s, 10)
