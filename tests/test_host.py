"""Product host side (libalvrl.so host harness, no GPU needed) against the
oracle: scene records, the VRL tracer, VRL file round trip, LightSlice slicing
and representative sampling must agree BIT FOR BIT (same float operations,
same counter-RNG streams; the product uses std::push_heap/pop_heap where the
oracle restates libstdc++'s heap in C)."""
import os
import tempfile

import numpy as np
import pytest


@pytest.fixture(scope="module")
def alvrl():
    import alvrl as a
    return a


def test_records_match_oracle(alvrl, oracle):
    s = alvrl.scene_default(96, 64)
    mine = alvrl.scene_records(s)
    ref = oracle.records(oracle.scene(96, 64))
    assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))
    ids = np.array([0, 5, 96 * 64 - 1, 1234], np.uint32)
    sub = alvrl.scene_records(s, pixel_ids=ids)
    assert np.array_equal(sub.view(np.uint32), ref[ids].view(np.uint32))


def test_tracer_matches_oracle(alvrl, oracle):
    s = alvrl.scene_default(16, 16)
    for target, short in ((700, True), (300, False)):
        mine, pc = alvrl.trace_vrls(s, target, seed=0x5EED0001, short_vrls=short)
        ref, rpc = oracle.trace(oracle.scene(16, 16), oracle.medium(), target, seed=0x5EED0001,
                                short_vrls=short)
        assert pc == rpc
        assert np.array_equal(mine.view(np.uint32), ref.view(np.uint32))


def test_vrl_file_roundtrip(alvrl):
    s = alvrl.scene_default(8, 8)
    v, pc = alvrl.trace_vrls(s, 200)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "vrls.txt")
        alvrl.write_vrl_file(p, v)
        v2, pc2 = alvrl.read_vrl_file(p)
        assert pc2 == v.shape[1]   # particleCount = #lines read (VRL.h:127)
        assert np.array_equal(v2, v)
        with open(p, "a") as f:    # zero-length / zero-power lines are filtered (VRL.h:148-158)
            f.write("0 0 0 0 0 0 1 1 1\n0.1 0.1 0.1 0.2 0.2 0.2 0 0 0\n")
        v3, pc3 = alvrl.read_vrl_file(p)
        assert v3.shape[1] == v.shape[1] and pc3 == pc2
        with open(p, "a") as f:
            f.write("0 0 0 1 1 1 -1 1 1\n")
        with pytest.raises(alvrl.AlvrlError):
            alvrl.read_vrl_file(p)


def test_golden_vrl_file_reader(alvrl):
    """The host reader of the reference ASCII format (VRL.h:43-54, :105-158)
    returns the committed fixture's VRLs exactly, particleCount = #VRLs."""
    path = os.path.join(os.path.dirname(__file__), "golden", "vrls_c1.txt")
    rows = np.array([list(map(float, l.split())) for l in open(path) if l.strip()], np.float32).T
    soa, pc = alvrl.read_vrl_file(path)
    assert pc == rows.shape[1] == soa.shape[1]
    assert np.array_equal(soa.view(np.uint32), np.ascontiguousarray(rows).view(np.uint32))


def test_integrator_properties_validation(alvrl):
    with pytest.raises(alvrl.AlvrlError, match="neighbourCount"):
        alvrl.Integrator("nc=3")
    with pytest.raises(alvrl.AlvrlError, match="volVolSamples"):
        alvrl.Integrator("volVolSamples=1")
    with pytest.raises(alvrl.AlvrlError, match="unknown"):
        alvrl.Integrator("noSuchParameter=1")
