"""The Mitsuba plugin's own C++ (mitsuba_plugin/vrlAmdIntegrator.cpp) executed.

It is linked with a mock implementation of the Mitsuba classes it uses
(tests/mitsuba_mock/: include/mitsuba/mock.h, src/mock_impl.cpp -> the shared
library libvrl_plugin_mock.so, built in-tree by __graft_entry__.build()) and
driven as Mitsuba's progressive render drives an integrator
(src/librender/integrator.cpp, renderproc.cpp): CreateInstance(props),
preprocess, then per pass prepass and renderBlock over 32x32 blocks, in frame
mode on the smoke box of alvrl_scene_default.

  * one device: the plugin's frame equals the library integrator's own frame
    (alvrl.Integrator on the same scene and properties) bit for bit;
  * amdDevices=0,0 (amdRehearseDevices=true: two library integrators on one
    GPU, the slice-sharded prepass through the in-process exchange, each
    rendering its 64x64 tiles, the frames summed): the same frame;
  * a remote worker (the master's serialize, the unserialization
    constructor, wakeup with the published "vrls" / "vrlClusterInfo"
    resources, vrlIntegrator.cpp:210-235, 353-384): the same frame.
"""
import ctypes as C
import os

import numpy as np
import pytest

from test_gpu_parity import SEED_RNG

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
MOCK = os.path.join(HERE, "mitsuba_mock", "libvrl_plugin_mock.so")
INV_PI = np.float32(0.31830988618379067154)


def _plugin():
    assert os.path.exists(MOCK), "build the mock plugin first (__graft_entry__.build / make -C tests/mitsuba_mock)"
    L = C.CDLL(MOCK)
    L.mock_run_frame.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
    L.mock_run_frame.restype = C.c_int
    L.mock_last_error.restype = C.c_char_p
    return L


def _run(L, props, w, h, passes, remote=0):
    out = np.zeros((h * w, 3), np.float32)
    rc = L.mock_run_frame(props.encode(), w, h, passes, remote, out.ctypes.data)
    assert rc == 0, L.mock_last_error().decode()
    return out


def _library_frame(props, w, h, passes):
    import torch
    import alvrl
    s = alvrl.scene_default(w, h)
    # the point light as the plugin describes it: samplePosition's power
    # (intensity * 4 pi, point.cpp:81-91) times 1 / (4 pi) in float
    for i in range(3):
        p = np.float32(np.float32(s.light_intensity[i]) * np.float32(4.0 * np.pi))
        s.light_intensity[i] = float(np.float32(p * np.float32(np.float32(0.25) * INV_PI)))
    it = alvrl.Integrator(props + ";sampleCount=1", device=0)
    it.preprocess(s)
    for p in range(passes):
        it.prepass(p)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    it.close()
    return fb.view(-1, 3).cpu().numpy()


@pytest.mark.parametrize("props", ["targetNumSlices=16;vrlTargetNum=3000",
                                   "targetNumSlices=12;vrlTargetNum=2000;neighbourCount=2"])
def test_plugin_frame_mode_runs(gpu_ok, props):
    L = _plugin()
    w, h, passes = 160, 96, 2
    props = props + f";seed={SEED_RNG}"
    ref = _library_frame(props, w, h, passes)
    assert ref.any()
    one = _run(L, props, w, h, passes)
    assert np.array_equal(one.view(np.uint32), ref.view(np.uint32)), "plugin (one device) vs library"
    two = _run(L, props + ";amdDevices=0,0;amdRehearseDevices=true", w, h, passes)
    assert np.array_equal(two.view(np.uint32), ref.view(np.uint32)), "plugin amdDevices=0,0 vs library"
    rem = _run(L, props, w, h, passes, remote=1)
    assert np.array_equal(rem.view(np.uint32), ref.view(np.uint32)), "plugin remote worker vs library"


def test_plugin_refuses_repeated_device_without_rehearsal(gpu_ok):
    L = _plugin()
    out = np.zeros((32 * 32, 3), np.float32)
    rc = L.mock_run_frame(b"amdDevices=0,0", 32, 32, 1, 0, out.ctypes.data)
    assert rc != 0 and b"distinct" in L.mock_last_error()
