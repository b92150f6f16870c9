"""The fused small split (refine.hip split_fused) against
split(): every cluster list of a C4-sized prepass (1024^2, 100k VRLs, 100
slices of 60-214 rows, so both the float2 and the means-only staging run) and
of the C3 configuration, bit for bit with ALVRL_SPLIT_FUSED = 0 (split() with
variance_split_small), 1 (float2 staging only) and 2 (the default).  The
oracle comparisons of the same lists are test_gpu_pipeline.py's
(test_refine_c4_scale) and test_gpu_parity.py's."""
import os

import numpy as np
import pytest

from test_gpu_parity import SEED_RNG, SEED_VRL

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("props", ["targetNumSlices=100;localUndersampling=-1",
                                   "targetNumSlices=100;localUndersampling=100"])
def test_fused_split_matches_split(gpu_ok, props):
    import alvrl
    scene = alvrl.scene_default(1024, 1024)
    vrls, pc = alvrl.trace_vrls(scene, 100000, seed=SEED_VRL)
    saved = os.environ.get("ALVRL_SPLIT_FUSED")
    lists = {}
    try:
        it = alvrl.Integrator(f"{props};seed={SEED_RNG}", device=0)
        try:
            it.set_vrls(vrls, pc)
            it.preprocess(scene)
            for mode in ("0", "1", "2"):
                os.environ["ALVRL_SPLIT_FUSED"] = mode
                it.prepass(3)
                lists[mode] = it.clusters()
        finally:
            it.close()
    finally:
        if saved is None:
            os.environ.pop("ALVRL_SPLIT_FUSED", None)
        else:
            os.environ["ALVRL_SPLIT_FUSED"] = saved
    ref = lists["0"]
    assert ref["reps"].size > 100 * 100
    for mode in ("1", "2"):
        for k in ref:
            assert np.array_equal(ref[k].view(np.uint32), lists[mode][k].view(np.uint32)), (mode, k)
