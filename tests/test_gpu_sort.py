"""The split sort's radix path (refine.hip radix8_sort) against
the bucket + bitonic path: every cluster list of a C4-sized prepass (1024^2,
100k VRLs, 100 slices of 60-214 rows, clusters up to 100k columns) and of the
C3 configuration, bit for bit with ALVRL_SORT_RADIX_MIN = 0 (never radix), 2
(radix for every split that reaches split()'s sort) and the default (radix
from 16,385 columns).  The keys are unique, so every correct sort gives the
same order; the oracle comparisons of the default lists are
test_gpu_pipeline.py's (test_refine_c4_scale) and test_gpu_parity.py's."""
import os

import numpy as np
import pytest

from test_gpu_parity import SEED_RNG, SEED_VRL

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("props", ["targetNumSlices=100;localUndersampling=-1",
                                   "targetNumSlices=100;localUndersampling=100"])
def test_radix_sort_matches_bitonic(gpu_ok, props):
    import alvrl
    scene = alvrl.scene_default(1024, 1024)
    vrls, pc = alvrl.trace_vrls(scene, 100000, seed=SEED_VRL)
    saved = os.environ.get("ALVRL_SORT_RADIX_MIN")
    lists = {}
    try:
        it = alvrl.Integrator(f"{props};seed={SEED_RNG}", device=0)
        try:
            it.set_vrls(vrls, pc)
            it.preprocess(scene)
            for mode in ("0", "2", None):
                if mode is None:
                    os.environ.pop("ALVRL_SORT_RADIX_MIN", None)
                else:
                    os.environ["ALVRL_SORT_RADIX_MIN"] = mode
                it.prepass(3)
                lists[mode] = it.clusters()
        finally:
            it.close()
    finally:
        if saved is None:
            os.environ.pop("ALVRL_SORT_RADIX_MIN", None)
        else:
            os.environ["ALVRL_SORT_RADIX_MIN"] = saved
    ref = lists["0"]
    assert ref["reps"].size > 100 * 100
    for mode in ("2", None):
        for k in ref:
            assert np.array_equal(ref[k].view(np.uint32), lists[mode][k].view(np.uint32)), (mode, k)
