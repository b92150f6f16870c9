"""Two large-cluster paths of split() against the ones they replace, on every
cluster list of a C4-sized prepass and of the C3 configuration, bit for bit:
the split sort's radix path (refine.hip radix8_sort) against
the bucket + bitonic path, and the weighted picks on every wave
(weighted_sample_wg) against the one-wave scan.

The sort: every cluster list of a C4-sized prepass (1024^2,
100k VRLs, 100 slices of 60-214 rows, clusters up to 100k columns) and of the
C3 configuration, bit for bit with ALVRL_SORT_RADIX_MIN = 0 (never radix), 2
(radix for every split that reaches split()'s sort) and the default (radix
from 1,024 columns).  The keys are unique, so every correct sort gives the
same order; the oracle comparisons of the default lists are
test_gpu_pipeline.py's (test_refine_c4_scale) and test_gpu_parity.py's."""
import os

import numpy as np
import pytest

from test_gpu_parity import SEED_RNG, SEED_VRL

pytestmark = pytest.mark.gpu


def _lists_by_setting(props, key):
    import alvrl
    scene = alvrl.scene_default(1024, 1024)
    vrls, pc = alvrl.trace_vrls(scene, 100000, seed=SEED_VRL)
    saved = os.environ.get(key)
    lists = {}
    try:
        it = alvrl.Integrator(f"{props};seed={SEED_RNG}", device=0)
        try:
            it.set_vrls(vrls, pc)
            it.preprocess(scene)
            for mode in ("0", "2", None):
                if mode is None:
                    os.environ.pop(key, None)
                else:
                    os.environ[key] = mode
                it.prepass(3)
                lists[mode] = it.clusters()
        finally:
            it.close()
    finally:
        if saved is None:
            os.environ.pop(key, None)
        else:
            os.environ[key] = saved
    return lists


PROPS = ["targetNumSlices=100;localUndersampling=-1", "targetNumSlices=100;localUndersampling=100"]


@pytest.mark.parametrize("props", PROPS)
def test_radix_sort_matches_bitonic(gpu_ok, props):
    lists = _lists_by_setting(props, "ALVRL_SORT_RADIX_MIN")
    ref = lists["0"]
    assert ref["reps"].size > 100 * 100
    for mode in ("2", None):
        for k in ref:
            assert np.array_equal(ref[k].view(np.uint32), lists[mode][k].view(np.uint32)), (mode, k)


@pytest.mark.parametrize("props", PROPS)
def test_weighted_pick_wg_matches_wave(gpu_ok, props):
    """ALVRL_WS_WG_MIN = 0 (the one-wave scan), 2 (every split that reaches
    split()'s picks) and the default (from 4,096 columns)."""
    lists = _lists_by_setting(props, "ALVRL_WS_WG_MIN")
    ref = lists["0"]
    assert ref["reps"].size > 100 * 100
    for mode in ("2", None):
        for k in ref:
            assert np.array_equal(ref[k].view(np.uint32), lists[mode][k].view(np.uint32)), (mode, k)
