"""The default (fast) pipeline against the CPU restatement's OWN pipeline at
the benchmark's config C4 (1024^2, 100k VRLs, Adaptive LightSlice): no device
result is fed to the oracle (bench.py unconditional_parity).

The fast R build rounds differently from the oracle (test_gpu_parity.py's
tolerance), so some of its discrete clustering decisions differ and its cluster
lists are not the oracle's: its frame is a different, equally valid estimate.
The stated bar is therefore the method's own noise: the per-pixel RMSE of the
fast frame against the oracle's frame of the same pass must stay below the RMSE
between the oracle's frames of two consecutive passes.  The oracle's lists
come from the strict device pipeline, pinned here at this scale: on the median
slice the oracle's own R rows equal the strict device's bit for bit and the
oracle's refinement of them gives the same list; the strict device frame meets
the gather tolerance against the oracle's frame.
"""
import numpy as np
import pytest

from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close

pytestmark = pytest.mark.gpu


def test_c4_fast_pipeline_vs_oracle_pipeline(gpu_ok):
    import torch
    import alvrl
    import bench
    cfg = bench.CONFIGS["C4"]
    W, H = cfg["w"], cfg["h"]
    scene = alvrl.scene_default(W, H)
    vrls, pc = alvrl.trace_vrls(scene, cfg["nvrl"], seed=SEED_VRL)
    it = alvrl.Integrator(cfg["props"] + f";seed={SEED_RNG}", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(scene)
    pass_ = 2
    it.prepass(pass_)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    fast_cl = it.clusters()
    r = bench.unconditional_parity(cfg, vrls, pc, pass_, fb.view(-1, 3).cpu().numpy(), row_stride=128,
                                   fast_clusters=fast_cl)
    it.close()
    print({k: v for k, v in r.items()})
    pin = r["oracle_lists_pinned_on_slice"]
    assert pin["R_bit_identical"] and pin["cluster_list_identical"], pin
    f, n, s = r["fast_vs_oracle_pipeline"], r["oracle_pass_to_pass"], r["strict_device_vs_oracle_pipeline"]
    # the strict device frame renders the oracle's lists: the gather tolerance
    assert s["median_rel"] <= 1e-6 and s["q99_rel"] <= 1e-4 and s["max_rel"] <= 5e-2, s
    # the fast pipeline's unconditional error is on the scale of the method's
    # pass-to-pass noise: its R rounds differently, so its discrete clustering
    # decisions differ (measured: in every slice at C4) and its frame is
    # another estimate of the same pass, as far from the oracle's as two of the
    # oracle's own passes are from each other (ratio 0.79-0.94 measured,
    # profiles/r05); bar 1.25
    assert n["rmse"] > 0 and f["rmse"] <= 1.25 * n["rmse"], (f, n)
