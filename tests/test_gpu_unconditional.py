"""The default pipeline (strict R build) against the CPU restatement's OWN
pipeline at the benchmark's config C4 (1024^2, 100k VRLs, Adaptive
LightSlice): no device result is fed to the oracle (bench.py
unconditional_parity).

The oracle re-derives three slices -- the median-size, the largest and the one
with the most clusters -- from scratch: its own R rows of their representatives
must equal the device's bit for bit, and its refinement of them the device's
cluster list; then it renders every 128th image row with the device's lists
(its own, by that identity), and the device frame must meet the gather
tolerance of test_gpu_parity.py.  The fast R build (strictRbuild=false) is run
beside it for the record: its R rounds differently, so some discrete
clustering decisions differ and its frame is another estimate of the pass,
held to the method's own noise (the RMSE between the oracle's frames of two
consecutive passes).
"""
import numpy as np
import pytest

from test_gpu_parity import SEED_RNG, SEED_VRL, _assert_close

pytestmark = pytest.mark.gpu


def test_c4_default_pipeline_vs_oracle_pipeline(gpu_ok):
    import torch
    import alvrl
    import bench
    cfg = bench.CONFIGS["C4"]
    W, H = cfg["w"], cfg["h"]
    scene = alvrl.scene_default(W, H)
    vrls, pc = alvrl.trace_vrls(scene, cfg["nvrl"], seed=SEED_VRL)
    it = alvrl.Integrator(cfg["props"] + f";seed={SEED_RNG}", device=0)   # the default: strict R build
    it.set_vrls(vrls, pc)
    it.preprocess(scene)
    pass_ = 2
    it.prepass(pass_)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    r = bench.unconditional_parity(cfg, vrls, pc, pass_, fb.view(-1, 3).cpu().numpy(), it, row_stride=128)
    it.close()
    print({k: v for k, v in r.items()})
    pins = r["oracle_pipeline_pinned_on_slices"]
    assert len(pins) == 3 and len({p["slice"] for p in pins}) >= 2, pins
    for p in pins:
        assert p["R_bit_identical"] and p["cluster_list_identical"], p
    d, n = r["default_vs_oracle_pipeline"], r["oracle_pass_to_pass"]
    # the default frame renders the oracle's own lists: the gather tolerance
    assert d["median_rel"] <= 1e-6 and d["q99_rel"] <= 1e-4 and d["max_rel"] <= 5e-2, d
    # the fast R build, for the record: another estimate of the same pass, as
    # far from the oracle's as two of the oracle's own passes are from each
    # other (ratio 0.79-0.94 measured in round 5); bar 1.25
    f = r["fast_rbuild_reference"]["vs_oracle_pipeline"]
    assert n["rmse"] > 0 and f["rmse"] <= 1.25 * n["rmse"], (f, n)
