"""BASELINE.json configs[4] (C5: 2048^2, 1M VRLs, adaptive LightSlice, 8 GPUs)
as rank 0's share on one GPU: the slice-sharded prepass
(alvrl_integrator_prepass_dist) with the seven other ranks stood in for by an
in-process exchange (tests/c5_share.py).  This rank builds its 1/8 of R (~61 GB)
and refines slices s % 8 == 0 -- local matrices of ~210-850 rows, so the
>256-row variance engine on 1M-column clusters.

The oracle's Clustering (Preprocessor.cpp:254-283: ctor, refineAdaptively,
sampleRepresentatives; strict build, speculative worker threads that do not
change a bit, oracle/alvrl_preproc.c) on the device's own job for the smallest
local slice and for the smallest one of more than 256 rows (refineSlice's
inputs through alvrl_integrator_slice_job) must give the device's
representatives and weights bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_c5_rank0_share(oracle, gpu_ok):
    import c5_share
    it, info, mine = c5_share.run_share()
    try:
        assert info["slices_local"] == len(mine) and info["slices_failed"] == 0
        off, _ = it.reps()
        rows = np.diff(off)
        # no neighbours: exactly this rank's slices' rows are built, each pair once
        assert info["rows_built"] == int(rows[mine].sum())
        assert info["contrib_preprocess"] == info["rows_built"] * info["vrls"]
        assert info["vrls"] >= 1_000_000
        cl = it.clusters()
        # the smallest slice (one row group of <= 256 rows) and the smallest of more than
        # 256 rows (the v3 engine over row groups, its sums carried from group to group)
        big = [s for s in mine if rows[s] > 256]
        picks = [mine[int(np.argmin(rows[mine]))]] + ([min(big, key=lambda s: rows[s])] if big else [])
        for s in picks:
            job = it.slice_job(s)
            n = job["R"].shape[1]
            reps, w, refined = oracle.cluster_refine(job["R"], np.arange(n, dtype=np.uint32), job["locw"],
                                                     job["init_vrls"], job["init_off"], job["pixel_undersampling"],
                                                     -1.0, seed=c5_share.SEED_RNG, pass_=0, stage_refine=3 + 2 * s,
                                                     stage_sample=4 + 2 * s)
            b, e = cl["slice_off"][s], cl["slice_off"][s + 1]
            print(f"C5 slice {s}: {n} rows x {job['R'].shape[0]} VRLs, {len(reps)} clusters (device {e - b}); "
                  f"share refine {info['ms_refine_kernel']:.0f} ms, R build {info['ms_rbuild']:.0f} ms")
            assert refined
            assert np.array_equal(reps, cl["reps"][b:e])
            assert np.array_equal(w.view(np.uint32), cl["weights"][b:e].view(np.uint32))
    finally:
        it.close()
