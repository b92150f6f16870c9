"""BASELINE.json configs[4] (C5: 2048^2, 1M VRLs, adaptive LightSlice, 8 GPUs)
end to end on one GPU: the eight ranks' slice-sharded prepasses
(alvrl_integrator_prepass_dist) run one after the other with the true OR of
the eight non-zero masks, their cluster lists are merged into one
vrlClusterInfo, and the 2048^2 frame is rendered as the eight ranks' 64x64
tiles plus the framebuffer sum (tests/c5_share.py, phases 1-3).

Checks against the oracle (oracle/alvrl_preproc.c, alvrl_oracle.c):
  * refinement (Preprocessor.cpp:254-283: Clustering ctor, refineAdaptively,
    sampleRepresentatives) of rank 0's smallest slice and of the smallest
    slice of more than 256 rows of the first rank that holds one (the v3
    engine over row groups; slices go to ranks by their cost, the
    integrator's default sliceSharding) on the
    device's own jobs (alvrl_integrator_slice_job): representatives and
    weights bit for bit;
  * the frame: every 64th image row against the oracle's clustered gather
    (getClusteredVrlContributions, vrlIntegrator.cpp:542-599) with the merged
    lists, on test_gpu_parity's tolerance; the tile-sharded sum equals one
    world-1 render bit for bit.
Per-rank refinement and R-build times are printed (and written to
$ALVRL_C5_REPORT as JSON when set)."""
import json
import os
import time

import numpy as np
import pytest

from test_gpu_parity import _assert_close

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_c5_end_to_end(oracle, gpu_ok, tmp_path):
    import torch
    import alvrl
    import c5_share
    W, H, world = c5_share.C5_W, c5_share.C5_H, c5_share.C5_WORLD
    checked = []
    checked_big = []

    def check(rank, it, info, mine):
        assert info["slices_local"] == len(mine) and info["slices_failed"] == 0
        assert info["exchange_calls"] == ["or", "counts", "data"]
        off, _ = it.reps()
        rows = np.diff(off)
        # no neighbours: exactly this rank's slices' rows are built, each pair once
        assert info["rows_built"] == int(rows[mine].sum())
        assert info["contrib_preprocess"] == info["rows_built"] * info["vrls"]
        assert info["vrls"] >= 1_000_000
        picks = []
        if rank == 0:
            picks.append(mine[int(np.argmin(rows[mine]))])
        big = [s for s in mine if rows[s] > 256]
        if big and not checked_big:           # the first rank holding a slice of > 256 rows (row groups)
            picks.append(min(big, key=lambda s: rows[s]))
            checked_big.append(rank)
        if not picks:
            return
        cl = it.clusters()
        for s in picks:
            t0 = time.time()
            job = it.slice_job(s)
            n = job["R"].shape[1]
            reps, w, refined = oracle.cluster_refine(job["R"], np.arange(n, dtype=np.uint32), job["locw"],
                                                     job["init_vrls"], job["init_off"], job["pixel_undersampling"],
                                                     -1.0, seed=c5_share.SEED_RNG, pass_=0, stage_refine=3 + 2 * s,
                                                     stage_sample=4 + 2 * s)
            b, e = cl["slice_off"][s], cl["slice_off"][s + 1]
            print(f"C5 rank {rank} slice {s}: {n} rows x {job['R'].shape[0]} VRLs, {len(reps)} clusters "
                  f"(device {e - b}), oracle {time.time() - t0:.1f} s")
            assert refined
            assert np.array_equal(reps, cl["reps"][b:e]), (rank, s)
            assert np.array_equal(w.view(np.uint32), cl["weights"][b:e].view(np.uint32)), (rank, s)
            checked.append(dict(rank=rank, slice=int(s), rows=int(n), clusters=int(len(reps))))
            del job

    it, info = c5_share.run_full(check=check, workdir=str(tmp_path))
    try:
        assert checked[0]["rank"] == 0 and len(checked) >= 2 and any(c["rows"] > 256 for c in checked), checked
        ns = info["slices"]
        assert len(info["slice_off"]) == ns + 1 and (np.diff(info["slice_off"]) > 0).all()
        # phase 3: the eight ranks' tiles and the framebuffer reduce
        t0 = time.time()
        total = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
        for r in range(world):
            fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
            it.render(fb, rank=r, world=world)
            torch.cuda.synchronize()   # the render ran on the integrator's stream
            total += fb
            del fb
        torch.cuda.synchronize()
        t_render = time.time() - t0
        one = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
        it.render(one)
        torch.cuda.synchronize()
        assert torch.equal(total, one)
        st = it.stats()
        img = total.view(H * W, 3).cpu().numpy()
        del total, one
        assert np.isfinite(img).all() and (img > 0).any()
        pid = (np.arange(0, H, 64, dtype=np.uint32)[:, None] * W + np.arange(W, dtype=np.uint32)[None, :]).ravel()
        p2s = info["p2s"]
        sl = p2s[(pid % W) * H + pid // W]                 # m_slices[y + H*x]
        assert (sl != 0xFFFFFFFF).all()
        vrls, pc = info["vrls"]
        t0 = time.time()
        recs = oracle.records(oracle.scene(W, H))[pid]
        P = oracle.params(oracle.medium(), seed=c5_share.SEED_RNG, pass_=0)
        cpu, _ = oracle.gather_clustered(P, recs, sl, vrls, pc, info["slice_off"], info["reps"], info["weights"],
                                         np.zeros(0, np.uint32), np.zeros(0, np.float32), rec_ids=pid)
        t_oracle = time.time() - t0
        _assert_close(img[pid], cpu, "C5 frame, every 64th row")
        report = dict(refine_ms_per_rank=info["refine_ms_per_rank"], rbuild_ms_per_rank=info["rbuild_ms_per_rank"],
                      rows_local=[x["rows_local"] for x in info["per_rank"]],
                      clusters_total=int(info["slice_off"][-1]), render_s_8_tiles=t_render,
                      render_kernel_ms=st["ms_render_kernel"], contrib_render=int(st["contrib_render"]),
                      s_phase1=info["s_phase1"], s_phase2=info["s_phase2"], oracle_rows_s=t_oracle, checked=checked)
        print("C5 end to end:", json.dumps(report))
        if os.environ.get("ALVRL_C5_REPORT"):
            with open(os.environ["ALVRL_C5_REPORT"], "w") as f:
                json.dump(report, f, indent=1)
    finally:
        it.close()
