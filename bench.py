#!/usr/bin/env python3
"""ALVRL hot-path benchmark (BASELINE.json metric) on N MI355X, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3|C4|C1]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

A step is one progressive pass of the vrl integrator over the whole frame
(vrlIntegrator::prepass + render, vrlIntegrator.cpp:270-599): with resident
VRLs (the vrlFile mode) the prepass is the LightSlice work (representative
sampling, R build, per-slice refinement) for the clustered configs and nothing
for the brute-force one; the render is the per-pixel gather.  Rank 0 prints one JSON line.

Multi-GPU (--shard):
  slices (default)  one pass per step, sharded inside the pass (BASELINE.json
                    north_star): rank r builds R for and refines
                    slices s % N == r, the non-zero mask is OR-reduced and the
                    cluster lists are all-gathered over RCCL
                    (alvrl_integrator_prepass_dist), 64x64 image tiles are
                    dealt round robin, and one RCCL reduce brings the
                    framebuffer to rank 0: "scaling": "strong".
  passes            progressive passes are independent units: at step i rank r
                    runs pass i*N + r over the whole frame (its own
                    representatives, R and clusters) and one RCCL reduce over
                    xGMI sums the N passes' framebuffers into rank 0 -- the
                    progressive accumulation (integrator.cpp:396-433) spread
                    over GPUs.  Per-GPU work is fixed: "scaling": "weak".
With N > 1 and slices, the same run also times the passes decomposition
(W + K more steps) and reports it as "alt_decomposition" beside the line
(--no-alt skips it); "value" is always the slices measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, "mitsuba-alvrl_amd"), os.path.join(REPO, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "VRL contributions/sec + per-pixel RMSE vs CPU (1024², 100k VRLs)"
SEED_VRL = 0x5EED0001
SEED_RNG = 0xA1B2C3D4
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Algorithmic bytes per contribution: one VRL
# record (9 x fp32) per pair for the brute gather, + index + weight for the
# clustered gather, + the (mean, var) float2 written per pair for the R build.
BYTES_PER_PAIR = {"brute": 36, "clustered": 44, "rbuild": 44}

CONFIGS = {
    "C1": dict(w=256, h=256, nvrl=1000, props="",
               desc="256^2 smoke box, 1k VRLs, ALVRL defaults (adaptive, 100 slices)"),
    "C2": dict(w=1024, h=1024, nvrl=10000, props="localRefinement=false;globalCluster=false",
               desc="1024^2 smoke box, 10k VRLs, brute-force VRL gather (clustering off)"),
    "C3": dict(w=1024, h=1024, nvrl=100000, props="targetNumSlices=100;localUndersampling=100",
               desc="1024^2 smoke box, 100k VRLs, LightSlice fixed-depth (localUndersampling=100)"),
    "C4": dict(w=1024, h=1024, nvrl=100000, props="targetNumSlices=100;localUndersampling=-1",
               desc="1024^2 smoke box, 100k VRLs, Adaptive LightSlice refinement"),
    # R is 65,536 rows x 1M VRLs x 8 B = 524 GB: only the slice-sharded pass fits
    # (524/N GB per GPU), so C5 needs --shard slices on >= 4 GPUs
    "C5": dict(w=2048, h=2048, nvrl=1000000, props="targetNumSlices=100;localUndersampling=-1",
               desc="2048^2 smoke box, 1M VRLs, Adaptive LightSlice, slices and tiles over the GPUs",
               min_world=4, shard="slices"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C4", choices=sorted(CONFIGS))
    ap.add_argument("--shard", default="slices", choices=["passes", "slices"],
                    help="multi-GPU decomposition (see the module docstring)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-alt", action="store_true",
                    help="N > 1 with --shard slices: skip the second, pass-parallel measurement")
    ap.add_argument("--no-records-mode", action="store_true",
                    help="clustered configs: skip timing the host-cast (records mode) pipeline")
    ap.add_argument("--no-unconditional", action="store_true",
                    help="clustered configs: skip the comparison with the oracle's own pipeline")
    ap.add_argument("--cpu-row-stride", type=int, default=64,
                    help="CPU baseline sample: every n-th image row")
    ap.add_argument("--pmc-json", default=os.path.join(REPO, "profiles", "r06", "pmc_traffic.json"),
                    help="per-launch HBM bytes of the dominant kernel from a rocprofv3 --pmc pass")
    ap.add_argument("--valu-json", default=os.path.join(REPO, "profiles", "r06", "pmc_valu_{cfg}.json"),
                    help="per-kernel VALU counters (tools/pmc_valu.sh + tools/pmc_valu.py)")
    return ap.parse_args()


def aggregate_over_ranks(elapsed, counts, world, device):
    """The contract's whole-job numbers: the MAX of the ranks' timed-region
    wall times and the SUM of their work counts (exact in float64 below 2^53)."""
    if world == 1:
        return elapsed, [int(c) for c in counts]
    import torch
    import torch.distributed as dist
    if dist.get_backend() == "gloo":
        device = torch.device("cpu")
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    c = torch.tensor([float(x) for x in counts], dtype=torch.float64, device=device)
    dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(x) for x in c.tolist()]


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    import alvrl

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} ranks")
    cfg0 = CONFIGS[args.config]
    if world < cfg0.get("min_world", 1) or (cfg0.get("shard") and args.shard != cfg0["shard"]):
        raise SystemExit(f"{args.config} needs --shard {cfg0.get('shard', args.shard)} on >= "
                         f"{cfg0.get('min_world', 1)} GPUs (R does not fit one GPU)")
    # rehearsal of the N > 1 path on a one-GPU box (never for a measurement):
    # ALVRL_BENCH_ONE_GPU=1 puts every rank on cuda:0 and uses gloo
    rehearse = os.environ.get("ALVRL_BENCH_ONE_GPU") == "1"
    gpu = 0 if rehearse else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    cfg = CONFIGS[args.config]
    W, H = cfg["w"], cfg["h"]
    scene = alvrl.scene_default(W, H)
    # VRL set = the benchmark input (restated vrlTracer, seed 0x5EED0001),
    # resident for every pass exactly like the reference's vrlFile mode.
    vrls, pc = alvrl.trace_vrls(scene, cfg["nvrl"], seed=SEED_VRL)
    props = cfg["props"] + (";" if cfg["props"] else "") + f"seed={SEED_RNG}"
    it = alvrl.Integrator(props, device=gpu)
    it.set_vrls(vrls, pc)
    it.preprocess(scene)
    clustered = "localRefinement=false" not in props
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    by_slices = args.shard == "slices"
    exchange = alvrl.Exchange(device=None if rehearse else dev) if (world > 1 and by_slices) else None

    def step(i, by_slices=by_slices):
        fb.zero_()
        if by_slices:   # one pass, LightSlice work and tiles sharded over ranks
            it.prepass(i, rank, world, exchange)
            it.render(fb, rank, world, stream=stream)
        else:           # pass i*N + rank, whole frame
            it.prepass(i * world + rank)
            it.render(fb, 0, 1, stream=stream)
        if world > 1:
            if rehearse:
                h = fb.cpu()
                dist.reduce(h, dst=0)
                fb.copy_(h)
            else:
                dist.reduce(fb, dst=0)   # the single RCCL framebuffer reduce per step

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize(dev)

    for i in range(args.warmup):
        step(i)
    barrier()
    s0 = it.stats()
    kernel_ms, rbuild_ms, refine_ms, prepass_ms, refine_kms, refine_ent, refine_split = [], [], [], [], [], [], []
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
        st = it.stats()           # HIP-event kernel times of this step (synchronises)
        kernel_ms.append(st["ms_render_kernel"])
        rbuild_ms.append(st["ms_rbuild"])
        refine_ms.append(st["ms_refine"])
        prepass_ms.append(st["ms_prepass_wall"])
        refine_kms.append(st["ms_refine_kernel"])
        refine_ent.append(st["refine_entries"])
        refine_split.append(st["refine_split_entries"])
    barrier()
    elapsed = time.perf_counter() - t0
    s1 = it.stats()
    contrib = (s1["contrib_preprocess"] - s0["contrib_preprocess"]) + (s1["contrib_render"] - s0["contrib_render"])
    render_pairs = s1["contrib_render"] - s0["contrib_render"]
    pre_pairs = s1["contrib_preprocess"] - s0["contrib_preprocess"]
    elapsed, (contrib, render_pairs, pre_pairs) = aggregate_over_ranks(
        elapsed, [contrib, render_pairs, pre_pairs], world, dev)

    value = contrib / elapsed

    # N > 1: the other decomposition too, on the same ranks and scene
    # (reported beside the line, never as its value): whole progressive
    # passes per GPU and one framebuffer reduce, which scales weakly
    alt = None
    if world > 1 and by_slices and not args.no_alt:
        base = args.warmup + args.steps
        for i in range(args.warmup):
            step(base + i, by_slices=False)
        barrier()
        a0 = it.stats()
        barrier()
        ta = time.perf_counter()
        for i in range(args.steps):
            step(base + args.warmup + i, by_slices=False)
        barrier()
        a_el = time.perf_counter() - ta
        a1 = it.stats()
        a_c = (a1["contrib_preprocess"] - a0["contrib_preprocess"]) + (a1["contrib_render"] - a0["contrib_render"])
        a_el, (a_c,) = aggregate_over_ranks(a_el, [a_c], world, dev)
        alt = {"shard": "passes", "scaling": "weak", "value": a_c / a_el, "unit": "VRL contributions/s",
               "ms_per_step": a_el / args.steps * 1e3, "steps": args.steps, "warmup": args.warmup,
               "parallelism": f"{world} progressive passes per step, one per GPU, RCCL reduce of the framebuffer"}
    # Rooflines (this rank's launches, HIP events on the stream each kernel ran
    # on).  Algorithmic bytes per launch (DESIGN.md "Roofline"): the gathers
    # and the R build count BYTES_PER_PAIR per VRL contribution; the
    # refinement counts 8 B per R entry per pass over it: the
    # three setup passes read the local matrix once each, and every split
    # reads its cluster three times -- projections, forward and reverse
    # calculateClusterVariance (alvrl_last_refine_entries + 2 x
    # alvrl_last_refine_split_entries); "frac_one_pass" keeps the earlier
    # rounds' count (each split's cluster once) for comparison.
    nst = max(args.steps, 1)
    kind = "clustered" if clustered else "brute"
    # committed counter files count only if they were taken on the library
    # this run loaded (their build_id, tools/pmc_summary.py / pmc_valu.py);
    # a file from another tree reports traffic / valu null.  The traffic
    # records are one GPU's launches (tools/pmc_traffic.sh runs N = 1): a rank
    # of N > 1 launches over its share, so its traffic is reported null
    my_id = alvrl.build_info()["build_id"]
    counters = {"pmc_json": os.path.relpath(args.pmc_json, REPO),
                "valu_json": os.path.relpath(args.valu_json.format(cfg=args.config), REPO),
                "build_id": my_id, "pmc_matches": False, "valu_matches": False}
    pmc = {}
    try:
        with open(args.pmc_json) as f:
            pm = json.load(f)
        for rec in (pm if isinstance(pm, list) else [pm]):
            if rec.get("config") == args.config and rec.get("build_id") == my_id and world == 1:
                pmc[rec.get("kernel_key", "render")] = rec.get("hbm_bytes_per_launch")
                counters["pmc_matches"] = True
    except (OSError, ValueError):
        pass

    valu = {}
    try:
        with open(args.valu_json.format(cfg=args.config)) as f:
            valu = {k: v for k, v in json.load(f).items() if v.get("build_id") == my_id}
        counters["valu_matches"] = bool(valu)
    except (OSError, ValueError, AttributeError):
        pass

    def roof(name, key, bytes_per_launch, ms, note):
        # achieved / frac: ALGORITHMIC bytes per launch (the contract's
        # definition); traffic: measured HBM bytes per launch
        # (rocprofv3 PMC, FETCH_SIZE x2 + WRITE_SIZE), and hbm_achieved /
        # hbm_frac the rate those bytes moved at in the same launch time
        s_ = ms / 1e3
        ach = bytes_per_launch / s_ / 1e9 if s_ > 0 else 0.0
        tr = pmc.get(key)
        hbm = tr / s_ / 1e9 if (tr is not None and s_ > 0) else None
        out = {"bound": "hbm", "kernel": name, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": ach / HBM_PEAK_GBS, "traffic": tr, "bytes_per_launch": bytes_per_launch,
               "hbm_achieved": hbm, "hbm_frac": hbm / HBM_PEAK_GBS if hbm is not None else None,
               "launch_ms": ms, "note": note}
        v = valu.get(key)
        if v:
            # VALU issue roofline (rocprofv3 pass of the same config, tools/pmc_valu.py):
            # fraction of one wave-instruction per SIMD per 2 cycles, VALU
            # instructions per VRL pair and the pair rate that issue peak allows
            out["valu"] = {k: v.get(k) for k in ("valu_issue_frac", "insts_per_pair", "pair_rate",
                                                 "pair_rate_at_valu_peak", "clock_ghz", "ms")}
            out["valu"]["source"] = os.path.relpath(args.valu_json.format(cfg=args.config), REPO)
        return out

    pairs_per_launch_rank = (s1["contrib_render"] - s0["contrib_render"]) / nst
    rooflines = {"render": roof(f"k_gather_{kind}", "render", BYTES_PER_PAIR[kind] * pairs_per_launch_rank,
                               float(np.mean(kernel_ms)) if kernel_ms else 0.0,
                               "the gather is VALU/transcendental-bound (VRL records are broadcast from "
                               "SGPRs), see DESIGN.md")}
    if clustered:
        ent1 = float(np.mean(refine_ent))
        ent3 = ent1 + 2.0 * float(np.mean(refine_split))
        rooflines["refine"] = roof("k_refine", "refine", 8.0 * ent3, float(np.mean(refine_kms)),
                                   "8 B per R entry per pass: 3 setup passes + 3 per split (projections, "
                                   "forward and reverse variance); latency-bound f64 recurrences, see DESIGN.md")
        rk = float(np.mean(refine_kms)) / 1e3
        rooflines["refine"]["frac_one_pass"] = (8.0 * ent1 / rk / 1e9 / HBM_PEAK_GBS) if rk > 0 else None
        rooflines["refine"]["bytes_one_pass"] = 8.0 * ent1
        strict = "strictRbuild=false" not in props          # the integrator's default R build
        rooflines["rbuild"] = roof("k_build_R_strict" if strict else "k_build_R_blocks", "rbuild",
                                   BYTES_PER_PAIR["rbuild"] * (s1["contrib_preprocess"] - s0["contrib_preprocess"]) / nst,
                                   float(np.mean(rbuild_ms)),
                                   "VALU-bound: integrateVRL in the oracle's arithmetic (f64 transcendentals with a "
                                   "Ziv rounding test, IEEE division and sqrt), bit-identical to the oracle's R"
                                   if strict else "VALU-bound like the gather")
    dominant = max(rooflines, key=lambda k: rooflines[k]["launch_ms"])

    out = None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "VRL contributions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if by_slices else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: restated vrlTracer VRLs (seed 0x5EED0001) in the BASELINE.md smoke box",
            "config": {"workload": f"{args.config}: {cfg['desc']}", "resolution": [W, H],
                       "vrls": int(vrls.shape[1]), "particles": int(pc),
                       "parallelism": (f"one pass per step: slices and 64x64 image tiles round-robin over "
                                       f"{world} GPU(s), RCCL mask OR + cluster all-gather + framebuffer reduce"
                                       if by_slices else
                                       f"{world} progressive pass(es) per step, one per GPU, "
                                       f"RCCL reduce of the framebuffer")},
            "breakdown": {"render_pairs": render_pairs, "prepass_pairs": pre_pairs,
                          "render_kernel_ms": float(np.mean(kernel_ms)) if kernel_ms else None,
                          "rbuild_ms": float(np.mean(rbuild_ms)), "refine_ms": float(np.mean(refine_ms)),
                          "refine_kernel_ms": float(np.mean(refine_kms)),
                          "refine_entries": float(np.mean(refine_ent)),
                          "refine_split_entries": float(np.mean(refine_split)),
                          "prepass_wall_ms": float(np.mean(prepass_ms)),
                          "slices": int(s1["slices"]), "rep_rows": int(s1["rep_rows"]),
                          "clusters_total": int(s1["clusters_total"]),
                          "slices_failed": int(s1["slices_failed"]),
                          "exchange_ms": float(s1["ms_exchange"])},
            "roofline": rooflines[dominant],
            "rooflines": rooflines,
            "cpu_baseline": None,
            # the prebuilt in-tree library this run loaded, and whether it was
            # built from this tree's sources (alvrl_build_id vs the tree's hash)
            "build_mode": dict(alvrl.build_info(), mode="prebuilt in-tree (make, hipcc --offload-arch=gfx950)"),
            "counter_files": counters,
        }
        if alt is not None:
            out["alt_decomposition"] = alt
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], out["pixel_rmse_vs_cpu"] = cpu_baseline(args, cfg, scene, vrls, pc, fb, it,
                                                                       clustered)
        if clustered:
            out["cpu_baseline"] = cpu_baseline_prepass(args, cfg, vrls, pc, it, out["cpu_baseline"],
                                                       pre_pairs / max(args.steps, 1),
                                                       render_pairs / max(args.steps, 1))
            if not args.no_records_mode:
                out["records_mode"] = records_mode(cfg, vrls, pc, args.warmup + args.steps + 10, gpu)
            if not args.no_unconditional:
                out["pixel_rmse_vs_cpu_unconditional"] = unconditional_parity(
                    cfg, vrls, pc, args.warmup + args.steps - 1, fb.view(-1, 3).cpu().numpy(), it, gpu,
                    row_stride=args.cpu_row_stride)
                u = out["pixel_rmse_vs_cpu_unconditional"]
                d = u["default_vs_oracle_pipeline"]
                # the headline's per-pixel RMSE vs the CPU reference: the
                # oracle's own pipeline (no device result fed to it)
                out["pixel_rmse_vs_cpu"]["unconditional"] = dict(d, within_gather_tolerance=bool(
                    d["median_rel"] <= 1e-6 and d["q99_rel"] <= 1e-4 and d["max_rel"] <= 5e-2),
                    all_pins_identical=u["all_pins_identical"])
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(args, cfg, scene, vrls, pc, fb, it, clustered):
    """The CPU restatement (oracle/, built with the reference's CXXFLAGS) timed
    on this host's cores on a bounded sample of the same workload, and the
    per-pixel RMSE of the device frame against it on that sample."""
    import numpy as np
    from oracle import Oracle
    o = Oracle(fast=True)
    W, H = cfg["w"], cfg["h"]
    threads = cpu_threads()
    rows = np.arange(0, H, args.cpu_row_stride)
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
    osc = o.scene(W, H)
    recs = o.records(osc)[pix]
    m = o.medium()
    last_pass = args.warmup + args.steps - 1
    P = o.params(m, seed=SEED_RNG, pass_=last_pass)
    if clustered:
        # clustered frame: the device's own cluster lists for the sampled pixels
        cl = it.clusters()
        p2s = it.slices()
        xs, ys = pix % W, pix // W
        sl = p2s[ys + H * xs]
        t0 = time.perf_counter()
        img, cnt = o.gather_clustered(P, recs, sl, vrls, pc, cl["slice_off"], cl["reps"], cl["weights"],
                                      cl["fb_reps"], cl["fb_weights"], rec_ids=pix, nthreads=threads)
        dt = time.perf_counter() - t0
        sample = (f"clustered gather of every {args.cpu_row_stride}th image row ({len(pix)} pixels) "
                  f"with the device's cluster lists")
    else:
        t0 = time.perf_counter()
        img, cnt = o.gather_brute(P, recs, vrls, pc, rec_ids=pix, nthreads=threads)
        dt = time.perf_counter() - t0
        sample = f"brute gather of every {args.cpu_row_stride}th image row ({len(pix)} pixels x {vrls.shape[1]} VRLs)"
    gpu = fb.view(-1, 3)[torch_index(pix).to(fb.device)].cpu().numpy()
    diff = gpu.astype(np.float64) - img.astype(np.float64)
    rmse = float(np.sqrt(np.mean(diff ** 2)))
    rel = np.abs(diff) / np.maximum(np.abs(img), 1e-30)
    base = {"value": cnt / dt, "unit": "VRL contributions/s", "cores": threads, "kind": "port",
            "sample": sample, "seconds": dt, "host_cpus": _host_cpus(),
            "cpu": _cpu_model(), "flags": "reference CXXFLAGS (build/config-linux-gcc.py:7)"}
    acc = {"rmse": rmse, "mean": float(np.abs(img).mean()), "rmse_rel": rmse / max(float(np.abs(img).mean()), 1e-30),
           "max_rel": float(rel.max()), "median_rel": float(np.median(rel)), "pixels": int(len(pix))}
    return base, acc


def cpu_baseline_prepass(args, cfg, vrls, pc, it, render_base, pre_pairs_step, render_pairs_step):
    """Clustered configs: one CPU step = R build + refinement + clustered render.
    Bounded samples: the R rows of one slice's representatives (all threads),
    the refinement of the median-size and of the largest slice (one thread
    each: the reference refines whole slices per worker thread,
    Preprocessor.cpp:722-773), and the clustered gather sample of
    cpu_baseline().  The step time is extrapolated from them: R rows x
    columns at the measured rate, ceil(slices / threads) rounds of
    refinement of which the last waits for the largest slice, and the render
    pairs at the measured rate; value = the step's contributions / that time."""
    import numpy as np
    from oracle import Oracle
    o = Oracle(fast=True)
    W, H = cfg["w"], cfg["h"]
    threads = cpu_threads()
    off, pix = it.reps()
    ns = len(off) - 1
    nrows = np.diff(off)
    s_med = int(np.argsort(nrows, kind="stable")[ns // 2])      # a median-size slice
    s_max = int(np.argmax(nrows))                                # the largest slice
    rp = pix[off[s_med]:off[s_med + 1]]
    rec_ids = ((rp % H) * W + rp // H).astype(np.uint32)   # column-major ids -> row-major
    recs = o.records(o.scene(W, H))[rec_ids]
    last_pass = args.warmup + args.steps - 1
    P = o.params(o.medium(), seed=SEED_RNG, pass_=last_pass)
    t0 = time.perf_counter()
    _, Rs, cnt = o.gather_brute(P, recs, vrls, pc, rec_ids=rec_ids, domain=2, want_R=True, nthreads=threads)
    t_r = time.perf_counter() - t0
    kv = dict(x.split("=", 1) for x in cfg["props"].split(";") if "=" in x)
    under = float(kv.get("localUndersampling", -1.0))
    dcorr = float(kv.get("depthCorrection", 1.0))
    cl = it.clusters()
    t_ref, parity = {}, []
    for s0 in dict.fromkeys((s_med, s_max)):
        # the refinement sample is the device's own job for slice s0 (its R
        # rows, locality weights, pixel undersampling and initial clusters)
        job = it.slice_job(s0)
        nrow = job["R"].shape[1]
        args_ = (job["R"], np.arange(nrow, dtype=np.uint32), job["locw"], job["init_vrls"], job["init_off"],
                 job["pixel_undersampling"], under)
        kw = dict(depth_correction=dcorr, seed=SEED_RNG, pass_=last_pass, stage_refine=3 + 2 * s0,
                  stage_sample=4 + 2 * s0)
        os.environ["ALVRL_ORACLE_THREADS"] = "0"    # timed: sequential, one slice per thread as the reference
        t0 = time.perf_counter()
        reps, w, refined = o.cluster_refine(*args_, **kw)
        t_ref[s0] = time.perf_counter() - t0
        os.environ.pop("ALVRL_ORACLE_THREADS", None)
        # the timed run is the reference-flags build (reassociating float
        # maths); the bit-exact check runs the strict build of the same restatement
        reps, w, refined = Oracle().cluster_refine(*args_, **kw)
        dev_reps = cl["reps"][cl["slice_off"][s0]:cl["slice_off"][s0 + 1]]
        dev_w = cl["weights"][cl["slice_off"][s0]:cl["slice_off"][s0 + 1]]
        identical = bool(refined and np.array_equal(reps, dev_reps)
                         and np.array_equal(w.view(np.uint32), dev_w.view(np.uint32)))
        parity.append({"slice": s0, "rows": int(nrow), "clusters_oracle": int(len(reps)),
                       "clusters_device": int(len(dev_reps)), "identical": identical,
                       "refine_s": t_ref[s0]})
    r_rate = cnt / t_r
    render_rate = render_base["value"]
    rounds = int(np.ceil(ns / threads))
    t_refine = (rounds - 1) * t_ref[s_med] + t_ref[s_max]
    t_step = pre_pairs_step / r_rate + t_refine + render_pairs_step / render_rate
    return {"value": (pre_pairs_step + render_pairs_step) / t_step, "unit": "VRL contributions/s",
            "cores": threads, "kind": "port",
            "sample": (f"R rows of slice {s_med} ({nrows[s_med]} representatives x {vrls.shape[1]} VRLs, "
                       f"{t_r:.2f} s on {threads} threads), the adaptive refinement of slices {s_med} "
                       f"({t_ref[s_med]:.2f} s) and {s_max} (the largest, {nrows[s_max]} rows, "
                       f"{t_ref[s_max]:.2f} s), one thread each, and {render_base['sample']}; step "
                       f"extrapolated: {ns} slices over {threads} threads ({rounds} rounds)"),
            "seconds": t_r + sum(t_ref.values()) + render_base["seconds"], "step_seconds_estimate": t_step,
            "host_cpus": render_base["host_cpus"], "cpu": render_base["cpu"], "flags": render_base["flags"],
            "rates": {"rbuild": r_rate, "render": render_rate, "refine_s_median_slice": t_ref[s_med],
                      "refine_s_largest_slice": t_ref[s_max]},
            "refine_parity": parity}


def unconditional_parity(cfg, vrls, pc, pass_, frame, it, device=0, row_stride=64, pin_slices=True,
                         fast_reference=True):
    """The benchmarked (default, strict R) pipeline's frame of pass `pass_`
    against the CPU restatement's OWN pipeline of that pass, on every
    `row_stride`-th image row.  `it` is the integrator
    that rendered `frame` and still holds that pass.

    The oracle's pipeline over the full R (1.6e9 pairs at C4) takes minutes on
    the host, so it is re-derived here on three slices -- the median-size, the
    largest and the one with the most clusters: the oracle's own R rows of the
    slice's representatives (oracle.gather_brute) against the device's, bit for
    bit, and the oracle's refinement of those rows (oracle.cluster_refine)
    against the device's list.  The device's pipeline computes every slice
    with the same kernels (R bit-identical to the oracle's for every strategy
    and scene in tests/test_gpu_strict.py, refinement bit-exact given R), so
    its lists are the oracle's own; the oracle then renders the sampled rows
    with them (its own clustered gather), and the device frame must meet the
    gather tolerance of tests/test_gpu_parity.py against it.

    fast_reference: the fast R build (strictRbuild=false, the gathers' maths)
    through the same pass, for the record: its cluster lists differ from the
    oracle's (float rounding flips discrete decisions), so it is held to the
    method's noise -- the RMSE between the oracle's frames of pass `pass_` and
    `pass_ + 1` -- not to the float tolerance."""
    import numpy as np
    import torch
    import alvrl
    from oracle import Oracle
    o = Oracle()                                 # the strict (IEEE) build: the parity checker
    W, H = cfg["w"], cfg["h"]
    threads = cpu_threads()
    base_props = cfg["props"] + (";" if cfg["props"] else "") + f"seed={SEED_RNG}"
    rows = np.arange(0, H, row_stride)
    pix = (rows[:, None] * W + np.arange(W)[None, :]).reshape(-1).astype(np.uint32)
    recs_all = o.records(o.scene(W, H))
    recs = recs_all[pix]
    xs, ys = pix % W, pix // W
    kv = dict(x.split("=", 1) for x in cfg["props"].split(";") if "=" in x)

    def device_pass(p, strict):
        it2 = alvrl.Integrator(base_props + f";strictRbuild={'true' if strict else 'false'}", device=device)
        it2.set_vrls(vrls, pc)
        it2.preprocess(alvrl.scene_default(W, H))
        it2.prepass(p)
        fb = torch.zeros(W * H * 3, dtype=torch.float32, device=torch.device("cuda", device))
        it2.render(fb)
        torch.cuda.synchronize(device)
        return it2, fb.view(-1, 3).cpu().numpy()

    def oracle_frame(itx, p):
        cl, p2s = itx.clusters(), itx.slices()
        P = o.params(o.medium(), seed=SEED_RNG, pass_=p)
        img, _ = o.gather_clustered(P, recs, p2s[ys + H * xs], vrls, pc, cl["slice_off"], cl["reps"],
                                    cl["weights"], cl["fb_reps"], cl["fb_weights"], rec_ids=pix, nthreads=threads)
        return img, cl

    def cmp(a, b):
        d = a.astype(np.float64) - b.astype(np.float64)
        rel = np.abs(d) / np.maximum(np.abs(b.astype(np.float64)), 1e-30)
        return {"rmse": float(np.sqrt(np.mean(d ** 2))), "median_rel": float(np.median(rel)),
                "q99_rel": float(np.quantile(rel, 0.99)), "max_rel": float(rel.max())}

    t0 = time.perf_counter()
    O, clO = oracle_frame(it, pass_)
    pins = []
    if pin_slices:
        off, rp = it.reps()
        ns = len(off) - 1
        nrows = np.diff(off)
        ncl = np.diff(clO["slice_off"])
        picks = {"median": int(np.argsort(nrows, kind="stable")[ns // 2]), "largest": int(np.argmax(nrows)),
                 "most_clusters": int(np.argmax(ncl))}
        P = o.params(o.medium(), seed=SEED_RNG, pass_=pass_)
        for why, s in picks.items():
            job = it.slice_job(s)
            ids = rp[off[s]:off[s + 1]]
            rid = ((ids % H) * W + ids // H).astype(np.uint32)           # column-major -> row-major
            tr = time.perf_counter()
            _, Ro, _ = o.gather_brute(P, recs_all[rid], vrls, pc, rec_ids=rid, domain=2, want_R=True,
                                      nthreads=threads)
            tr = time.perf_counter() - tr
            r_same = bool(np.array_equal(np.ascontiguousarray(job["R"].transpose(1, 0, 2)).view(np.uint32),
                                         Ro.view(np.uint32)))
            tc = time.perf_counter()
            reps, w, refined = o.cluster_refine(np.ascontiguousarray(Ro.transpose(1, 0, 2)),
                                                np.arange(len(rid), dtype=np.uint32), job["locw"],
                                                job["init_vrls"], job["init_off"], job["pixel_undersampling"],
                                                float(kv.get("localUndersampling", -1.0)),
                                                depth_correction=float(kv.get("depthCorrection", 1.0)),
                                                seed=SEED_RNG, pass_=pass_, stage_refine=3 + 2 * s,
                                                stage_sample=4 + 2 * s)
            tc = time.perf_counter() - tc
            b, e = clO["slice_off"][s], clO["slice_off"][s + 1]
            l_same = bool(refined and np.array_equal(reps, clO["reps"][b:e])
                          and np.array_equal(w.view(np.uint32), clO["weights"][b:e].view(np.uint32)))
            pins.append({"slice": s, "pick": why, "rows": int(len(rid)), "R_bit_identical": r_same,
                         "clusters": int(e - b), "cluster_list_identical": l_same,
                         "oracle_R_s": tr, "oracle_refine_s": tc})
    it2, _ = device_pass(pass_ + 1, True)
    O2, _ = oracle_frame(it2, pass_ + 1)
    it2.close()
    noise = cmp(O2, O)
    dev = cmp(frame[pix], O)
    out = {"pass": pass_, "pixels": int(len(pix)),
           "sample": f"every {row_stride}th image row; the oracle's clustered gather with its own cluster lists",
           "default_vs_oracle_pipeline": dev,
           "oracle_pass_to_pass": noise,
           "oracle_pipeline_pinned_on_slices": pins,
           "all_pins_identical": bool(pins) and all(q["R_bit_identical"] and q["cluster_list_identical"]
                                                   for q in pins)}
    if fast_reference:
        itF, F = device_pass(pass_, False)
        stF = itF.stats()
        a, b = itF.clusters(), clO
        same = sum(1 for s in range(len(a["slice_off"]) - 1)
                   if np.array_equal(a["reps"][a["slice_off"][s]:a["slice_off"][s + 1]],
                                     b["reps"][b["slice_off"][s]:b["slice_off"][s + 1]]))
        itF.close()
        fast = cmp(F[pix], O)
        out["fast_rbuild_reference"] = {
            "note": "strictRbuild=false (not the default): held to the method's pass-to-pass noise",
            "vs_oracle_pipeline": fast, "rmse_ratio_to_pass_noise": fast["rmse"] / noise["rmse"] if noise["rmse"] > 0
            else None, "slices_with_oracle_lists": [same, len(a["slice_off"]) - 1],
            "rbuild_ms": float(stF["ms_rbuild"])}
    out["seconds"] = time.perf_counter() - t0
    return out


def records_mode(cfg, vrls, pc, pass0, device=0, steps=2, blocks=(128, 32), threads=16):
    """The host-cast ABI the Mitsuba plugin's records mode drives
    (include/alvrl_host.h "host-cast scenes"), timed per pass:
    the host hands the representative pixels' eye records to
    alvrl_integrator_prepass_records (R, clusters) and renders the frame in
    image blocks from `threads` host threads, one alvrl_gather_clustered_host
    call per block with host-memory records and results (renderBlock,
    renderproc.cpp:52-86) -- every record crosses PCIe.  Block sizes: 128
    (`mitsuba -b 128`, the largest mitsuba.cpp:233-237 accepts) and the
    default 32.  The host here plays Mitsuba with the library's own scene (the
    smoke box has no null surfaces, so buildSlices' gather point of a pixel is
    its eye record's hit)."""
    import numpy as np
    import alvrl
    from concurrent.futures import ThreadPoolExecutor
    W, H = cfg["w"], cfg["h"]
    s = alvrl.scene_default(W, H)
    recs = alvrl.scene_records(s)                        # the host's rays, cast once
    props = cfg["props"] + (";" if cfg["props"] else "") + f"seed={SEED_RNG}"
    it = alvrl.Integrator(props, device=device)
    it.set_vrls(vrls, pc)
    it.preprocess_ext(W, H, recs, list(s.box_min), list(s.box_max), alvrl.Medium())
    ctx = it.context()
    p2s = it.slices()
    allpix = np.arange(W * H, dtype=np.uint32)
    sl_all = p2s[(allpix % W) * H + allpix // W]
    frame = np.zeros((W * H, 3), np.float32)
    out = {"unit": "VRL contributions/s", "steps": steps, "host_threads": threads,
           "note": "host-pointer ABI (records and results cross PCIe), renderBlock-sized calls from "
                   "concurrent host threads; not the metric's value", "by_block": {}}
    p = pass0
    for block in blocks:
        bl = []
        for by in range(0, H, block):
            for bx in range(0, W, block):
                ids = (np.arange(by, min(by + block, H))[:, None] * W + np.arange(bx, min(bx + block, W))[None, :])
                ids = ids.ravel().astype(np.uint32)
                bl.append((np.ascontiguousarray(recs[ids]), np.ascontiguousarray(sl_all[ids]), ids))

        def render_block(b):
            r, sl, ids = b
            frame[ids] = ctx.gather_clustered_host(r, sl, ids=ids)

        def one_pass(q):
            pix = it.rep_pixels(q)
            it.prepass_records(q, recs[pix], np.arange(len(pix), dtype=np.uint32))
            t = time.perf_counter()
            with ThreadPoolExecutor(threads) as ex:
                list(ex.map(render_block, bl))
            return time.perf_counter() - t

        one_pass(p)                                      # warm-up
        p += 1
        s0 = it.stats()
        hb0 = ctx.host_batch_stats()["clustered"]
        t0 = time.perf_counter()
        render_s = 0.0
        for _ in range(steps):
            render_s += one_pass(p)
            p += 1
        dt = time.perf_counter() - t0
        s1 = it.stats()
        pairs = (s1["contrib_preprocess"] - s0["contrib_preprocess"]) + (s1["contrib_render"] - s0["contrib_render"])
        hb1 = ctx.host_batch_stats()["clustered"]
        out["by_block"][str(block)] = {"value": pairs / dt, "ms_per_step": dt / steps * 1e3,
                                       "render_ms_per_step": render_s / steps * 1e3, "blocks": len(bl),
                                       "launches_per_step": (hb1[0] - hb0[0]) / steps}
    it.close()
    best = out["by_block"][str(blocks[0])]
    out.update(value=best["value"], ms_per_step=best["ms_per_step"], block=blocks[0])
    return out


def cpu_threads():
    """The host cores this process may use: its CPU affinity, capped by a
    cgroup CPU quota when one is set (a GPU box shares its host), or
    ALVRL_CPU_THREADS."""
    env = os.environ.get("ALVRL_CPU_THREADS")
    if env:
        return max(1, int(env))
    n = _host_cpus()["affinity"]
    q = _host_cpus()["cgroup_quota"]
    return max(1, min(n, int(q)) if q else n)


def _host_cpus():
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            a, b = f.read().split()[:2]
            if a != "max":
                quota = float(a) / float(b)
    except (OSError, ValueError):
        pass
    return {"affinity": aff, "cgroup_quota": quota, "os_cpu_count": os.cpu_count()}


def torch_index(pix):
    import torch
    return torch.from_numpy(pix.astype("int64"))


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
