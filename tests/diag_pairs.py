"""Diagnostic (not a test): find the worst pixel of the 64x64x1k brute gather and
compare per-pair contributions device vs oracle to see which pairs diverge."""
import sys, numpy as np, torch
sys.path[:0] = ['oracle', 'mitsuba-alvrl_amd']
import alvrl
from oracle import Oracle
o = Oracle()
sc = o.scene(64, 64); m = o.medium()
vrls, pc = o.trace(sc, m, 1000, seed=0x5EED0001)
recs = o.records(sc)
P = o.params(m, seed=0xA1B2C3D4)
cpu, _ = o.gather_brute(P, recs, vrls, pc)
ctx = alvrl.Context(device=0, seed=0xA1B2C3D4); ctx.set_medium(alvrl.Medium()); ctx.upload_vrls(vrls, pc)
gpu = ctx.gather_brute_host(recs)
rel = np.abs(gpu - cpu) / np.maximum(np.abs(cpu), 1e-30)
print("rel error quantiles", np.quantile(rel, [0.5, 0.9, 0.99, 0.999, 1.0]))
bad = np.argsort(rel.max(1))[::-1][:4]
for p in bad:
    # per-pair: single-VRL sets keep vrl ids through rec ids? use each VRL alone with
    # the same vrl id by uploading all VRLs and a weight vector selecting one.
    rows = []
    for v in range(vrls.shape[1]):
        c_rgb, _, _ = o.integrate(P, recs[p], p, vrls, v)
        rows.append(c_rgb)
    rows = np.array(rows)
    ctx.set_clusters(np.arange(vrls.shape[1] + 1, dtype=np.uint32), np.arange(vrls.shape[1], dtype=np.uint32),
                     np.ones(vrls.shape[1], np.float32), np.zeros(1, np.uint32), np.ones(1, np.float32))
    sl = np.arange(vrls.shape[1], dtype=np.uint32)
    g = ctx.gather_clustered_host(np.repeat(recs[p:p+1], vrls.shape[1], 0), sl, ids=np.full(vrls.shape[1], p, np.uint32)) * pc
    d = np.abs(g - rows).max(1) / np.maximum(np.abs(rows).max(1), 1e-30)
    k = np.argsort(np.abs(g - rows).max(1))[::-1][:3]
    print(f"pixel {p} rel {rel[p].max():.2e} pixel value {cpu[p]}")
    for v in k:
        S, E = vrls[0:3, v], vrls[3:6, v]
        print(f"   vrl {v} cpu {rows[v]} gpu {g[v]} pair-rel {d[v]:.2e} share {rows[v].max()/ (cpu[p].max()*pc):.3f} len {np.linalg.norm(E-S):.3e}")
