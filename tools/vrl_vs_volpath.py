"""Diagnostic: per-pass VRL frame means vs per-batch volpath frame means
(the statistics behind tests/test_gpu_volpath.py).
  python tools/vrl_vs_volpath.py [vrl props] [volpath max_depth] [volpath rr_depth]"""
import os
import sys

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "mitsuba-alvrl_amd")]
import alvrl  # noqa: E402

props = sys.argv[1] if len(sys.argv) > 1 else "vrlTargetNum=50000;maxParticleDepth=30;rrDepth=1000"
md = int(sys.argv[2]) if len(sys.argv) > 2 else 32
rr = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
w, h, K, B, spp = 24, 16, 32, 16, 512
s = alvrl.scene_default(w, h)
it = alvrl.Integrator("localRefinement=false;globalCluster=false;seed=0xA1B2C3D4;" + props, device=0)
it.preprocess(s)
vm = []
for p in range(K):
    it.prepass(p)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    it.render(fb)
    torch.cuda.synchronize()
    vm.append(fb.cpu().numpy().reshape(h * w, 3))
it.close()
vm = np.asarray(vm, np.float64)
vp = np.asarray([alvrl.volpath_render(s, spp, pass_=1000 + b, max_depth=md, rr_depth=rr).cpu().numpy()
                 for b in range(B)], np.float64)
a, b = vm.mean(axis=(1, 2)), vp.mean(axis=(1, 2))
print("vrl per-pass frame means:", np.round(a, 4))
print("volpath per-batch frame means:", np.round(b, 4))
print(f"vrl {a.mean():.4f} +- {a.std(ddof=1) / np.sqrt(K):.4f}   volpath {b.mean():.4f} +- {b.std(ddof=1) / np.sqrt(B):.4f}")
pix_v, pix_p = vm.mean(0).mean(1), vp.mean(0).mean(1)
r = pix_v / np.maximum(pix_p, 1e-9)
print("per-pixel ratio vrl/volpath: median %.4f q05 %.4f q95 %.4f" % (np.median(r), np.quantile(r, 0.05), np.quantile(r, 0.95)))
print("worst pixels:", np.argsort(np.abs(r - 1))[-5:], r[np.argsort(np.abs(r - 1))[-5:]])
