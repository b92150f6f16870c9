"""Team-mode probe: one small refinement job set with and without helpers,
printing timings as it goes (each case runs in the same process)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mitsuba-alvrl_amd"))
import alvrl  # noqa: E402
import torch  # noqa: E402


def run(props, w, h, nvrl):
    scene = alvrl.scene_default(w, h)
    vrls, pc = alvrl.trace_vrls(scene, nvrl, seed=0x5EED0001)
    it = alvrl.Integrator(props + ";seed=2712847316", device=0)
    it.set_vrls(vrls, pc)
    it.preprocess(scene)
    t = time.time()
    it.prepass(0)
    st = it.stats()
    cl = it.clusters()
    print(f"  {props}: prepass {time.time() - t:.3f} s, refine kernel {st['ms_refine_kernel']:.1f} ms, "
          f"{len(cl['reps'])} reps, failed {st['slices_failed']}", flush=True)
    return cl


for team in sys.argv[1:]:
    os.environ["ALVRL_REFINE_TEAM"] = team
    print(f"team cap {team}", flush=True)
    a = run("targetNumSlices=5", 96, 64, 300)
    b = run("targetNumSlices=40", 256, 192, 3000)
    if team == sys.argv[1]:
        ref = (a, b)
    else:
        same = all(np.array_equal(x[k], y[k]) for x, y in zip((a, b), ref) for k in x)
        print(f"  identical to team {sys.argv[1]}: {same}", flush=True)
