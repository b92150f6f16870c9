"""Host vs device VRL tracer (vrlTracer::randomWalk) at the C4 target (100k
VRLs in the 1024^2 smoke box): wall time of each, and the sets' equality."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mitsuba-alvrl_amd"))
import alvrl  # noqa: E402

s = alvrl.scene_default(1024, 1024)
target = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
alvrl.trace_vrls_gpu(s, 1000)                      # device init
t0 = time.perf_counter(); h, hp = alvrl.trace_vrls(s, target); t1 = time.perf_counter()
d, dp = alvrl.trace_vrls_gpu(s, target); t2 = time.perf_counter()
print({"target": target, "vrls": int(h.shape[1]), "particles": hp, "host_ms": round(1e3 * (t1 - t0), 2),
       "gpu_ms_incl_copies": round(1e3 * (t2 - t1), 2),
       "identical": bool(dp == hp and np.array_equal(h.view(np.uint32), d.view(np.uint32)))})
