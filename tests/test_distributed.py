"""The multi-GPU path on CPU: two gloo ranks launched the way the driver
launches bench.py (torch.distributed.run, 127.0.0.1 rendezvous).  Each rank
renders its 64x64 tiles (alvrl_tile_pixels) with the oracle; the framebuffer
reduce to rank 0 must equal the single-process frame bit for bit (every pixel
is owned by exactly one rank), and bench.aggregate_over_ranks must give the
max of the ranks' times and the sum of their counts.  The same run checks the
collectives of the slice-sharded prepass (alvrl.Exchange over gloo:
variable-size all-gather, mask OR, cluster-list merge)."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("world", [2, 3])
def test_tile_sharding_gloo(tmp_path, world):
    out = tmp_path / "verdict.json"
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(HERE, "dist_worker.py"), str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    v = json.loads(out.read_text())
    assert v["world"] == world and v["frame_bit_exact"]
    assert v["pixels_total"] == 150 * 70
    assert v["elapsed_max"] == float(world) and v["ranks"] == world
    assert v["count_sum"] == v["count_full"]
    assert v["exchange"] == {"allgatherv": True, "or": True, "clusters": True, "duplicate_rejected": True}


def test_local_exchange_threads():
    """alvrl_local_exchange (ranks = threads of one process, the plugin's
    amdDevices): variable-size all-gather and mask OR over 3 threads give
    every rank the same rank-ordered result; a rank calling with a different
    message size fails the round on every rank instead of hanging."""
    import threading
    import numpy as np
    import alvrl
    world = 3
    g = alvrl.LocalExchange(world)
    out, err = [None] * world, []

    def run(r):
        try:
            ex = g.rank(r)
            for it in range(4):                      # several rounds reuse the group
                parts = ex.allgatherv(np.full(r + it + 1, 10 * r + it, np.uint8))
                m = np.zeros(8, np.uint8)
                m[(r + it) % 8] = 1
                out[r] = (parts, ex.or_(m))
        except Exception as e:   # pragma: no cover - reported below
            err.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    [t.start() for t in th]
    [t.join(60) for t in th]
    assert not err, err
    for r in range(world):
        parts, m = out[r]
        assert [len(p) for p in parts] == [q + 4 for q in range(world)]
        assert all((p == 10 * q + 3).all() for q, p in enumerate(parts))
        assert np.array_equal(m, np.isin(np.arange(8), [(q + 3) % 8 for q in range(world)]).astype(np.uint8))
    g.close()

    # mismatched sizes on the raw all-gather: every rank's call fails
    g = alvrl.LocalExchange(2)
    L = alvrl._host()
    rcs = [None, None]

    def bad(r):
        a = np.zeros(4 + 4 * r, np.uint8)
        rcs[r] = L.alvrl_exchange_or(alvrl.C.byref(g.rank(r).desc), 2, alvrl._ptr(a), a.size)

    th = [threading.Thread(target=bad, args=(r,)) for r in range(2)]
    [t.start() for t in th]
    [t.join(60) for t in th]
    assert all(rc == alvrl.ALVRL_ERR_COMM for rc in rcs), rcs
    g.close()
