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
