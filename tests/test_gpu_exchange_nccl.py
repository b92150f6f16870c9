"""The multi-GPU bench path's collectives on the RCCL ("nccl") backend, at one
rank (the one-GPU box cannot host two RCCL ranks): alvrl.Exchange moves its
bytes as device tensors through all_gather_into_tensor, and bench.py reduces
the framebuffer with dist.reduce.  The gloo tests (test_distributed.py) cover
two and three ranks; this covers the device-tensor code path those run on
8 GPUs."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_exchange_and_reduce_on_rccl(gpu_ok):
    import torch
    import torch.distributed as dist
    import alvrl
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dev = torch.device("cuda", 0)
    own = not dist.is_initialized()
    if own:
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        ex = alvrl.Exchange()
        assert ex.device.type == "cuda"
        rng = np.random.default_rng(5)
        mask = (rng.random(1000) < 0.3).astype(np.uint8)
        assert np.array_equal(ex.or_(mask), mask)
        data = rng.integers(0, 255, size=12345, dtype=np.uint8)
        parts = ex.allgatherv(data)
        assert len(parts) == 1 and np.array_equal(parts[0], data)
        # at one rank the library skips its collectives: call the all-gather
        # the library is handed directly (device tensors through RCCL)
        out = np.zeros_like(data)
        assert ex._fn(None, data.ctypes.data, data.size, out.ctypes.data) == 0, ex.error
        assert ex.error is None and ex.calls == 1 and np.array_equal(out, data)
        fb = torch.arange(48, dtype=torch.float32, device=dev)
        dist.reduce(fb, dst=0)
        torch.cuda.synchronize()
        assert torch.equal(fb.cpu(), torch.arange(48, dtype=torch.float32))
    finally:
        if own:
            dist.destroy_process_group()
