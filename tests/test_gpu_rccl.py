"""The RCCL (`nccl` backend) calls of the multi-GPU bench path, on the one GPU a test box has.

`bench.py --gpus N` runs one process per GPU: `init_process_group("nccl", device_id=…)`, one float64
`all_reduce` of the per-step NMSE_Split sums, one `all_gather` of the last step's predictions and one of the
per-rank timings (`bench.py`, `sharding.py`).  The world-2 logic is covered on gloo (tests/test_dist_gloo.py);
this runs the same calls through RCCL in a one-rank group in a child process (127.0.0.1 rendezvous), so the
backend, the device binding and the dtypes the bench hands it are exercised on the GPU stack itself.
"""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

pytestmark = pytest.mark.gpu

CHILD = textwrap.dedent("""
    import os, sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.environ["REPO"])
    from channelestimationtransformer_amd.sharding import collate_step_sums, gather_predictions

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    sums = torch.rand(20, 2, 5, dtype=torch.float64, device=dev) + 0.5
    ref = sums.clone()
    dist.all_reduce(sums)                                   # what collate_step_sums does at world > 1
    assert torch.equal(sums, ref)
    ratios, mean = collate_step_sums(sums, 1)
    assert ratios.shape == (20, 5) and torch.allclose(mean, (ref[:, 0] / ref[:, 1]).mean(0))
    pred = torch.randn(512, 5, 16, device=dev)
    out = [torch.empty_like(pred)]
    dist.all_gather(out, pred.contiguous())                 # gather_predictions at world > 1
    assert torch.equal(out[0], pred) and torch.equal(gather_predictions(pred, 1)[0], pred)
    allt = [torch.zeros(1, dtype=torch.float64, device=dev)]
    dist.all_gather(allt, torch.tensor([0.125], dtype=torch.float64, device=dev))   # the per-rank timings
    assert float(allt[0].item()) == 0.125
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok")
""")


def test_rccl_calls_of_the_bench_path():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, REPO=repo, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29000 + os.getpid() % 1000),
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl ok" in r.stdout
