"""GPU parameter-server data-plane probe: 1 ps + 2 workers sharing GPU 0 (gloo control plane).
The chief uploads known values, the other worker pulls; reports how many elements reached the
non-chief's buffer when read (a) at once through a D2H copy, (b) through a device clone, (c) after
a sleep -- for the ps copying with its copy kernel (mode 1) and with hipMemcpyAsync (mode 0).

    python tools/debug/ps_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from dist_util import run_ranks  # noqa: E402


def _probe(rank, world, mode):
    from tensorflow_distributed_amd import _native
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd.parallel.async_ps import mnist_layout
    from tensorflow_distributed_amd.parallel.gpu_ps import GpuParameterServerService, GpuPSClient
    from tensorflow_distributed_amd.training.optimizers import AdamOptimizer

    _native.require()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    layout = mnist_layout(1)
    if rank == 0:
        svc = GpuParameterServerService(0, 1, 2, layout, AdamOptimizer(0.01), dev, sync=True, replicas_to_aggregate=2)
        svc.shard.set_copy_kernel(bool(mode))
        svc.serve()
        return {}
    w = rank - 1
    params = torch.zeros(M.TOTAL, device=dev)
    torch.cuda.synchronize()
    client = GpuPSClient(w, layout, params, lambda: None)
    client.port.set_copy_kernel(bool(mode))
    init = torch.arange(M.TOTAL, dtype=torch.float32) * 1e-3
    if w == 0:
        params.copy_(init.to(dev))
        client.init(step=0, t=0)
    client.pull()
    a = (params.cpu() == init).float().mean().item()
    b = (params.clone().cpu() == init).float().mean().item()
    torch.cuda.synchronize()
    time.sleep(0.2)
    c = (params.cpu() == init).float().mean().item()
    first_bad = int(((params.cpu() != init).nonzero().flatten()[:1].tolist() or [-1])[0])
    client.stop()
    return {"at_once": a, "clone": b, "after_sleep": c, "first_bad": first_bad}


if __name__ == "__main__":
    for mode in (1, 0):
        res = run_ranks(_probe, 3, mode, timeout=120)
        print(f"copy_kernel={mode}: chief {res[1]}  other {res[2]}", flush=True)
