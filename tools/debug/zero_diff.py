"""Debug: where do ZeRO and replicated DP (IPC, 2 ranks on one GPU) differ?"""
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from dist_util import run_ranks
from test_ipc_gpu import _engine_zero_worker
from tensorflow_distributed_amd.models import mnist_cnn as M



def _solo_worker(rank, world, B, steps, graph):
    """independent world=1 engines, all on the same data: must agree bit-for-bit"""
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd import _native
    _native.require()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = torch.classes.tfd.MnistEngine(B, 0, 1.0, 5, 0)
    eng.set_adam(0.01, 0.9, 0.999, 1e-8)
    g = torch.Generator().manual_seed(7)
    x = torch.rand(steps, B, 784, generator=g)
    y = torch.randint(0, 10, (steps, B), generator=g, dtype=torch.int32)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(dev))
        eng.sync_shadow()
        for i in range(steps):
            eng.feed_x().copy_(x[i].to(dev))
            eng.feed_y().copy_(y[i].to(dev))
            if i == 0 or not graph:
                eng.train_step()
                if graph:
                    eng.capture_train_step("t")
            else:
                eng.replay("t", 1)
            torch.cuda.current_stream().synchronize()
    torch.cuda.synchronize()
    return eng.params().cpu(), 0


if __name__ == "__main__":
    B, steps, world = 16, int(sys.argv[1]), int(sys.argv[2])
    for graph in (False, True):
        so = run_ranks(_solo_worker, 4, B, 6, graph, timeout=300)
        print("solo graph", graph, "max diff vs rank0", [(p - so[0][0]).abs().max().item() for p, _ in so])
    zr = run_ranks(_engine_zero_worker, world, B, steps, True, timeout=300)
    rp = run_ranks(_engine_zero_worker, world, B, steps, False, timeout=300)
    rp2 = run_ranks(_engine_zero_worker, world, B, steps, False, timeout=300)
    print("errors", [e for _, e in zr + rp + rp2])
    print("replicated run-to-run max diff", (rp[0][0] - rp2[0][0]).abs().max().item())
    print("replicated rank0 vs rank1", (rp[0][0] - rp[1][0]).abs().max().item())
    d = (zr[0][0] - rp[0][0]).abs()
    for k, off in M.OFFSETS.items():
        n = 1
        for s in M.SHAPES[k]:
            n *= s
        dd = d[off:off + n]
        print(f"{k:6s} max {dd.max().item():.4g} frac>1e-2 {(dd > 1e-2).float().mean().item():.4g}")
    W0, W1 = M.OFFSETS["wd1"], M.OFFSETS["bd1"]
    S = (W1 - W0) // world
    for r in range(world):
        dd = d[W0 + r * S:W0 + (r + 1) * S]
        print(f"wd1 shard {r}: max {dd.max().item():.4g} frac {(dd > 1e-2).float().mean().item():.4g}")

