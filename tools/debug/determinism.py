"""Debug: is every stage of the MNIST engine step deterministic when 4 processes share the GPU?
Each process repeats the same forward/backward R times on fixed params and records, per stage,
whether any repeat differs from its first result; rank 0's first results are compared across
processes."""
import os, sys
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
from dist_util import run_ranks


def _worker(rank, world, B, R, unfused):
    from tensorflow_distributed_amd.models import mnist_cnn as M
    from tensorflow_distributed_amd import _native
    _native.require()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    eng = torch.classes.tfd.MnistEngine(B, 0, 1.0, 5, 0)
    eng.set_adam(0.01, 0.9, 0.999, 1e-8)
    assert not unfused, 'the two-kernel conv forward was removed (fused conv12 only)'
    g = torch.Generator().manual_seed(7)
    x = torch.rand(B, 784, generator=g)
    y = torch.randint(0, 10, (B,), generator=g, dtype=torch.int32)
    s = torch.cuda.Stream()
    first, bad = {}, {}
    with torch.cuda.stream(s):
        eng.params().copy_(M.flat_from_dict({k: v * 0.05 for k, v in M.init_params(3).items()}).to(dev))
        eng.sync_shadow()
        eng.feed_x().copy_(x.to(dev))
        eng.feed_y().copy_(y.to(dev))
        for it in range(R):
            eng.grads().zero_()
            snaps = {"x": eng.feed_x().clone(), "params": eng.params().clone()}
            eng.forward(True)
            snaps["pool1"] = eng.pool1().clone(); snaps["pool2"] = eng.pool2().clone()
            snaps["hidden"] = eng.hidden().clone(); snaps["loss"] = eng.loss_rows().clone()
            eng.backward_a()
            snaps["grad_a"] = eng.grads().clone()
            eng.backward_b()
            snaps["grad_b"] = eng.grads().clone()
            torch.cuda.current_stream().synchronize()
            for k, v in snaps.items():
                v = v.float().cpu()
                if it == 0:
                    first[k] = v
                else:
                    d = (v - first[k]).abs().max().item()
                    bad[k] = max(bad.get(k, 0.0), d)
                    if d > 0 and k == "pool1":
                        dm = ((v - first[k]).abs() > 0).reshape(B, 14, 14, 32)
                        imgs = dm.flatten(1).any(1).nonzero().flatten().tolist()
                        chans = dm.any(0).any(0).any(0).nonzero().flatten().tolist()
                        print(f"rank {rank} it {it}: pool1 differs in images {imgs} channels {chans} "
                              f"count {int(dm.sum())}", flush=True)
                        vv, ff = v.reshape(B, 14, 14, 32), first[k].reshape(B, 14, 14, 32)
                        for (bi, hh, ww, cc) in dm.nonzero().tolist()[:12]:
                            print(f"   b{bi} px{hh * 14 + ww} c{cc}: first {ff[bi, hh, ww, cc].item():.5f} now "
                                  f"{vv[bi, hh, ww, cc].item():.5f} ch-1 {vv[bi, hh, ww, cc - 1].item():.5f}/"
                                  f"{ff[bi, hh, ww, cc - 1].item():.5f}", flush=True)
    return {k: v for k, v in bad.items()}, {k: v for k, v in first.items()}


if __name__ == "__main__":
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    unfused = int(sys.argv[2]) if len(sys.argv) > 2 else 0  # 1: conv1_pool_fwd (VALU conv1) + conv2 kernels
    res = run_ranks(_worker, world, 16, 60, unfused, timeout=400)
    for r, (bad, first) in enumerate(res):
        print("rank", r, "within-process max diff:", {k: f"{v:.3g}" for k, v in bad.items()})
        print("rank", r, "vs rank0:", {k: f"{(first[k] - res[0][1][k]).abs().max().item():.3g}" for k in first})
