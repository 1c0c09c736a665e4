"""Slot-mode statistics partials at a ResNet-50 stage-1 shape: conv2d_fwd_stats with a zeroed
[S,2,K] buffer, the slot sums (read right after the kernel by a GPU reduction, and after a sync)
against torch sums of the stored output. Lost or late atomics show as a mismatch."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_amd import _native  # noqa: E402

_native.require()
ops = torch.ops.tfd
cuda = torch.device("cuda", 0)
torch.manual_seed(0)
N, H, W, C, K = 128, 56, 56, 64, 256
x = (torch.randn(N, H, W, C, device=cuda) * 0.5).bfloat16()
w = (torch.randn(1, 1, C, K, device=cuda) * 0.1).bfloat16()
for slots in (4, 1, 8):
    ops.set_bn_part_slots(slots)
    part = torch.zeros(slots, 2, K, device=cuda)
    worst_gpu, worst_sync = 0.0, 0.0
    for it in range(20):
        part.zero_()
        y, p = ops.conv2d_fwd_stats(x, w, 1, 0, part_out=part)
        s_gpu = p.sum(0)[0].clone()  # a GPU kernel right behind the producer
        torch.cuda.synchronize()
        ref = y.float().reshape(-1, K).sum(0)
        s_sync = p.sum(0)[0]
        worst_gpu = max(worst_gpu, ((s_gpu - ref).abs() / ref.abs().clamp_min(1.0)).max().item())
        worst_sync = max(worst_sync, ((s_sync - ref).abs() / ref.abs().clamp_min(1.0)).max().item())
    print(f"slots={slots}: worst rel err of sum(y) read by the next kernel {worst_gpu:.3e}, after sync {worst_sync:.3e}",
          flush=True)
ops.set_bn_part_slots(4)
