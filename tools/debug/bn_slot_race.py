"""Stress the BN slot mode: the same ResNet forward repeated, loss spread in slot mode vs row mode.
A stale slot read (cache coherence across XCDs, a missing zero) shows up as an outlier loss."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_amd import _native  # noqa: E402

_native.require()
from tensorflow_distributed_amd.models.resnet import ResNet  # noqa: E402

cuda = torch.device("cuda", 0)
torch.manual_seed(0)
x = torch.randn(4, 64, 64, 3).to(cuda)
lab = torch.randint(0, 16, (4,), dtype=torch.int32).to(cuda)
for slots in (0, 4, 1):
    torch.ops.tfd.set_bn_part_slots(slots)
    m = ResNet(50, num_classes=16, device=cuda, seed=1, width=16, zero_init_residual=False)
    vals = []
    for i in range(200):
        loss, _ = m.loss(x, lab)
        vals.append(loss.item())
    v = torch.tensor(vals, dtype=torch.float64)
    print(f"slots={slots} loss min {v.min().item():.6f} max {v.max().item():.6f} first {vals[0]:.6f} "
          f"distinct {len(set(vals))}", flush=True)
    rm = torch.cat([b.rmean for b in m.bns])
    print(f"  rmean finite {bool(torch.isfinite(rm).all())}", flush=True)
torch.ops.tfd.set_bn_part_slots(4)
