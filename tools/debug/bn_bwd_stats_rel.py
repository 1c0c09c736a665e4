"""rel. gradient difference of bn_bwd_stats on/off (fused BN-backward statistics vs the partial pass)
at a few batch/image sizes, in row mode -- how chaotic the tiny-batch comparison is."""
import os
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_amd import _native  # noqa: E402

_native.require()
torch.ops.tfd.set_bn_part_slots(0)
from tensorflow_distributed_amd.models import resnet as R  # noqa: E402

cuda = torch.device("cuda", 0)
for depth in (18, 50):
    for B, hw in ((4, 32), (8, 64), (16, 64)):
        torch.manual_seed(depth)
        x = torch.randn(B, hw, hw, 3, device=cuda)
        lab = torch.randint(0, 16, (B,), dtype=torch.int32, device=cuda)
        out = []
        for on in (False, True):
            m = R.ResNet(depth, num_classes=16, device=cuda, seed=3, width=16, zero_init_residual=False, bn_bwd_stats=on)
            m.fp.grad.zero_()
            loss, _ = m.loss(x, lab)
            loss.backward()
            torch.cuda.synchronize()
            out.append(m.fp.grad.clone())
        rel = ((out[1] - out[0]).norm() / out[0].norm()).item()
        print(f"defer={R._JOIN_DEFER} depth {depth} B {B} hw {hw}: rel {rel:.4f}", flush=True)
