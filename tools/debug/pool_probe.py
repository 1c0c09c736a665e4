"""Device time of the stem's pool ops at ResNet B=128 (112x112x64 -> 56x56): bn_relu_maxpool,
maxpool2d_bwd_bn, maxpool2d_bwd, in the loaded library's slot mode."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_amd import _native  # noqa: E402

_native.require()
ops = torch.ops.tfd
cuda = torch.device("cuda", 0)
N, H, W, C = 128, 112, 112, 64
torch.manual_seed(0)
y = (torch.randn(N, H, W, C, device=cuda) * 2).bfloat16()
S = ops.bn_part_slots()
part = torch.zeros(max(S, 1), 2, C, device=cuda)
part[0, 0] = y.float().reshape(-1, C).sum(0)
part[0, 1] = (y.float().reshape(-1, C) ** 2).sum(0)
if S == 0:
    part = part[:1]
g, b = torch.ones(C, device=cuda), torch.zeros(C, device=cuda)
rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
out, am, mean, invstd = ops.bn_relu_maxpool(y, g, b, rm, rv, 0.9, 1e-5, part, 3, 2, 1)
dp = torch.randn_like(out)
acc = torch.zeros(max(S, 1), 2, C, device=cuda)


def t(fn, n=30):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


if len(sys.argv) > 1 and sys.argv[1] == "rows":
    ops.set_bn_part_slots(0)
    S, acc = 0, None
print(f"slots {S}: bn_relu_maxpool {t(lambda: ops.bn_relu_maxpool(y, g, b, rm, rv, 0.9, 1e-5, part, 3, 2, 1)):.1f} us, "
      f"maxpool2d_bwd_bn {t(lambda: ops.maxpool2d_bwd_bn(dp, am, [N, H, W, C], 3, 2, 1, y, mean, invstd, g, b, acc)):.1f} us, "
      f"maxpool2d_bwd {t(lambda: ops.maxpool2d_bwd(dp, am, [N, H, W, C], 3, 2, 1)):.1f} us", flush=True)
