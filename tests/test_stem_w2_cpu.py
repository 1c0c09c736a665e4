"""The width-paired stem (models/resnet.py _StemW2, csrc/bindings/conv_ops.cpp w2_shape) on CPU in fp32:
a 7x7 stride-2 pad-3 conv over 3 channels equals the 7x4 conv over width-paired 8-channel pixels with
the paired filter (height stride 2 / pad 3, width stride 1, left pad 2), and the paired filter's
gradient maps back onto the original filter's (reference stem: the ResNet configs of BASELINE.md)."""
import torch
import torch.nn.functional as F

from tensorflow_distributed_amd.models.resnet import pair_stem_weight, unpair_stem_grad


def pack(x):  # [N, H, W, 3] -> [N, H, W/2, 8], what ops.stem_pack writes (before bf16 rounding)
    N, H, W, _ = x.shape
    return F.pad(x.reshape(N, H, W // 2, 6), (0, 2))


def conv_nhwc(x, w, stride, pad_hw):  # x NHWC, w [R, S, C, K]; pad_hw = (left, right, top, bottom)
    y = F.conv2d(F.pad(x.permute(0, 3, 1, 2), pad_hw), w.permute(3, 2, 0, 1), stride=stride)
    return y.permute(0, 2, 3, 1)


def test_paired_stem_equals_the_7x7_conv_and_maps_its_gradient():
    torch.manual_seed(0)
    N, H, W, K = 2, 20, 18, 16
    x = torch.randn(N, H, W, 3, dtype=torch.float64)
    w = torch.randn(7, 7, 8, K, dtype=torch.float64, requires_grad=True)
    xpad = F.pad(x, (0, 5))  # channels 3..7 zero, as pad_channels
    y = conv_nhwc(xpad, w, 2, (3, 3, 3, 3))
    wp = pair_stem_weight(w)
    assert wp.shape == (7, 4, 8, K)
    Wo = (W + 6 - 7) // 2 + 1
    yp = conv_nhwc(pack(x), wp, (2, 1), (2, Wo + 1 - W // 2, 3, 3))  # right pad so that Wo columns come out
    assert yp.shape == y.shape
    assert torch.allclose(yp, y, rtol=1e-12, atol=1e-12)
    dy = torch.randn_like(y)
    (gw,) = torch.autograd.grad(y, w, dy)
    wp_leaf = wp.detach().requires_grad_(True)
    yq = conv_nhwc(pack(x), wp_leaf, (2, 1), (2, Wo + 1 - W // 2, 3, 3))
    (gwp,) = torch.autograd.grad(yq, wp_leaf, dy)
    dw = torch.full_like(gw, float("nan"))
    unpair_stem_grad(gwp, dw)
    assert torch.allclose(dw, gw, rtol=1e-12, atol=1e-12)
    assert torch.equal(dw[:, :, 3:], torch.zeros_like(dw[:, :, 3:]))
