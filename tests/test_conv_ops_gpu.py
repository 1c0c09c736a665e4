"""Numerics of the generic NHWC HIP kernel library (conv fwd/dgrad/wgrad, dense, batch norm,
pooling, softmax-xent) against plain PyTorch fp32 references of the same ops."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
ops = None


@pytest.fixture(autouse=True, params=[(0, 0), (2, 0), (1, 2)], ids=["core128", "core256", "halo"])
def _ops(cuda, request):
    """Every conv test runs on every GEMM path: the 128-row register-staged core and the 256-row DMA
    core with the im2col gather (each forced for every shape it applies to; the default picks the
    256-row core where its tiles fill the chip), and the LDS halo-tile kernel (csrc/conv_halo.h) for
    every 3x3 stride-1 conv with 64-channel multiples, narrow maps included."""
    global ops
    ops = torch.ops.tfd
    core, halo = request.param
    old = ops.conv_gemm_core(core), ops.conv_halo_mode(halo)
    yield
    ops.conv_gemm_core(old[0])
    ops.conv_halo_mode(old[1])


@pytest.fixture(params=[0, 4], ids=["rowmode", "slots4"])
def bn_mode(request):
    """BN statistics partials in row mode (one row per producer block, bn_final) and in slot mode
    (fp32 atomics into 4 zeroed slots, the apply pass finalizes inline)."""
    old = torch.ops.tfd.set_bn_part_slots(request.param)
    yield request.param
    torch.ops.tfd.set_bn_part_slots(old)


def rb(t):  # round to bf16 and back (the kernels' operand precision)
    return t.to(torch.bfloat16).float()


def relerr(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()


def same_sums(a, b, rtol=1e-5, atol=1e-5):
    """BN statistics from two runs: bit-identical in row mode (fixed order); in slot mode
    (bn_part_slots() > 0) the producers' fp32 atomics may add in another order."""
    if torch.ops.tfd.bn_part_slots() == 0:
        assert torch.equal(a, b)
    else:
        torch.testing.assert_close(a, b, rtol=rtol, atol=atol)


CONVS = [  # N, H, W, C, K, R, stride, pad
    (2, 9, 7, 16, 24, 3, 1, 1),
    (2, 10, 10, 16, 32, 3, 2, 1),
    (3, 8, 8, 32, 16, 1, 1, 0),
    (2, 9, 9, 16, 32, 1, 2, 0),
    (2, 16, 16, 8, 16, 7, 2, 3),
    (4, 14, 14, 64, 64, 3, 1, 1),
]


# (48, 28, 28, 128, ...): its dgrad (M = 37632, C = 128) takes the 128x128 tiles of the LDS-staged
# epilogue; (48, 28, 28, 64, 64): 128x64 output tiles for fwd and dgrad; (48, 56, 56, 64, 64, s2): the
# strided phase dgrad on 128x64 tiles
# halo-tile shapes (3x3 s1, 64-channel multiples): partial tiles in both directions with 128-wide
# output tiles, three input-channel chunks, a 7-wide map (halo mode 2), C != K both ways
HALO = [(2, 20, 36, 64, 128, 3, 1, 1), (2, 9, 23, 192, 64, 3, 1, 1), (3, 7, 7, 128, 64, 3, 1, 1),
        (2, 16, 16, 64, 192, 3, 1, 1)]


@pytest.mark.parametrize("N,H,W,C,K,R,st,pad", CONVS + HALO + [(48, 28, 28, 128, 32, 3, 1, 1), (48, 28, 28, 64, 64, 3, 1, 1),
                                                          (48, 56, 56, 64, 64, 3, 2, 1)])
def test_conv_fwd_dgrad_wgrad(cuda, N, H, W, C, K, R, st, pad):
    torch.manual_seed(0)
    x = rb(torch.randn(N, H, W, C))
    w = rb(torch.randn(R, R, C, K) * 0.2)
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    wr = w.permute(3, 2, 0, 1).clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, stride=st, padding=pad)
    dy = rb(torch.randn_like(yr))
    yr.backward(dy)
    y = ops.conv2d_fwd(x.to(cuda, torch.bfloat16), w.to(cuda, torch.bfloat16), st, pad)
    assert relerr(y.cpu().permute(0, 3, 1, 2), yr.detach()) < 1e-2
    dyn = dy.permute(0, 2, 3, 1).contiguous().to(cuda, torch.bfloat16)
    dx = ops.conv2d_dgrad(dyn, w.to(cuda, torch.bfloat16), [N, H, W, C], st, pad)
    assert relerr(dx.cpu().permute(0, 3, 1, 2), xr.grad) < 1e-2
    dw = torch.zeros(R, R, C, K, device=cuda)
    ops.conv2d_wgrad(x.to(cuda, torch.bfloat16), dyn, dw, st, pad)
    assert relerr(dw.cpu(), wr.grad.permute(2, 3, 1, 0)) < 1e-3
    # residual-join form: dx = acc + dgrad in the dgrad epilogue
    acc0 = rb(torch.randn(N, H, W, C))
    acc = acc0.to(cuda, torch.bfloat16)
    dx2 = ops.conv2d_dgrad(dyn, w.to(cuda, torch.bfloat16), [N, H, W, C], st, pad, acc)
    assert dx2.data_ptr() != acc.data_ptr()
    assert relerr(dx2.cpu().float().permute(0, 3, 1, 2), xr.grad + acc0.permute(0, 3, 1, 2)) < 1e-2
    # pre-zeroed weight-gradient buffer: no per-call memset
    dw2 = torch.zeros(R, R, C, K, device=cuda)
    ops.conv2d_wgrad(x.to(cuda, torch.bfloat16), dyn, dw2, st, pad, True)
    assert relerr(dw2.cpu(), wr.grad.permute(2, 3, 1, 0)) < 1e-3


@pytest.mark.parametrize("N,H,W,C,K,R,st,pad", [(32, 14, 14, 256, 1024, 1, 1, 0), (64, 7, 7, 512, 2048, 1, 1, 0),
                                                  (16, 14, 14, 128, 128, 3, 1, 1), (32, 14, 14, 256, 128, 1, 2, 0)])
def test_conv_wgrad_long_split_k(cuda, N, H, W, C, K, R, st, pad):
    """Weight gradients of ResNet-50 stage-3/4 shapes: 33-49 K-tiles per split and (tile x split)
    grids divisible by 8 (the XCD renumbering of the wgrad launch), against the fp32 oracle."""
    torch.manual_seed(1)
    x = rb(torch.randn(N, H, W, C))
    Ho = (H + 2 * pad - R) // st + 1
    dy = rb(torch.randn(N, Ho, Ho, K))
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2), (K, C, R, R), dy.permute(0, 3, 1, 2),
                                      stride=st, padding=pad)
    for zeroed in (False, True):
        dw = torch.zeros(R, R, C, K, device=cuda)
        ops.conv2d_wgrad(x.to(cuda, torch.bfloat16), dy.to(cuda, torch.bfloat16), dw, st, pad, zeroed)
        assert relerr(dw.cpu(), ref.permute(2, 3, 1, 0)) < 1e-5


@pytest.mark.parametrize("N,H,W,C,K,R,st,pad", CONVS + HALO + [(8, 28, 28, 64, 256, 1, 1, 0), (48, 28, 28, 32, 64, 3, 1, 1)])
def test_conv_fwd_stats_feeds_bn(cuda, bn_mode, N, H, W, C, K, R, st, pad):
    """conv2d_fwd_stats: same output as conv2d_fwd, and per-row-block sums of the stored bf16 output
    that bn_fwd(partials=...) turns into the same normalisation as its own statistics pass. The
    last shape takes the 128x128 tiles."""
    torch.manual_seed(5)
    x = rb(torch.randn(N, H, W, C)).to(cuda, torch.bfloat16)
    w = rb(torch.randn(R, R, C, K) * 0.2).to(cuda, torch.bfloat16)
    y0 = ops.conv2d_fwd(x, w, st, pad)
    y, part = ops.conv2d_fwd_stats(x, w, st, pad)
    assert torch.equal(y, y0)
    yf = y.float().reshape(-1, K)
    assert part.shape[1:] == (2, K)
    torch.testing.assert_close(part[:, 0].sum(0), yf.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(part[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-4, atol=1e-3)
    y2, part2 = ops.conv2d_fwd_stats(x, w, st, pad)  # row mode: bit-identical partials on a rerun
    assert torch.equal(y2, y)
    same_sums(part2, part, rtol=1e-5, atol=1e-3)
    g, b = torch.rand(K, device=cuda) + 0.5, torch.randn(K, device=cuda)
    rm0, rv0 = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
    rm1, rv1 = rm0.clone(), rv0.clone()
    o0, m0, i0 = ops.bn_fwd(y, g, b, None, True, rm0, rv0, 0.9, 1e-5)
    o1, m1, i1 = ops.bn_fwd(y, g, b, None, True, rm1, rv1, 0.9, 1e-5, part)
    torch.testing.assert_close(m1, m0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(i1, i0, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv1, rv0, rtol=1e-4, atol=1e-5)
    assert relerr(o1, o0) < 1e-2


# forward BN fold: padded 3x3 (zero taps must stay zero after the affine + relu), strided 3x3,
# 1x1, a channel count that is not a multiple of the 64-wide K tile, 128x128 / 128x64 output tiles
@pytest.mark.parametrize("N,H,W,C,K,R,st,pad", [(2, 9, 7, 16, 24, 3, 1, 1), (2, 10, 10, 16, 32, 3, 2, 1),
                                               (3, 8, 8, 40, 16, 1, 1, 0), (48, 28, 28, 64, 128, 1, 1, 0),
                                               (48, 28, 28, 32, 64, 3, 1, 1), (4, 14, 14, 512, 64, 3, 1, 1)])
def test_conv_folded_bn_input_is_bit_identical(cuda, bn_mode, N, H, W, C, K, R, st, pad):
    """conv2d_fwd / conv2d_fwd_stats / conv2d_wgrad with the input's batch norm + relu applied by the
    operand loader (mean, invstd, gamma, beta passed) against the same ops on bn_fwd's materialised
    output: bit-identical outputs, statistics partials and weight gradients."""
    torch.manual_seed(7)
    ops.conv_gemm_core(0)  # the folded form always takes the 128-row core with the im2col gather
    ops.conv_halo_mode(0)  # (the fixture restores both modes)
    y = rb(torch.randn(N, H, W, C) * 2 + 0.3).to(cuda, torch.bfloat16)
    w = rb(torch.randn(R, R, C, K) * 0.2).to(cuda, torch.bfloat16)
    g, b = (torch.rand(C) + 0.5).to(cuda), torch.randn(C).to(cuda)
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    out, mean, invstd = ops.bn_fwd(y, g, b, None, True, rm, rv, 0.9, 1e-5)
    assert (out.float() == 0).any() and (out.float() > 0).any()  # the relu acts
    act = (mean, invstd, g, b)
    y0 = ops.conv2d_fwd(out, w, st, pad)
    assert torch.equal(ops.conv2d_fwd(y, w, st, pad, *act), y0)
    y1, p1 = ops.conv2d_fwd_stats(out, w, st, pad)
    y2, p2 = ops.conv2d_fwd_stats(y, w, st, pad, *act)
    assert torch.equal(y2, y1) and torch.equal(y2, y0)
    same_sums(p2, p1, rtol=1e-5, atol=1e-3)
    dy = rb(torch.randn(N, y0.shape[1], y0.shape[2], K)).to(cuda, torch.bfloat16)
    dw0, dw1 = torch.zeros(R, R, C, K, device=cuda), torch.zeros(R, R, C, K, device=cuda)
    ops.conv2d_wgrad(out, dy, dw0, st, pad, True)
    ops.conv2d_wgrad(y, dy, dw1, st, pad, True, *act)
    assert relerr(dw1, dw0) < 1e-5  # split-K atomics: the fp32 add order may differ
    # bn_stats: the finalize alone, same statistics and running-stat update as bn_fwd
    rm2, rv2 = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
    yk, pk = ops.conv2d_fwd_stats(y, w, st, pad)
    m3, i3 = ops.bn_stats(yk, pk, rm2, rv2, 0.9, 1e-5)
    rm3, rv3 = torch.zeros(K, device=cuda), torch.ones(K, device=cuda)
    _, m4, i4 = ops.bn_fwd(yk, torch.ones(K, device=cuda), torch.zeros(K, device=cuda), None, False, rm3, rv3, 0.9, 1e-5,
                           pk)
    for u, v in ((m3, m4), (i3, i4), (rm2, rm3), (rv2, rv3)):
        same_sums(u, v)
    with pytest.raises(RuntimeError):
        ops.conv2d_fwd(y, w, st, pad, mean, invstd, g, None)


def test_linear(cuda):
    torch.manual_seed(1)
    M, Kin, N = 24, 64, 40
    x, w, b = rb(torch.randn(M, Kin)), rb(torch.randn(Kin, N) * 0.1), torch.randn(N)
    y = ops.linear_fwd(x.to(cuda, torch.bfloat16), w.to(cuda, torch.bfloat16), b.to(cuda))
    assert relerr(y.cpu(), x @ w + b) < 1e-4
    dy = rb(torch.randn(M, N))
    dx = ops.linear_dgrad(dy.to(cuda, torch.bfloat16), w.to(cuda, torch.bfloat16))
    assert relerr(dx.cpu(), dy @ w.t()) < 1e-2
    dw = torch.empty(Kin, N, device=cuda)
    ops.linear_wgrad(x.to(cuda, torch.bfloat16), dy.to(cuda, torch.bfloat16), dw)
    assert relerr(dw.cpu(), x.t() @ dy) < 1e-4


@pytest.mark.parametrize("relu,res", [(True, False), (False, True), (True, True)])
def test_batchnorm_train(cuda, bn_mode, relu, res):
    torch.manual_seed(2)
    M, C = 300, 64
    y = rb(torch.randn(M, C) * 3 + 1)
    g, b = torch.rand(C) + 0.5, torch.randn(C)
    r = rb(torch.randn(M, C)) if res else None
    rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    out, mean, invstd = ops.bn_fwd(y.to(cuda, torch.bfloat16), g.to(cuda), b.to(cuda),
                                   r.to(cuda, torch.bfloat16) if res else None, relu, rm, rv, 0.9, 1e-5)
    yr = y.clone().requires_grad_(True)
    z = F.batch_norm(yr, None, None, g, b, training=True, eps=1e-5)
    if res:
        z = z + r
    if relu:
        z = torch.relu(z)
    assert relerr(out.cpu(), z.detach()) < 1e-2
    torch.testing.assert_close(mean.cpu(), y.mean(0), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rm.cpu(), 0.1 * y.mean(0), rtol=1e-4, atol=1e-4)
    dout = rb(torch.randn(M, C))
    dg, db = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
    dy, dres = ops.bn_bwd(dout.to(cuda, torch.bfloat16), out, y.to(cuda, torch.bfloat16), g.to(cuda), mean, invstd,
                          relu, res, dg, db)
    gr = torch.autograd.grad(z, [yr], dout)[0]
    # dgamma / dbeta reference
    yh = (y - y.mean(0)) / torch.sqrt(y.var(0, unbiased=False) + 1e-5)
    mask = (z.detach() > 0).float() if relu else torch.ones_like(y)
    dz = dout * mask
    assert relerr(dy.cpu(), gr) < 2e-2
    assert relerr(db.cpu(), dz.sum(0)) < 1e-3 and relerr(dg.cpu(), (dz * yh).sum(0)) < 1e-2
    if res:
        assert relerr(dres.cpu(), dz) < 1e-2
    if relu and res:  # relu bits from the forward instead of `out`: same output, same gradients
        mask = torch.empty(M, C // 8, dtype=torch.uint8, device=cuda)
        out3, _, _ = ops.bn_fwd(y.to(cuda, torch.bfloat16), g.to(cuda), b.to(cuda), r.to(cuda, torch.bfloat16), relu,
                                torch.zeros(C, device=cuda), torch.ones(C, device=cuda), 0.9, 1e-5, None, mask)
        assert torch.equal(out3, out)
        bits = ((mask.cpu().long().unsqueeze(-1) >> torch.arange(8)) & 1).reshape(M, C).bool()
        assert torch.equal(bits, out.cpu().float() > 0)
        dg3, db3 = torch.empty_like(dg), torch.empty_like(db)
        dy3, dres3 = ops.bn_bwd(dout.to(cuda, torch.bfloat16), torch.empty_like(out), y.to(cuda, torch.bfloat16),
                                g.to(cuda), mean, invstd, relu, res, dg3, db3, None, mask)
        assert torch.equal(dres3, dres)
        same_sums(dg3, dg)
        same_sums(db3, db)
        same_sums(dy3.float(), dy.float(), rtol=1e-2, atol=1e-2)  # bf16: a changed sum may flip a rounding
    if relu and not res:  # mask recomputed from y (beta given): `out` is not read, same gradients
        dg2, db2 = torch.empty_like(dg), torch.empty_like(db)
        dy2, _ = ops.bn_bwd(dout.to(cuda, torch.bfloat16), torch.empty_like(out), y.to(cuda, torch.bfloat16),
                            g.to(cuda), mean, invstd, relu, res, dg2, db2, b.to(cuda))
        same_sums(dg2, dg)
        same_sums(db2, db)
        same_sums(dy2.float(), dy.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("M,C", [(100000, 64), (20000, 520)])
def test_batchnorm_totals_many_groups(cuda, bn_mode, M, C):
    """Large M (1024 partial rows): statistics and dgamma/dbeta against fp64 sums, bit-identical when
    repeated in row mode (fixed summation order; slot mode: close)."""
    torch.manual_seed(6)
    y = rb(torch.randn(M, C) * 2 + 0.5)
    g, b = torch.rand(C) + 0.5, torch.randn(C)
    yd = y.to(cuda, torch.bfloat16)
    outs = []
    for _ in range(2):
        rm, rv = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
        out, mean, invstd = ops.bn_fwd(yd, g.to(cuda), b.to(cuda), None, True, rm, rv, 0.9, 1e-5)
        dout = rb(torch.randn(M, C, generator=torch.Generator().manual_seed(1))).to(cuda, torch.bfloat16)
        dg, db = torch.empty(C, device=cuda), torch.empty(C, device=cuda)
        dy, _ = ops.bn_bwd(dout, out, yd, g.to(cuda), mean, invstd, True, False, dg, db)
        outs.append([t.cpu() for t in (out, mean, invstd, rm, rv, dg, db, dy)])
    for a, c in zip(outs[0], outs[1]):
        # slot mode: M = 1e5 rows of fp32 atomics in any order (sums of both signs: 1e-4 relative)
        same_sums(a.float(), c.float(), rtol=1e-2 if a.dtype == torch.bfloat16 else 1e-4,
                  atol=1e-2 if a.dtype == torch.bfloat16 else 1e-3)
    out, mean, invstd, rm, rv, dg, db, dy = outs[0]
    y64 = y.double()
    mu, var = y64.mean(0), y64.var(0, unbiased=False)
    torch.testing.assert_close(mean.double(), mu, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(invstd.double(), 1 / torch.sqrt(var + 1e-5), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(rv.double(), 0.9 + 0.1 * y64.var(0, unbiased=True), rtol=1e-4, atol=1e-5)
    dout64 = rb(torch.randn(M, C, generator=torch.Generator().manual_seed(1))).double()
    mask = (out.double() > 0).double()
    dz = dout64 * mask
    yh = (y64 - mu) / torch.sqrt(var + 1e-5)
    assert relerr(db, dz.sum(0)) < 1e-4 and relerr(dg, (dz * yh).sum(0)) < 2e-3


def test_maxpool_avgpool(cuda):
    torch.manual_seed(3)
    x = rb(torch.randn(2, 11, 9, 16))
    y, am = ops.maxpool2d_fwd(x.to(cuda, torch.bfloat16), 3, 2, 1)
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.cpu().float().permute(0, 3, 1, 2), yr.detach())
    dy = rb(torch.randn_like(yr))
    yr.backward(dy)
    dx = ops.maxpool2d_bwd(dy.permute(0, 2, 3, 1).contiguous().to(cuda, torch.bfloat16), am, [2, 11, 9, 16], 3, 2, 1)
    assert relerr(dx.cpu().permute(0, 3, 1, 2), xr.grad) < 1e-2
    a = ops.avgpool_fwd(x.to(cuda, torch.bfloat16))
    assert relerr(a.cpu(), x.mean((1, 2))) < 1e-2
    da = ops.avgpool_bwd(rb(torch.ones(2, 16)).to(cuda, torch.bfloat16), [2, 11, 9, 16])
    assert torch.allclose(da.cpu().float(), torch.full((2, 11, 9, 16), 1 / 99.0), rtol=1e-2)


def test_softmax_xent_and_pad(cuda):
    torch.manual_seed(4)
    z = torch.randn(5, 1000) * 3
    lab = torch.randint(0, 1000, (5,), dtype=torch.int32)
    loss, corr, dl = ops.softmax_xent(z.to(cuda), lab.to(cuda))
    zr = z.clone().requires_grad_(True)
    lr = F.cross_entropy(zr, lab.long(), reduction="none")
    lr.mean().backward()
    torch.testing.assert_close(loss.cpu(), lr.detach(), rtol=1e-4, atol=1e-4)
    assert relerr(dl.cpu().float(), zr.grad) < 1e-2
    assert torch.equal(corr.cpu(), (z.argmax(1) == lab.long()).float())
    x = torch.randn(2, 4, 4, 3)
    p = ops.pad_channels(x.to(cuda), 8)
    assert p.shape == (2, 4, 4, 8) and torch.equal(p.cpu()[..., :3].float(), rb(x)) and p[..., 3:].abs().sum() == 0


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 264, 72), (1000, 520, 1032), (513, 2048, 576)])
def test_gemm256_nt_matches_fp32(cuda, M, N, K):
    """The 256 x 256 core (buffer-load-to-LDS staging, 32x32x16 MFMA, XCD-grouped tiles): C = A Bt^T
    against an fp32 reference of the same bf16 operands, ragged M / N / K tails included."""
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = (torch.rand(M, K, device=cuda, generator=g) * 2 - 1).bfloat16()
    Bt = (torch.rand(N, K, device=cuda, generator=g) * 2 - 1).bfloat16()
    C = torch.ops.tfd.gemm_nt(A, Bt).float()
    ref = A.float() @ Bt.float().t()
    torch.testing.assert_close(C, ref.bfloat16().float(), rtol=1e-2, atol=1e-2 * ref.abs().max().item())


@pytest.mark.parametrize("N,H,W,C", [(2, 16, 16, 64), (3, 15, 13, 32), (8, 112, 112, 64)])
def test_bn_relu_maxpool_equals_bn_then_pool(cuda, bn_mode, N, H, W, C):
    """The stem's fused relu(bn(y)) -> 3x3/2 max pool (bn_relu_maxpool) against bn_fwd + maxpool2d_fwd
    from the same conv-epilogue partials: output and argmax bit for bit, the same statistics and running
    stats (row mode: bit for bit; slot mode: both finalize the same slot sums)."""
    torch.manual_seed(9)
    x = rb(torch.randn(N, H, W, 8)).to(cuda, torch.bfloat16)
    w = rb(torch.randn(3, 3, 8, C) * 0.3).to(cuda, torch.bfloat16)
    y, part = ops.conv2d_fwd_stats(x, w, 1, 1)
    g, b = (torch.rand(C) + 0.5).to(cuda), torch.randn(C).to(cuda)
    rm0, rv0 = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    rm1, rv1 = rm0.clone(), rv0.clone()
    bo, m0, i0 = ops.bn_fwd(y, g, b, None, True, rm0, rv0, 0.9, 1e-5, part)
    p0, a0 = ops.maxpool2d_fwd(bo, 3, 2, 1)
    p1, a1, m1, i1 = ops.bn_relu_maxpool(y, g, b, rm1, rv1, 0.9, 1e-5, part, 3, 2, 1)
    torch.cuda.synchronize()
    assert torch.equal(p1, p0) and torch.equal(a1, a0)
    for u, v in ((m1, m0), (i1, i0), (rm1, rm0), (rv1, rv0)):
        assert torch.equal(u, v)


@pytest.mark.parametrize("N,H,W,C,k,st,pad", [(2, 16, 16, 64, 3, 2, 1), (3, 15, 13, 32, 3, 2, 1), (8, 112, 112, 64, 3, 2, 1),
                                            (2, 9, 11, 16, 2, 2, 0), (2, 10, 10, 8, 3, 3, 1), (2, 8, 8, 16, 3, 1, 1)])
def test_maxpool_bwd_matches_torch(cuda, N, H, W, C, k, st, pad):
    """Max-pool backward (the row-walking 2x2-window kernel where ceil(k / stride) <= 2, the generic
    one else) against torch's max_pool2d backward on the same bf16 input."""
    torch.manual_seed(11)
    x = rb(torch.randn(N, H, W, C))
    y, am = ops.maxpool2d_fwd(x.to(cuda, torch.bfloat16), k, st, pad)
    xr = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    yr = F.max_pool2d(xr, k, st, pad)
    assert torch.equal(y.cpu().float().permute(0, 3, 1, 2), yr.detach())
    dy = rb(torch.randn_like(yr))
    yr.backward(dy)
    dx = ops.maxpool2d_bwd(dy.permute(0, 2, 3, 1).contiguous().to(cuda, torch.bfloat16), am, [N, H, W, C], k, st, pad)
    assert relerr(dx.cpu().permute(0, 3, 1, 2), xr.grad) < 1e-2


@pytest.mark.parametrize("N,H,W,C,K", [(2, 14, 14, 64, 32), (3, 9, 7, 32, 16), (16, 28, 28, 256, 128)])
def test_dgrad_with_stride2_add_operand(cuda, N, H, W, C, K):
    """conv2d_dgrad / conv2d_dgrad_bn with acc_sub2: a [N, ceil(H/2), ceil(W/2), C] operand added at the
    even pixels equals adding its zero-filled full-grid form (the 1x1 stride-2 shortcut dgrad)."""
    torch.manual_seed(12)
    dy = rb(torch.randn(N, H, W, K)).to(cuda, torch.bfloat16)
    w = rb(torch.randn(1, 1, C, K) * 0.2).to(cuda, torch.bfloat16)
    comp = rb(torch.randn(N, (H + 1) // 2, (W + 1) // 2, C)).to(cuda, torch.bfloat16)
    full = torch.zeros(N, H, W, C, device=cuda, dtype=torch.bfloat16)
    full[:, ::2, ::2, :] = comp
    ref = ops.conv2d_dgrad(dy, w, [N, H, W, C], 1, 0, full)
    got = ops.conv2d_dgrad(dy, w, [N, H, W, C], 1, 0, comp, None, True)
    assert torch.equal(got, ref)
    y = rb(torch.randn(N, H, W, C)).to(cuda, torch.bfloat16)
    mean, invstd = torch.zeros(C, device=cuda), torch.ones(C, device=cuda)
    g = torch.ones(C, device=cuda)
    r0, p0 = ops.conv2d_dgrad_bn(dy, w, [N, H, W, C], 1, 0, full, y, mean, invstd, g, None, None, False)
    r1, p1 = ops.conv2d_dgrad_bn(dy, w, [N, H, W, C], 1, 0, comp, y, mean, invstd, g, None, None, False, None, None, True)
    assert torch.equal(r1, r0)
    torch.testing.assert_close(p1.sum(0), p0.sum(0), rtol=1e-4, atol=1e-3)
    # a strided 3x3 consumer (phase GEMMs): the odd pixels get no add
    w3 = rb(torch.randn(3, 3, C, K) * 0.1).to(cuda, torch.bfloat16)
    dy2 = rb(torch.randn(N, (H + 1) // 2, (W + 1) // 2, K)).to(cuda, torch.bfloat16)
    ref2 = ops.conv2d_dgrad(dy2, w3, [N, H, W, C], 2, 1, full)
    got2 = ops.conv2d_dgrad(dy2, w3, [N, H, W, C], 2, 1, comp, None, True)
    assert torch.equal(got2, ref2)


@pytest.mark.parametrize("N,H,W,K", [(2, 32, 30, 64), (3, 23, 16, 16)])
def test_width_paired_stem_matches_the_padded_conv(cuda, N, H, W, K):
    """stem_pack + conv2d_fwd_stats_w2 / conv2d_wgrad_w2 (the ResNet stem, models/resnet.py _StemW2)
    against the channel-padded 7x7 stride-2 conv on the same bf16 operands: output, BN partials'
    column sums, and the filter gradient mapped back by unpair_stem_grad."""
    from tensorflow_distributed_amd.models.resnet import pair_stem_weight, unpair_stem_grad
    torch.manual_seed(2)
    x = torch.randn(N, H, W, 3, device=cuda)
    w = (torch.randn(7, 7, 8, K, device=cuda) * 0.2).to(torch.bfloat16)
    w[:, :, 3:] = 0
    xpad = ops.pad_channels(x, 8)
    xp = ops.stem_pack(x)
    assert torch.equal(xp.view(N, H, W // 2, 8)[..., :6].reshape(N, H, W, 3), xpad[..., :3])
    assert torch.equal(xp[..., 6:], torch.zeros_like(xp[..., 6:]))
    y0, p0 = ops.conv2d_fwd_stats(xpad, w, 2, 3)
    y1, p1 = ops.conv2d_fwd_stats_w2(xp, pair_stem_weight(w), 2, 3)
    assert y1.shape == y0.shape
    assert relerr(y1.float(), y0.float()) < 1e-2
    torch.testing.assert_close(p1.sum(0), p0.sum(0), rtol=2e-2, atol=2e-2)
    dy = rb(torch.randn(y0.shape)).to(cuda, torch.bfloat16)
    dw0 = torch.zeros(7, 7, 8, K, device=cuda)
    ops.conv2d_wgrad(xpad, dy, dw0, 2, 3)
    dwp = torch.empty(7, 4, 8, K, device=cuda)
    ops.conv2d_wgrad_w2(xp, dy, dwp, 2, 3, False)
    dw1 = torch.full_like(dw0, float("nan"))
    unpair_stem_grad(dwp, dw1)
    assert relerr(dw1, dw0) < 1e-5


MEMSET_RACE = ("platform: a captured hipMemsetAsync node (a root node, 32 KB) is intermittently not ordered "
               "before the kernel that depends on it on graph replays -- 2048 of 8192 accumulator elements "
               "garbage from replay 1 on some boxes, clean on others (profiles/memset_capture_probe_r6.log)")


@pytest.mark.parametrize("clear", [0, pytest.param(1, marks=pytest.mark.xfail(strict=False, reason=MEMSET_RACE))])
def test_captured_split_k_wgrad_zeroes_its_accumulator_on_every_replay(cuda, clear):
    """conv2d_wgrad(zeroed=False) with split-K clears dw itself; captured in a graph and replayed, every
    replay must give the eager result. clear 0: the fill kernel (the library's); 1: hipMemsetAsync, kept
    as the platform reproducer (xfail, not strict: it passes on some boxes) -- which is why no capturable
    path issues a memset (tests/test_source_hygiene_cpu.py, docs/DESIGN.md §8)."""
    old = ops.conv_wgrad_clear_mode(clear)
    try:
        _split_k_replay(cuda)
    finally:
        ops.conv_wgrad_clear_mode(old)


def _split_k_replay(cuda):
    torch.manual_seed(4)
    x = rb(torch.randn(16, 14, 14, 64)).to(cuda, torch.bfloat16)  # 3,136 pixels: split-K
    dy = rb(torch.randn(16, 14, 14, 128)).to(cuda, torch.bfloat16)
    ref = torch.zeros(1, 1, 64, 128, device=cuda)
    ops.conv2d_wgrad(x, dy, ref, 1, 0)
    dw = torch.full((1, 1, 64, 128), 7.0, device=cuda)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.conv2d_wgrad(x, dy, dw, 1, 0)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.conv2d_wgrad(x, dy, dw, 1, 0)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert relerr(dw, ref) < 1e-5


@pytest.mark.parametrize("C", [64, 12])
def test_avgpool_chunk_and_scalar_forms(cuda, C):
    """avgpool_fwd / avgpool_bwd: the 8-channel chunk kernels (C % 8 == 0) and the scalar ones (C = 12):
    forward within bf16 rounding of the fp64 mean, backward exactly bf16(dy / HW) (fp32 divide, RNE)."""
    torch.manual_seed(5)
    x = rb(torch.randn(3, 7, 7, C))
    a = ops.avgpool_fwd(x.to(cuda, torch.bfloat16)).cpu().double()
    ref = x.double().mean((1, 2))
    assert (a - ref).abs().max().item() <= 2 ** -7 * ref.abs().max().item() + 1e-6
    dy = rb(torch.randn(3, C))
    da = ops.avgpool_bwd(dy.to(cuda, torch.bfloat16), [3, 7, 7, C]).cpu()
    want = (dy.float() / 49.0).to(torch.bfloat16)[:, None, None, :].expand(3, 7, 7, C)
    assert torch.equal(da, want)
