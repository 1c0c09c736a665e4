"""Debug: per-block forward agreement of the native ResNet vs a PyTorch fp32 reference."""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
import torch.nn.functional as F
from tensorflow_distributed_amd.models.resnet import ResNet, _MaxPool

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = ResNet(50, num_classes=16, device=dev, seed=1, width=16, zero_init_residual=False)
x = torch.randn(4, 64, 64, 3)
from tensorflow_distributed_amd import _native; _native.require(); ops = torch.ops.tfd
def rb(t): return t.to(torch.bfloat16).float()
def W(L): return m.fp.w(L.name).float().cpu().permute(3, 2, 0, 1)
def conv(h, L): return rb(F.conv2d(h, W(L), stride=L.stride, padding=L.pad))
def bn(y, L, relu=True, res=None):
    z = F.batch_norm(y, None, None, m.fp.p(L.name + "/gamma").cpu(), m.fp.p(L.name + "/beta").cpu(), training=True, eps=1e-5)
    if res is not None: z = z + res
    return rb(torch.relu(z) if relu else z)
def cos(a, b): return F.cosine_similarity(a.flatten().float(), b.flatten().float(), dim=0).item()

with torch.no_grad():
    xn = ops.pad_channels(x.to(dev), 8)
    hn = m.stem_bn(m.stem(xn))
    hn = _MaxPool.apply(hn, 3, 2, 1)
    h = F.pad(rb(x).permute(0, 3, 1, 2), (0, 0, 0, 0, 0, 5))
    h = bn(conv(h, m.stem), m.stem_bn)
    h = F.max_pool2d(h, 3, 2, 1)
    print("stem", cos(hn.cpu().permute(0, 3, 1, 2), h))
    for i, blk in enumerate(m.blocks):
        # native, step by step
        scn = hn
        if "cd" in blk:
            yd = blk["cd"](hn); scn = blk["bd"](yd, relu=False)
        t1n = blk["c1"](hn); a1n = blk["b1"](t1n)
        t2n = blk["c2"](a1n); a2n = blk["b2"](t2n)
        t3n = blk["c3"](a2n); hn2 = blk["b3"](t3n, relu=True, res=scn)
        # reference from the NATIVE input of this block (isolate per-block error)
        hin = hn.cpu().float().permute(0, 3, 1, 2)
        sc = hin
        if "cd" in blk:
            ydr = conv(hin, blk["cd"]); sc = bn(ydr, blk["bd"], relu=False)
            print(f"  blk{i} downsample conv", cos(yd.cpu().permute(0, 3, 1, 2), ydr), "bn", cos(scn.cpu().permute(0,3,1,2), sc))
        t1 = conv(hin, blk["c1"]); a1 = bn(t1, blk["b1"])
        t2 = conv(a1n.cpu().float().permute(0,3,1,2), blk["c2"]); a2 = bn(t2, blk["b2"])
        t3 = conv(a2n.cpu().float().permute(0,3,1,2), blk["c3"])
        out = bn(t3n.cpu().float().permute(0,3,1,2), blk["b3"], True, scn.cpu().float().permute(0,3,1,2))
        print(f"blk{i} c1 {cos(t1n.cpu().permute(0,3,1,2), t1):.5f} b1 {cos(a1n.cpu().permute(0,3,1,2), a1):.5f} "
              f"c2 {cos(t2n.cpu().permute(0,3,1,2), t2):.5f} c3 {cos(t3n.cpu().permute(0,3,1,2), t3):.5f} out {cos(hn2.cpu().permute(0,3,1,2), out):.5f}"
              f" shape {tuple(hn2.shape)} c2cfg st={blk['c2'].stride}")
        hn = hn2

print("---- backward per block ----")
class RB(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x): return x.to(torch.bfloat16).float()
    @staticmethod
    def backward(ctx, g): return g.to(torch.bfloat16).float()
def convg(h, L, Wt): return RB.apply(F.conv2d(h, Wt, stride=L.stride, padding=L.pad))
def bng(y, L, g, b, relu=True, res=None):
    z = F.batch_norm(y, None, None, g, b, training=True, eps=1e-5)
    if res is not None: z = z + res
    return RB.apply(torch.relu(z) if relu else z)

for bi in (0, 1, 3, 13):
    blk = m.blocks[bi]
    cin = blk["c1"].model.fp.by_name[blk["c1"].name].shape[2]
    hw = {0: 16, 1: 16, 3: 16, 13: 4}[bi]
    xin = rb(torch.randn(4, hw, hw, cin))
    gout_shape = None
    # native
    xn_ = xin.to(dev, torch.bfloat16).requires_grad_(True)
    scn = xn_
    if "cd" in blk: scn = blk["bd"](blk["cd"](xn_), relu=False)
    a = blk["b1"](blk["c1"](xn_)); a = blk["b2"](blk["c2"](a)); outn = blk["b3"](blk["c3"](a), relu=True, res=scn)
    g = rb(torch.randn(outn.shape))
    m.fp.grad.zero_()
    outn.backward(g.to(dev, torch.bfloat16))
    torch.cuda.synchronize()
    # reference
    xr = xin.permute(0, 3, 1, 2).clone().requires_grad_(True)
    Ws = {k: W(L).clone().requires_grad_(True) for k, L in blk.items() if k.startswith("c")}
    Gs = {k: (m.fp.p(L.name + "/gamma").cpu().clone().requires_grad_(True), m.fp.p(L.name + "/beta").cpu().clone().requires_grad_(True)) for k, L in blk.items() if k.startswith("b")}
    sc = xr
    if "cd" in blk: sc = bng(convg(xr, blk["cd"], Ws["cd"]), blk["bd"], *Gs["bd"], relu=False)
    t = bng(convg(xr, blk["c1"], Ws["c1"]), blk["b1"], *Gs["b1"])
    t = bng(convg(t, blk["c2"], Ws["c2"]), blk["b2"], *Gs["b2"])
    outr = bng(convg(t, blk["c3"], Ws["c3"]), blk["b3"], *Gs["b3"], True, sc)
    outr.backward(g.permute(0, 3, 1, 2))
    res = [f"out {cos(outn.detach().cpu().permute(0,3,1,2), outr):.4f}", f"dx {cos(xn_.grad.cpu().permute(0,3,1,2), xr.grad):.4f}"]
    for k, L in blk.items():
        if k.startswith("c"):
            res.append(f"{k} {cos(m.fp.g(L.name).cpu(), Ws[k].grad.permute(2,3,1,0)):.4f}")
        else:
            res.append(f"{k}g {cos(m.fp.g(L.name + '/gamma').cpu(), Gs[k][0].grad):.4f}")
    print(f"blk{bi}", " ".join(res))
