"""Per-phase clocks of the conv12, head and conv2-dgrad kernels from a TFD_STAMP build (TFD_NATIVE_LIB=..._C_stamp.so):
median over blocks of the s_memtime deltas between consecutive stamps, after warm replays."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from tensorflow_distributed_amd import _native  # noqa: E402
from tensorflow_distributed_amd.models import mnist_cnn as M  # noqa: E402

_native.require()
dev = torch.device("cuda", 0)
B = 128
eng = torch.classes.tfd.MnistEngine(B, 0, 0.75, 1, 0)
eng.set_adam(0.01, 0.9, 0.999, 1e-8)
dbg = torch.zeros(10 * B * 8, dtype=torch.int64, device=dev)
eng.set_debug_buffer(dbg)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    data = torch.rand(55000, 784, device=dev)
    labels = torch.randint(0, 10, (55000,), device=dev, dtype=torch.int32)
    perm = torch.randperm(55000, device=dev).to(torch.int32)
    eng.params().copy_(M.flat_from_dict(M.init_params(1)).to(dev))
    eng.sync_shadow()
    eng.set_dataset(data, labels, perm)
    eng.set_input_mode(1)
    eng.train_step()
    eng.capture_train_steps("g", 20)
    eng.replay("g", 50)
torch.cuda.synchronize()
MODE = sys.argv[1] if len(sys.argv) > 1 else "train"
if MODE == "fwd_after_idle":  # conv12 + head with no write-heavy kernel before them
    import time
    time.sleep(0.01)
    with torch.cuda.stream(s):
        eng.forward(True)
    torch.cuda.synchronize()
elif MODE == "fwd_after_fill":  # conv12 + head right after a 45 MB write-only fill
    junk = torch.empty(45 * 2**20 // 4, device=dev)
    with torch.cuda.stream(s):
        for _ in range(3):
            junk.fill_(1.0)
            eng.forward(True)
    torch.cuda.synchronize()
print("mode", MODE)
d = dbg.view(-1, 8).cpu()
h = d[4 * B:]
w4 = d[1:4 * B:2]
d = d[0:4 * B:2]
names = ["issue loads", "zero+stage+2 barriers", "conv1", "W2 store+copyout+barrier", "conv2 loop", "epilogue"]
base = d[:, 0].min()
print("block span (cycles): median", (d[:, 6] - d[:, 0]).median().item(), "max", (d[:, 6] - d[:, 0]).max().item(),
      "start spread", (d[:, 0] - base).max().item())
for k in range(6):
    dd = d[:, k + 1] - d[:, k]
    print(f"{names[k]:28s} median {dd.median().item():8d}  p90 {dd.float().quantile(0.9).item():8.0f}")
wn = ["w4 issue loads", "w4 vmcnt(0) wait", "w4 zero LDS", "w4 barrier 1", "w4 x/W1 LDS stores", "w4 barrier 2"]
for k in range(6):
    dd = w4[:, k + 1] - w4[:, k]
    print(f"{wn[k]:28s} median {dd.median().item():8d}  p90 {dd.float().quantile(0.9).item():8.0f}")
print("wave4 start - wave0 start: median", (w4[:, 0] - d[:, 0]).median().item())
if (d[:, 7] > 0).all():  # TFD_EXP_C12REP=2: conv1 section twice (second pass with a warm I-cache)
    print("conv1 rep0", (d[:, 7] - d[:, 2]).median().item(), "rep1", (d[:, 3] - d[:, 7]).median().item())
hn = ["bias+slab loads", "dropout+wout+lp", "reduce+softmax", "dl/dh+stores"]
print("head block span: median", (h[:, 4] - h[:, 0]).median().item())
for k in range(4):
    dd = h[:, k + 1] - h[:, k]
    print(f"head {hn[k]:23s} median {dd.median().item():8d}  p90 {dd.float().quantile(0.9).item():8.0f}")

dg = dbg.view(-1, 8).cpu()[5 * B:5 * B + 2 * B]
if (dg[:, 7] > 0).all():
    dn = ["issue staging loads", "image LDS stores + barrier", "K loop (MFMA)", "barrier + tail LDS zeroing",
          "gsl / x / argmax + barrier", "conv1-wgrad accumulate", "partial reduce + slab store"]
    print("dgrad block span: median", (dg[:, 7] - dg[:, 0]).median().item())
    for k in range(7):
        dd = dg[:, k + 1] - dg[:, k]
        print(f"dgrad {dn[k]:28s} median {dd.median().item():8d}  p90 {dd.float().quantile(0.9).item():8.0f}")

wg = dbg.view(-1, 8).cpu()[7 * B:9 * B]
if (wg[:, 7] > 0).all():
    wn2 = ["zero + image 0 loads + LDS stores + barrier", "image 0 MFMAs", "image 1 LDS stores + barrier",
           "image 1 MFMAs"]
    print("wgrad block span: median", (wg[:, 7] - wg[:, 0]).median().item())
    for k in range(4):
        dd = wg[:, k + 1] - wg[:, k]
        print(f"wgrad {wn2[k]:44s} median {dd.median().item():8d}  p90 {dd.float().quantile(0.9).item():8.0f}")
    dd = wg[:, 7] - wg[:, 4]
    print(f"wgrad {'slab epilogue (+ bias sum)':44s} median {dd.median().item():8d}")
