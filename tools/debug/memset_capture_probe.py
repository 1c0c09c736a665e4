"""Does a hipMemsetAsync issued into a stream capture clear its buffer on every graph replay?
(native side: csrc/runtime/graph_probe.cpp.)

Pattern per graph:  +1 (atomics)  ->  clear  ->  +1 (atomics);  the buffer starts at 5.0, so after
any number of replays every element is 1.0 exactly when the clear ran on each replay.

Cases: clear = hipMemsetAsync / hipMemsetD32Async / a fill kernel; capture mode global /
thread-local / relaxed (native capture); buffer 256-B aligned or a 4-B aligned view of a flat
buffer (the ResNet stem gradient's situation); sizes of the stem's width-paired filter gradient
(7 x 4 x 8 x 64) and its padded one (7 x 7 x 8 x 64) and an odd 1001. Then the same sequence
captured by torch.cuda.graph (the path the ResNet wgrad took), memset issued on torch's capture
stream.

    python tools/debug/memset_capture_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from tensorflow_distributed_amd import _native  # noqa: E402

CLEAR = {0: "hipMemsetAsync", 1: "hipMemsetD32Async", 2: "fill kernel"}
MODE = {0: "global", 1: "thread-local", 2: "relaxed"}


def buffers(n, dev):
    flat = torch.empty(n + 64, device=dev)
    return {"aligned": torch.empty(n, device=dev), "view+4B": flat[1:1 + n], "view+8B": flat[2:2 + n]}


def main():
    _native.require()
    dev = torch.device("cuda", 0)
    ops = torch.ops.tfd
    bad = 0
    print("native capture: nodes kernel/memset/other | memset dst-off elem width height deps | "
          "elements != 1.0 after 3 replays, buf[0], buf[-1]")
    for n in (7 * 4 * 8 * 64, 7 * 7 * 8 * 64, 1001, 8192, 16384, 65536):
        for bname, buf in buffers(n, dev).items():
            for clear in (0, 1, 2):
                for mode in (0, 1, 2):
                    i = ops.memset_capture_probe(buf, 3, clear, mode).tolist()
                    ok = i[10] == 0
                    bad += not ok
                    print(f"n={n:6d} {bname:8s} {CLEAR[clear]:18s} {MODE[mode]:12s} nodes {i[0]} "
                          f"{i[1]}/{i[2]}/{i[3]} | memset off {i[4]} elem {i[5]} w {i[6]} h {i[7]} deps {i[9]} | "
                          f"bad {i[10]} first {i[11] / 1000:.1f} last {i[12] / 1000:.1f} {'OK' if ok else 'FAIL'}",
                          flush=True)
    print("native capture, the clear as the graph's ROOT node (clear -> +1; expect 1.0 after every replay):")
    for n in (8192, 7 * 4 * 8 * 64, 1001, 65536):
        for bname, buf in buffers(n, dev).items():
            for clear in (0, 1, 2):
                i = ops.memset_capture_probe(buf, 3, clear, 4).tolist()
                # the +1-only replays leave every element at 1.0 when the clear ran on each
                ok = i[10] == 0
                bad += not ok
                print(f"n={n:6d} {bname:8s} {CLEAR[clear]:18s} root   nodes {i[0]} {i[1]}/{i[2]}/{i[3]} | memset "
                      f"elem {i[5]} w {i[6]} deps {i[9]} | bad {i[10]} first {i[11] / 1000:.1f} last {i[12] / 1000:.1f} "
                      f"{'OK' if ok else 'FAIL'}", flush=True)
    print("torch.cuda.graph capture (memset on torch's capture stream):")
    for n in (7 * 4 * 8 * 64, 1001):
        for bname, buf in buffers(n, dev).items():
            for clear in ("memset", "fill_"):
                buf.fill_(5.0)
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                with torch.cuda.stream(s):
                    with torch.cuda.graph(g, stream=s):
                        ops.probe_atomic_add_one(buf)
                        if clear == "memset":
                            ops.memset_zero_async(buf)
                        else:
                            buf.zero_()
                        ops.probe_atomic_add_one(buf)
                for _ in range(3):
                    g.replay()
                torch.cuda.synchronize()
                nb = int((buf != 1.0).sum().item())
                bad += nb != 0
                print(f"n={n:6d} {bname:8s} {clear:8s} bad {nb} first {buf[0].item():.1f} last {buf[-1].item():.1f} "
                      f"{'OK' if nb == 0 else 'FAIL'}", flush=True)
                del g
    print("split-K weight gradient in a torch.cuda.graph (tests/test_conv_ops_gpu.py "
          "test_captured_split_k_wgrad_zeroes_its_accumulator_on_every_replay), per clear mode:")
    for clear in (0, 1):
        old = ops.conv_wgrad_clear_mode(clear)
        try:
            torch.manual_seed(4)
            x = torch.randn(16, 14, 14, 64).to(torch.bfloat16).to(dev)
            dy = torch.randn(16, 14, 14, 128).to(torch.bfloat16).to(dev)
            ref = torch.zeros(1, 1, 64, 128, device=dev)
            ops.conv2d_wgrad(x, dy, ref, 1, 0)
            dw = torch.full((1, 1, 64, 128), 7.0, device=dev)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                ops.conv2d_wgrad(x, dy, dw, 1, 0)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            eager_ok = torch.allclose(dw, ref, rtol=1e-5, atol=1e-4)
            g = torch.cuda.CUDAGraph(keep_graph=True)
            with torch.cuda.graph(g):
                ops.conv2d_wgrad(x, dy, dw, 1, 0)
            rows = ops.graph_memset_nodes(int(g.raw_cuda_graph())).tolist()
            print(f"  clear {clear}: eager {'OK' if eager_ok else 'WRONG'}; graph nodes {rows[0][0]} "
                  f"(kernels {rows[0][1]}), memset nodes {len(rows) - 1}", flush=True)
            for r in rows[1:]:
                print(f"    memset dst {r[0]:#x} (dw {dw.data_ptr():#x}) elem {r[1]} width {r[2]} height {r[3]} "
                      f"value {r[4]} deps in {r[5]} out {r[6]}", flush=True)
            for i in range(3):
                g.replay()
                torch.cuda.synchronize()
                d = (dw - ref).abs()
                nb = int((d > 1e-3 * ref.abs().max()).sum().item())
                bad += nb != 0
                print(f"    replay {i}: {nb} / {dw.numel()} elements off, max |d| {d.max().item():.3e}", flush=True)
            del g
        finally:
            ops.conv_wgrad_clear_mode(old)
    print(f"# {bad} failing case(s)")
    return 0  # a finding, not a failure: the table above is the result


if __name__ == "__main__":
    sys.exit(main())
