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
    for n in (7 * 4 * 8 * 64, 7 * 7 * 8 * 64, 1001):
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
    print(f"# {bad} failing case(s)")
    return 0  # a finding, not a failure: the table above is the result


if __name__ == "__main__":
    sys.exit(main())
