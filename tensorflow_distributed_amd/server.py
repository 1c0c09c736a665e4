"""Standalone coordination server for ``--existing_servers=True`` (reference
``/root/reference/mnist_python_m.py:76-80, 268-273``: attach to servers launched outside the
training scripts).

Hosts the rendezvous ``TCPStore`` at ``--address`` (the first ``--ps_hosts`` entry) and exits once
``--num_workers`` workers have signalled completion (or never, with ``--forever``).

    python -m tensorflow_distributed_amd.server --address 127.0.0.1:2222 --num_workers 2
"""
from __future__ import annotations

import argparse
import datetime
import sys
import time

import torch.distributed as dist

from .parallel.cluster import split_hostport


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--address", required=True)
    ap.add_argument("--num_workers", type=int, default=1)
    ap.add_argument("--forever", action="store_true")
    ap.add_argument("--timeout", type=float, default=3600.0)
    a = ap.parse_args(argv)
    host, port = split_hostport(a.address)
    store = dist.TCPStore(host, port, is_master=True, timeout=datetime.timedelta(seconds=a.timeout),
                          wait_for_workers=False)
    print(f"coordination server listening on {host}:{port}", flush=True)
    t0 = time.time()
    while a.forever or int(store.add("tfd/workers_done", 0)) < a.num_workers:
        if time.time() - t0 > a.timeout:
            print("coordination server: timeout", flush=True)
            return 1
        time.sleep(0.2)
    time.sleep(1.0)  # let the last clients finish their final store operations
    return 0


if __name__ == "__main__":
    sys.exit(main())
