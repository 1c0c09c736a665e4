"""Helpers to run a function in N gloo processes on 127.0.0.1 (CPU distributed tests)."""
import os
import traceback

import torch.multiprocessing as mp


def free_port():
    from tensorflow_distributed_amd.parallel.spawn import free_port as _free_port  # below the ephemeral range

    return _free_port()


def _to_plain(x):
    """Tensors -> numpy (plain pickles): avoids torch's fd-passing, which races with child exit."""
    import torch

    if isinstance(x, torch.Tensor):
        return ("__tensor__", x.detach().cpu().numpy())
    if isinstance(x, (list, tuple)):
        return type(x)(_to_plain(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_plain(v) for k, v in x.items()}
    return x


def _from_plain(x):
    import torch

    if isinstance(x, tuple) and len(x) == 2 and isinstance(x[0], str) and x[0] == "__tensor__":
        return torch.from_numpy(x[1])
    if isinstance(x, (list, tuple)):
        return type(x)(_from_plain(v) for v in x)
    if isinstance(x, dict):
        return {k: _from_plain(v) for k, v in x.items()}
    return x


def _entry(rank, world, port, fn, args, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        import torch

        if world > 4:  # many ranks share the host's cores (fewer keep torch's default: the tests that
            # compare a worker's result bit for bit with the parent's use the same thread count)
            torch.set_num_threads(max(1, (os.cpu_count() or 8) // world))
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        out = fn(rank, world, *args)
        q.put((rank, "ok", _to_plain(out)))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_ranks(fn, world, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, status, out = q.get(timeout=timeout)
            if status != "ok":
                raise AssertionError(f"rank {rank} failed:\n{out}")
            res[rank] = _from_plain(out)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    return [res[r] for r in range(world)]
