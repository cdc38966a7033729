"""Spawn helpers for multi-process tests (gloo on 127.0.0.1)."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _detach(x):
    """Tensors cannot outlive the child through an mp.Queue: ship numpy copies."""
    import torch

    if isinstance(x, torch.Tensor):
        return ("__tensor__", x.detach().cpu().numpy().copy())
    if isinstance(x, (list, tuple)):
        return type(x)(_detach(v) for v in x)
    if isinstance(x, dict):
        return {k: _detach(v) for k, v in x.items()}
    return x


def _attach(x):
    import torch

    if isinstance(x, tuple) and len(x) == 2 and isinstance(x[0], str) and x[0] == "__tensor__":
        return torch.from_numpy(x[1])
    if isinstance(x, (list, tuple)):
        return type(x)(_attach(v) for v in x)
    if isinstance(x, dict):
        return {k: _attach(v) for k, v in x.items()}
    return x


def _entry(rank, world, port, fn, args, q, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    try:
        import torch.distributed as dist

        if backend == "nccl":
            import torch

            torch.cuda.set_device(0)
        dist.init_process_group(backend, rank=rank, world_size=world)
        out = _detach(fn(rank, world, *args))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", out))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


def run_ranks(fn, world: int = 2, args=(), timeout: float = 240.0, backend: str = "gloo"):
    """Run fn(rank, world, *args) in `world` spawned processes; return {rank: result}."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q, backend)) for r in range(world)]
    for p in ps:
        p.start()
    res, errs = {}, []
    try:
        for _ in range(world):
            rank, st, out = q.get(timeout=timeout)
            if st == "ok":
                res[rank] = _attach(out)
            else:
                errs.append(f"rank {rank}:\n{out}")
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if errs:
        raise AssertionError("\n".join(errs))
    return res
