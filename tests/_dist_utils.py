"""Spawn helpers for multi-process tests (gloo on CPU, 127.0.0.1 rendezvous)."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(rank, world, port, fn, args, backend, errq):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["RANK"] = str(rank)
    os.environ["WORLD_SIZE"] = str(world)
    os.environ["LOCAL_RANK"] = str(rank)
    try:
        dist.init_process_group(backend, rank=rank, world_size=world)
        fn(rank, world, *args)
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        errq.put((rank, traceback.format_exc()))
        raise


def run_multiprocess(fn, world=2, args=(), backend="gloo", timeout=240):
    ctx = mp.get_context("spawn")
    errq = ctx.SimpleQueue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, backend, errq)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    for p in procs:
        if p.is_alive():
            p.kill()
            errs.append((-1, "timeout"))
        elif p.exitcode != 0 and not errs:
            errs.append((-1, f"exit code {p.exitcode}"))
    if errs:
        raise AssertionError("\n".join(f"rank {r}: {e}" for r, e in errs))
