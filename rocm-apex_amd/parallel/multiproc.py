"""One-process-per-GPU launcher (reference apex/parallel/multiproc.py:1-35).

``python -m apex.parallel.multiproc train.py args...`` spawns ``train.py`` once per visible GPU
with ``--world-size`` / ``--rank`` appended and RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* exported
(127.0.0.1 rendezvous); ranks >= 1 log to ``GPU_<rank>.log``.  ``torch.distributed.run`` is the
recommended launcher; this is kept for parity."""
import os
import subprocess
import sys

import torch


def docstring_hack():
    """Multiproc file which will launch a set of processes locally for multi-gpu usage."""
    pass


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    world_size = torch.cuda.device_count() or 1
    argv.append("--world-size={}".format(world_size))
    workers = []
    env0 = dict(os.environ)
    env0.setdefault("MASTER_ADDR", "127.0.0.1")
    env0.setdefault("MASTER_PORT", "29500")
    for i in range(world_size):
        env = dict(env0, RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(world_size))
        args = argv + ["--rank={}".format(i)]
        stdout = None if i == 0 else open("GPU_" + str(i) + ".log", "w")
        workers.append(subprocess.Popen([sys.executable] + args, stdout=stdout, env=env))
    rc = 0
    for p in workers:
        rc = p.wait() or rc
    return rc


if __name__ == "__main__":
    sys.exit(main())
