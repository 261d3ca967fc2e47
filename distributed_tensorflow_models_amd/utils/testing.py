"""Multi-process test harness: run ``fn(rank, world, *args)`` in ``world`` spawned processes over
a gloo process group on 127.0.0.1 (CPU), collecting each rank's return value."""
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, fn, world, port, outdir, args, backend="gloo"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DTM_RUN_ID="t%d" % port)
    # the CPU share, not the machine: os.cpu_count() on a GPU box is the whole host (hundreds), and that many OpenMP
    # threads per rank under a 16-CPU quota turn every CPU op (a model's weight init) into minutes of spin-waiting
    cpus = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0)) or 2
    torch.set_num_threads(max(1, cpus // world))
    from ..parallel import process_group as pg
    if backend == "nccl":
        pg.rccl_env(0, timing=True)  # per-collective durations (bucket_ms)
    pg.init(backend=backend, timeout_s=120, force=backend == "nccl")
    ok = False
    try:
        out = fn(rank, world, *args)
        torch.save(out, os.path.join(outdir, "r%d.pt" % rank))
        ok = True
    finally:
        # a failed rank leaves at once (no barrier): the others' pending collectives then fail instead of waiting
        # for the gloo timeout, and start_processes reports the first error
        if ok:
            pg.barrier()
        pg.destroy()


def run_workers(fn, world, *args, backend="gloo"):
    """Returns [result_rank0, result_rank1, ...]; raises if any rank fails.  backend "nccl" (RCCL): one rank per GPU
    (RCCL refuses two ranks on one device)."""
    port = free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_entry, args=(fn, world, port, d, args, backend), nprocs=world, join=True,
                           start_method="spawn")
        return [torch.load(os.path.join(d, "r%d.pt" % r), weights_only=True) for r in range(world)]
