"""Process-group bring-up (replaces the reference's gRPC ClusterSpec/Server).

One process per MI355X: ``LOCAL_RANK`` -> device; ``backend='nccl'`` is RCCL over xGMI on ROCm,
``gloo`` for CPU runs and tests.  Rendezvous through the c10d TCPStore on rank 0 (127.0.0.1 by
default for single-node runs).
"""
import datetime
import os

import torch
import torch.distributed as dist


def rccl_env(channels=0, timing=False):
    """RCCL knobs that must be set before the communicator exists.

    channels > 0 pins the number of RCCL channels (NCCL_MIN/MAX_NCHANNELS): each channel is one ring
    over the xGMI links driven by its own workgroup, so the count trades all-reduce bandwidth against
    CUs taken from the overlapped backward kernels.  timing: per-collective start/end events
    (TORCH_NCCL_ENABLE_TIMING) so BSPDataParallel.bucket_ms() can report every bucket's duration."""
    if channels and channels > 0:
        os.environ["NCCL_MIN_NCHANNELS"] = str(int(channels))
        os.environ["NCCL_MAX_NCHANNELS"] = str(int(channels))
    if timing:
        os.environ["TORCH_NCCL_ENABLE_TIMING"] = "1"


def nccl_options(high_priority=True):
    """ProcessGroupNCCL options: the collectives' internal stream at high priority, so bucket
    all-reduces issued mid-backward are scheduled ahead of the compute stream's queued kernels."""
    try:
        from torch.distributed import ProcessGroupNCCL
        return ProcessGroupNCCL.Options(is_high_priority_stream=bool(high_priority))
    except Exception:  # (a build without the NCCL/RCCL backend)
        return None


def init(rank=None, world_size=None, master_addr=None, master_port=None, backend=None, timeout_s=1800,
         high_priority=True, force=False):
    """force: create the process group even for one rank (tests of the RCCL path on a one-GPU box)."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    rank = int(os.environ.get("RANK", 0) if rank is None else rank)
    world_size = int(os.environ.get("WORLD_SIZE", 1) if world_size is None else world_size)
    if world_size <= 1 and not force:
        return 0, 1
    os.environ.setdefault("MASTER_ADDR", master_addr or "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(master_port or 29500))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    kw = {}
    if backend == "nccl":
        local = int(os.environ.get("LOCAL_RANK", rank % max(torch.cuda.device_count(), 1)))
        torch.cuda.set_device(local)
        kw["device_id"] = torch.device("cuda", local)
        opts = nccl_options(high_priority)
        if opts is not None:
            kw["pg_options"] = opts
    dist.init_process_group(backend, rank=rank, world_size=world_size,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rank, world_size


def rank():
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def is_chief():
    return rank() == 0


def barrier():
    if world_size() > 1:
        dist.barrier()


def broadcast_tensors(tensors, src=0):
    """Chief -> all (initial parameters / restored checkpoint), coalesced per dtype+device."""
    if world_size() <= 1:
        return
    groups = {}
    for t in tensors:
        groups.setdefault((t.dtype, t.device), []).append(t)
    for (_dt, _dev), ts in groups.items():
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        dist.broadcast(flat, src)
        off = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view_as(t))
                off += n


def device():
    if torch.cuda.is_available():
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)))
    return torch.device("cpu")


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
