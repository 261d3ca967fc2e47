"""ASP: asynchronous parameter-store data parallelism (reference vgg/cifar10_vgg_asp.py,
inception/imagenet_inception_asp.py).

The reference keeps variables on PS tasks and every worker runs ``apply_gradients`` on them
independently (Hogwild at op granularity).  MI355X-native redesign: the parameter store is a set
of *owner shards* (round-robin over tensors, like ``replica_device_setter``) that every worker
maps directly:

  * GPU mode: owner k's shard lives in GPU k's HBM; the other ranks open it through HIP IPC
    handles (exchanged via the c10d TCPStore) and read / update it in place over xGMI peer
    access - no owner-side server loop, no message matching;
  * host mode (CPU runs, tests, or when peer IPC is unavailable): shards live in a file-backed
    shared mapping under /dev/shm (``torch.from_file(shared=True)``) - exactly the reference's
    "variables on the PS CPU" placement.

Per worker step: pull (copy every shard into the local replica) -> forward/backward on local
weights -> push (apply this worker's gradient to the owner shard with the TF update rule; no
averaging, no barrier).  ``global_step`` is an atomic counter in the TCPStore, incremented once
per worker step (TF ASP semantics).  Concurrent pushes to one shard race exactly as Hogwild does.
"""
import datetime
import os
import pickle
import time

import torch
import torch.distributed as dist

from ..ops import _lib
from . import process_group as pg

STORE_PREFIX = "dtm_asp"


def owner_map(params, world):
    """Round-robin tensor -> owner rank (replica_device_setter semantics, C14)."""
    return {i: i % world for i in range(len(params))}


def _enable_peer_access(me, peers):
    """hipDeviceEnablePeerAccess(peer) from device ``me``'s context for every peer (already-enabled is fine)."""
    import ctypes
    try:
        hip = ctypes.CDLL("libamdhip64.so")
    except OSError:
        return False
    if hip.hipSetDevice(ctypes.c_int(me)) != 0:
        return False
    for d in peers:
        rc = hip.hipDeviceEnablePeerAccess(ctypes.c_int(d), ctypes.c_uint(0))
        if rc not in (0, 704):  # hipSuccess, hipErrorPeerAccessAlreadyEnabled
            return False
    return True


class ParamStore:
    def __init__(self, params, optimizer="sgd", lr=0.01, momentum=0.9, rho=0.9, epsilon=1e-10, mode=None,
                 store=None, run_id="0", weight_decays=None, buffers=()):
        self.params = [p for p in params if p.requires_grad]
        # non-trainable state every worker's forward updates in place (BN moving statistics): in the
        # reference they are PS variables too, written by each worker's AssignMovingAvg ops
        # (inception/imagenet_inception_asp.py:119-145 runs the UPDATE_OPS with the train op).  They
        # live in one flat region of owner 0's shard; a worker pulls them with the parameters and
        # pushes the delta its forward made (shared += local - pulled), Hogwild-style.
        from .bsp import flatten_tensors
        self.buffers = [b for b in buffers]
        self._buf_local = flatten_tensors(self.buffers) if self.buffers else None
        self._buf_snap = self._buf_local.clone() if self._buf_local is not None else None
        self.rank, self.world = pg.rank(), pg.world_size()
        self.owner = owner_map(self.params, self.world)
        self.kind, self.lr, self.mu, self.rho, self.eps = optimizer, lr, momentum, rho, epsilon
        self.wd = [float(getattr(p, "weight_decay", 0.0)) for p in self.params] if weight_decays is None \
            else list(weight_decays)
        self.store = store if store is not None else _default_store()
        self.run_id = run_id
        gpu = self.params[0].is_cuda
        self.mode = mode or ("ipc" if gpu else "shm")
        if self.mode == "ipc" and self.world > 1:
            self.mode = self._negotiate_ipc()
        self.shards = {}   # param index -> dict(param=..., s1=..., s2=...) views into owner memory
        self._build()

    # -----------------------------------------------------------------------------------------
    def _build(self):
        nslots = {"sgd": 0, "momentum": 1, "rmsprop": 2}[self.kind]
        # one flat buffer per owner: [params | slot1 | slot2]
        per_owner = {}
        for i, p in enumerate(self.params):
            per_owner.setdefault(self.owner[i], []).append(i)
        # within an owner: the tensors with a bf16 compute copy (conv / FC weights) first, so the pull
        # refreshes those copies with ONE cast over a prefix of the owner's region
        for k in per_owner:
            per_owner[k].sort(key=lambda i: (self._bf16(self.params[i]) is None, i))
        self.owned = {k: list(v) for k, v in per_owner.items()}
        self.layout = {}
        for k, idxs in per_owner.items():
            off = 0
            for i in idxs:
                self.layout[i] = (k, off)
                off += self.params[i].numel()
            per_owner[k] = (idxs, off)
        self.flat = {}
        nbuf = self._buf_local.numel() if self._buf_local is not None else 0
        self._nslot = {k: n for k, (idxs, n) in per_owner.items()}
        for k, (idxs, n) in per_owner.items():
            total = n * (1 + nslots) + (nbuf if k == 0 else 0)
            self.flat[k] = self._open_flat(k, total, init_from=(idxs, n) if k == self.rank or self.mode == "shm"
                                           else None)
        if self.mode == "shm" and self.rank == 0:
            pass
        pg.barrier()
        for i, p in enumerate(self.params):
            k, off = self.layout[i]
            n_owner = per_owner[k][1]
            buf = self.flat[k]
            sh = {"param": buf[off:off + p.numel()].view(p.shape)}
            if nslots >= 1:
                sh["s1"] = buf[n_owner + off:n_owner + off + p.numel()].view(p.shape)
            if nslots >= 2:
                sh["s2"] = buf[2 * n_owner + off:2 * n_owner + off + p.numel()].view(p.shape)
            self.shards[i] = sh
        if nbuf:
            base = self._nslot[0] * (1 + nslots)
            self.buf_shard = self.flat[0][base:base + nbuf]
        self._flatten_local()

    @staticmethod
    def _bf16(p):
        w16 = getattr(p, "bf16", None)
        return w16 if (w16 is not None and w16.dtype == torch.bfloat16 and w16.shape == p.shape) else None

    def _flatten_local(self):
        """Re-home the local replica in the owner shards' layout (``flatten_tensors`` keeps every
        parameter object; only its storage moves): per owner one fp32 region mirroring the shard, and
        one bf16 region for the compute copies of its leading weights.  The pull is then 2 launches per
        owner instead of 2 per tensor (ResNet-50: 322)."""
        from .bsp import flatten_tensors
        self._local, self._local16 = {}, {}
        for k, idxs in self.owned.items():
            ps = [self.params[i] for i in idxs]
            if len({(p.dtype, p.device) for p in ps}) != 1:
                self._local = None
                return
            self._local[k] = flatten_tensors(ps)
            w16 = [self._bf16(p) for p in ps if self._bf16(p) is not None]
            self._local16[k] = flatten_tensors(w16) if w16 else None

    def _negotiate_ipc(self):
        """Owner shards are written from other GPUs over xGMI: the ranks exchange their device indices
        through the store, every rank checks (and enables, from its own device) peer access to the OTHER
        ranks' devices only; if any pair cannot, ALL ranks fall back to the host (/dev/shm) store - the
        decision is collective, since the owners' allocations depend on it.  Nothing is allocated on a peer
        device (no extra HIP context / HBM there)."""
        me = self.params[0].device.index
        key = "%s/%s/p2p" % (STORE_PREFIX, self.run_id)
        self.store.set("%s_dev%d" % (key, self.rank), str(me))
        self.store.wait(["%s_dev%d" % (key, r) for r in range(self.world)], datetime.timedelta(seconds=300))
        peers = sorted({int(self.store.get("%s_dev%d" % (key, r))) for r in range(self.world)} - {me})
        ok = all(torch.cuda.can_device_access_peer(me, d) for d in peers)
        if ok and peers:
            ok = _enable_peer_access(me, peers)
        self.peers = peers
        self.store.add(key + "_n", 1)
        if not ok:
            self.store.add(key + "_bad", 1)
        t0 = time.time()
        while int(self.store.add(key + "_n", 0)) < self.world:
            if time.time() - t0 > 300:
                raise TimeoutError("ASP peer-access negotiation")
            time.sleep(0.005)
        if int(self.store.add(key + "_bad", 0)):
            import logging
            logging.getLogger(__name__).warning(
                "ASP: peer access between the ranks' GPUs is unavailable; using the host (/dev/shm) store")
            return "shm"
        return "ipc"

    def _open_flat(self, k, total, init_from):
        if self.mode == "shm":
            path = "/dev/shm/%s_%s_owner%d" % (STORE_PREFIX, self.run_id, k)
            if self.rank == k:
                buf = torch.from_file(path, shared=True, size=total, dtype=torch.float32)
                self._init_owner(buf, k)
                self.store.set("%s/%s/ready%d" % (STORE_PREFIX, self.run_id, k), "1")
            else:
                self.store.wait(["%s/%s/ready%d" % (STORE_PREFIX, self.run_id, k)])
                buf = torch.from_file(path, shared=True, size=total, dtype=torch.float32)
            return buf
        # ipc: owner allocates in its HBM, publishes the handle; others open it
        from torch.multiprocessing.reductions import reduce_tensor
        key = "%s/%s/ipc%d" % (STORE_PREFIX, self.run_id, k)
        if self.rank == k:
            buf = torch.zeros(total, dtype=torch.float32, device=self.params[0].device)
            self._init_owner(buf, k)
            torch.cuda.synchronize()
            self._owned = buf
            if self.world == 1:
                return buf
            fn, args = reduce_tensor(buf)
            self.store.set(key, pickle.dumps((fn, args)))
            return buf
        self.store.wait([key])
        fn, args = pickle.loads(self.store.get(key))
        return fn(*args)

    def _init_owner(self, buf, k):
        n_owner = sum(self.params[i].numel() for i in self.layout if self.layout[i][0] == k)
        with torch.no_grad():
            for i, p in enumerate(self.params):
                kk, off = self.layout[i]
                if kk == k:
                    buf[off:off + p.numel()].copy_(p.detach().reshape(-1).to(buf.device))
            if self.kind == "rmsprop":
                buf[2 * n_owner:3 * n_owner].fill_(1.0)  # TF RMSProp ms slot init 1.0
            if k == 0 and self._buf_local is not None:
                nsl = {"sgd": 0, "momentum": 1, "rmsprop": 2}[self.kind]
                base = n_owner * (1 + nsl)
                buf[base:base + self._buf_local.numel()].copy_(self._buf_local.to(buf.device))

    # -----------------------------------------------------------------------------------------
    @torch.no_grad()
    def pull(self):
        """Copy the current shared parameters into the local replica (M1)."""
        from ..ops.nn import WEIGHT_VERSION
        if self._local is not None:
            for k, loc in self._local.items():
                loc.copy_(self.flat[k][:loc.numel()].to(loc.device, non_blocking=True))
                l16 = self._local16[k]
                if l16 is not None:
                    l16.copy_(loc[:l16.numel()])
        else:
            for i, p in enumerate(self.params):
                p.copy_(self.shards[i]["param"].to(p.device, non_blocking=True))
                w16 = getattr(p, "bf16", None)
                if w16 is not None:
                    w16.copy_(p)
        if self._buf_local is not None:
            self._buf_local.copy_(self.buf_shard.to(self._buf_local.device, non_blocking=True))
            self._buf_snap.copy_(self._buf_local)
        WEIGHT_VERSION[0] += 1

    @torch.no_grad()
    def push_buffers(self):
        """Apply this worker's forward-time buffer updates to the shared copy (delta since the pull)."""
        if self._buf_local is None:
            return
        delta = self._buf_local - self._buf_snap
        self.buf_shard.add_(delta.to(self.buf_shard.device, non_blocking=True))

    # ---- fused GPU push: one multi-tensor optimizer launch on the owner shards -----------------
    def _fused_tables(self):
        """Static part of the multi-tensor table (shard / slot pointers, sizes, wd) + the chunk list."""
        import numpy as np

        from ..ops import _lib
        L = _lib.lib()
        tb, chunk = L.dtm_opt_tensor_bytes(), L.dtm_opt_chunk_size()
        assert tb == 64, tb
        tens = np.zeros((len(self.params), 8), dtype=np.uint64)
        chunks = []
        for i, p in enumerate(self.params):
            sh = self.shards[i]
            tens[i, 0] = sh["param"].data_ptr()
            tens[i, 2] = sh["s1"].data_ptr() if "s1" in sh else 0
            tens[i, 3] = sh["s2"].data_ptr() if "s2" in sh else 0
            tens[i, 6] = p.numel()
            tens[i, 7] = np.array([self.wd[i], 1.0], dtype=np.float32).view(np.uint64)[0]
            for st in range(0, p.numel(), chunk):
                chunks.append((i, st))
        ct = np.zeros((len(chunks), 2), dtype=np.int64)
        for j, (i, st) in enumerate(chunks):
            ct[j, 0], ct[j, 1] = i, st
        dev = self.params[0].device
        self._ftens = tens
        self._fchunks = torch.from_numpy(ct.view(np.uint8).reshape(-1).copy()).to(dev)
        self._fnchunks = len(chunks)
        self._fring = [(torch.empty(tens.nbytes, dtype=torch.uint8).pin_memory(),
                        torch.zeros(3, dtype=torch.float32).pin_memory(), None) for _ in range(4)]
        self._fi = 0
        self._fdev_tens = torch.empty(tens.nbytes, dtype=torch.uint8, device=dev)
        self._fdyn = torch.zeros(3, dtype=torch.float32, device=dev)

    @torch.no_grad()
    def _push_fused(self, grads, lr, grad_scale, sync):
        """GPU mode: every shard updated by ONE dtm_multi_tensor_opt launch on this rank's stream; the
        kernel writes the owners' HBM directly through the IPC mappings (xGMI peer access).  The grad
        pointers change per step, so the per-step table row is staged through a pinned ring."""
        import numpy as np

        from ..ops import _lib
        from ..ops.optim import KINDS
        if getattr(self, "_ftens", None) is None:
            self._fused_tables()
        keep = []
        tens = self._ftens.copy()
        for i, g in enumerate(grads):
            if g is None:
                tens[i, 6] = 0  # no gradient this step: the rows of this tensor do nothing
                continue
            g = g.detach().float().contiguous()
            keep.append(g)
            tens[i, 1] = g.data_ptr()
        host, dyn, ev = self._fring[self._fi]
        if ev is not None:
            ev.synchronize()  # the copy that last read this ring slot has executed
        host.numpy()[:] = tens.view(np.uint8).reshape(-1)
        dyn[0], dyn[1], dyn[2] = float(lr), 0.0, float(grad_scale)
        self._fdev_tens.copy_(host, non_blocking=True)
        self._fdyn.copy_(dyn, non_blocking=True)
        L = _lib.lib()
        L.dtm_multi_tensor_opt(_lib.ptr(self._fdev_tens), _lib.ptr(self._fchunks), self._fnchunks, KINDS[self.kind],
                               float(lr), float(self.mu), float(self.rho), float(self.eps), float(grad_scale), 0.0, 0,
                               None, _lib.ptr(self._fdyn), _lib.stream_ptr())
        ev = torch.cuda.Event()
        ev.record()
        self._fring[self._fi] = (host, dyn, ev)
        self._fi = (self._fi + 1) % len(self._fring)
        if sync:
            ev.synchronize()

    @torch.no_grad()
    def push(self, grads, lr=None, grad_scale=1.0, sync=True):
        """Apply this worker's gradients to the owner shards with the TF rule (M2).  GPU shards: one
        fused multi-tensor launch (``sync``: wait for it, e.g. before an SSP clock tick); host shards
        (shm mode): per-tensor torch ops."""
        lr = self.lr if lr is None else lr
        if self.params[0].is_cuda and self.mode == "ipc":
            return self._push_fused(grads, lr, grad_scale, sync)
        for i, p in enumerate(self.params):
            g = grads[i]
            if g is None:
                continue
            sh = self.shards[i]
            w = sh["param"]
            g = g.to(w.device, non_blocking=True).float() * grad_scale + self.wd[i] * w
            if self.kind == "sgd":
                w.sub_(lr * g)
            elif self.kind == "momentum":
                sh["s1"].mul_(self.mu).add_(g)
                w.sub_(lr * sh["s1"])
            else:
                sh["s2"].mul_(self.rho).add_((1 - self.rho) * g * g)
                sh["s1"].mul_(self.mu).add_(lr * g * torch.rsqrt(sh["s2"] + self.eps))
                w.sub_(sh["s1"])
        if self.params[0].is_cuda:
            torch.cuda.synchronize()

    def increment_global_step(self):
        return int(self.store.add("%s/%s/global_step" % (STORE_PREFIX, self.run_id), 1))

    def global_step(self):
        return int(self.store.add("%s/%s/global_step" % (STORE_PREFIX, self.run_id), 0))

    def set_global_step(self, n):
        """Resume: move the shared counter to ``n`` (chief only, before workers start)."""
        cur = self.global_step()
        if n != cur:
            self.store.add("%s/%s/global_step" % (STORE_PREFIX, self.run_id), int(n) - cur)

    def close(self):
        pg.barrier()
        if self.mode == "shm" and self.rank in self.flat:
            try:
                os.remove("/dev/shm/%s_%s_owner%d" % (STORE_PREFIX, self.run_id, self.rank))
            except OSError:
                pass


def _default_store():
    if pg.world_size() > 1:
        # the default process group's store (TCPStore on rank 0)
        from torch.distributed import distributed_c10d as c10d
        return c10d._get_default_store()
    return _LocalStore()


class _LocalStore:
    """Single-process stand-in for the c10d store API used here."""

    def __init__(self):
        self.d = {}

    def set(self, k, v):
        self.d[k] = v if isinstance(v, bytes) else str(v).encode()

    def get(self, k):
        return self.d[k]

    def add(self, k, n):
        v = int(self.d.get(k, b"0")) + n
        self.d[k] = str(v).encode()
        return v

    def wait(self, keys, timeout=None):
        for k in keys:
            if k not in self.d:
                raise KeyError(k)


class ASPTrainStep:
    """Worker step in ASP mode: pull -> fwd/bwd -> push; no collective on the critical path."""

    def __init__(self, model, loss_fn, store: ParamStore, lr_schedule=None, ssp_clock=None):
        self.model, self.loss_fn, self.store = model, loss_fn, store
        self.lr_schedule = lr_schedule
        self.ssp = ssp_clock
        self.local_step = 0

    def __call__(self, images, labels):
        self.store.pull()
        for p in self.store.params:
            p.grad = None
        out = self.model(images, training=True)
        loss = self.loss_fn(out, labels)
        loss.backward()
        if images.is_cuda:
            _lib.side_join()  # weight gradients enqueued on the side stream (ops/_lib.py)
        gs = self.store.global_step()
        lr = self.lr_schedule(gs) if self.lr_schedule else None
        self.store.push_buffers()
        # ASP: nothing waits for the update (Hogwild: the next pull on this stream sees it); SSP ticks
        # the staleness clock only after the update has landed
        self.store.push([getattr(p, "main_grad", None) if p.grad is None else p.grad for p in self.store.params],
                        lr=lr, sync=self.ssp is not None)
        gstep = self.store.increment_global_step()
        self.local_step += 1
        if self.ssp is not None:
            self.ssp.tick(self.local_step)
        return loss.detach(), gstep


def wait_all_done(store, world, run_id, timeout_s=600):
    """Workers finishing at different speeds (ASP) meet here before teardown."""
    k = "%s/%s/done" % (STORE_PREFIX, run_id)
    store.add(k, 1)
    t0 = time.time()
    while int(store.add(k, 0)) < world:
        if time.time() - t0 > timeout_s:
            raise TimeoutError("ASP teardown")
        time.sleep(0.01)
    if dist.is_available() and dist.is_initialized():
        pass
