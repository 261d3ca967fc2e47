"""BSP data parallelism: bucketed gradient all-reduce over RCCL (xGMI), overlapped with backward.

Replaces the reference's PS-side SyncReplicasOptimizer (ConditionalAccumulator per variable +
chief queue runner + sync token queue; e.g. reference
alexnet/cifar10_alexnet_bsp.py:79-94, inception/imagenet_inception_bsp.py:123-157).

Design (MI355X-first):
  * all fp32 gradients live in ONE flat buffer laid out in backward (reverse-registration)
    order; every parameter gets ``param.main_grad`` = its view.  Conv wgrad kernels add into it
    directly with fp32 atomics, so there is no per-parameter grad copy or bucket pack kernel;
  * the buffer is cut into ~``bucket_mb`` contiguous buckets (a tensor larger than a bucket - e.g.
    VGG-16's 411 MB fc6 gradient - is split across several buckets so its all-reduce pipelines); the
    last bucket of backward (the first layers, whose gradients come last and whose collective nothing
    can hide) is cut at ``tail_mb`` (ResNet-50: stem + stage 1 ~ 1 MB instead of a 6 MB remainder);
  * when the last gradient of a bucket is produced (``grad_ready`` fired by the ops, or autograd
    post-accumulate hooks for plain torch ops), the bucket's all_reduce(SUM) is issued
    asynchronously; RCCL's internal stream waits on the compute stream at issue time, so the
    reduction overlaps the rest of backward;
  * averaging (1/W) and the per-rank batch weight (C15, b_r / b_nominal) are folded into the
    optimizer's grad_scale / the loss scale - no extra pass over the gradients;
  * conv weights with dead taps (taps that only ever read zero padding, e.g. VGG-16 fc6 as a 7x7 conv
    over a 1x1 map in the reference's CIFAR geometry: 48 of 49 taps) have a provably-zero gradient
    outside their live window on EVERY rank; such a parameter gets its own compact bucket: the window
    is gathered into a contiguous buffer, all-reduced, and scattered back - the dead part never
    travels (VGG-16 DP: 537 MB -> ~134 MB of fp32 per step; reference vgg/nets/vgg.py:202);
  * ``comm_dtype=torch.bfloat16`` (opt-in) sends each bucket as bf16: the bucket is cast into a
    bf16 shadow right before its all-reduce and cast back after the wait - half the bytes on the
    xGMI links for communication-bound models (VGG-16: 537 MB of fp32 gradient per step), at the
    cost of bf16 rounding of the per-rank and summed gradients.
With world_size == 1 no collective is issued.
"""
import os

import torch
import torch.distributed as dist

from ..ops import _lib
from ..ops import nn as opsnn
from ..utils.profiler import roctx


class BSPDataParallel:
    def __init__(self, params, bucket_mb=32.0, process_group=None, device=None, overlap=True, grad_dtype=torch.float32,
                 comm_dtype=None, tail_mb=1.0, check=None, names=None, force_comm=False):
        self.params = [p for p in params if p.requires_grad]
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        # force_comm: issue the bucket collectives even with one rank (tests: the RCCL path on a one-GPU box)
        self.comm_on = self.world > 1 or bool(force_comm)
        dev = device or self.params[0].device
        total = sum(p.numel() for p in self.params)
        self.flat = torch.zeros(total, dtype=grad_dtype, device=dev)
        self.comm_dtype = comm_dtype if comm_dtype is not None else grad_dtype
        # low-precision shadow of the flat buffer for the wire (only with more than one rank)
        self.comm = (torch.empty(total, dtype=self.comm_dtype, device=dev)
                     if (self.comm_dtype != grad_dtype and self.comm_on) else None)
        # backward order ~ reverse of registration order
        self.order = list(reversed(self.params))
        self.offsets = {}
        off = 0
        for p in self.order:
            self.offsets[p] = off
            p.main_grad = self.flat[off:off + p.numel()].view(p.shape)
            off += p.numel()
        self.cap = max(1, int(bucket_mb * (1 << 20) / self.flat.element_size()))
        # the LAST bucket of backward is the exposed one (nothing is left to overlap it): keep it small
        self.tail = max(0, int(tail_mb * (1 << 20) / self.flat.element_size()))
        # param -> live-tap window (r0, r1, s0, s1): compact bucket (windows announced to an earlier
        # instance are remembered on the parameter).  Feature bsp_compact (ops/features.py; off: DTM_DISABLE).
        from ..ops import features
        self._compact_on = features.on("bsp_compact")
        self.windows = {p: p._live_win for p in self.params
                        if self._compact_on and getattr(p, "_live_win", None) is not None and p.dim() == 4}
        self._works = []
        self._done_works = []
        self._build_buckets()
        self._win_hook = opsnn.add_live_window_hook(self._on_live_window)
        self.overlap = overlap
        self._have = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._works = []
        self._seen = set()
        self._hook = opsnn.add_grad_ready_hook(self._on_ready)
        self._acc_hooks = []
        for p in self.params:
            if hasattr(p, "register_post_accumulate_grad_hook"):
                self._acc_hooks.append(p.register_post_accumulate_grad_hook(self._on_accumulated))
        # debug mode (DTM_BSP_CHECK=1): every gradient write must precede its parameter's ready notification,
        # which must come once per step; a write into a bucket whose all-reduce was already issued would be
        # clobbered by the collective's copy-back or left out of the sum
        self.check = (os.environ.get("DTM_BSP_CHECK", "0") not in ("", "0")) if check is None else bool(check)
        self._names = {}
        if names is not None:
            self._names = {p: n for n, p in names}
        self._write_hook = opsnn.add_grad_write_hook(self._on_write) if self.check else None
        self.writes_checked = 0
        self.unreported = []

    def _build_buckets(self):
        """Contiguous cap-sized buckets over the flat buffer, skipping the segments of windowed
        parameters, plus one compact bucket per windowed parameter (its live window, gathered)."""
        segs, cur = [], None
        for p in self.order:
            s, e = self.offsets[p], self.offsets[p] + p.numel()
            if p in self.windows:
                if cur is not None:
                    segs.append(cur)
                    cur = None
                continue
            cur = (cur[0], e) if cur is not None else (s, e)
        if cur is not None:
            segs.append(cur)
        self.buckets = []  # (start, end) of the flat buffer, or (param, window) for a compact bucket
        for i, (s, e) in enumerate(segs):
            # the final segment ends with a tail bucket of at most `tail` elements (the first layers'
            # gradients, produced last), so the collective left exposed after backward is short
            cut = e - self.tail if (i == len(segs) - 1 and 0 < self.tail < e - s) else e
            while s < cut:
                self.buckets.append((s, min(cut, s + self.cap)))
                s += self.cap
            if cut < e:
                self.buckets.append((cut, e))
        self.compact = {}  # bucket index -> (param, window, fp32 buffer, comm-dtype buffer or None)
        for p in self.order:
            if p in self.windows:
                r0, r1, s0, s1 = self.windows[p]
                K, _R, _S, C = p.shape
                buf = torch.empty((K, r1 - r0, s1 - s0, C), dtype=self.flat.dtype, device=self.flat.device)
                low = (torch.empty(buf.shape, dtype=self.comm_dtype, device=buf.device)
                       if (self.comm is not None) else None)
                self.compact[len(self.buckets)] = (p, self.windows[p], buf, low)
                self.buckets.append((p, self.windows[p]))
        # param -> list of (bucket index, element count inside that bucket)
        self.contrib = {}
        self.need = [0] * len(self.buckets)
        for p in self.order:
            if p in self.windows:
                bi = [i for i, v in self.compact.items() if v[0] is p][0]
                self.contrib[p] = [(bi, 1)]
                self.need[bi] = 1
                continue
            s, e = self.offsets[p], self.offsets[p] + p.numel()
            lst = []
            for bi, b in enumerate(self.buckets):
                if bi in self.compact:
                    continue
                lo, hi = max(s, b[0]), min(e, b[1])
                if lo < hi:
                    lst.append((bi, hi - lo))
                    self.need[bi] += hi - lo
            self.contrib[p] = lst
        self._have = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)

    def _on_live_window(self, p, win):
        """A conv announced its live-tap window (forward, before any bucket of this step launched)."""
        if not self._compact_on or p not in self.offsets or self.windows.get(p) == win or p.dim() != 4:
            return
        if any(self._launched) or self._works:
            raise RuntimeError("live-tap window changed while gradients were in flight")
        self.windows[p] = win
        self._build_buckets()

    def wire_elements(self):
        """Gradient elements sent per all-reduce step (compact buckets count their window only)."""
        n = 0
        for bi, b in enumerate(self.buckets):
            n += self.compact[bi][2].numel() if bi in self.compact else b[1] - b[0]
        return n

    def close(self):
        opsnn.remove_live_window_hook(self._win_hook)
        opsnn.remove_grad_ready_hook(self._hook)
        if self._write_hook is not None:
            opsnn.remove_grad_write_hook(self._write_hook)
        for h in self._acc_hooks:
            h.remove()

    # ------------------------------------------------------------------------------------------
    def zero_grad(self):
        self.flat.zero_()
        self._have = [0] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._works = []
        self._seen = set()
        self.unreported = []

    def _on_accumulated(self, p):
        # plain autograd path (CPU ops / torch fallbacks): move .grad into the flat buffer.  (autograd also
        # runs this hook with no .grad when a HIP op already wrote main_grad and returned None for p: that
        # op notified p itself)
        if p.grad is None:
            return
        if self.check:
            self._on_write(p)
        p.main_grad.add_(p.grad.to(p.main_grad.dtype))
        p.grad = None
        self._on_ready(p)

    def _pname(self, p):
        return self._names.get(p, "<param %s>" % (tuple(p.shape),))

    def _on_write(self, p):
        """(check mode) a kernel / op is about to write p's gradient."""
        lst = self.contrib.get(p)
        if lst is None:
            return
        self.writes_checked += 1
        if p in self._seen:
            raise RuntimeError("BSP check: gradient of %s written after it was reported ready" % self._pname(p))
        for bi, _n in lst:
            if self._launched[bi]:
                raise RuntimeError("BSP check: gradient of %s written after the all-reduce of its bucket %d was issued"
                                   % (self._pname(p), bi))

    def _on_ready(self, p):
        lst = self.contrib.get(p)
        if lst is None:
            return
        if p in self._seen:
            if self.check:
                raise RuntimeError("BSP check: %s reported ready twice in one step" % self._pname(p))
            return
        self._seen.add(p)
        for bi, n in lst:
            self._have[bi] += n
            if self.overlap and self._have[bi] == self.need[bi]:
                self._launch(bi)

    def _launch(self, bi):
        if self._launched[bi]:
            return
        self._launched[bi] = True
        if not self.comm_on:
            return
        side = _lib.side_active() if self.flat.is_cuda else None
        if side is not None and torch.cuda.current_stream() != side:
            # weight gradients run on the side stream (ops/_lib.py): the all-reduce goes after both
            # streams' work so far without making the main stream wait for the side one
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                self._launch_now(bi)
        else:
            self._launch_now(bi)

    def _launch_now(self, bi):
        with roctx("allreduce_bucket_%d" % bi):
            if bi in self.compact:
                p, (r0, r1, s0, s1), buf, low = self.compact[bi]
                buf.copy_(p.main_grad[:, r0:r1, s0:s1, :])  # gather the live window
                if low is not None:
                    low.copy_(buf)
                    buf = low
            else:
                s, e = self.buckets[bi]
                buf = self.flat[s:e]
                if self.comm is not None:
                    buf = self.comm[s:e]
                    buf.copy_(self.flat[s:e])
            self._works.append((bi, dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)))

    def finish(self):
        """Launch any bucket not yet reduced (unused params / no overlap) and make the current
        stream wait for every reduction."""
        if self.check:
            # parameters that never reported a gradient this step (legal - an unused head - but listed)
            self.unreported = [self._pname(p) for p in self.order if p not in self._seen]
        for bi in range(len(self.buckets)):
            if not self._launched[bi]:
                self._launch(bi)
        if self.flat.is_cuda:
            _lib.side_join()
        for bi, w in self._works:
            w.wait()
            if bi in self.compact:
                p, (r0, r1, s0, s1), buf, low = self.compact[bi]
                p.main_grad[:, r0:r1, s0:s1, :].copy_(low if low is not None else buf)  # scatter back
            elif self.comm is not None:
                s, e = self.buckets[bi]
                self.flat[s:e].copy_(self.comm[s:e])
        if self.check:
            # nothing may write a gradient between the waits above and the next zero_grad
            self._seen = set(self.contrib)
        self._done_works = self._works
        self._works = []

    def bucket_elements(self):
        """Elements each bucket sends, in bucket order."""
        return [self.compact[bi][2].numel() if bi in self.compact else b[1] - b[0]
                for bi, b in enumerate(self.buckets)]

    def bucket_ms(self):
        """Per-bucket collective durations (ms) of the last step, in issue order - available when the
        RCCL communicator records timing events (process_group.rccl_env(timing=True)); [] otherwise.
        Synchronizes with the last collective: call on log steps only."""
        out = []
        for _bi, w in self._done_works:
            try:
                out.append(round(float(w._get_duration()), 4))
            except Exception:
                return []
        return out

    @property
    def grad_scale(self):
        return 1.0 / self.world


def flatten_tensors(tensors):
    """Re-home ``tensors`` (same dtype and device) into ONE contiguous buffer and return it.

    Object identity is kept - every tensor's ``.data`` is re-pointed at its view of the buffer - so
    module buffers, slim variable stores and checkpoint variable lists that already hold the
    tensors keep working, while one collective / one copy now covers all of them.  Must run before
    anything caches raw device pointers of the tensors (FusedOptimizer tables)."""
    tensors = list(tensors)
    if not tensors:
        return None
    dt, dev = tensors[0].dtype, tensors[0].device
    assert all(t.dtype == dt and t.device == dev for t in tensors), "flatten_tensors: mixed dtype/device"
    flat = torch.empty(sum(t.numel() for t in tensors), dtype=dt, device=dev)
    off = 0
    with torch.no_grad():
        for t in tensors:
            n = t.numel()
            v = flat[off:off + n].view(t.shape)
            v.copy_(t.detach())
            t.data = v
            off += n
    return flat


class BufferSync:
    """Replica-consistent BN moving statistics under BSP, with the reference's update semantics.

    In the reference every worker's BN update op (``AssignMovingAvg`` in UPDATE_OPS, run as control
    dependencies of each worker's train op: inception/imagenet_inception_bsp.py:145-149,
    inception/slim/ops.py:117-131) writes the ONE PS-resident ``moving_mean`` / ``moving_variance``, so one
    global step applies W updates m <- d*m + (1-d)*b_r, one per worker batch, to a single copy - the same as
    the ASP store here (parallel/asp.py push_buffers: each worker adds its forward's delta).  Here each replica
    updates its own copy in its forward (k local steps since the last sync, k = ``every``); this class makes
    every replica end the synced step with
        m = d^(W*k) * m_prev + (1 - d^(W*k)) * mean_r(B_r),    B_r = (m_r - d^k * m_prev) / (1 - d^k),
    i.e. W*k sequential moving-average updates of the one shared copy, each replica contributing its own
    implied (decay-weighted) batch statistic B_r.  This is exact for W = 1, equal to the reference's W
    sequential updates up to the order in which the workers' batches land, and a convex combination of
    m_prev and the replicas' statistics for ANY decay (NASNet-CIFAR's d = 0.9 at W = 8 included: a
    first-order form m_prev + sum_r (m_r - m_prev) would weight m_prev by 1 - W(1-d) <= 0 there and could drive
    a variance negative).  Statistics whose decay is unknown get d = 0: plain averaging over the replicas.
    Mechanics: the statistics live in one flat fp32 buffer (``flatten_tensors``); ``issue`` (right after the
    forward: the statistics are final then, backward never reads them) computes B_r into a separate send
    buffer and issues its SUM all-reduce, which runs on the comm stream underneath the whole backward;
    ``finish`` waits and writes the combined statistics.  The live statistics are never overwritten by a
    partial result, so an exception between ``issue`` and ``finish`` (``abort``) leaves them at this replica's
    own values.  EMA shadows of the statistics are updated by the optimizer from the synced values, so they
    stay replica-identical without a collective of their own."""

    def __init__(self, buffers, process_group=None, every=1, decays=None, force_comm=False):
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1
        self.buffers = [b for b in buffers]
        self.every = max(1, int(every))
        comm = self.world > 1 or bool(force_comm)
        self.flat = flatten_tensors(self.buffers) if (comm and self.buffers) else None
        self.prev = self.send = self.decay = None
        if self.flat is not None:
            # the statistics as of the last sync (every replica holds the same values there)
            self.prev = self.flat.detach().clone()
            self.send = torch.empty_like(self.flat)
            ds = list(decays) if decays is not None else [None] * len(self.buffers)
            assert len(ds) == len(self.buffers), "BufferSync: one decay per buffer"
            # per-element decay, fp64 so d^(W*k) keeps its digits; unknown decay -> 0 (averaging)
            self.decay = torch.cat([torch.full((b.numel(),), float(d) if d is not None else 0.0,
                                               dtype=torch.float64) for b, d in zip(self.buffers, ds)]
                                   ).to(self.flat.device)
            assert bool(((self.decay >= 0) & (self.decay < 1)).all()), "BN decay must lie in [0, 1)"
        self._work = None
        self._n = 0       # steps since construction
        self._local = 0   # local (unsynced) moving-average updates since the last sync
        self._k = 0       # local updates covered by the in-flight all-reduce
        self._pow = {}    # k -> (d^k, 1 / (1 - d^k), d^(W*k)) (k is constant in steady state)

    def _powers(self, k):
        if k not in self._pow:
            dk = self.decay.pow(k)
            self._pow[k] = (dk, 1.0 / (1.0 - dk), self.decay.pow(self.world * k))
        return self._pow[k]

    def begin(self):
        """(kept for API symmetry: the snapshot is the state after the last sync, see finish)"""

    def issue(self):
        if self.flat is None:
            return
        self._n += 1
        self._local += 1
        if (self._n - 1) % self.every:
            return
        k = self._local
        with roctx("bn_stats_allreduce"):
            dk, inv, _ = self._powers(k)
            # B_r = (m_r - d^k m_prev) / (1 - d^k)   (this replica's implied batch statistic)
            self.send.copy_((self.flat.double() - dk * self.prev.double()) * inv)
            self._k = k
            self._work = dist.all_reduce(self.send, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def finish(self):
        if self._work is None:
            return
        self._work.wait()
        self._work = None
        dwk = self._powers(self._k)[2]
        m = dwk * self.prev.double() + (1.0 - dwk) * (self.send.double() / self.world)
        self.flat.copy_(m)
        self.prev.copy_(self.flat)
        self._local = 0

    def abort(self):
        """An exception between issue() and finish(): drain the collective, keep this replica's own statistics
        (the live buffer was never overwritten) - the next completed sync folds them in."""
        if self._work is not None:
            try:
                self._work.wait()
            finally:
                self._work = None

    def resync(self):
        """The statistics were overwritten outside a step (checkpoint restore, broadcast): re-snapshot."""
        if self.flat is not None:
            self.prev.copy_(self.flat)
            self._local = 0

    def numel(self):
        return 0 if self.flat is None else self.flat.numel()
