"""Single training step: forward -> loss -> backward (+ overlapped bucket all-reduce) -> fused update.

This is the MI355X replacement for the reference's per-step ``sess.run([train_op, loss,
global_step])``: no PS round trips, gradients reduced over RCCL while backward
runs, one multi-tensor optimizer launch, TF 1.x optimizer / loss semantics.
"""
import os

import torch

from .ops import _lib
from .ops import elementwise as _elementwise
from .ops import fused as _fused
from .ops import nn as F
from .ops.optim import FusedOptimizer
from .parallel.bsp import BSPDataParallel, BufferSync
from .utils.profiler import range_pop, range_push, roctx


def prepare_compute_copies(model):
    """Create the bf16 compute copy of every matrix/conv weight (refreshed by the optimizer).  Weight groups the
    model declares (``sibling_weight_groups``: the 1x1 branch heads of an Inception mixed block, same input
    channels) get their copies as consecutive views of ONE [sum K][1][1][C] buffer, recorded as ``p._sib_cat =
    (buffer, row offset)``: the merged head conv reads them as one weight (ops.fused._SiblingGroup.forward_all)."""
    groups = model.sibling_weight_groups() if hasattr(model, "sibling_weight_groups") else []
    for grp in groups:
        if not grp or not all(p.is_cuda and p.dim() == 4 and p.shape[1:] == grp[0].shape[1:] for p in grp):
            continue
        if any(getattr(p, "_sib_cat", None) is not None for p in grp):
            continue
        buf = torch.empty((sum(p.shape[0] for p in grp),) + tuple(grp[0].shape[1:]), device=grp[0].device,
                          dtype=torch.bfloat16)
        off = 0
        for p in grp:
            v = buf[off:off + p.shape[0]]
            v.copy_(p.detach())
            p.bf16 = v
            p._sib_cat = (buf, off)
            off += p.shape[0]
    for p in model.parameters():
        if p.is_cuda and p.dim() >= 2 and getattr(p, "bf16", None) is None:
            p.bf16 = p.detach().to(torch.bfloat16)


def moving_average_buffers(model):
    """The tensors TF puts in moving_average_variables(): every BN moving mean / variance."""
    from .models.layers import tf_variables
    return [t for _n, t, _l, trainable in tf_variables(model)
            if not trainable and t.dtype == torch.float32 and t.is_floating_point()]


def moving_average_decays(model, buffers):
    """The moving-average decay of each BN statistic in ``buffers`` (None where unknown): a module BatchNorm
    (models/layers.py) carries ``decay``; slim / old-slim batch_norm tag their variables with ``_bn_decay``."""
    by_id = {}
    for m in model.modules():
        names = getattr(m, "tf_buffer_names", None)
        if names and getattr(m, "decay", None) is not None:
            for b in names:
                by_id[id(getattr(m, b))] = float(m.decay)
    return [getattr(b, "_bn_decay", by_id.get(id(b))) for b in buffers]


def reserved_cus_default():
    """CUs kept out of the compute grids' sizing under data parallelism (ops/_lib.set_reserved_cus):
    DTM_RESERVED_CUS if set, else RESERVED_CUS_DP.  (A pinned RCCL channel count - NCCL_MAX_NCHANNELS, trainer
    --rccl_channels - does not reserve anything by itself: reserving measured slower, see below.)"""
    v = os.environ.get("DTM_RESERVED_CUS")
    if v is not None:
        return int(v)
    return RESERVED_CUS_DP


# Measured on one MI355X with a CU-occupying copy kernel on a second stream for 8 ms of every backward standing in
# for the RCCL channels (profiles/ab/r4_ab_hog_reserve.log, ResNet-50): 16 CUs taken +2.4 % step, 32 CUs +3.5 %;
# reserving the same CUs from the compute grids' sizing made both worse (+3.3 %, +4.8 %; +0.8 % with no
# contention): the non-persistent tiles rebalance by themselves, so nothing is reserved by default.
RESERVED_CUS_DP = 0


class TrainStep:
    def __init__(self, model, optimizer="momentum", lr=0.1, momentum=0.9, rho=0.9, epsilon=1e-10, bucket_mb=32.0,
                 label_smoothing=0.0, aux_weight=0.4, ema_decay=None, lr_schedule=None, use_graph=False,
                 process_group=None, weight_decay=None, batch_weight=1.0, nan_guard=True, timer=None,
                 grad_comm_dtype=None, ema_buffers=True, bn_sync_every=1, wgrad_stream=None, bsp_check=None,
                 overlap=True, force_comm=False, graph_comm=False):
        self.model = model
        if wgrad_stream is not None:
            # conv+BN weight gradients on the side stream (ops/_lib.py side_stream; process-wide): ResNet-50
            # -4.3 % step time, Inception-v3 +3.4 % eager (its per-conv stream forks cost more host time than
            # they overlap)
            _lib.set_side_enabled(wgrad_stream)
        prepare_compute_copies(model)
        params = [p for p in model.parameters() if p.requires_grad]
        # bsp_check (or DTM_BSP_CHECK=1): assert every gradient write precedes its bucket's all-reduce (debug)
        # force_comm: issue the collectives even with one rank (tests of the RCCL path on a one-GPU box)
        self.dp = BSPDataParallel(params, bucket_mb, process_group, comm_dtype=grad_comm_dtype, overlap=overlap,
                                  check=bsp_check, names=list(model.named_parameters()), force_comm=force_comm)
        if use_graph and self.dp.comm_on and not graph_comm:
            # a captured step holds the bucket all-reduces, the BN-statistics sync and their waits inside the graph
            # (RCCL collectives captured on the current stream, replayed every step): opt in with graph_comm=True -
            # validated bit-identical to the eager step at world 1 over RCCL
            # (tests/test_distributed.py::test_bsp_rccl_captured_step_matches_eager)
            raise ValueError("use_graph (hipGraph step capture) is only for steps without collectives unless "
                             "graph_comm=True; world size %d, force_comm %s" % (self.dp.world, bool(force_comm)))
        # BN moving statistics: one flat buffer, averaged over the replicas every step (reference
        # keeps ONE PS-resident copy that every worker updates); must precede the optimizer tables
        bufs = moving_average_buffers(model)
        self.bufsync = BufferSync(bufs, process_group, every=bn_sync_every,
                                  decays=moving_average_decays(model, bufs), force_comm=force_comm)
        # ema_buffers: whether the statistics also get EMA shadows (slim BN lists them in
        # moving_average_variables(); tf.layers BN - the CIFAR ResNet preset - does not)
        self.opt = FusedOptimizer(params, optimizer, lr, momentum, rho, epsilon, ema_decay, weight_decay,
                                  ema_buffers=moving_average_buffers(model)
                                  if (ema_decay is not None and ema_buffers) else ())
        self.lr = lr
        self.lr_schedule = lr_schedule
        self.smoothing = label_smoothing
        self.aux_weight = aux_weight
        self.batch_weight = batch_weight
        self.global_step = 0
        self.use_graph = use_graph
        self.nan_guard = nan_guard
        self.last_skip = None   # device int32 flag of the last step (1 = non-finite grads, update skipped)
        self.skipped = 0        # host count, updated by poll_skipped()
        self.timer = timer      # utils.metrics.StepTimer for fwd/bwd/allreduce/optimizer HIP-event sections
        self._graph = None
        self._eager_steps = 0
        self._skip_total = None  # device int32: number of skipped (non-finite) steps so far
        self._skip_seen = 0
        self.on_backward = None  # optional callable run right before loss.backward() (tools/ab_step.py 'hog')
        if self.dp.world > 1 and params and params[0].is_cuda:
            _lib.set_reserved_cus(reserved_cus_default())

    def loss_fn(self, out, labels):
        aux = None
        if isinstance(out, tuple):
            out, aux = out
        bw = self.batch_weight
        heads = [(out, bw)] + ([(aux, self.aux_weight * bw)] if aux is not None and self.aux_weight else [])
        return F.mean_xent_loss(heads, labels, self.smoothing)

    def current_lr(self):
        if self.lr_schedule is not None:
            return float(self.lr_schedule(self.global_step))
        return self.lr

    def _mark(self, name):
        if self.timer is not None:
            self.timer.mark(name)

    def _forward_backward(self, images, labels):
        self.dp.zero_grad()
        self._mark("start")
        if images.is_cuda:
            _fused.arena.begin_step(images.device)
            _elementwise.advance_seed_offset(images.device)  # fresh dropout masks, replay included
        try:
            with roctx("forward"):
                out = self.model(images, training=True)
            with roctx("loss"):
                loss = self.loss_fn(out, labels)
            self._mark("fwd")
            self.bufsync.issue()  # forward has finished every moving-statistics update
            if self.on_backward is not None:
                self.on_backward()
            with roctx("backward"):  # bucket all-reduces are issued (own ranges) from the grad hooks
                loss.backward()
            if images.is_cuda:
                _lib.side_join()  # weight gradients enqueued on the side stream (ops/_lib.py)
            self._mark("bwd")
        except BaseException:
            self.bufsync.abort()  # the live BN statistics stay this replica's own (never a partial sum)
            raise
        finally:
            _fused.arena.end_step()
        with roctx("allreduce_wait"):
            self.dp.finish()
            self.bufsync.finish()
        self._mark("allreduce")
        skip = None
        if self.nan_guard:
            # NaN/Inf guard on the reduced gradient: identical on every rank after the all-reduce,
            # so all replicas skip the same update
            flat = self.dp.flat
            if flat.is_cuda:
                skip = torch.zeros(1, device=flat.device, dtype=torch.int32)
                with roctx("nan_guard"):
                    _lib.lib().dtm_check_finite(_lib.ptr(flat), flat.numel(), _lib.ptr(skip), _lib.stream_ptr())
            else:
                skip = torch.tensor([0 if bool(torch.isfinite(flat).all()) else 1], dtype=torch.int32)
            self.last_skip = skip
            if self._skip_total is None:
                self._skip_total = torch.zeros(1, device=flat.device, dtype=torch.int32)
            self._skip_total.add_(skip)  # sticky device count: read on log steps only, no per-step sync
        return loss.detach(), skip

    def __call__(self, images, labels):
        if self.use_graph and images.is_cuda:
            return self._graph_step(images, labels)
        return self._eager_step(images, labels)

    def _eager_step(self, images, labels):
        rng = range_push("train_step")
        loss, skip = self._forward_backward(images, labels)
        with roctx("optimizer"):
            self.opt.step(self.current_lr(), grad_scale=self.dp.grad_scale, skip_flag=skip)
        self._mark("optimizer")
        self.global_step += 1
        range_pop(rng)
        return loss

    # ---- hipGraph path -----------------------------------------------------------------------
    # The whole step (zero-grad memset, forward, backward with its hook-issued bucket all-reduces,
    # NaN guard, fused optimizer, dgrad weight-copy refresh) is captured once into a hipGraph and
    # replayed: one host submission per step instead of ~600 kernel launches, so launch-bound
    # models (LeNet, CIFAR nets, small batches) stop being host-bound.  Per-step scalars (lr, EMA
    # decay, 1/W) live in a device buffer staged before every replay (FusedOptimizer.set_dynamic);
    # host counters (global_step, EMA num_updates) advance outside the graph.  The first
    # ``graph_warmup`` steps run eagerly so every lazily grown workspace, the zero-arena high-water
    # mark and the weight-flip table exist before capture (no allocation inside the graph).
    graph_warmup = 2

    def _graph_step(self, images, labels):
        if self._graph is None and self._eager_steps < self.graph_warmup:
            self._eager_steps += 1
            self.use_graph = False
            try:
                return self(images, labels)
            finally:
                self.use_graph = True
        if self._graph is None:
            self._static_x = images.clone()
            self._static_y = labels.clone()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            timer, self.timer = self.timer, None  # no event records inside the capture
            try:
                with torch.cuda.graph(g):
                    loss, skip = self._forward_backward(self._static_x, self._static_y)
                    self.opt.launch(skip)
                    from .ops.nn import refresh_flipped
                    refresh_flipped()
            finally:
                self.timer = timer
            self._graph, self._static_loss = g, loss
        else:
            if images.data_ptr() != self._static_x.data_ptr():
                self._static_x.copy_(images, non_blocking=True)
            if labels.data_ptr() != self._static_y.data_ptr():
                self._static_y.copy_(labels, non_blocking=True)
        self.opt.set_dynamic(self.current_lr(), self.dp.grad_scale)
        self._graph.replay()
        self.opt.num_updates += 1
        self.global_step += 1
        return self._static_loss.clone()

    def poll_skipped(self):
        """Host-side check (one small sync; call on log steps): True if any step since the last poll
        had non-finite gradients and skipped its update.  ``self.skipped`` = total so far."""
        if self._skip_total is None:
            return False
        n = int(self._skip_total.item())
        new = n - self._skip_seen
        self._skip_seen = n
        self.skipped = n
        return new > 0
