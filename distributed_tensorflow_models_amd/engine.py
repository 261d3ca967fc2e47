"""Single training step: forward -> loss -> backward (+ overlapped bucket all-reduce) -> fused update.

This is the MI355X replacement for the reference's per-step ``sess.run([train_op, loss,
global_step])``: no PS round trips, gradients reduced over RCCL while backward
runs, one multi-tensor optimizer launch, TF 1.x optimizer / loss semantics.
"""
import torch

from .ops import fused as _fused
from .ops import nn as F
from .ops.optim import FusedOptimizer
from .parallel.bsp import BSPDataParallel


def prepare_compute_copies(model):
    """Create the bf16 compute copy of every matrix/conv weight (refreshed by the optimizer)."""
    for p in model.parameters():
        if p.is_cuda and p.dim() >= 2 and getattr(p, "bf16", None) is None:
            p.bf16 = p.detach().to(torch.bfloat16)


class TrainStep:
    def __init__(self, model, optimizer="momentum", lr=0.1, momentum=0.9, rho=0.9, epsilon=1e-10, bucket_mb=32.0,
                 label_smoothing=0.0, aux_weight=0.4, ema_decay=None, lr_schedule=None, use_graph=False,
                 process_group=None, weight_decay=None, batch_weight=1.0):
        self.model = model
        prepare_compute_copies(model)
        params = [p for p in model.parameters() if p.requires_grad]
        self.dp = BSPDataParallel(params, bucket_mb, process_group)
        self.opt = FusedOptimizer(params, optimizer, lr, momentum, rho, epsilon, ema_decay, weight_decay)
        self.lr = lr
        self.lr_schedule = lr_schedule
        self.smoothing = label_smoothing
        self.aux_weight = aux_weight
        self.batch_weight = batch_weight
        self.global_step = 0
        self.use_graph = use_graph

    def loss_fn(self, out, labels):
        aux = None
        if isinstance(out, tuple):
            out, aux = out
        loss = F.softmax_cross_entropy(out, labels, self.smoothing).mean()
        if aux is not None and self.aux_weight:
            loss = loss + self.aux_weight * F.softmax_cross_entropy(aux, labels, self.smoothing).mean()
        if self.batch_weight != 1.0:
            loss = loss * self.batch_weight
        return loss

    def current_lr(self):
        if self.lr_schedule is not None:
            return float(self.lr_schedule(self.global_step))
        return self.lr

    def __call__(self, images, labels):
        self.dp.zero_grad()
        if images.is_cuda:
            _fused.arena.begin_step(images.device)
        try:
            out = self.model(images, training=True)
            loss = self.loss_fn(out, labels)
            loss.backward()
        finally:
            _fused.arena.end_step()
        self.dp.finish()
        self.opt.step(self.current_lr(), grad_scale=self.dp.grad_scale)
        self.global_step += 1
        return loss.detach()
