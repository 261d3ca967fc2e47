"""Fused multi-tensor optimizers (one HIP launch per step for every parameter).

TF 1.x update semantics:
  GradientDescentOptimizer  p -= lr*g                                  (C20)
  MomentumOptimizer         a = mu*a + g; p -= lr*a   (use_nesterov=False)  (C20b)
  RMSPropOptimizer          ms = rho*ms + (1-rho)g^2 (ms init 1.0); mom = mu*mom + lr*g/sqrt(ms+eps);
                            p -= mom                                       (C21)
  g = grad*grad_scale + weight_decay*p   (coupled L2 = d/dp of wd*sum(p^2)/2; K14)
  optional ExponentialMovingAverage shadows: ema -= (1-d)(ema - p), d = min(decay,(1+n)/(10+n)) (C22)
and a bf16 copy-out of every updated weight (the compute copy read by the conv kernels).

On CPU the same math runs as torch ops (gloo plumbing tests, reference checks).
"""
import ctypes

import numpy as np
import torch

from . import _lib

KINDS = {"sgd": 0, "momentum": 1, "rmsprop": 2}


class FusedOptimizer:
    def __init__(self, params, kind="momentum", lr=0.1, momentum=0.9, rho=0.9, epsilon=1e-10, ema_decay=None,
                 weight_decay=None, lr_mults=None, ema_buffers=()):
        self.params = [p for p in params if p.requires_grad]
        # non-trainable tensors that also get an EMA shadow (BN moving mean/variance: the reference
        # averages trainable_variables() + moving_average_variables(), e.g. reference
        # alexnet/cifar10_alexnet_bsp.py:79-86, inception/imagenet_inception_bsp.py:123-126)
        self.ema_buffers = [b for b in ema_buffers] if ema_decay is not None else []
        self.buffer_ema = {id(b): b.detach().clone().float() for b in self.ema_buffers}
        if kind not in KINDS:
            raise ValueError(kind)
        self.kind, self.lr, self.mu, self.rho, self.eps = kind, lr, momentum, rho, epsilon
        self.ema_decay = ema_decay
        self.num_updates = 0
        self.state = {}
        for p in self.params:
            st = {}
            if kind in ("momentum", "rmsprop"):
                st["s1"] = torch.zeros_like(p, dtype=torch.float32)
            if kind == "rmsprop":
                st["s2"] = torch.ones_like(p, dtype=torch.float32)  # TF RMSProp ms slot init 1.0
            if ema_decay is not None:
                st["ema"] = p.detach().clone().float()
            st["wd"] = float(getattr(p, "weight_decay", 0.0) if weight_decay is None else weight_decay)
            st["lr_mult"] = 1.0 if lr_mults is None else float(lr_mults.get(p, 1.0))
            self.state[p] = st
        self._dev = None
        if self.params and self.params[0].is_cuda:
            self._build_tables()

    # ---- device tables ---------------------------------------------------------------------
    def _build_tables(self):
        L = _lib.lib()
        tb, cb, chunk = L.dtm_opt_tensor_bytes(), L.dtm_opt_chunk_bytes(), L.dtm_opt_chunk_size()
        assert tb == 64 and cb == 16, (tb, cb)
        dev = self.params[0].device
        tens = np.zeros((len(self.params), 8), dtype=np.uint64)
        chunks = []
        self._keep = []
        for i, p in enumerate(self.params):
            st = self.state[p]
            g = self._grad_tensor(p)
            w16 = getattr(p, "bf16", None)
            if w16 is not None and (w16.dtype != torch.bfloat16 or w16.shape != p.shape):
                w16 = None
            ptrs = [p.data_ptr(), g.data_ptr(), st["s1"].data_ptr() if "s1" in st else 0,
                    st["s2"].data_ptr() if "s2" in st else 0, w16.data_ptr() if w16 is not None else 0,
                    st["ema"].data_ptr() if "ema" in st else 0]
            tens[i, :6] = ptrs
            tens[i, 6] = p.numel()
            tens[i, 7] = np.array([st["wd"], st["lr_mult"]], dtype=np.float32).view(np.uint64)[0]
            for s in range(0, p.numel(), chunk):
                chunks.append((i, 0, s))
        # EMA-only rows (grad pointer 0): the kernel just moves the shadow towards the buffer
        base = len(self.params)
        if self.ema_buffers:
            tens = np.concatenate([tens, np.zeros((len(self.ema_buffers), 8), dtype=np.uint64)])
        for j, b in enumerate(self.ema_buffers):
            assert b.dtype == torch.float32 and b.is_contiguous(), "EMA buffers must be contiguous fp32"
            tens[base + j, 0] = b.data_ptr()
            tens[base + j, 5] = self.buffer_ema[id(b)].data_ptr()
            tens[base + j, 6] = b.numel()
            for s in range(0, b.numel(), chunk):
                chunks.append((base + j, 0, s))
        ct = np.zeros((len(chunks), 2), dtype=np.int64)
        for j, (i, _, s) in enumerate(chunks):
            ct[j, 0] = i  # int t, int pad packed little-endian into first 8 bytes
            ct[j, 1] = s
        self._tens_dev = torch.from_numpy(tens.view(np.uint8).reshape(-1).copy()).to(dev)
        self._chunks_dev = torch.from_numpy(ct.view(np.uint8).reshape(-1).copy()).to(dev)
        self._nchunks = len(chunks)
        self._dyn = torch.zeros(3, dtype=torch.float32, device=dev)
        # ring of pinned staging rows: the host runs ahead of the GPU, so a row is reused only
        # after the copy that last read it has executed (its event), never overwritten in flight
        self._dyn_ring = torch.zeros((16, 3), dtype=torch.float32).pin_memory()
        self._dyn_ev = [None] * 16
        self._dyn_i = 0
        self._dev = dev

    @staticmethod
    def _grad_tensor(p):
        g = getattr(p, "main_grad", None)
        if g is None:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            g = p.grad
        return g

    def ema_decay_now(self):
        if self.ema_decay is None:
            return 0.0
        n = self.num_updates
        return min(self.ema_decay, (1.0 + n) / (10.0 + n))

    def set_dynamic(self, lr, grad_scale=1.0):
        """Stage per-step scalars on the device (safe to call before a hipGraph replay)."""
        i = self._dyn_i
        self._dyn_i = (i + 1) % len(self._dyn_ev)
        if self._dyn_ev[i] is not None:
            self._dyn_ev[i].synchronize()
        row = self._dyn_ring[i]
        row[0] = float(lr)
        row[1] = float(self.ema_decay_now())
        row[2] = float(grad_scale)
        self._dyn.copy_(row, non_blocking=True)
        ev = self._dyn_ev[i] or torch.cuda.Event()
        ev.record()
        self._dyn_ev[i] = ev

    def launch(self, skip_flag=None):
        """Issue the fused update reading lr/ema/grad_scale from the device scalars."""
        L = _lib.lib()
        L.dtm_multi_tensor_opt(_lib.ptr(self._tens_dev), _lib.ptr(self._chunks_dev), self._nchunks, KINDS[self.kind],
                               0.0, float(self.mu), float(self.rho), float(self.eps), 1.0, 0.0,
                               int(self.ema_decay is not None), _lib.ptr(skip_flag), _lib.ptr(self._dyn),
                               _lib.stream_ptr())

    def step(self, lr=None, grad_scale=1.0, skip_flag=None):
        lr = self.lr if lr is None else lr
        if self._dev is not None:
            self.set_dynamic(lr, grad_scale)
            self.launch(skip_flag)
            from .nn import refresh_flipped
            refresh_flipped()
        else:
            self._step_cpu(lr, grad_scale, skip_flag)
        self.num_updates += 1

    @torch.no_grad()
    def _step_cpu(self, lr, grad_scale, skip_flag):
        if skip_flag is not None and int(skip_flag.item()) != 0:
            return
        d = self.ema_decay_now()
        for p in self.params:
            st = self.state[p]
            g = getattr(p, "main_grad", None)
            if g is None:
                g = p.grad
            if g is None:
                continue
            g = g.float() * grad_scale + st["wd"] * p
            lr_p = lr * st["lr_mult"]
            if self.kind == "sgd":
                p.sub_(lr_p * g)
            elif self.kind == "momentum":
                st["s1"].mul_(self.mu).add_(g)
                p.sub_(lr_p * st["s1"])
            else:
                st["s2"].mul_(self.rho).add_((1 - self.rho) * g * g)
                st["s1"].mul_(self.mu).add_(lr_p * g / torch.sqrt(st["s2"] + self.eps))
                p.sub_(st["s1"])
            w16 = getattr(p, "bf16", None)
            if w16 is not None:
                w16.copy_(p)
            if "ema" in st:
                st["ema"].sub_((1 - d) * (st["ema"] - p))
        for b in self.ema_buffers:
            e = self.buffer_ema[id(b)]
            e.sub_((1 - d) * (e - b.float()))

    # ---- state for checkpoints (TF slot names) -------------------------------------------------
    def slot_variables(self):
        """(tf_name, tensor) for optimizer slots: Momentum -> <v>/Momentum, RMSProp -> <v>/RMSProp (ms),
        <v>/RMSProp_1 (mom), EMA -> <v>/ExponentialMovingAverage."""
        out = []
        for p in self.params:
            name = getattr(p, "tf_name", None)
            if name is None:
                continue
            st = self.state[p]
            if self.kind == "momentum":
                out.append((name + "/Momentum", st["s1"]))
            elif self.kind == "rmsprop":
                out.append((name + "/RMSProp", st["s2"]))
                out.append((name + "/RMSProp_1", st["s1"]))
            if "ema" in st:
                out.append((name + "/ExponentialMovingAverage", st["ema"]))
        return out

    def buffer_shadows(self):
        """[(buffer, shadow)] for the EMA-averaged non-trainable tensors (BN moving statistics)."""
        return [(b, self.buffer_ema[id(b)]) for b in self.ema_buffers]
