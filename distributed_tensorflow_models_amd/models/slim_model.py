"""Wrap functional slim-style model code (compat.slim) as an nn.Module.

The first (build) pass creates every variable in a private VariableStore with its TF name; the
Module registers them so ``.to(device)``, optimizers, DP buckets and the Saver see them.  Each
forward re-executes the model function, re-using the variables by name (graph = code).
"""
import re

import torch

from ..compat import slim


class SlimModel(torch.nn.Module):
    def __init__(self, fn, image_size, num_classes=None, in_channels=3, build_batch=1, name=None, quantize=None,
                 **kw):
        super().__init__()
        self.fn, self.kw = fn, kw
        self.num_classes = num_classes
        self.default_image_size = image_size
        self.scope = name or getattr(fn, "__name__", "slim_model")
        self.store = slim.VariableStore()
        # compat.quantize.QuantConfig: fake-quant graph (its state variables are created by the
        # build pass below, so they are registered and checkpointed like the weights)
        self.store.quant = quantize
        hw = image_size if isinstance(image_size, (tuple, list)) else (image_size, image_size)
        # build in training mode so training-only variables (e.g. NASNet aux heads) exist too;
        # the pass's moving-statistics update is undone below (moving_* are constant-initialised)
        saved_q = None
        if quantize is not None:  # the build pass must not move the quantiser averages
            saved_q, quantize.is_training = quantize.is_training, False
        with torch.no_grad():
            self._run(torch.zeros(max(build_batch, 2), hw[0], hw[1], in_channels), training=True, end_points=None)
            for n, v in self.store.vars.items():
                if n.endswith("moving_mean"):
                    v.data.zero_()
                elif n.endswith("moving_variance"):
                    v.data.fill_(1.0)
        if quantize is not None:
            quantize.is_training = saved_q
        for n, v in self.store.vars.items():
            if v.dtype.is_floating_point:
                self.register_parameter(re.sub(r"[^0-9a-zA-Z_]", "_", n), v)
            else:
                self.register_buffer(re.sub(r"[^0-9a-zA-Z_]", "_", n), v.data)

    def _run(self, x, training, end_points):
        with slim.use_store(self.store):
            slim.begin_pass()
            with slim.training_mode(training):
                kw = dict(self.kw)
                if self.num_classes is not None:
                    kw["num_classes"] = self.num_classes
                out = self.fn(x, is_training=training, **kw)
        if isinstance(out, tuple) and len(out) == 2 and isinstance(out[1], dict):
            out, ep = out
            if end_points is not None:
                end_points.update(ep)
        return out

    def forward(self, x, training=True, end_points=None):
        out = self._run(x, training, end_points)
        q = self.store.quant
        if training and q is not None and q.is_training:
            q.advance()  # one training forward = one step of the quant_delay count
        return out
