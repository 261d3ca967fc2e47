"""Fake-quantised (quantisation-aware) training for slim models - the ``tf.contrib.quantize``
capability behind the reference's ``--quantize`` flag (vgg/nets/mobilenet_v1_train.py:40,71-76,138-139:
``create_training_graph(quant_delay=...)``; mobilenet_v1_eval.py:126-127: ``create_eval_graph()``).

TF rewrites the graph; here the slim layers consult the active ``QuantConfig`` of their
VariableStore (set before the model's build pass, so the quantiser state variables are created,
registered and checkpointed like every other variable):

* weights of conv2d / separable_conv2d (depthwise and pointwise) / fully_connected go through an
  8-bit fake quantiser with the last-value range [min(w, 0), max(w, 0)] and TF's narrow range
  [1, 255] (``weights_quant/min``, ``weights_quant/max`` record the range used);
* each such layer's output (after its normaliser and activation) goes through an 8-bit fake
  quantiser whose range is an exponential moving average (decay 0.999) of the batch min / max in
  training and the stored average at evaluation (``act_quant/min``, ``act_quant/max``);
* until ``quant_delay`` training steps have run both quantisers are identity (the averages are
  still tracked), exactly the reference's delayed start;
* gradients use the straight-through estimator, zero outside the clamp range.

* BatchNorm after a conv2d / separable_conv2d is folded into that conv's weights, as TF's
  ``fold_batch_norms`` does (``compat/slim.py::_folded_bn``): in training the plain conv gives the
  batch moments (moving averages updated from them) and the layer computes
  ``conv(x, Q(w * gamma/sqrt(var+eps))) + beta - mean * gamma/sqrt(var+eps)``; in evaluation the
  moving moments replace the batch ones.  ``QuantConfig(fold_bn=False)`` keeps BN a separate op.

Deviation (documented): TF's optional ``freeze_bn_delay`` (switch to moving moments with the
correction factors after N steps) is not implemented -- the reference's scripts never set it.
Quantisation runs in fp32 torch ops (the model is small; not a hot path).
"""
import torch


class QuantConfig:
    def __init__(self, quant_delay=0, num_bits=8, ema_decay=0.999, is_training=True, fold_bn=True):
        self.fold_bn = bool(fold_bn)  # fold slim.batch_norm into the producing conv's weights (TF default)
        self.quant_delay = int(quant_delay or 0)
        self.num_bits = int(num_bits)
        self.ema_decay = float(ema_decay)
        self.is_training = bool(is_training)
        self.step = 0            # training steps seen (advanced by ``advance``)

    def active(self):
        return (not self.is_training) or self.step >= self.quant_delay

    def advance(self, n=1):
        self.step += n


def create_training_graph(model, quant_delay=0, num_bits=8):
    """Enable fake-quant training on a slim-built model (must be called before its build pass ->
    use ``nets_factory.build(..., quantize=QuantConfig(...))``); kept for reference call sites that
    hold a model: sets the delay / training mode of the model's existing config."""
    cfg = _cfg_of(model)
    cfg.quant_delay, cfg.num_bits, cfg.is_training = int(quant_delay or 0), int(num_bits), True
    return cfg


def create_eval_graph(model):
    cfg = _cfg_of(model)
    cfg.is_training = False
    return cfg


def _cfg_of(model):
    cfg = getattr(getattr(model, "store", None), "quant", None)
    if cfg is None:
        raise ValueError("model was not built with quantize=QuantConfig(...)")
    return cfg


def _qrange(num_bits, narrow):
    return (1 if narrow else 0), (1 << num_bits) - 1


def fake_quant(x, lo, hi, num_bits=8, narrow=False):
    """TF FakeQuantWithMinMaxVars on device (no host sync): range widened to contain 0.0 and the zero
    point rounded so 0.0 is exact; straight-through gradient inside the range.  lo / hi: 0-d or
    1-element fp32 tensors."""
    qmin, qmax = _qrange(num_bits, narrow)
    lo = torch.clamp(lo.reshape(1).float(), max=0.0)
    hi = torch.clamp(hi.reshape(1).float(), min=0.0)
    scale = (hi - lo) / float(qmax - qmin)
    scale = torch.where(scale > 1e-12, scale, torch.ones_like(scale))
    zp = torch.clamp(torch.round(qmin - lo / scale), qmin, qmax).to(torch.int32)
    y = torch.fake_quantize_per_tensor_affine(x.float(), scale, zp, qmin, qmax)
    return y.to(x.dtype)


def quantize_weights(w, var_fn, cfg):
    """w: fp32 master (Parameter); var_fn(name, init) creates/reuses the layer scope's state."""
    vmin = var_fn("weights_quant/min", 0.0)
    vmax = var_fn("weights_quant/max", 0.0)
    if not cfg.active():
        return w
    with torch.no_grad():
        lo, hi = w.detach().aminmax()
        vmin.data.copy_(torch.clamp(lo, max=0.0))
        vmax.data.copy_(torch.clamp(hi, min=0.0))
    return fake_quant(w, vmin.detach(), vmax.detach(), cfg.num_bits, narrow=True)


def quantize_activations(y, var_fn, cfg, training):
    vmin = var_fn("act_quant/min", 0.0)
    vmax = var_fn("act_quant/max", 6.0)
    if training and cfg.is_training:
        with torch.no_grad():
            d = cfg.ema_decay
            lo, hi = y.detach().float().aminmax()
            vmin.data.mul_(d).add_((1 - d) * torch.clamp(lo, max=0.0))
            vmax.data.mul_(d).add_((1 - d) * torch.clamp(hi, min=0.0))
    if not cfg.active():
        return y
    return fake_quant(y, vmin.detach(), vmax.detach(), cfg.num_bits, narrow=False)
