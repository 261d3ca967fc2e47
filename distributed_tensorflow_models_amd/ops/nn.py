"""Autograd front-end of the gfx950 kernels (NHWC bf16 activations, fp32 master params).

Each public function dispatches on the device of its input:
  * cuda tensors -> hand-written HIP kernels through ``_lib`` (hard error if missing);
  * cpu tensors  -> ``reference`` (pure torch, autograd by composition).

Weight gradients of conv/linear layers are accumulated straight into ``param.main_grad`` when
the parameter has one (a view into the flat fp32 gradient buffer that the BSP all-reduce
buckets and the fused optimizer consume), and ``grad_ready(param)`` hooks are fired so the
data-parallel engine can launch a bucket's all-reduce while backward continues.
"""
import ctypes


import torch

from . import _lib, features
from . import reference as ref
from .geometry import conv_geom, cropped_geom, live_taps, pool_geom
from .lazy import LazyBN, as_tensor

_grad_ready_hooks = []


def add_grad_ready_hook(fn):
    _grad_ready_hooks.append(fn)
    return fn


def remove_grad_ready_hook(fn):
    if fn in _grad_ready_hooks:
        _grad_ready_hooks.remove(fn)


def _notify(p):
    for h in _grad_ready_hooks:
        h(p)


# gradient-write hooks: every kernel launch (or torch op) that writes into a parameter's main_grad asks for
# the target through grad_target() right before it is enqueued, so a checker (BSPDataParallel with
# check=True / DTM_BSP_CHECK=1) can assert that the write precedes the parameter's ready notification and
# the launch of its bucket's all-reduce - a later write would be clobbered by (or missing from) the collective
_grad_write_hooks = []


def add_grad_write_hook(fn):
    _grad_write_hooks.append(fn)
    return fn


def remove_grad_write_hook(fn):
    if fn in _grad_write_hooks:
        _grad_write_hooks.remove(fn)


def grad_target(p):
    """``p.main_grad`` (or None) for a write about to be enqueued; write hooks see the parameter."""
    mg = getattr(p, "main_grad", None)
    if mg is not None:
        for h in _grad_write_hooks:
            h(p)
    return mg


# live-tap windows: a conv whose outer taps only ever read zero padding has a provably-zero weight
# gradient outside its live window (VGG-16 fc6 on a 1x1 map: 48 of 49 taps).  The window is announced
# during the forward (geometry only, identical on every rank) so the data-parallel layer can leave the
# dead part of the gradient out of the all-reduce (parallel/bsp.py).
_live_window_hooks = []


def add_live_window_hook(fn):
    _live_window_hooks.append(fn)
    return fn


def remove_live_window_hook(fn):
    if fn in _live_window_hooks:
        _live_window_hooks.remove(fn)


def _note_live_window(w, win):
    if getattr(w, "_live_win", None) == win:
        return
    try:
        w._live_win = win
    except Exception:
        return
    for h in _live_window_hooks:
        h(w, win)


def _accum_param_grad(p, g):
    """Route a computed fp32 grad for parameter p; returns what autograd should receive."""
    mg = grad_target(p)
    if mg is not None:
        mg.add_(g)
        _notify(p)
        return None
    return g


def _check(rc, what):
    if rc == -9:
        raise RuntimeError("%s: the kernel library's device state belongs to another device (one process per "
                           "GPU; csrc/kernels/workspace.hip dtm_device_ok)" % what)
    if rc == -4 and _lib.lib().dtm_ws_last_error() == -10:
        raise RuntimeError("%s: its scratch arena would have to grow while the stream is being captured into a "
                           "hipGraph (run eager warm-up steps at the captured shapes first; "
                           "csrc/kernels/workspace.hip dtm_ws_get_stream)" % what)
    if rc != 0:
        raise RuntimeError("%s failed with code %d" % (what, rc))


def weight_bf16(w):
    """bf16 compute copy of a fp32 master weight (kept fresh by the fused optimizer)."""
    w16 = getattr(w, "bf16", None)
    if w16 is None or w16.shape != w.shape:
        w16 = w.detach().to(torch.bfloat16)
        try:
            w.bf16 = w16
        except Exception:
            pass
    return w16


# flipped/transposed bf16 weight copies for dgrad ([C][R][S][K] from [K][R][S][C]).  A copy is valid
# for one weights version; FusedOptimizer bumps the version and refreshes every registered copy in
# one batched launch right after its update, so backward normally finds them ready.
WEIGHT_VERSION = [0]
FLIP_REGISTRY = {}   # (id(param), dec) -> (param, wt buffer, dec)


def dgrad_decomposable(g):
    """A stride > 1 dgrad runs as one stride-1 conv per output parity class (ConvDesc.dec, the
    decomposed flipped weight) when every class has taps (R, S >= stride)."""
    return g.stride > 1 and g.R >= g.stride and g.S >= g.stride


def _flip_attr(dec):
    return "_flip" if dec is None else ("_flippad" if dec[0] == "pad" else "_flipdec")


def weight_flipped(w, K, R, S, C, dec=None, pad_to=None):
    """Flipped / transposed bf16 dgrad copy [C][R][S][K] of w [K][R][S][C]; with dec = (stride, pad_h,
    pad_w) the same elements in the stride-decomposed layout (per output parity class (a, b) a block
    [C][Tr][Tu][K] of that class's taps, conv_igemm.hip dec_dim).  pad_to: the copy lives in the first C rows of a
    zero-initialised [pad_to][R][S][K] buffer, which is returned (the FC forward's 8-aligned output width: the
    refresh after every update rewrites the C real rows, the zero rows stay)."""
    if pad_to is not None and pad_to != C:
        dec = ("pad", int(pad_to))
    attr = _flip_attr(dec)
    c = getattr(w, attr, None)
    if c is not None and c[0] == WEIGHT_VERSION[0] and c[1].shape == (C, R, S, K) and c[2] == dec:
        return c[1] if dec is None or dec[0] != "pad" else c[1]._pad_full
    L = _lib.lib()
    if c is not None and c[1].shape == (C, R, S, K) and c[2] == dec:
        wt = c[1]
    elif dec is not None and dec[0] == "pad":
        full = torch.zeros((dec[1], R, S, K), device=w.device, dtype=torch.bfloat16)
        wt = full[:C]  # (contiguous: the first C rows)
        wt._pad_full = full
    else:
        wt = torch.empty((C, R, S, K), device=w.device, dtype=torch.bfloat16)
    if dec is None or dec[0] == "pad":
        L.dtm_weight_flip_transpose(_lib.ptr(weight_bf16(w)), _lib.ptr(wt), K, R, S, C, _lib.stream_ptr())
    else:
        L.dtm_weight_flip_transpose_dec(_lib.ptr(weight_bf16(w)), _lib.ptr(wt), K, R, S, C, int(dec[0]), int(dec[1]),
                                        int(dec[2]), _lib.stream_ptr())
    if isinstance(w, torch.nn.Parameter):
        try:
            setattr(w, attr, (WEIGHT_VERSION[0], wt, dec))
            FLIP_REGISTRY[(id(w), dec)] = (w, wt, dec)
        except Exception:
            pass
    return wt if dec is None or dec[0] != "pad" else wt._pad_full


_RETIRED = []  # device tables a captured graph may still point into (kept for the process lifetime)


def _padded_copy(src, attr, shape, fill):
    """A zero-padded copy of src (bf16 weight [Kin][N] -> [Kin][Np], or fp32 bias [N] -> [Np]) kept on the parameter and
    refreshed once per weights version: one strided copy per step instead of a zero fill + copy per use."""
    c = getattr(src, attr, None)
    if c is not None and c[0] == WEIGHT_VERSION[0] and tuple(c[1].shape) == tuple(shape):
        return c[1]
    buf = c[1] if (c is not None and tuple(c[1].shape) == tuple(shape)) else \
        torch.zeros(shape, device=src.device, dtype=fill.dtype)
    with torch.no_grad():
        if buf.dim() == 2:
            buf[:, :fill.shape[1]].copy_(fill)
        else:
            buf[:fill.shape[0]].copy_(fill)
    try:
        setattr(src, attr, (WEIGHT_VERSION[0], buf))
    except Exception:
        pass
    return buf


def refresh_flipped(stream=None):
    """After a weight update: one batched launch re-deriving every registered dgrad copy."""
    WEIGHT_VERSION[0] += 1
    if not FLIP_REGISTRY:
        return
    L = _lib.lib()
    entries = list(FLIP_REGISTRY.values())
    key = tuple((id(w), d) for w, _, d in entries)
    cache = refresh_flipped.__dict__.get("table")
    if cache is None or cache[0] != key:
        nb = L.dtm_flip_desc_bytes()
        import numpy as np
        tab = np.zeros((len(entries), nb // 8), dtype=np.int64)
        for i, (w, wt, d) in enumerate(entries):
            C, R, S, K = wt.shape
            tab[i, 0] = weight_bf16(w).data_ptr()
            tab[i, 1] = wt.data_ptr()
            tab[i, 2:4] = np.array([K, R, S, C], dtype=np.int32).view(np.int64)
            st, ph, pw = d if (d is not None and d[0] != "pad") else (1, 0, 0)
            tab[i, 4:6] = np.array([st, ph, pw, 0], dtype=np.int32).view(np.int64)
        dev_tab = torch.from_numpy(tab.view(np.uint8).reshape(-1).copy()).to(entries[0][0].device)
        if cache is not None:
            # a captured hipGraph may hold the old table's pointer (its refresh launch): never free it
            _RETIRED.append(cache[1])
        refresh_flipped.table = cache = (key, dev_tab, len(entries))
    L.dtm_weight_flip_transpose_batched(_lib.ptr(cache[1]), cache[2], stream or _lib.stream_ptr())
    for w, wt, d in entries:
        setattr(w, _flip_attr(d), (WEIGHT_VERSION[0], wt, d))


def invalidate_weight_copies(params):
    """Weights changed outside the optimizer (checkpoint restore, ASP pull, broadcast): refresh the
    bf16 compute copies and drop the flipped dgrad copies."""
    with torch.no_grad():
        for p in params:
            w16 = getattr(p, "bf16", None)
            if w16 is not None and w16.shape == p.shape:
                w16.copy_(p)
    WEIGHT_VERSION[0] += 1


# ---------------------------------------------------------------------------------------------
# convolution
class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, geom, relu):
        L = _lib.lib()
        x = x.contiguous()
        w16 = weight_bf16(w)
        y = torch.empty((geom.N, geom.P, geom.Q, geom.K), device=x.device, dtype=torch.bfloat16)
        d = geom.as_desc(_lib.ConvDesc)
        _check(L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w16), _lib.ptr(y), None, _lib.ptr(b), None, None,
                              int(relu), ctypes.byref(d), _lib.stream_ptr()), "conv_fwd")
        ctx.geom, ctx.relu, ctx.has_b = geom, relu, b is not None
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.bias_param = b
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        x, w, y = ctx.saved_tensors
        g = ctx.geom
        dy = dy.contiguous()
        gb = None
        if ctx.relu and _relu_bias_bwd_ok(dy):
            # one pass: ReLU mask from y and the bias-gradient column sums (the BN-apply backward
            # kernel with unit scale), instead of compare + where + cast + reduce torch ops
            dy, gb = _relu_bias_bwd(dy, y)
        elif ctx.relu:
            dy = torch.where(y > 0, dy, torch.zeros((), dtype=dy.dtype, device=dy.device))
        d = g.as_desc(_lib.ConvDesc)
        s = _lib.stream_ptr()
        dx = None
        if ctx.needs_input_grad[0]:
            dec = (g.stride, g.pad_h, g.pad_w) if dgrad_decomposable(g) else None
            wt = weight_flipped(w, g.K, g.R, g.S, g.C, dec)
            dx = torch.empty((g.N, g.H, g.W, g.C), device=dy.device, dtype=torch.bfloat16)
            d.dec = int(dec is not None)
            _check(L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), s), "conv_dgrad")
            d.dec = 0
        dw = None
        if ctx.needs_input_grad[1]:
            mg = grad_target(w)
            target = mg if mg is not None else torch.zeros(w.shape, device=dy.device, dtype=torch.float32)
            _check(L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(target), None, None,
                                                         ctypes.byref(d), _lib.num_cus(), s), "conv_wgrad")
            if mg is not None:
                _notify(w)
            else:
                dw = target
        db = None
        if ctx.has_b and ctx.needs_input_grad[2]:
            if gb is None:
                gb = _col_sums(dy.reshape(-1, g.K), ctx.bias_param)
            db = _accum_param_grad(ctx.bias_param, gb)
        return dx, dw, db, None, None


_UNIT_SS = {}


def _col_sums(g, param):
    """fp32 column sums of a [M][K] gradient (a bias gradient).  bf16 with K % 8 == 0 and a data-parallel gradient
    slot on the parameter (consumed at once by _accum_param_grad): one BN-statistics pass + its row reduction into the
    step's zero arena instead of a float cast + torch reduction; otherwise the torch form (its result may become
    param.grad, which must not live in the arena)."""
    K = g.shape[-1]
    if (g.is_cuda and g.dtype == torch.bfloat16 and K % 8 == 0 and K // 8 <= 256 and g.is_contiguous()
            and getattr(param, "main_grad", None) is not None):
        from .fused import arena
        st = arena.zeros((2, K), g.device)
        # (one row chunk: a fixed summation order, so bias gradients reproduce run to run - ADVICE r5)
        if _lib.lib().dtm_col_sums(_lib.ptr(g), _lib.ptr(st), g.numel() // K, K, _lib.stream_ptr()) == 0:
            return st[0]
    return g.reshape(-1, K).float().sum(0)


def _relu_bias_bwd_ok(dy):
    K = dy.shape[-1]
    return dy.dtype == torch.bfloat16 and K % 8 == 0 and K // 8 <= 256 and dy.numel() // K < (1 << 31)


def _relu_bias_bwd(dy, y):
    """g = dy * [y > 0] and sum_rows(g) (fp32) in one HIP pass (dtm_bn_apply_bwd, mode 1, unscaled)."""
    L = _lib.lib()
    K = dy.shape[-1]
    M = dy.numel() // K
    key = (dy.device, K)
    ss = _UNIT_SS.get(key)
    if ss is None:
        ss = _UNIT_SS[key] = torch.ones((4, K), device=dy.device, dtype=torch.float32)
    g = torch.empty_like(dy)
    sums = torch.zeros((4, K), device=dy.device, dtype=torch.float32)
    _check(L.dtm_bn_apply_bwd(_lib.ptr(dy), _lib.ptr(y), None, _lib.ptr(y), _lib.ptr(ss), None, None, _lib.ptr(g),
                              None, _lib.ptr(sums), None, M, K, 1, 0, 1, _lib.stream_ptr()), "relu_bias_bwd")
    return g, sums[1]


def conv2d(x, w, bias=None, stride=1, padding="SAME", relu=False, dilation=1):
    """NHWC conv. x [N,H,W,C]; w fp32 master [K,R,S,C]; bias [K] or None."""
    x = as_tensor(x)
    if dilation == 1 and isinstance(w, torch.nn.Parameter) and w.requires_grad and torch.is_grad_enabled():
        gl = conv_geom(tuple(x.shape), tuple(w.shape), stride, padding, dilation)
        win = live_taps(gl)
        if (win[1] - win[0], win[3] - win[2]) != (gl.R, gl.S):
            _note_live_window(w, win)
    if not x.is_cuda:
        return ref.conv2d(x, w, bias, stride, padding, relu, dilation)
    if dilation != 1:
        return _atrous_conv2d(x, w, bias, stride, padding, relu, dilation)
    g = conv_geom(tuple(x.shape), tuple(w.shape), stride, padding, dilation)
    r0, r1, s0, s1 = live_taps(g)
    if (r1 - r0, s1 - s0) != (g.R, g.S):
        # taps that only ever read zero padding are skipped: their products are zero, and so is
        # their weight gradient (VGG-16 fc6 on a 1x1 map: 49x fewer MACs in fwd, dgrad and wgrad)
        w = _CropTaps.apply(w, r0, r1, s0, s1)
        g = cropped_geom(g, r0, r1, s0, s1)
    if g.C % 8 != 0:
        # pad input channels with zeros (first layer: RGB) so every gather chunk is 16 B
        cp = (g.C + 7) // 8 * 8
        x = torch.nn.functional.pad(x, (0, cp - g.C))
        w = _PadChannels.apply(w, cp)
        g = conv_geom(tuple(x.shape), tuple(w.shape), stride, padding, dilation)
    if g.K % 8 != 0:
        # pad output channels (e.g. 10 / 1001 classes) to the 8-channel store granule
        kp = (g.K + 7) // 8 * 8
        wp = _PadOutChannels.apply(w, kp)
        bp = _PadOutChannels.apply(bias, kp) if bias is not None else None
        g = conv_geom(tuple(x.shape), tuple(wp.shape), stride, padding, dilation)
        y = _Conv2dFn.apply(x.to(torch.bfloat16), wp, bp, g, relu)
        return y[..., :w.shape[0]].contiguous()
    return _Conv2dFn.apply(x.to(torch.bfloat16), w, bias, g, relu)


def _atrous_conv2d(x, w, bias, stride, padding, relu, rate):
    """Dilated (atrous) conv as space-to-batch -> dense VALID conv -> batch-to-space, the
    decomposition TF's atrous_conv2d uses (the conv itself runs on the dense HIP implicit-GEMM
    kernel; the two re-layouts are plain strided copies whose backward autograd derives).

    Output pixel o = a + rate*i (phase a) only reads input pixels a + rate*(i + k), so each of the
    rate x rate phases is an ordinary conv over the phase-subsampled, padded input.  Used by the
    ResNet ``output_stride`` (atrous) mode (reference vgg/nets/resnet_utils.py:125-219)."""
    if stride != 1:
        raise ValueError("atrous conv requires stride 1 (TF atrous_conv2d has no stride)")
    g = conv_geom(tuple(x.shape), tuple(w.shape), 1, padding, rate)
    N, H, W, C = x.shape
    Hp, Wp = H + g.pad_h + g.pad_b, W + g.pad_w + g.pad_r
    Hq, Wq = -(-Hp // rate) * rate, -(-Wp // rate) * rate
    xp = torch.nn.functional.pad(x, (0, 0, g.pad_w, g.pad_r + Wq - Wp, g.pad_h, g.pad_b + Hq - Hp))
    xs = xp.reshape(N, Hq // rate, rate, Wq // rate, rate, C).permute(2, 4, 0, 1, 3, 5)
    xs = xs.reshape(rate * rate * N, Hq // rate, Wq // rate, C)
    ys = conv2d(xs, w, bias, 1, "VALID", relu)
    ho, wo, K = ys.shape[1], ys.shape[2], ys.shape[3]
    y = ys.reshape(rate, rate, N, ho, wo, K).permute(2, 3, 0, 4, 1, 5).reshape(N, ho * rate, wo * rate, K)
    return y[:, :g.P, :g.Q].contiguous()


class _Conv2dTransposeFn(torch.autograd.Function):
    """y = C^T x for the conv C: y-space -> x-space with weight w [Cx, R, S, Cy] (KRSC) and
    geometry ``geom`` (input = y-space).  Forward is C's dgrad kernel, backward is C's forward
    (dx) and C's wgrad with the roles of input / output-grad swapped (dw)."""

    @staticmethod
    def forward(ctx, x, w, geom):
        L = _lib.lib()
        s = _lib.stream_ptr()
        g = geom
        x = x.contiguous()
        w16 = weight_bf16(w)
        wt = torch.empty((g.C, g.R, g.S, g.K), device=x.device, dtype=torch.bfloat16)
        L.dtm_weight_flip_transpose(_lib.ptr(w16), _lib.ptr(wt), g.K, g.R, g.S, g.C, s)
        y = torch.empty((g.N, g.H, g.W, g.C), device=x.device, dtype=torch.bfloat16)
        d = g.as_desc(_lib.ConvDesc)
        _check(L.dtm_conv_dgrad(_lib.ptr(x), _lib.ptr(wt), _lib.ptr(y), ctypes.byref(d), s), "conv_transpose")
        ctx.geom = g
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        s = _lib.stream_ptr()
        x, w = ctx.saved_tensors
        g = ctx.geom
        dy = dy.contiguous().to(torch.bfloat16)
        d = g.as_desc(_lib.ConvDesc)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty((g.N, g.P, g.Q, g.K), device=dy.device, dtype=torch.bfloat16)
            _check(L.dtm_conv_fwd(_lib.ptr(dy), _lib.ptr(weight_bf16(w)), _lib.ptr(dx), None, None, None, None, 0,
                                  ctypes.byref(d), s), "conv_transpose_bwd_data")
        dw = None
        if ctx.needs_input_grad[1]:
            mg = grad_target(w)
            target = mg if mg is not None else torch.zeros(w.shape, device=dy.device, dtype=torch.float32)
            _check(L.dtm_conv_wgrad(_lib.ptr(dy), _lib.ptr(x), _lib.ptr(target), None, None,
                                                         ctypes.byref(d), _lib.num_cus(), s),
                   "conv_transpose_bwd_filter")
            if mg is not None:
                _notify(w)
            else:
                dw = target
        return dx, dw, None


def conv2d_transpose(x, w, bias=None, stride=2, padding="SAME", relu=False):
    """TF conv2d_transpose, NHWC.  x [N,Hx,Wx,Cx]; w fp32 master [Cx, R, S, Cy] (KRSC of the conv
    this op is the gradient of; TF filter [R,S,Cy,Cx] = w.permute(1,2,3,0)); -> [N,Hy,Wy,Cy] with
    Hy = Hx*stride (SAME) or (Hx-1)*stride+R (VALID)."""
    x = as_tensor(x)
    Cx, R, S, Cy = w.shape
    N, Hx, Wx, _ = x.shape
    if str(padding).upper() == "SAME":
        Hy, Wy = Hx * stride, Wx * stride
    else:
        Hy, Wy = (Hx - 1) * stride + R, (Wx - 1) * stride + S
    if not x.is_cuda:
        y = ref.conv2d_transpose(x, w.permute(1, 2, 3, 0), stride, padding, (Hy, Wy))
    else:
        wp, xp = w, x.to(torch.bfloat16)
        if Cy % 8:
            wp = _PadChannels.apply(wp, (Cy + 7) // 8 * 8)
        if Cx % 8:
            cxp = (Cx + 7) // 8 * 8
            wp = _PadOutChannels.apply(wp, cxp)
            xp = torch.nn.functional.pad(xp, (0, cxp - Cx))
        g = conv_geom((N, Hy, Wy, wp.shape[-1]), tuple(wp.shape), stride, padding)
        if (g.P, g.Q) != (Hx, Wx):
            raise ValueError("conv2d_transpose geometry mismatch: %s vs input %s" % ((g.P, g.Q), (Hx, Wx)))
        y = _Conv2dTransposeFn.apply(xp, wp, g)
        if Cy % 8:
            y = y[..., :Cy].contiguous()
    if bias is not None:
        y = y + bias.to(y.dtype)
    return torch.relu(y) if relu else y


class _CropTaps(torch.autograd.Function):
    """fp32 master [K,R,S,C] -> its live-tap window [K, r0:r1, s0:s1, C] (contiguous) with the bf16
    compute copy cropped alongside; the window's gradient lands in the master's main_grad slice."""

    @staticmethod
    def forward(ctx, w, r0, r1, s0, s1):
        ctx.src, ctx.win = w, (r0, r1, s0, s1)
        out = w.detach()[:, r0:r1, s0:s1, :].contiguous()
        out.bf16 = weight_bf16(w)[:, r0:r1, s0:s1, :].contiguous()
        return out

    @staticmethod
    def backward(ctx, g):
        r0, r1, s0, s1 = ctx.win
        p = ctx.src
        mg = grad_target(p)
        if mg is not None:
            mg[:, r0:r1, s0:s1, :].add_(g)
            _notify(p)
            return None, None, None, None, None
        full = torch.zeros(p.shape, device=g.device, dtype=g.dtype)
        full[:, r0:r1, s0:s1, :] = g
        return full, None, None, None, None


class _PadOutChannels(torch.autograd.Function):
    """Zero-pad dim 0 (output channels) of a fp32 weight / bias."""

    @staticmethod
    def forward(ctx, w, kp):
        ctx.k = w.shape[0]
        ctx.src = w
        pad = [0, 0] * (w.dim() - 1) + [0, kp - w.shape[0]]
        return torch.nn.functional.pad(w, pad)

    @staticmethod
    def backward(ctx, g):
        return _accum_param_grad(ctx.src, g[:ctx.k].contiguous()), None


class _PadChannels(torch.autograd.Function):
    """Zero-pad the input-channel dim of a fp32 weight; grads flow back to the unpadded master."""

    @staticmethod
    def forward(ctx, w, cp):
        ctx.c = w.shape[-1]
        ctx.src = w
        out = torch.nn.functional.pad(w, (0, cp - w.shape[-1]))
        return out

    @staticmethod
    def backward(ctx, g):
        gw = g[..., :ctx.c].contiguous()
        return _accum_param_grad(ctx.src, gw), None


# ---------------------------------------------------------------------------------------------
# batch norm (+ReLU, +residual)
class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, res, moving_mean, moving_var, training, decay, eps, relu, bessel):
        L = _lib.lib()
        s = _lib.stream_ptr()
        C = x.shape[-1]
        M = x.numel() // C
        x = x.contiguous()
        ss = torch.empty((4, C), device=x.device, dtype=torch.float32)
        if training:
            from .fused import arena  # (per-step zeroed scratch: no fill launch)
            stats = arena.zeros((2, C), x.device)
            L.dtm_bn_stats(_lib.ptr(x), _lib.ptr(stats), M, C, s)
            L.dtm_bn_finalize(_lib.ptr(stats), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(moving_mean),
                              _lib.ptr(moving_var), _lib.ptr(ss), C, float(M), float(eps), float(decay),
                              int(moving_mean is not None), int(bessel), s)
        else:
            L.dtm_bn_inference_params(_lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(moving_mean), _lib.ptr(moving_var),
                                      _lib.ptr(ss), C, float(eps), s)
        y = torch.empty_like(x)
        if res is not None:
            res = res.contiguous()
        L.dtm_bn_apply(_lib.ptr(x), _lib.ptr(ss), _lib.ptr(res), None, _lib.ptr(y), M, C,
                       1 if res is not None else 0, int(relu), s)
        ctx.training, ctx.relu, ctx.has_res = training, relu, res is not None
        ctx.gamma, ctx.beta = gamma, beta
        ctx.save_for_backward(x, ss, y if relu else None)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        s = _lib.stream_ptr()
        x, ss, y = ctx.saved_tensors
        C = x.shape[-1]
        M = x.numel() // C
        dy = dy.contiguous()
        mask_mode = 1 if ctx.relu else 0
        from .fused import arena
        sums = arena.zeros((2, C), x.device)
        L.dtm_bn_bwd_reduce(_lib.ptr(dy), _lib.ptr(x), _lib.ptr(y), _lib.ptr(ss), _lib.ptr(sums), M, C, mask_mode, s)
        dx = torch.empty_like(x)
        gout = torch.empty_like(x) if ctx.has_res else None
        L.dtm_bn_bwd_apply(_lib.ptr(dy), _lib.ptr(x), _lib.ptr(y), _lib.ptr(ss), _lib.ptr(sums), _lib.ptr(dx),
                           _lib.ptr(gout), M, C, mask_mode, int(ctx.training), s)
        dg = db = None
        if ctx.gamma is not None and ctx.needs_input_grad[1]:
            dg = _accum_param_grad(ctx.gamma, sums[1].clone())
        if ctx.beta is not None and ctx.needs_input_grad[2]:
            db = _accum_param_grad(ctx.beta, sums[0].clone())
        return dx, dg, db, gout, None, None, None, None, None, None, None


def batch_norm(x, gamma, beta, moving_mean, moving_var, training=True, decay=0.999, eps=1e-3, relu=False,
               residual=None, bessel=True):
    x = as_tensor(x)
    residual = as_tensor(residual) if residual is not None else None
    if not x.is_cuda:
        return ref.batch_norm(x, gamma, beta, moving_mean, moving_var, training, decay, eps, relu, residual, bessel)
    return _BatchNormFn.apply(x.to(torch.bfloat16), gamma, beta,
                              None if residual is None else residual.to(torch.bfloat16),
                              moving_mean, moving_var, bool(training), float(decay), float(eps), bool(relu),
                              bool(bessel))


# ---------------------------------------------------------------------------------------------
# pooling
def _pool_slot(x):
    """Join the gradient hand-off of a tensor shared with fused conv consumers (an Inception block
    input feeds three 1x1 convs and a pooling branch): see ops.fused._GradSlot."""
    from .fused import _slot_register
    return _slot_register(x)


def _pool_grad_out(slot, dx):
    """Pool backward's input gradient under the hand-off: the pool branch is built last in an
    Inception block, so its backward runs first and stashes; the last conv consumer folds the stash
    into its dgrad epilogue - no separate add over the block input."""
    from .fused import _slot_stash, _slot_take, _unstride
    if slot is None:
        return dx
    last, buf, bst = _slot_take(slot)
    if not last:
        _slot_stash(slot, dx, 1)
        return None
    if buf is not None:
        dx = dx + _unstride(slot, buf, bst)
    # (not recorded as the slot's main gradient for a tail consumer: a pool that is the last slot consumer may
    # share x with generic consumers whose gradients autograd adds out of place - the recorded tensor would then be
    # stale and the tail's in-place add lost.  Only a conv dgrad epilogue that folded the stash records it.)
    return dx


TAIL_FUSED = [0]  # tail avg-pool gradients added in place into the main-path gradient (tests / diagnostics)


def _pixel_pitch(t):
    """Element pitch between consecutive pixels of an NHWC bf16 tensor whose channels are contiguous (a concat
    gradient's channel slice: pitch = the concat width), or None."""
    if t.dim() != 4 or t.dtype != torch.bfloat16 or t.stride(3) != 1:
        return None
    ld = t.stride(2)
    if t.stride(1) != ld * t.shape[2] or t.stride(0) != t.stride(1) * t.shape[1]:
        return None
    return ld


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, slot=None):
        L = _lib.lib()
        x = x.contiguous()
        y = torch.empty((g.N, g.P, g.Q, g.C), device=x.device, dtype=x.dtype)
        arg = torch.empty((g.N, g.P, g.Q, g.C), device=x.device, dtype=torch.uint8)
        a = g.as_args(_lib.PoolArgs)
        L.dtm_maxpool_fwd(_lib.ptr(x), _lib.ptr(y), _lib.ptr(arg), ctypes.byref(a), _lib.stream_ptr())
        ctx.g, ctx.slot = g, slot
        ctx.save_for_backward(arg)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        (arg,) = ctx.saved_tensors
        g = ctx.g
        dx = torch.empty((g.N, g.H, g.W, g.C), device=dy.device, dtype=torch.bfloat16)
        a = g.as_args(_lib.PoolArgs)
        ld = _pixel_pitch(dy)
        if ld is None or L.dtm_maxpool_bwd_ld(_lib.ptr(dy), ld, _lib.ptr(arg), _lib.ptr(dx), ctypes.byref(a),
                                              _lib.stream_ptr()) != 0:
            L.dtm_maxpool_bwd(_lib.ptr(dy.contiguous()), _lib.ptr(arg), _lib.ptr(dx), ctypes.byref(a),
                              _lib.stream_ptr())
        return _pool_grad_out(ctx.slot, dx), None, None


class _MaxPoolBNReluFn(torch.autograd.Function):
    """maxpool(relu(raw*scale + shift)) without storing the normalised activation (the ResNet stem's
    BN -> ReLU -> max pool); backward returns the raw-input gradient and the [4, C] scale/shift sums."""

    @staticmethod
    def forward(ctx, raw, ss, g, unscaled=False):
        L = _lib.lib()
        y = torch.empty((g.N, g.P, g.Q, g.C), device=raw.device, dtype=torch.bfloat16)
        arg = torch.empty((g.N, g.P, g.Q, g.C), device=raw.device, dtype=torch.uint8)
        a = g.as_args(_lib.PoolArgs)
        _check(L.dtm_maxpool_bnrelu_fwd(_lib.ptr(raw), _lib.ptr(ss), _lib.ptr(y), _lib.ptr(arg), ctypes.byref(a),
                                        _lib.stream_ptr()), "maxpool_bnrelu_fwd")
        ctx.g, ctx.unscaled = g, bool(unscaled)
        ctx.save_for_backward(raw, ss, arg)
        return y

    @staticmethod
    def backward(ctx, dy):
        from .fused import arena
        L = _lib.lib()
        raw, ss, arg = ctx.saved_tensors
        g = ctx.g
        dx = torch.empty_like(raw)
        sums = arena.zeros((4, g.C), raw.device)
        a = g.as_args(_lib.PoolArgs)
        _check(L.dtm_maxpool_bnrelu_bwd(_lib.ptr(dy.contiguous()), _lib.ptr(arg), _lib.ptr(raw), _lib.ptr(ss),
                                        _lib.ptr(dx), _lib.ptr(sums), ctypes.byref(a), int(ctx.unscaled),
                                        _lib.stream_ptr()), "maxpool_bnrelu_bwd")
        return dx, sums, None, None


def max_pool(x, kernel, stride, padding="VALID", grad_handoff=False):
    """``grad_handoff``: x is also read by fused conv consumers whose backward is certain to run
    (an Inception block input); the pool then joins their gradient hand-off instead of leaving an
    add to autograd.  Off by default: a registered consumer whose backward never runs (an unused
    branch) would strand the hand-off."""
    if isinstance(x, LazyBN) and x.relu and x.raw.is_cuda and x.raw.dtype == torch.bfloat16 \
            and x.raw.shape[-1] % 8 == 0 and x.raw.is_contiguous():
        g = pool_geom(tuple(x.raw.shape), kernel, stride, padding)
        if g.KH * g.KW <= 255 and -(-g.KH // g.SH) <= 3 and -(-g.KW // g.SW) <= 3:
            return _MaxPoolBNReluFn.apply(x.raw, x.ss.contiguous(), g, x.unscaled)
    x = as_tensor(x)
    if not x.is_cuda:
        return ref.max_pool(x, kernel, stride, padding)
    g = pool_geom(tuple(x.shape), kernel, stride, padding)
    if g.KH * g.KW > 255:
        raise ValueError("max-pool window too large for the uint8 argmax")
    xb = x.to(torch.bfloat16)
    share = grad_handoff and xb is x and xb.is_contiguous()
    return _MaxPoolFn.apply(xb, g, _pool_slot(xb) if share else None)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, count_pad, slot=None, tail=None):
        L = _lib.lib()
        y = torch.empty((g.N, g.P, g.Q, g.C), device=x.device, dtype=torch.bfloat16)
        a = g.as_args(_lib.PoolArgs)
        L.dtm_avgpool_fwd(_lib.ptr(x.contiguous()), _lib.ptr(y), ctypes.byref(a), int(count_pad), _lib.stream_ptr())
        ctx.g, ctx.cp, ctx.slot, ctx.tail = g, count_pad, slot, tail
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        g = ctx.g
        a = g.as_args(_lib.PoolArgs)
        main = ctx.tail.main if ctx.tail is not None else None
        if main is not None and tuple(main.shape) == (g.N, g.H, g.W, g.C) and main.dtype == torch.bfloat16 \
                and main.is_contiguous() and L.dtm_avgpool_bwd_acc(_lib.ptr(dy.contiguous()), _lib.ptr(main),
                                                                    ctypes.byref(a), int(ctx.cp),
                                                                    _lib.stream_ptr()) == 0:
            # (tail consumer: its gradient added into the main path's, which autograd still holds for x)
            ctx.tail.main = None
            TAIL_FUSED[0] += 1
            return None, None, None, None, None
        dx = torch.empty((g.N, g.H, g.W, g.C), device=dy.device, dtype=torch.bfloat16)
        L.dtm_avgpool_bwd(_lib.ptr(dy.contiguous()), _lib.ptr(dx), ctypes.byref(a), int(ctx.cp), _lib.stream_ptr())
        return _pool_grad_out(ctx.slot, dx), None, None, None, None


def avg_pool(x, kernel, stride, padding="VALID", count_pad=False, grad_handoff=False, grad_tail=False):
    """TF avg pool (SAME excludes the padding from the divisor unless count_pad); grad_handoff as in
    max_pool.  ``grad_tail``: x's other consumers are all slot consumers recorded AFTER this pool (Inception's
    aux head on the Mixed_6e output): the backward adds into their gradient in place (ops.fused._slot_tail)."""
    x = as_tensor(x)
    if not x.is_cuda:
        return ref.avg_pool(x, kernel, stride, padding, count_pad)
    g = pool_geom(tuple(x.shape), kernel, stride, padding)
    xb = x.to(torch.bfloat16)
    share = grad_handoff and xb is x and xb.is_contiguous()
    tail = None
    # (the tail needs every other consumer of x on the slot: with fused_bn off the convs take the generic path and
    # autograd sums their gradients, so the tail stays off)
    if (grad_tail and not share and xb is x and xb.is_contiguous() and features.on("pool_tail")
            and features.on("fused_bn")):
        from .fused import _slot_tail
        tail = _slot_tail(xb)
    return _AvgPoolFn.apply(xb, g, bool(count_pad), _pool_slot(xb) if share else None, tail)


class _GlobalAvgFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_bf16):
        L = _lib.lib()
        N, H, W, C = x.shape
        y = torch.empty((N, C), device=x.device, dtype=torch.bfloat16 if out_bf16 else torch.float32)
        (L.dtm_global_avg_fwd_bf16 if out_bf16 else L.dtm_global_avg_fwd)(_lib.ptr(x.contiguous()), _lib.ptr(y), N,
                                                                          H * W, C, _lib.stream_ptr())
        ctx.shape = x.shape
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        N, H, W, C = ctx.shape
        dx = torch.empty((N, H, W, C), device=dy.device, dtype=torch.bfloat16)
        if dy.dtype == torch.bfloat16:  # (the bf16-output form: its gradient comes back in bf16)
            L.dtm_global_avg_bwd_bf16(_lib.ptr(dy.contiguous()), _lib.ptr(dx), N, H * W, C, _lib.stream_ptr())
        else:
            L.dtm_global_avg_bwd(_lib.ptr(dy.float().contiguous()), _lib.ptr(dx), N, H * W, C, _lib.stream_ptr())
        return dx, None


def global_avg_pool(x, out_bf16=False):
    """mean over H, W -> [N, C] fp32 (out_bf16: bf16, rounded as a cast of the fp32 mean would be - for a consumer that
    computes in bf16 anyway, e.g. the logits layer)."""
    x = as_tensor(x)
    if not x.is_cuda:
        return ref.global_avg_pool(x)
    return _GlobalAvgFn.apply(x.to(torch.bfloat16), bool(out_bf16))


# ---------------------------------------------------------------------------------------------
# loss
def _rows(t):
    """(t, row pitch): a [B][K] tensor with unit column stride is read in place (an FC's padded output viewed as its
    first K columns), anything else made contiguous."""
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return t, t.stride(0)
    t = t.contiguous()
    return t, t.shape[1]


class _SoftmaxXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, smoothing, row_weight):
        L = _lib.lib()
        logits, ld = _rows(logits)
        B, K = logits.shape
        loss = torch.empty((B,), device=logits.device, dtype=torch.float32)
        dl = torch.empty((B, K), device=logits.device, dtype=logits.dtype)
        lab = labels.to(torch.int32).contiguous()
        L.dtm_softmax_xent(_lib.ptr(logits), int(logits.dtype == torch.bfloat16), _lib.ptr(lab), _lib.ptr(loss),
                           _lib.ptr(dl), B, K, float(smoothing), 1.0,
                           _lib.ptr(row_weight.float().contiguous()) if row_weight is not None else None, ld,
                           _lib.stream_ptr())
        ctx.save_for_backward(dl)
        return loss

    @staticmethod
    def backward(ctx, gl):
        (dl,) = ctx.saved_tensors
        B, N = dl.shape
        if not dl.is_cuda or gl.dtype != torch.float32 or gl.dim() != 1 or gl.stride(0) not in (0, 1):
            return (dl.float() * gl.view(-1, 1)).to(dl.dtype), None, None, None
        # one HIP pass (dl * gl per row); an FC producer's 8-aligned padded width is written here with zero columns,
        # and its backward takes that buffer as is (_LinearHipFn: no zero fill + copy of the padded operand)
        Np = _pad8(N) if dl.dtype == torch.bfloat16 else N
        out = torch.empty((B, Np), device=dl.device, dtype=dl.dtype)
        _check(_lib.lib().dtm_scale_rows_pad(_lib.ptr(dl), int(dl.dtype == torch.bfloat16), _lib.ptr(gl),
                                             int(gl.stride(0)), _lib.ptr(out), B, N, Np, _lib.stream_ptr()),
               "scale_rows_pad")
        if Np == N:
            return out, None, None, None
        g = out[:, :N]
        g._dtm_pad_base = out
        return g, None, None, None


def softmax_cross_entropy(logits, labels, smoothing=0.0, row_weight=None):
    """Per-row softmax cross-entropy with TF label smoothing."""
    if not logits.is_cuda:
        return ref.softmax_cross_entropy(logits, labels, smoothing, row_weight)
    if logits.dtype not in (torch.float32, torch.bfloat16):
        logits = logits.float()
    return _SoftmaxXentFn.apply(logits, labels, float(smoothing), row_weight)


def _scaled_rows_grad(dl, gl):
    """dl * gl[0] for every row (gl: the 0-dim upstream gradient) in one HIP pass, written into the FC producer's
    8-aligned padded width as _SoftmaxXentFn.backward does."""
    B, N = dl.shape
    Np = _pad8(N) if dl.dtype == torch.bfloat16 else N
    out = torch.empty((B, Np), device=dl.device, dtype=dl.dtype)
    _check(_lib.lib().dtm_scale_rows_pad(_lib.ptr(dl), int(dl.dtype == torch.bfloat16), _lib.ptr(gl), 0, _lib.ptr(out),
                                         B, N, Np, _lib.stream_ptr()), "scale_rows_pad")
    if Np == N:
        return out
    g = out[:, :N]
    g._dtm_pad_base = out
    return g


class _MeanXentFn(torch.autograd.Function):
    """sum_h w_h * mean_r xent(logits_h[r], labels[r]) as ONE scalar op: each head's xent kernel writes its gradient
    pre-scaled by w_h / B, one launch combines the per-row losses (dtm_loss_combine), and the backward is one
    scale pass per head - in place of the per-head mean, the weight multiply, the add and their backwards
    (eight small launches at ~4.7 us each in a captured Inception step)."""

    @staticmethod
    def forward(ctx, labels, smoothing, weights, *logits):
        L = _lib.lib()
        B = labels.shape[0]
        lab = labels.to(torch.int32).contiguous()
        losses = torch.empty((len(logits), B), device=lab.device, dtype=torch.float32)
        dls = []
        for i, (lg, w) in enumerate(zip(logits, weights)):
            lg, ld = _rows(lg)
            dl = torch.empty(lg.shape, device=lg.device, dtype=lg.dtype)
            L.dtm_softmax_xent(_lib.ptr(lg), int(lg.dtype == torch.bfloat16), _lib.ptr(lab), _lib.ptr(losses[i]),
                               _lib.ptr(dl), B, lg.shape[1], float(smoothing), float(w) / B, None, ld,
                               _lib.stream_ptr())
            dls.append(dl)
        out = torch.empty((), device=lab.device, dtype=torch.float32)
        ws = (ctypes.c_float * len(weights))(*[float(w) / B for w in weights])
        _check(L.dtm_loss_combine(_lib.ptr(losses), len(logits), B, ctypes.cast(ws, ctypes.c_void_p), _lib.ptr(out),
                                  _lib.stream_ptr()), "loss_combine")
        ctx.save_for_backward(*dls)
        return out

    @staticmethod
    def backward(ctx, gl):
        gl = gl.float().reshape(1).contiguous()
        return (None, None, None) + tuple(_scaled_rows_grad(dl, gl) for dl in ctx.saved_tensors)


def mean_xent_loss(heads, labels, smoothing=0.0):
    """sum over (logits, weight) heads of weight * mean softmax cross-entropy (the training loss with Inception's
    weighted aux head); one fused op on the GPU, the plain composition elsewhere."""
    heads = [(lg, float(w)) for lg, w in heads]
    ok = all(lg.is_cuda and lg.dim() == 2 and lg.dtype in (torch.float32, torch.bfloat16) for lg, _ in heads)
    if ok and labels.is_cuda and 1 <= len(heads) <= 4 and labels.shape[0] <= 65535:
        return _MeanXentFn.apply(labels, float(smoothing), [w for _, w in heads], *[lg for lg, _ in heads])
    loss = None
    for lg, w in heads:
        term = softmax_cross_entropy(lg, labels, smoothing).mean()
        term = term if w == 1.0 else w * term
        loss = term if loss is None else loss + term
    return loss


# ---------------------------------------------------------------------------------------------
# fully connected (reference cnn/cifar10.py:262-279 local3/local4,
# inception/slim/ops.py:305,317 logits / aux FC).  An FC layer IS a 1x1 convolution over a 1x1
# image, so it runs on the hand-written MFMA implicit-GEMM kernels (conv_igemm.hip) with the bias and
# ReLU in the GEMM epilogue:  forward  y[B][N]  = conv(x [B,1,1,Kin], W^T [N][Kin])  (the dgrad copy of
#                            the [Kin][N] TF-layout weight, refreshed with the conv weights);
#                            dgrad    dx[B][Kin] = conv(dy [B,1,1,N], W [Kin][N]);
#                            wgrad    dW[Kin][N] = conv_wgrad with the roles of x / dy swapped.
# Output widths that are not a multiple of 8 (logits: 10, 1001) run on zero-padded copies.
PAD_BASE_USED = [0]  # FC backwards that took the loss backward's padded gradient buffer as is (tests)


def _pad8(n):
    return (n + 7) // 8 * 8


def _fc_desc(B, C, K):
    return _lib.ConvDesc(B, 1, 1, C, K, 1, 1, 1, 1, 1, 0, 0, 0)


class _LinearHipFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        L = _lib.lib()
        s = _lib.stream_ptr()
        Kin, N = w.shape
        Np = _pad8(N)
        B = x.shape[0]
        x16 = x.to(torch.bfloat16).contiguous()
        if Np == N:
            wt = weight_flipped(w, Kin, 1, 1, N).view(N, Kin)
            bias = b.float().contiguous() if b is not None else None
        else:  # (padded copies kept per weights version: no zero fill + copy per step)
            wt = weight_flipped(w, Kin, 1, 1, N, pad_to=Np).view(Np, Kin)
            bias = _padded_copy(b, "_pad8", (Np,), b.detach().float()) if b is not None else None
        y = torch.empty((B, Np), device=x.device, dtype=torch.bfloat16)
        d = _fc_desc(B, Kin, Np)
        _check(L.dtm_conv_fwd(_lib.ptr(x16), _lib.ptr(wt), _lib.ptr(y), None, _lib.ptr(bias), None, None, int(relu),
                              ctypes.byref(d), s), "fc_fwd")
        if Np != N:
            # the first N columns, read in place by the loss (ops.nn._rows); a consumer needing a dense tensor copies
            y = y[:, :N] if not relu else y[:, :N].contiguous()
        ctx.save_for_backward(x16, w, y if relu else None)
        ctx.b, ctx.relu = b, relu
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        s = _lib.stream_ptr()
        x16, w, y = ctx.saved_tensors
        Kin, N = w.shape
        Np = _pad8(N)
        B = x16.shape[0]
        gb = None
        base = getattr(dy, "_dtm_pad_base", None)
        if (base is not None and Np != N and not ctx.relu and base.dtype == torch.bfloat16
                and tuple(base.shape) == (B, Np)):
            # the loss backward already wrote this gradient into a zero-padded [B][Np] buffer (_SoftmaxXentFn)
            PAD_BASE_USED[0] += 1
            dyp = base
            dy16 = base[:, :N]
        else:
            dy = dy.contiguous()
            if ctx.relu and ctx.b is not None and _relu_bias_bwd_ok(dy):
                dy, gb = _relu_bias_bwd(dy, y)  # mask + bias-gradient sums in one HIP pass
            elif ctx.relu:
                dy = torch.where(y > 0, dy, torch.zeros((), dtype=dy.dtype, device=dy.device))
            dy16 = dy.to(torch.bfloat16).contiguous()
            if Np != N:
                dyp = torch.zeros((B, Np), device=dy.device, dtype=torch.bfloat16)
                dyp[:, :N].copy_(dy16)
            else:
                dyp = dy16
        dx = None
        if ctx.needs_input_grad[0]:
            if Np == N:
                w16 = weight_bf16(w)
            else:
                w16 = _padded_copy(w, "_pad8w", (Kin, Np), weight_bf16(w))
            dx = torch.empty((B, Kin), device=dy.device, dtype=torch.bfloat16)
            d = _fc_desc(B, Np, Kin)
            _check(L.dtm_conv_fwd(_lib.ptr(dyp), _lib.ptr(w16), _lib.ptr(dx), None, None, None, None, 0,
                                  ctypes.byref(d), s), "fc_dgrad")
        dw = None
        if ctx.needs_input_grad[1]:
            mg = grad_target(w)
            direct = mg is not None and Np == N
            target = mg if direct else torch.zeros((Kin, Np), device=dy.device, dtype=torch.float32)
            d = _fc_desc(B, Np, Kin)  # "input" dy (C = Np), "output gradient" x (K = Kin): dW[Kin][Np]
            _check(L.dtm_conv_wgrad(_lib.ptr(dyp), _lib.ptr(x16), _lib.ptr(target), None, None,
                                                 ctypes.byref(d), _lib.num_cus(), s), "fc_wgrad")
            if direct:
                _notify(w)
            else:
                dw = _accum_param_grad(w, target[:, :N] if Np != N else target)
        db = None
        if ctx.b is not None and ctx.needs_input_grad[2]:
            if gb is None:
                gb = _col_sums(dyp, ctx.b)[:N] if Np != N else _col_sums(dy16, ctx.b)
            db = _accum_param_grad(ctx.b, gb)
        return dx, dw, db, None


class _LinearFn(torch.autograd.Function):
    """hipBLASLt fallback (input width not a multiple of 8)."""
    @staticmethod
    def forward(ctx, x, w, b, relu):
        w16 = weight_bf16(w)
        x16 = x.to(torch.bfloat16)
        if b is not None:  # bias in the GEMM epilogue (w stored TF-style [in, out])
            y = torch.addmm(b.to(torch.bfloat16), x16, w16)
        else:
            y = x16 @ w16
        if relu:
            y = torch.relu(y)
        ctx.save_for_backward(x16, w, y if relu else None)
        ctx.b, ctx.relu = b, relu
        return y

    @staticmethod
    def backward(ctx, dy):
        x16, w, y = ctx.saved_tensors
        gb = None
        dy = dy.contiguous()
        if ctx.relu and ctx.b is not None and _relu_bias_bwd_ok(dy):
            dy, gb = _relu_bias_bwd(dy, y)  # mask + bias-gradient sums in one HIP pass
        elif ctx.relu:
            dy = torch.where(y > 0, dy, torch.zeros((), dtype=dy.dtype, device=dy.device))
        dy16 = dy.to(torch.bfloat16)
        dx = dy16 @ weight_bf16(w).t() if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            gw = (x16.t() @ dy16).float()
            dw = _accum_param_grad(w, gw)
        db = None
        if ctx.b is not None and ctx.needs_input_grad[2]:
            db = _accum_param_grad(ctx.b, gb if gb is not None else dy16.float().sum(0))
        return dx, dw, db, None


def linear(x, w, b=None, relu=False):
    """x [B, in] @ w [in, out] (+b)."""
    x = as_tensor(x)
    if not x.is_cuda:
        y = x.float() @ w
        if b is not None:
            y = y + b
        return torch.relu(y) if relu else y
    if w.shape[0] % 8 == 0 and x.dim() == 2:
        return _LinearHipFn.apply(x, w, b, bool(relu))
    return _LinearFn.apply(x, w, b, bool(relu))
