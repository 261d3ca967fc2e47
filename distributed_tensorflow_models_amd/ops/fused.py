"""Conv + BatchNorm(+ReLU)(+residual) fusion on the HIP path.

A BatchNorm that follows a conv is split into:
  * statistics  - accumulated in the producing conv's epilogue (``_ConvBNFn``),
  * finalize    - per-channel scale/shift (+ moving averages), fused into the statistics reduction
                  (``_ConvBNFn``; ``_BNFinalizeFn`` is the standalone form),
  * apply       - either folded into the NEXT conv's operand prologue (the normalised activation is
                  never written to HBM: ``LazyBN`` consumed by ``conv_bn``), or materialised once by
                  ``_BNApplyFn`` (block outputs, residual add, pool inputs).
Each piece is an autograd Function with a hand-written backward kernel, so gradients compose
exactly to TF's fused BatchNorm gradient (tests/test_fused_gpu.py checks it against torch).
"""
import ctypes

import torch

from . import _lib, features
from .geometry import conv_geom
from .lazy import LazyBN, Subsampled, as_tensor  # noqa: F401
from .nn import _accum_param_grad, _check, _notify, dgrad_decomposable, grad_target, weight_bf16, weight_flipped


class ZeroArena:
    """Per-step pool of zero-initialised fp32 scratch (BN statistics, per-channel grad sums).

    One memset at step start replaces ~150 small zero-fill kernels per ResNet-50 step.  Only used
    between ``begin_step`` and ``end_step`` (the training engine brackets every step)."""

    def __init__(self, floats=1 << 22):
        self.floats = floats
        self.buf = None
        self.off = 0
        self.high = 0
        self.active = False

    def begin_step(self, device):
        if self.buf is None or self.buf.device != device:
            self.buf = torch.zeros(self.floats, device=device, dtype=torch.float32)
            self.high = 0
        elif self.high:
            self.buf[:self.high].zero_()
        self.off = 0
        self.active = True

    def end_step(self):
        self.high = max(self.high, self.off)
        self.active = False

    def zeros(self, shape, device):
        n = 1
        for s in shape:
            n *= int(s)
        if self.active and self.buf is not None and self.buf.device == device:
            n_al = (n + 63) // 64 * 64
            if self.off + n_al <= self.floats:
                v = self.buf[self.off:self.off + n].view(*shape)
                self.off += n_al
                return v
        return torch.zeros(shape, device=device, dtype=torch.float32)


arena = ZeroArena()


class _GradSlot:
    """Gradient hand-off for a tensor read by several fused ops (a ResNet block input feeds conv1
    and the shortcut).  Every consumer's backward but the last stashes its input-gradient here and
    returns None; the last one folds the stash into its own dgrad epilogue (``add_src``), so the
    autograd engine never launches a separate add over the whole activation.  A stash may be the
    gradient of a stride-s subsample of the tensor (``stride`` > 1): the dgrad epilogue adds it at
    the subsampled pixels."""
    __slots__ = ("pending", "buf", "stride", "shape", "main", "tail")

    def __init__(self, shape):
        self.pending = 0
        self.buf = None
        self.stride = 1
        self.shape = tuple(shape)
        self.main = None  # the gradient the last consumer returned (a tail consumer may still add into it)
        self.tail = False  # a tail consumer is registered (only then is main kept)


class _BNOutInfo:
    """Block-output BN-apply y = relu(x*scale+shift [+ res]) whose backward can run inside the dgrad
    epilogue of the conv that consumes y last (dtm_conv_dgrad_bnout): that conv writes g = d(y) * mask
    and the scale/shift gradient sums; the BN-apply's own backward then only hands them on."""
    __slots__ = ("mask", "x", "r", "sums", "g")

    def __init__(self, mask, x, r):
        self.mask, self.x, self.r = mask, x, r
        self.sums = None  # [4 or 8, C]: sum g*x, sum g, 0, 0 (, sum g*r, sum g, 0, 0)  (set by the fusing dgrad)
        self.g = None     # the tensor the fusing dgrad returned


BNOUT_FUSED = [0]  # count of block-output BN backwards absorbed by a dgrad epilogue (tests / diagnostics)


def _bnout_enabled():
    return features.on("bnout_fuse")


def _bnout_strided():
    """The dgrad-epilogue BN-apply backward also for the outputs of stride-2 units (strided identity residual):
    part of feature bnout_fuse (profiles/ab/r3_ab_dgrp_bnst.log)."""
    return features.on("bnout_fuse")


def _slot_register(x):
    if not (torch.is_grad_enabled() and x.requires_grad and x.is_cuda):
        return None
    s = getattr(x, "_dtm_slot", None)
    if s is None:
        s = _GradSlot(x.shape)
        try:
            x._dtm_slot = s
        except Exception:
            return None
    s.pending += 1
    return s


def _slot_tail(x):
    """The slot of x for a tail consumer (Inception's aux-head pool): one whose backward the engine runs after
    every registered consumer's (it was recorded before them) and that is not counted as pending.  It adds its
    gradient in place into the one the last consumer returned (``_slot_done``) and returns None; when that is
    absent (the order differs, or no consumer recorded one) it returns its own gradient as usual.  Only for a
    tensor whose other consumers all use the slot: an autograd-added gradient would make the recorded one stale."""
    if not (torch.is_grad_enabled() and x.requires_grad and x.is_cuda):
        return None
    s = getattr(x, "_dtm_slot", None)
    if s is None:
        s = _GradSlot(x.shape)
        try:
            x._dtm_slot = s
        except Exception:
            return None
    s.tail = True
    return s


def _slot_done(slot, dx):
    """Record the full gradient the last consumer returns (for a tail consumer)."""
    if slot is not None and slot.tail and dx is not None and slot.pending == 0:
        slot.main = dx
    return dx


def _unstride(slot, g, stride):
    """Full-resolution gradient of x from the gradient of x[:, ::stride, ::stride]."""
    if stride == 1:
        return g
    full = torch.zeros(slot.shape, device=g.device, dtype=g.dtype)
    full[:, ::stride, ::stride, :] = g
    return full


def _slot_take(slot):
    """-> (is_last_consumer, stashed_gradient_or_None, its stride)"""
    if slot is None:
        return True, None, 1
    slot.pending -= 1
    buf, stride = slot.buf, slot.stride
    if slot.pending == 0:
        slot.buf, slot.stride = None, 1
        return True, buf, stride
    return False, buf, stride


def _slot_stash(slot, g, stride=1):
    if slot.buf is None:
        slot.buf, slot.stride = g, stride
    elif slot.stride == stride:
        slot.buf = slot.buf + g
    else:
        slot.buf, slot.stride = _unstride(slot, slot.buf, slot.stride) + _unstride(slot, g, stride), 1


def _full_window(g):
    """A VALID conv whose kernel covers the whole input (1x1 output, e.g. Inception's 5x5 aux conv on its 5x5
    map): its dgrad is the plain GEMM dx[n, (r, s, c)] = dy[n, :] . W[:, (r, s, c)]; as an implicit-GEMM conv
    over the zero-padded dy it ran 25x the work in 25 blocks (282 us) - see _full_window_dgrad_act."""
    return g.P == 1 and g.Q == 1 and g.pad_h == 0 and g.pad_w == 0 and g.R == g.H and g.S == g.W


def _full_window_dgrad_act(g, dy, w, x_raw, in_ss, d_in, dx, unscaled, add_src=None):
    """dgrad of a full-window conv with the input's BN+ReLU backward, on the MFMA conv kernels: the GEMM
    dx[n, (r, s, c)] = dy[n, :] . W[:, (r, s, c)] is the dgrad of a 1x1 conv from R*S*C input channels to K outputs
    on a 1x1 map, whose transposed weight [R*S*C][K] is the flipped-weight copy of W viewed as [K][1][1][R*S*C]
    (cached and refreshed by the optimizer like every dgrad copy).  The act epilogue sees pixel n's R*S*C
    channels, i.e. x_raw[n] flattened, so it takes the BN scale / shift tiled R*S times and its partial sums
    [sum g*x_raw | sum g] per (r, s, c) are folded over the R*S taps into d_in[0:2]."""
    L = _lib.lib()
    s = _lib.stream_ptr()
    rsc, rs = g.R * g.S * g.C, g.R * g.S
    wt = weight_flipped(w, g.K, 1, 1, rsc)
    d = _lib.ConvDesc(g.N, 1, 1, rsc, g.K, 1, 1, 1, 1, 1, 0, 0, 0, 0)
    ss_t = in_ss[:2].repeat(1, rs)  # [2][R*S*C]: channel (r, s, c) -> the BN's channel c
    sums = arena.zeros((2, rsc), dy.device)
    _check(L.dtm_conv_dgrad_ex(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d),
                               _lib.ptr(add_src) if add_src is not None else None, 1, _lib.ptr(x_raw), _lib.ptr(ss_t),
                               _lib.ptr(sums), int(unscaled), s), "conv_dgrad_act(full window)")
    torch.sum(sums.view(2, rs, g.C), 1, out=d_in[0:2])


# ---------------------------------------------------------------------------------------------
class _ConvBNFn(torch.autograd.Function):
    """Training: (y_raw, ss) = conv(relu(x_raw*in_scale+in_shift) or x_raw, w) with the BatchNorm
    statistics from the conv epilogue and the finalize (ss = [scale; shift; mean; rstd], moving averages)
    fused into the statistics reduction.  Inference (bn=None): y_raw only.
    Backward: the finalize backward is folded into the stats-combine pass (dgamma / dbeta included)."""

    @staticmethod
    def forward(ctx, x, in_ss, w, gamma, beta, geom, bn, slot=None, in_unscaled=False, x_mat=None, grp=None):
        L = _lib.lib()
        s = _lib.stream_ptr()
        # (popped: the group must not keep the members' outputs - ctx -> group -> output -> grad_fn -> ctx would be
        # a reference cycle through C++ autograd nodes that the garbage collector cannot break: a per-step leak)
        pre = grp[0].fwd.pop(id(w), None) if (grp is not None and grp[0].fwd is not None) else None
        if pre is not None:
            # computed by the group's merged forward (_SiblingGroup.forward_all): nothing to launch
            ctx.geom, ctx.slot, ctx.grp, ctx.in_unscaled = geom, slot, grp, bool(in_unscaled)
            ctx.mat = False
            ctx.bnout = getattr(x, "_dtm_bnout", None)
            ctx.has_gamma, ctx.has_beta = gamma is not None, beta is not None
            y, ss = pre
            if ss is not None:
                ctx.count = float(geom.N * geom.P * geom.Q)
            ctx.save_for_backward(x, in_ss, w, y, ss, gamma, beta, None)
            return y if ss is None else (y, ss)
        w16 = weight_bf16(w)
        y = torch.empty((geom.N, geom.P, geom.Q, geom.K), device=x.device, dtype=torch.bfloat16)
        d = geom.as_desc(_lib.ConvDesc)
        # x_mat: relu(x*scale+shift) already materialised (``_prologue_mode`` 'mat'): forward conv and
        # wgrad read it without the prologue; the dgrad epilogue still does the activation backward from
        # the raw x and in_ss, so the materialisation has no backward pass of its own
        ctx.mat = x_mat is not None
        sc = in_ss[0] if (in_ss is not None and x_mat is None) else None
        sh = in_ss[1] if (in_ss is not None and x_mat is None) else None
        if x_mat is not None:
            x, x_raw = x_mat, x
        else:
            x_raw = None
        ss = None
        if bn is not None:
            ss = torch.empty((4, geom.K), device=x.device, dtype=torch.float32)
            count = float(geom.N * geom.P * geom.Q)
            _check(L.dtm_conv_fwd_bn(_lib.ptr(x), _lib.ptr(w16), _lib.ptr(y), _lib.ptr(sc), _lib.ptr(sh),
                                     _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(bn.moving_mean),
                                     _lib.ptr(bn.moving_variance), _lib.ptr(ss), count, float(bn.eps),
                                     float(bn.decay), 1, int(bn.bessel), ctypes.byref(d), s), "conv_fwd_bn")
            ctx.count = count
        else:
            _check(L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w16), _lib.ptr(y), None, None, _lib.ptr(sc), _lib.ptr(sh), 0,
                                  ctypes.byref(d), s), "conv_fwd")
        ctx.geom = geom
        ctx.slot = slot
        ctx.grp = grp  # (_SiblingGroup, member index): backward merged with the sibling 1x1 convs of x
        ctx.in_unscaled = bool(in_unscaled)
        # the input is a block output whose BN-apply backward this conv's dgrad can absorb (if it turns
        # out to be the input's last consumer)
        ctx.bnout = getattr(x, "_dtm_bnout", None) if (in_ss is None and x_mat is None) else None
        ctx.has_gamma, ctx.has_beta = gamma is not None, beta is not None
        ctx.save_for_backward(x, in_ss, w, y, ss, gamma, beta, x_raw)
        if ss is None:
            return y
        return y, ss

    @staticmethod
    def backward(ctx, dy, dss=None):
        L = _lib.lib()
        s = _lib.stream_ptr()
        x, in_ss, w, y, ss, gamma, beta, x_raw = ctx.saved_tensors
        if x_raw is None:
            x_raw = x
        g = ctx.geom
        M_out = g.N * g.P * g.Q
        dy = dy.contiguous()
        dgamma = dbeta = None
        if ctx.grp is not None:
            if ss is not None and dss is None:  # (no statistics gradient reached this member: zero keeps it complete)
                dss = torch.zeros((4, g.K), device=dy.device, dtype=torch.float32)
            return _SiblingGroup.backward_member(ctx, dy, dss, x, w, y, ss, gamma, beta)
        if ss is not None and dss is not None and _bwd1x1_ok(ctx, g):
            out = _ConvBNFn._backward_1x1_fused(ctx, dy, dss, x_raw, in_ss, w, y, ss, gamma, beta)
            if out is not None:
                return out
        if ss is not None and dss is not None:
            gmg = grad_target(gamma) if gamma is not None else None
            bmg = grad_target(beta) if beta is not None else None
            if gamma is not None and gmg is None:
                dgamma = torch.zeros(g.K, device=dy.device)
            if beta is not None and bmg is None:
                dbeta = torch.zeros(g.K, device=dy.device)
            comb = torch.empty_like(dy)
            # dy is the unscaled g (every consumer of a training LazyBN returns it, see LazyBN)
            _check(L.dtm_stats_combine_fin(_lib.ptr(dy), _lib.ptr(y), _lib.ptr(dss.contiguous()), _lib.ptr(ss),
                                           _lib.ptr(gamma), ctx.count,
                                           _lib.ptr(gmg if gmg is not None else dgamma),
                                           _lib.ptr(bmg if bmg is not None else dbeta), _lib.ptr(comb), M_out, g.K, 1,
                                           s),
                   "stats_combine_fin")
            if gmg is not None:
                _notify(gamma)
            if bmg is not None:
                _notify(beta)
            dy = comb
        elif ss is not None:
            dy = (dy.float() * ss[0]).to(dy.dtype)  # no statistics gradient: only the BN-apply scale
        d = g.as_desc(_lib.ConvDesc)
        sc = in_ss[0] if (in_ss is not None and not ctx.mat) else None
        sh = in_ss[1] if (in_ss is not None and not ctx.mat) else None
        dx = d_in = None
        # the weight gradient on the side stream (ops/_lib.py side_stream), enqueued BEFORE the dgrad so
        # the two run concurrently; its bucket all-reduce is launched from that stream (parallel/bsp.py)
        wg_side = False
        if ctx.needs_input_grad[2] and getattr(w, "main_grad", None) is not None:
            st = _lib.side_fork(x, dy, in_ss)
            if st is not None:
                with torch.cuda.stream(st):
                    _check(L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(grad_target(w)), _lib.ptr(sc),
                                            _lib.ptr(sh), ctypes.byref(d), _lib.side_cus(), _lib.stream_ptr()),
                           "conv_wgrad(side)")
                    _notify(w)
                wg_side = True
        if ctx.needs_input_grad[0] or (in_ss is not None and ctx.needs_input_grad[1]):
            last, add_src, add_stride = _slot_take(ctx.slot)
            # stride > 1: one stride-1 conv per output parity class instead of the zero-dilated dgrad
            dec = (g.stride, g.pad_h, g.pad_w) if dgrad_decomposable(g) else None
            fullw = in_ss is not None and _full_window(g)
            wt = weight_flipped(w, g.K, g.R, g.S, g.C, dec) if not fullw else None
            d.dec = int(dec is not None)
            dx = torch.empty((g.N, g.H, g.W, g.C), device=dy.device, dtype=torch.bfloat16)
            if fullw:
                d_in = arena.zeros((4, g.C), dy.device)
                _full_window_dgrad_act(g, dy, w, x_raw, in_ss, d_in, dx, ctx.in_unscaled, add_src)
            elif in_ss is not None:
                # BN+ReLU of the input was fused into the forward prologue: mask, scale and the BN
                # parameter-gradient sums are done in the dgrad epilogue (+ the other conv consumers' masked
                # gradient of the same activation, added before the mask: act hand-off, see conv_bn)
                d_in = arena.zeros((4, g.C), dy.device)
                _check(L.dtm_conv_dgrad_ex(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d),
                                           _lib.ptr(add_src) if add_src is not None else None, 1,
                                           _lib.ptr(x_raw), _lib.ptr(in_ss), _lib.ptr(d_in), int(ctx.in_unscaled), s),
                       "conv_dgrad_act")
            else:
                # every conv consumer folds the pending stash into its own dgrad epilogue (free), so
                # a tensor read by k consumers costs no separate add at all; a non-last consumer
                # then leaves its (now cumulative) gradient as the new stash
                use_add = add_src is not None
                info = ctx.bnout
                if last and info is not None and info.sums is None and tuple(info.x.shape) == tuple(dx.shape):
                    # last consumer of a block output: the BN-apply backward (mask, scale/shift sums)
                    # runs in this dgrad's epilogue; the BN-apply node just hands the results on
                    # [8][C]: rows 0-3 / 4-7 = the ss gradients of bn(x) / bn(r) (rows 2-3, 6-7 stay 0)
                    sums = arena.zeros((8 if info.r is not None else 4, g.C), dy.device)
                    _check(L.dtm_conv_dgrad_bnout(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d),
                                                  _lib.ptr(add_src) if use_add else None,
                                                  add_stride if use_add else 1, _lib.ptr(info.mask),
                                                  _lib.ptr(info.x), _lib.ptr(info.r), _lib.ptr(sums), s),
                           "conv_dgrad_bnout")
                    info.sums, info.g = sums, dx
                    BNOUT_FUSED[0] += 1
                else:
                    _check(L.dtm_conv_dgrad_ex(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d),
                                               _lib.ptr(add_src) if use_add else None, add_stride if use_add else 1,
                                               None, None, None, 0, s), "conv_dgrad")
                if not last:
                    ctx.slot.buf, ctx.slot.stride = dx, 1
                    dx = None
                else:
                    _slot_done(ctx.slot, dx)
            if in_ss is not None and not last:
                # act hand-off (conv_bn): the cumulative masked gradient waits for the next conv consumer, whose
                # BN-gradient sums cover every consumer
                ctx.slot.buf, ctx.slot.stride = dx, 1
                dx = d_in = None
            d.dec = 0
        if wg_side:
            dw = None
        elif ctx.needs_input_grad[2]:
            mg = grad_target(w)
            target = mg if mg is not None else torch.zeros(w.shape, device=dy.device, dtype=torch.float32)
            _check(L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(target), _lib.ptr(sc),
                                                         _lib.ptr(sh), ctypes.byref(d), _lib.wgrad_cus(), s),
                   "conv_wgrad")
            if mg is not None:
                _notify(w)
                dw = None
            else:
                dw = target
        else:
            dw = None
        return dx, d_in, dw, dgamma, dbeta, None, None, None, None, None, None


    @staticmethod
    def _backward_1x1_fused(ctx, dy, dss, x_raw, in_ss, w, y, ss, gamma, beta):
        """Stats-combine + dgrad + wgrad of a 1x1 conv+BN in one pass over dy / y (dtm_conv1x1_bnbwd).
        With an activation input (in_ss) the dgrad epilogue does that BN+ReLU backward; with a plain
        input it adds the input's stashed gradient (_GradSlot) instead.  Returns the backward's
        outputs, or None if the kernel declines (the caller runs the three-kernel path)."""
        g = ctx.geom
        act = in_ss is not None
        add_src = None
        if act and ctx.slot is not None and (ctx.slot.pending > 1 or ctx.slot.buf is not None):
            return None  # (an activation shared by several conv consumers: the dgrad-epilogue hand-off path)
        if not act:
            sl = ctx.slot
            if ctx.bnout is not None or (sl is not None and sl.buf is not None and sl.stride != 1):
                return None  # (block-output input: the dgrad-epilogue BN-apply backward wins)
        L = _lib.lib()
        s = _lib.stream_ptr()
        gmg = grad_target(gamma) if gamma is not None else None
        bmg = grad_target(beta) if beta is not None else None
        dgamma = torch.zeros(g.K, device=dy.device) if (gamma is not None and gmg is None) else None
        dbeta = torch.zeros(g.K, device=dy.device) if (beta is not None and bmg is None) else None
        wt = weight_flipped(w, g.K, g.R, g.S, g.C)  # 1x1: [C][K] = W transposed
        dx = torch.empty((g.N, g.H, g.W, g.C), device=dy.device, dtype=torch.bfloat16)
        d_in = arena.zeros((4, g.C), dy.device) if act else None
        mg = grad_target(w)
        target = mg if mg is not None else torch.zeros(w.shape, device=dy.device, dtype=torch.float32)
        last = True
        if not act:
            sl = ctx.slot
            add_src = sl.buf if sl is not None else None
        rc = L.dtm_conv1x1_bnbwd(_lib.ptr(dy), _lib.ptr(y), _lib.ptr(dss.contiguous()), _lib.ptr(ss),
                                 _lib.ptr(gamma), ctx.count, _lib.ptr(gmg if gmg is not None else dgamma),
                                 _lib.ptr(bmg if bmg is not None else dbeta), _lib.ptr(wt), _lib.ptr(x_raw),
                                 _lib.ptr(in_ss), int(ctx.in_unscaled), _lib.ptr(add_src), _lib.ptr(dx),
                                 _lib.ptr(d_in), _lib.ptr(target), g.N * g.P * g.Q, g.K, g.C, s)
        if rc == -1:
            return None
        _check(rc, "conv1x1_bnbwd")
        last, _buf, _st = _slot_take(ctx.slot)
        if not act and not last:
            # (the kernel already folded the pending stash in: dx is the cumulative gradient)
            ctx.slot.buf, ctx.slot.stride = dx, 1
            dx = None
        elif not act:
            _slot_done(ctx.slot, dx)
        BWD1X1_FUSED[0] += 1
        for p, m in ((gamma, gmg), (beta, bmg), (w, mg)):
            if m is not None:
                _notify(p)
        return dx, d_in, (None if mg is not None else target), dgamma, dbeta, None, None, None, None, None, None


BWD1X1_FUSED = [0]  # count of 1x1 conv+BN backwards done by the one-pass kernel (tests / diagnostics)


def _bwd1x1_ok(ctx, g):
    """The one-pass 1x1 backward covers the ResNet 64 -> 256 channel shape (stage-1 expansion conv and
    projection shortcut)."""
    return (features.on("bwd1x1_fuse") and g.R == 1 and g.S == 1 and g.stride == 1 and
            g.pad_h == 0 and g.pad_w == 0 and g.P == g.H and g.Q == g.W and g.K == 256 and g.C == 64 and
            ctx.needs_input_grad[0] and ctx.needs_input_grad[2])


class _BNFinalizeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, stats, gamma, beta, mm, mv, count, eps, decay, bessel, update):
        L = _lib.lib()
        C = stats.shape[1]
        ss = torch.empty((4, C), device=stats.device, dtype=torch.float32)
        L.dtm_bn_finalize(_lib.ptr(stats), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(mm), _lib.ptr(mv), _lib.ptr(ss),
                          C, float(count), float(eps), float(decay), int(update and mm is not None), int(bessel),
                          _lib.stream_ptr())
        ctx.save_for_backward(ss)
        ctx.gamma, ctx.beta, ctx.count = gamma, beta, count
        return ss

    @staticmethod
    def backward(ctx, dss):
        L = _lib.lib()
        (ss,) = ctx.saved_tensors
        C = ss.shape[1]
        dstats = torch.empty((2, C), device=ss.device, dtype=torch.float32)
        gmg = grad_target(ctx.gamma) if ctx.gamma is not None else None
        bmg = grad_target(ctx.beta) if ctx.beta is not None else None
        dg = None if (ctx.gamma is None or gmg is not None) else torch.zeros(C, device=ss.device)
        db = None if (ctx.beta is None or bmg is not None) else torch.zeros(C, device=ss.device)
        L.dtm_bn_finalize_bwd(_lib.ptr(dss.contiguous()), _lib.ptr(ss), _lib.ptr(ctx.gamma), _lib.ptr(dstats),
                              _lib.ptr(gmg if gmg is not None else dg), _lib.ptr(bmg if bmg is not None else db), C,
                              float(ctx.count), _lib.stream_ptr())
        if gmg is not None:
            _notify(ctx.gamma)
        if bmg is not None:
            _notify(ctx.beta)
        return dstats, dg, db, None, None, None, None, None, None, None


class _BNApplyFn(torch.autograd.Function):
    """y = act(x*scale + shift [+ res | + res*rscale + rshift]); ReLU mask kept as a bitmask.
    unscaled: bit 0 / bit 1 = x / the BN'd residual comes from a training conv+BN (LazyBN.unscaled)."""

    @staticmethod
    def forward(ctx, x, ss, res, res_ss, relu, res_slot=None, res_stride=1, unscaled=0):
        L = _lib.lib()
        C = x.shape[-1]
        M = x.numel() // C
        y = torch.empty_like(x)
        res_mode = 0 if res is None else (2 if res_ss is not None else 1)
        # (grad mode is off inside Function.forward: whether a backward will run is needs_input_grad)
        want_mask = relu and any(ctx.needs_input_grad) and C % 8 == 0
        mask = torch.empty(M * C // 8, device=x.device, dtype=torch.uint8) if want_mask else None
        if res_stride > 1:
            N, Ho, Wo, _ = x.shape
            _check(L.dtm_bn_apply_res_strided(_lib.ptr(x), _lib.ptr(ss), _lib.ptr(res), _lib.ptr(y), _lib.ptr(mask), N,
                                              Ho, Wo, C, res.shape[1], res.shape[2], res_stride, int(relu),
                                              _lib.stream_ptr()), "bn_apply_res_strided")
        else:
            rc = L.dtm_bn_apply2(_lib.ptr(x), _lib.ptr(ss), _lib.ptr(res), _lib.ptr(res_ss), _lib.ptr(y), _lib.ptr(mask),
                                 M, C, res_mode, int(relu), _lib.stream_ptr())
            if rc == -7:  # no bitmask on this shape: keep y for the mask
                mask = None
                L.dtm_bn_apply2(_lib.ptr(x), _lib.ptr(ss), _lib.ptr(res), _lib.ptr(res_ss), _lib.ptr(y), None, M, C,
                                res_mode, int(relu), _lib.stream_ptr())
        ctx.relu, ctx.res_mode, ctx.res_slot, ctx.res_stride = relu, res_mode, res_slot, res_stride
        ctx.unscaled = int(unscaled) if res_mode == 2 else int(unscaled) & 1
        # eligible for the dgrad-epilogue backward: bitmask ReLU and every gradient this backward hands out
        # equal to g itself (unscaled producers).  A strided identity residual (the subsampled block input of
        # a stride-2 unit) qualifies too: its gradient is g at the subsampled pixels, handed to the block
        # input's other consumer with the stride exactly as the separate pass does
        ctx.bnout = None
        if (mask is not None and relu and (res_stride == 1 or (res_mode == 1 and _bnout_strided())) and
                (ctx.unscaled & 1) and
                (res_mode != 2 or (ctx.unscaled & 2)) and C % 8 == 0 and _bnout_enabled()):
            ctx.bnout = _BNOutInfo(mask, x, res if res_mode == 2 else None)
            try:
                y._dtm_bnout = ctx.bnout
            except Exception:
                ctx.bnout = None
        ctx.res_shape = None if res is None else tuple(res.shape)
        # the residual itself is only read back for a BN'd residual (res_mode 2)
        ctx.save_for_backward(x, ss, res if res_mode == 2 else None, res_ss,
                              y if (relu and mask is None) else None, mask)
        return y

    @staticmethod
    def backward(ctx, dy):
        L = _lib.lib()
        x, ss, res, rss, y, mask = ctx.saved_tensors
        C = x.shape[-1]
        M = x.numel() // C
        ux, ur = bool(ctx.unscaled & 1), bool(ctx.unscaled & 2)
        # dres aliases dx when both are g (identity residual with an unscaled x, or both BN'd unscaled)
        alias = (ctx.res_mode == 1 and ux) or (ctx.res_mode == 2 and ux and ur)
        info = ctx.bnout
        if info is not None and info.sums is not None:
            # the consuming conv's dgrad epilogue already applied this backward: dy is g (= d(y) * mask)
            sx = info.sums[:4]
            sr = info.sums[4:8] if ctx.res_mode == 2 else None
            dx = info.g
            if dy.data_ptr() != dx.data_ptr():
                # another (non-hand-off) consumer of y added its gradient: push the remainder through
                # the regular kernel (masking is linear) and add it
                rest = (dy.float() - dx.float()).to(dx.dtype).contiguous()
                dx2 = torch.empty_like(x)
                sx2 = arena.zeros((4, C), x.device)
                sr2 = arena.zeros((4, C), x.device) if ctx.res_mode == 2 else None
                _check(L.dtm_bn_apply_bwd(_lib.ptr(rest), None, _lib.ptr(mask), _lib.ptr(x), _lib.ptr(ss),
                                          _lib.ptr(res), _lib.ptr(rss), _lib.ptr(dx2), _lib.ptr(dx2), _lib.ptr(sx2),
                                          _lib.ptr(sr2), M, C, 3, ctx.res_mode, ctx.unscaled, _lib.stream_ptr()),
                       "bn_apply_bwd")
                dx = dx + dx2
                sx = sx + sx2
                if sr is not None:
                    sr = sr + sr2
            info.g = info.sums = None
            dres = None if not ctx.res_mode else dx
        else:
            dx = torch.empty_like(x)
            dres = None if not ctx.res_mode else (dx if alias else torch.empty_like(x))
            sx = arena.zeros((4, C), x.device)
            sr = arena.zeros((4, C), x.device) if ctx.res_mode == 2 else None
            mode = 3 if mask is not None else (1 if ctx.relu else 0)
            _check(L.dtm_bn_apply_bwd(_lib.ptr(dy.contiguous()), _lib.ptr(y), _lib.ptr(mask), _lib.ptr(x),
                                      _lib.ptr(ss), _lib.ptr(res), _lib.ptr(rss), _lib.ptr(dx), _lib.ptr(dres),
                                      _lib.ptr(sx), _lib.ptr(sr), M, C, mode, ctx.res_mode, ctx.unscaled,
                                      _lib.stream_ptr()), "bn_apply_bwd")
        st = ctx.res_stride
        if ctx.res_slot is not None:
            last, buf, bst = _slot_take(ctx.res_slot)
            if not last:
                _slot_stash(ctx.res_slot, dres, st)
                dres = None
            elif buf is not None or st > 1:
                dres = _unstride(ctx.res_slot, dres, st)
                if buf is not None:
                    dres = dres + _unstride(ctx.res_slot, buf, bst)
        elif st > 1:
            full = torch.zeros(ctx.res_shape, device=dres.device, dtype=dres.dtype)
            full[:, ::st, ::st, :] = dres
            dres = full
        return dx, sx, dres, sr, None, None, None, None


class _StemConvBNFn(torch.autograd.Function):
    """Training/inference conv+BN of a stem convolution (few input channels, stride 2, explicit pad;
    the ResNet 7x7/2 on RGB: reference vgg/nets/resnet_v1.py:226 via resnet_utils.conv2d_same) as a
    packed-row implicit GEMM.  The zero-bordered input is stored [N][Hp][Wp][4] (8-byte pixels), so
    one kernel row of taps for one output pixel -- S taps x 4 channels -- is a single contiguous
    64-byte run: the conv is run as an R x 1 conv over 32 'channels' with an 8-byte pixel pitch
    (ConvDesc.pix_bytes).  Reduction K*R*S*C = 7*32 = 224 instead of 7*7*8 = 392 (C padded to 8), and
    64-B contiguous gathers instead of 16-B ones.  No input gradient (images)."""

    @staticmethod
    def forward(ctx, x, w, gamma, beta, geom, bn, pad):
        L = _lib.lib()
        s = _lib.stream_ptr()
        N, H, W, C = x.shape
        K, R, S, _ = w.shape
        st, P, Q = geom.stride, geom.P, geom.Q
        Hp = max(H + 2 * pad, st * (P - 1) + R)
        Wp = max(W + 2 * pad, st * (Q - 1) + 8)
        Wp += Wp % 2  # 16-B aligned rows (the 64-B runs start at 16*q bytes)
        if x.dtype in (torch.float32, torch.bfloat16) and x.is_contiguous():
            # zero border + channel pad + bf16 in one pass
            xp = torch.empty((N, Hp, Wp, 4), device=x.device, dtype=torch.bfloat16)
            _check(L.dtm_stem_pack(_lib.ptr(x), 0 if x.dtype == torch.float32 else 1, _lib.ptr(xp), N, H, W, C, Hp,
                                   Wp, pad, s), "stem_pack")
        else:
            xp = torch.nn.functional.pad(x.to(torch.bfloat16), (0, 4 - C, pad, Wp - W - pad, pad, Hp - H - pad))
        wv = torch.zeros((K, R, 8, 4), device=x.device, dtype=torch.bfloat16)
        wv[:, :, :S, :C] = weight_bf16(w)
        d = _lib.ConvDesc(N, Hp, Wp, 32, K, R, 1, P, Q, st, 0, 0, 8)
        y = torch.empty((N, P, Q, K), device=x.device, dtype=torch.bfloat16)
        ss = None
        if bn is not None:
            ss = torch.empty((4, K), device=x.device, dtype=torch.float32)
            ctx.count = float(N * P * Q)
            _check(L.dtm_conv_fwd_bn(_lib.ptr(xp), _lib.ptr(wv), _lib.ptr(y), None, None, _lib.ptr(gamma),
                                     _lib.ptr(beta), _lib.ptr(bn.moving_mean), _lib.ptr(bn.moving_variance),
                                     _lib.ptr(ss), ctx.count, float(bn.eps), float(bn.decay), 1, int(bn.bessel),
                                     ctypes.byref(d), s), "stem_conv_fwd_bn")
        else:
            _check(L.dtm_conv_fwd(_lib.ptr(xp), _lib.ptr(wv), _lib.ptr(y), None, None, None, None, 0,
                                  ctypes.byref(d), s), "stem_conv_fwd")
        ctx.d = (N, Hp, Wp, K, R, S, C, P, Q, st)
        ctx.save_for_backward(xp, w, y, ss, gamma, beta)
        if ss is None:
            return y
        return y, ss

    @staticmethod
    def backward(ctx, dy, dss=None):
        L = _lib.lib()
        s = _lib.stream_ptr()
        xp, w, y, ss, gamma, beta = ctx.saved_tensors
        N, Hp, Wp, K, R, S, C, P, Q, st = ctx.d
        dy = dy.contiguous()
        dgamma = dbeta = None
        if (ss is not None and dss is not None and ctx.needs_input_grad[1] and features.on("stem_wgrad_fuse")):
            # no input gradient: comb (the BN backward of dy) has the wgrad as its only reader, so it is
            # formed in the wgrad's operand staging instead of being written and read back
            gmg = grad_target(gamma) if gamma is not None else None
            bmg = grad_target(beta) if beta is not None else None
            dgamma = torch.zeros(K, device=dy.device) if (gamma is not None and gmg is None) else None
            dbeta = torch.zeros(K, device=dy.device) if (beta is not None and bmg is None) else None
            d = _lib.ConvDesc(N, Hp, Wp, 32, K, R, 1, P, Q, st, 0, 0, 8)
            tv = torch.zeros((K, R, 8, 4), device=dy.device, dtype=torch.float32)
            _check(L.dtm_conv_wgrad_bnbwd(_lib.ptr(xp), _lib.ptr(dy), _lib.ptr(y), _lib.ptr(dss.contiguous()),
                                          _lib.ptr(ss), _lib.ptr(gamma), ctx.count,
                                          _lib.ptr(gmg if gmg is not None else dgamma),
                                          _lib.ptr(bmg if bmg is not None else dbeta), _lib.ptr(tv), ctypes.byref(d),
                                          _lib.wgrad_cus("stem"), s), "stem_conv_wgrad_bnbwd")
            for p, m in ((gamma, gmg), (beta, bmg)):
                if m is not None:
                    _notify(p)
            dw = _accum_param_grad(w, tv[:, :, :S, :C])
            return None, dw, dgamma, dbeta, None, None, None
        if ss is not None and dss is not None:
            gmg = grad_target(gamma) if gamma is not None else None
            bmg = grad_target(beta) if beta is not None else None
            if gamma is not None and gmg is None:
                dgamma = torch.zeros(K, device=dy.device)
            if beta is not None and bmg is None:
                dbeta = torch.zeros(K, device=dy.device)
            comb = torch.empty_like(dy)
            _check(L.dtm_stats_combine_fin(_lib.ptr(dy), _lib.ptr(y), _lib.ptr(dss.contiguous()), _lib.ptr(ss),
                                           _lib.ptr(gamma), ctx.count,
                                           _lib.ptr(gmg if gmg is not None else dgamma),
                                           _lib.ptr(bmg if bmg is not None else dbeta), _lib.ptr(comb), N * P * Q, K,
                                           1, s), "stats_combine_fin")
            if gmg is not None:
                _notify(gamma)
            if bmg is not None:
                _notify(beta)
            dy = comb
        elif ss is not None:
            dy = (dy.float() * ss[0]).to(dy.dtype)
        dw = None
        if ctx.needs_input_grad[1]:
            d = _lib.ConvDesc(N, Hp, Wp, 32, K, R, 1, P, Q, st, 0, 0, 8)
            tv = torch.zeros((K, R, 8, 4), device=dy.device, dtype=torch.float32)
            _check(L.dtm_conv_wgrad(_lib.ptr(xp), _lib.ptr(dy), _lib.ptr(tv), None, None, ctypes.byref(d),
                                    _lib.wgrad_cus("stem"), s), "stem_conv_wgrad")
            dw = _accum_param_grad(w, tv[:, :, :S, :C])
        return None, dw, dgamma, dbeta, None, None, None


def _stem_eligible(x, w, stride, g):
    """The packed-row stem path: a plain (non-lazy) input without gradient, <= 4 channels, stride 2,
    S <= 7 taps per kernel row (S x 4 channels fit one 64-byte run), equal top / left pads (explicit,
    'VALID', or TF 'SAME'; the bottom / right zero fill comes from the packed buffer's extent)."""
    if isinstance(x, (LazyBN, Subsampled)):
        return False
    if not (x.is_cuda and x.dim() == 4 and w.dim() == 4) or x.requires_grad:
        return False
    K, R, S, C = w.shape
    st = stride if isinstance(stride, int) else stride[0]
    return (C <= 4 and x.shape[-1] == C and st == 2 and S <= 7 and K % 4 == 0 and g.pad_h == g.pad_w and
            g.pad_h >= 0 and g.dilation == 1)


def bn_apply(raw, ss, relu, residual=None, unscaled=False):
    """y = relu?(raw*scale+shift + residual); residual may be a tensor, a LazyBN (BN'd shortcut) or a
    Subsampled block input (strided identity shortcut).  ``unscaled``: raw's LazyBN.unscaled."""
    ux = 1 if unscaled else 0
    if residual is None:
        return _BNApplyFn.apply(raw, ss, None, None, bool(relu), None, 1, ux)
    if isinstance(residual, Subsampled):
        src = residual.src
        if isinstance(src, LazyBN):
            src = src.materialize()
        res = src.to(torch.bfloat16).contiguous()
        slot = _slot_register(res) if res is src else None
        return _BNApplyFn.apply(raw, ss, res, None, bool(relu), slot, residual.stride, ux)
    if isinstance(residual, LazyBN):
        if residual.relu:
            residual = residual.materialize()
        else:
            return _BNApplyFn.apply(raw, ss, residual.raw, residual.ss, bool(relu), None, 1,
                                    ux | (2 if residual.unscaled else 0))
    res = residual.to(torch.bfloat16).contiguous()
    slot = _slot_register(res) if res is residual else None
    return _BNApplyFn.apply(raw, ss, res, None, bool(relu), slot, 1, ux)


def bn_apply_nograd(raw, ss):
    """relu(raw*scale + shift) as a plain bf16 tensor (no autograd node, no ReLU mask)."""
    L = _lib.lib()
    C = raw.shape[-1]
    y = torch.empty_like(raw)
    _check(L.dtm_bn_apply2(_lib.ptr(raw), _lib.ptr(ss), None, None, _lib.ptr(y), None, raw.numel() // C, C, 0, 1,
                           _lib.stream_ptr()), "bn_apply")
    return y


def bn_inference_ss(bn):
    """Differentiable [4, C] scale/shift from moving statistics (frozen BN / eval)."""
    rstd = torch.rsqrt(bn.moving_variance + bn.eps)
    scale = rstd if bn.gamma is None else bn.gamma * rstd
    shift = -bn.moving_mean * scale if bn.beta is None else bn.beta - bn.moving_mean * scale
    return torch.stack([scale, shift, bn.moving_mean.expand_as(scale), rstd.expand_as(scale)]).contiguous()


class _SiblingGroup:
    """1x1 stride-1 conv+BN siblings on one plain input - the first convs of an Inception mixed block's branches
    (reference inception/slim/inception_model.py:67-320: branch1x1 / branch5x5 / branch3x3dbl / ... all start
    with a 1x1 conv of the block input).  Forward is unchanged (one conv each).  In backward every member writes
    its BN-combined output gradient into its column slice of ONE [M][sum K] buffer (stats_combine_fin with a row
    pitch); the member whose backward runs last issues ONE dgrad with the members' transposed weights laid side
    by side ([C][sum K]) and ONE weight gradient whose split-K slabs are reduced row range by row range into
    each member's dW (dtm_conv_wgrad_multi).  Instead of one dgrad per member - each re-reading and
    re-writing the whole block-input gradient through the _GradSlot hand-off - and one wgrad per member.
    The group is one consumer of the input's _GradSlot."""
    __slots__ = ("x", "members", "ktot", "slot", "buf", "done", "bnout", "pend", "heads", "fwd")

    def __init__(self, x, heads=None):
        self.x, self.members, self.ktot, self.slot, self.buf, self.done = x, [], 0, None, None, 0
        # heads: the members' (weight, BatchNorm or None) in call order, declared by the model: the first member's
        # forward then runs ONE conv + ONE finalize for all of them (forward_all); fwd: weight -> (y, ss)
        self.heads, self.fwd = heads, None
        # deferred stats-combines (one grouped launch at the last member): (keep-alive tensors, 7 pointers, C, off,
        # parameters to notify)
        self.pend = []
        # x is a block output whose BN-apply backward the merged dgrad's epilogue can absorb (ResNet unit 1)
        self.bnout = getattr(x, "_dtm_bnout", None)

    def join(self, w, geom):
        if self.slot is None:
            self.slot = _slot_register(self.x)
        if self.heads is not None and (len(self.members) >= len(self.heads) or
                                       self.heads[len(self.members)][0] is not w):
            raise RuntimeError("sibling group: member %d joined out of the declared head order" % len(self.members))
        self.members.append((w, geom.K, self.ktot))
        self.ktot += geom.K
        return (self, len(self.members) - 1)

    def forward_all(self, geom, training):
        """The declared heads' forward as ONE conv over their concatenated bf16 weights (the members' compute
        copies are views of one buffer, engine.prepare_compute_copies) storing each member's own output, and ONE
        BatchNorm finalize writing each BN member's ss and moving statistics (dtm_conv_fwd_bn_multi).  Returns
        False (per-member launches instead) when the heads do not form such a group."""
        heads = self.heads
        if self.fwd is not None:
            return True
        cat = getattr(heads[0][0], "_sib_cat", None)
        if cat is None or len(heads) > 8:
            return False
        buf, off = cat[0], 0
        bns = [bn for _w, bn in heads if bn is not None]
        for w, bn in heads:
            c = getattr(w, "_sib_cat", None)
            if c is None or c[0] is not buf or c[1] != off or w.shape[1:3] != (1, 1) or w.shape[0] % 8:
                return False
            if bn is not None and (bn.eps, bn.decay, bn.bessel) != (bns[0].eps, bns[0].decay, bns[0].bessel):
                return False
            off += w.shape[0]
        if buf.shape[0] != off or geom.stride != 1 or geom.pad_h or geom.pad_w:
            return False
        L = _lib.lib()
        x = self.x
        N, H, W, C = x.shape
        M = N * H * W
        ys = [torch.empty((N, H, W, w.shape[0]), device=x.device, dtype=torch.bfloat16) for w, _bn in heads]
        sss = [torch.empty((4, w.shape[0]), device=x.device, dtype=torch.float32) if bn is not None else None
               for w, bn in heads]
        ptrs = []
        dp = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        for (w, bn), ss in zip(heads, sss):
            ptrs += ([dp(bn.gamma), dp(bn.beta), dp(bn.moving_mean), dp(bn.moving_variance), dp(ss)]
                     if bn is not None else [0, 0, 0, 0, 0])
        d = _lib.ConvDesc(N, H, W, C, off, 1, 1, H, W, 1, 0, 0, 0, 0)
        b0 = bns[0] if bns else None
        _check(L.dtm_conv_fwd_bn_multi(_lib.ptr(x), _lib.ptr(buf), (ctypes.c_void_p * len(ys))(*[y.data_ptr() for y in ys]),
                                       (ctypes.c_int * len(ys))(*[w.shape[0] for w, _bn in heads]), len(ys),
                                       (ctypes.c_void_p * len(ptrs))(*ptrs), float(M),
                                       float(b0.eps) if b0 else 1e-3, float(b0.decay) if b0 else 0.9, 1 if training else 0,
                                       int(b0.bessel) if b0 else 0, ctypes.byref(d), _lib.stream_ptr()),
               "conv_fwd_bn_multi(sibling heads)")
        self.fwd = {id(w): (y, ss) for (w, _bn), y, ss in zip(heads, ys, sss)}
        SIBLING_FWD_MERGED[0] += 1
        return True

    @staticmethod
    def backward_member(ctx, dy, dss, x, w, y, ss, gamma, beta):
        grp, idx = ctx.grp
        g = ctx.geom
        L = _lib.lib()
        s = _lib.stream_ptr()
        M = g.N * g.P * g.Q
        if grp.buf is None:
            grp.buf = torch.empty((M, grp.ktot), device=dy.device, dtype=torch.bfloat16)
        off = grp.members[idx][2]
        dgamma = dbeta = None
        gmg = grad_target(gamma) if (ss is not None and gamma is not None) else None
        bmg = grad_target(beta) if (ss is not None and beta is not None) else None
        # every BN parameter gradient lands in main_grad: the members' combines are deferred to ONE grouped launch
        # at the last member (dgamma / dbeta written there, then reported); otherwise per member, now
        grouped = (features.on("sibling_combine") and len(grp.members) <= 8 and g.K % 8 == 0 and
                   (gamma is None or gmg is not None) and (beta is None or bmg is not None))
        if grouped:
            dyc = dy.contiguous()
            dssc = dss.contiguous() if ss is not None else None
            grp.pend.append(((dyc, dssc, y), [dyc.data_ptr(), y.data_ptr() if ss is not None else 0,
                                              dssc.data_ptr() if ss is not None else 0,
                                              ss.data_ptr() if ss is not None else 0,
                                              gamma.data_ptr() if (ss is not None and gamma is not None) else 0,
                                              gmg.data_ptr() if gmg is not None else 0,
                                              bmg.data_ptr() if bmg is not None else 0],
                             g.K, off, [p for p, m in ((gamma, gmg), (beta, bmg)) if m is not None],
                             getattr(ctx, "count", None) if ss is not None else None))
        elif ss is None:
            # a member without BatchNorm (Inception's commuted pool-branch conv: its gradient comes from the pool's
            # backward): a strided copy into its column slice
            grp.buf[:, off:off + g.K].copy_(dy.reshape(M, g.K))
        else:
            dgamma = torch.zeros(g.K, device=dy.device) if (gamma is not None and gmg is None) else None
            dbeta = torch.zeros(g.K, device=dy.device) if (beta is not None and bmg is None) else None
            _check(L.dtm_stats_combine_fin_ld(_lib.ptr(dy.contiguous()), _lib.ptr(y), _lib.ptr(dss.contiguous()),
                                              _lib.ptr(ss), _lib.ptr(gamma), ctx.count,
                                              _lib.ptr(gmg if gmg is not None else dgamma),
                                              _lib.ptr(bmg if bmg is not None else dbeta),
                                              ctypes.c_void_p(grp.buf.data_ptr() + 2 * off), M, g.K, 1, grp.ktot, s),
                   "stats_combine_fin(sibling)")
            for p, m in ((gamma, gmg), (beta, bmg)):
                if m is not None:
                    _notify(p)
        grp.done += 1
        if grp.done < len(grp.members):
            return None, None, None, dgamma, dbeta, None, None, None, None, None, None
        if grp.pend:
            # (members' geometry is the shared input's: one pixel count; the count of a BN'd member is its N*P*Q)
            cnt = next((c for *_r, c in grp.pend if c), float(M))
            ptrs = (ctypes.c_void_p * (7 * len(grp.pend)))(*[q for _k, pp, *_r in grp.pend for q in pp])
            dims = (ctypes.c_int * (2 * len(grp.pend)))(*[v for _k, _p, K_, off_, *_r in grp.pend for v in (K_, off_)])
            _check(L.dtm_stats_combine_multi(ptrs, dims, len(grp.pend), float(cnt), _lib.ptr(grp.buf), M, grp.ktot, s),
                   "stats_combine_multi(sibling)")
            for _k, _p, _K, _off, params, _c in grp.pend:
                for p in params:
                    _notify(p)
            grp.pend = []
        # the last member: one dgrad and one wgrad over every member's output gradient
        buf, n = grp.buf, len(grp.members)
        d = _lib.ConvDesc(g.N, g.H, g.W, g.C, grp.ktot, 1, 1, g.P, g.Q, 1, 0, 0, 0)
        mgs = [grad_target(m[0]) for m in grp.members]
        dws = [mg if mg is not None else torch.zeros(m[0].shape, device=dy.device, dtype=torch.float32)
               for mg, m in zip(mgs, grp.members)]
        ptrs = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dws])
        rows = (ctypes.c_int * n)(*[m[1] for m in grp.members])
        st = _lib.side_fork(x, buf)

        def wgrad(stream, cus):
            _check(L.dtm_conv_wgrad_multi(_lib.ptr(x), _lib.ptr(buf), ptrs, rows, n, ctypes.byref(d), cus, stream),
                   "conv_wgrad_multi")
            # (the bucket all-reduces these notifications may launch are issued from the stream that wrote dW)
            for m, mg in zip(grp.members, mgs):
                if mg is not None:
                    _notify(m[0])
        if st is not None:
            with torch.cuda.stream(st):
                wgrad(_lib.stream_ptr(), _lib.side_cus())
        else:
            wgrad(s, _lib.wgrad_cus())
        wt = _group_flipped(grp, g.C)
        if wt is None:
            wts = [weight_flipped(m[0], m[1], 1, 1, g.C) for m in grp.members]
            wt = wts[0] if n == 1 else torch.cat([t.view(g.C, m[1]) for t, m in zip(wts, grp.members)], dim=1)
        last, add_src, add_stride = _slot_take(grp.slot)
        use_add = add_src is not None
        dx = torch.empty((g.N, g.H, g.W, g.C), device=dy.device, dtype=torch.bfloat16)
        info = grp.bnout
        if last and info is not None and info.sums is None and tuple(info.x.shape) == tuple(dx.shape):
            # last consumer of a block output: its BN-apply backward in this dgrad's epilogue (as _ConvBNFn)
            sums = arena.zeros((8 if info.r is not None else 4, g.C), dy.device)
            _check(L.dtm_conv_dgrad_bnout(_lib.ptr(buf), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d),
                                          _lib.ptr(add_src) if use_add else None, add_stride if use_add else 1,
                                          _lib.ptr(info.mask), _lib.ptr(info.x), _lib.ptr(info.r), _lib.ptr(sums), s),
                   "conv_dgrad_bnout(sibling)")
            info.sums, info.g = sums, dx
            BNOUT_FUSED[0] += 1
        else:
            _check(L.dtm_conv_dgrad_ex(_lib.ptr(buf), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d),
                                       _lib.ptr(add_src) if use_add else None, add_stride if use_add else 1,
                                       None, None, None, 0, s), "conv_dgrad(sibling)")
        if not last:
            grp.slot.buf, grp.slot.stride = dx, 1
            dx = None
        else:
            _slot_done(grp.slot, dx)
        grp.buf = None
        SIBLING_MERGED[0] += 1
        # member weights whose gradient has no main_grad: hand the fresh tensors back through this member only
        dw = None if mgs[idx] is not None else dws[idx]
        return dx, None, dw, dgamma, dbeta, None, None, None, None, None, None


_CAT_PARAMS = {}  # id(concatenated bf16 weight buffer) -> a bf16 pseudo-parameter over it (its flipped-copy owner)


def _group_flipped(grp, C):
    """The merged dgrad's [C][sum K] weight when the members' bf16 copies are consecutive rows of one buffer
    (engine.prepare_compute_copies): the flipped (for a 1x1: transposed) copy of that buffer as ONE weight, cached
    and refreshed by the optimizer like every dgrad copy (ops.nn.refresh_flipped) - no per-step concatenation."""
    ms = grp.members
    cat = getattr(ms[0][0], "_sib_cat", None)
    if len(ms) < 2 or cat is None or cat[1] != 0:
        return None
    buf = cat[0]
    for w, K, off in ms:
        c = getattr(w, "_sib_cat", None)
        if c is None or c[0] is not buf or c[1] != off:
            return None
    if buf.shape[0] != grp.ktot:
        return None
    cp = _CAT_PARAMS.get(id(buf))
    if cp is None or cp.data_ptr() != buf.data_ptr():
        cp = torch.nn.Parameter(buf, requires_grad=False)
        cp.bf16 = buf
        _CAT_PARAMS[id(buf)] = cp
    return weight_flipped(cp, grp.ktot, 1, 1, C)


SIBLING_MERGED = [0]  # merged sibling backwards (tests / diagnostics)
SIBLING_FWD_MERGED = [0]  # merged sibling forwards
_SIBLINGS = [None]


class sibling_group:
    """Context: the eligible 1x1 conv+BN calls on ``x`` inside it share one backward (see _SiblingGroup).
    Feature sibling_group (default on: Inception-v3 -4.8 %, ResNet-50 -0.24 % step on one GPU,
    profiles/ab/r3_ab_sibling_*).  Data-parallel exactness: the step-1 and step-2 per-parameter gradients of 2 ranks
    equal the single-rank ones bit for bit (profiles/r4/r4_diag_resnet_sib_2steps.log, tests/test_distributed.py
    test_bsp_gpu_step1_gradients_match_single_rank); the round-3 2-rank mismatch no longer reproduces
    (profiles/r4/README.md)."""

    def __init__(self, x, training=True, heads=None):
        on = (training and torch.is_grad_enabled() and isinstance(x, torch.Tensor) and x.is_cuda and
              x.requires_grad and features.on("sibling_group"))
        if heads is not None and (len(heads) < 2 or not features.on("sibling_fwd")):
            heads = None
        self.grp = _SiblingGroup(x, heads) if on else None

    def __enter__(self):
        self.prev, _SIBLINGS[0] = _SIBLINGS[0], self.grp
        return self.grp

    def __exit__(self, *exc):
        _SIBLINGS[0] = self.prev
        return False


def _sibling_join(xb, w, g, training, bn, plain=False):
    """The sibling group member handle of a conv(+BN) on x, or None.  plain: a conv without BatchNorm (its output
    gradient is copied into the group buffer instead of stats-combined)."""
    grp = _SIBLINGS[0]
    if (grp is None or not training or (bn is None and not plain) or xb is not grp.x or g.R != 1 or g.S != 1 or
            g.stride != 1 or
            g.pad_h or g.pad_w or g.P != g.H or g.Q != g.W or g.K % 8 or g.C % 8 or
            getattr(w, "main_grad", None) is None):
        return None
    if g.K == 256 and g.C == 64 and features.on("bwd1x1_fuse"):
        return None  # (the ResNet stage-1 64 -> 256 projection keeps its one-pass backward, dtm_conv1x1_bnbwd)
    h = grp.join(w, g)
    if grp.heads is not None and len(grp.members) == 1 and not grp.forward_all(g, training):
        grp.heads = None  # (not a mergeable head set: per-member forwards)
    return h


# How a conv consumes a LazyBN input (see _prologue_mode); None = the measured shape policy.  Tests and the A/B
# tool pin a mode by setting this attribute (it is not an environment knob).
PROLOGUE_MODE = None


def _prologue_mode(x_shape, w_shape, stride):
    """How a conv consumes its input's BatchNorm-apply + ReLU (a LazyBN):

    'fused' - in the conv's operand prologue (and again in its wgrad): the normalised activation is
              never stored, but every gathered element is re-transformed R*S times per pass and the
              conv stays off the pipelined LDS-DMA tile;
    'mat'   - materialised once by a forward-only BN-apply pass (read raw + write bf16); the conv and its
              wgrad read it plainly, and the dgrad epilogue still does the activation backward from the
              raw tensor, so there is no backward pass for it;
    'apply' - the autograd BN-apply (its own backward pass).
    Measured per ResNet-50 layer (tools/conv_tile_sweep.py with WGRAD=1, batch 256): the prologue
    costs fwd +13..+66 us and wgrad +12..+68 us per layer, a materialising pass 6..35 us -> 'mat' wins
    every conv except the stride-2 3x3 at 56x56, where it is neutral (profiles/ab/r2_ab_prologue_fused_vs_mat.log),
    and the stage-1 expansion 1x1, whose one-pass backward recomputes relu(bn(x)) from the raw x anyway
    (profiles/ab/r2_ab_prologue_expand.log).  Re-measured in round 5 with the pipelined prologue tiles: the prologue
    for every 1x1 consumer is still +1.71 % step (profiles/ab/r5_ab_prologue_1x1_fdir.log)."""
    _, H, W, _ = x_shape
    _, R, S, _ = w_shape
    if PROLOGUE_MODE == "spatial":  # (A/B: the prologue for every spatial consumer)
        return "fused" if R * S > 1 else "mat"
    if PROLOGUE_MODE is not None:
        return PROLOGUE_MODE
    st = stride if isinstance(stride, int) else stride[0]
    if st > 1 and H * W >= 56 * 56:
        return "fused"
    K, C = w_shape[0], w_shape[3]
    if R * S == 1 and st == 1 and C == 64 and K == 256:
        return "fused"
    return "mat"


def conv_bn(x, w, bn, stride, padding, training, relu):
    """Fused conv -> BatchNorm; returns a LazyBN.  x: tensor or LazyBN(relu=True) (prologue-fused)."""
    act_slot = None
    in_ss = None
    in_unscaled = False
    x_mat = None
    if isinstance(x, LazyBN):
        mode = _prologue_mode(tuple(x.shape), tuple(w.shape), stride) if x.relu else "apply"
        if mode == "apply" or x.ss.shape[1] % 8 != 0:
            x = x.materialize()
        else:
            lz = x
            in_ss, in_unscaled, x = x.ss, x.unscaled, x.raw
            if (training and lz.unscaled and torch.is_grad_enabled() and x.requires_grad and x.is_cuda and
                    features.on("act_handoff")):
                # conv consumers of one activation hand the (unscaled, masked) input gradient on: the last one's
                # act epilogue adds the others' before its mask and sums (Inception's split 1x3 / 3x1 pairs), so
                # autograd adds neither the gradients nor the BN-gradient sums
                if lz.aslot is None:
                    lz.aslot = _GradSlot(x.shape)
                lz.aslot.pending += 1
                act_slot = lz.aslot
            if mode == "mat":
                # one materialisation per LazyBN, whatever the number of conv consumers (Inception's split
                # 1x3 / 3x1 pairs read the same activation)
                if lz.mat is None:
                    lz.mat = bn_apply_nograd(x, in_ss)
                x_mat = lz.mat
    g = conv_geom(tuple(x.shape), tuple(w.shape), stride, padding)
    if in_ss is None and _stem_eligible(x, w, stride, g):
        if training:
            y, ss = _StemConvBNFn.apply(x, w, bn.gamma, bn.beta, g, bn, int(g.pad_h))
        else:
            y = _StemConvBNFn.apply(x, w, None, None, g, None, int(g.pad_h))
            ss = bn_inference_ss(bn)
        return LazyBN(y, ss, relu, unscaled=training)
    if g.C % 8 != 0:
        from .nn import _PadChannels
        if in_ss is not None:
            raise ValueError("prologue fusion needs C % 8 == 0")
        cp = (g.C + 7) // 8 * 8
        x = torch.nn.functional.pad(x, (0, cp - g.C))
        w = _PadChannels.apply(w, cp)
        g = conv_geom(tuple(x.shape), tuple(w.shape), stride, padding)
    xb = x.to(torch.bfloat16).contiguous()
    grp = _sibling_join(xb, w, g, training, bn) if (xb is x and in_ss is None) else None
    # a shared (materialised) input: hand the gradient between its consumers (see _GradSlot); sibling-group
    # members share the group's registration
    slot = _slot_register(xb) if (xb is x and in_ss is None and grp is None) else act_slot
    x = xb
    if training:
        y, ss = _ConvBNFn.apply(x, in_ss, w, bn.gamma, bn.beta, g, bn, slot, in_unscaled, x_mat, grp)
    else:
        y = _ConvBNFn.apply(x, in_ss, w, None, None, g, None, slot, in_unscaled)
        ss = bn_inference_ss(bn)
    return LazyBN(y, ss, relu, unscaled=training)


class _BNStatsFn(torch.autograd.Function):
    """stats = [sum y; sum y^2] per channel (HIP reduction), returned with an alias of y that the
    consumers use instead of y: backward then receives both of y's gradients at once and forms
    dy = d(alias) + dsum + 2*y*dsumsq in one HIP pass (no separate autograd accumulation launch)."""

    @staticmethod
    def forward(ctx, y):
        C = y.shape[-1]
        stats = arena.zeros((2, C), y.device)  # (per-step zeroed scratch: no fill launch)
        _lib.lib().dtm_bn_stats(_lib.ptr(y), _lib.ptr(stats), y.numel() // C, C, _lib.stream_ptr())
        ctx.save_for_backward(y)
        return stats, y.view_as(y)

    @staticmethod
    def backward(ctx, dstats, dalias):
        (y,) = ctx.saved_tensors
        C = y.shape[-1]
        if dstats is None:
            return dalias
        if y.is_cuda and y.dtype == torch.bfloat16 and C % 8 == 0 and y.is_contiguous():
            g = None
            if dalias is not None:
                g = dalias.to(torch.bfloat16).contiguous()
            # write dy into g only when nobody else can see g: a copy made just above, or a gradient its
            # producer marked private (the concat BN-apply backward's fresh dx).  A gradient autograd
            # shares between several inputs (or a view of a shared one) gets a fresh dy instead.
            private = g is not None and (g is not dalias or getattr(dalias, "_dtm_private_grad", False))
            dy = g if (private and g.data_ptr() != y.data_ptr()) else torch.empty_like(y)
            _check(_lib.lib().dtm_bn_stats_bwd(_lib.ptr(y), _lib.ptr(dstats.float().contiguous()),
                                               _lib.ptr(g) if g is not None else None, _lib.ptr(dy),
                                               y.numel() // C, C, _lib.stream_ptr()), "dtm_bn_stats_bwd")
            return dy
        dy = (dstats[0] + 2.0 * y.float() * dstats[1]).to(y.dtype)
        return dy if dalias is None else dy + dalias


def pool_commute_enabled():
    """Feature pool_commute (default on): Inception pool branches as conv -> avg_pool -> BN."""
    return features.on("pool_commute")


def conv_avgpool_bn(x, w, bn, training, relu=True):
    """An Inception pool branch - avg_pool 3x3/1 'SAME' -> 1x1 conv -> BatchNorm (+ReLU), reference
    inception/slim/inception_model.py:88-92 etc. - computed as 1x1 conv -> avg_pool -> BatchNorm.  The two
    linear maps commute exactly (the pool mixes pixels per channel, the 1x1 conv channels per pixel, and
    TF's 'SAME' divisor depends on the pixel only), so the pool runs over the conv's K output channels
    instead of the block input's C (Inception: 288 -> 64, 768 -> 192, 2048 -> 192), forward and backward.
    The conv keeps the block input's gradient hand-off; the BatchNorm statistics come from the pooled
    tensor.  Returns a LazyBN like conv_bn."""
    from .nn import avg_pool
    xb = as_tensor(x).to(torch.bfloat16).contiguous()
    g = conv_geom(tuple(xb.shape), tuple(w.shape), 1, "SAME")
    grp = _sibling_join(xb, w, g, training, None, plain=True) if xb is x else None
    slot = _slot_register(xb) if (xb is x and grp is None) else None
    z = _ConvBNFn.apply(xb, None, w, None, None, g, None, slot, False, None, grp)
    y = avg_pool(z, 3, 1, "SAME")
    if training:
        stats, y = _BNStatsFn.apply(y)  # (y: the alias whose gradient the statistics backward folds in)
        ss = _BNFinalizeFn.apply(stats, bn.gamma, bn.beta, bn.moving_mean, bn.moving_variance,
                                 float(y.numel() // y.shape[-1]), float(bn.eps), float(bn.decay), bool(bn.bessel), True)
    else:
        ss = bn_inference_ss(bn)
    return LazyBN(y, ss, relu, unscaled=False)


# ---------------------------------------------------------------------------------------------
class _ConcatBNApplyFn(torch.autograd.Function):
    """Zero-copy channel concat (Inception mixed blocks, reference
    inception/slim/inception_model.py tf.concat(axis=3, ...)): every LazyBN part's BN-apply(+ReLU)
    writes straight into its channel slice of the block output (row pitch = total channels), and in
    backward its BN-apply gradient reads the slice of the concat gradient in place - neither the
    concat copy nor the split copies of its gradient exist.  Plain-tensor parts (max-pool branches)
    are copied into their slice.  meta: per part ('bn', C, relu, unscaled) or ('t', C)."""

    @staticmethod
    def _descs(parts):
        """Host table of CatPart (fused_bn.hip) for dtm_cat_bn_apply(_bwd): per part (raw, ss, mask, dx, C,
        channel offset, flags)."""
        import numpy as np
        nb = _lib.lib().dtm_cat_desc_bytes()
        tab = np.zeros((len(parts), nb // 8), dtype=np.int64)
        off = 0
        for i, (raw, ss, mask, dx, C, flags) in enumerate(parts):
            tab[i, 0:4] = [t.data_ptr() if t is not None else 0 for t in (raw, ss, mask, dx)]
            tab[i, 4:6] = np.array([C, off, flags, 0], dtype=np.int32).view(np.int64)
            off += C
        return tab

    @staticmethod
    def forward(ctx, meta, *ts):
        L = _lib.lib()
        first = ts[0]
        N, H, W = first.shape[:3]
        Ct = sum(m[1] for m in meta)
        M = N * H * W
        out = torch.empty((N, H, W, Ct), device=first.device, dtype=torch.bfloat16)
        saved, off, i = [], 0, 0
        s = _lib.stream_ptr()
        cm = _cat_multi()
        ctx.multi = (cm and any(m[0] == "bn" for m in meta) and len(meta) <= 8 and
                     all(m[0] == "bn" or (cm == 1 and ts[i].dtype == torch.bfloat16 and ts[i].is_contiguous())
                         for m, i in zip(meta, _part_index(meta))))
        if ctx.multi:
            # every part's BN-apply (plain parts: a copy) in one launch (fused_bn.hip cat_bn_apply_kernel)
            parts = []
            for m, i in zip(meta, _part_index(meta)):
                if m[0] == "bn":
                    raw, ss = ts[i], ts[i + 1]
                    mask = torch.empty(M * m[1] // 8, device=raw.device, dtype=torch.uint8)
                    parts.append((raw, ss, mask, None, m[1], int(m[2])))
                    saved += [raw, ss, mask]
                else:
                    parts.append((ts[i], None, None, None, m[1], 2))
            tab = _ConcatBNApplyFn._descs(parts)
            _check(L.dtm_cat_bn_apply(ctypes.c_void_p(tab.ctypes.data), len(parts), _lib.ptr(out), M, Ct, s),
                   "cat_bn_apply")
            ctx.meta = meta
            ctx.save_for_backward(*saved)
            return out
        for m in meta:
            C = m[1]
            if m[0] == "bn":
                raw, ss = ts[i], ts[i + 1]
                i += 2
                mask = torch.empty(M * C // 8, device=raw.device, dtype=torch.uint8)
                _check(L.dtm_bn_apply_ld(_lib.ptr(raw), _lib.ptr(ss), ctypes.c_void_p(out.data_ptr() + 2 * off),
                                         _lib.ptr(mask), M, C, int(m[2]), Ct, s), "bn_apply_ld")
                saved += [raw, ss, mask]
            else:
                out[..., off:off + C].copy_(ts[i])
                i += 1
            off += C
        ctx.meta = meta
        ctx.save_for_backward(*saved)
        return out

    @staticmethod
    def backward(ctx, dout):
        L = _lib.lib()
        dout = dout.contiguous()
        saved = list(ctx.saved_tensors)
        Ct = dout.shape[-1]
        M = dout.numel() // Ct
        s = _lib.stream_ptr()
        if ctx.multi:
            # every part's BN-apply backward and ONE reduction: sums holds the parts' [4][C] dss back to back
            # (a plain part's gradient is its view of dout; its sums slots stay zero)
            parts, grads = [], []
            sums = arena.zeros((4 * Ct,), dout.device)
            off, j = 0, 0
            for m in ctx.meta:
                if m[0] == "bn":
                    raw, ss, mask = saved[j:j + 3]
                    j += 3
                    dx = torch.empty_like(raw)
                    dx._dtm_private_grad = True  # fresh, single-owner: _BNStatsFn may write into it
                    parts.append((raw, ss, mask, dx, m[1], int(m[3])))
                    grads += [dx, sums[4 * off:4 * (off + m[1])].view(4, m[1])]
                else:
                    parts.append((dout, None, None, None, m[1], 2))
                    grads.append(dout[..., off:off + m[1]])
                off += m[1]
            tab = _ConcatBNApplyFn._descs(parts)
            _check(L.dtm_cat_bn_apply_bwd(ctypes.c_void_p(tab.ctypes.data), len(parts), _lib.ptr(dout), _lib.ptr(sums),
                                          M, Ct, s), "cat_bn_apply_bwd")
            return (None,) + tuple(grads)
        grads, off, j = [], 0, 0
        for m in ctx.meta:
            C = m[1]
            if m[0] == "bn":
                raw, ss, mask = saved[j:j + 3]
                j += 3
                dx = torch.empty_like(raw)
                dx._dtm_private_grad = True
                sx = arena.zeros((4, C), raw.device)
                _check(L.dtm_bn_apply_bwd_ld(ctypes.c_void_p(dout.data_ptr() + 2 * off), _lib.ptr(mask), _lib.ptr(raw),
                                             _lib.ptr(ss), _lib.ptr(dx), _lib.ptr(sx), M, C, int(m[3]), Ct, s),
                       "bn_apply_bwd_ld")
                grads += [dx, sx]
            else:
                grads.append(dout[..., off:off + C])
            off += C
        return (None,) + tuple(grads)


def _part_index(meta):
    """Index of each concat part's first tensor in the flat (raw, ss | tensor) argument list."""
    idx, i = [], 0
    for m in meta:
        idx.append(i)
        i += 2 if m[0] == "bn" else 1
    return idx


def _cat_multi():
    """Feature cat_multi: 1 (default) = the one-launch multi-part concat BN-apply, plain tensor parts included;
    0 = one launch per part."""
    return 1 if features.on("cat_multi") else 0


def concat_channels(parts):
    """Channel concat of NHWC parts (LazyBN or tensors) with the zero-copy path when every slice is
    16-byte aligned and each LazyBN part fits the fast BN-apply (C % 8 == 0); otherwise torch.cat."""
    cuda = all(p.is_cuda for p in parts)
    ok = cuda and all(p.shape[-1] % 8 == 0 and tuple(p.shape[:3]) == tuple(parts[0].shape[:3]) for p in parts)
    ok = ok and any(isinstance(p, LazyBN) for p in parts)
    if not ok:
        return torch.cat([as_tensor(p) for p in parts], dim=-1)
    meta, ts = [], []
    for p in parts:
        if isinstance(p, LazyBN) and p.relu and p.raw.dtype == torch.bfloat16 and p.shape[-1] // 8 <= 256:
            meta.append(("bn", p.shape[-1], True, bool(p.unscaled)))
            ts += [p.raw.contiguous(), p.ss]
        else:
            t = as_tensor(p)
            meta.append(("t", t.shape[-1]))
            ts.append(t)
    return _ConcatBNApplyFn.apply(meta, *ts)
