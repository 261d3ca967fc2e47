"""Stride-decomposed dgrad (conv_igemm.hip dec_dim / ConvDesc.dec): a stride-s conv's input gradient as
s*s stride-1 convolutions of dy, one per output parity class, each with that class's taps of the flipped
weight - instead of one conv over the zero-dilated dy (which spends (s*s-1)/(s*s) of its MFMA work on
zeros).  CPU: the decomposition algebra against torch's dgrad in fp64.  GPU: the HIP kernels (plain,
shared-input add, BatchNorm+ReLU activation-backward and block-output epilogues) against the undecomposed
path and the fp32 reference."""
import ctypes

import pytest
import torch
import torch.nn.functional as tF


def dec_dim(R, st, pad, a):
    """Python mirror of conv_igemm.hip dec_dim: (r0, T, off) of parity class a along one dimension."""
    r0 = ((a + pad) % st + st) % st
    T = (R - r0 + st - 1) // st if r0 < R else 0
    return r0, T, (a + pad - r0) // st


def decomposed_layout(w, st, ph, pw):
    """w [K][R][S][C] -> the decomposed flipped layout as a flat tensor (blocks [C][Tr][Tu][K], classes
    a-major), built from the definition W'[c][t'][u'][k] = w[k][r0 + st(Tr-1-t')][s0 + st(Tu-1-u')][c]."""
    K, R, S, C = w.shape
    out = []
    for a in range(st):
        for b in range(st):
            r0, Tr, _ = dec_dim(R, st, ph, a)
            s0, Tu, _ = dec_dim(S, st, pw, b)
            blk = torch.empty(C, Tr, Tu, K, dtype=w.dtype)
            for t in range(Tr):
                for u in range(Tu):
                    blk[:, t, u, :] = w[:, r0 + st * (Tr - 1 - t), s0 + st * (Tu - 1 - u), :].t()
            out.append(blk.reshape(-1))
    return torch.cat(out)


def dgrad_by_classes(dy, w, H, W, st, ph, pw):
    """dx [N][H][W][C] from dy [N][P][Q][K] via the per-class stride-1 correlations (NHWC, fp64)."""
    N, P, Q, K = dy.shape
    _, R, S, C = w.shape
    dx = torch.zeros(N, H, W, C, dtype=dy.dtype)
    flat = decomposed_layout(w, st, ph, pw)
    off = 0
    for a in range(st):
        for b in range(st):
            r0, Tr, oa = dec_dim(R, st, ph, a)
            s0, Tu, ob = dec_dim(S, st, pw, b)
            n = C * Tr * Tu * K
            wb = flat[off:off + n].reshape(C, Tr, Tu, K)
            off += n
            Hc, Wc = (H - a + st - 1) // st, (W - b + st - 1) // st
            if Hc <= 0 or Wc <= 0 or Tr == 0 or Tu == 0:
                continue
            pt, pl = Tr - 1 - oa, Tu - 1 - ob
            for i in range(Hc):
                for j in range(Wc):
                    acc = torch.zeros(N, C, dtype=dy.dtype)
                    for t in range(Tr):
                        for u in range(Tu):
                            p, q = i - pt + t, j - pl + u
                            if 0 <= p < P and 0 <= q < Q:
                                acc += dy[:, p, q, :] @ wb[:, t, u, :].t()
                    dx[:, st * i + a, st * j + b, :] = acc
    return dx


@pytest.mark.parametrize("H, R, st, pad, P", [
    (8, 3, 2, 1, 4),      # ResNet conv2d_same 3x3/2 (explicit pad 1, VALID)
    (9, 3, 2, 0, 4),      # Inception 3x3/2 VALID, odd extent
    (15, 3, 2, 1, 8),     # TF SAME on an odd extent (top pad 1)
    (8, 3, 2, 0, 4),      # TF SAME on an even extent (top pad 0, bottom 1)
    (12, 7, 2, 3, 6),     # 7x7/2 stem geometry
    (9, 4, 2, 1, 5),      # even kernel (conv2d_same: pads 1 / 2)
    (10, 5, 3, 2, 4),     # stride 3
])
def test_decomposition_algebra_matches_dgrad(H, R, st, pad, P):
    torch.manual_seed(0)
    N, C, K = 2, 3, 4
    x = torch.randn(N, C, H, H, dtype=torch.float64, requires_grad=True)
    w = torch.randn(K, C, R, R, dtype=torch.float64)
    # forward with top/left pad `pad` and output extent P (the rest of the bottom/right pad is implicit)
    need = (P - 1) * st + R
    xp = tF.pad(x, (pad, max(need - H - pad, 0), pad, max(need - H - pad, 0)))
    y = tF.conv2d(xp, w, stride=st)[:, :, :P, :P]
    dy = torch.randn_like(y)
    y.backward(dy)
    got = dgrad_by_classes(dy.permute(0, 2, 3, 1).contiguous(), w.permute(0, 2, 3, 1).contiguous(), H, H, st, pad,
                           pad)
    assert torch.allclose(got.permute(0, 3, 1, 2), x.grad, atol=1e-9)


DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.gpu
@pytest.mark.parametrize("case", [
    # N, H, C(in), K(out), R, stride, padding
    (4, 56, 64, 64, 3, 2, (1, 1)),        # ResNet-50 stage-2 conv2 (56 -> 28)
    (2, 28, 128, 128, 3, 2, (1, 1)),
    (2, 35, 288, 384, 3, 2, "VALID"),     # Inception mixed_17x17x768a
    (2, 17, 192, 320, 3, 2, "VALID"),     # Inception mixed_8x8x1280a
    (2, 15, 32, 64, 3, 2, "SAME"),
    (2, 16, 64, 96, 7, 2, (3, 3)),
    (2, 9, 64, 64, 4, 2, ((1, 2), (1, 2))),
    (2, 12, 64, 64, 5, 3, "SAME"),
])
def test_decomposed_dgrad_kernels(case):
    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops import reference as ref
    from distributed_tensorflow_models_amd.ops.geometry import conv_geom
    N, H, C, K, R, st, pad = case
    torch.manual_seed(0)
    L = _lib.lib()
    s = _lib.stream_ptr()
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=DEV) / (R * R * C) ** 0.5).to(torch.bfloat16)
    g = conv_geom(tuple(x.shape), tuple(w.shape), st, pad)
    # layout of the batched/tiled flip against the Python definition
    wdec = torch.empty(C, R, R, K, device=DEV, dtype=torch.bfloat16)
    L.dtm_weight_flip_transpose_dec(_lib.ptr(w), _lib.ptr(wdec), K, R, R, C, st, g.pad_h, g.pad_w, s)
    torch.cuda.synchronize()
    assert torch.equal(wdec.reshape(-1).cpu(), decomposed_layout(w.cpu(), st, g.pad_h, g.pad_w))
    wt = torch.empty(C, R, R, K, device=DEV, dtype=torch.bfloat16)
    L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, s)
    xr = x.float().requires_grad_()
    yr = ref.conv2d(xr, w.float(), None, st, pad)
    dy = torch.randn_like(yr).to(torch.bfloat16)
    yr.backward(dy.float())

    plain = st <= 2  # (the zero-dilated path covers strides 1 and 2 only)

    def run(dec, **kw):
        if not dec and not plain:
            dec = 1
        d = g.as_desc(_lib.ConvDesc)
        d.dec = dec
        dx = torch.empty_like(x)
        if not kw:
            rc = L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wdec if dec else wt), _lib.ptr(dx), ctypes.byref(d), s)
            assert rc == 0
            return dx, None
        sums = torch.zeros(kw.get("rows", 4), C, device=DEV)
        if "mask" in kw:
            rc = L.dtm_conv_dgrad_bnout(_lib.ptr(dy), _lib.ptr(wdec if dec else wt), _lib.ptr(dx), ctypes.byref(d),
                                        _lib.ptr(kw["add"]), 1, _lib.ptr(kw["mask"]), _lib.ptr(kw["ax"]),
                                        _lib.ptr(kw.get("ar")), _lib.ptr(sums), s)
        else:
            rc = L.dtm_conv_dgrad_ex(_lib.ptr(dy), _lib.ptr(wdec if dec else wt), _lib.ptr(dx), ctypes.byref(d),
                                     _lib.ptr(kw.get("add")), 1, _lib.ptr(kw.get("ax")), _lib.ptr(kw.get("ss")),
                                     _lib.ptr(sums) if "ax" in kw else None, 0, s)
        assert rc == 0
        return dx, sums

    dx0, _ = run(0)
    dx1, _ = run(1)
    torch.cuda.synchronize()
    assert _rel(dx1, xr.grad) < 1e-2
    assert _rel(dx1, dx0) < 1e-2
    # shared-input gradient added in the epilogue
    add = torch.randn_like(x)
    a0, _ = run(0, add=add)
    a1, _ = run(1, add=add)
    torch.cuda.synchronize()
    assert _rel(a1, xr.grad + add.float()) < 1e-2 and _rel(a1, a0) < 1e-2
    # BatchNorm+ReLU activation backward of the conv's input (act epilogue): mask, scale, scale/shift sums
    ax = torch.randn_like(x)
    ss = torch.stack([torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3,
                      torch.zeros(C, device=DEV), torch.ones(C, device=DEV)]).contiguous()
    b0, s0 = run(0, ax=ax, ss=ss)
    b1, s1 = run(1, ax=ax, ss=ss)
    torch.cuda.synchronize()
    m = (ax.float() * ss[0] + ss[1] > 0).float()
    gm = xr.grad * m
    assert _rel(b1, gm * ss[0]) < 1e-2 and _rel(b1, b0) < 1e-2
    assert _rel(s1[0], (gm * ax.float()).sum((0, 1, 2))) < 2e-2 and _rel(s1[1], gm.sum((0, 1, 2))) < 2e-2
    assert _rel(s1[:2], s0[:2]) < 1e-2
    if C % 8 == 0:
        # block-output form: the ReLU bitmask of the forward, sums against the raw input and a BN'd residual
        bits = torch.rand(x.numel(), device=DEV) > 0.4
        mask = (bits.view(-1, 8).to(torch.uint8) << torch.arange(8, device=DEV, dtype=torch.uint8)).sum(
            1).to(torch.uint8)
        ar = torch.randn_like(x)
        c0, t0 = run(0, mask=mask, ax=ax, ar=ar, add=add, rows=8)
        c1, t1 = run(1, mask=mask, ax=ax, ar=ar, add=add, rows=8)
        torch.cuda.synchronize()
        gb = (xr.grad + add.float()) * bits.view(x.shape).float()
        assert _rel(c1, gb) < 1e-2 and _rel(c1, c0) < 1e-2
        assert _rel(t1[0], (gb * ax.float()).sum((0, 1, 2))) < 2e-2
        assert _rel(t1[4], (gb * ar.float()).sum((0, 1, 2))) < 2e-2
        assert _rel(t1, t0) < 1e-2
