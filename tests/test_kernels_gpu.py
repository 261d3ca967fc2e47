"""Numerics of the HIP kernels against plain PyTorch fp32 references (GPU only)."""
import pytest
import torch

from distributed_tensorflow_models_amd.ops import nn as dnn
from distributed_tensorflow_models_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CONV_CASES = [
    # N, H, W, C, K, (R, S), stride, padding
    (2, 14, 14, 64, 64, (3, 3), 1, "SAME"),
    (2, 14, 14, 64, 128, (1, 1), 1, "SAME"),
    (2, 15, 15, 32, 64, (3, 3), 2, "SAME"),      # asymmetric SAME
    (2, 16, 16, 64, 64, (3, 3), 2, (1, 1)),       # conv2d_same style explicit pad
    (2, 9, 9, 128, 256, (3, 3), 1, "VALID"),
    (2, 32, 32, 3, 64, (7, 7), 2, (3, 3)),        # stem (C=3 -> padded)
    (3, 7, 7, 512, 512, (3, 3), 1, "SAME"),
    (2, 8, 8, 256, 1000, (1, 1), 1, "SAME"),      # K not a multiple of the tile
    # Inception-v3 factorised convs (reference inception/slim/inception_model.py:127-317)
    (2, 17, 17, 128, 128, (1, 7), 1, "SAME"),
    (2, 17, 17, 160, 192, (7, 1), 1, "SAME"),
    (2, 8, 8, 384, 384, (1, 3), 1, "SAME"),
    (2, 8, 8, 448, 384, (3, 1), 1, "SAME"),
    (2, 35, 35, 288, 384, (3, 3), 2, "VALID"),    # mixed_17x17x768a 3x3/2 VALID
    (2, 17, 17, 192, 320, (3, 3), 2, "VALID"),    # mixed_8x8x1280a
    (2, 9, 9, 64, 64, (4, 4), 2, ((1, 2), (1, 2))),  # even-kernel conv2d_same (resnet_utils.py:77-122)
    # the direct 3x3 kernel (C in {32, 64}; ragged 8 x 16 spatial tiles): ResNet stage 1, Inception stem
    (2, 56, 56, 64, 64, (3, 3), 1, "SAME"),
    (3, 19, 21, 32, 32, (3, 3), 1, "VALID"),
    (2, 17, 23, 32, 64, (3, 3), 1, "SAME"),
    (2, 9, 30, 64, 32, (3, 3), 1, "VALID"),
    (1, 41, 37, 64, 96, (3, 3), 1, "SAME"),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_bwd(case):
    torch.manual_seed(0)
    N, H, W, C, K, (R, S), st, pad = case
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(K, R, S, C, device=DEV) * (1.0 / (R * S * C) ** 0.5)).to(torch.bfloat16).float()
    xr = x.clone().requires_grad_()
    wr = w.clone().requires_grad_()
    yr = ref.conv2d(xr, wr, None, st, pad)
    gy = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(gy)

    xk = x.to(torch.bfloat16).requires_grad_()
    wk = w.clone().requires_grad_()
    yk = dnn.conv2d(xk, wk, None, st, pad)
    assert yk.shape == yr.shape
    yk.backward(gy.to(torch.bfloat16))
    torch.cuda.synchronize()
    assert _rel(yk, yr) < 1e-2
    assert _rel(xk.grad, xr.grad) < 1e-2
    assert _rel(wk.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("N,H,C,K,R,rate,pad", [(2, 21, 64, 64, 3, 2, "SAME"), (2, 11, 128, 64, 3, 4, "SAME"),
                                                 (1, 17, 32, 48, 3, 2, "VALID")])
def test_atrous_conv_fwd_bwd(N, H, C, K, R, rate, pad):
    """Dilated conv (ResNet output_stride mode): space-to-batch around the dense HIP conv."""
    torch.manual_seed(3)
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(K, R, R, C, device=DEV) * (1.0 / (R * R * C) ** 0.5)).to(torch.bfloat16).float()
    xr, wr = x.clone().requires_grad_(), w.clone().requires_grad_()
    yr = ref.conv2d(xr, wr, None, 1, pad, False, rate)
    gy = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(gy)
    xk, wk = x.to(torch.bfloat16).requires_grad_(), w.clone().requires_grad_()
    yk = dnn.conv2d(xk, wk, None, 1, pad, dilation=rate)
    assert yk.shape == yr.shape
    yk.backward(gy.to(torch.bfloat16))
    torch.cuda.synchronize()
    assert _rel(yk, yr) < 1e-2
    assert _rel(xk.grad, xr.grad) < 1e-2
    assert _rel(wk.grad, wr.grad) < 1e-2


def test_conv_bias_relu_and_stats_free():
    torch.manual_seed(1)
    x = torch.randn(2, 12, 12, 64, device=DEV).to(torch.bfloat16).float()
    w = (torch.randn(96, 3, 3, 64, device=DEV) * 0.05).to(torch.bfloat16).float()
    b = torch.randn(96, device=DEV)
    yr = ref.conv2d(x, w, b, 1, "SAME", relu=True)
    yk = dnn.conv2d(x.to(torch.bfloat16), w, b, 1, "SAME", relu=True)
    assert _rel(yk, yr) < 1e-2


@pytest.mark.parametrize("C,relu,res", [(64, True, False), (256, False, True), (40, True, True), (2048, True, False), (80, True, True), (1280, False, False), (192, True, False)])
def test_batch_norm(C, relu, res):
    torch.manual_seed(2)
    x = (torch.randn(4, 7, 7, C, device=DEV) * 2 + 0.5).to(torch.bfloat16).float()
    g = torch.rand(C, device=DEV) + 0.5
    b = torch.randn(C, device=DEV)
    r = torch.randn_like(x).to(torch.bfloat16).float() if res else None
    mm_r, mv_r = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    mm_k, mv_k = mm_r.clone(), mv_r.clone()
    xr, gr, br = x.clone().requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
    rr = r.clone().requires_grad_() if res else None
    yr = ref.batch_norm(xr, gr, br, mm_r, mv_r, True, 0.9, 1e-3, relu, rr)
    gy = torch.randn_like(yr).to(torch.bfloat16).float()
    yr.backward(gy)
    xk, gk, bk = x.to(torch.bfloat16).requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
    rk = r.to(torch.bfloat16).requires_grad_() if res else None
    yk = dnn.batch_norm(xk, gk, bk, mm_k, mv_k, True, 0.9, 1e-3, relu, rk)
    yk.backward(gy.to(torch.bfloat16))
    assert _rel(yk, yr) < 1e-2
    assert _rel(xk.grad, xr.grad) < 2e-2
    assert _rel(gk.grad, gr.grad) < 1e-2
    assert _rel(bk.grad, br.grad) < 1e-2
    assert _rel(mm_k, mm_r) < 1e-4 and _rel(mv_k, mv_r) < 1e-4
    if res:
        assert _rel(rk.grad, rr.grad) < 1e-2


@pytest.mark.parametrize("k,s,pad", [(3, 2, "SAME"), (2, 2, "VALID"), (3, 2, "VALID"), (1, 2, "VALID"), (3, 1, "SAME")])
def test_pools(k, s, pad):
    torch.manual_seed(3)
    x = torch.randn(2, 13, 13, 64, device=DEV).to(torch.bfloat16).float()
    for fk, fr in ((dnn.max_pool, ref.max_pool), (dnn.avg_pool, ref.avg_pool)):
        xr = x.clone().requires_grad_()
        yr = fr(xr, k, s, pad)
        gy = torch.randn_like(yr).to(torch.bfloat16).float()
        yr.backward(gy)
        xk = x.to(torch.bfloat16).requires_grad_()
        yk = fk(xk, k, s, pad)
        yk.backward(gy.to(torch.bfloat16))
        assert _rel(yk, yr) < 1e-2
        assert _rel(xk.grad, xr.grad) < 1e-2


def test_global_avg_and_xent():
    torch.manual_seed(4)
    x = torch.randn(8, 7, 7, 256, device=DEV).to(torch.bfloat16).float()
    xr = x.clone().requires_grad_()
    xk = x.to(torch.bfloat16).requires_grad_()
    pr, pk = ref.global_avg_pool(xr), dnn.global_avg_pool(xk)
    assert _rel(pk, pr) < 1e-3
    lab = torch.randint(0, 256, (8,), device=DEV)
    lr_ = ref.softmax_cross_entropy(pr, lab, 0.1).mean()
    lk = dnn.softmax_cross_entropy(pk, lab, 0.1).mean()
    assert abs(lr_.item() - lk.item()) < 1e-3
    lr_.backward()
    lk.backward()
    assert _rel(xk.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("distort,size", [(True, 24), (False, 24), (True, 32)])
def test_image_augment_kernel_matches_oracle(distort, size):
    """HIP crop/flip/brightness/contrast/standardise kernel vs the torch oracle, same random params."""
    import numpy as np
    from distributed_tensorflow_models_amd.data import cifar10
    imgs = torch.randint(0, 256, (16, 32, 32, 3), dtype=torch.uint8)
    ref_out = cifar10.augment(imgs, size, distort, np.random.RandomState(3), torch.float32)
    got = cifar10.augment(imgs.to(DEV), size, distort, np.random.RandomState(3), torch.float32)
    torch.cuda.synchronize()
    assert got.is_cuda and _rel(got.cpu(), ref_out) < 1e-4


@pytest.mark.parametrize("tile", [20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 40, 41, 42, 43])
@pytest.mark.parametrize("prologue", [False, True])
@pytest.mark.parametrize("case", [(4, 15, 15, 64, 96, 3, 2), (2, 14, 14, 128, 256, 3, 1), (3, 7, 7, 512, 200, 1, 1),
                                  (2, 9, 9, 24, 40, 3, 1), (4, 12, 12, 64, 256, 1, 1), (3, 7, 7, 128, 96, 1, 1),
                                  (2, 9, 9, 64, 64, 1, 1), (2, 30, 30, 128, 64, 1, 1), (4, 16, 16, 256, 512, 3, 1),
                                  (2, 19, 19, 32, 32, 3, 1), (2, 17, 17, 32, 24, 3, 2)])
def test_conv_pipelined_tiles_match_reference(tile, prologue, case):
    """The pipelined LDS-DMA conv kernels (DTM_CONV_TILE=20..23; ring of k-tiles, counted vmcnt, the
    BatchNorm-apply prologue transformed in LDS) against the fp32 reference: forward (with and without
    the prologue, zero padding kept zero), dgrad (stride-2 through the dilated path)."""
    import ctypes

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import conv_geom
    N, H, W, C, K, R, st = case
    torch.manual_seed(0)
    L = _lib.lib()
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=DEV) / (R * R * C) ** 0.5).to(torch.bfloat16)
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    g = conv_geom(tuple(x.shape), tuple(w.shape), st, "SAME")
    d = g.as_desc(_lib.ConvDesc)
    xin = torch.relu(x.float() * sc + sh).to(torch.bfloat16).float() if prologue else x.float()
    yr = ref.conv2d(xin, w.float(), None, st, "SAME")
    dy = torch.randn_like(yr).to(torch.bfloat16)
    xr = xin.clone().requires_grad_()
    ref.conv2d(xr, w.float(), None, st, "SAME").backward(dy.float())
    wt = torch.empty(C, R, R, K, device=DEV, dtype=torch.bfloat16)
    L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, _lib.stream_ptr())
    y = torch.empty(N, g.P, g.Q, K, device=DEV, dtype=torch.bfloat16)
    dx = torch.empty_like(x)
    stats = torch.zeros(2, K, device=DEV)
    L.dtm_conv_set_tile(tile)
    try:
        rc = L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), _lib.ptr(stats), None,
                            _lib.ptr(sc) if prologue else None, _lib.ptr(sh) if prologue else None, 0,
                            ctypes.byref(d), _lib.stream_ptr())
        assert rc == 0
        rc = L.dtm_conv_dgrad(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), _lib.stream_ptr())
        assert rc == 0
        torch.cuda.synchronize()
    finally:
        L.dtm_conv_set_tile(-1)
    assert _rel(y, yr) < 1e-2
    assert _rel(dx, xr.grad) < 1e-2
    # BatchNorm statistics from the epilogue = sums of the kernel's own bf16 outputs
    yf = y.float().reshape(-1, K)
    assert _rel(stats[0], yf.sum(0)) < 1e-3 and _rel(stats[1], yf.square().sum(0)) < 1e-3


@pytest.mark.parametrize("tile", [-1, 4, 21, 24, 26, 32, 40, 41])
@pytest.mark.parametrize("case", [(2, 14, 14, 128, 256, 3, 1), (3, 7, 7, 512, 200, 1, 1), (4, 15, 15, 96, 64, 3, 2),
                                  (2, 28, 28, 128, 128, 3, 2), (2, 9, 9, 64, 40, 3, 1), (2, 30, 30, 64, 128, 1, 1)])
def test_conv_act_dgrad_tiles_match_reference(tile, case):
    """dgrad with the input's BatchNorm+ReLU backward in the epilogue (the bottleneck conv2 / conv3 dgrads) on every
    tile the policy can pick: g = dgrad * [x*scale + shift > 0] (unscaled output), sums = (sum g*x, sum g) per
    channel; strided cases through the grouped parity-class dgrad."""
    import ctypes

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import conv_geom
    N, H, W, C, K, R, st = case
    torch.manual_seed(0)
    L = _lib.lib()
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=DEV) / (R * R * C) ** 0.5).to(torch.bfloat16)
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    g = conv_geom(tuple(x.shape), tuple(w.shape), st, "SAME")
    yr = ref.conv2d(x.float(), w.float(), None, st, "SAME")
    dy = torch.randn_like(yr).to(torch.bfloat16)
    xr = x.float().clone().requires_grad_()
    ref.conv2d(xr, w.float(), None, st, "SAME").backward(dy.float())
    mask = (x.float() * sc + sh) > 0
    gref = xr.grad * mask
    wt = torch.empty(C, R, R, K, device=DEV, dtype=torch.bfloat16)
    d = g.as_desc(_lib.ConvDesc)
    if st > 1:
        L.dtm_weight_flip_transpose_dec(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, st, g.pad_h, g.pad_w, _lib.stream_ptr())
        d.dec = 1
    else:
        L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, R, C, _lib.stream_ptr())
    ss4 = torch.stack([sc, sh, sh, sc]).contiguous()
    sums = torch.zeros(2, C, device=DEV)
    dx = torch.empty_like(x)
    L.dtm_conv_set_tile(tile)
    try:
        rc = L.dtm_conv_dgrad_ex(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), None, 1, _lib.ptr(x),
                                 _lib.ptr(ss4), _lib.ptr(sums), 1, _lib.stream_ptr())
        assert rc == 0
        torch.cuda.synchronize()
    finally:
        L.dtm_conv_set_tile(-1)
    assert _rel(dx, gref) < 1e-2
    assert _rel(sums[0], (gref * x.float()).sum((0, 1, 2))) < 1e-2
    assert _rel(sums[1], gref.sum((0, 1, 2))) < 1e-2


@pytest.mark.parametrize("case", [(4, 35, 35, 64, "SAME"), (4, 17, 17, 192, "SAME"), (3, 8, 8, 192, "SAME"),
                                  (2, 13, 11, 16, "VALID"), (2, 9, 10, 8, "SAME")])
@pytest.mark.parametrize("count_pad", [0, 1])
def test_avgpool_k3s1_matches_generic(case, count_pad):
    """3x3 / stride-1 average pools (Inception's pool branches) on the strip kernels vs the generic ones: output and
    input gradient bit-identical (same tap / window order and divisors); and against fp32 torch."""
    import ctypes

    import torch.nn.functional as tF

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import pool_geom
    N, H, W, C, pad = case
    torch.manual_seed(9)
    L = _lib.lib()
    s = _lib.stream_ptr()
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    g = pool_geom(tuple(x.shape), 3, 1, pad)
    a = g.as_args(_lib.PoolArgs)
    dy = torch.randn(N, g.P, g.Q, C, device=DEV).to(torch.bfloat16)
    out = {}
    for fast in (1, 0):
        L.dtm_pool_set_k3s2(fast)
        try:
            y = torch.empty(N, g.P, g.Q, C, device=DEV, dtype=torch.bfloat16)
            L.dtm_avgpool_fwd(_lib.ptr(x), _lib.ptr(y), ctypes.byref(a), count_pad, s)
            dx = torch.empty_like(x)
            L.dtm_avgpool_bwd(_lib.ptr(dy), _lib.ptr(dx), ctypes.byref(a), count_pad, s)
            torch.cuda.synchronize()
        finally:
            L.dtm_pool_set_k3s2(1)
        out[fast] = (y, dx)
    assert torch.equal(out[1][0], out[0][0]) and torch.equal(out[1][1], out[0][1])
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    yr = tF.avg_pool2d(tF.pad(xr, (g.PW, g.PR, g.PH, g.PB)), 3, 1)
    if not count_pad:  # TF SAME: divide by the in-bounds taps
        ones = tF.pad(torch.ones_like(xr[:, :1]), (g.PW, g.PR, g.PH, g.PB))
        yr = yr * 9.0 / (tF.avg_pool2d(ones, 3, 1) * 9.0)
    assert _rel(out[1][0].float().permute(0, 3, 1, 2), yr) < 1e-2
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(out[1][1].float(), xr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.parametrize("case", [(4, 17, 17, 768, 5, 3, "VALID"), (3, 8, 8, 2048, 8, 1, "VALID"),
                                  (2, 11, 9, 24, 3, 2, "SAME"), (2, 12, 12, 16, 2, 2, "SAME")])
@pytest.mark.parametrize("count_pad", [0, 1])
def test_avgpool_generic8_and_accumulating_backward(case, count_pad):
    """The generic 8-channel avg pool (32-bit index kernels: Inception's 5x5/3 aux-head pool) against fp32 torch,
    and its accumulating backward dx += pool_bwd(dy) (the aux head's gradient added into the main path's) against
    the plain backward plus the prior dx."""
    import ctypes

    import torch.nn.functional as tF

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import pool_geom
    N, H, W, C, k, st, pad = case
    torch.manual_seed(4)
    L = _lib.lib()
    s = _lib.stream_ptr()
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    g = pool_geom(tuple(x.shape), k, st, pad)
    a = g.as_args(_lib.PoolArgs)
    dy = torch.randn(N, g.P, g.Q, C, device=DEV).to(torch.bfloat16)
    y = torch.empty(N, g.P, g.Q, C, device=DEV, dtype=torch.bfloat16)
    L.dtm_avgpool_fwd(_lib.ptr(x), _lib.ptr(y), ctypes.byref(a), count_pad, s)
    dx = torch.empty_like(x)
    L.dtm_avgpool_bwd(_lib.ptr(dy), _lib.ptr(dx), ctypes.byref(a), count_pad, s)
    prior = torch.randn_like(x, dtype=torch.float32).to(torch.bfloat16)
    acc = prior.clone()
    assert L.dtm_avgpool_bwd_acc(_lib.ptr(dy), _lib.ptr(acc), ctypes.byref(a), count_pad, s) == 0
    torch.cuda.synchronize()
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    yr = tF.avg_pool2d(tF.pad(xr, (g.PW, g.PR, g.PH, g.PB)), k, st)
    if not count_pad:
        ones = tF.pad(torch.ones_like(xr[:, :1]), (g.PW, g.PR, g.PH, g.PB))
        yr = yr / tF.avg_pool2d(ones, k, st)
    assert _rel(y.float().permute(0, 3, 1, 2), yr) < 1e-2
    yr.backward(dy.float().permute(0, 3, 1, 2))
    gx = xr.grad.permute(0, 2, 3, 1)
    assert _rel(dx.float(), gx) < 1e-2
    assert _rel(acc.float(), prior.float() + gx) < 1e-2
    # one rounding of (prior + exact fp32 pool gradient): within half a bf16 ulp of it
    ref = prior.float() + dx.float()
    assert float((acc.float() - ref).abs().max()) <= float(ref.abs().max()) * 2 ** -7


@pytest.mark.parametrize("case", [(4, 35, 35, 288, "VALID"), (4, 17, 17, 768, "VALID"), (2, 15, 14, 16, "SAME"),
                                  (3, 9, 10, 8, "VALID"), (2, 13, 13, 2048, "SAME")])
def test_maxpool_k3s2_matches_generic(case):
    """The plain 3x3 / stride-2 max pool (Inception's grid-reduction branches) on the specialised kernels vs the
    generic ones: output, argmax bytes and input gradient bit-identical; and against fp32 torch."""
    import ctypes

    import torch.nn.functional as tF

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import pool_geom
    N, H, W, C, pad = case
    torch.manual_seed(8)
    L = _lib.lib()
    s = _lib.stream_ptr()
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    g = pool_geom(tuple(x.shape), 3, 2, pad)
    a = g.as_args(_lib.PoolArgs)
    dy = torch.randn(N, g.P, g.Q, C, device=DEV).to(torch.bfloat16)
    out = {}
    for fast in (1, 0):
        L.dtm_pool_set_k3s2(fast)
        try:
            y = torch.empty(N, g.P, g.Q, C, device=DEV, dtype=torch.bfloat16)
            arg = torch.empty(N, g.P, g.Q, C, device=DEV, dtype=torch.uint8)
            L.dtm_maxpool_fwd(_lib.ptr(x), _lib.ptr(y), _lib.ptr(arg), ctypes.byref(a), s)
            dx = torch.empty_like(x)
            L.dtm_maxpool_bwd(_lib.ptr(dy), _lib.ptr(arg), _lib.ptr(dx), ctypes.byref(a), s)
            torch.cuda.synchronize()
        finally:
            L.dtm_pool_set_k3s2(1)
        out[fast] = (y, arg, dx)
    for i in range(3):
        assert torch.equal(out[1][i], out[0][i]), i
    if C % 8 == 0:  # dy read in place as the channel slice of a wider (concat) gradient
        wide = torch.randn(N, g.P, g.Q, C + 24, device=DEV).to(torch.bfloat16)
        wide[..., 8:8 + C] = dy
        dxs = torch.empty_like(x)
        assert L.dtm_maxpool_bwd_ld(_lib.ptr(wide[..., 8:8 + C]), C + 24, _lib.ptr(out[1][1]), _lib.ptr(dxs),
                                    ctypes.byref(a), s) == 0
        torch.cuda.synchronize()
        assert torch.equal(dxs, out[1][2])
    xr = x.float().permute(0, 3, 1, 2).contiguous().requires_grad_()
    yr = tF.max_pool2d(tF.pad(xr, (g.PW, g.PR, g.PH, g.PB), value=-1e30), 3, 2)
    assert torch.equal(out[1][0].float().permute(0, 3, 1, 2), yr)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(out[1][2].float(), xr.grad.permute(0, 2, 3, 1)) < 2e-2  # (bf16 ties may route differently)


@pytest.mark.parametrize("case", [(4, 112, 112, 64, "SAME"), (3, 147, 147, 64, "VALID"), (2, 71, 71, 192, "VALID"),
                                  (2, 15, 14, 16, "SAME"), (3, 9, 10, 8, "VALID"), (2, 13, 13, 24, "SAME")])
@pytest.mark.parametrize("unscaled", [0, 1])
def test_maxpool_bnrelu_k3s2_matches_generic(case, unscaled):
    """The 3x3 / stride-2 stem-pool kernels (two outputs per lane forward, a 2x2 input block per lane backward) vs the
    generic gather kernels: pooled output and argmax bytes bit-identical (same scan order, strict comparison), input
    gradient bit-identical (same window order), the BN-gradient sums equal up to the summation order; and both
    against fp32 torch (max_pool2d of relu(x*scale+shift), its gradient)."""
    import ctypes

    import torch.nn.functional as tF

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import pool_geom
    N, H, W, C, pad = case
    torch.manual_seed(7)
    L = _lib.lib()
    s = _lib.stream_ptr()
    raw = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    sc, sh = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV) * 0.3
    ss = torch.stack([sc, sh, sh, sc]).contiguous()
    g = pool_geom(tuple(raw.shape), 3, 2, pad)
    a = g.as_args(_lib.PoolArgs)
    dy = torch.randn(N, g.P, g.Q, C, device=DEV).to(torch.bfloat16)
    out = {}
    for fast in (1, 0):
        L.dtm_pool_set_k3s2(fast)
        try:
            y = torch.empty(N, g.P, g.Q, C, device=DEV, dtype=torch.bfloat16)
            arg = torch.empty(N, g.P, g.Q, C, device=DEV, dtype=torch.uint8)
            assert L.dtm_maxpool_bnrelu_fwd(_lib.ptr(raw), _lib.ptr(ss), _lib.ptr(y), _lib.ptr(arg), ctypes.byref(a),
                                            s) == 0
            dx = torch.empty_like(raw)
            sums = torch.zeros(4, C, device=DEV)
            assert L.dtm_maxpool_bnrelu_bwd(_lib.ptr(dy), _lib.ptr(arg), _lib.ptr(raw), _lib.ptr(ss), _lib.ptr(dx),
                                            _lib.ptr(sums), ctypes.byref(a), unscaled, s) == 0
            torch.cuda.synchronize()
        finally:
            L.dtm_pool_set_k3s2(1)
        out[fast] = (y, arg, dx, sums)
    for i in range(3):
        assert torch.equal(out[1][i], out[0][i]), i
    assert _rel(out[1][3][:2], out[0][3][:2]) < 1e-5
    # fp32 reference (NCHW torch pooling; TF SAME padding as explicit -inf pads)
    act = torch.relu(raw.float() * sc + sh).permute(0, 3, 1, 2).contiguous().requires_grad_()
    padded = tF.pad(act, (g.PW, g.PR, g.PH, g.PB), value=-1e30)
    yr = tF.max_pool2d(padded, 3, 2)
    assert _rel(out[1][0].float().permute(0, 3, 1, 2), yr) < 1e-2
    yr.backward(dy.float().permute(0, 3, 1, 2))
    m = (raw.float() * sc + sh > 0).float()
    gref = act.grad.permute(0, 2, 3, 1) * m  # (ties: torch and the kernels may route to different maxima)
    want = gref if unscaled else gref * sc
    assert _rel(out[1][2].float(), want) < 2e-2
    assert _rel(out[1][3][0], (gref * raw.float()).sum((0, 1, 2))) < 2e-2
    assert _rel(out[1][3][1], gref.sum((0, 1, 2))) < 2e-2


@pytest.mark.parametrize("case", [(4, 28, 28, 64, 256, True, True), (4, 28, 28, 64, 256, False, True),
                                  (3, 13, 13, 128, 512, True, False), (2, 9, 11, 128, 384, False, True),
                                  (5, 14, 14, 64, 128, True, True), (3, 14, 14, 256, 1024, False, True),
                                  (2, 7, 9, 256, 256, True, True)])
def test_conv_bnout_dgrad(case):
    """Block-output dgrad (the next unit's 1x1 conv1 consuming relu(bn(conv3) + residual)): total = dgrad +
    add_src, g = total * ReLU bit, sums rows 0-1 = (sum g*x_raw, sum g), rows 4-5 = (sum g*r_raw, sum g) with a BN'd
    residual (ragged pixel tails; reductions of 64 / 128 / 256)."""
    import ctypes

    import numpy as np

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import conv_geom
    N, H, W, Kc, C, has_r, has_add = case  # Kc: conv1's output channels (the dgrad's reduction), C: its input
    torch.manual_seed(0)
    L = _lib.lib()
    w = (torch.randn(Kc, 1, 1, C, device=DEV) / C ** 0.5).to(torch.bfloat16)
    g = conv_geom((N, H, W, C), tuple(w.shape), 1, "SAME")
    dy = torch.randn(N, H, W, Kc, device=DEV).to(torch.bfloat16)
    wt = torch.empty(C, 1, 1, Kc, device=DEV, dtype=torch.bfloat16)
    L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), Kc, 1, 1, C, _lib.stream_ptr())
    add = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16) if has_add else None
    xr = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    rr = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16) if has_r else None
    bits = np.random.RandomState(1).rand(N * H * W * C) > 0.4
    mask = torch.from_numpy(np.packbits(bits, bitorder="little")).to(DEV)
    bm = torch.from_numpy(bits.reshape(N, H, W, C)).to(DEV).float()
    tot = torch.einsum("nhwk,kc->nhwc", dy.float(), w.float().reshape(Kc, C))
    if has_add:
        tot = tot + add.float()
    gref = tot * bm
    dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    sums = torch.zeros(8, C, device=DEV)
    d = g.as_desc(_lib.ConvDesc)
    rc = L.dtm_conv_dgrad_bnout(_lib.ptr(dy), _lib.ptr(wt), _lib.ptr(dx), ctypes.byref(d), _lib.ptr(add), 1,
                                _lib.ptr(mask), _lib.ptr(xr), _lib.ptr(rr), _lib.ptr(sums), _lib.stream_ptr())
    assert rc == 0
    torch.cuda.synchronize()
    assert _rel(dx, gref) < 1e-2
    assert _rel(sums[0], (gref * xr.float()).sum((0, 1, 2))) < 1e-2
    assert _rel(sums[1], gref.sum((0, 1, 2))) < 1e-2
    if has_r:
        assert _rel(sums[4], (gref * rr.float()).sum((0, 1, 2))) < 1e-2
        assert _rel(sums[5], gref.sum((0, 1, 2))) < 1e-2


@pytest.mark.parametrize("case", [(2, 8, 1280, [320, 384, 448, 192]), (128, 8, 2048, [320, 384, 448, 192]),
                                  (3, 35, 288, [64, 48, 64, 32]), (8, 17, 768, [192, 128, 128, 192]),
                                  (4, 14, 256, [512, 128]), (2, 17, 768, [192, 192])])
def test_conv_fwd_bn_multi_matches_separate(case):
    """Merged sibling forward (dtm_conv_fwd_bn_multi): one 1x1 conv over the members' concatenated weights writing
    each member's own output + one grouped finalize, vs one dtm_conv_fwd_bn per member: outputs, ss and moving
    statistics (the last member without BatchNorm: its ss untouched)."""
    import ctypes

    from distributed_tensorflow_models_amd.ops import _lib
    N, H, C, ks = case
    torch.manual_seed(0)
    L = _lib.lib()
    st = _lib.stream_ptr()
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    ws = [(torch.randn(k, 1, 1, C, device=DEV) / C ** 0.5).to(torch.bfloat16) for k in ks]
    wcat = torch.cat(ws).contiguous()
    nbn = len(ks) - 1  # the last member has no BatchNorm
    beta = [torch.randn(k, device=DEV) for k in ks]
    mm = [torch.randn(k, device=DEV) * 0.1 for k in ks]
    mv = [torch.rand(k, device=DEV) + 0.5 for k in ks]
    M = N * H * H
    ref_y, ref_ss, ref_mm, ref_mv = [], [], [], []
    for i, (w, k) in enumerate(zip(ws, ks)):
        d = _lib.ConvDesc(N, H, H, C, k, 1, 1, H, H, 1, 0, 0, 0, 0)
        y = torch.empty(N, H, H, k, device=DEV, dtype=torch.bfloat16)
        m2, v2 = mm[i].clone(), mv[i].clone()
        ss = torch.zeros(4, k, device=DEV)
        if i < nbn:
            assert L.dtm_conv_fwd_bn(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, None, _lib.ptr(beta[i]),
                                     _lib.ptr(m2), _lib.ptr(v2), _lib.ptr(ss), float(M), 1e-3, 0.9997, 1, 0,
                                     ctypes.byref(d), st) == 0
        else:
            assert L.dtm_conv_fwd(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, None, None, 0, ctypes.byref(d),
                                  st) == 0
        ref_y.append(y); ref_ss.append(ss); ref_mm.append(m2); ref_mv.append(v2)
    ys = [torch.empty(N, H, H, k, device=DEV, dtype=torch.bfloat16) for k in ks]
    sss = [torch.zeros(4, k, device=DEV) for k in ks]
    m3, v3 = [t.clone() for t in mm], [t.clone() for t in mv]
    ptrs = []
    for i in range(len(ks)):
        ptrs += ([0, beta[i].data_ptr(), m3[i].data_ptr(), v3[i].data_ptr(), sss[i].data_ptr()] if i < nbn
                 else [0, 0, 0, 0, 0])
    d = _lib.ConvDesc(N, H, H, C, sum(ks), 1, 1, H, H, 1, 0, 0, 0, 0)
    rc = L.dtm_conv_fwd_bn_multi(_lib.ptr(x), _lib.ptr(wcat), (ctypes.c_void_p * len(ys))(*[y.data_ptr() for y in ys]),
                                 (ctypes.c_int * len(ks))(*ks), len(ks), (ctypes.c_void_p * len(ptrs))(*ptrs),
                                 float(M), 1e-3, 0.9997, 1, 0, ctypes.byref(d), st)
    assert rc == 0
    torch.cuda.synchronize()
    for i in range(len(ks)):
        assert torch.equal(ys[i], ref_y[i]), (i, _rel(ys[i], ref_y[i]))
        if i < nbn:
            assert _rel(sss[i], ref_ss[i]) < 1e-5, (i, _rel(sss[i], ref_ss[i]))
            assert _rel(m3[i], ref_mm[i]) < 1e-5 and _rel(v3[i], ref_mv[i]) < 1e-5
        else:
            assert not sss[i].any()


@pytest.mark.parametrize("prologue", [False, True])
@pytest.mark.parametrize("case", [(2, 19, 21, 32, 32, "SAME"), (3, 17, 18, 32, 64, "VALID"), (2, 13, 15, 64, 64, "SAME"),
                                  (1, 8, 40, 64, 96, "SAME"), (2, 25, 9, 32, 32, "VALID")])
def test_conv3x3_wgrad_direct_matches_reference(prologue, case):
    """conv3x3_wgrad_direct_kernel (wgrad tile 20: per 8x16 output tile, dy^T and three column-shifted x halo copies
    staged once, channel-major, in LDS; the optional BN-apply prologue applied to the staged x with the zero padding
    kept zero) against the fp32 reference: partial edge tiles, VALID / SAME padding, 32 / 64 input channels, one and
    several 32-row dW tiles."""
    import ctypes

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import conv_geom
    N, H, W, C, K, pad = case
    torch.manual_seed(1)
    L = _lib.lib()
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    w = torch.randn(K, 3, 3, C, device=DEV).to(torch.bfloat16)
    sc = torch.rand(C, device=DEV) + 0.5
    sh = torch.randn(C, device=DEV) * 0.5
    g = conv_geom(tuple(x.shape), tuple(w.shape), 1, pad)
    d = g.as_desc(_lib.ConvDesc)
    dy = torch.randn(N, g.P, g.Q, K, device=DEV).to(torch.bfloat16)
    xin = torch.relu(x.float() * sc + sh).to(torch.bfloat16).float() if prologue else x.float()
    wr = w.float().clone().requires_grad_()
    ref.conv2d(xin, wr, None, 1, pad).backward(dy.float())
    dw = torch.zeros(K, 3, 3, C, device=DEV)
    L.dtm_conv_set_wgrad_tile(20, 0)
    try:
        rc = L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), _lib.ptr(sc) if prologue else None,
                              _lib.ptr(sh) if prologue else None, ctypes.byref(d), _lib.num_cus(), _lib.stream_ptr())
        torch.cuda.synchronize()
    finally:
        L.dtm_conv_set_wgrad_tile(-1, 4)
    assert rc == 0
    assert _rel(dw, wr.grad) < 1e-3, _rel(dw, wr.grad)


@pytest.mark.parametrize("tile", [0, 1, 6, 10, 11, 12, 13])
@pytest.mark.parametrize("case", [(4, 15, 15, 64, 96, 3, 2), (2, 14, 14, 128, 256, 3, 1), (3, 7, 7, 512, 200, 1, 1),
                                  (2, 9, 9, 24, 40, 3, 1), (5, 8, 8, 64, 64, 1, 1), (4, 9, 9, 256, 512, 3, 1),
                                  (3, 13, 13, 32, 32, 3, 1), (2, 11, 11, 32, 24, 3, 2), (16, 14, 14, 512, 512, 3, 1)])
def test_conv_wgrad_pipelined_tiles_match_reference(tile, case):
    """The wgrad kernels - register-staged tiles 0 / 1 / 6 (128 / 64 / 32 rows x 128 columns) and the pipelined (10: 128 x 128, 11: 64 x 256, 12: 256 x 256,
    13: its ping-pong form) LDS-DMA ones (inverse transposed-read image mapping for the DMA slots) - with split-K slabs against the
    fp32 reference, including K / R*S*C tails and empty splits."""
    import ctypes

    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.geometry import conv_geom
    N, H, W, C, K, R, st = case
    torch.manual_seed(0)
    L = _lib.lib()
    x = torch.randn(N, H, W, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, R, R, C, device=DEV) / (R * R * C) ** 0.5).to(torch.bfloat16)
    g = conv_geom(tuple(x.shape), tuple(w.shape), st, "SAME")
    d = g.as_desc(_lib.ConvDesc)
    wr = w.float().clone().requires_grad_()
    yr = ref.conv2d(x.float(), wr, None, st, "SAME")
    dy = torch.randn_like(yr).to(torch.bfloat16)
    yr.backward(dy.float())
    dw = torch.zeros(K, R, R, C, device=DEV)
    L.dtm_conv_set_wgrad_tile(tile, 0)
    try:
        rc = L.dtm_conv_wgrad(_lib.ptr(x), _lib.ptr(dy), _lib.ptr(dw), None, None, ctypes.byref(d), _lib.num_cus(),
                              _lib.stream_ptr())
        assert rc == 0
        torch.cuda.synchronize()
    finally:
        L.dtm_conv_set_wgrad_tile(-1, 0)
    assert _rel(dw, wr.grad) < 1e-2


@pytest.mark.parametrize("shape", [(256, 1000), (48, 1008), (4, 7, 7, 64), (3, 24), (128, 35, 35, 64)])
def test_bias_column_sums_match_torch(shape):
    """Bias gradients (column sums of a bf16 [.., K] gradient) on the BN-statistics kernel into the step's zero arena
    when the parameter has a data-parallel gradient slot, vs the fp32 torch reduction; other cases take torch."""
    from distributed_tensorflow_models_amd.ops import nn as F
    from distributed_tensorflow_models_amd.ops.fused import arena
    torch.manual_seed(13)
    g = torch.randn(*shape, device=DEV).to(torch.bfloat16)
    K = shape[-1]
    p = torch.nn.Parameter(torch.zeros(K, device=DEV))
    want = g.reshape(-1, K).float().sum(0)
    assert _rel(F._col_sums(g.reshape(-1, K), p), want) < 1e-5  # (no slot: torch)
    p.main_grad = torch.zeros(K, device=DEV)
    outs = []
    for _ in range(2):  # (fixed summation order: bit-identical run to run, outside DTM_DETERMINISTIC too)
        arena.begin_step(g.device)
        try:
            outs.append(F._col_sums(g.reshape(-1, K), p).clone())
            torch.cuda.synchronize()
        finally:
            arena.end_step()
    assert _rel(outs[0], want) < 1e-5
    assert torch.equal(outs[0], outs[1])


def test_softmax_xent_backward_beyond_grid_y_limit():
    """Per-row loss backward (dtm_scale_rows_pad) at a batch past the 65535 grid.y limit: rows grid-stride, same
    values as the torch expression (it returned -1 there)."""
    from distributed_tensorflow_models_amd.ops import nn as F
    torch.manual_seed(5)
    B, N = 70000, 10
    logits = torch.randn(B, N, device=DEV).requires_grad_()
    labels = torch.randint(0, N, (B,), device=DEV)
    loss = F.softmax_cross_entropy(logits, labels)
    gl = torch.rand(B, device=DEV)
    (loss * gl).sum().backward()
    lr = logits.detach().clone().requires_grad_()
    ref_loss = torch.nn.functional.cross_entropy(lr, labels, reduction="none")
    (ref_loss * gl).sum().backward()
    assert _rel(loss.detach(), ref_loss.detach()) < 1e-4
    assert _rel(logits.grad, lr.grad) < 1e-4


@pytest.mark.parametrize("shape", [(64, 8, 8, 2048), (16, 7, 7, 2048), (3, 5, 3, 24), (2, 3, 3, 12)])
@pytest.mark.parametrize("out_bf16", [False, True])
def test_global_avg_pool_shapes_match_torch(shape, out_bf16):
    """Global mean pool (8-channel split-row kernel when C % 8 == 0, the per-channel one otherwise) forward and
    backward against fp32 torch, for fp32 and bf16 outputs."""
    from distributed_tensorflow_models_amd.ops import nn as F
    torch.manual_seed(15)
    x = torch.randn(*shape, device=DEV).to(torch.bfloat16)
    xk = x.clone().requires_grad_()
    y = F.global_avg_pool(xk, out_bf16=out_bf16)
    xr = x.float().requires_grad_()
    yr = xr.mean(dim=(1, 2))
    assert y.shape == yr.shape
    assert _rel(y.float(), yr) < (4e-3 if out_bf16 else 1e-5)
    dy = torch.randn_like(yr)
    y.backward(dy.to(y.dtype))
    yr.backward(dy.to(y.dtype).float())
    assert _rel(xk.grad.float(), xr.grad) < 4e-3


@pytest.mark.parametrize("C", [2048, 64])
def test_global_avg_pool_bf16_output_matches_cast(C):
    """The bf16-output global average pool (the ResNet logits input) == the fp32 pool cast to bf16, forward and
    backward (a bf16 incoming gradient)."""
    from distributed_tensorflow_models_amd.ops import nn as F
    torch.manual_seed(14)
    x = torch.randn(8, 7, 7, C, device=DEV).to(torch.bfloat16)
    xa, xb = x.clone().requires_grad_(), x.clone().requires_grad_()
    ya = F.global_avg_pool(xa).to(torch.bfloat16)
    yb = F.global_avg_pool(xb, out_bf16=True)
    assert yb.dtype == torch.bfloat16 and torch.equal(ya, yb)
    dy = torch.randn_like(yb)
    ya.backward(dy)
    yb.backward(dy)
    assert torch.equal(xa.grad, xb.grad)


@pytest.mark.parametrize("N", [1001, 1000, 10])
def test_fc_softmax_xent_padded_head_matches_torch(N):
    """Logits FC + label-smoothed softmax cross-entropy (the Inception-v3 / ResNet heads): the loss backward writes the
    row-scaled gradient in one HIP pass, into an 8-aligned zero-padded buffer that the FC backward takes as its padded
    operand (N % 8 != 0), and the padded flipped / bf16 weight copies persist per weights version - loss, input, weight
    and bias gradients against fp32 torch, over two versions of the weights."""
    from distributed_tensorflow_models_amd.ops import nn as F
    torch.manual_seed(12)
    B, Kin = 48, 256
    x = torch.randn(B, Kin, device=DEV)
    labels = torch.randint(0, N, (B,), device=DEV)
    w = torch.nn.Parameter((torch.randn(Kin, N, device=DEV) / Kin ** 0.5))
    b = torch.nn.Parameter(torch.randn(N, device=DEV) * 0.1)
    used0 = F.PAD_BASE_USED[0]
    for version in range(2):
        if version:
            with torch.no_grad():
                w.add_(0.01)
                b.add_(0.02)
            F.invalidate_weight_copies([w])
            F.refresh_flipped()
        w.grad = b.grad = None
        xi = x.clone().requires_grad_()
        logits = F.linear(xi.to(torch.bfloat16), w, b)
        assert logits.is_contiguous() == (N % 8 == 0)  # (a padded head's output is read in place by the loss)
        loss = 0.4 * F.softmax_cross_entropy(logits, labels, 0.1).mean()
        loss.backward()
        torch.cuda.synchronize()
        xr = x.clone().requires_grad_()
        wr, br = w.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
        lr = xr.to(torch.bfloat16).float() @ wr.to(torch.bfloat16).float() + br
        lref = 0.4 * ref.softmax_cross_entropy(lr, labels, 0.1).mean()
        lref.backward()
        assert abs(float(loss.detach()) - float(lref.detach())) < 2e-2 * max(1.0, abs(float(lref.detach())))
        assert _rel(xi.grad, xr.grad) < 3e-2
        assert _rel(w.grad, wr.grad) < 3e-2 and _rel(b.grad, br.grad) < 3e-2
    if N % 8:
        assert F.PAD_BASE_USED[0] >= used0 + 2


@pytest.mark.parametrize("bw", [1.0, 0.5])
def test_mean_xent_loss_fused_matches_composition(bw):
    """The fused training loss (main head + 0.4-weighted aux head, batch weight bw) against the composition of
    per-row xent, means and weights: the loss to fp32 rounding, and both heads' logits gradients and the FCs' padded
    backward hand-off (PAD_BASE_USED) through a real FC pair."""
    from distributed_tensorflow_models_amd.ops import nn as F
    torch.manual_seed(13)
    B, Kin, N = 64, 128, 1001
    x = torch.randn(B, Kin, device=DEV).to(torch.bfloat16)
    labels = torch.randint(0, N, (B,), device=DEV)
    ws = [torch.nn.Parameter(torch.randn(Kin, N, device=DEV) / Kin ** 0.5) for _ in range(2)]
    out = []
    for fused in (True, False):
        for w in ws:
            w.grad = None
        xi = x.clone().requires_grad_()
        used0 = F.PAD_BASE_USED[0]
        la, lb = F.linear(xi, ws[0], None), F.linear(xi * 2, ws[1], None)
        if fused:
            loss = F.mean_xent_loss([(la, bw), (lb, 0.4 * bw)], labels, 0.1)
        else:
            loss = (F.softmax_cross_entropy(la, labels, 0.1).mean()
                    + 0.4 * F.softmax_cross_entropy(lb, labels, 0.1).mean()) * bw
        loss.backward()
        torch.cuda.synchronize()
        out.append((float(loss.detach()), xi.grad.float(), [w.grad.clone() for w in ws], F.PAD_BASE_USED[0] - used0))
    (l1, gx1, gw1, u1), (l2, gx2, gw2, u2) = out
    assert abs(l1 - l2) <= 1e-5 * abs(l2), (l1, l2)
    assert _rel(gx1, gx2) < 1e-2
    for a, b in zip(gw1, gw2):
        assert _rel(a, b) < 1e-2
    assert u1 == 2 and u2 == 2


@pytest.mark.parametrize("tile", [10, 11, 12, 13, 14, 15])
def test_conv_lds_dma_tiles_match_default(tile):
    """The opt-in LDS-DMA conv kernels (DTM_CONV_TILE=10..12) give the default kernel's results
    (fwd with padding, stride-2 dgrad through the dilated path)."""
    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops import nn as F
    outs = []
    for t in (-1, tile):
        _lib.lib().dtm_conv_set_tile(t)
        try:
            torch.manual_seed(0)
            x = torch.randn(4, 15, 15, 64, device="cuda").to(torch.bfloat16).requires_grad_()
            w = (torch.randn(96, 3, 3, 64, device="cuda") * 0.05).requires_grad_()
            y = F.conv2d(x, w, None, 2, "SAME")
            y.float().square().sum().backward()
            torch.cuda.synchronize()
            outs.append((y.detach().float(), x.grad.float()))
        finally:
            _lib.lib().dtm_conv_set_tile(-1)
    for i, k in enumerate(("y", "dx")):
        a, b = outs[0][i], outs[1][i]
        assert ((a - b).norm() / b.norm()).item() < 1e-2, k


@pytest.mark.parametrize("dtype,n", [(torch.bfloat16, 4096 * 33 + 5), (torch.float32, 1000003), (torch.bfloat16, 7)])
def test_dropout_kernel_matches_hash_mask(dtype, n):
    """HIP dropout regenerates exactly the CPU hash mask (forward and backward, nothing stored)."""
    from distributed_tensorflow_models_amd.ops import elementwise as E
    E.seed_offset(torch.device(DEV, 0)).zero_()  # engine steps earlier in this process advance it
    x = torch.randn(n, device=DEV).to(dtype).requires_grad_()
    y = E.dropout(x, 0.7, seed=123456789)
    mask = E.dropout_mask((n,), 0.7, 123456789).to(DEV)
    want = torch.where(mask, x.detach().float() / 0.7, torch.zeros((), device=DEV))
    torch.testing.assert_close(y.float(), want, rtol=1e-2 if dtype == torch.bfloat16 else 1e-6, atol=1e-6)
    g = torch.randn(n, device=DEV).to(dtype)
    y.backward(g)
    torch.testing.assert_close(x.grad.float(), torch.where(mask, g.float() / 0.7, torch.zeros((), device=DEV)),
                               rtol=1e-2 if dtype == torch.bfloat16 else 1e-6, atol=1e-6)


@pytest.mark.parametrize("B,K,dtype", [(256, 1000, torch.bfloat16), (37, 10, torch.float32), (5, 1001, torch.float32)])
def test_in_top_k_kernel(B, K, dtype):
    from distributed_tensorflow_models_amd.ops import elementwise as E
    torch.manual_seed(5)
    p = torch.randn(B, K).to(dtype)
    p[0, :] = 0.0                      # all-tie row
    t = torch.randint(0, K, (B,))
    t[1] = -1                          # invalid label
    for k in (1, 5):
        got = E.in_top_k(p.to(DEV), t.to(DEV), k).cpu()
        assert torch.equal(got, E.in_top_k(p.float(), t, k))


def test_weight_flip_tiled_and_batched():
    """dgrad weight copies [C][R'][S'][K] (taps flipped) from [K][R][S][C]: the single-weight and the
    batched (post-optimizer refresh) launches, ragged 64-tiles included."""
    import numpy as np
    from distributed_tensorflow_models_amd.ops import _lib
    L = _lib.lib()
    shapes = [(64, 3, 3, 64), (100, 7, 7, 24), (2048, 1, 1, 512), (8, 1, 1, 8), (72, 5, 3, 136)]
    ws = [torch.randn(s, device=DEV).to(torch.bfloat16) for s in shapes]
    want = [w.flip(1, 2).permute(3, 1, 2, 0).contiguous() for w in ws]
    for w, ref_ in zip(ws, want):
        K, R, S, C = w.shape
        wt = torch.empty(C, R, S, K, device=DEV, dtype=torch.bfloat16)
        L.dtm_weight_flip_transpose(_lib.ptr(w), _lib.ptr(wt), K, R, S, C, _lib.stream_ptr())
        assert torch.equal(wt, ref_)
    outs = [torch.empty_like(r) for r in want]
    nb = L.dtm_flip_desc_bytes()
    tab = np.zeros((len(ws), nb // 8), dtype=np.int64)
    for i, (w, o) in enumerate(zip(ws, outs)):
        tab[i, 0], tab[i, 1] = w.data_ptr(), o.data_ptr()
        K, R, S, C = w.shape
        tab[i, 2:4] = np.array([K, R, S, C], dtype=np.int32).view(np.int64)
    dev_tab = torch.from_numpy(tab.view(np.uint8).reshape(-1).copy()).to(DEV)
    L.dtm_weight_flip_transpose_batched(_lib.ptr(dev_tab), len(ws), _lib.stream_ptr())
    torch.cuda.synchronize()
    for o, r in zip(outs, want):
        assert torch.equal(o, r)


@pytest.mark.parametrize("H,R,K,C,use_main_grad", [(1, 7, 256, 64, True), (2, 5, 24, 16, False), (3, 7, 16, 8, True)])
def test_conv_dead_taps_cropped(H, R, K, C, use_main_grad):
    """Taps that only ever read zero padding are cropped away (VGG fc6 on a 1x1 map): y, dx and
    the full-size dw (zeros on the dead taps) match the fp32 reference of the uncropped conv."""
    from distributed_tensorflow_models_amd.ops import nn as F
    from distributed_tensorflow_models_amd.ops import reference as ref
    torch.manual_seed(0)
    x = torch.randn(8, H, H, C)
    w = torch.nn.Parameter(torch.randn(K, R, R, C) * 0.1)
    dy = torch.randn(8, H, H, K)
    xr = x.clone().requires_grad_()
    wr = w.detach().clone().requires_grad_()
    yr = ref.conv2d(xr, wr, None, 1, "SAME", False, 1)
    yr.backward(dy)
    wg = torch.nn.Parameter(w.detach().to(DEV))
    if use_main_grad:
        wg.main_grad = torch.zeros(wg.shape, device=DEV)
    xg = x.to(DEV, torch.bfloat16).requires_grad_()
    y = F.conv2d(xg, wg, None, 1, "SAME")
    y.backward(dy.to(DEV, torch.bfloat16))
    dw = wg.main_grad if use_main_grad else wg.grad
    for a, b in ((y, yr), (xg.grad, xr.grad), (dw, wr.grad)):
        a = a.float().cpu()
        assert ((a - b).norm() / b.norm()).item() < 2e-2
    c = R // 2
    if H == 1:
        assert float(dw.abs().sum() - dw[:, c, c].abs().sum()) == 0.0  # only the centre tap is live


@pytest.mark.parametrize("K,H", [(64, 16), (200, 7), (512, 2)])
def test_conv_relu_bias_backward_fused(K, H):
    """conv + bias + ReLU backward: mask and bias-gradient sums from one HIP pass, vs fp32 torch.

    The fp32 reference back-propagates through the GPU's own ReLU mask (y > 0 of the bf16 output):
    elements within bf16 rounding of zero would otherwise flip and dominate the bias-sum error."""
    torch.manual_seed(0)
    x = torch.randn(8, H, H, 32).bfloat16().float()
    w = torch.randn(K, 3, 3, 32) * 0.1
    b = torch.randn(K) * 0.1
    dy = torch.randn(8, H, H, K).bfloat16().float()
    xg = x.to(DEV, torch.bfloat16).requires_grad_()
    wg = torch.nn.Parameter(w.to(DEV))
    bg = torch.nn.Parameter(b.to(DEV))
    y = dnn.conv2d(xg, wg, bg, 1, "SAME", relu=True)
    y.backward(dy.to(DEV, torch.bfloat16))
    mask = (y.detach().float().cpu() > 0).float()
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    ref.conv2d(xr, wr, br, 1, "SAME", False, 1).backward(dy * mask)
    assert _rel(bg.grad.cpu(), br.grad) < 5e-3
    assert _rel(wg.grad.cpu(), wr.grad) < 2e-2
    assert _rel(xg.grad.float().cpu(), xr.grad) < 2e-2


@pytest.mark.parametrize("B,N,relu", [(64, 384, True), (37, 192, True), (16, 1000, False), (8, 24, True), (32, 10, False), (5, 1001, True)])
def test_linear_bias_relu_fused(B, N, relu):
    """FC layer: bias in the GEMM epilogue, ReLU mask + bias sums in one HIP pass, vs fp32 torch
    through the GPU's own ReLU mask."""
    torch.manual_seed(0)
    x = torch.randn(B, 96).bfloat16().float()
    w = torch.randn(96, N) * 0.1
    b = torch.randn(N) * 0.1
    dy = torch.randn(B, N).bfloat16().float()
    xg = x.to(DEV, torch.bfloat16).requires_grad_()
    wg = torch.nn.Parameter(w.to(DEV))
    bg = torch.nn.Parameter(b.to(DEV))
    y = dnn.linear(xg, wg, bg, relu=relu)
    y.backward(dy.to(DEV, torch.bfloat16))
    mask = (y.detach().float().cpu() > 0).float() if relu else torch.ones(B, N)
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    yr = xr @ wr + br
    assert _rel(y.float().cpu(), torch.relu(yr) if relu else yr) < 2e-2
    yr.backward(dy * mask)
    assert _rel(bg.grad.cpu(), br.grad) < 5e-3
    assert _rel(wg.grad.cpu(), wr.grad) < 2e-2
    assert _rel(xg.grad.float().cpu(), xr.grad) < 2e-2


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 17, 13, 3, 3, 26, 20), (3, 8, 8, 1, 2, 14, 14), (1, 5, 7, 4, 0, 6, 8)])
def test_stem_pack_kernel(dtype, shape):
    """dtm_stem_pack (zero border + channel pad to 4 + bf16 in one pass) = torch pad of the bf16 input."""
    from distributed_tensorflow_models_amd.ops import _lib
    N, H, W, C, pad, Hp, Wp = shape
    x = torch.randn(N, H, W, C, device=DEV).to(dtype)
    xp = torch.full((N, Hp, Wp, 4), 7.0, device=DEV, dtype=torch.bfloat16)
    rc = _lib.lib().dtm_stem_pack(_lib.ptr(x), 0 if dtype == torch.float32 else 1, _lib.ptr(xp), N, H, W, C, Hp, Wp,
                                  pad, _lib.stream_ptr())
    assert rc == 0
    ref_p = torch.nn.functional.pad(x.to(torch.bfloat16), (0, 4 - C, pad, Wp - W - pad, pad, Hp - H - pad))
    torch.cuda.synchronize()
    assert torch.equal(xp, ref_p)


def test_device_state_bound_to_first_device():
    """The kernel library's device state (scratch arenas, finalize accumulators, zero chunk) belongs to the
    first device the process uses; from that device the check passes (another device gets -9, which
    nn._check turns into a clear error - not testable on a one-GPU box)."""
    from distributed_tensorflow_models_amd.ops import _lib
    L = _lib.lib()
    x = torch.zeros(8, device="cuda")  # (initialises the device)
    assert L.dtm_device_check() == 0
    assert x.sum().item() == 0


@pytest.mark.parametrize("case", [(16, 14, 256, 256), (8, 7, 512, 2048), (4, 35, 288, 48), (2, 8, 1280, 320),
                                  (64, 56, 64, 64), (3, 17, 768, 192)])
def test_bn_stats_finalize_direct_matches_counter_path_and_fp32(case):
    """The one-block-per-channel-group BN finalize (stats_finalize_direct_kernel, taken when one row chunk covers
    every statistics row) vs the accumulator + completion-counter path it replaces: ss = [scale; shift; mean; rstd]
    and the moving averages bit-identical under deterministic reductions (the persistent conv kernels' partial rows
    are otherwise summed in arrival order: 1e-6 then); both against the fp32 batch statistics of the conv output."""
    import ctypes

    from distributed_tensorflow_models_amd.ops import _lib
    N, H, C, K = case
    torch.manual_seed(1)
    L = _lib.lib()
    st = _lib.stream_ptr()
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    w = (torch.randn(K, 1, 1, C, device=DEV) / C ** 0.5).to(torch.bfloat16)
    beta = torch.randn(K, device=DEV)
    mm0, mv0 = torch.randn(K, device=DEV) * 0.1, torch.rand(K, device=DEV) + 0.5
    M = N * H * H
    d = _lib.ConvDesc(N, H, H, C, K, 1, 1, H, H, 1, 0, 0, 0, 0)
    out = {}
    try:
        for direct, det in ((1, 1), (0, 1), (1, 0)):
            L.dtm_set_fin_direct(direct)
            L.dtm_set_deterministic(det)
            y = torch.empty(N, H, H, K, device=DEV, dtype=torch.bfloat16)
            mm, mv, ss = mm0.clone(), mv0.clone(), torch.zeros(4, K, device=DEV)
            assert L.dtm_conv_fwd_bn(_lib.ptr(x), _lib.ptr(w), _lib.ptr(y), None, None, None, _lib.ptr(beta),
                                     _lib.ptr(mm), _lib.ptr(mv), _lib.ptr(ss), float(M), 1e-3, 0.9, 1, 0,
                                     ctypes.byref(d), st) == 0
            torch.cuda.synchronize()
            out[(direct, det)] = (y, ss, mm, mv)
    finally:
        L.dtm_set_fin_direct(1)
        L.dtm_set_deterministic(0)
    assert torch.equal(out[(0, 1)][0], out[(1, 1)][0])
    for a, b in zip(out[(1, 1)][1:], out[(0, 1)][1:]):
        assert torch.equal(a, b), _rel(a, b)
    for a, b in zip(out[(1, 0)][1:], out[(0, 1)][1:]):
        assert _rel(a, b) < 1e-6, _rel(a, b)
    out[1] = out[(1, 0)]
    yf = (x.float().reshape(M, C) @ w.float().reshape(K, C).t())
    mean, var = yf.mean(0), yf.var(0, unbiased=False)
    ss = out[1][1]
    assert _rel(ss[2], mean) < 2e-2 and _rel(ss[3], torch.rsqrt(var + 1e-3)) < 2e-2
    assert _rel(ss[1], beta - mean * ss[0]) < 2e-2
    assert _rel(out[1][2], mm0 * 0.9 + 0.1 * mean) < 2e-2 and _rel(out[1][3], mv0 * 0.9 + 0.1 * var) < 2e-2


@pytest.mark.parametrize("case", [(128, 35, 288, [64, 48, 64, 32]), (8, 17, 768, [192, 160, 160, 192]),
                                  (4, 8, 1280, [320, 384, 448]), (2, 9, 64, [16, 8])])
@pytest.mark.parametrize("det", [0, 1])
def test_conv_wgrad_multi_matches_separate(case, det):
    """The weight gradient of merged sibling 1x1 convs (dtm_conv_wgrad_multi: ONE wgrad over the members' output
    gradients side by side, its split-K slabs' row ranges reduced into each member's dW in one launch) vs one
    dtm_conv_wgrad per member, and vs fp32 torch; deterministic mode: bit-identical to the per-member runs' sums of
    the same slabs is not promised (other split counts), so both are held to the fp32 reference."""
    import ctypes

    from distributed_tensorflow_models_amd.ops import _lib
    N, H, C, ks = case
    torch.manual_seed(3)
    L = _lib.lib()
    st = _lib.stream_ptr()
    x = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    K = sum(ks)
    dy = torch.randn(N, H, H, K, device=DEV).to(torch.bfloat16)
    L.dtm_set_deterministic(det)
    try:
        dws = [torch.zeros(k, 1, 1, C, device=DEV) for k in ks]
        d = _lib.ConvDesc(N, H, H, C, K, 1, 1, H, H, 1, 0, 0, 0, 0)
        ptrs = (ctypes.c_void_p * len(ks))(*[t.data_ptr() for t in dws])
        rows = (ctypes.c_int * len(ks))(*ks)
        assert L.dtm_conv_wgrad_multi(_lib.ptr(x), _lib.ptr(dy), ptrs, rows, len(ks), ctypes.byref(d),
                                      _lib.num_cus(), st) == 0
        torch.cuda.synchronize()
    finally:
        L.dtm_set_deterministic(0)
    ref = (dy.float().reshape(-1, K).t() @ x.float().reshape(-1, C))
    off = 0
    for k, got in zip(ks, dws):
        assert _rel(got.reshape(k, C), ref[off:off + k]) < 1e-4, (k, _rel(got.reshape(k, C), ref[off:off + k]))
        off += k


@pytest.mark.parametrize("tile", [1, 7, 8, 14, 15, 16])
@pytest.mark.parametrize("N", [2, 5])
def test_stem_wgrad_bn_fused_tiles_match_unfused(tile, N):
    """The stem's weight gradient with its BN backward fused into the A-operand staging (dtm_conv_wgrad_bnbwd) on
    every tile that can take it - register-staged 64 x 128 (1) / 64 x 256 (7, 8) and the pipelined 64 x 256 with the
    in-LDS transform (14, 15, 16) - against the unfused form (stats_combine_fin -> comb, then a plain wgrad), and
    dgamma / dbeta against the combine's: packed-row 7x7/2 view at 224 x 224."""
    import ctypes

    from distributed_tensorflow_models_amd.ops import _lib
    torch.manual_seed(21)
    L = _lib.lib()
    st = _lib.stream_ptr()
    Hp = Wp = 230
    P = Q = 112
    xp = torch.randn(N, Hp, Wp, 4, device=DEV).to(torch.bfloat16)
    d = _lib.ConvDesc(N, Hp, Wp, 32, 64, 7, 1, P, Q, 2, 0, 0, 8)
    g = torch.randn(N, P, Q, 64, device=DEV).to(torch.bfloat16)
    y = torch.randn(N, P, Q, 64, device=DEV).to(torch.bfloat16)
    count = float(N * P * Q)
    dss = torch.randn(4, 64, device=DEV) * 1e-2 * count
    ss = torch.cat([torch.rand(1, 64, device=DEV) + 0.5, torch.randn(1, 64, device=DEV),
                    torch.randn(1, 64, device=DEV) * 0.1, torch.rand(1, 64, device=DEV) + 0.5]).contiguous()
    gamma = torch.rand(64, device=DEV) + 0.5
    comb = torch.empty_like(g)
    dg0, db0 = torch.zeros(64, device=DEV), torch.zeros(64, device=DEV)
    assert L.dtm_stats_combine_fin(_lib.ptr(g), _lib.ptr(y), _lib.ptr(dss), _lib.ptr(ss), _lib.ptr(gamma), count,
                                   _lib.ptr(dg0), _lib.ptr(db0), _lib.ptr(comb), N * P * Q, 64, 1, st) == 0
    dw0 = torch.zeros(64, 7, 8, 4, device=DEV)
    L.dtm_conv_set_wgrad_tile(1, 0)
    try:
        assert L.dtm_conv_wgrad(_lib.ptr(xp), _lib.ptr(comb), _lib.ptr(dw0), None, None, ctypes.byref(d),
                                _lib.num_cus(), st) == 0
        dw = torch.zeros(64, 7, 8, 4, device=DEV)
        dg, db = torch.zeros(64, device=DEV), torch.zeros(64, device=DEV)
        L.dtm_conv_set_wgrad_tile(tile, 0)
        assert L.dtm_conv_wgrad_bnbwd(_lib.ptr(xp), _lib.ptr(g), _lib.ptr(y), _lib.ptr(dss), _lib.ptr(ss),
                                      _lib.ptr(gamma), count, _lib.ptr(dg), _lib.ptr(db), _lib.ptr(dw),
                                      ctypes.byref(d), _lib.num_cus(), st) == 0
        torch.cuda.synchronize()
    finally:
        L.dtm_conv_set_wgrad_tile(-1, 4)
    assert _rel(dw, dw0) < 2e-3, _rel(dw, dw0)
    assert _rel(dg, dg0) < 1e-5 and _rel(db, db0) < 1e-5
