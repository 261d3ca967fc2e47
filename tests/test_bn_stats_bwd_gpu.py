"""HIP backward of the per-channel [sum y; sum y^2] statistics (ops/fused.py _BNStatsFn, the
Inception pool branches' BatchNorm over the pooled tensor) vs the fp32 PyTorch reference."""
import pytest
import torch

from distributed_tensorflow_models_amd.ops import _lib
from distributed_tensorflow_models_amd.ops import fused

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(4, 35, 35, 64), (3, 17, 17, 192), (2, 8, 8, 8), (5, 7, 3, 40)])
def test_bn_stats_bwd_matches_fp32(shape):
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    y = torch.randn(shape, device=dev).to(torch.bfloat16)
    C = shape[-1]
    dstats = torch.randn(2, C, device=dev)
    dy = torch.empty_like(y)
    rc = _lib.lib().dtm_bn_stats_bwd(_lib.ptr(y), _lib.ptr(dstats), None, _lib.ptr(dy), y.numel() // C, C,
                                     _lib.stream_ptr())
    assert rc == 0
    ref = dstats[0] + 2.0 * y.float() * dstats[1]
    err = (dy.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2
    # with the tensor's other gradient added, written in place into it
    g = torch.randn(shape, device=dev).to(torch.bfloat16)
    ref2 = ref + g.float()
    rc = _lib.lib().dtm_bn_stats_bwd(_lib.ptr(y), _lib.ptr(dstats), _lib.ptr(g), _lib.ptr(g), y.numel() // C, C,
                                     _lib.stream_ptr())
    assert rc == 0
    assert (g.float() - ref2).abs().max() / ref2.abs().max() < 1e-2


def test_bn_stats_fn_gradient_through_autograd():
    torch.manual_seed(1)
    dev = torch.device("cuda", 0)
    y = torch.randn(2, 9, 9, 32, device=dev).to(torch.bfloat16).requires_grad_(True)
    stats, alias = fused._BNStatsFn.apply(y)
    ref_stats = torch.stack([y.float().sum((0, 1, 2)), (y.float() ** 2).sum((0, 1, 2))])
    assert (stats - ref_stats).abs().max() / ref_stats.abs().max() < 1e-2
    w = torch.randn(2, 32, device=dev)
    v = torch.randn(y.shape, device=dev)
    ((stats * w).sum() + (alias.float() * v).sum()).backward()
    ref = w[0] + 2.0 * y.detach().float() * w[1] + v
    assert (y.grad.float() - ref).abs().max() / ref.abs().max() < 1e-2
