"""ctypes binding of the gfx950 kernel library ``_native/libdtm_kernels.so``.

Every entry point launches on the caller's current HIP stream (``torch.cuda.current_stream()``)
so whole training steps can be captured into a hipGraph.  On a GPU machine a missing library is a
hard error (no silent eager fallback); on a CPU-only machine the pure-PyTorch reference path in
``ops.reference`` is used instead.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("DTM_KERNELS_SO") or os.path.join(_HERE, "_native", "libdtm_kernels.so")  # A/B override

_lib = None


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("N", "H", "W", "C", "K", "R", "S", "P", "Q", "stride", "pad_h", "pad_w", "pix_bytes", "dec")]


class PoolArgs(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("N", "H", "W", "C", "P", "Q", "KH", "KW", "SH", "SW", "PH", "PW")]


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float

_SIGS = {
    "dtm_conv_fwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, ctypes.POINTER(ConvDesc), _P]),
    "dtm_act_fwd": (_I, [_P, _P, _L, _I, _F, _I, _P]),
    "dtm_prep_params_bytes": (_I, []),
    "dtm_jpeg_desc_bytes": (_I, []),
    "dtm_jpeg_decode_gpu": (_I, [_P, _P, _I, _I, _L, _P, _P, _P]),
    "dtm_jpeg_huff_desc_bytes": (_I, []),
    "dtm_jpeg_huff_gpu": (_I, [_P, _P, _P, _I, _P, _P, _P]),
    "dtm_jpeg_set_huff": (None, [_I, _I]),
    "dtm_imagenet_prep": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _P]),
    "dtm_act_bwd": (_I, [_P, _P, _P, _L, _I, _F, _I, _P]),
    "dtm_instnorm_fwd": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _F, _I, _I, _P]),
    "dtm_instnorm_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "dtm_reflect_pad": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "dtm_reflect_pad_bwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "dtm_conv_dgrad": (_I, [_P, _P, _P, ctypes.POINTER(ConvDesc), _P]),
    "dtm_conv_dgrad_ex": (_I, [_P, _P, _P, ctypes.POINTER(ConvDesc), _P, _I, _P, _P, _P, _I, _P]),
    "dtm_conv_dgrad_bnout": (_I, [_P, _P, _P, ctypes.POINTER(ConvDesc), _P, _I, _P, _P, _P, _P, _P]),
    "dtm_conv1x1_bnbwd": (_I, [_P, _P, _P, _P, _P, _F, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _L, _I, _I, _P]),
    "dtm_conv_wgrad_bnbwd": (_I, [_P, _P, _P, _P, _P, _P, _F, _P, _P, _P, ctypes.POINTER(ConvDesc), _I, _P]),
    "dtm_conv_wgrad": (_I, [_P, _P, _P, _P, _P, ctypes.POINTER(ConvDesc), _I, _P]),
    "dtm_conv_wgrad_multi": (_I, [_P, _P, _P, _P, _I, ctypes.POINTER(ConvDesc), _I, _P]),
    "dtm_conv_set_policy2": (None, [_I]),
    "dtm_set_grid_cpt": (None, [_I]),
    "dtm_conv_set_k32": (None, [_I]),
    "dtm_conv_set_stem_stream": (None, [_I]),
    "dtm_ws_set_side_stream": (None, [_I, _P]),
    "dtm_device_check": (_I, []),
    "dtm_conv_set_direct3": (None, [_I]),
    "dtm_conv_set_dec_group": (None, [_I]),
    "dtm_cat_desc_bytes": (_I, []),
    "dtm_cat_bn_apply": (_I, [_P, _I, _P, _L, _I, _P]),
    "dtm_cat_bn_apply_bwd": (_I, [_P, _I, _P, _P, _L, _I, _P]),
    "dtm_weight_flip_transpose": (None, [_P, _P, _I, _I, _I, _I, _P]),
    "dtm_weight_flip_transpose_batched": (None, [_P, _I, _P]),
    "dtm_weight_flip_transpose_dec": (None, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "dtm_flip_desc_bytes": (_I, []),
    "dtm_bn_stats": (None, [_P, _P, _L, _I, _P]),
    "dtm_col_sums": (_I, [_P, _P, _L, _I, _P]),
    "dtm_bn_stats_bwd": (_I, [_P, _P, _P, _P, _L, _I, _P]),
    "dtm_bn_finalize": (None, [_P, _P, _P, _P, _P, _P, _I, _F, _F, _F, _I, _I, _P]),
    "dtm_bn_inference_params": (None, [_P, _P, _P, _P, _P, _I, _F, _P]),
    "dtm_bn_apply": (None, [_P, _P, _P, _P, _P, _L, _I, _I, _I, _P]),
    "dtm_bn_apply2": (_I, [_P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _P]),
    "dtm_maxpool_bnrelu_fwd": (_I, [_P, _P, _P, _P, ctypes.POINTER(PoolArgs), _P]),
    "dtm_maxpool_bnrelu_bwd": (_I, [_P, _P, _P, _P, _P, _P, ctypes.POINTER(PoolArgs), _I, _P]),
    "dtm_conv_set_tile": (None, [_I]),
    "dtm_conv_set_wgrad_tile": (None, [_I, _I]),
    "dtm_loss_combine": (_I, [_P, _I, _I, _P, _P, _P]),
    "dtm_scale_rows_pad": (_I, [_P, _I, _P, _I, _P, _I, _I, _I, _P]),
    "dtm_conv_set_wgrad_k64": (None, [_I]),
    "dtm_pool_set_k3s2": (None, [_I]),
    "dtm_conv_fwd_bn": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _I, _I, ctypes.POINTER(ConvDesc), _P]),
    "dtm_stats_combine_fin": (_I, [_P, _P, _P, _P, _P, _F, _P, _P, _P, _L, _I, _I, _P]),
    "dtm_stats_combine_fin_ld": (_I, [_P, _P, _P, _P, _P, _F, _P, _P, _P, _L, _I, _I, _I, _P]),
    "dtm_bn_apply_res_strided": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P]),
    "dtm_bn_bwd_reduce": (None, [_P, _P, _P, _P, _P, _L, _I, _I, _P]),
    "dtm_bn_bwd_apply": (None, [_P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _P]),
    "dtm_bn_param_grad": (None, [_P, _P, _P, _I, _P]),
    "dtm_maxpool_fwd": (None, [_P, _P, _P, ctypes.POINTER(PoolArgs), _P]),
    "dtm_maxpool_bwd": (None, [_P, _P, _P, ctypes.POINTER(PoolArgs), _P]),
    "dtm_maxpool_bwd_ld": (_I, [_P, _I, _P, _P, ctypes.POINTER(PoolArgs), _P]),
    "dtm_avgpool_fwd": (None, [_P, _P, ctypes.POINTER(PoolArgs), _I, _P]),
    "dtm_avgpool_bwd": (None, [_P, _P, ctypes.POINTER(PoolArgs), _I, _P]),
    "dtm_avgpool_bwd_acc": (_I, [_P, _P, ctypes.POINTER(PoolArgs), _I, _P]),
    "dtm_global_avg_fwd": (None, [_P, _P, _I, _I, _I, _P]),
    "dtm_global_avg_bwd": (None, [_P, _P, _I, _I, _I, _P]),
    "dtm_global_avg_fwd_bf16": (None, [_P, _P, _I, _I, _I, _P]),
    "dtm_global_avg_bwd_bf16": (None, [_P, _P, _I, _I, _I, _P]),
    "dtm_softmax_xent": (None, [_P, _I, _P, _P, _P, _I, _I, _F, _F, _P, _I, _P]),
    "dtm_opt_chunk_size": (_I, []),
    "dtm_opt_tensor_bytes": (_I, []),
    "dtm_opt_chunk_bytes": (_I, []),
    "dtm_multi_tensor_opt": (None, [_P, _P, _I, _I, _F, _F, _F, _F, _F, _F, _I, _P, _P, _P]),
    "dtm_check_finite": (None, [_P, _L, _P, _P]),
    "dtm_f32_to_bf16": (None, [_P, _P, _L, _P]),
    "dtm_scale": (None, [_P, _L, _F, _P]),
    "dtm_bn_apply_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _I, _P]),
    "dtm_stats_combine": (_I, [_P, _P, _P, _P, _L, _I, _P]),
    "dtm_bn_finalize_bwd": (None, [_P, _P, _P, _P, _P, _P, _I, _F, _P]),
    "dtm_lrn": (_I, [_P, _P, _P, _L, _I, _I, _F, _F, _F, _I, _P]),
    "dtm_ws_reserve": (_I, [_L]),
    "dtm_ws_last_error": (_I, []),
    "dtm_ws_retired": (_L, []),
    "dtm_ws_reserve_stream": (_I, [_L, _P]),
    "dtm_ws_capacity": (_L, [_P]),
    "dtm_depthwise_fwd": (_I, [_P, _P, _P, _P, _P]),
    "dtm_depthwise_dgrad": (_I, [_P, _P, _P, _P, _P]),
    "dtm_depthwise_wgrad": (_I, [_P, _P, _P, _P, _P]),
    "dtm_set_reduce_policy": (None, [_I, _I, _I]),
    "dtm_bn_apply_ld": (_I, [_P, _P, _P, _P, _L, _I, _I, _I, _P]),
    "dtm_bn_apply_bwd_ld": (_I, [_P, _P, _P, _P, _P, _P, _L, _I, _I, _I, _P]),
    "dtm_set_sc_policy": (None, [_I, _I]),
    "dtm_set_ntld_policy": (None, [_I]),
    "dtm_set_deterministic": (None, [_I]),
    "dtm_get_deterministic": (_I, []),
    "dtm_conv_set_k64_tile": (None, [_I]),
    "dtm_conv_set_w8": (None, [_I]),
    "dtm_conv_set_kwide": (None, [_I]),
    "dtm_set_reduce_few": (None, [_I]),
    "dtm_set_reserved_cus": (None, [_I]),
    "dtm_stats_combine_multi": (_I, [_P, _P, _I, _F, _P, _L, _I, _P]),
    "dtm_conv_fwd_bn_multi": (_I, [_P, _P, _P, _P, _I, _P, _F, _F, _F, _I, _I, ctypes.POINTER(ConvDesc), _P]),
    "dtm_conv_set_dec_lpt": (None, [_I]),
    "dtm_conv_set_dec_tile": (None, [_I]),
    "dtm_conv_set_split_tile": (None, [_I]),
    "dtm_get_reserved_cus": (_I, []),
    "dtm_compute_cus_api": (_I, []),
    "dtm_cu_hog": (_I, [_I, _F, _P]),
    "dtm_conv_set_stream_act": (None, [_I]),
    "dtm_conv_set_act_tile": (None, [_I]),
    "dtm_stem_pack": (_I, [_P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "dtm_dropout": (_I, [_P, _P, _L, _I, _F, ctypes.c_ulonglong, _P, _P]),
    "dtm_in_top_k": (_I, [_P, _P, _P, _I, _I, _I, _I, _P]),
}


def gpu_present():
    try:
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False


def lib():
    """Load (once) and return the kernel library; raise loudly if it is missing on a GPU box."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "native kernel library %s is missing: run `python tools/build_native.py` "
                "(or __graft_entry__.build())" % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        ab = bool(os.environ.get("DTM_KERNELS_SO"))
        for name, (res, args) in _SIGS.items():
            if ab and not hasattr(L, name):  # an A/B baseline build older than this binding: its missing entry
                continue                     # points stay unbound (only the default library is checked in full)
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        if os.environ.get("DTM_DETERMINISTIC", "0") not in ("", "0"):
            L.dtm_set_deterministic(1)
    return _lib


def set_deterministic(on=True):
    """Bit-reproducible GPU reductions (BN statistics, BN-gradient sums, split-K wgrad): every
    output column summed by one block in a fixed order instead of fp32 atomics across blocks.
    Also enabled by DTM_DETERMINISTIC=1.  Costs a little latency on tall partial-sum slabs."""
    lib().dtm_set_deterministic(int(bool(on)))


def available():
    return os.path.exists(LIB_PATH) and gpu_present()


def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


# ---- weight-gradient side stream ----------------------------------------------------------------------
# The conv+BN backward enqueues its weight gradient on a second HIP stream (after waiting for the main
# stream's gradient), so it runs concurrently with the dgrad chain on the main stream and fills the CUs
# the latter's tails and small launches leave idle.  The C++ side gives that stream its own scratch
# arena (dtm_ws_set_side_stream).  The data-parallel layer launches bucket all-reduces from the side
# stream after it has waited for the main one (parallel/bsp.py), and the engine joins the side stream
# before the optimizer (side_join).  Feature wgrad_stream (ops/features.py; default on) or set_side_enabled().  Measured
# (profiles/ab/r3_ab_wgrad_side_stream.log): ResNet-50 b256 step 18.02 -> 17.26 ms (-4.3 %).
_side = {"stream": None, "on": None, "used": False}


def set_side_enabled(on):
    _side["on"] = bool(on)


def side_enabled():
    if _side["on"] is None:
        from . import features
        _side["on"] = features.on("wgrad_stream")
    return _side["on"]


def side_stream():
    """The weight-gradient side stream, or None when off / not on a GPU."""
    if not side_enabled() or not torch.cuda.is_available():
        return None
    if torch.cuda.is_current_stream_capturing():
        # captured steps are single-stream: with the side stream inside the capture Inception-v3 ran 6.3 % slower
        # (profiles/ab/r4_ab_graph_side_inception.log; that capture mode was removed in round 5)
        return None
    dev = torch.cuda.current_device()
    st = _side["stream"]
    if st is None or st.device.index != dev:
        st = torch.cuda.Stream(device=dev)
        _side["stream"] = st
        lib().dtm_ws_set_side_stream(1, ctypes.c_void_p(st.cuda_stream))  # scratch slot 1
    return st


SIDE_CU_FRAC = 0.75
_side_cu = {"frac": None}


def set_side_cu_fraction(frac):
    _side_cu["frac"] = float(frac)


def side_cus():
    """CU count the split-K policy of a side-stream weight gradient sizes its grid for (SIDE_CU_FRAC x the
    device's CUs; set_side_cu_fraction for A/B runs): the side stream shares the chip with the dgrad chain, so fewer splits mean fewer fp32
    partial slabs to write and reduce and fewer workgroups taken from the main stream.  Measured on ResNet-50
    (profiles/ab/r3_ab_side_cus.log, r3_ab_dgrp_bnst.log): 0.75 -1.0..-1.5 % step vs 1.0; 0.5 neutral; 0.35 +4 %."""
    if _side_cu["frac"] is None:
        _side_cu["frac"] = SIDE_CU_FRAC
    return max(8, int(num_cus() * _side_cu["frac"]))


_wgrad_cu = {"main": None, "stem": None}


def set_wgrad_cu_percent(kind, pct):
    _wgrad_cu[kind] = float(pct)


def wgrad_cus(kind="main"):
    """CU count the split-K policy of a main-stream weight gradient sizes its grid for: ``kind`` 'main' (every
    conv wgrad not on the side stream) or 'stem' (the packed-row stem's BN-fused wgrad, the last kernel of the
    backward): 100 % of the CUs unless set_wgrad_cu_percent (A/B runs: profiles/ab/r3_ab_wgrad_cus_*.log,
    r3_ab_stem_wgrad_cus.log)."""
    if _wgrad_cu[kind] is None:
        _wgrad_cu[kind] = 100.0
    return max(8, int(num_cus() * _wgrad_cu[kind] / 100.0))


def side_fork(*tensors):
    """Make the side stream wait for the main stream's work so far and mark ``tensors`` as used by it (the
    caching allocator keeps them until the side stream is done).  Returns the stream or None."""
    st = side_stream()
    if st is None:
        return None
    st.wait_stream(torch.cuda.current_stream())
    for t in tensors:
        if t is not None:
            t.record_stream(st)
    _side["used"] = True
    return st


def side_active():
    """The side stream if work was enqueued on it since the last join."""
    return _side["stream"] if _side["used"] else None


def side_join():
    """The current stream waits for everything enqueued on the side stream."""
    if _side["used"]:
        torch.cuda.current_stream().wait_stream(_side["stream"])
        _side["used"] = False


def ptr(t):
    """Raw device pointer of a tensor (or None)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


_num_cus = None
_reserved = [0]


def set_reserved_cus(n):
    """Take ``n`` CUs out of the count that the persistent conv kernels and the split-K weight-gradient policies
    size their grids for (the RCCL channels' workgroups share the chip with the overlapped backward under data
    parallelism: a grid sized for every CU would run a short second round behind them).  0 = all CUs."""
    _reserved[0] = max(0, int(n))
    lib().dtm_set_reserved_cus(_reserved[0])


def reserved_cus():
    return _reserved[0]


def num_cus():
    """CUs available to compute grids: the device's CUs minus the reserved ones (set_reserved_cus)."""
    global _num_cus
    if _num_cus is None:
        _num_cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    return max(8, _num_cus - _reserved[0])
