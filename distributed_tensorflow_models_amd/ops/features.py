"""The switchable fused paths of the HIP training step, in one registry (profiles/ab/README.md lists every knob,
its default, its A/B evidence and its data-parallel test coverage).

Every feature is ON by default - each was kept because a same-process whole-step A/B measured it faster (the logs
named below).  A feature is turned off for an A/B run or a numerics comparison with the ONE environment variable
``DTM_DISABLE=<name>[,<name>...]`` (read at each use, so a process can flip it between steps) or, in-process, with
``features.override(name=False)``.  Off means the generic (unfused) kernels of the same op run instead; nothing
about the math changes.  ``ROUTES_GRADIENTS`` marks the features that change how a gradient reaches its
parameter's main_grad (and so the BSP bucket bookkeeping): each has a row in the data-parallel gradient matrix
(tests/test_distributed.py _DP_MATRIX, run log profiles/r5/r5_dp_matrix.log)."""
import contextlib
import os

# name -> (what it fuses, A/B evidence)
FEATURES = {
    "fused_bn": ("conv -> BatchNorm as one lazily applied pair: statistics in the conv epilogue, the BN-apply + ReLU "
                 "folded into the consumer (models/layers.py)", "profiles/r1_resnet50_b256_fused_v1_summary.txt (vs r1_torch_eager_baseline_probe.log)"),
    "sibling_group": ("one backward for the sibling 1x1 conv+BNs reading one input (Inception branch heads, a ResNet "
                      "projection unit's shortcut + conv1)", "profiles/ab/r3_ab_sibling_resnet.log, r4_ab_sibling_inception.log"),
    "sibling_fwd": ("Inception mixed blocks: the branch-head 1x1 conv+BNs as ONE conv over their concatenated weights "
                    "+ one grouped BN finalize", "profiles/ab/r4_ab_sibfwd_inception.log"),
    "sibling_combine": ("the sibling members' BN stats-combines as one grouped launch",
                        "profiles/ab/r4_ab_knobs_inception.log"),
    "act_handoff": ("conv consumers of one activation hand the masked input gradient on (the last one's act epilogue "
                    "adds it)", "profiles/ab/r4_ab_sibling_inception.log"),
    "bnout_fuse": ("the block-output BN-apply backward inside the consuming conv's dgrad epilogue",
                   "profiles/ab/r2_ab_bnout.log, r3_ab_dgrp_bnst.log"),
    "bwd1x1_fuse": ("one-pass backward of ResNet's 64->256 expansion 1x1 conv+BN", "profiles/ab/r2_ab_bwd1x1.log"),
    "stem_wgrad_fuse": ("the stem's BN backward inside its wgrad operand staging", "profiles/ab/r2_ab_stem_wgrad_bn.log"),
    "cat_multi": ("an Inception block's concat BN-apply as one multi-part launch", "profiles/ab/r2_ab_cat_multi_inception.log"),
    "pool_commute": ("Inception pool branches as conv -> pool -> BN (the pool over the conv's output channels)",
                     "profiles/ab/r2_ab_pool_commute_inception.log"),
    "wgrad_stream": ("conv+BN weight gradients on a second HIP stream, concurrent with the dgrad chain "
                     "(TrainStep(wgrad_stream=...) overrides per model)", "profiles/ab/r3_ab_wgrad_side_stream.log"),
    "pool_tail": ("Inception's aux-head pool gradient added in place into the Mixed_6e-output gradient the main path "
                  "returned (no separate add over the 17x17x768 map)", "profiles/ab/r5_ab_pool_tail.log"),
    "bsp_compact": ("dead-tap conv weights get a compact all-reduce bucket holding their live window only",
                    "tests/test_distributed.py test_bsp_dead_tap_gradients_left_out_of_the_allreduce"),
}

ROUTES_GRADIENTS = ("fused_bn", "sibling_group", "sibling_fwd", "sibling_combine", "act_handoff", "bnout_fuse",
                    "bwd1x1_fuse", "stem_wgrad_fuse", "cat_multi", "pool_commute", "wgrad_stream", "bsp_compact")

_override = {}


def _disabled_env():
    v = os.environ.get("DTM_DISABLE", "")
    return {n.strip() for n in v.split(",") if n.strip()}


def on(name):
    """Whether fused path ``name`` is enabled (override > DTM_DISABLE > default on)."""
    if name not in FEATURES:
        raise KeyError("unknown feature %r (ops/features.py)" % name)
    if name in _override:
        return _override[name]
    return name not in _disabled_env()


def check_env():
    """Unknown names in DTM_DISABLE are an error (a typo would silently measure the default)."""
    bad = sorted(_disabled_env() - set(FEATURES))
    if bad:
        raise ValueError("DTM_DISABLE names unknown features %s (known: %s)" % (bad, ", ".join(sorted(FEATURES))))


@contextlib.contextmanager
def override(**kw):
    """features.override(sibling_fwd=False): in-process switch for tests / A/B tools."""
    for k in kw:
        if k not in FEATURES:
            raise KeyError("unknown feature %r" % k)
    saved = {k: _override.get(k) for k in kw}
    _override.update({k: bool(v) for k, v in kw.items()})
    try:
        yield
    finally:
        for k, v in saved.items():
            if v is None:
                _override.pop(k, None)
            else:
                _override[k] = v


def disable_env(names):
    """The environment entry that turns ``names`` off (for child processes / DP test workers)."""
    return {"DTM_DISABLE": ",".join(names)}
