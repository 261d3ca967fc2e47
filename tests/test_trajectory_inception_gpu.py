"""Inception-v3 (old slim, config #4) as the reference trains it - label smoothing 0.1, 0.4 x aux xent, L2 4e-5,
RMSProp(0.9, 0.9, eps 1.0), BatchNorm decay 0.9997 (/root/reference/inception/imagenet_inception_bsp.py:109-152,
/root/reference/inception/slim/inception_model.py:54-332) - through the default HIP training path (merged sibling
head forward and backward, act-input hand-off, zero-copy concat, pool commute, aux-head full-window dgrad on the
MFMA tiles, grouped stats-combines) against CPU fp32 (ops/reference.py) on the same weights and batches
(tests/fixtures/inception_v3_299_b16_*, written by tools/make_inception_trajectory_fixture.py: 299x299, batch 16,
5 steps, dropout off).

The random-init network's gradient is chaotic: a 1e-6 relative input perturbation moves the fp32 gradients by a
median 4 % (~4e4 x eps), at batch 4, 16 or 48 alike (profiles/r5/r5_grad_sensitivity_inception_b16.log; ResNet-50
too, r5_grad_sensitivity_resnet50_b16.log).  bf16 storage alone therefore leaves the deep layers' step-1 updates
uncorrelated with fp32 (the fixture's emulation error per tensor: median 1.3), which makes a per-tensor comparison
of two independent whole backward passes blind below the top layers.  Hence three tests:

1. test_inception_v3_trajectory_matches_cpu_fp32 (the round-4 verdict's criteria): the 5-step loss curve within
   the emulation's noise; per-tensor step-1 updates within 1.5x the emulation's own error (+2 %: meaningful for the
   logits / aux head / last blocks only, see above); no systematic update scaling (median norm ratio within 3 %,
   the one per-tensor statistic that survives the chaos: emulation p10-p90 0.94-1.08); default path and
   DTM_SIBLING_FWD=0; the merged path no farther from fp32 than the per-head path.
2. test_inception_v3_merged_forward_within_reduction_noise: merged vs per-head whole-model gradients bounded by
   the per-head path's own reduction-order noise floor (deterministic vs atomic order) at the same batch.
3. test_inception_v3_step_teacher_forced_per_segment: the discriminating whole-step check - one real GPU
   training step, every segment (stem, 11 mixed blocks, aux head, logits head) recomputed on the CPU from the
   GPU's own segment inputs and output gradients; every parameter gradient and every block's input gradient within
   2x the bf16-emulation floor (+3 %) of that recomputation, and the median / p90 over tensors within 1.1x / 1.2x of
   the emulation's (measured: 0.0805 vs 0.0803, profiles/r5/r5_s3_pytest_fixed.log)."""
import json
import os
import sys

import numpy as np
import pytest
import torch
from distributed_tensorflow_models_amd.ops import features

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEV = torch.device("cuda", 0)


def _fixture():
    sys.path.insert(0, ROOT)
    from tools import make_inception_trajectory_fixture as T
    return T


def _trajectory(monkeypatch, sib_fwd):
    T = _fixture()
    monkeypatch.setitem(features._override, "sibling_fwd", (sib_fwd) != "0")
    net = T.build().to(DEV)
    tr = T.tracked(net)
    w0 = {k: v.detach().clone() for k, (v, _i) in tr.items()}
    step = T.make_step(net)
    losses, d1 = [], {}
    for i, (x, y) in enumerate(T.batches()):
        losses.append(float(step(x.to(DEV).to(torch.bfloat16), y.to(DEV))))
        if i == 0:
            d1 = {k: T.step1_update(v.detach(), w0[k], idx) for k, (v, idx) in tr.items()}
    step.dp.close()
    return losses, d1


def _errors(d1, fx):
    """per tensor: (GPU rel err, emulation rel err, GPU/fp32 full-norm ratio) of the step-1 update."""
    out = {}
    for k, (g, gn) in d1.items():
        f32 = torch.from_numpy(fx["fp32:" + k])
        em = torch.from_numpy(fx["emul:" + k])
        n = f32.norm().item()
        if n == 0:
            continue
        out[k] = ((g - f32).norm().item() / n, (em - f32).norm().item() / n,
                  gn / float(fx["fp32_norm:" + k][0]))
    return out


def test_inception_v3_trajectory_matches_cpu_fp32(monkeypatch):
    T = _fixture()
    ref = json.load(open(T.FIXTURE + "_trajectory.json"))
    fx = np.load(T.FIXTURE + "_deltas.npz")
    fp32, emul = ref["losses"], ref["losses_bf16_storage"]

    def mrel(a, b):
        return sum(abs(u - v) / v for u, v in zip(a, b)) / len(a)
    res = {}
    for path, sib in (("merged", "1"), ("per-head", "0")):
        got, d1 = _trajectory(monkeypatch, sib)
        errs = _errors(d1, fx)
        d_gpu, d_emul = mrel(got, fp32), mrel(emul, fp32)
        ratios = sorted(r for _e, _em, r in errs.values())
        med = ratios[len(ratios) // 2]
        # per tensor where bf16-scale noise still determines the update (emulation error < 0.1: the logits and the
        # top blocks); the chaos-dominated rest (emulation error 0.1 .. 1.5) as a distribution
        sharp = {k: v for k, v in errs.items() if v[1] < 0.1}
        chaotic = {k: v for k, v in errs.items() if v[1] >= 0.1}
        print("%s: losses %s (fp32 %s); loss dev %.4g (emulation %.4g); update norm ratio median %.4f; %d sharp "
              "tensors: GPU rel err median %.3g max %.3g (emulation %.3g / %.3g); %d chaotic tensors: GPU median %.3g "
              "p90 %.3g (emulation %.3g / %.3g)" % (
                  path, ["%.4f" % v for v in got], ["%.4f" % v for v in fp32], d_gpu, d_emul, med, len(sharp),
                  _pct([v[0] for v in sharp.values()])[0], _pct([v[0] for v in sharp.values()])[2],
                  _pct([v[1] for v in sharp.values()])[0], _pct([v[1] for v in sharp.values()])[2], len(chaotic),
                  *_pct([v[0] for v in chaotic.values()])[:2], *_pct([v[1] for v in chaotic.values()])[:2]))
        msg = "%s\ngpu  %s\nfp32 %s\nemul %s" % ((path,) + tuple(["%.4f" % v for v in t] for t in (got, fp32, emul)))
        assert len(errs) > 180, len(errs)  # every trainable tensor of the 388-variable layout
        assert len(sharp) >= 4, sorted(sharp)
        bad = ["%s: step-1 rel err %.4f (emulation %.4f)" % (k, e, em) for k, (e, em, _r) in sharp.items()
               if e > 1.5 * em + 0.02]
        assert not bad, path + "\n" + "\n".join(bad[:20])
        gc, ec = _pct([v[0] for v in chaotic.values()]), _pct([v[1] for v in chaotic.values()])
        assert gc[0] < 1.25 * ec[0] + 0.02 and gc[1] < 1.25 * ec[1] + 0.02, (path, gc, ec)
        assert abs(med - 1.0) < 0.03, (path, med)  # no systematic scaling of the update
        assert abs(got[0] - fp32[0]) / fp32[0] < 2e-2, msg  # same weights and batch at step 0
        assert d_gpu < 1.5 * d_emul + 5e-3, (d_gpu, d_emul, msg)
        res[path] = errs
    # the merged head forward is no farther from fp32 than the per-head path
    m = _pct([v[0] for v in res["merged"].values()])
    p = _pct([v[0] for v in res["per-head"].values()])
    assert m[0] <= 1.25 * p[0] + 2e-3 and m[1] <= 1.25 * p[1] + 5e-3, (m, p)


def _pct(v):
    v = sorted(v)
    return v[len(v) // 2], v[int(0.9 * (len(v) - 1))], v[-1]


def _grads(monkeypatch, net, step, x, y, sib_fwd, det, init):
    from distributed_tensorflow_models_amd.engine import moving_average_buffers
    from distributed_tensorflow_models_amd.ops import _lib
    monkeypatch.setitem(features._override, "sibling_fwd", (sib_fwd) != "0")
    _lib.lib().dtm_set_deterministic(int(det))
    try:
        with torch.no_grad():
            for b, v in zip(moving_average_buffers(net), init):
                b.copy_(v)
        loss, _skip = step._forward_backward(x, y)
        torch.cuda.synchronize()
        return float(loss), {k: p.main_grad.detach().float().clone() for k, p in net.named_parameters()
                             if getattr(p, "main_grad", None) is not None}
    finally:
        _lib.lib().dtm_set_deterministic(0)


def test_inception_v3_merged_forward_within_reduction_noise(monkeypatch):
    """The merged sibling head forward sums each member's BatchNorm statistics over other partial rows than the
    per-head convs do, so it differs from the per-head path in the last bits of the statistics - the same kind of
    difference the per-head path has with itself between deterministic (one block per column, fixed order) and
    default (cross-block fp32 atomics, arrival order) reductions.  Through the whole network, at the trajectory
    fixture's batch (16 x 299 x 299), the merged-vs-per-head gradient difference must stay within that noise floor
    (measured here, not assumed); a wrong merged forward or backward shows as an O(1) difference."""
    T = _fixture()
    from distributed_tensorflow_models_amd.engine import moving_average_buffers
    net = T.build().to(DEV)
    step = T.make_step(net)
    x, y = T.batches()[0]
    x, y = x.to(DEV).to(torch.bfloat16), y.to(DEV)
    init = [b.detach().clone() for b in moving_average_buffers(net)]
    ref_l, ref = _grads(monkeypatch, net, step, x, y, "0", True, init)
    rep_l, rep = _grads(monkeypatch, net, step, x, y, "0", True, init)
    assert rep_l == ref_l and all(torch.equal(rep[k], ref[k]) for k in ref)  # deterministic means bit-identical
    floors = [_grads(monkeypatch, net, step, x, y, "0", False, init)[1] for _ in range(2)]
    merged_l, merged = _grads(monkeypatch, net, step, x, y, "1", True, init)
    step.dp.close()

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))
    live = [k for k, v in ref.items() if float(v.abs().max()) > 0]
    noise = [max(rel(f[k], ref[k]) for f in floors) for k in live]
    diff = [rel(merged[k], ref[k]) for k in live]
    n, d = _pct(noise), _pct(diff)
    print("per-head atomic-order vs deterministic (noise floor): median %.3g p90 %.3g max %.3g" % n)
    print("merged vs per-head (both deterministic):              median %.3g p90 %.3g max %.3g" % d)
    assert abs(merged_l - ref_l) < 1e-3 * abs(ref_l), (merged_l, ref_l)
    # (measured: the floor itself is O(1) - median 1.06 - the reduction order alone decorrelates the deep layers'
    # gradients of this chaotic network, so this bound only shows the merged path is no worse than that noise;
    # the discriminating whole-step check is the teacher-forced test below)
    assert d[0] <= 3.0 * n[0] + 1e-4 and d[1] <= 3.0 * n[1] + 1e-3, (d, n)


# ---------------------------------------------------------------------------------------------------------------
# Whole-model, teacher-forced: the random-init network's gradient is chaotic (a 1e-6 relative input perturbation
# moves the fp32 CPU gradients by a median 4 %, 1e-4 by 37 %, at any batch size; profiles/r5/
# r5_grad_sensitivity_inception_b16.log - ResNet-50 the same, r5_grad_sensitivity_resnet50_b16.log), so bf16
# storage alone decorrelates the deep layers' step-1 gradients from fp32 (the emulation's own per-tensor error in the
# fixture: median 1.3) and a per-tensor comparison of two whole backward passes cannot see a kernel error there.
# Instead, ONE real training step of the default GPU path (merged sibling heads, hand-offs, zero-copy concat, pool
# commute, grouped combines, aux dgrad on the MFMA tiles: nothing changed, hooks only observe) records every
# segment's input (the previous end point, bf16) and the gradient arriving at its output; the CPU then recomputes
# each segment - stem, 11 mixed blocks, aux head, logits head - in fp32 from exactly those inputs and output
# gradients, and in the bf16-storage emulation for the noise floor.  Every parameter gradient and every block's input
# gradient must match within 1.5x that floor (+2 %): each segment is checked in its real context without the
# cross-network amplification.

_SEGMENT_EPS = ("pool2", "mixed_35x35x256a", "mixed_35x35x288a", "mixed_35x35x288b", "mixed_17x17x768a",
                "mixed_17x17x768b", "mixed_17x17x768c", "mixed_17x17x768d", "mixed_17x17x768e", "mixed_17x17x1280a",
                "mixed_8x8x2048a", "mixed_8x8x2048b")


def _gpu_step_with_taps(monkeypatch, sib_fwd):
    T = _fixture()
    monkeypatch.setitem(features._override, "sibling_fwd", (sib_fwd) != "0")
    net = T.build().to(DEV)
    step = T.make_step(net)
    x, y = T.batches()[0]
    ep, grads = {}, {}
    orig = net.forward

    def fwd(images, training=True):
        out = orig(images, training, end_points=ep)
        for k in _SEGMENT_EPS:
            ep[k].register_hook(lambda g, k=k: grads.__setitem__(k, g.detach().float().cpu()))
        return out
    monkeypatch.setattr(net, "forward", fwd)
    loss, _skip = step._forward_backward(x.to(DEV).to(torch.bfloat16), y.to(DEV))
    torch.cuda.synchronize()
    acts = {k: ep[k].detach().float().cpu() for k in _SEGMENT_EPS}
    pg = {k: p.main_grad.detach().float().cpu() for k, p in net.named_parameters()
          if getattr(p, "main_grad", None) is not None}
    step.dp.close()
    assert set(grads) == set(_SEGMENT_EPS), sorted(set(_SEGMENT_EPS) - set(grads))
    return float(loss), x, y, acts, grads, pg


def _cpu_segments(x, y, acts, grads, emulate):
    """CPU recomputation of every segment from the GPU's inputs and output gradients -> (param grads, input grads
    per end point)."""
    import contextlib
    T = _fixture()
    from distributed_tensorflow_models_amd.ops import nn as F
    from distributed_tensorflow_models_amd.ops.lazy import as_tensor
    net = T.build()
    dx = {}
    ctx = T.bf16_storage() if emulate else contextlib.nullcontext()
    with ctx:
        def seg(inp_key, fn, out_grad=None, loss_fn=None):
            xin = (x if inp_key is None else acts[inp_key]).clone().requires_grad_(inp_key is not None)
            out = as_tensor(fn(xin))
            if loss_fn is not None:
                loss_fn(out.float()).backward()
            else:
                torch.autograd.backward(out, out_grad)
            if inp_key is not None:
                dx[inp_key] = dx.get(inp_key, 0) + xin.grad
        seg(None, lambda t: net.run_stem(t, True), grads["pool2"])
        prev = "pool2"
        for name, kind, branches in net.plan:
            if kind == "aux":
                seg(prev, lambda t: net.run_aux(t, True),
                    loss_fn=lambda o: 0.4 * F.softmax_cross_entropy(o, y, 0.1).mean())
                continue
            seg(prev, lambda t, b=branches: net.run_block(b, t, True), grads[name])
            prev = name
        seg(prev, lambda t: net.run_logits(t, True), loss_fn=lambda o: F.softmax_cross_entropy(o, y, 0.1).mean())
    pg = {k: p.grad.detach().clone() for k, p in net.named_parameters() if p.grad is not None}
    return pg, dx


@pytest.mark.parametrize("sib_fwd", ["1", "0"], ids=["merged", "per-head"])
def test_inception_v3_step_teacher_forced_per_segment(monkeypatch, sib_fwd):
    _loss, x, y, acts, grads, gpu_pg = _gpu_step_with_taps(monkeypatch, sib_fwd)
    f32_pg, f32_dx = _cpu_segments(x, y, acts, grads, False)
    emu_pg, emu_dx = _cpu_segments(x, y, acts, grads, True)

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))
    bad, e_g, e_e = [], [], []
    for k, f in f32_pg.items():
        if float(f.norm()) == 0:
            continue
        eg, ee = rel(gpu_pg[k], f), rel(emu_pg[k], f)
        e_g.append(eg)
        e_e.append(ee)
        if eg > 2.0 * ee + 0.03:
            bad.append("param %s: rel err %.4g (emulation %.4g)" % (k, eg, ee))
    # the gradient each block hands to the one below it (its input gradient, aux head included at 768e)
    for k in _SEGMENT_EPS[:-1]:
        eg, ee = rel(grads[k], f32_dx[k]), rel(emu_dx[k], f32_dx[k])
        e_g.append(eg)
        e_e.append(ee)
        if eg > 2.0 * ee + 0.03:
            bad.append("input gradient of the block after %s: rel err %.4g (emulation %.4g)" % (k, eg, ee))
    assert len(e_g) > 190, len(e_g)
    print("%s: %d tensors, GPU vs fp32 rel err median %.3g p90 %.3g max %.3g; emulation median %.3g p90 %.3g "
          "max %.3g" % ((sib_fwd, len(e_g)) + _pct(e_g) + _pct(e_e)))
    assert not bad, "\n".join(bad[:20])
    # and typically as close as the emulation: no systematic error hiding under the per-tensor slack (the slack is for
    # single tensors whose rounding points differ from the emulation's - the commuted pool branch rounds the conv
    # output before the pool, the reference after it - and for atomic-order noise; measured medians agree to 1 %)
    assert _pct(e_g)[0] < 1.1 * _pct(e_e)[0] + 2e-3 and _pct(e_g)[1] < 1.2 * _pct(e_e)[1] + 5e-3, (
        _pct(e_g), _pct(e_e))
