"""Training-step engine on CPU: fused-optimizer semantics (TF 1.x) and the NaN/Inf guard."""
import math

import torch

from distributed_tensorflow_models_amd.engine import TrainStep
from distributed_tensorflow_models_amd.models import nets_factory
from distributed_tensorflow_models_amd.ops.optim import FusedOptimizer


def test_nan_guard_skips_update():
    torch.manual_seed(0)
    m = nets_factory.build("lenet", 10)
    step = TrainStep(m, optimizer="momentum", lr=0.1)
    x = torch.randn(4, 28, 28, 1)
    y = torch.randint(0, 10, (4,))
    step(x, y)
    assert not step.poll_skipped()
    before = [p.detach().clone() for p in m.parameters()]
    x_bad = x.clone()
    x_bad[0, 0, 0, 0] = float("nan")
    loss = step(x_bad, y)
    assert math.isnan(float(loss))
    assert step.poll_skipped() and step.skipped == 1
    for a, p in zip(before, m.parameters()):
        assert torch.equal(a, p.detach())
    step(x, y)   # recovers on the next finite step
    assert not step.poll_skipped()


def test_tf_optimizer_semantics_cpu():
    for kind in ("sgd", "momentum", "rmsprop"):
        p = torch.nn.Parameter(torch.tensor([1.0, -2.0]))
        p.weight_decay = 0.1
        p.main_grad = torch.tensor([0.5, 0.25])
        opt = FusedOptimizer([p], kind, lr=0.1, momentum=0.9, rho=0.9, epsilon=1.0, ema_decay=0.99)
        opt.step(0.1, grad_scale=1.0)
        w0 = torch.tensor([1.0, -2.0])
        g = torch.tensor([0.5, 0.25]) + 0.1 * w0
        if kind == "sgd":
            exp = w0 - 0.1 * g
        elif kind == "momentum":
            exp = w0 - 0.1 * g                      # accum = 0*0.9 + g
        else:
            ms = 0.9 * 1.0 + 0.1 * g * g            # TF ms slot starts at 1.0
            exp = w0 - 0.1 * g / torch.sqrt(ms + 1.0)
        torch.testing.assert_close(p.detach(), exp, rtol=1e-6, atol=1e-6)
        # EMA with num_updates=0 -> decay = min(0.99, 1/10) = 0.1
        ema = opt.state[p]["ema"]
        torch.testing.assert_close(ema, w0 - (1 - 0.1) * (w0 - exp), rtol=1e-6, atol=1e-6)


import pytest  # noqa: E402


@pytest.mark.gpu
def test_nan_guard_skips_update_gpu():
    torch.manual_seed(0)
    m = nets_factory.build("resnet_v1_50", 10).cuda()
    step = TrainStep(m, optimizer="momentum", lr=0.1)
    x = torch.randn(2, 64, 64, 3, device="cuda").to(torch.bfloat16)
    y = torch.randint(0, 10, (2,), device="cuda")
    step(x, y)
    assert not step.poll_skipped()
    before = [p.detach().clone() for p in m.parameters()]
    x_bad = x.clone()
    x_bad[0, 5, 5, 0] = float("inf")
    step(x_bad, y)
    torch.cuda.synchronize()
    assert step.poll_skipped()
    assert all(torch.equal(a, p.detach()) for a, p in zip(before, m.parameters()))


def _run_steps(name, use_graph, steps, size, ncls, opt="momentum", ema=None, sched=None, lr=0.05,
               reset_seed=False, wgrad_stream=None, **kw):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if reset_seed:  # the same dropout masks in both runs of a comparison (the device offset is process state)
        from distributed_tensorflow_models_amd.ops import elementwise as E
        E.seed_offset(dev).zero_()
        E.set_base_seed(1234)
    model = nets_factory.build(name, num_classes=ncls, **kw).to(dev)
    step = TrainStep(model, optimizer=opt, lr=lr, momentum=0.9, use_graph=use_graph, ema_decay=ema,
                     lr_schedule=sched, wgrad_stream=wgrad_stream)
    g = torch.Generator().manual_seed(3)
    cin = 1 if name == "lenet" else 3
    xs = [torch.randn(4, size, size, cin, generator=g).to(dev, torch.bfloat16) for _ in range(2)]
    ys = [torch.randint(0, ncls, (4,), generator=g).to(dev) for _ in range(2)]
    losses = [float(step(xs[i % 2], ys[i % 2])) for i in range(steps)]
    torch.cuda.synchronize()
    params = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()])
    emas = (torch.cat([step.opt.state[p]["ema"].reshape(-1) for p in step.opt.params]) if ema else None)
    step.dp.close()
    return losses, params, emas, step


@pytest.mark.gpu
@pytest.mark.parametrize("name,size,ncls", [("resnet_v1_50", 64, 16), ("cifar10_cnn", 24, 10)])
def test_hipgraph_step_matches_eager(name, size, ncls):
    """Captured-and-replayed steps (alternating input buffers, lr schedule and EMA decay staged per
    replay) follow the eager trajectory (a captured step is single-stream: the weight-gradient side stream is
    left out of captures, ops/_lib.py side_stream)."""
    sched = lambda s: 0.05 * (0.5 ** (s // 3))  # noqa: E731
    le, pe, ee, _ = _run_steps(name, False, 6, size, ncls, ema=0.99, sched=sched, reset_seed=True)
    lg, pg_, eg, st = _run_steps(name, True, 6, size, ncls, ema=0.99, sched=sched, reset_seed=True)
    assert st._graph is not None and st.global_step == 6 and st.opt.num_updates == 6
    assert lg == pytest.approx(le, rel=2e-2, abs=2e-3)
    # BN statistics are summed with fp32 atomics, so two runs are not bit-identical, and the 2x2
    # last-block BN of this tiny ResNet amplifies that on a few elements: compare in norm
    for a, b in ((pg_, pe), (eg, ee)):
        assert ((a - b).norm() / b.norm()).item() < 1e-3


@pytest.mark.gpu
def test_hipgraph_inception_bit_exact_vs_eager():
    """Inception-v3 (299, batch 4: the aux head, merged sibling heads, dropout, concat BN) in deterministic mode:
    the captured step replays the eager trajectory bit for bit (a random-init Inception at batch 4 is chaotic enough that fp32-atomic reductions alone make two eager runs
    drift apart, so the comparison is made where every reduction has a fixed order)."""
    from distributed_tensorflow_models_amd.ops import _lib
    _lib.set_deterministic(True)
    side_was = _lib.side_enabled()
    try:
        # the eager run routes the weight gradients like the captured one (main stream: the side stream's split-K
        # sizing differs, another summation order); no dropout (an eager step draws a new host seed per step, a
        # replayed graph keeps the captured one and advances the device offset)
        kw = dict(lr=0.005, reset_seed=True, dropout_keep_prob=1.0)
        le, pe, _, _ = _run_steps("inception_v3_slim_old", False, 5, 299, 11, wgrad_stream=False, **kw)
        lg, pg_, _, st = _run_steps("inception_v3_slim_old", True, 5, 299, 11, wgrad_stream=False, **kw)
    finally:
        _lib.set_deterministic(False)
        _lib.set_side_enabled(side_was)
    assert st._graph is not None and st.global_step == 5
    assert all(math.isfinite(v) for v in le)
    assert lg == le
    assert torch.equal(pg_, pe)


@pytest.mark.gpu
def test_hipgraph_replay_draws_fresh_dropout_masks():
    """LeNet (dropout before the logits) under hipGraph replay: the device seed offset advances
    every replayed step, so masks differ step to step although the host seed was baked in."""
    from distributed_tensorflow_models_amd.ops import elementwise as E
    dev = torch.device("cuda", 0)
    off0 = int(E.seed_offset(dev).item())
    losses, params, _, st = _run_steps("lenet", True, 6, 28, 10, opt="sgd", lr=1e-4)
    assert st._graph is not None
    assert int(E.seed_offset(dev).item()) == off0 + 6
    assert all(math.isfinite(v) for v in losses) and bool(torch.isfinite(params).all())
    x = torch.randn(1 << 16, device=dev)
    E._seed_off[dev.index].fill_(5)
    a = E.dropout(x, 0.5, seed=99)
    E._seed_off[dev.index].fill_(6)
    b = E.dropout(x, 0.5, seed=99)
    assert not torch.equal(a, b)
    want = E.dropout_mask(x.shape, 0.5, E.mix_seed(99, 6)).to(dev)
    assert torch.equal(b != 0, want & (x != 0))


def test_bench_cpu_plumbing_json():
    """bench.py contract on the CPU plumbing config (BASELINE.json config 1: LeNet, no GPU)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--model", "lenet", "--device", "cpu",
                          "--steps", "2", "--warmup", "1", "--batch", "16"], capture_output=True, text=True,
                         timeout=300, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    r = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in r
    assert r["steps"] == 2 and r["n_gpus"] == 1 and r["value"] > 0 and r["config"]["model"] == "lenet"


@pytest.mark.gpu
def test_deterministic_mode_bit_reproducible_across_allocation_histories():
    """DTM_DETERMINISTIC / ops._lib.set_deterministic: two ResNet training runs whose allocation
    histories differ (a dummy allocation shifts every buffer) end bit-identical; BN statistics and
    gradient sums are summed in a fixed order instead of cross-block fp32 atomics."""
    from distributed_tensorflow_models_amd.ops import _lib
    _lib.set_deterministic(True)
    try:
        outs = []
        for pad in (0, 3 << 20):
            junk = torch.empty(pad + 1, device="cuda", dtype=torch.uint8)
            losses, params, _, st = _run_steps("resnet_v1_50", False, 3, 64, 16)
            outs.append((losses, params))
            del junk
        assert outs[0][0] == outs[1][0]
        assert torch.equal(outs[0][1], outs[1][1])
    finally:
        _lib.set_deterministic(False)


def _run_bench(args, env_extra=None, timeout=300):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, cwd=root, env=env)


def test_bench_self_launches_ranks():
    """``bench.py --gpus 2`` with no WORLD_SIZE starts its own 2 ranks (gloo on CPU here)."""
    import json
    out = _run_bench(["--model", "lenet", "--device", "cpu", "--gpus", "2", "--steps", "2", "--warmup", "1",
                      "--batch", "16"])
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["parallelism"] == "dp2" and r["config"]["global_batch"] == 32


def test_bench_refuses_world_size_mismatch():
    out = _run_bench(["--model", "lenet", "--device", "cpu", "--gpus", "4", "--steps", "1", "--warmup", "0"],
                     env_extra={"WORLD_SIZE": "2"})
    assert out.returncode == 2 and "WORLD_SIZE" in out.stderr


def test_bsp_bucket_layout_small_tail():
    """Buckets cover the flat gradient buffer exactly, at most bucket_mb each, and the last one of
    backward (the first layers' gradients) is cut at tail_mb so the exposed collective is short."""
    from distributed_tensorflow_models_amd.parallel.bsp import BSPDataParallel
    params = [torch.nn.Parameter(torch.zeros(n)) for n in (1000, 300_000, 50_000, 700_000, 20_000, 5_000)]
    dp = BSPDataParallel(params, bucket_mb=1.0, tail_mb=0.1)
    try:
        spans = [b for b in dp.buckets if isinstance(b[0], int)]
        assert spans[0][0] == 0 and spans[-1][1] == dp.flat.numel()
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
        assert all(e - s <= (1 << 20) // 4 for s, e in spans)
        assert spans[-1][1] - spans[-1][0] <= int(0.1 * (1 << 20)) // 4
        # every parameter's elements are accounted for exactly once
        assert sum(n for p in dp.params for _, n in dp.contrib[p]) == dp.flat.numel()
    finally:
        dp.close()


@pytest.mark.gpu
def test_scratch_growth_refused_inside_capture_and_graph_safe_after():
    """Scratch arenas never grow inside a hipGraph capture (a clear error instead of a hipMalloc in the
    captured region) and never free a retired arena (a graph captured earlier may point into it)."""
    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops.nn import _check
    L = _lib.lib()
    torch.cuda.synchronize()
    cap = int(L.dtm_ws_capacity(_lib.stream_ptr()))
    g = torch.cuda.CUDAGraph()
    t = torch.zeros(16, device="cuda")
    with torch.cuda.graph(g):
        t.add_(1.0)  # (a non-empty capture)
        rc = L.dtm_ws_reserve_stream(cap + 1, _lib.stream_ptr())
        err = L.dtm_ws_last_error()
        with pytest.raises(RuntimeError, match="captured into a hipGraph"):
            _check(rc, "probe")
    assert rc == -4 and err == -10
    r0 = int(L.dtm_ws_retired())
    assert L.dtm_ws_reserve_stream(cap + 1, _lib.stream_ptr()) == 0  # eager: grows
    assert int(L.dtm_ws_capacity(_lib.stream_ptr())) > cap and int(L.dtm_ws_retired()) == r0 + (1 if cap else 0)


@pytest.mark.gpu
def test_hipgraph_replay_after_larger_eager_step_matches_eager():
    """Capture a ResNet step, then run a much larger eager step in the same process (the scratch arenas and the
    flip-refresh table grow), then keep replaying: the replayed trajectory still follows the eager one (the
    round-3 illegal-address-after-capture mode: a captured graph pointing into a freed arena)."""
    from distributed_tensorflow_models_amd.ops import _lib
    le, pe, _, _ = _run_steps("resnet_v1_50", False, 6, 64, 16)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = nets_factory.build("resnet_v1_50", num_classes=16).to(dev)
    step = TrainStep(model, optimizer="momentum", lr=0.05, momentum=0.9, use_graph=True)
    g = torch.Generator().manual_seed(3)
    xs = [torch.randn(4, 64, 64, 3, generator=g).to(dev, torch.bfloat16) for _ in range(2)]
    ys = [torch.randint(0, 16, (4,), generator=g).to(dev) for _ in range(2)]
    losses = [float(step(xs[i % 2], ys[i % 2])) for i in range(3)]
    assert step._graph is not None
    # a second model, eager, at 16x the pixels and 8x the batch: every growable arena grows
    r0 = int(_lib.lib().dtm_ws_retired())
    other = nets_factory.build("resnet_v1_50", num_classes=1000).to(dev)
    big = TrainStep(other, optimizer="momentum", lr=0.01, momentum=0.9)
    big(torch.randn(32, 256, 256, 3, device=dev).to(torch.bfloat16), torch.randint(0, 1000, (32,), device=dev))
    torch.cuda.synchronize()
    if int(_lib.lib().dtm_ws_retired()) == r0:
        # (earlier tests of this process already grew the arenas past the big step's needs: force a growth of the
        # main-stream arena the captured graph points into)
        cap = int(_lib.lib().dtm_ws_capacity(_lib.stream_ptr()))
        assert _lib.lib().dtm_ws_reserve_stream(cap + 1, _lib.stream_ptr()) == 0
    assert int(_lib.lib().dtm_ws_retired()) > r0
    big.dp.close()
    del big, other
    losses += [float(step(xs[i % 2], ys[i % 2])) for i in range(3, 6)]
    torch.cuda.synchronize()
    params = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()])
    step.dp.close()
    assert losses == pytest.approx(le, rel=2e-2, abs=2e-3)
    assert ((params - pe).norm() / pe.norm()).item() < 1e-3
