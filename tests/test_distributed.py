"""Multi-process CPU tests (gloo, 127.0.0.1) of the distributed paths: BSP gradient all-reduce
equivalence and determinism, ASP owner-sharded shared-memory store, SSP staleness bound, and the
launcher's restart-and-resume after an injected rank failure."""
import os
import time

import pytest
import torch

from distributed_tensorflow_models_amd.utils.testing import run_workers

B, S = 8, 24


def _batch():
    g = torch.Generator().manual_seed(123)
    return torch.randn(B, S, S, 3, generator=g), torch.randint(0, 10, (B,), generator=g)


def _bsp_worker(rank, world, steps=2, comm=None):
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory
    from distributed_tensorflow_models_amd.parallel import process_group as pg
    torch.manual_seed(0)
    model = nets_factory.build("cifar10_cnn", num_classes=10)
    pg.broadcast_tensors(list(model.parameters()))
    step = TrainStep(model, optimizer="momentum", lr=0.05, momentum=0.9, ema_decay=0.99, bucket_mb=0.25,
                     grad_comm_dtype=comm)
    x, y = _batch()
    per = B // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    losses = []
    for _ in range(steps):
        losses.append(float(step(xs, ys)))
    return {"params": torch.cat([p.detach().reshape(-1) for p in model.parameters()]),
            "ema": torch.cat([step.opt.state[p]["ema"].reshape(-1) for p in step.opt.params]),
            "mom": torch.cat([step.opt.state[p]["s1"].reshape(-1) for p in step.opt.params]),
            "losses": losses, "buckets": len(step.dp.buckets)}


def test_bsp_two_ranks_equal_single_rank_full_batch():
    single = _bsp_worker(0, 1)
    two = run_workers(_bsp_worker, 2)
    assert two[0]["buckets"] > 1  # the gradient really travelled in several buckets
    for r in range(2):
        assert torch.equal(two[r]["params"], two[0]["params"])  # replicas stay bit-identical
    for k in ("params", "ema", "mom"):
        torch.testing.assert_close(two[0][k], single[k], rtol=2e-4, atol=2e-6)


def test_bsp_bf16_gradient_communication():
    """bf16 on the wire: replicas stay identical and track the fp32 all-reduce to bf16 precision."""
    ref_ = run_workers(_bsp_worker, 2)
    lo = run_workers(_bsp_worker, 2, 2, torch.bfloat16)
    assert torch.equal(lo[0]["params"], lo[1]["params"])
    assert not torch.equal(lo[0]["params"], ref_[0]["params"])  # the bf16 path really ran
    for k in ("params", "mom"):
        torch.testing.assert_close(lo[0][k], ref_[0][k], rtol=2e-2, atol=2e-3)


def test_bsp_deterministic():
    a = run_workers(_bsp_worker, 2)
    b = run_workers(_bsp_worker, 2)
    assert torch.equal(a[0]["params"], b[0]["params"])


def _asp_worker(rank, world, lr=0.5):
    from distributed_tensorflow_models_amd.parallel.asp import ParamStore, wait_all_done
    torch.manual_seed(0)
    params = [torch.nn.Parameter(torch.full((5,), 1.0)), torch.nn.Parameter(torch.full((3, 2), 2.0)),
              torch.nn.Parameter(torch.zeros(4))]
    store = ParamStore(params, "sgd", lr, mode="shm", run_id="asp%d" % world)
    g = [torch.full_like(p, float(rank + 1)) for p in params]
    store.push(g)
    store.increment_global_step()
    wait_all_done(store.store, world, store.run_id)
    store.pull()
    out = {"params": [p.detach().clone() for p in params], "gs": store.global_step(),
           "owners": sorted(set(store.owner.values()))}
    store.close()
    return out


def test_asp_shared_store_applies_every_worker_update():
    res = run_workers(_asp_worker, 2)
    total = 0.5 * (1 + 2)
    for r in res:
        assert r["gs"] == 2
        assert r["owners"] == [0, 1]  # variables are round-robin sharded over the ranks (C14)
        torch.testing.assert_close(r["params"][0], torch.full((5,), 1.0 - total))
        torch.testing.assert_close(r["params"][1], torch.full((3, 2), 2.0 - total))
        torch.testing.assert_close(r["params"][2], torch.full((4,), -total))


def _ssp_worker(rank, world, s=2, steps=12):
    from distributed_tensorflow_models_amd.parallel.ssp import StalenessClock
    clock = StalenessClock(s, run_id="ssp%d" % world, poll_s=0.001, timeout_s=60)
    worst = 0
    for i in range(1, steps + 1):
        if rank == world - 1:
            time.sleep(0.03)  # the straggler
        m = clock.tick(i)
        worst = max(worst, i - m)
    clock.finish()
    return {"worst": worst, "waited": clock.waited_s}


def test_ssp_bounds_staleness():
    res = run_workers(_ssp_worker, 3)
    assert all(r["worst"] <= 2 for r in res)
    assert res[0]["waited"] > 0.05  # fast workers were actually held back


def test_launcher_restart_resumes_after_rank_failure(tmp_path):
    from distributed_tensorflow_models_amd.ckpt.saver import get_checkpoint_state
    from distributed_tensorflow_models_amd.parallel import launcher
    train_dir = str(tmp_path / "train")
    extra = ["--max_steps=6", "--batch_size=4", "--train_dir=" + train_dir, "--data_dir=/nonexistent",
             "--save_every_steps=1", "--fault_inject=1:3", "--fresh"]
    env_keep = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "2"
    try:
        rc = launcher.launch("cnn", "bsp", 2, extra, str(tmp_path / "logs"), max_restarts=1)
    finally:
        os.environ.clear()
        os.environ.update(env_keep)
    log0 = open(tmp_path / "logs" / "worker_0.log").read()
    assert rc == 0, log0[-3000:]
    assert "==== restart 1 ====" in log0 and "restored" in log0
    st = get_checkpoint_state(train_dir)
    assert st.model_checkpoint_path.endswith("model.ckpt-6")


# ---------------------------------------------------------------------------------------------
# GPU: the bucketed, hook-driven all-reduce with the real HIP kernels producing the gradients.
# RCCL refuses two ranks on one device, so the 1-GPU box runs two gloo ranks that share cuda:0
# (gloo reduces device tensors through host staging).  Both ranks see the SAME batch, so the
# averaged gradient equals the single-rank gradient exactly (x + x then * 1/2) even with BN.

def _bsp_gpu_worker(rank, world, steps=2, comm=None):
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    model = nets_factory.build("resnet_v1_50", num_classes=16).to(dev)
    step = TrainStep(model, optimizer="momentum", lr=0.05, momentum=0.9, bucket_mb=4.0, grad_comm_dtype=comm)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(4, 64, 64, 3, generator=g).to(dev, torch.bfloat16)
    y = torch.randint(0, 16, (4,), generator=g).to(dev)
    losses = [float(step(x, y)) for _ in range(steps)]
    torch.cuda.synchronize()
    out = {"params": torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu(),
           "losses": losses, "buckets": len(step.dp.buckets), "launched": sum(step.dp._launched)}
    step.dp.close()
    return out


@pytest.mark.gpu
def test_bsp_gpu_two_ranks_hip_kernels_match_single_rank():
    single = _bsp_gpu_worker(0, 1)
    two = run_workers(_bsp_gpu_worker, 2)
    assert two[0]["buckets"] > 4 and two[0]["launched"] == two[0]["buckets"]
    assert torch.equal(two[0]["params"], two[1]["params"])
    # BN statistics are summed with fp32 atomics (order varies run to run): not bit-exact across runs
    torch.testing.assert_close(two[0]["params"], single["params"], rtol=1e-3, atol=1e-5)
    assert two[0]["losses"] == pytest.approx(single["losses"], rel=1e-4)


# Step-1 gradients of every BASELINE data-parallel model, per parameter, W = 2 ranks each on ITS OWN batch vs the
# mean of the two single-rank gradients, over the gradient-routing fused paths (ops/features.py ROUTES_GRADIENTS,
# each switched off on its own): deterministic reductions make a correct run bit-exact, the BSP write checker
# (DTM_BSP_CHECK) raises on a gradient written after its bucket's all-reduce was issued.
_DP_MATRIX = [("resnet_v1_50", ())] + [("resnet_v1_50", (f,)) for f in (
    "fused_bn", "sibling_group", "bnout_fuse", "bwd1x1_fuse", "stem_wgrad_fuse", "wgrad_stream")] + [
    ("inception_v3_slim_old", ())] + [("inception_v3_slim_old", (f,)) for f in (
        "sibling_fwd", "sibling_combine", "sibling_group", "act_handoff", "cat_multi", "pool_commute",
        "wgrad_stream")] + [
    ("vgg_16", ()), ("vgg_16", ("wgrad_stream",)), ("vgg_16", ("bsp_compact",))]


def test_dp_matrix_covers_every_gradient_routing_feature():
    from distributed_tensorflow_models_amd.ops import features
    covered = {f for _m, fs in _DP_MATRIX for f in fs}
    assert covered == set(features.ROUTES_GRADIENTS), set(features.ROUTES_GRADIENTS) ^ covered


# the driver's GPU suite runs the default configs; DTM_DP_MATRIX=1 runs every row
_DP_RUN = _DP_MATRIX if os.environ.get("DTM_DP_MATRIX") == "1" else [c for c in _DP_MATRIX if not c[1]]


@pytest.mark.gpu
@pytest.mark.parametrize("model,off", _DP_RUN, ids=lambda v: v if isinstance(v, str) else
                         ("no-" + "-".join(v) if v else "defaults"))
def test_bsp_gpu_step1_gradients_match_single_rank(model, off):
    """Per-parameter step-1 gradients of 2 ranks, rank r on its own batch b_r, vs the mean over r of the single-rank
    gradient on b_r (each computed inside the same 2-rank job in a singleton group), deterministic reductions, BSP
    write checker on.  Distinct batches: a permuted, offset or dropped contribution of one rank cannot hide."""
    from distributed_tensorflow_models_amd.ops import features
    from distributed_tensorflow_models_amd.utils import dp_check
    res = run_workers(dp_check.grad_worker_pair, 2, model, features.disable_env(off) if off else None)
    two = [r["multi"] for r in res]
    ref = dp_check.mean_grads([r["single"] for r in res])
    assert two[0]["launched"] == two[0]["buckets"] > 1 and two[0]["writes_checked"] > 0
    if model == "vgg_16":
        assert two[0]["compact"] == (0 if "bsp_compact" in off else 1)  # fc6's live window travels alone
    # the two ranks' own gradients differ (distinct batches), so the check can see a mixed-up contribution
    d01 = dp_check.compare(res[0]["single"], res[1]["single"])
    assert sorted(r[1] for r in d01)[len(d01) // 2] > 1e-3
    rows = dp_check.compare(two[0], ref)
    bad = [r for r in rows if r[1] > 1e-5]
    print("%s %s: %d tensors, max rel err %.3g" % (model, off or "defaults", len(rows), max(r[1] for r in rows)))
    assert not bad, (len(bad), len(rows), bad[:6])
    assert torch.equal(two[0]["params"], two[1]["params"])


# The round-3 sibling-merge data-parallel mismatch, reduced to its mechanism (profiles/r4/README.md): a fused op
# that returns None for a parameter whose gradient a LATER op of the same backward writes into main_grad (the
# non-last members of a merged sibling group).  PyTorch still runs the parameter's post-accumulate-grad hook when
# the op returned None; the round-3 hook treated that as "ready", so the bucket's all-reduce was issued before the
# real gradient was written and the write was lost from the sum (world 1 never launches a collective, hence
# invisible single-rank).
class _DeferredGradFn(torch.autograd.Function):
    """y = x * w; the gradient of w is left to a later op (returned as None here, stashed in PENDING)."""
    PENDING = []

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        return x * w

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        _DeferredGradFn.PENDING.append((g * x).sum(0))
        return g * ctx.w_value, None


class _MergedGradFn(torch.autograd.Function):
    """y = x * v; writes v's gradient and the deferred one of w straight into main_grad, then notifies both."""

    @staticmethod
    def forward(ctx, x, v, w):
        ctx.save_for_backward(x, v)
        ctx.w = w
        return x * v

    @staticmethod
    def backward(ctx, g):
        from distributed_tensorflow_models_amd.ops import nn as opsnn
        x, v = ctx.saved_tensors
        w = ctx.w
        opsnn.grad_target(v).add_((g * x).sum(0))
        opsnn._notify(v)
        opsnn.grad_target(w).add_(_DeferredGradFn.PENDING.pop())
        opsnn._notify(w)
        return g * v, None, None


def _deferred_grad_worker(rank, world):
    from distributed_tensorflow_models_amd.parallel.bsp import BSPDataParallel
    torch.manual_seed(0)
    v = torch.nn.Parameter(torch.randn(5))
    w = torch.nn.Parameter(torch.randn(5))
    dp = BSPDataParallel([v, w], bucket_mb=1e-5, check=True, names=[("v", v), ("w", w)])
    try:
        x = torch.randn(3, 5, generator=torch.Generator().manual_seed(1 + rank))
        dp.zero_grad()
        ctx_w = w.detach()
        y = _MergedGradFn.apply(x, v, w)      # backward runs second: writes both gradients
        z = _DeferredGradFn.apply(y, w)       # backward runs first: returns None for w
        z.grad_fn.w_value = ctx_w
        z.sum().backward()
        dp.finish()
        return {"v": v.main_grad.clone() / world, "w": w.main_grad.clone() / world, "x": x, "vv": v.detach(),
                "wv": w.detach(), "launched": sum(dp._launched), "buckets": len(dp.buckets)}
    finally:
        dp.close()


def test_bsp_deferred_gradient_not_reported_early():
    res = run_workers(_deferred_grad_worker, 2)
    xs = [r["x"] for r in res]
    v, w = res[0]["vv"], res[0]["wv"]
    # d/dw sum((x*v)*w) = sum_rows x*v ; d/dv = sum_rows x*w ; mean over the two ranks' batches
    want_w = sum((x * v).sum(0) for x in xs) / 2
    want_v = sum((x * w).sum(0) for x in xs) / 2
    for r in res:
        assert r["launched"] == r["buckets"] > 1
        torch.testing.assert_close(r["w"], want_w)
        torch.testing.assert_close(r["v"], want_v)


def test_bsp_post_accumulate_hook_without_grad_is_not_ready():
    """The unit form: the hook with p.grad None (an op returned None and will write main_grad itself) must not
    mark p ready."""
    from distributed_tensorflow_models_amd.parallel.bsp import BSPDataParallel
    a, b = torch.nn.Parameter(torch.zeros(4)), torch.nn.Parameter(torch.zeros(3))
    dp = BSPDataParallel([a, b], bucket_mb=1e-5)
    try:
        dp.zero_grad()
        a.grad = None
        dp._on_accumulated(a)
        assert a not in dp._seen and not any(dp._launched)
        a.grad = torch.ones(4)
        dp._on_accumulated(a)
        assert a in dp._seen and a.grad is None and torch.equal(a.main_grad, torch.ones(4))
    finally:
        dp.close()


def test_bsp_check_catches_late_gradient_write():
    """The BSP write checker: a ready notification before the gradient write (the defect class that drops a
    write from the all-reduce) raises, naming the parameter."""
    from distributed_tensorflow_models_amd.ops import nn as opsnn
    from distributed_tensorflow_models_amd.parallel.bsp import BSPDataParallel
    a, b = torch.nn.Parameter(torch.zeros(4)), torch.nn.Parameter(torch.zeros(3))
    dp = BSPDataParallel([a, b], bucket_mb=1e-5, check=True, names=[("a", a), ("b", b)])
    try:
        dp.zero_grad()
        opsnn.grad_target(b).add_(1.0)
        opsnn._notify(b)  # b's bucket is complete -> issued
        with pytest.raises(RuntimeError, match="gradient of b written after"):
            opsnn.grad_target(b)
        with pytest.raises(RuntimeError, match="b reported ready twice"):
            opsnn._notify(b)
        dp.finish()
        assert dp.unreported == ["a"] and dp.writes_checked == 2
    finally:
        dp.close()


def test_launcher_detects_hung_rank_and_resumes(tmp_path):
    """A rank that stops making progress (alive, silent) is caught by the heartbeat monitor; the job
    is stopped and restarted from the latest checkpoint."""
    from distributed_tensorflow_models_amd.ckpt.saver import get_checkpoint_state
    from distributed_tensorflow_models_amd.parallel import launcher
    train_dir = str(tmp_path / "train")
    extra = ["--max_steps=6", "--batch_size=4", "--train_dir=" + train_dir, "--data_dir=/nonexistent",
             "--save_every_steps=1", "--fault_inject=1:3:hang", "--fresh"]
    env_keep = dict(os.environ)
    os.environ["OMP_NUM_THREADS"] = "2"
    t0 = time.time()
    try:
        rc = launcher.launch("cnn", "bsp", 2, extra, str(tmp_path / "logs"), max_restarts=1, hang_timeout=20.0)
    finally:
        os.environ.clear()
        os.environ.update(env_keep)
    log1 = open(tmp_path / "logs" / "worker_1.log").read()
    assert rc == 0, log1[-3000:]
    assert "hangs at step 3" in log1 and "==== restart 1 ====" in log1
    assert get_checkpoint_state(train_dir).model_checkpoint_path.endswith("model.ckpt-6")
    assert time.time() - t0 < 240


def test_heartbeat_staleness(tmp_path):
    from distributed_tensorflow_models_amd.utils import heartbeat as hb
    d = str(tmp_path / "hb")
    h = hb.Heartbeat(0, d, min_interval_s=0.0)
    h.beat(5)
    assert hb.read(d, 0)[0] == 5
    now = time.time()
    assert hb.stale_ranks(d, 2, 10.0, started_at=now - 5, now=now) == []         # rank 1 still starting
    assert hb.stale_ranks(d, 2, 10.0, started_at=now - 30, now=now) == [1]       # rank 1 never beat
    assert hb.stale_ranks(d, 2, 10.0, started_at=now - 30, now=now + 60) == [0, 1]


@pytest.mark.gpu
def test_bsp_gpu_two_ranks_bf16_wire():
    # one step: params = p0 - lr*g, so the difference is the bf16 rounding of the gradient itself
    # (over several steps the 2x2-pixel BN of this tiny ResNet amplifies any rounding chaotically)
    single = _bsp_gpu_worker(0, 1, 1)
    two = run_workers(_bsp_gpu_worker, 2, 1, torch.bfloat16)
    assert torch.equal(two[0]["params"], two[1]["params"])
    assert ((two[0]["params"] - single["params"]).norm() / single["params"].norm()).item() < 1e-3


def _dropout_worker(rank, world, seed):
    from distributed_tensorflow_models_amd.ops import elementwise as E
    E.set_base_seed(seed, rank)
    x = torch.ones(4096)
    return {"a": E.dropout(x, 0.5), "b": E.dropout(x, 0.5)}


def test_dropout_masks_differ_across_ranks_and_reproduce():
    """Every replica draws its own dropout masks (reference workers sample independently); a fixed
    (seed, rank) reproduces them exactly."""
    r1 = run_workers(_dropout_worker, 2, 7)
    r2 = run_workers(_dropout_worker, 2, 7)
    assert not torch.equal(r1[0]["a"], r1[1]["a"])
    assert not torch.equal(r1[0]["a"], r1[0]["b"])
    for r in range(2):
        assert torch.equal(r1[r]["a"], r2[r]["a"]) and torch.equal(r1[r]["b"], r2[r]["b"])


class _DeadTapNet(torch.nn.Module):
    """VGG-16 fc6 in miniature: a 7x7 'SAME' conv over a 1x1 map (48 of its 49 taps only read zero
    padding), between an ordinary conv stem and a 1x1 classifier."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.w1 = torch.nn.Parameter(torch.randn(16, 3, 3, 3, generator=g) * 0.2)
        self.w6 = torch.nn.Parameter(torch.randn(32, 7, 7, 16, generator=g) * 0.05)
        self.w8 = torch.nn.Parameter(torch.randn(10, 1, 1, 32, generator=g) * 0.1)

    def forward(self, x, training=True):
        from distributed_tensorflow_models_amd.ops import nn as F
        h = F.conv2d(x, self.w1, None, 2, "SAME", relu=True)
        h = F.max_pool(h, h.shape[1], h.shape[1], "VALID")
        h = F.conv2d(h, self.w6, None, 1, "SAME", relu=True)
        h = F.conv2d(h, self.w8, None, 1, "SAME")
        return h.reshape(h.shape[0], -1)


def _dead_tap_worker(rank, world, compact):
    os.environ["DTM_DISABLE"] = "" if compact else "bsp_compact"
    from distributed_tensorflow_models_amd.engine import TrainStep
    torch.manual_seed(0)
    model = _DeadTapNet()
    step = TrainStep(model, optimizer="momentum", lr=0.05, momentum=0.9, bucket_mb=0.01)
    x, y = _batch()
    per = B // world
    for _ in range(3):
        step(x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per])
    return {"params": torch.cat([p.detach().reshape(-1) for p in model.parameters()]),
            "wire": step.dp.wire_elements(), "compact": len(step.dp.compact)}


def test_bsp_dead_tap_gradients_left_out_of_the_allreduce():
    """The provably-zero gradient of dead taps never travels: the compact-bucket run sends 1/49 of the
    fc6-like weight and ends bit-identical to the full-buffer all-reduce (and across replicas)."""
    full = run_workers(_dead_tap_worker, 2, False)
    comp = run_workers(_dead_tap_worker, 2, True)
    assert comp[0]["compact"] == 1 and full[0]["compact"] == 0
    assert full[0]["wire"] - comp[0]["wire"] == 32 * 16 * 48  # the 48 dead taps of w6
    assert torch.equal(comp[0]["params"], comp[1]["params"])
    assert torch.equal(comp[0]["params"], full[0]["params"])


def _asp_ipc_worker(rank, world, kind="sgd", lr=0.5):
    """Two ranks sharing cuda:0: owner shards in HBM opened through HIP IPC by the other rank; every
    push is ONE fused multi-tensor optimizer launch writing the owners' memory directly."""
    from distributed_tensorflow_models_amd.parallel.asp import ParamStore, wait_all_done
    dev = torch.device("cuda", 0)
    params = [torch.nn.Parameter(torch.full((5,), 1.0, device=dev)),
              torch.nn.Parameter(torch.full((3, 20000), 2.0, device=dev)),  # several optimizer chunks
              torch.nn.Parameter(torch.zeros(4, device=dev))]
    store = ParamStore(params, kind, lr, momentum=0.9, mode="ipc", run_id="aspipc%s%d" % (kind, world))
    from distributed_tensorflow_models_amd.parallel import process_group as pg
    for step in range(2):
        g = [torch.full_like(p, float(rank + 1)) for p in params]
        for r in range(world):  # one pusher at a time: this test checks the update math, not Hogwild races
            if r == rank:
                store.push(g, sync=True)
                store.increment_global_step()
            pg.barrier()
    wait_all_done(store.store, world, store.run_id)
    store.pull()
    torch.cuda.synchronize()
    out = {"params": [p.detach().cpu().clone() for p in params], "gs": store.global_step(),
           "fused": getattr(store, "_ftens", None) is not None}
    store.close()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sgd", "momentum"])
def test_asp_gpu_ipc_fused_push(kind):
    res = run_workers(_asp_ipc_worker, 2, kind)
    # pushes land in the order rank 0, rank 1, rank 0, rank 1 with g = 1, 2, 1, 2 (lr 0.5)
    gs_seq = [1.0, 2.0, 1.0, 2.0]
    dec, a = 0.0, 0.0
    for g in gs_seq:
        if kind == "sgd":
            dec += 0.5 * g
        else:  # TF Momentum: a <- 0.9 a + g ; w -= lr a  (the accumulator lives in the owner shard)
            a = 0.9 * a + g
            dec += 0.5 * a
    for r in res:
        assert r["gs"] == 4 and r["fused"]
        torch.testing.assert_close(r["params"][1], torch.full((3, 20000), 2.0 - dec))
        torch.testing.assert_close(r["params"][2], torch.full((4,), -dec))
        torch.testing.assert_close(r["params"][0], torch.full((5,), 1.0 - dec))


# ---------------------------------------------------------------------------------------------
# BN moving statistics under BSP: the reference keeps ONE PS-resident copy that every worker's
# update op writes (inception/imagenet_inception_bsp.py:145-149); here every replica must end each
# step with the same statistics = the pre-step value plus every replica's update of it.

def _bn_sync_worker(rank, world, steps=3, gpu=False):
    import copy

    from distributed_tensorflow_models_amd.engine import TrainStep, moving_average_buffers
    from distributed_tensorflow_models_amd.models import nets_factory
    if gpu:  # the HIP kernels (conv epilogue statistics, stats_reduce_finalize moving-average update)
        os.environ["DTM_DETERMINISTIC"] = "1"
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
    torch.manual_seed(0)
    if gpu:
        model = nets_factory.build("resnet_v1_50", num_classes=16).to(dev)
        S, ncls, bdt = 64, 16, torch.bfloat16
    else:
        dev = torch.device("cpu")
        model = nets_factory.build("cifar10_resnet_v2", num_classes=10, resnet_size=8)
        S, ncls, bdt = 32, 10, torch.float32
    step = TrainStep(model, optimizer="momentum", lr=0.05, momentum=0.9, ema_decay=0.99, bucket_mb=0.05)
    g = torch.Generator().manual_seed(100 + rank)  # a DIFFERENT batch on every rank
    local, synced = [], []
    init = torch.cat([b.reshape(-1) for b in moving_average_buffers(model)]).clone()
    for _ in range(steps):
        x = (torch.randn(4, S, S, 3, generator=g) * (1 + rank)).to(dev, bdt)
        y = torch.randint(0, ncls, (4,), generator=g).to(dev)
        shadow = copy.deepcopy(model)  # what this replica's forward alone makes of the statistics
        with torch.no_grad():
            shadow(x, training=True)
        local.append(torch.cat([b.reshape(-1) for b in moving_average_buffers(shadow)]).cpu())
        step(x, y)
        synced.append(torch.cat([b.reshape(-1) for b in moving_average_buffers(model)]).cpu().clone())
    shadows = torch.cat([s.reshape(-1) for _b, s in step.opt.buffer_shadows()]).cpu()
    from distributed_tensorflow_models_amd.engine import moving_average_decays
    decays = set(moving_average_decays(model, moving_average_buffers(model)))
    out = {"local": torch.stack(local), "synced": torch.stack(synced), "shadows": shadows, "init": init.cpu(),
           "flat": step.bufsync.numel(), "nbuf": len(moving_average_buffers(model)),
           "decay": decays.pop() if len(decays) == 1 else None}
    step.dp.close()
    return out


@pytest.mark.parametrize("gpu", [False, pytest.param(True, marks=pytest.mark.gpu)], ids=["cpu", "gpu"])
def test_bsp_bn_moving_statistics_replica_consistent(gpu):
    """CPU: reference ops; GPU: two gloo ranks sharing cuda:0 with the HIP kernels computing the statistics."""
    res = run_workers(_bn_sync_worker, 2, 3, gpu)
    assert res[0]["nbuf"] > 0 and res[0]["flat"] > 0
    # bit-identical replicas after every step (and so are the EMA shadows of the statistics)
    assert torch.equal(res[0]["synced"], res[1]["synced"])
    assert torch.equal(res[0]["shadows"], res[1]["shadows"])
    # the ranks saw different data, so their own statistics differ ...
    assert not torch.allclose(res[0]["local"][0], res[1]["local"][0])
    # ... and the synced value applies BOTH replicas' updates to the one shared copy, as the reference's W
    # per-worker AssignMovingAvg ops on the PS variable do: d^W prev + (1 - d^W) mean_r B_r with B_r the
    # replica's implied batch statistic (m_r - d prev) / (1 - d), from the same pre-step state on both ranks
    d = res[0]["decay"]
    assert d is not None and 0.9 < d < 1.0
    prev = torch.cat([res[0]["init"][None], res[0]["synced"][:-1]]).double()
    loc = [r["local"].double() for r in res]
    b = [(lr - d * prev) / (1 - d) for lr in loc]
    want = d ** 2 * prev + (1 - d ** 2) * (b[0] + b[1]) / 2
    torch.testing.assert_close(res[0]["synced"].double(), want, rtol=1e-5, atol=1e-6)
    # to first order in (1 - d) this is prev + sum_r (m_r - prev)
    first = prev + (loc[0] - prev) + (loc[1] - prev)
    torch.testing.assert_close(res[0]["synced"].double(), first, rtol=1e-3, atol=1e-4)


def _bn_sync_convex_worker(rank, world, decay, every, steps):
    """BufferSync alone, on hand-made statistics: replica r's forward moves m towards its own batch value."""
    from distributed_tensorflow_models_amd.parallel.bsp import BufferSync
    mm, mv = torch.zeros(3), torch.ones(3)
    bs = BufferSync([mm, mv], every=every, decays=[decay, decay])
    hist = []
    for t in range(steps):
        bmean = torch.full((3,), 5.0 * (rank + 1) + t)
        bvar = torch.full((3,), 0.01 * (rank + 1))
        mm.sub_((mm - bmean) * (1 - decay))
        mv.sub_((mv - bvar) * (1 - decay))
        bs.issue()
        bs.finish()
        hist.append((mm.clone(), mv.clone()))
    return hist


@pytest.mark.parametrize("decay,every", [(0.9, 1), (0.9, 3), (0.997, 1)])
def test_bsp_bn_sync_convex_for_any_decay(decay, every):
    """with W = 8 replicas and NASNet-CIFAR's decay 0.9 (1 - W(1-d) < 0) the combined statistics stay
    a convex combination (variance positive, mean inside the replicas' range) and equal W*k sequential updates
    with the replicas' batch statistics averaged."""
    W, steps = 8, 6
    res = run_workers(_bn_sync_convex_worker, W, decay, every, steps)
    prev_m, prev_v = torch.zeros(3, dtype=torch.float64), torch.ones(3, dtype=torch.float64)
    loc = [(prev_m.clone(), prev_v.clone()) for _ in range(W)]
    k = 0
    for t in range(steps):
        k += 1
        for r in range(W):  # each replica's own forward update
            lm, lv = loc[r]
            loc[r] = (lm - (lm - (5.0 * (r + 1) + t)) * (1 - decay), lv - (lv - 0.01 * (r + 1)) * (1 - decay))
        if t % every == 0:  # a synced step (steps 1, 1 + every, ...)
            dk, dwk = decay ** k, decay ** (W * k)
            bm = sum((loc[r][0] - dk * prev_m) / (1 - dk) for r in range(W)) / W
            bv = sum((loc[r][1] - dk * prev_v) / (1 - dk) for r in range(W)) / W
            prev_m, prev_v = dwk * prev_m + (1 - dwk) * bm, dwk * prev_v + (1 - dwk) * bv
            loc = [(prev_m.clone(), prev_v.clone()) for _ in range(W)]
            k = 0
            assert all(torch.equal(res[0][t][i], r[t][i]) for r in res for i in (0, 1))
        for r in range(W):
            torch.testing.assert_close(res[r][t][0].double(), loc[r][0], rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(res[r][t][1].double(), loc[r][1], rtol=1e-5, atol=1e-6)
            mv = res[r][t][1]
            assert bool((mv > 0).all()) and bool((mv <= 1.0).all())
    if every == 1 and decay == 0.9:
        # the old first-order form would have weighted prev by 1 - W (1 - d) = 0.2 instead of d^W = 0.43
        assert abs(decay ** W - (1 - W * (1 - decay))) > 0.2


def test_bsp_bn_sync_abort_keeps_own_statistics():
    """An exception between issue() and finish(): the live statistics are this replica's own values, never a
    partial sum (single process: a 1-rank gloo group)."""
    res = run_workers(_bn_abort_worker, 2)
    for r in res:
        assert r["ok"]


def _bn_abort_worker(rank, world):
    from distributed_tensorflow_models_amd.parallel.bsp import BufferSync
    mm = torch.zeros(4)
    bs = BufferSync([mm], decays=[0.9])
    mm.fill_(1.0 + rank)  # this replica's forward
    bs.issue()
    own = mm.clone()
    bs.abort()
    return {"ok": torch.equal(mm, own)}


def test_bsp_single_rank_keeps_buffers_unflattened():
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory
    model = nets_factory.build("cifar10_resnet_v2", num_classes=10, resnet_size=8)
    step = TrainStep(model, optimizer="sgd", lr=0.01)
    assert step.bufsync.flat is None  # world 1: no collective, no re-homing


def _graph_refusal_worker(rank, world):
    from distributed_tensorflow_models_amd.engine import TrainStep
    from distributed_tensorflow_models_amd.models import nets_factory
    model = nets_factory.build("cifar10_cnn", num_classes=10)
    try:
        TrainStep(model, optimizer="sgd", lr=0.01, use_graph=True)
    except ValueError as e:
        return {"refused": "without collectives unless graph_comm" in str(e)}
    return {"refused": False}


def test_hipgraph_capture_refused_with_more_than_one_rank():
    assert all(r["refused"] for r in run_workers(_graph_refusal_worker, 2))


def _asp_buffer_worker(rank, world):
    """ASP: BN moving statistics live in the shared store; each worker pushes its forward's delta."""
    from distributed_tensorflow_models_amd.parallel import process_group as pg
    from distributed_tensorflow_models_amd.parallel.asp import ParamStore, wait_all_done
    p = torch.nn.Parameter(torch.ones(3))
    mm, mv = torch.zeros(4), torch.ones(4)
    store = ParamStore([p], "sgd", 0.1, mode="shm", run_id="aspbuf%d" % world, buffers=[mm, mv])
    for r in range(world):  # one worker at a time (this checks the bookkeeping, not the race)
        if r == rank:
            store.pull()
            mm.sub_((mm - float(rank + 1)) * 0.5)  # the forward's moving-average update, decay 0.5
            mv.mul_(0.5)
            store.push_buffers()
        pg.barrier()
    wait_all_done(store.store, world, store.run_id)
    store.pull()
    out = {"mm": mm.clone(), "mv": mv.clone()}
    store.close()
    return out


def test_asp_shared_bn_statistics():
    res = run_workers(_asp_buffer_worker, 2)
    # rank 0: mm 0 -> 0.5 ; rank 1 (sees 0.5): 0.5 -> 1.25 ; mv 1 -> 0.5 -> 0.25
    for r in res:
        torch.testing.assert_close(r["mm"], torch.full((4,), 1.25))
        torch.testing.assert_close(r["mv"], torch.full((4,), 0.25))


def test_ssp_debug_clock_is_read_only():
    """The SSP debug CLI observes a live job's clock without publishing a key of its own."""
    import torch.distributed as dist
    from distributed_tensorflow_models_amd.parallel.ssp import StalenessClock
    st = dist.HashStore()
    workers = [StalenessClock(2, store=st, rank=r, world=2, run_id="ro") for r in range(2)]
    workers[1].store.set(workers[1].prefix + "1", "3")
    obs = StalenessClock(store=st, rank=-1, world=2, run_id="ro", read_only=True)
    assert obs.steps() == [0, 3]
    assert not st.check([obs.prefix + "-1"])
    with pytest.raises(RuntimeError):
        obs.tick(1)
    obs.finish()
    assert obs.steps() == [0, 3]


def _rccl_single_rank_worker(rank, world):
    """One rank over RCCL (backend nccl) with the BSP bucket all-reduces and the BN-statistics sync forced on: the
    communicator, the bucket collectives issued from the backward hooks (side stream included), their timing events
    and the waits run for real - the part of the data-parallel path a one-GPU box can execute."""
    import torch.distributed as dist

    from distributed_tensorflow_models_amd.engine import TrainStep, moving_average_buffers
    from distributed_tensorflow_models_amd.models import nets_factory
    import sys
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    dev = torch.device("cuda", 0)
    out = {}
    for forced in (False, True):
        print("rccl worker: forced %s" % forced, file=sys.stderr, flush=True)
        torch.manual_seed(0)
        model = nets_factory.build("resnet_v1_50", num_classes=16).to(dev)
        step = TrainStep(model, optimizer="momentum", lr=0.05, momentum=0.9, bucket_mb=2.0, force_comm=forced)
        g = torch.Generator().manual_seed(5)
        x = torch.randn(8, 64, 64, 3, generator=g).to(dev, torch.bfloat16)
        y = torch.randint(0, 16, (8,), generator=g).to(dev)
        for i in range(2):
            step(x, y)
            print("rccl worker: step %d issued" % i, file=sys.stderr, flush=True)
        torch.cuda.synchronize()
        print("rccl worker: synchronized", file=sys.stderr, flush=True)
        out[forced] = {"params": torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu(),
                       "bufs": torch.cat([b.detach().reshape(-1) for b in moving_average_buffers(model)]).cpu(),
                       "works": len(step.dp._done_works), "buckets": len(step.dp.buckets),
                       "ms": step.dp.bucket_ms(), "bn_flat": step.bufsync.numel()}
        step.dp.close()
    return out


def _rccl_graph_worker(rank, world):
    """One rank over RCCL with every collective forced on (bucket all-reduces from the backward hooks, the BN-statistics
    sync): the eager step vs the step captured in a hipGraph WITH those collectives inside (graph_comm=True) and
    replayed - 2 eager warm-up steps, then the capture and 3 replays."""
    import sys

    import torch.distributed as dist

    from distributed_tensorflow_models_amd.engine import TrainStep, moving_average_buffers
    from distributed_tensorflow_models_amd.models import nets_factory
    from distributed_tensorflow_models_amd.ops import _lib
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    dev = torch.device("cuda", 0)
    _lib.set_deterministic(True)
    out = {}
    try:
        for graph in (False, True):
            print("rccl graph worker: graph %s" % graph, file=sys.stderr, flush=True)
            torch.manual_seed(0)
            model = nets_factory.build("resnet_v1_50", num_classes=16).to(dev)
            step = TrainStep(model, optimizer="momentum", lr=0.05, momentum=0.9, bucket_mb=2.0, force_comm=True,
                             use_graph=graph, graph_comm=True)
            g = torch.Generator().manual_seed(5)
            xs = [torch.randn(8, 64, 64, 3, generator=g).to(dev, torch.bfloat16) for _ in range(2)]
            ys = [torch.randint(0, 16, (8,), generator=g).to(dev) for _ in range(2)]
            losses = []
            for i in range(5):
                losses.append(float(step(xs[i % 2], ys[i % 2])))
                print("rccl graph worker: step %d" % i, file=sys.stderr, flush=True)
            torch.cuda.synchronize()
            out[graph] = {"params": torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu(),
                          "bufs": torch.cat([b.detach().reshape(-1) for b in moving_average_buffers(model)]).cpu(),
                          "losses": losses, "captured": step._graph is not None}
            step.dp.close()
    finally:
        _lib.set_deterministic(False)
    return out


@pytest.mark.gpu
def test_bsp_rccl_captured_step_matches_eager():
    """RCCL collectives inside a captured hipGraph step (graph_comm=True): at world 1 with every collective forced on,
    the captured-and-replayed steps are bit-identical to the eager ones (losses, parameters, BN moving statistics)."""
    res = run_workers(_rccl_graph_worker, 1, backend="nccl")[0]
    eager, graph = res[False], res[True]
    assert graph["captured"] and not eager["captured"]
    assert eager["losses"] == graph["losses"], (eager["losses"], graph["losses"])
    assert torch.equal(eager["params"], graph["params"]) and torch.equal(eager["bufs"], graph["bufs"])


@pytest.mark.gpu
def test_bsp_rccl_single_rank_collectives_are_identity():
    res = run_workers(_rccl_single_rank_worker, 1, backend="nccl")[0]
    off, on = res[False], res[True]
    assert off["works"] == 0 and on["works"] == on["buckets"] > 4 and on["bn_flat"] > 0
    assert len(on["ms"]) == on["works"] and all(v >= 0 for v in on["ms"])
    # a one-rank all-reduce is the identity: the same parameters as without collectives, bit for bit (BSP buckets);
    # the BN statistics go through the fp64 combine (d m_prev + (1 - d) B_r with B_r = (m_r - d m_prev) / (1 - d))
    assert torch.equal(on["params"], off["params"])
    torch.testing.assert_close(on["bufs"], off["bufs"], rtol=1e-6, atol=1e-7)
