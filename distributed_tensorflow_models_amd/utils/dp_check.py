"""Gradient-exactness check of BSP data parallelism on the real kernels.

The reference's BSP step applies exactly the mean of the W workers' gradients
(/root/reference/inception/imagenet_inception_bsp.py:123-157, /root/reference/vgg/cifar10_vgg_bsp.py:85-95).
Here every rank reduces its flat fp32 gradient buffer with bucketed all-reduces issued from inside backward,
so a kernel that writes a gradient after its bucket's collective was issued - or a ready notification that
comes before the write - silently drops or clobbers part of the sum.  ``grad_worker`` runs ONE training step
of a model, every rank on ITS OWN batch b_r (batch seed + rank; the same batch everywhere with ``distinct=False``),
with deterministic reductions (bit-reproducible kernels) and the BSP write checker on, and returns every
parameter's step-1 gradient (flat buffer / W) in backward order.  ``grad_worker_pair`` also runs each rank alone
(a singleton group) on its b_r; the W-rank gradient must equal the mean over r of those single-rank gradients -
with distinct batches a permutation, offset or dropped contribution between ranks cannot hide.  ``compare``
reports the per-tensor relative error.

Used by tests/test_distributed.py (GPU matrix over models and gradient-routing knobs) and
tools/dp_grad_diag.py (the per-parameter table).
"""
import os

import torch

# model name -> (builder kwargs, image size, batch, optimizer kwargs)
CONFIGS = {
    "resnet_v1_50": (dict(num_classes=16), 64, 4, dict(optimizer="momentum", lr=0.05, momentum=0.9)),
    # 299: the aux head's 5x5 VALID conv needs the 17x17 map (reference inception/slim/inception_model.py:227-236)
    "inception_v3_slim_old": (dict(num_classes=11), 299, 2,
                              dict(optimizer="rmsprop", lr=0.045, rho=0.9, epsilon=1.0, label_smoothing=0.1,
                                   aux_weight=0.4)),
    # the reference's CIFAR geometry: fc6 a 7x7 'SAME' conv over a 1x1 map -> compact dead-tap bucket
    "vgg_16": (dict(num_classes=10, fc_conv_padding="SAME"), 32, 4, dict(optimizer="momentum", lr=0.01,
                                                                          momentum=0.9)),
}


def grad_worker(rank, world, model_name, knobs=None, bucket_mb=2.0, overlap=True, steps=1, group=None,
                batch_seed=7):
    """One rank (world 1 = the reference run).  knobs: environment overrides (e.g. DTM_DISABLE=<features>, the
    gradient-routing fused paths of ops/features.py), set before any kernel call of this fresh process.  group:
    the process group of the data-parallel run (a singleton group gives the single-rank reference inside a
    multi-rank job); gradients are divided by its size."""
    os.environ.update({k: str(v) for k, v in (knobs or {}).items()})
    os.environ["DTM_DETERMINISTIC"] = "1"
    os.environ.setdefault("DTM_BSP_CHECK", "1")
    from ..engine import TrainStep
    from ..models import nets_factory
    from ..ops import elementwise as ew
    from ..ops import fused
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.manual_seed(0)
    ew.set_base_seed(0, 0)  # the same dropout masks in the singleton and the W-rank run of a rank ...
    ew.seed_offset(dev).zero_()  # ... and in every run of this process (the per-step offset is process state)
    kw, S, B, okw = CONFIGS[model_name]
    model = nets_factory.build(model_name, **kw).to(dev)
    step = TrainStep(model, bucket_mb=bucket_mb, overlap=overlap, process_group=group, **okw)
    world = step.dp.world
    g = torch.Generator().manual_seed(batch_seed)
    x = torch.randn(B, S, S, 3, generator=g).to(dev, torch.bfloat16)
    y = torch.randint(0, kw["num_classes"], (B,), generator=g).to(dev)
    n_sib = fused.SIBLING_MERGED[0]
    grads = []
    import sys
    import time
    t0 = time.time()
    for i in range(steps):
        step(x, y)
        torch.cuda.synchronize()
        print("dp_check rank %d/%d %s %s: step %d done (%.1f s)" % (rank, world, model_name, knobs or {}, i + 1,
                                                                   time.time() - t0), file=sys.stderr, flush=True)
        names = {p: n for n, p in model.named_parameters()}
        grads.append([(names[p], (p.main_grad.detach().float() / world).cpu()) for p in step.dp.order])
    out = {"grads": grads, "buckets": len(step.dp.buckets), "launched": sum(step.dp._launched),
           "compact": len(step.dp.compact), "sibling_merged": fused.SIBLING_MERGED[0] - n_sib,
           "writes_checked": step.dp.writes_checked, "unreported": list(step.dp.unreported),
           "params": torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu()}
    step.dp.close()
    return out


def compare(multi, single, step=0):
    """[(name, relative error, max abs error)] in backward order (relative: ||a - b|| / max(||b||, tiny))."""
    rows = []
    for (na, a), (nb, b) in zip(multi["grads"][step], single["grads"][step]):
        assert na == nb, (na, nb)
        d = (a - b).double()
        rel = float(d.norm() / max(float(b.double().norm()), 1e-30))
        rows.append((na, rel, float(d.abs().max()) if d.numel() else 0.0))
    return rows


def grad_worker_pair(rank, world, model_name, knobs=None, bucket_mb=2.0, overlap=True, steps=1, distinct=True):
    """The single-rank reference AND the world-rank run in ONE multi-rank job (process start-up and the rendezvous
    dominate the cost of a config): each rank first runs the model alone in a singleton process group (no
    collective: the reference) on its batch, then in the full group on the same batch.  Returns
    {"single": ..., "multi": ...}; the caller averages the ranks' "single" gradients (mean_grads)."""
    import torch.distributed as dist
    seed = 7 + (rank if distinct else 0)
    singles = [dist.new_group([r]) for r in range(world)]  # (every rank creates every group, in one order)
    single = grad_worker(rank, world, model_name, knobs, bucket_mb, overlap, steps, group=singles[rank],
                         batch_seed=seed)
    torch.cuda.empty_cache()
    multi = grad_worker(rank, world, model_name, knobs, bucket_mb, overlap, steps, batch_seed=seed)
    return {"single": single, "multi": multi}


def mean_grads(singles):
    """The reference of a W-rank BSP step: per parameter, the mean of the W single-rank gradients (the
    reference's SyncReplicasOptimizer applies the mean of the workers' gradients:
    /root/reference/inception/imagenet_inception_bsp.py:137-152).  Summed in rank order in fp32, then / W: the
    order the W-rank all-reduce of two ranks produces bit for bit."""
    W = len(singles)
    out = {"grads": []}
    for step in range(len(singles[0]["grads"])):
        rows = []
        for i, (name, g) in enumerate(singles[0]["grads"][step]):
            acc = g.clone()
            for s in singles[1:]:
                assert s["grads"][step][i][0] == name
                acc += s["grads"][step][i][1]
            rows.append((name, acc / W))
        out["grads"].append(rows)
    return out
