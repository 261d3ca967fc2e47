#!/usr/bin/env python3
"""Merged sibling-head forward (feature sibling_fwd) vs per-head forward (DTM_DISABLE=sibling_fwd) on Inception-v3: per-parameter main_grad
relative errors of one training step, grouped by mixed block (deterministic reductions, pinned dropout), so a real
backward difference of the merged path (it would show in the blocks nearest the loss) can be told from random-init
drift (which grows towards the stem).

  python tools/diag_sibfwd.py [--batch 2] [--size 299]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--size", type=int, default=299)
    ap.add_argument("--model", default="inception_v3_slim_old")
    ap.add_argument("--block", default="", help="backprop a fixed gradient from this end point only (no loss): "
                    "the merged path of the blocks up to it, without the whole random-init net's drift")
    args = ap.parse_args()
    from distributed_tensorflow_models_amd.engine import TrainStep, moving_average_buffers
    from distributed_tensorflow_models_amd.models import nets_factory
    from distributed_tensorflow_models_amd.ops import _lib
    from distributed_tensorflow_models_amd.ops import elementwise as ew
    ew.advance_seed_offset = lambda device: None
    ew.next_seed = lambda: 1234
    _lib.lib().dtm_set_deterministic(1)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    net = nets_factory.build(args.model, num_classes=11).to(dev)
    step = TrainStep(net, optimizer="momentum", lr=0.0, momentum=0.9, wgrad_stream=False)
    x = torch.randn(args.batch, args.size, args.size, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 11, (args.batch,), device=dev)
    init = [b.detach().clone() for b in moving_average_buffers(net)]
    out = {}
    for run in ("0", "1", "0b"):
        os.environ["DTM_DISABLE"] = "" if run[0] == "1" else "sibling_fwd"
        with torch.no_grad():
            for b, v in zip(moving_average_buffers(net), init):
                b.copy_(v)
        if args.block:
            from distributed_tensorflow_models_amd.ops import fused as _fz
            step.dp.zero_grad()
            _fz.arena.begin_step(dev)  # (the per-step zero arena, as TrainStep does around every step)
            try:
                ep = {}
                net(x, training=True, end_points=ep)
                t = ep[args.block]
                g = torch.Generator(device="cpu").manual_seed(7)
                G = torch.randn(tuple(t.shape), generator=g).to(dev, t.dtype)
                torch.autograd.backward(t, G)
                _lib.side_join()
                loss = float(t.detach().float().norm())
                del ep, t
            finally:
                _fz.arena.end_step()
        else:
            loss, _ = step._forward_backward(x, y)
        torch.cuda.synchronize()
        out[run] = (float(loss), {k: p.main_grad.detach().float().clone() for k, p in net.named_parameters()
                                  if getattr(p, "main_grad", None) is not None},
                    [b.detach().clone() for b in moving_average_buffers(net)])
        print("run %s loss %.6f" % (run, out[run][0]), flush=True)

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-30))

    if args.block:
        live = [n for n, t in out["0"][1].items() if float(t.abs().max()) > 0]  # the parameters the gradient reached
        out = {k: (v[0], {n: v[1][n] for n in live}, v[2]) for k, v in out.items()}
    print("per-head repeat (0 vs 0b) identical:", all(torch.equal(out["0"][1][k], out["0b"][1][k]) for k in out["0"][1]))
    errs = {k: rel(out["1"][1][k], out["0"][1][k]) for k in out["0"][1]}
    blocks = {}
    for k, v in errs.items():
        b = k.split("__")[0] if k.startswith("layers.") else k.split(".")[0]
        blocks.setdefault(b, []).append(v)
    print("block                               n    median      max")
    for b, vs in blocks.items():
        print("%-34s %3d  %.3e  %.3e" % (b, len(vs), statistics.median(vs), max(vs)))
    srt = sorted(((v, k) for k, v in errs.items()), reverse=True)
    print("top 15:")
    for v, k in srt[:15]:
        print("  %.3e  %s" % (v, k))
    print("overall median %.3e" % statistics.median(errs.values()))
    mv = [rel(a, b) for a, b in zip(out["1"][2], out["0"][2])]
    print("moving statistics: median rel %.3e max %.3e" % (statistics.median(mv), max(mv)))


if __name__ == "__main__":
    main()
