#!/usr/bin/env python3
"""Why bench.py's final_loss differs run to run: the same ResNet-50 bench step (224^2, batch B, one fixed random batch
with random labels, momentum SGD + WD, bench.py's TrainStep) run REPS times from the same init, at the bench's lr 0.1
and at lr 0.01, with the default (atomic-order) reductions and with DTM_DETERMINISTIC.  Prints the loss at a few
steps per run.  Expected if the spread is reduction-order noise amplified by an optimisation at the edge of
stability: deterministic runs identical; default runs at lr 0.1 spread widely by step 25, at lr 0.01 stay close.
Usage: B=256 STEPS=25 REPS=3 python tools/loss_spread.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_tensorflow_models_amd.engine import TrainStep  # noqa: E402
from distributed_tensorflow_models_amd.models import nets_factory  # noqa: E402
from distributed_tensorflow_models_amd.ops import _lib  # noqa: E402


def run(lr, det, B, steps, x, y):
    _lib.set_deterministic(det)
    try:
        torch.manual_seed(0)
        net = nets_factory.build("resnet_v1_50", num_classes=1000).to("cuda")
        step = TrainStep(net, optimizer="momentum", lr=lr, momentum=0.9, weight_decay=1e-4)
        out = [float(step(x, y)) for _ in range(steps)]
        torch.cuda.synchronize()
        step.dp.close()
        return out
    finally:
        _lib.set_deterministic(False)


def main():
    B, steps, reps = int(os.environ.get("B", "256")), int(os.environ.get("STEPS", "25")), int(os.environ.get("REPS", "3"))
    g = torch.Generator().manual_seed(1)
    x = torch.randn(B, 224, 224, 3, generator=g).to("cuda", torch.bfloat16)
    y = torch.randint(0, 1000, (B,), generator=g).to("cuda")
    marks = [0, 4, 9, 14, 19, steps - 1]
    print("lr     mode           run  " + " ".join("step%-3d" % (m + 1) for m in marks), flush=True)
    for lr in (0.1, 0.01):
        for det in (False, True):
            finals = []
            for r in range(reps):
                ls = run(lr, det, B, steps, x, y)
                finals.append(ls[-1])
                print("%-6g %-14s %-4d " % (lr, "deterministic" if det else "default", r) +
                      " ".join("%7.4f" % ls[m] for m in marks), flush=True)
            print("%-6g %-14s final loss spread (max - min) %.4f" % (lr, "deterministic" if det else "default",
                                                                      max(finals) - min(finals)), flush=True)


if __name__ == "__main__":
    main()
