"""Observability: the reference per-step log line, node-wide throughput, JSONL
metrics stream and HIP-event step timers."""
import datetime
import json
import os
import time

import torch

LOG_FORMATS = {
    # alexnet/cifar10_alexnet_bsp.py:133-134, vgg bsp:135-136, cifarnet:128-129
    "standard": "time: {unix}; {now}: step {step} (global_step {gs}), loss = {loss:.2f} ({eps:.1f} examples/sec; "
                "{spb:.3f} sec/batch)",
    # cnn/cifar10_cnn_bsp.py:104 (no time: prefix)
    "cnn": "{now}: step {step} (global_step {gs}), loss = {loss:.2f} ({eps:.1f} examples/sec; {spb:.3f} sec/batch)",
    # resnet/cifar10_resnet_bsp.py:142, inception/imagenet_inception_bsp.py:196
    "short": "{now}: step {step} (gs {gs}), loss= {loss:.2f} ({eps:.1f} samples/s; {spb:.3f} s/batch)",
}


def format_step(style, step, gs, loss, examples_per_sec, sec_per_batch):
    return LOG_FORMATS[style].format(unix=time.time(), now=datetime.datetime.now(), step=step, gs=gs, loss=loss,
                                     eps=examples_per_sec, spb=sec_per_batch)


class JsonlMetrics:
    """Rank-0 JSONL stream: step, loss, lr, images/sec (per rank and node), step_ms, ..."""

    def __init__(self, path=None):
        self.f = None
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
            self.f = open(path, "a")

    def write(self, **kv):
        if self.f:
            kv.setdefault("wall", time.time())
            self.f.write(json.dumps(kv) + "\n")
            self.f.flush()

    def close(self):
        if self.f:
            self.f.close()
            self.f = None


class StepTimer:
    """Wall time per step plus optional HIP-event sections (fwd / bwd / allreduce / optimizer)."""

    def __init__(self, cuda=None):
        self.cuda = torch.cuda.is_available() if cuda is None else cuda
        self.events = {}
        self.t0 = None

    def start(self):
        self.t0 = time.perf_counter()

    def mark(self, name):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.events[name] = e

    def sections(self):
        out = {}
        if not self.events:
            return out
        torch.cuda.synchronize()
        names = list(self.events)
        for a, b in zip(names, names[1:]):
            out[b + "_ms"] = self.events[a].elapsed_time(self.events[b])
        self.events = {}
        return out

    def stop(self):
        return time.perf_counter() - self.t0
