"""--trace_steps a:b -> torch.profiler (roctracer on ROCm) Chrome trace per rank; the reference
collected FULL_TRACE RunMetadata every step and never exported it."""
import contextlib
import os

import torch


def range_push(name):
    """roctx range push (torch.cuda.nvtx maps to roctx on ROCm builds); False when unavailable.
    Shows up in rocprofv3 --marker-trace and in the torch profiler timeline."""
    try:
        if torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
            return True
    except Exception:
        pass
    return False


def range_pop(active):
    if active:
        try:
            torch.cuda.nvtx.range_pop()
        except Exception:
            pass


@contextlib.contextmanager
def roctx(name):
    """Per-phase roctx range (fwd, loss, bwd, allreduce bucket issue / wait, nan guard, optimizer)."""
    a = range_push(name)
    try:
        yield
    finally:
        range_pop(a)


class StepTracer:
    def __init__(self, spec, outdir, rank=0):
        self.start = self.stop = None
        if spec:
            a, b = spec.split(":")
            self.start, self.stop = int(a), int(b)
        self.outdir, self.rank = outdir, rank
        self.prof = None

    def step(self, i):
        if self.start is None:
            return
        if i == self.start:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self.prof = torch.profiler.profile(activities=acts, record_shapes=False)
            self.prof.__enter__()
        elif i == self.stop and self.prof is not None:
            self.prof.__exit__(None, None, None)
            os.makedirs(self.outdir, exist_ok=True)
            path = os.path.join(self.outdir, "trace_rank%d_steps%d-%d.json" % (self.rank, self.start, self.stop))
            self.prof.export_chrome_trace(path)
            self.prof = None
            return path
        return None
